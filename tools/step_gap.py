"""Per-step host wall time vs the exec kernels' own time over back-to-back reruns (the bench's
timed loop), to price what lies between replays.  usage: python tools/step_gap.py n slots engine"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
m = importlib.import_module("chandy-lamport-distributed-snapshot-algorithm_amd")
G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/test_data/")
n = int(sys.argv[1]); slots = int(sys.argv[2]); eng = sys.argv[3]
s = m.ChandyLamportSim(n_instances=n, fifo_lds_slots=slots or None)
s.set_exec_engine({"lanes": 2, "nodes": 1, "auto": 0}[eng])
s.read_topology_file(G + "8nodes.top")
s.read_events_file(G + "8nodes-concurrent-snapshots.events")
s.flush()
for _ in range(20):
    s.rerun()
s.synchronize()
s.kernel_time()
K = 200
t0 = time.perf_counter()
for _ in range(K):
    s.rerun()
s.synchronize()
wall = (time.perf_counter() - t0) / K * 1e3
tot, k = s.kernel_time()
print(f"n={n} slots={slots} engine={s.exec_engine()} split={s.replay_split()} step_ms={wall:.4f} "
      f"kernel_ms={tot / k:.4f} gap_us={(wall - tot / k) * 1e3:.1f}", flush=True)
