"""A/B timing of the instance-per-lane kernel on a headline batch: per variant (a cl_lanes.h
copy named by CLSNAP_LANES_HEADER, or a build), kernel ms per replay and the checksums against the
node-parallel engine's.  usage: python tools/lanes_ab.py [c3|c2] [reruns] [lanes|nodes|auto] [instances]"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
m = importlib.import_module("chandy-lamport-distributed-snapshot-algorithm_amd")
G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests/golden/test_data/")
cfgs = {"c3": ("8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20),
        "c2": ("10nodes.top", "10nodes.events", 65536)}
name = sys.argv[1] if len(sys.argv) > 1 else "c3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
eng = {"lanes": m.ChandyLamportSim.ENGINE_LANES, "nodes": m.ChandyLamportSim.ENGINE_NODES,
       "auto": m.ChandyLamportSim.ENGINE_AUTO}[sys.argv[3] if len(sys.argv) > 3 else "lanes"]
top, ev, n = cfgs[name]
if len(sys.argv) > 4:
    n = int(sys.argv[4])
s = m.ChandyLamportSim(n_instances=n)
s.set_exec_engine(eng)
s.read_topology_file(G + top)
s.read_events_file(G + ev)
s.flush()
s.synchronize()
fresh_ms, _ = s.kernel_time()   # the first launch: no replay plan (spill-capable kernel)
for _ in range(3):
    s.rerun()
s.synchronize()
s.kernel_time()
for _ in range(reps):
    s.rerun()
s.synchronize()
tot, k = s.kernel_time()
print(f"{name} n={n} engine={s.exec_engine()} variant={os.environ.get('CLSNAP_VARIANT', '')} rerun_ms={tot / k:.4f} fresh_ms={fresh_ms:.4f} "
      f"sums={s.checksums().tolist()}", flush=True)
