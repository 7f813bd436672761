"""GPU check of the instance-per-lane kernel: which engine ran, JIT time, kernel times of both
engines on the same batch, and that their results agree (checksums)."""
import sys, time, importlib, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
m = importlib.import_module("chandy-lamport-distributed-snapshot-algorithm_amd")
G = "tests/golden/test_data/"
cfgs = {"c3": ("8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20, 0),
        "c3s8": ("8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20, 8),
        "c3s2": ("8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20, 2),
        "c2": ("10nodes.top", "10nodes.events", 65536, 0)}
for name in sys.argv[1:] or ["c3", "c2"]:
    top, ev, n, slots = cfgs[name]
    res = {}
    for eng in (m.ChandyLamportSim.ENGINE_NODES, m.ChandyLamportSim.ENGINE_LANES):
        s = m.ChandyLamportSim(n_instances=n)
        s.set_exec_engine(eng)
        if slots:
            s.set_limits(fifo_lds_slots=slots)
        s.read_topology_file(G + top)
        t0 = time.time()
        s.read_events_file(G + ev)
        s.flush()
        t1 = time.time()
        used = s.exec_engine()
        for _ in range(3):
            s.rerun()
        s.synchronize()
        s.kernel_time()
        for _ in range(10):
            s.rerun()
        s.synchronize()
        tot, k = s.kernel_time()
        res[eng] = s.checksums()
        print(f"{name} engine={eng} used={used} first_flush_s={t1-t0:.2f} rerun_ms={tot/k:.4f} "
              f"jit={m.jit_stats()} split={s.replay_split()}", flush=True)
    print(name, "checksums equal:", res[1] == res[2], res[1][:6], flush=True)
