"""Cycle attribution of the exec kernel (diagnostic `prof` variant, CLSNAP_PROF=1).

usage: CLSNAP_VARIANT=prof python tools/prof_c2.py [c2|c3]
Prints shader-clock cycles per program part, per wave and per wave-tick."""
import ctypes as C
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
top, events, n, _ = bench.CONFIGS[cfg]
cl = importlib.import_module(bench.PKG)
sim = cl.ChandyLamportSim(n, device=0, seed_base=cl.REFERENCE_SEED)
sim.read_topology_file(os.path.join(bench.TEST_DATA, top))
sim.read_events_file(os.path.join(bench.TEST_DATA, events))
sim.flush()
sim.synchronize()
L = cl.lib()
buf = (C.c_ulonglong * 8)()
L.cl_prof_read(buf, 1)
reps = 10
for _ in range(reps):
    sim.rerun()
sim.synchronize()
L.cl_prof_read(buf, 1)
names = ["send ops", "snap ops", "tick A+B", "tick C/D", "loop ctl", "prologue", "epilogue", "ticks"]
waves = (n + 64 // sim.num_nodes - 1) // (64 // sim.num_nodes)
tot = sum(buf[k] for k in range(7))
for k in range(8):
    print(f"{names[k]:10s} {buf[k] / reps / waves:12.1f} per wave  {100.0 * buf[k] / tot if k < 7 else 0:5.1f}%")
print(f"ticks/wave {buf[7] / reps / waves:.1f}; cycles per wave-tick (A+B+C/D) "
      f"{(buf[2] + buf[3]) / max(buf[7], 1):.1f}")
