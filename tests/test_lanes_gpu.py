"""The GPU parity suite (test_gpu_parity.py) re-run on the instance-per-lane kernel
(cl_lanes.h, compiled per topology at run time by cl_jit.cpp), plus that kernel against
the node-parallel one on the headline batch.  Under AUTO the library runs small batches
node-parallel (kLanesAutoMinInstances), so most parity cases would never reach the lanes
kernel without ENGINE_LANES; cases whose topology it cannot run (over 16 nodes, a degree
over 4) are skipped here and covered by test_gpu_parity.py."""
import numpy as np
import pytest

import enginecheck
from enginecheck import cl, engine_run
from test_gpu_parity import *  # noqa: F401,F403  (the parity cases, collected again here)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _lanes_engine():
    enginecheck.ENGINE = cl.ChandyLamportSim.ENGINE_LANES
    yield
    enginecheck.ENGINE = None


def test_lanes_equals_nodes_headline_with_spills():
    """2^20 instances of BASELINE config 3 with 2 LDS FIFO slots and with the default layout
    (split replays: the spilling instances -- over 65,536 of them, a wave per SIMD -- on the lanes
    spill kernel, the rest on the spill-free lanes kernel): every output plane equal between the
    two engines."""
    top, events, n = "8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20
    for slots in (None, 2):
        out = {}
        for eng in (cl.ChandyLamportSim.ENGINE_NODES, cl.ChandyLamportSim.ENGINE_LANES):
            enginecheck.ENGINE = eng
            sim = engine_run(top, events, n, fifo_lds_slots=slots)
            sim.rerun()
            sim.synchronize()
            assert sim.exec_engine() == eng
            out[eng] = (sim.checksums(), sim.status(), sim.time(), sim.counters(only_ok=False))
        a, b = out[cl.ChandyLamportSim.ENGINE_NODES], out[cl.ChandyLamportSim.ENGINE_LANES]
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
        assert a[3] == b[3]


def test_lanes_refuses_what_it_cannot_run():
    """ENGINE_LANES on a topology with a degree over 4 is an E_LIMIT error, not a silent
    node-parallel run; AUTO runs it node-parallel."""
    top = "6\nH 9\nA 0\nB 0\nC 0\nD 0\nE 0\n" + "".join(f"H {x}\n{x} H\n" for x in "ABCDE")
    sim = cl.ChandyLamportSim(64)
    sim.set_exec_engine(cl.ChandyLamportSim.ENGINE_LANES)
    sim.read_topology_text(top)
    sim.read_events_text("snapshot H\n")
    with pytest.raises(cl.ClSnapError) as e:
        sim.flush()
    assert e.value.code == cl.E_LIMIT
    sim2 = cl.ChandyLamportSim(64)
    sim2.read_topology_text(top)
    sim2.read_events_text("snapshot H\n")
    sim2.flush()
    assert sim2.exec_engine() == cl.ChandyLamportSim.ENGINE_NODES


@pytest.mark.parametrize("n", [1 << 17, 1 << 20])
def test_back_to_back_split_replays(n):
    """Split replays back to back do not fork the second stream from the main one (they touch
    disjoint instances): 2^17 instances put the spilling half on the node-parallel kernel, 2^20
    on the lanes spill kernel.  Ten replays in a row leave the same outputs as one, and a launch's
    kernel time (the longer half, each timed by its own events) stays within the wall time of a
    replay -- a half timed from the other stream's events would count the queueing."""
    import time
    sim = engine_run("8nodes.top", "8nodes-concurrent-snapshots.events", n)
    sim.rerun()
    sim.synchronize()
    spilled, split = sim.replay_split()
    assert 0 < split < n and 0 < spilled <= n - split
    one = (sim.checksums(), sim.status(), sim.counters(only_ok=False))
    sim.kernel_time()
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        sim.rerun()
    sim.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3 / reps
    k_total, k_n = sim.kernel_time()
    assert k_n == reps
    assert 0.5 * wall_ms < k_total / k_n < 1.2 * wall_ms
    many = (sim.checksums(), sim.status(), sim.counters(only_ok=False))
    assert np.array_equal(one[0], many[0]) and np.array_equal(one[1], many[1]) and one[2] == many[2]
