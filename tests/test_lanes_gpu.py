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
    """2^20 instances of BASELINE config 3 with 2 LDS FIFO slots (a split replay: the spilling
    instances on the node-parallel spill kernel, the rest on the lanes kernel) and with the
    default layout: every output plane equal between the two engines."""
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
