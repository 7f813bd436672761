"""CPU checks of the instance-per-lane engine's host side: the engine switch, and that the
kernels hipRTC generates for each reference topology compile for gfx950 (no device needed;
the GPU runs are test_lanes_gpu.py)."""
import pytest

from enginecheck import cl
from snapcheck import read_text, scenarios


def test_engine_switch_and_query():
    sim = cl.ChandyLamportSim(8)
    assert sim.exec_engine() == 0                    # nothing launched yet
    for e in (sim.ENGINE_NODES, sim.ENGINE_LANES, sim.ENGINE_AUTO):
        sim.set_exec_engine(e)
    with pytest.raises(cl.ClSnapError) as err:
        sim.set_exec_engine(7)
    assert err.value.code == cl.E_INVALID


_TOPS = sorted({sc["top"] for sc in scenarios()})


@pytest.mark.parametrize("top", _TOPS)
def test_lanes_kernels_compile_for_reference_topologies(top):
    sc = [s for s in scenarios() if s["top"] == top][0]
    sim = cl.ChandyLamportSim(64)
    sim.read_topology_text(read_text(top))
    sim.read_events_text(read_text(sc["events"]))
    ms, log = sim.lanes_compile_check()
    assert ms > 0
    assert "error" not in log.lower()


def test_lanes_compile_check_refuses_high_degree():
    top = "6\nH 9\nA 0\nB 0\nC 0\nD 0\nE 0\n" + "".join(f"H {x}\n{x} H\n" for x in "ABCDE")
    sim = cl.ChandyLamportSim(8)
    sim.read_topology_text(top)
    sim.read_events_text("snapshot H\n")
    with pytest.raises(cl.ClSnapError) as err:
        sim.lanes_compile_check()
    assert err.value.code == cl.E_LIMIT
