"""Graph-partitioned mode on the device: ONE simulation
split over 2 or 3 processes that share the box's GPU, each owning a block-aligned node
range, exchanging deliveries, trigger reports, trigger totals and draw replies every tick
over gloo (graph.py PartitionedGraphSim -> cl_graph_part_*).  The gathered run must equal
the oracle's unpartitioned run bit for bit: status, time, final tokens, completion ticks,
snapshot token maps, per-channel recorded messages and the reference counters.

Both transports are covered: "host" stages every exchanged row through host arrays;
"device" keeps them in device buffers (cl_graph_part_dev_*: fixed-capacity buckets, the
collectives on the engine's stream, no host round trip per tick), here with gloo staging
the buckets through host memory since the ranks share one GPU.  The 8-GPU form (one rank
per GPU, RCCL on the device buffers) is the same code with exchange_device="cuda"; it is
not measured."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from snapcheck import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _program(kind, n, steps, seed):
    import graphcheck as GC
    if kind == "regular":
        return GC.regular_program(n, steps=steps, seed=seed, snaps=((5, None), (5, 0), (9, None), (17, None)))
    p = GC.powerlaw_program(n, steps, 12, seed=seed, fifo_slots=512)   # (hub channels queue deep)
    p.traffic_steps = 60
    return p


def _worker(rank, world, port, case, out):
    import sys
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import graphcheck as GC
        kind, n, steps, seed, _, lanes, drain, transport = case
        p = _program(kind, n, steps, seed)
        g = GC.clg.GraphSim(device=0, fifo_slots=p.fifo_slots, max_snapshots=len(p.snap_step))
        g.set_push_lanes(lanes)
        g.set_topology(p.tokens, p.src, p.dst, id_width=p.width())
        g.set_delay_hash(p.delay_seed)
        g.set_traffic(p.traffic_seed, p.thresh, p.traffic_steps)
        ps = GC.clg.PartitionedGraphSim(g, rank, world, transport=transport)
        ps.run_program(p.steps, p.snap_step, p.snap_rank)
        if drain:
            assert ps.drain()
        res = ps.results()
        if rank == 0:
            out["r"] = res + (ps.time,)
    except Exception as e:  # surfaced in the parent
        out[f"error{rank}"] = repr(e)
        raise
    finally:
        dist.destroy_process_group()


CASES = [("regular", 4096, 90, 3, 2, 0, False, "host"), ("regular", 4096, 100, 5, 3, 1, False, "host"),
         ("powerlaw", 2000, 300, 7, 2, 0, False, "host"), ("powerlaw", 2000, 70, 9, 2, 4, True, "host"),
         ("regular", 4096, 90, 3, 2, 0, False, "device"), ("regular", 4096, 100, 5, 3, 1, False, "device"),
         ("powerlaw", 2000, 300, 7, 2, 0, False, "device"), ("powerlaw", 2000, 70, 9, 3, 4, True, "device")]


@pytest.mark.parametrize("case", CASES,
                         ids=lambda c: f"{c[0]}{c[1]}_w{c[4]}_l{c[5]}{'_drain' if c[6] else ''}_{c[7]}")
def test_partitioned_device_run_vs_oracle(case):
    import graphcheck as GC
    kind, n, steps, seed, world, _, drain, _ = case
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), case, out), nprocs=world, join=True)
    assert "r" in out, dict(out)
    status, tokens, ctick, cnt, snaps, time = out["r"]
    p = _program(kind, n, steps, seed)
    o = GC.oracle_program(p, drain=drain)
    assert status == 0 and o.status == 0
    assert time == o.time
    nt = o.node_tokens()
    np.testing.assert_array_equal(tokens, np.array([nt[k] for k in o.node_ids()], dtype=np.int64))
    assert ctick == [o.completion_tick(s) for s in range(o.num_snapshots)]
    assert sum(x >= 0 for x in ctick) >= 1
    if drain:
        assert all(x >= 0 for x in ctick)
    oc = o.counters()
    for k in ("push", "peek", "pop_tok", "pop_mk", "recorded", "completed"):
        assert cnt[k] == oc[k], f"{k}: partitioned {cnt[k]} vs oracle {oc[k]}"
    assert set(snaps) == {s for s in range(o.num_snapshots) if o.complete(s)}
    for sid, (tok, off, vals) in snaps.items():
        otok, ooff, ovals = o.collect_channels(sid)
        np.testing.assert_array_equal(tok, otok)
        np.testing.assert_array_equal(off, ooff)
        np.testing.assert_array_equal(vals, ovals)


def _freeze_worker(rank, world, port, transport, out):
    import sys
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import graphcheck as GC
        p = _program("powerlaw", 2000, 120, 9)
        g = GC.clg.GraphSim(device=0, fifo_slots=4, max_snapshots=len(p.snap_step))
        g.set_topology(p.tokens, p.src, p.dst, id_width=p.width())
        g.set_delay_hash(p.delay_seed)
        g.set_traffic(p.traffic_seed, p.thresh, p.traffic_steps)
        ps = GC.clg.PartitionedGraphSim(g, rank, world, transport=transport)
        ps.run_program(p.steps, p.snap_step, p.snap_rank)
        out[rank] = (g.status(), ps.frozen, ps.time)
    except Exception as e:  # surfaced in the parent
        out[f"error{rank}"] = repr(e)
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("transport", ["host", "device"])
def test_partitioned_freeze_stops_every_rank(transport):
    """Four FIFO slots per channel overflow at the power-law hubs on one rank (an engine
    limit, CL_INST_FIFO_OVERFLOW): the status is allgathered with the tick totals, so every
    rank stops at the same step with the same status instead of drawing from the frozen
    rank's stale totals -- the whole-graph engine freezes with that status too."""
    import graphcheck as GC
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_freeze_worker, args=(2, _free_port(), transport, out), nprocs=2, join=True)
    (s0, f0, t0), (s1, f1, t1) = out[0], out[1]
    assert f0 == f1 != 0 and s0 == s1 == f0 and t0 == t1
    p = _program("powerlaw", 2000, 120, 9)
    p.fifo_slots = 4
    g = GC.engine_program(p)
    assert g.status() == s0
