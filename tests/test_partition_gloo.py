"""The graph-partitioned single-simulation protocol
on 2 and 3 gloo ranks on the CPU, bit-exact against the oracle's unpartitioned run.

Every rank runs its node range of ONE simulation (tests/partition_model.py, the CPU
stand-in of the engine halves) and exchanges deliveries, broadcast-trigger reports,
trigger totals and draw bases through the package's exchange layer (dist.py
exchange_rows / allgather_ints -- the same calls the device mode makes over RCCL).
The oracle runs the same program on one simulator; final tokens, completion ticks,
snapshot token maps, per-channel recorded messages and the reference counters (pushes,
peeks, delivered tokens and markers, recorded copies, completed snapshots) must agree.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from snapcheck import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _program(kind, n, steps, seed):
    import graphcheck as GC
    if kind == "regular":
        return GC.regular_program(n, steps=steps, seed=seed, snaps=((5, None), (5, 0), (9, None), (17, None)))
    p = GC.powerlaw_program(n, steps, 12, seed=seed)
    p.traffic_steps = 60          # traffic stops, so snapshots complete inside the window
    return p


def _worker(rank, world, port, kind, n, steps, seed, out):
    import sys
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from partition_model import PartitionedSim
    p = _program(kind, n, steps, seed)
    sim = PartitionedSim(rank, world, p.tokens, p.src, p.dst, p.delay_seed)
    sim.run_program(p.steps, p.traffic_seed, p.thresh, p.traffic_steps, p.snap_step, p.snap_rank)
    tokens, ctick, cnt, snaps = sim.results()
    if rank == 0:
        out["r"] = (tokens, ctick, dict(cnt), {sid: (tok, msgs) for sid, (tok, msgs) in snaps.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,n,steps,seed,world", [("regular", 4096, 90, 3, 2), ("regular", 1000, 110, 5, 3),
                                                     ("powerlaw", 2000, 300, 7, 2)])
def test_partitioned_protocol_vs_oracle(kind, n, steps, seed, world):
    import graphcheck as GC
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), kind, n, steps, seed, out), nprocs=world, join=True)
    tokens, ctick, cnt, snaps = out["r"]
    p = _program(kind, n, steps, seed)
    o = GC.oracle_program(p)
    assert o.status == 0
    nt = o.node_tokens()
    np.testing.assert_array_equal(tokens, np.array([nt[k] for k in o.node_ids()], dtype=np.int64))
    assert ctick == [o.completion_tick(s) for s in range(o.num_snapshots)]
    assert sum(x >= 0 for x in ctick) >= 1
    oc = o.counters()
    for k in ("push", "peek", "pop_tok", "pop_mk", "recorded", "completed"):
        assert cnt.get(k, 0) == oc[k], f"{k}: partitioned {cnt.get(k, 0)} vs oracle {oc[k]}"
    src, dst = GC.G.dedup(p.src, p.dst)
    for sid, (tok, msgs) in snaps.items():
        otok, ooff, ovals = o.collect_channels(sid)
        np.testing.assert_array_equal(tok, otok)
        for c in range(len(src)):
            want = ovals[ooff[c]:ooff[c + 1]].tolist()
            assert msgs.get((int(src[c]), int(dst[c])), []) == want, (sid, c)
