"""Helpers that compare the GPU engine with the oracle, instance by instance."""
import importlib
import os

import numpy as np

import oracle as O
from snapcheck import TEST_DATA, read_text

cl = importlib.import_module("chandy-lamport-distributed-snapshot-algorithm_amd")


# The exec engine the parity tests run on: None = the library's choice (AUTO); test_lanes_gpu
# sets ENGINE_LANES to re-run the parity suite on the instance-per-lane kernel.
ENGINE = None


def new_sim(n, **kw):
    sim = cl.ChandyLamportSim(n, **kw)
    if ENGINE is not None:
        sim.set_exec_engine(ENGINE)
    return sim


def checked_flush(sim):
    """flush(); under a forced engine, a topology that engine cannot run skips the test and
    a completed launch must have used it."""
    try:
        sim.flush()
    except cl.ClSnapError as e:
        if ENGINE is not None and e.code == cl.E_LIMIT:
            import pytest
            pytest.skip(f"engine {ENGINE} does not fit this case: {e}")
        raise
    if ENGINE is not None and sim.exec_engine() != 0:
        assert sim.exec_engine() == ENGINE


def engine_run(top, events, n, seed_base=O.REFERENCE_SEED, schedule=None, fifo_lds_slots=None,
               max_drain_ticks=None, flush=True):
    sim = new_sim(n, seed_base=seed_base, fifo_lds_slots=fifo_lds_slots, max_drain_ticks=max_drain_ticks)
    sim.read_topology_text(top if "\n" in top else read_text(top))
    if schedule is not None:
        sim.set_delay_schedule(schedule)
    sim.read_events_text(events if "\n" in events else read_text(events))
    if flush:
        checked_flush(sim)
    return sim


def oracle_run(top, events, seed=None, schedule=None, max_drain=O.MAX_DRAIN_TICKS):
    ref = O.OracleSim()
    if schedule is not None:
        ref.use_schedule(schedule)
    else:
        ref.seed_go(seed)
    assert ref.read_topology_text(top if "\n" in top else read_text(top)) == 0
    assert ref.read_events_text(events if "\n" in events else read_text(events), max_drain) >= 0
    return ref


def canonical(msgs):
    """Per-channel message lists: the comparison unit (test_common.go:253-284)."""
    out = {}
    for m in msgs:
        t = m.astuple() if hasattr(m, "astuple") else tuple(m)
        out.setdefault((t[0], t[1]), []).append(t[2])
    return out


def compare_instance(sim, i, ref, status=None, times=None):
    """Bit-exact comparison of instance i with one oracle run."""
    st = sim.status()[i] if status is None else status[i]
    assert st == ref.status, f"instance {i}: status {st} vs oracle {ref.status}"
    if st != 0:
        return
    t = sim.time()[i] if times is None else times[i]
    assert t == ref.time, f"instance {i}: time {t} vs oracle {ref.time}"
    assert sim.node_tokens(i) == ref.node_tokens(), f"instance {i}: final tokens differ"
    for sid in range(ref.num_snapshots):
        done = ref.complete(sid)
        tick = sim.snapshot_tick(sid, i)
        assert (tick >= 0) == done, f"instance {i} snapshot {sid}: completion differs"
        if not done:
            continue
        assert tick == ref.completion_tick(sid), f"instance {i} snapshot {sid}: completion tick"
        got = sim.CollectSnapshot(sid, instance=i)
        want = ref.collect(sid)
        assert got.tokenMap == want.tokens, f"instance {i} snapshot {sid}: tokens {got.tokenMap} vs {want.tokens}"
        assert canonical(got.messages) == canonical(want.messages), \
            f"instance {i} snapshot {sid}: messages {got.messages} vs {want.messages}"


def oracle_batch(top, events, n, seed_base=O.REFERENCE_SEED, threads=8, schedule=None, draws=0):
    return O.run_batch(top if "\n" in top else read_text(top),
                       events if "\n" in events else read_text(events), n, sched=schedule,
                       draws=draws, seed_base=seed_base, threads=threads)


def batch_sums_from_oracle(status, counters, hashes):
    ok = status == 0
    return {
        "instances": len(status),
        "ok": int(ok.sum()),
        "fatal": int(((status == 1) | (status == 2)).sum()),
        "delivered": int((counters[ok, 2] + counters[ok, 3]).sum()),
        "snapshot_hash": int(np.uint64(hashes[ok].sum(dtype=np.uint64)).astype(np.int64)),
        "completed": int(counters[ok, 6].sum()),
    }
