"""GPU parity: the gfx950 engine against the reference goldens and the CPU oracle.

All comparisons are bit-exact (integer simulation): statuses, simulator time, final node
tokens, snapshot completion ticks, snapshot token maps and per-channel recorded
message sequences.  Full-size batches (BASELINE configs 2 and 3 per GPU) are checked
through batch checksums against the oracle's own full-batch run plus sampled
instance-by-instance comparisons.
"""
import os

import numpy as np
import pytest

import oracle as O
from enginecheck import (batch_sums_from_oracle, canonical, cl, compare_instance, engine_run,
                         new_sim, oracle_batch, oracle_run)
from snapcheck import TEST_DATA, assert_equal, check_tokens, read_snapshot_file, scenarios

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s["name"])
def test_reference_goldens_and_neighbours(sc):
    """Instance 0 uses the reference seed: it must reproduce the golden files exactly.
    Instances 1..255 use seeds +1..+255 and must match the oracle bit for bit."""
    n = 256
    sim = engine_run(sc["top"], sc["events"], n)
    status = sim.status()
    assert status[0] == 0
    actual = []
    for sid in range(sim.num_snapshots):
        s = sim.CollectSnapshot(sid, 0)
        actual.append((s.id, s.tokenMap, [m.astuple() for m in s.messages]))
    check_tokens(sim.node_tokens(0), actual)
    expected = sorted((read_snapshot_file(f) for f in sc["snaps"]), key=lambda s: s[0])
    assert len(expected) == len(actual)
    for e, a in zip(expected, actual):
        assert_equal(e, a)
    assert sim.time()[0] == sc["ticks"]
    times = sim.time()
    for i in range(n):
        compare_instance(sim, i, oracle_run(sc["top"], sc["events"], seed=O.REFERENCE_SEED + i),
                         status=status, times=times)


def test_counters_match_oracle():
    sc = [s for s in scenarios() if s["name"] == "Test8NodesConcurrentSnapshots"][0]
    n = 2048
    sim = engine_run(sc["top"], sc["events"], n)
    _, st, ticks, cnt, _ = oracle_batch(sc["top"], sc["events"], n)
    got = sim.counters(only_ok=False)
    assert got["push"] == cnt[:, 0].sum()
    assert got["peek"] == cnt[:, 1].sum()
    assert got["pop_tok"] == cnt[:, 2].sum()
    assert got["pop_mk"] == cnt[:, 3].sum()
    assert got["ticks"] == ticks.sum()
    ok = st == 0
    got_ok = sim.counters(only_ok=True)
    assert got_ok["recorded"] == cnt[ok, 4].sum()
    assert got_ok["completed"] == cnt[ok, 6].sum()


def _checksums(sim):
    return dict(zip(cl.SUM_NAMES, sim.checksums().tolist()))


@pytest.mark.parametrize("cfg", [("10nodes.top", "10nodes.events", 65536),
                                 ("8nodes.top", "8nodes-concurrent-snapshots.events", 131072)],
                         ids=["C2_10nodes_x65536", "C3_8nodes_concurrent_x131072"])
def test_full_batch_checksums(cfg):
    """BASELINE configs at full per-GPU size: checksum of checksums vs the oracle's run
    of every instance, plus conservation properties and sampled exact comparisons."""
    top, events, n = cfg
    sim = engine_run(top, events, n)
    sums = _checksums(sim)
    _, st, ticks, cnt, hashes = oracle_batch(top, events, n, threads=16)
    want = batch_sums_from_oracle(st, cnt, hashes)
    for k, v in want.items():
        assert sums[k] == v, f"{k}: engine {sums[k]} vs oracle {v}"
    assert sums["cut_residual"] == 0          # every snapshot is a consistent cut
    assert sums["final_residual"] == 0        # checkTokens (test_common.go:298-328)
    status = sim.status()
    assert np.array_equal(status, st)
    assert np.array_equal(sim.time()[st == 0], ticks[st == 0])
    rng = np.random.default_rng(7)
    sample = np.concatenate([[0, n - 1], rng.choice(n, 48, replace=False), np.nonzero(st != 0)[0][:16]])
    times = sim.time()
    for i in sample:
        compare_instance(sim, int(i), oracle_run(top, events, seed=O.REFERENCE_SEED + int(i)),
                         status=status, times=times)


def test_fifo_spill_to_hbm():
    """Two LDS slots per channel force deep channels through the HBM spill ring."""
    top, events, n = "10nodes.top", "10nodes.events", 4096
    sim = engine_run(top, events, n, fifo_lds_slots=2)
    _, st, ticks, cnt, hashes = oracle_batch(top, events, n)
    sums = _checksums(sim)
    want = batch_sums_from_oracle(st, cnt, hashes)
    for k, v in want.items():
        assert sums[k] == v
    for i in (0, 1, 17, 4095):
        compare_instance(sim, i, oracle_run(top, events, seed=O.REFERENCE_SEED + i))


def test_explicit_schedule_matches_oracle():
    top, events, n = "8nodes.top", "8nodes-concurrent-snapshots.events", 512
    rng = np.random.default_rng(3)
    sched = rng.integers(0, 5, size=(n, 97), dtype=np.uint8)
    sim = engine_run(top, events, n, schedule=sched)
    status, times = sim.status(), sim.time()
    for i in range(0, n, 7):
        compare_instance(sim, i, oracle_run(top, events, schedule=sched[i]), status=status, times=times)


def test_delay_exhausted():
    top, events, n = "3nodes.top", "3nodes-simple.events", 64
    sched = np.zeros((n, 4), dtype=np.uint8)  # 10 draws needed
    sim = engine_run(top, events, n, schedule=sched)
    assert (sim.status() == cl.INST_DELAY_EXHAUSTED).all()
    ref = oracle_run(top, events, schedule=sched[0])
    assert ref.status == O.DELAY_EXHAUSTED


def test_incremental_flush_equals_one_shot():
    """Flushing after every event (state saved/restored through HBM) == one launch."""
    top = "8nodes.top"
    lines = open(os.path.join(TEST_DATA, "8nodes-concurrent-snapshots.events")).read().split("\n")
    n = 256
    a = engine_run(top, "8nodes-concurrent-snapshots.events", n)
    b = new_sim(n)
    b.read_topology_file(os.path.join(TEST_DATA, top))
    for line in lines:
        if not line:
            continue
        f = line.split()
        if f[0] == "send":
            b.ProcessEvent(cl.PassTokenEvent(f[1], f[2], int(f[3])))
        elif f[0] == "snapshot":
            b.ProcessEvent(cl.SnapshotEvent(f[1]))
        else:
            b.Tick(int(f[1]) if len(f) > 1 else 1)
        b.flush()
    b.drain()
    b.flush()
    assert np.array_equal(a.status(), b.status())
    assert np.array_equal(a.time(), b.time())
    assert np.array_equal(a.checksums(), b.checksums())


def test_hang_and_unknown_dest():
    top = "3\nA 5\nB 5\nC 0\nA B\nB C\nC B\n"      # A has no in-links
    sim = engine_run(top, "snapshot A\ntick 3\n", 64, max_drain_ticks=200)
    assert (sim.status() == cl.INST_HANG).all()
    ref = oracle_run(top, "snapshot A\ntick 3\n", seed=O.REFERENCE_SEED, max_drain=200)
    assert ref.status == O.HANG
    sim2 = engine_run(top, "send A B 1\nsend A C 1\ntick\n", 64)
    assert (sim2.status() == cl.INST_FATAL_UNKNOWN_DEST).all()
    sim3 = engine_run(top, "send C B 1\n", 64)
    assert (sim3.status() == cl.INST_FATAL_INSUFFICIENT_TOKENS).all()


def _random_scenario(rng, n_nodes, n_events):
    ids = [f"N{k}" for k in range(1, n_nodes + 1)]   # lexicographic != numeric order (N10 < N2)
    tokens = {i: int(rng.integers(0, 30)) for i in ids}
    edges = set()
    for k in range(n_nodes):                          # a ring keeps every node reachable
        edges.add((ids[k], ids[(k + 1) % n_nodes]))
    for _ in range(int(rng.integers(0, 3 * n_nodes))):
        a, b = rng.choice(ids, 2, replace=False)
        edges.add((str(a), str(b)))
    top = f"{n_nodes}\n" + "".join(f"{i} {tokens[i]}\n" for i in ids) + "".join(f"{a} {b}\n" for a, b in sorted(edges))
    ev = []
    snaps = 0
    out = {}
    for a, b in edges:
        out.setdefault(a, []).append(b)
    for _ in range(n_events):
        r = rng.random()
        if r < 0.6:
            a = str(rng.choice(ids))
            b = str(rng.choice(out[a]))
            ev.append(f"send {a} {b} {int(rng.integers(0, 4))}")
        elif r < 0.75 and snaps < 12:
            ev.append(f"snapshot {rng.choice(ids)}")
            snaps += 1
        else:
            ev.append(f"tick {int(rng.integers(1, 4))}")
    return top, "\n".join(ev) + "\n"


@pytest.mark.parametrize("seed", range(12))
def test_random_scenarios(seed):
    """Random digraphs (up to 14 nodes, multi-source receivers, overlapping snapshots,
    data-dependent fatals) against the oracle."""
    rng = np.random.default_rng(100 + seed)
    top, events = _random_scenario(rng, int(rng.integers(2, 15)), int(rng.integers(5, 60)))
    n = 128
    sim = engine_run(top, events, n, fifo_lds_slots=4)
    status, times = sim.status(), sim.time()
    for i in range(n):
        compare_instance(sim, i, oracle_run(top, events, seed=O.REFERENCE_SEED + i),
                         status=status, times=times)


@pytest.mark.parametrize("seed,tlo,thi", [(0, 4, 8), (3, 4, 8), (1, 3, 7), (2, 3, 7)])
def test_send_groups_with_midgroup_fatals(seed, tlo, thi):
    """Event lines of sends from distinct senders run as one lane-parallel group
    (OP_SENDS).  Low balances make delay-dependent insufficient-token fatals land in the
    middle of groups (about 40% of the instances): every instance must freeze exactly
    where the sequential reference does (status and frozen node balances), and OK
    instances must match exactly."""
    rng = np.random.default_rng(500 + seed)
    n_nodes = int(rng.integers(3, 12))
    ids = [f"N{k}" for k in range(1, n_nodes + 1)]
    top = f"{n_nodes}\n" + "".join(f"{i} {int(rng.integers(tlo, thi))}\n" for i in ids)
    top += "".join(f"{ids[k]} {ids[(k + 1) % n_nodes]}\n{ids[k]} {ids[(k - 1) % n_nodes]}\n"
                   for k in range(n_nodes))
    ev = []
    for r in range(12):
        order = rng.permutation(n_nodes)
        for k in order[: int(rng.integers(2, n_nodes + 1))]:
            ev.append(f"send {ids[k]} {ids[(k + int(rng.integers(0, 2)) * 2 - 1) % n_nodes]} 1")
        if r % 3 == 0:
            ev.append(f"snapshot {ids[int(rng.integers(0, n_nodes))]}")
        ev.append("tick 3")
    events = "\n".join(ev) + "\n"
    n = 256
    sim = engine_run(top, events, n)
    status, times = sim.status(), sim.time()
    assert (status == cl.INST_FATAL_INSUFFICIENT_TOKENS).any() and (status == cl.INST_OK).any()
    for i in range(n):
        ref = oracle_run(top, events, seed=O.REFERENCE_SEED + i)
        compare_instance(sim, i, ref, status=status, times=times)
        if status[i] == cl.INST_FATAL_INSUFFICIENT_TOKENS:
            assert sim.node_tokens(i) == ref.node_tokens(), f"instance {i}: frozen balances differ"


@pytest.mark.parametrize("cfg", [("10nodes.top", "10nodes.events", 65536, None),
                                 ("8nodes.top", "8nodes-concurrent-snapshots.events", 131072, None),
                                 ("10nodes.top", "10nodes.events", 4096, 2),
                                 ("8nodes.top", "8nodes-concurrent-snapshots.events", 8192, 2)],
                         ids=["C2_x65536", "C3_x131072", "C2_spill_x4096", "C3_spill_x8192"])
def test_rerun_equals_flush_and_oracle(cfg):
    """The benchmark's timed path: cl_rerun replays the program from the initial state
    with the kernel prologue resetting completion ticks and HBM spill-ring heads (no fill
    launch).  Three reruns after the first flush must reproduce the flush and the oracle
    exactly -- statuses, times, batch checksums, and sampled instances in full.  Every
    output plane is poisoned before each rerun, so a rerun that skipped (or only partly
    made) its stores would fail."""
    top, events, n, slots = cfg
    sim = engine_run(top, events, n, fifo_lds_slots=slots)
    first = (sim.status().copy(), sim.time().copy(), sim.checksums().copy())
    # the replay plan of the flush (the probe): instances that spilled run last, on the
    # spill-capable kernel, the rest spill-free -- with two LDS slots, deep channels spill
    spilled, split = sim.replay_split()
    assert 0 <= spilled <= n and (split == 0 or n - spilled - 64 < split <= n - spilled)
    if slots == 2:
        assert spilled > 0 and not sim.spill_free_replays()
    if 0 < spilled < n - 64:
        assert sim.mapped_replays() and split > 0
    if n == 131072 and slots is None:  # C3: instance lengths spread (13..50 ticks): mapped replays
        assert sim.mapped_replays()
    _, st, ticks, cnt, hashes = oracle_batch(top, events, n, threads=16)
    want = batch_sums_from_oracle(st, cnt, hashes)
    # the poison reaches every plane the results are read from: without a rerun, nothing
    # the flush wrote survives
    sim.poison_outputs()
    assert not np.array_equal(sim.checksums(), first[2])
    assert not np.array_equal(sim.status(), first[0]) and not np.array_equal(sim.time(), first[1])
    for r in range(3):
        sim.poison_outputs()      # results below can only come from this rerun
        sim.rerun()
        sim.synchronize()
        assert sim.replay_split() == (spilled, split), f"rerun {r}: plan"
        status, times, sums = sim.status(), sim.time(), sim.checksums()
        assert np.array_equal(status, first[0]) and np.array_equal(status, st), f"rerun {r}: status"
        assert np.array_equal(times, first[1]), f"rerun {r}: times"
        assert np.array_equal(times[st == 0], ticks[st == 0]), f"rerun {r}: times vs oracle"
        assert np.array_equal(sums, first[2]), f"rerun {r}: checksums"
        got = dict(zip(cl.SUM_NAMES, sums.tolist()))
        for k, v in want.items():
            assert got[k] == v, f"rerun {r} {k}: engine {got[k]} vs oracle {v}"
        assert got["cut_residual"] == 0 and got["final_residual"] == 0
    rng = np.random.default_rng(11)
    for i in np.concatenate([[0, n - 1], rng.choice(n, 24, replace=False)]):
        compare_instance(sim, int(i), oracle_run(top, events, seed=O.REFERENCE_SEED + int(i)),
                         status=status, times=times)


def test_wait_snapshot_after_back_to_back_split_reruns():
    """back-to-back split reruns leave the spill-capable half running on the
    second stream, whose prologue resets completion ticks.  A collector's cl_wait_snapshot
    (and cl_poll_snapshot) must join that stream before reading them: the wait returns at
    once (CL_E_NOT_COMPLETE because some instances stopped FATAL, with every completed
    instance counted) instead of waiting out its timeout on ticks of instances still
    being replayed."""
    import ctypes
    import time
    top, events, n = "8nodes.top", "8nodes-concurrent-snapshots.events", 8192
    sim = engine_run(top, events, n, fifo_lds_slots=2)
    spilled, split = sim.replay_split()
    assert spilled > 0 and split > 0 and (sim.status() != cl.INST_OK).any()
    want = [sim.poll_snapshot(sid) for sid in range(sim.num_snapshots)]
    for sid in range(sim.num_snapshots):
        sim.rerun()
        sim.rerun()   # back to back: no join of the second stream in between
        v = ctypes.c_int64(-1)
        timeout_ms = 20_000
        t0 = time.perf_counter()
        rc = sim._L.cl_wait_snapshot(sim._h, sid, 0, n, timeout_ms, ctypes.byref(v))
        waited = time.perf_counter() - t0
        # returning at once, not after the timeout (half of it: room for a slow box)
        assert rc == cl.E_NOT_COMPLETE and v.value == want[sid] and waited < timeout_ms / 2000, \
            (sid, rc, v.value, want[sid], waited)
        sim.rerun()
        assert sim.poll_snapshot(sid) == want[sid]


def test_replay_plan_spill_free_and_split():
    """The first full run of a program is the probe: per-instance spill flags and final
    ticks.  A program that never spills replays wholly on the spill-free kernel; one in which
    some instances spill replays split -- the slot map puts the spilling instances last, the
    clean whole waves run spill-free and the rest on the spill-capable kernel, concurrently
    -- and appending events invalidates the plan until the next full run.  Every launch
    equals the flush and the oracle; output planes are poisoned before every rerun."""
    # A->B carries a send and two markers (depth bound 3 > 2 LDS slots: spill rings are
    # provisioned), but the ticks between them keep at most one packet queued
    top = "3\nA 10\nB 10\nC 10\nA B\nB C\nC A\nB A\n"
    ev = "send A B 2\ntick 6\nsnapshot A\ntick 6\nsnapshot B\n"
    n = 512
    sim = new_sim(n, fifo_lds_slots=2)
    sim.read_topology_text(top)
    sim.read_events_text(ev)
    sim.flush()
    first = (sim.status().copy(), sim.time().copy(), sim.checksums().copy())
    assert sim.spill_free_replays() and sim.replay_split() == (0, 0)
    for i in range(0, n, 37):
        compare_instance(sim, i, oracle_run(top, ev, seed=O.REFERENCE_SEED + i), status=first[0], times=first[1])
    for _ in range(2):
        sim.poison_outputs()
        sim.rerun()
        sim.synchronize()
        assert np.array_equal(sim.status(), first[0]) and np.array_equal(sim.time(), first[1])
        assert np.array_equal(sim.checksums(), first[2])
    ev2 = "send A B 1\nsend A B 1\nsend A B 1\nsend A B 1\nsend A B 1\ntick 1\n"
    sim.read_events_text(ev2)
    assert not sim.spill_free_replays() and sim.replay_split() == (-1, 0)   # (not run in full yet)
    sim.rerun()                   # the new program's probe: every instance spills, no split
    sim.synchronize()
    assert sim.replay_split() == (n, 0)
    ref = new_sim(n, fifo_lds_slots=2)  # the same two readEventsFile calls, one flush
    ref.read_topology_text(top)
    ref.read_events_text(ev)
    ref.read_events_text(ev2)
    ref.flush()
    assert np.array_equal(sim.status(), ref.status()) and np.array_equal(sim.time(), ref.time())
    assert np.array_equal(sim.checksums(), ref.checksums())
    # random delays on 8nodes-concurrent with two LDS slots: some instances spill, most not
    top3, ev3, n3 = "8nodes.top", "8nodes-concurrent-snapshots.events", 4096
    sim3 = engine_run(top3, ev3, n3, fifo_lds_slots=2)
    spilled, split = sim3.replay_split()
    assert 0 < spilled < n3 - 64 and split > 0 and sim3.mapped_replays()
    base = (sim3.status().copy(), sim3.time().copy(), sim3.checksums().copy())
    for _ in range(2):
        sim3.poison_outputs()
        sim3.rerun()
        sim3.synchronize()
        assert np.array_equal(sim3.status(), base[0]) and np.array_equal(sim3.time(), base[1])
        assert np.array_equal(sim3.checksums(), base[2])
    _, st, ticks, cnt, hashes = oracle_batch(top3, ev3, n3)
    want = batch_sums_from_oracle(st, cnt, hashes)
    got = dict(zip(cl.SUM_NAMES, base[2].tolist()))
    for k, v in want.items():
        assert got[k] == v, k
    for i in (0, 1, 77, 1234, n3 - 1):
        compare_instance(sim3, i, oracle_run(top3, ev3, seed=O.REFERENCE_SEED + i), status=base[0], times=base[1])


def test_headline_batch_2p20_matches_fixture():
    """The north_star batch itself (BASELINE config 3, 2^20 instances on one GPU): the
    batch checksums of a flush and of a rerun equal the oracle's values over every
    instance (tests/golden/bench_sums.json, tools/gen_bench_fixture.py); the rerun's outputs
    are poisoned beforehand, so they come from the rerun alone."""
    import json
    fx = json.load(open(os.path.join(os.path.dirname(TEST_DATA), "bench_sums.json")))
    want = fx["batches"]["c3"]["sums"]
    n = fx["batches"]["c3"]["instances"]
    assert n == 1 << 20 and fx["seed_base"] == O.REFERENCE_SEED
    sim = engine_run("8nodes.top", "8nodes-concurrent-snapshots.events", n)
    for rnd in range(2):
        got = dict(zip(cl.SUM_NAMES, sim.checksums().tolist()))
        got["recorded"] = sim.counters(only_ok=True)["recorded"]
        for k in want:
            assert (got[k] - want[k]) % (1 << 64) == 0, f"pass {rnd} {k}: engine {got[k]} vs oracle {want[k]}"
        sim.poison_outputs()      # the next pass reads only what the rerun wrote
        sim.rerun()
        sim.synchronize()


def test_headline_batch_fresh_path_matches_fixture():
    """The fresh path on the north_star batch: the FIRST launch of a new sim is
    a rerun with no replay plan (the whole batch, unordered, on the spill-capable kernel) and
    its batch checksums equal the oracle's over every instance (tests/golden/bench_sums.json).
    The replays after it, through the plan that first run built (length order, split between
    the spill-free and spill-capable kernels), agree too."""
    import json
    fx = json.load(open(os.path.join(os.path.dirname(TEST_DATA), "bench_sums.json")))
    want = fx["batches"]["c3"]["sums"]
    n = fx["batches"]["c3"]["instances"]
    sim = new_sim(n, seed_base=O.REFERENCE_SEED)
    sim.read_topology_file(os.path.join(TEST_DATA, "8nodes.top"))
    sim.read_events_file(os.path.join(TEST_DATA, "8nodes-concurrent-snapshots.events"))
    sim.rerun()                    # the first launch: nothing derived from a prior run
    sim.synchronize()
    spilled, split = sim.replay_split()       # (the plan that first run built)
    assert spilled > 0 and split > 0           # the replays below run split
    for rnd in range(2):
        got = dict(zip(cl.SUM_NAMES, sim.checksums().tolist()))
        got["recorded"] = sim.counters(only_ok=True)["recorded"]
        for k in want:
            assert (got[k] - want[k]) % (1 << 64) == 0, f"pass {rnd} {k}: engine {got[k]} vs oracle {want[k]}"
        sim.poison_outputs()
        sim.rerun()                # a replay through the plan
        sim.synchronize()


def test_two_event_texts_and_snapshot_after_drain():
    """Two readEventsFile calls on one batch, then a snapshot after the last drain and
    more ticks: every instance equals the oracle running the same calls; a rerun
    replays the whole program identically."""
    top = "4\nA 10\nB 10\nC 10\nD 10\nA B\nB C\nC D\nD A\nB A\nC B\n"
    ev1 = "send A B 3\nsnapshot A\ntick 2\nsend C D 1\n"
    ev2 = "snapshot C\nsend B A 2\ntick 3\nsnapshot D\n"
    n = 128
    sim = new_sim(n)
    sim.read_topology_text(top)
    sim.read_events_text(ev1)
    sim.flush()
    sim.read_events_text(ev2)
    sim.StartSnapshot("B")
    sim.Tick(12)
    sim.flush()
    first = (sim.status().copy(), sim.time().copy(), sim.checksums().copy())
    refs = []
    for i in range(n):
        o = O.OracleSim()
        o.seed_go(O.REFERENCE_SEED + i)
        assert o.read_topology_text(top) == 0
        if o.read_events_text(ev1) == 0 and o.read_events_text(ev2) == 0:
            o.start_snapshot("B")
            for _ in range(12):
                o.tick()
        refs.append(o)
        compare_instance(sim, i, o, status=first[0], times=first[1])
    sim.poison_outputs()
    sim.rerun()
    sim.synchronize()
    assert np.array_equal(sim.status(), first[0]) and np.array_equal(sim.time(), first[1])
    assert np.array_equal(sim.checksums(), first[2])


def test_packed_collect_equals_host_expansion_and_oracle():
    """CollectSnapshot packed on the GPU (cl_collect_snapshot_packed: node records expanded
    over the channels' token histories into one CSR over (instance, channel), finalizeSnapshot
    node.go:188-195 / CollectSnapshot sim.go:134-173) equals the host expansion of each
    instance's records (cl_collect_snapshot) and the oracle, on the C3 batch: every snapshot,
    a sub-range that starts mid-batch, and totals that match the recorded-copy counter."""
    top, events, n = "8nodes.top", "8nodes-concurrent-snapshots.events", 65536
    sim = engine_run(top, events, n)
    status = sim.status()
    ids, chans = sim.node_ids(), sim.channels()
    C = len(chans)
    total = 0
    rng = np.random.default_rng(5)
    sample = np.concatenate([[0, 1, n - 1], rng.choice(n, 40, replace=False), np.nonzero(status != 0)[0][:8]])
    refs = {int(i): oracle_run(top, events, seed=O.REFERENCE_SEED + int(i)) for i in sample}
    for sid in range(sim.num_snapshots):
        tok, done, off, msg = sim.collect_snapshot_packed(sid)
        assert off[0] == 0 and np.all(np.diff(off) >= 0) and off[-1] == msg.size
        total += msg.size
        ticks = np.array([sim.snapshot_tick(sid, int(i)) for i in sample])
        assert np.array_equal(done[sample], ticks >= 0)
        for i, t in zip(sample, ticks):
            i = int(i)
            if t < 0:
                assert (tok[i] == -1).all() and off[i * C] == off[(i + 1) * C]
                continue
            g = sim.CollectSnapshot(sid, i)                    # host expansion of the records
            assert dict(zip(ids, tok[i].tolist())) == g.tokenMap
            got = {}
            for c in range(C):
                for k in range(off[i * C + c], off[i * C + c + 1]):
                    got.setdefault((ids[chans[c][0]], ids[chans[c][1]]), []).append(int(msg[k]))
            assert got == canonical(g.messages)
            ref = refs[i]
            if ref.status == 0 or ref.complete(sid):
                w = ref.collect(sid)
                assert g.tokenMap == w.tokens and canonical(g.messages) == canonical(w.messages)
        # a sub-range equals the same slice of the whole-batch CSR
        lo, hi = 12345, 40000
        t2, d2, o2, m2 = sim.collect_snapshot_packed(sid, lo, hi)
        assert np.array_equal(t2, tok[lo:hi]) and np.array_equal(d2, done[lo:hi])
        assert np.array_equal(o2, off[lo * C:hi * C + 1] - off[lo * C])
        assert np.array_equal(m2, msg[off[lo * C]:off[hi * C]])
        rt, rd, ro, rm = sim.collect_snapshot_range(sid, lo, hi)    # the int64 form
        assert np.array_equal(rt, t2) and np.array_equal(rd, d2) and np.array_equal(ro, o2)
        assert np.array_equal(rm, m2)
    assert total == sim.counters(only_ok=False)["recorded"]
    assert sim.collect_time() > 0


def test_uneven_fan_out_runtime_loop_kernel():
    """a hub with 10 out-links (degree bound 16: the run-time-loop kernel with its
    heads in LDS) next to leaves of in-degree <= 2 -- marker broadcasts at the hub must touch
    only its own channels' heads.  1-4 overlapping snapshots, sends from the hub."""
    leaves = [f"L{k}" for k in range(10)]
    top = f"{len(leaves) + 1}\nH 40\n" + "".join(f"{x} 5\n" for x in leaves)
    top += "".join(f"H {x}\n" for x in leaves)
    top += "".join(f"{leaves[k]} {leaves[(k + 1) % 10]}\n" for k in range(10)) + "L0 H\n"
    for n_snap in (1, 2, 4):
        ev = []
        for r in range(n_snap):
            ev += [f"send H {leaves[(3 * r) % 10]} 2", f"snapshot {'H' if r % 2 == 0 else leaves[r]}",
                   f"send L{r} L{r + 1} 1", "tick 2"]
        events = "\n".join(ev) + "\n"
        n = 512
        sim = engine_run(top, events, n)
        status, times = sim.status(), sim.time()
        assert (status == cl.INST_OK).all()
        for i in range(n):
            compare_instance(sim, i, oracle_run(top, events, seed=O.REFERENCE_SEED + i),
                             status=status, times=times)
