"""GPU parity of the graph engine (include/clgraph.h) against the reference goldens and
the CPU oracle.  All comparisons are bit-exact: status, simulator time, final node
tokens, snapshot completion ticks, token maps, per-channel recorded messages, and the
reference-level counters (pushes = delay draws, peeks, delivered tokens / markers,
recorded copies, completed snapshots).

At BASELINE config 4's full size (2^20-node regular digraph, one snapshot under
continuous traffic) the benchmark's exact program is compared with the CPU oracle's
full-size run (tests/golden/graph_runs.json c4_full), and checked through
size-independent properties: the snapshot completes, its cut is consistent (snapshot
tokens + recorded messages = total), final tokens + in-flight tokens = total, and
reruns into poisoned result planes reproduce the run.
"""
import os

import numpy as np
import pytest

import graphgen as G
import oracle as O
from graphcheck import (clg, cl, compare, digest_from_oracle, engine_program, engine_summary, oracle_program,
                        powerlaw_program, program_files, regular_program, scenario_engine, scenario_oracle, Program)
from snapcheck import assert_equal, check_tokens, read_snapshot_file, scenarios

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s["name"])
def test_reference_goldens(sc):
    """The reference's own test_data runs (reference seed) reproduce the golden files."""
    g = scenario_engine(sc["top"], sc["events"], O.REFERENCE_SEED)
    assert g.status() == 0
    actual = []
    for sid in range(g.num_snapshots):
        s = g.CollectSnapshot(sid)
        actual.append((s.id, s.tokenMap, [m.astuple() for m in s.messages]))
    check_tokens(g.node_tokens(), actual)
    expected = sorted((read_snapshot_file(f) for f in sc["snaps"]), key=lambda s: s[0])
    assert len(expected) == len(actual)
    for e, a in zip(expected, actual):
        assert_equal(e, a)
    assert g.time() == sc["ticks"]
    c = g.counters()
    assert (c["push"], c["peek"], c["pop_tok"], c["pop_mk"], c["recorded"]) == \
        (sc["draws"], sc["peek"], sc["pop_tok"], sc["pop_mk"], sc["recorded"])


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s["name"])
def test_scenarios_other_seeds_vs_oracle(sc):
    """Other Go seeds: fatal and hang statuses included, everything bit-exact."""
    for i in range(1, 17):
        seed = O.REFERENCE_SEED + 1000 * i
        compare(scenario_engine(sc["top"], sc["events"], seed), scenario_oracle(sc["top"], sc["events"], seed))


@pytest.mark.parametrize("n,steps,seed", [(64, 60, 1), (1000, 80, 2), (4096, 90, 3)])
def test_regular_traffic_vs_oracle(n, steps, seed):
    """C4-shaped runs (8-out regular digraph, continuous traffic, snapshots) at sizes the
    oracle runs in seconds."""
    p = regular_program(n, steps=steps, seed=seed, snaps=((5, None), (5, 0), (17, None), (30, None)))
    g = engine_program(p)
    o = oracle_program(p)
    assert o.status == 0
    compare(g, o)
    sums = g.checksums()
    assert sums["cut_residual"] == 0 and sums["final_residual"] == 0
    assert sums["digest"] == digest_from_oracle(o)


def test_regular_one_thread_per_node_push_vs_oracle():
    """A 2^18-node graph: k_push runs one thread per node (graphs below 2^18 nodes use 8
    lanes per node), bit-exact against the oracle over 25 traffic steps (~2.5M pushes)."""
    p = regular_program(1 << 18, steps=25, seed=4, snaps=((5, None), (5, 0), (17, None)))
    g = engine_program(p)
    o = oracle_program(p)
    assert o.status == 0
    compare(g, o)
    assert g.checksums()["digest"] == digest_from_oracle(o)


@pytest.mark.parametrize("lanes", [0, 1, 4])
@pytest.mark.parametrize("n,steps,snaps", [(300, 300, 8), (300, 300, 24), (1500, 400, 48)])
def test_powerlaw_overlapping_snapshots_vs_oracle(n, steps, snaps, lanes):
    """C5-shaped runs: skewed in-degree hub, one snapshot start per tick, long
    recording logs, most snapshots still in flight at the end.  lanes forces the push
    kernel's one-thread-per-node path (1) or its 4-lane path (4); 0 = automatic."""
    p = powerlaw_program(n, steps, snaps, fifo_slots=512)
    g = engine_program(p, lanes=lanes)
    o = oracle_program(p)
    compare(g, o)
    assert g.checksums()["digest"] == digest_from_oracle(o)


def _random_graph(rng, n):
    m = int(rng.integers(n, 4 * n))
    return rng.integers(0, n, m).astype(np.int32), rng.integers(0, n, m).astype(np.int32)


def _random_events_run(rng, n, src, dst, gseed, n_events, drain=500, tokens=(0, 50),
                       link_sends=False, lanes=0):
    ids = [f"n{r}" for r in rng.permutation(n)]
    top = f"{n}\n" + "".join(f"{ids[r]} {int(rng.integers(*tokens))}\n" for r in range(n)) + \
        "".join(f"{ids[a]} {ids[b]}\n" for a, b in zip(src, dst))
    ev = []
    for _ in range(n_events):
        x = rng.random()
        if x < 0.45:
            a, b = int(rng.integers(0, n)), int(rng.integers(0, n))
            if link_sends:  # an existing channel: no unknown-dest fatal
                e = int(rng.integers(0, len(src)))
                a, b = int(src[e]), int(dst[e])
            ev.append(f"send {ids[a]} {ids[b]} {int(rng.integers(0, 8))}")
        elif x < 0.6:
            ev.append(f"snapshot {ids[int(rng.integers(0, n))]}")
        else:
            ev.append(f"tick {int(rng.integers(1, 4))}")
    events = "\n".join(ev) + "\n"
    o = O.OracleSim()
    o.seed_go(gseed)
    assert o.read_topology_text(top) == 0
    o.read_events_text(events, drain)
    if os.environ.get("CG_ORACLE_ONLY"):  # sizing aid on a CPU host
        return o
    g = clg.GraphSim(max_drain_ticks=drain)
    g.set_push_lanes(lanes)
    g.read_topology_text(top)
    g.set_delay_go_seed(gseed)
    g.read_events_text(events)
    g.flush()
    compare(g, o)
    return o


@pytest.mark.parametrize("seed", range(12))
def test_random_host_events_vs_oracle(seed):
    """Random digraphs with host sends of arbitrary sizes (payload history), snapshots
    at random nodes, ticks, fatals (insufficient tokens, unknown dest) -- string API and
    Go delay stream, exactly like readEventsFile."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 30))
    src, dst = _random_graph(rng, n)
    _random_events_run(rng, n, src, dst, O.REFERENCE_SEED + seed, int(rng.integers(5, 40)))


@pytest.mark.parametrize("kind", ["insufficient", "unknown_dest", "none"])
def test_large_send_group_with_late_fatal_vs_oracle(kind):
    """A run of 700 sends from pairwise distinct senders executes as one parallel send
    group over three 256-thread blocks (k_sg_check / k_sg_apply).  The first failing send
    (program order) sits in the last block: every earlier send must run, none after it,
    and the draw index must advance by exactly the sends that ran (node.go:112-131,
    sim.go:101) -- however the blocks are scheduled."""
    n = 720
    rng = np.random.default_rng(41)
    ids = [f"v{r:03d}" for r in range(n)]
    tok = [5] * n
    order = [int(x) for x in rng.permutation(n)[:700]]
    bad = order[600]
    if kind == "insufficient":
        tok[bad] = 0
    top = f"{n}\n" + "".join(f"{ids[r]} {tok[r]}\n" for r in range(n)) + \
        "".join(f"{ids[r]} {ids[(r + 1) % n]}\n{ids[r]} {ids[(r - 1) % n]}\n" for r in range(n))
    ev = ["tick"]
    for v in order:
        dest = ids[(v + 1) % n]
        if kind == "unknown_dest" and v == bad:
            dest = ids[(v + 7) % n]             # no such link
        ev.append(f"send {ids[v]} {dest} 1")
    ev += ["snapshot v000", "tick 3"] + [f"send {ids[v]} {ids[(v - 1) % n]} 1" for v in order[:300]] + ["tick 2"]
    events = "\n".join(ev) + "\n"
    gseed = O.REFERENCE_SEED + 5
    o = O.OracleSim()
    o.seed_go(gseed)
    assert o.read_topology_text(top) == 0
    o.read_events_text(events, 2000)
    want = {"insufficient": 1, "unknown_dest": 2, "none": 0}[kind]
    assert o.status == want
    for _ in range(3):                           # (block scheduling varies run to run)
        g = clg.GraphSim(max_drain_ticks=2000)
        g.read_topology_text(top)
        g.set_delay_go_seed(gseed)
        g.read_events_text(events)
        g.flush()
        compare(g, o)


@pytest.mark.parametrize("lanes", [0, 1, 4])
@pytest.mark.parametrize("n,deg,seed", [(24, 23, 0), (70, 40, 1), (100, 62, 2)])
def test_high_out_degree_vs_oracle(n, deg, seed, lanes):
    """Dense digraphs: broadcasts over out-degrees up to 62 (k_push pushes them in chunks
    of 8 channels: multi-chunk and partial tail chunks), and one pick block whose
    out-channels exceed k_pick's LDS stage (3,072 head words; n=70/100 have 2,800 /
    6,200), so the fallback reads HBM.  Both push paths (lanes 1 and 4) are forced."""
    rng = np.random.default_rng(100 + seed)
    src = np.repeat(np.arange(n), deg)
    dst = np.concatenate([rng.choice(np.delete(np.arange(n), v), deg, replace=False) for v in range(n)])
    _random_events_run(rng, n, src.astype(np.int32), dst.astype(np.int32), O.REFERENCE_SEED + 77 + seed, 60,
                       drain=4000, tokens=(100, 200), link_sends=True, lanes=lanes)


@pytest.mark.parametrize("lanes", [1, 4])
def test_hub_expansion_both_push_paths_vs_oracle(lanes):
    """Power-law hubs with in-degree > 64 (the grid-wide expansion of k_push<1>) and
    nodes of out-degree 9-10 (a partial second chunk), on both push paths."""
    p = powerlaw_program(2000, 250, 16, seed=5, fifo_slots=512)
    assert np.bincount(p.dst).max() > 64
    g = engine_program(p, lanes=lanes)
    o = oracle_program(p)
    compare(g, o)
    assert g.checksums()["digest"] == digest_from_oracle(o)


def test_two_event_texts_and_snapshot_after_drain_vs_oracle():
    """Two readEventsFile calls on one simulator (test_common.go:79-140 twice): the
    second drain waits only for the snapshots started before it.  Then a rerun after
    more events were appended (snapshot after the last drain, more ticks) replays the
    whole program identically to the incremental run and to the oracle."""
    top = "4\nA 10\nB 10\nC 10\nD 10\nA B\nB C\nC D\nD A\nB A\nC B\n"
    ev1 = "send A B 3\nsnapshot A\ntick 2\nsend C D 1\n"
    ev2 = "snapshot C\nsend B A 2\ntick 3\nsnapshot D\n"
    for seed in range(6):
        gseed = O.REFERENCE_SEED + 31 * seed
        o = O.OracleSim()
        o.seed_go(gseed)
        assert o.read_topology_text(top) == 0
        assert o.read_events_text(ev1) == 0 and o.read_events_text(ev2) == 0
        g = clg.GraphSim()
        g.read_topology_text(top)
        g.set_delay_go_seed(gseed)
        g.read_events_text(ev1)
        g.flush()                    # incremental: first file executed on its own
        g.read_events_text(ev2)
        g.flush()
        compare(g, o)
        one = clg.GraphSim()         # both files in one flush
        one.read_topology_text(top)
        one.set_delay_go_seed(gseed)
        one.read_events_text(ev1)
        one.read_events_text(ev2)
        one.flush()
        compare(one, o)
        # a snapshot after the last drain, then ticks: incremental == rerun == oracle
        g.StartSnapshot("B")
        g.Tick(12)
        g.flush()
        o.start_snapshot("B")
        for _ in range(12):
            o.tick()
        compare(g, o)
        first = (g.status(), g.time(), g.checksums())
        g.rerun()
        g.synchronize()
        assert (g.status(), g.time(), g.checksums()) == first
        compare(g, o)


def test_hang_freezes_later_ops():
    """A drain that never completes (a node without in-links) is HANG and freezes the
    run: later events do not execute, as in the oracle."""
    top = "3\nA 5\nB 5\nC 0\nA B\nB C\nC B\n"
    o = O.OracleSim()
    o.seed_go(O.REFERENCE_SEED)
    assert o.read_topology_text(top) == 0
    o.read_events_text("snapshot A\ntick 3\n", 50)
    assert o.status == O.HANG
    g = clg.GraphSim(max_drain_ticks=50)
    g.read_topology_text(top)
    g.set_delay_go_seed(O.REFERENCE_SEED)
    g.read_events_text("snapshot A\ntick 3\n")
    g.read_events_text("send B C 1\ntick 4\n")   # after the hang: never executed
    g.flush()
    assert g.status() == cl.INST_HANG
    assert g.time() == o.time
    assert g.node_tokens() == o.node_tokens()


def test_rerun_and_incremental_equal_one_shot():
    p = regular_program(2000, steps=70, seed=9)
    g = engine_program(p)
    first = g.checksums()
    cnt = g.counters()
    for _ in range(3):
        g.rerun()
        g.synchronize()
        assert g.checksums() == first
        assert g.counters() == cnt
    # the same program flushed tick by tick
    h = engine_program(p, run=False)
    inc = clg.GraphSim()
    inc.set_topology(p.tokens, p.src, p.dst, id_width=p.width())
    inc.set_delay_hash(p.delay_seed)
    inc.set_traffic(p.traffic_seed, p.thresh, p.traffic_steps)
    si = 0
    for k in range(p.steps):
        while si < len(p.snap_step) and p.snap_step[si] == k:
            inc.start_snapshot_rank(int(p.snap_rank[si]))
            si += 1
        inc.Tick(1)
        if k % 7 == 3:
            inc.flush()
    inc.flush()
    assert inc.checksums() == first
    assert inc.counters() == cnt
    del h


def test_fifo_overflow_status():
    p = powerlaw_program(300, 200, 24, fifo_slots=2)
    g = engine_program(p)
    assert g.status() == cl.INST_FIFO_OVERFLOW


def test_explicit_schedule_and_exhaustion():
    sc = [s for s in scenarios() if s["name"] == "Test8NodesConcurrentSnapshots"][0]
    from graphcheck import TEST_DATA
    d = cl.go_delay_schedule(O.REFERENCE_SEED + 5, 1, 200)[0]
    for length, want in ((200, None), (20, O.DELAY_EXHAUSTED)):
        g = clg.GraphSim()
        g.read_topology_file(os.path.join(TEST_DATA, sc["top"]))
        g.set_delay_schedule(d[:length])
        g.read_events_file(os.path.join(TEST_DATA, sc["events"]))
        g.flush()
        o = O.OracleSim()
        o.use_schedule(d[:length])
        o.read_topology(os.path.join(TEST_DATA, sc["top"]))
        o.read_events(os.path.join(TEST_DATA, sc["events"]))
        if want is None:
            compare(g, o)
        else:   # engine limit: the run freezes at the failing draw
            assert o.status == want and g.status() == want
            assert g.time() == o.time


def test_c4_full_size_properties():
    """BASELINE config 4 at full size: 2^20 nodes, 8 random permutations, 100 tokens
    each, continuous traffic (p = 1/4), one snapshot at step 5."""
    n, steps = 1 << 20, 80
    g = clg.GraphSim(fifo_slots=16)
    g.generate_regular(n, 8, 100, seed=20240)
    g.set_delay_hash(20241)
    g.set_traffic(20242, 1 << 30, steps)
    for k in range(steps):
        if k == 5:
            g.start_snapshot_rank(G.mulhi(G.counter_hash(20243, 0, 0), n))
        g.Tick(1)
    g.flush()
    assert g.status() == 0
    sums = g.checksums()
    assert sums["completed"] == 1
    assert sums["cut_residual"] == 0 and sums["final_residual"] == 0
    c = g.counters()
    assert c["pop_mk"] == g.num_channels           # one marker per channel
    assert c["push"] == c["pop_tok"] + c["pop_mk"] + sums["in_flight"]  # unit tokens; no marker left
    tok, off, msg = g.collect_arrays(0)
    assert tok.sum() + msg.sum() == 100 * n
    g.rerun()
    g.synchronize()
    assert g.checksums() == sums


def test_c4_full_size_bench_program_vs_oracle_fixture():
    """BASELINE config 4 exactly as bench.py runs it (2^20 nodes, 8-out regular digraph
    from the engine's generator, 80 ticks of traffic, one snapshot at step 5, rank 0's
    seeds): the engine's run summary -- status, time, push / peek / delivered / recorded
    / completed counters, completion tick, snapshot content digest, final token sum and
    hash -- equals the CPU oracle's full-size run (tests/golden/graph_runs.json c4_full,
    tools/gen_graph_fixture.py; sim.go:71-95, node.go:149-185 at scale).  A rerun into
    poisoned result planes must reproduce it too (the benchmark's timed path)."""
    import json
    from graphcheck import bench_program
    from snapcheck import ROOT
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "graph_runs.json")))["runs"]["c4_full"]
    p, cfg = bench_program("c4")
    assert (p.n, p.steps, len(p.snap_step)) == (fx["nodes"], fx["steps"], fx["snapshots"])
    g = clg.GraphSim(fifo_slots=cfg["fifo"], max_snapshots=1, max_drain_ticks=1_000_000)
    g.generate_regular(p.n, cfg["degree"], cfg["tokens"], cfg["seed"])     # bench.py's own path
    g.set_delay_hash(p.delay_seed)
    g.set_traffic(p.traffic_seed, p.thresh, p.traffic_steps)
    for k in range(p.steps):
        if k in p.snap_step:
            g.start_snapshot_rank(int(p.snap_rank[list(p.snap_step).index(k)]))
        g.Tick(1)
    g.flush()
    want = fx["summary"]
    for rnd in range(2):
        got = engine_summary(g)
        for k in want:
            assert got[k] == want[k], f"pass {rnd} {k}: engine {got[k]} vs oracle {want[k]}"
        g.poison_outputs()
        g.rerun()
        g.synchronize()


@pytest.mark.parametrize("lanes", [1, 4])
def test_powerlaw_with_drain_vs_oracle(lanes):
    """C5-shaped run followed by readEventsFile's drain (test_common.go:123-137, on the
    device: k_drain_ctl before every tick): every snapshot completes, bit-exact."""
    p = powerlaw_program(2000, 60, 32, fifo_slots=512)
    g = engine_program(p, lanes=lanes, drain=True)
    o = oracle_program(p, drain=True)
    assert o.status == 0 and all(o.complete(s) for s in range(32))
    compare(g, o)
    assert g.checksums()["digest"] == digest_from_oracle(o)
    g.rerun()
    g.synchronize()
    compare(g, o)


def test_c5_shape_20k_nodes_256_snapshots_vs_oracle_fixture():
    """The largest C5-shaped run the CPU oracle finishes in minutes (20,000 nodes, one
    snapshot start per tick for 256 ticks under traffic, then the drain until all 256
    complete: ~52M delivered packets): the engine's exact run summary equals the
    oracle's (tests/golden/graph_runs.json, tools/gen_graph_fixture.py)."""
    import json
    from snapcheck import ROOT
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "graph_runs.json")))["runs"]["c5_shape_20k_256"]
    p = powerlaw_program(fx["nodes"], fx["steps"], fx["snapshots"], fifo_slots=fx["fifo_slots"])
    g = engine_program(p, drain=True, max_drain=fx["max_drain"])
    want = fx["summary"]
    got = engine_summary(g)
    assert got["status"] == 0 and all(t >= 0 for t in got["ctick"])
    for k in want:
        assert got[k] == want[k], k
    sums = g.checksums()
    assert sums["completed"] == fx["snapshots"] and sums["cut_residual"] == 0 and sums["final_residual"] == 0
    g.poison_outputs()                  # a rerun into poisoned planes reproduces it
    g.rerun()
    g.synchronize()
    got = engine_summary(g)
    for k in want:
        assert got[k] == want[k], f"rerun {k}"


def test_c5_full_size_properties():
    """BASELINE config 5 at full size: 100k-node power-law digraph (8 Zipf(0.9) targets
    + ring), one snapshot start per tick for 4,096 ticks under continuous traffic for
    4,100 ticks, then readEventsFile's drain until all 4,096 snapshots complete (+6).
    Head-of-line scanning in dest order (sim.go:76-90) serializes each sender's marker
    fan-out, so channels hold up to all 4,096 markers (8,192 slots) and the drain runs
    for tens of thousands of ticks."""
    n, steps, snaps = 100_000, 4100, 4096
    g = clg.GraphSim(fifo_slots=8192, max_snapshots=snaps, max_drain_ticks=200_000)
    g.generate_powerlaw(n, 8, 0.9, True, 100, seed=30240)
    g.set_delay_hash(30241)
    g.set_traffic(30242, 1 << 30, steps)
    for k in range(steps):
        if 1 <= k <= snaps:
            g.start_snapshot_rank(G.mulhi(G.counter_hash(30243, k - 1, 1), n))
        g.Tick(1)
    g.drain()
    g.flush()
    assert g.status() == 0
    sums = g.checksums()
    assert sums["completed"] == snaps
    assert sums["final_residual"] == 0 and sums["cut_residual"] == 0
    c = g.counters()
    assert c["pop_mk"] == snaps * g.num_channels       # every marker of every snapshot delivered
    assert c["pop_tok"] + c["pop_mk"] == sums["delivered"]
    assert c["push"] >= sums["delivered"]
    g.rerun()
    g.synchronize()
    assert g.checksums() == sums


def test_event_file_driven_c4_shape_vs_oracle():
    """a C4-shaped workload given as .top / .events files -- one
    `send` line per traffic send (~1,000 per step, run as parallel send groups), the
    snapshots, `tick` lines, then readEventsFile's drain -- read by the engine's
    streaming parsers and by the oracle's readEventsFile restatement: bit-exact."""
    p = regular_program(4096, steps=70, seed=12, snaps=((5, None), (9, 0), (20, None)))
    o = oracle_program(p, log=True)
    top, events = program_files(p, o.log())
    assert events.count("send") > 50_000
    ref = O.OracleSim()
    ref.use_counter_hash(p.delay_seed)
    assert ref.read_topology_text(top) == 0
    assert ref.read_events_text(events) == 0
    g = clg.GraphSim(fifo_slots=p.fifo_slots)
    g.read_topology_text(top)
    g.set_delay_hash(p.delay_seed)
    assert g.read_events_text(events) == 3
    g.flush()
    compare(g, ref)
    assert all(ref.complete(s) for s in range(3))
    assert g.checksums()["digest"] == digest_from_oracle(ref)


def test_event_file_driven_large_equals_synthetic_run():
    """2^18 nodes, 24 steps: the same traffic as send lines (~1.5M, the Logger of the
    synthetic run) replayed from files equals the synthetic device-driven run with its
    drain -- checksums, counters, status, time."""
    p = regular_program(1 << 18, steps=24, seed=14, snaps=((3, None), (4, 0)))
    s = engine_program(p, run=False, drain=True)
    s.trace_enable(1 << 24)
    s.flush()
    top, events = program_files(p, s.trace())
    assert events.count("send") > 1_000_000
    g = clg.GraphSim(fifo_slots=p.fifo_slots)
    g.read_topology_text(top)
    g.set_delay_hash(p.delay_seed)
    g.read_events_text(events)
    g.flush()
    assert g.status() == s.status() == 0 and g.time() == s.time()
    assert g.checksums() == s.checksums()
    assert g.counters() == s.counters()
