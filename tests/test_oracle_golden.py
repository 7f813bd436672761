"""The oracle is pinned before anything is checked against it (CPU only).

* Go math/rand restatement vs Go's published known answers and the reference seed's
  stream (tests/golden/go_rng_kat.json).
* The regenerated rngCooked table vs its SHA-256 / first / last entries.
* All 7 reference tests (snapshot_test.go:46-108) with their 21 golden snapshots,
  token conservation (checkTokens) and the structural counts of SURVEY.md section 6.
"""
import hashlib
import json
import os

import pytest

import oracle as O
from snapcheck import (ROOT, TEST_DATA, assert_equal, check_tokens, read_snapshot_file,
                       read_text, scenarios)

KAT = json.load(open(os.path.join(ROOT, "tests", "golden", "go_rng_kat.json")))


def test_go_rand_seed1_known_answers():
    assert O.go_int63(1, 3).tolist() == KAT["seed1_int63"]
    assert O.go_intn(1, 100, 10).tolist() == KAT["seed1_intn100"]


def test_go_rand_reference_seed_stream():
    assert O.go_int63(KAT["refseed"], 3).tolist() == KAT["refseed_int63"]
    s = "".join(str(v) for v in O.go_intn(KAT["refseed"], 5, 200).tolist())
    assert s == KAT["refseed_intn5_200"]


def test_rng_cooked_table():
    with open(os.path.join(ROOT, "tests", "golden", "go_rng_cooked.txt")) as f:
        text = f.read().rstrip("\n")
    vals = [int(v) for v in text.split("\n")]
    assert len(vals) == 607
    assert vals[:4] == KAT["cooked_first4"] and vals[606] == KAT["cooked_last"]
    assert hashlib.sha256(text.encode()).hexdigest() == KAT["cooked_sha256"]


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s["name"])
def test_reference_goldens(sc):
    sim = O.OracleSim()
    sim.seed_go(O.REFERENCE_SEED)          # rand.Seed(seed + 1)
    assert sim.read_topology(os.path.join(TEST_DATA, sc["top"])) == 0
    assert sim.read_events(os.path.join(TEST_DATA, sc["events"])) == 0
    assert sim.num_snapshots == len(sc["snaps"])
    actual = []
    for sid in range(sim.num_snapshots):
        snap = sim.collect(sid)
        actual.append((snap.id, snap.tokens, snap.messages))
    check_tokens(sim.node_tokens(), actual)
    expected = sorted((read_snapshot_file(f) for f in sc["snaps"]), key=lambda s: s[0])
    for e, a in zip(expected, actual):
        assert_equal(e, a)
    c = sim.counters()
    assert sim.time == sc["ticks"]
    assert c["draws"] == c["push"] == sc["draws"]
    assert c["peek"] == sc["peek"]
    assert c["pop_tok"] == sc["pop_tok"] and c["pop_mk"] == sc["pop_mk"]
    assert c["recorded"] == sc["recorded"]
    assert c["completed"] == len(sc["snaps"])


def test_golden_mutation_is_detected():
    """A wrong delay stream must break the 10-node goldens (the fixtures really pin it)."""
    sim = O.OracleSim()
    sim.seed_go(O.REFERENCE_SEED + 1)
    sim.read_topology(os.path.join(TEST_DATA, "10nodes.top"))
    sim.read_events(os.path.join(TEST_DATA, "10nodes.events"))
    mismatches = 0
    for i in range(10):
        e = read_snapshot_file(f"10nodes{i}.snap")
        s = sim.collect(i)
        try:
            assert_equal(e, (s.id, s.tokens, s.messages))
        except AssertionError:
            mismatches += 1
    assert mismatches > 0


def test_fatal_insufficient_tokens():
    sim = O.OracleSim()
    sim.add_node("N1", 1)
    sim.add_node("N2", 0)
    sim.add_link("N1", "N2")
    assert sim.send_tokens("N1", "N2", 2) == O.FATAL_INSUFFICIENT_TOKENS
    assert sim.status == O.FATAL_INSUFFICIENT_TOKENS


def test_fatal_unknown_dest_and_hang():
    sim = O.OracleSim()
    sim.add_node("A", 5)
    sim.add_node("B", 0)
    sim.add_link("A", "B")
    assert sim.send_tokens("B", "A", 0) == O.FATAL_UNKNOWN_DEST
    sim2 = O.OracleSim()
    sim2.add_node("A", 5)
    sim2.add_node("B", 0)
    sim2.add_link("A", "B")          # A has no in-links: a snapshot at A never completes
    rc, sid = sim2.start_snapshot("A")
    assert rc == 0 and sid == 0
    for _ in range(50):
        sim2.tick()
    assert not sim2.complete(0)


def test_logger_restatement_simple_run():
    """The oracle's Logger (logger.go:12-76) on 2nodes-simple at the golden seed, derived
    by hand from the reference source: StartSnapshotRecord + the broadcast at time 0
    (sim.go:109, node.go:100), N1's first marker at time 4 (sim.go:86, node.go:100,
    sim.go:127: N1 has one in-link, so it completes at once), N2's closing marker at 7."""
    ref = O.OracleSim()
    ref.seed_go(O.REFERENCE_SEED)
    assert ref.read_topology_text(read_text("2nodes.top")) == 0
    ref.log_enable()
    ref.read_events_text(read_text("2nodes-simple.events"))
    # (epoch, kind, node rank, other rank, data, nodeTokens); ranks: N1 = 0, N2 = 1
    assert ref.log() == [(0, 4, 1, -1, 0, 0), (0, 1, 1, 0, 0, 0),
                         (4, 3, 0, 1, 0, 1), (4, 1, 0, 1, 0, 1), (4, 5, 0, -1, 0, 1),
                         (7, 3, 1, 0, 0, 0), (7, 5, 1, -1, 0, 0)]


@pytest.mark.parametrize("sc", scenarios(), ids=lambda s: s["name"])
def test_logger_counts_match_counters(sc):
    """Every scenario: one Received record per delivery, one Sent record per push, one
    StartSnapshotRecord per snapshot, N EndSnapshotRecords per completed snapshot."""
    ref = O.OracleSim()
    ref.seed_go(O.REFERENCE_SEED)
    assert ref.read_topology_text(read_text(sc["top"])) == 0
    ref.log_enable()
    ref.read_events_text(read_text(sc["events"]))
    log, c = ref.log(), ref.counters()
    kinds = [r[1] for r in log]
    assert kinds.count(2) + kinds.count(3) == c["pop_tok"] + c["pop_mk"]
    assert kinds.count(0) + kinds.count(1) == c["push"]
    assert kinds.count(4) == ref.num_snapshots
    n = len(ref.node_ids())
    assert kinds.count(5) >= n * c["completed"]
    assert [r[0] for r in log] == sorted(r[0] for r in log)  # epochs never go back
