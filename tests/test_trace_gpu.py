"""Device event trace (the reference's debug Logger, logger.go:12-76) vs the oracle's
Logger restatement (oracle/cl_oracle.c log_event), record for record.

Parity here is against the oracle only: the reference's tests never check the log
(snapshot_test.go:29 only prints it under `debug`), so no reference fixture pins it."""
import importlib

import numpy as np
import pytest

import oracle as O
from enginecheck import engine_run
from snapcheck import read_text
from test_gpu_parity import _random_scenario

cl = importlib.import_module("chandy-lamport-distributed-snapshot-algorithm_amd")

SCENARIOS = [
    ("2nodes.top", "2nodes-simple.events"),
    ("2nodes.top", "2nodes-message.events"),
    ("3nodes.top", "3nodes-simple.events"),
    ("3nodes.top", "3nodes-bidirectional-messages.events"),
    ("8nodes.top", "8nodes-sequential-snapshots.events"),
    ("8nodes.top", "8nodes-concurrent-snapshots.events"),
    ("10nodes.top", "10nodes.events"),
]


def oracle_log(top, events, seed):
    ref = O.OracleSim()
    ref.seed_go(seed)
    assert ref.read_topology_text(top if "\n" in top else read_text(top)) == 0
    ref.log_enable()
    ref.read_events_text(events if "\n" in events else read_text(events), O.MAX_DRAIN_TICKS)
    return ref


def traced_run(top, events, n, traced, capacity=8192):
    sim = engine_run(top, events, n, flush=False)
    sim.trace_enable(0, traced, capacity)
    sim.flush()
    return sim


def check_instances(sim, top, events, traced):
    status = sim.status()
    for i in range(traced):
        ref = oracle_log(top, events, O.REFERENCE_SEED + i)
        if status[i] != ref.status:
            raise AssertionError(f"instance {i}: status {status[i]} vs oracle {ref.status}")
        got, want = sim.trace(i), ref.log()
        assert len(got) == len(want), f"instance {i}: {len(got)} records vs oracle {len(want)}"
        for k, (g, w) in enumerate(zip(got, want)):
            assert g == w, f"instance {i} record {k}: {g} vs oracle {w}"


@pytest.mark.gpu
@pytest.mark.parametrize("top,events", SCENARIOS)
def test_trace_matches_oracle_logger(top, events):
    """The 7 reference scenarios, 32 traced instances of a 256-instance batch."""
    sim = traced_run(top, events, 256, 32)
    check_instances(sim, top, events, 32)


@pytest.mark.gpu
def test_trace_pretty_print_golden_run():
    """Instance 0 of 2nodes-message (the golden seed): the PrettyPrint text restates
    logger.go:55-64 / common.go:75-122 on the oracle's log."""
    sim = traced_run("2nodes.top", "2nodes-message.events", 64, 1)
    ref = oracle_log("2nodes.top", "2nodes-message.events", O.REFERENCE_SEED)
    text = sim.pretty_print(0)
    ids = ref.node_ids()
    assert text.startswith("Time 0:\n")
    n_lines = sum(2 if k in (cl.LOG_SENT_TOKEN, cl.LOG_RECV_TOKEN, cl.LOG_START) else 1 for _, k, *_ in ref.log())
    n_epochs = len({e for e, *_ in ref.log()})
    assert text.count("\n") == n_lines + n_epochs
    first = ref.log()[0]
    assert f"\t{ids[first[2]]} has {first[5]} token(s)\n" in text


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_trace_random_scenarios(seed):
    """Random digraphs: multi-source receivers (several Received records per node per
    tick), overlapping snapshots, data-dependent fatals (the unknown-dest record is
    logged before the exit, the insufficient-tokens one is not)."""
    rng = np.random.default_rng(100 + seed)
    top, events = _random_scenario(rng, int(rng.integers(2, 15)), int(rng.integers(5, 60)))
    sim = traced_run(top, events, 128, 48)
    check_instances(sim, top, events, 48)


@pytest.mark.gpu
def test_trace_off_by_default_and_results_unchanged():
    """Tracing changes no snapshot result: traced and untraced batches agree."""
    top, events = "8nodes.top", "8nodes-concurrent-snapshots.events"
    a = engine_run(top, events, 512)
    b = traced_run(top, events, 512, 16)
    assert (a.status() == b.status()).all() and (a.time() == b.time()).all()
    assert (a.checksums() == b.checksums()).all()
    with pytest.raises(cl.ClSnapError):
        a.trace(0)


@pytest.mark.gpu
def test_trace_overflow_reports_limit():
    sim = traced_run("10nodes.top", "10nodes.events", 64, 2, capacity=16)
    with pytest.raises(cl.ClSnapError):
        sim.trace(0)
