"""The bench parity fixture (tests/golden/bench_sums.json) re-derived from the CPU oracle.

bench.py compares the checksums of its timed batch with this file; here the file is
checked against a fresh oracle run of every instance of each batch."""
import json
import os

import oracle as O
from snapcheck import ROOT, TEST_DATA

FIXTURE = os.path.join(os.path.dirname(TEST_DATA), "bench_sums.json")


def test_fixture_matches_oracle():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_bench_fixture import batch_sums
    fx = json.load(open(FIXTURE))
    assert fx["seed_base"] == O.REFERENCE_SEED
    for cfg, b in fx["batches"].items():
        t = open(os.path.join(TEST_DATA, b["top"])).read()
        e = open(os.path.join(TEST_DATA, b["events"])).read()
        _, st, _, cnt, h = O.run_batch_prepared(t, e, b["instances"], threads=os.cpu_count() or 1)
        assert batch_sums(st, cnt, h) == b["sums"], cfg


def test_prepared_runner_equals_parsing_runner():
    """The cpu_baseline's prepared runner (parse once, reset per instance) computes the
    same per-instance results as the runner that parses every instance's files."""
    import numpy as np
    for top, ev in (("8nodes.top", "8nodes-concurrent-snapshots.events"), ("10nodes.top", "10nodes.events"),
                    ("3nodes.top", "3nodes-bidirectional-messages.events")):
        t = open(os.path.join(TEST_DATA, top)).read()
        e = open(os.path.join(TEST_DATA, ev)).read()
        a = O.run_batch(t, e, 3000, threads=4)
        b = O.run_batch_prepared(t, e, 3000, threads=3)
        for x, y in zip(a[1:], b[1:]):
            assert np.array_equal(x, y)
