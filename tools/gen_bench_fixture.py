"""Generate tests/golden/bench_sums.json: the oracle's batch checksums for the bench batches.

bench.py compares the all-reduced checksums of its timed batch with these values and
prints "parity": true/false in its line; tests/test_bench_fixture.py re-derives them.
The values come from the CPU oracle (oracle/cl_oracle.c, pinned by the reference's 21
golden snapshots), run here over EVERY instance of each batch: instance i uses Go's
rand.Seed(REFERENCE_SEED + i) delay stream (snapshot_test.go:20).

usage: python tools/gen_bench_fixture.py [threads]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

TEST_DATA = os.path.join(ROOT, "tests", "golden", "test_data")
BATCHES = {
    # BASELINE.json configs[2]: the north_star's 2^20-instance batch
    "c3": ("8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20),
    # BASELINE.json configs[1]
    "c2": ("10nodes.top", "10nodes.events", 65536),
}


def batch_sums(status, counters, hashes):
    """The CL_SUM_* values the oracle can state (include/clsnap.h); hash sum mod 2^64 as int64."""
    ok = status == 0
    return {
        "instances": int(status.size),
        "ok": int(ok.sum()),
        "fatal": int(((status == 1) | (status == 2)).sum()),
        "other": int((~ok & (status != 1) & (status != 2)).sum()),
        "delivered": int((counters[ok, 2] + counters[ok, 3]).sum()),
        "snapshot_hash": int(np.uint64(hashes[ok].sum(dtype=np.uint64)).astype(np.int64)),
        "completed": int(counters[ok, 6].sum()),
        "recorded": int(counters[ok, 4].sum()),
        "cut_residual": 0,
        "final_residual": 0,
    }


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    out = {"generator": "tools/gen_bench_fixture.py (CPU oracle, oracle/cl_oracle.c)",
           "seed_base": O.REFERENCE_SEED, "batches": {}}
    for cfg, (top, events, n) in BATCHES.items():
        t_text = open(os.path.join(TEST_DATA, top)).read()
        e_text = open(os.path.join(TEST_DATA, events)).read()
        t0 = time.time()
        _, st, _, cnt, h = O.run_batch_prepared(t_text, e_text, n, seed_base=O.REFERENCE_SEED, threads=threads)
        out["batches"][cfg] = {"top": top, "events": events, "instances": n,
                               "sums": batch_sums(st, cnt, h)}
        print(cfg, n, f"{time.time() - t0:.1f}s", out["batches"][cfg]["sums"])
    with open(os.path.join(ROOT, "tests", "golden", "bench_sums.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
