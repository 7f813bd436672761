"""Generate tests/golden/graph_runs.json: exact summaries of C5-shaped graph runs that
the CPU oracle needs minutes for (too slow to run inside a GPU test).

Each run is tests/graphcheck.py's powerlaw_program (BASELINE config 5's shape: 8
Zipf(0.9) targets + ring, continuous unit-token traffic, one snapshot start per tick),
followed by readEventsFile's drain (test_common.go:123-137) so that every snapshot
completes.  The summary (graphcheck.run_summary) holds status, time, the reference
counters, every completion tick, a content digest per snapshot (token map + per-channel
recorded payloads) and a digest of the final node tokens; tests/test_graph_gpu.py
compares the engine's summary of the same run with it.

usage: python tools/gen_graph_fixture.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from graphcheck import oracle_program, oracle_summary, powerlaw_program  # noqa: E402

RUNS = {
    # name: (nodes, traffic/snapshot window in ticks, snapshots)
    "c5_shape_20k_256": (20000, 300, 256),
}


def main():
    out = {"generator": "tools/gen_graph_fixture.py (CPU oracle, oracle/cl_oracle.c)", "runs": {}}
    for name, (n, steps, snaps) in RUNS.items():
        p = powerlaw_program(n, steps, snaps, fifo_slots=512)
        t0 = time.time()
        o = oracle_program(p, drain=True, max_drain=100000)
        summ = oracle_summary(o)
        out["runs"][name] = {"nodes": n, "steps": steps, "snapshots": snaps, "fifo_slots": 512,
                             "max_drain": 100000, "summary": summ}
        print(name, f"{time.time() - t0:.0f}s", summ["status"], summ["time"], summ["counters"])
    with open(os.path.join(ROOT, "tests", "golden", "graph_runs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
