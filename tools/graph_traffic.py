"""HBM bytes per graph-engine run from the gpu_pmc_graph.sh passes -> profiles/traffic_<cfg>.json.

usage: python tools/graph_traffic.py <cfg> <nodes> <ticks> [drain]
(env PMCG_DIR: the passes' directory, default gpurun_out/pmcg_<cfg>; OUT_DIR: default profiles/)
A run is k_reset + the tick kernels (k_hostops, k_tally, k_pick, k_marker, k_scan, k_push);
the post-run checks (k_finish, k_checks_*) are excluded.  Runs = k_reset dispatches.
Bytes: raw (FETCH_SIZE + WRITE_SIZE) KB and fetch-doubled, per kernel, with the justified
one (tools/traffic_model.py) as hbm_bytes_per_launch."""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUN_KERNELS = {"k_reset", "k_sn_reset", "k_hostops", "k_tally", "k_pick", "k_marker", "k_scan", "k_push",
               "k_drain_begin", "k_drain_ctl", "k_drain_end"}


def sums(pattern):
    tot = collections.Counter()
    per_kernel = collections.Counter()
    resets = set()
    for p in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(p)):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            if not m or m.group(1) not in RUN_KERNELS:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            per_kernel[m.group(1)] += float(r["Counter_Value"])
            if m.group(1) == "k_reset":
                resets.add(r["Dispatch_Id"])
    return tot, len(resets), per_kernel


cfg, nodes, ticks = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
base = os.environ.get("PMCG_DIR") or os.path.join(ROOT, "gpurun_out", f"pmcg_{cfg}")
drain = len(sys.argv) > 4 and sys.argv[4] == "drain"
f, runs_f, fk = sums(os.path.join(base, "pass3", "**", "*counter_collection.csv"))
w, runs_w, wk = sums(os.path.join(base, "pass4", "**", "*counter_collection.csv"))
assert runs_f and runs_w, "no k_reset dispatches found"
fetch_kb = f["FETCH_SIZE"] / runs_f
write_kb = w["WRITE_SIZE"] / runs_w
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import traffic_model as tm  # noqa: E402
per = {}
for k in sorted(set(fk) | set(wk)):
    r, co, j = tm.bytes_both(fk[k] / runs_f, wk[k] / runs_w, tm.streaming(k))
    per[k] = {"raw": r, "corrected": co, "justified": j, "fetch_correction": tm.streaming(k), "reason": tm.reason(k)}
out = {"config": cfg, "nodes": nodes, "steps": ticks, "drain": drain, "runs_profiled": runs_f,
       "fetch_kb_per_run": fetch_kb, "write_kb_per_run": write_kb,
       "raw_bytes_per_launch": sum(v["raw"] for v in per.values()),
       "corrected_bytes_per_launch": sum(v["corrected"] for v in per.values()),
       "hbm_bytes_per_launch": sum(v["justified"] for v in per.values()),
       "per_kernel": per,
       "per_kernel_fetch_kb_per_run": {k: fk[k] / runs_f for k in sorted(fk)},
       "per_kernel_write_kb_per_run": {k: wk[k] / runs_w for k in sorted(wk)},
       "note": "one launch = one full run of the tick pipeline; raw = (FETCH_SIZE + WRITE_SIZE) KB, corrected = "
               "(2 FETCH_SIZE + WRITE_SIZE) KB (the guide's gfx950 factor, for wide coalesced streaming reads only); "
               "per kernel the justified figure is raw unless its reads are such streams (tools/traffic_model.py)"}
out_dir = os.environ.get("OUT_DIR") or os.path.join(ROOT, "profiles")
os.makedirs(out_dir, exist_ok=True)
json.dump(out, open(os.path.join(out_dir, f"traffic_{cfg}.json"), "w"), indent=1)
print(json.dumps(out))
