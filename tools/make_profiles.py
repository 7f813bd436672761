"""Turn a gpurun_out/pmc_<cfg> directory into committed profile summaries.

usage: python tools/make_profiles.py <round> <cfg> [instances] [timed steps] [dispatches per step] [dir suffix]
(reads gpurun_out/pmc_<cfg><dir suffix>, the directory tools/gpu_pmc.sh wrote with SUFFIX=...)
writes profiles/<round>_<cfg>_kernel_stats.csv  (rocprofv3 --kernel-trace --stats)
       profiles/<round>_<cfg>_pmc.json          (per-dispatch PMC means, timed dispatches)
       profiles/traffic_<cfg>.json              (HBM bytes per launch for bench.py)
HBM bytes: FETCH_SIZE/WRITE_SIZE are KB; both raw and fetch-doubled figures are written
(tools/traffic_model.py: the doubling is for wide coalesced streaming reads only).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the exec kernels: node-parallel, and the instance-per-lane kernels compiled at run time
KERNELS = ("cl_exec_kernel", "clsnap_lanes")
KERNEL = " + ".join(KERNELS)


def is_exec(name):
    return any(k in name for k in KERNELS)


def per_dispatch(paths):
    vals = collections.defaultdict(dict)  # counter -> dispatch -> value
    for p in paths:
        for r in csv.DictReader(open(p)):
            if not is_exec(r["Kernel_Name"]):
                continue
            d = int(r["Dispatch_Id"])
            vals[r["Counter_Name"]][d] = vals[r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
    return vals


def main():
    rnd, cfg = sys.argv[1], sys.argv[2]
    inst = int(sys.argv[3]) if len(sys.argv) > 3 else {"c2": 65536, "c3": 1 << 20}[cfg]
    src = os.path.join(ROOT, "gpurun_out", f"pmc_{cfg}" + (sys.argv[6] if len(sys.argv) > 6 else ""))
    out = os.environ.get("OUT_DIR") or os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, "trace", "p_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{rnd}_{cfg}_kernel_stats.csv"))
    # one step = every exec-kernel dispatch of one rerun: split replays dispatch the spill-free
    # and the spill-capable kernels concurrently.  Counters are summed over the timed steps'
    # dispatches (the last steps * per_step of the pass) and divided by the steps; the active
    # GPU cycles (GRBM_GUI_ACTIVE) of concurrent dispatches overlap, so the step's maximum.
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    per_step = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    summary = {}
    for name, per in per_dispatch(glob.glob(os.path.join(src, "pass*", "p_counter_collection.csv"))).items():
        ds = sorted(per)[-steps * per_step:]
        groups = [ds[k:k + per_step] for k in range(0, len(ds), per_step)]
        agg = max if name == "GRBM_GUI_ACTIVE" else sum
        summary[name] = sum(agg(per[d] for d in g) for g in groups) / len(groups)
    with open(os.path.join(out, f"{rnd}_{cfg}_pmc.json"), "w") as f:
        json.dump({"kernel": KERNEL, "config": cfg, "instances": inst, "dispatches_per_step": per_step,
                   "note": "per timed step (sum over its exec-kernel dispatches; GRBM_GUI_ACTIVE the "
                           "max); SQ_* cycle counters are quad-cycles",
                   "counters": summary}, f, indent=1, sort_keys=True)
    if "FETCH_SIZE" in summary and "WRITE_SIZE" in summary:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import traffic_model as tm
        raw, cor, just = tm.bytes_both(summary["FETCH_SIZE"], summary["WRITE_SIZE"], tm.streaming("cl_exec_kernel"))
        with open(os.path.join(out, f"traffic_{cfg}.json"), "w") as f:
            json.dump({"config": cfg, "instances": inst, "fifo_slots": 0,
                       "hbm_bytes_per_launch": just, "raw_bytes_per_launch": raw,
                       "corrected_bytes_per_launch": cor, "fetch_correction": False,
                       "reason": tm.reason("cl_exec_kernel"), "fetch_kb": summary["FETCH_SIZE"],
                       "write_kb": summary["WRITE_SIZE"], "round": rnd}, f, indent=1)
    for row in csv.DictReader(open(stats)):
        if is_exec(row["Name"]):
            print(cfg, "avg kernel ns", row["AverageNs"], "calls", row["Calls"])
    print(json.dumps({k: round(v) for k, v in sorted(summary.items())}))


if __name__ == "__main__":
    main()
