"""Per-dispatch view of a graph-engine run: where a kernel's average comes from.

Reads a rocprofv3 `--kernel-trace --output-format csv` kernel_trace.csv and prints, for each
tick kernel (k_pick, k_marker, k_push, k_scan), the dispatch-duration percentiles, the total,
and the share of the total taken by its longest 10 % of dispatches (a per-kernel average over
a C4 run mixes ~75 quiet ticks with the few ticks the snapshot sweeps through).
usage: python tools/tick_profile.py <kernel_trace.csv> [out.json]
"""
import collections
import csv
import json
import sys

KERNELS = ("k_pick", "k_marker", "k_push", "k_scan")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    dur = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        for k in KERNELS:
            if k + "<" in name or k + "I" in name or name.endswith(k):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                break
    # idle time between consecutive dispatches (launch gaps on the one stream)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    gaps = sorted((b[0] - a[1]) / 1e3 for a, b in zip(ev, ev[1:]) if b[0] > a[1])
    out = {}
    if gaps:
        out["gaps"] = {"count": len(gaps), "p50_us": round(gaps[len(gaps) // 2], 2),
                       "p90_us": round(gaps[int(0.9 * len(gaps))], 2), "total_us": round(sum(gaps), 1)}
        print("gaps", json.dumps(out["gaps"]))
    for k in KERNELS:
        d = dur.get(k)
        if not d:
            continue
        s = sorted(d)
        n = len(s)
        top = s[n - max(1, n // 10):]
        pct = lambda q: s[min(n - 1, int(q * n))]
        out[k] = {"dispatches": n, "total_us": round(sum(s), 1), "mean_us": round(sum(s) / n, 2),
                  "p10_us": round(pct(0.1), 2), "p50_us": round(pct(0.5), 2), "p90_us": round(pct(0.9), 2),
                  "max_us": round(s[-1], 2), "top10pct_share": round(sum(top) / sum(s), 3),
                  "longest_in_order": [round(x, 1) for x in d if x >= top[0]][:16]}
        print(k, json.dumps(out[k]))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
