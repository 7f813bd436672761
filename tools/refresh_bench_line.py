"""Fill a batch-engine bench line's roofline.traffic / roofline.valu from the committed PMC
summary of the same build (profiles/<round>_<cfg>_pmc.json), as bench.py does when that
file exists at bench time -- for lines measured in the same GPU call as the PMC passes that
produced the summary.

usage: python tools/refresh_bench_line.py <bench.json> <cfg> > profiles/<round>_bench_<cfg>.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (constants and profile lookup only)

path, cfg = sys.argv[1], sys.argv[2]
lines = [ln for ln in open(path) if ln.lstrip().startswith("{")]
d = json.loads(lines[-1])
prof = bench.profile_entry(cfg, d["config"]["instances_per_gpu"])
if prof is not None:
    p, doc, scale = prof
    c = {k: (v * scale if k != "SQ_WAVE_CYCLES" and k != "GRBM_GUI_ACTIVE" else v) for k, v in doc["counters"].items()}
    r = d["roofline"]
    kms = r["kernel_ms"]
    # raw bytes (the exec kernels' reads are not wide coalesced streams: tools/traffic_model.py)
    r["traffic"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    r["traffic_detail"] = {"raw": r["traffic"], "fetch_doubled": (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024,
                           "write": c["WRITE_SIZE"] * 1024, "used": "raw", "source": os.path.relpath(p, ROOT)}
    rate = c["SQ_INSTS_VALU"] / (kms * 1e-3)
    r["valu"] = {"achieved": rate, "peak": bench.VALU_PEAK, "unit": "wave64 VALU instr/s",
                 "frac": rate / bench.VALU_PEAK, "insts_per_launch": c["SQ_INSTS_VALU"],
                 "source": os.path.relpath(p, ROOT),
                 "waves_per_simd": 4 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8) / bench.SIMDS}
print(json.dumps(d))
