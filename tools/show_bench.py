import json
import sys
for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().split("\n")[-1])
        print(f, f"{d['value']:.4g} pkt/s", f"step {d['ms_per_step']:.4f} ms", f"kernel {d['roofline']['kernel_ms']:.4f} ms",
              f"frac {d['roofline']['frac']:.4f}", d["status"], d["checks"]["cut_residual"], d["checks"]["final_residual"])
    except Exception as e:  # noqa
        print(f, "unreadable:", e)
