"""What a replay plan's length order is worth, and whether a fresh launch could predict it.

Runs the CPU oracle over the C3 bench batch (8nodes-concurrent, instance i seeded
REFERENCE_SEED + i) and reports, from every instance's final tick:
  - wave-ticks per wave (the longest of each wave's 8 instances) in launch order and in
    length order, against the mean instance length (the floor of any schedule);
  - the R^2 of a least-squares fit of the final tick on the instance's delay row (the
    97 Go rand.Intn(5) draws), on a held-out half of a 2^17-instance sample.
usage: python tools/length_model.py [instances]   (default 2^20; ~5 s of oracle time on 8 threads)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

TD = os.path.join(ROOT, "tests", "golden", "test_data")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    top = open(os.path.join(TD, "8nodes.top")).read()
    ev = open(os.path.join(TD, "8nodes-concurrent-snapshots.events")).read()
    _, st, ticks, _, _ = O.run_batch_prepared(top, ev, n, threads=os.cpu_count() or 1, want_hash=False)
    t = ticks.astype(np.float64)
    ipw = 8
    m = n // ipw * ipw
    print(f"instances {n}: mean final tick {t.mean():.2f}, fatal {(st != 0).mean():.4f}")
    print(f"wave-ticks per wave: launch order {t[:m].reshape(-1, ipw).max(1).mean():.2f}, "
          f"length order {np.sort(t[:m])[::-1].reshape(-1, ipw).max(1).mean():.2f}")
    k = min(n, 1 << 17)
    X = np.stack([O.go_intn(O.REFERENCE_SEED + i, 5, 97) for i in range(k)]).astype(np.float64)
    A = np.hstack([X, np.ones((k, 1))])
    tr = k // 2
    w, *_ = np.linalg.lstsq(A[:tr], t[:tr], rcond=None)
    p = A[tr:k] @ w
    r2 = 1 - ((p - t[tr:k]) ** 2).mean() / t[tr:k].var()
    pred = np.argsort(-p)
    print(f"final tick ~ delay row (linear, held-out half of {k}): R^2 {r2:.3f}; "
          f"predicted-order wave-ticks {t[tr:k][pred][: (k - tr) // ipw * ipw].reshape(-1, ipw).max(1).mean():.2f}")


if __name__ == "__main__":
    main()
