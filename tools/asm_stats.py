"""Instruction mix, spill sites and loop back-edges of one kernel in build/cl_kernels.s.

usage: python tools/asm_stats.py [asm] [kernel-substring]   (default: the D=3 staged exec kernel)
"""
import re
import sys
from collections import Counter

asm = sys.argv[1] if len(sys.argv) > 1 else "chandy-lamport-distributed-snapshot-algorithm_amd/build/cl_kernels.s"
pat = sys.argv[2] if len(sys.argv) > 2 else "cl_exec_kernelILi3ELb1ELb0E"
lines = open(asm).read().split("\n")
start = next(i for i, l in enumerate(lines) if pat in l and l.endswith(":") or (pat in l and ": ; @" in l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for n, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = n
cls = Counter()
ops = Counter()
for l in body:
    t = l.strip().split()
    if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
        continue
    ops[t[0]] += 1
    k = t[0]
    cls["valu" if k.startswith("v_") else "salu" if k.startswith("s_") and not k.startswith(("s_load", "s_buffer", "s_cbranch", "s_branch", "s_waitcnt")) else
        "branch" if "branch" in k else "lds" if k.startswith("ds_") else "vmem" if k.startswith(("global_", "buffer_", "scratch_", "flat_")) else
        "smem" if k.startswith(("s_load", "s_buffer")) else "wait" if k.startswith("s_waitcnt") else "other"] += 1
print(f"{len(body)} lines; static mix: {dict(cls)}")
for k, v in ops.most_common(40):
    print(f"  {k:28s} {v}")
print("back-edges (branch to an earlier label):")
for n, l in enumerate(body):
    m = re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)
    if m and labels.get(m.group(1), 1 << 30) < n:
        print(f"  {labels[m.group(1)]:5d} <- {n:5d} {l.strip()}")
print("spill / scratch sites:")
for n, l in enumerate(body):
    if "scratch_" in l or "buffer_store" in l or "buffer_load" in l or "v_writelane" in l and False:
        print(f"  {n:5d} {l.strip()}")
