#!/usr/bin/env python3
"""Benchmark: delivered packets/s of the batched Chandy-Lamport engine (BASELINE.json).

A step = one pass of the hot path over one batch: every instance of the batch runs the
whole event program (BASELINE config 2: 10nodes.top + 10nodes.events, 65,536 replicas
per GPU, each with its own Go delay stream) from the initial topology to the end of the
drain (test_common.go:79-140).  Inputs (topology, event program, delay schedule) are
resident in HBM before timing; the timed region is K launches of the exec kernel.

Multi-GPU: one process per GPU, each owning a disjoint instance range (seeds
base + rank * I + i); instances are independent so there is no data-path collective
("scaling": "weak").  RCCL all-reduces the batch checksums once, after timing.

Prints ONE JSON line (rank 0).  See DESIGN.md §6 for the byte model behind "roofline".
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "chandy-lamport-distributed-snapshot-algorithm_amd"
TEST_DATA = os.path.join(ROOT, "tests", "golden", "test_data")

CONFIGS = {
    # BASELINE.json configs[1]: the headline single-GPU workload
    "c2": ("10nodes.top", "10nodes.events", 65536,
           "10nodes.top + 10nodes.events, 65,536 replicas per GPU, Go delay streams"),
    # BASELINE.json configs[2]: 2^20 instances over 8 GPUs = 131,072 per GPU
    "c3": ("8nodes.top", "8nodes-concurrent-snapshots.events", 131072,
           "8nodes.top + 8nodes-concurrent-snapshots.events, 131,072 instances per GPU"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

# BASELINE.json configs[3] and [4]: one large simulation per GPU on the graph engine
# (include/clgraph.h).  Ranks run replicas of the same graph with their own delay,
# traffic and snapshot-placement seeds ("replicas only").
GRAPH_CONFIGS = {
    "c4": dict(kind="regular", n=1 << 20, degree=8, tokens=100, steps=80, snap_steps=[5], fifo=16,
               seed=20240,
               desc="random 8-out regular digraph, 2^20 nodes, one snapshot under continuous token "
                    "traffic (p=1/4 per node per tick), 80 ticks"),
    "c5": dict(kind="powerlaw", n=100_000, targets=8, exponent=0.9, ring=True, tokens=100, steps=4100,
               snap_steps=list(range(1, 4097)), fifo=8192, seed=30240,
               desc="power-law digraph (8 Zipf(0.9) targets + ring), 100k nodes, 4,096 overlapping "
                    "snapshots (one start per tick), 4,100-tick window under continuous traffic"),
}


def b_alg(c, n_nodes):
    """8 push + 8 peek + 8 pop + 4 recorded + 1 draw + 4 N completed."""
    pops = c["pop_tok"] + c["pop_mk"]
    return 8 * c["push"] + 8 * c["peek"] + 8 * pops + 4 * c["recorded"] + 1 * c["push"] \
        + 4 * n_nodes * c["completed"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + sorted(GRAPH_CONFIGS))
    ap.add_argument("--graph-nodes", type=int, default=0, help="override the graph size (c4/c5)")
    ap.add_argument("--graph-steps", type=int, default=0, help="override the tick window (c4/c5)")
    ap.add_argument("--graph-fifo", type=int, default=0, help="override FIFO slots per channel (c4/c5)")
    ap.add_argument("--instances", type=int, default=0, help="instances per GPU (default: config)")
    ap.add_argument("--fifo-slots", type=int, default=0, help="LDS ring slots per channel (0 = automatic)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config in GRAPH_CONFIGS:
        return bench_graph(args, rank, world, local_rank)
    top, events, per_gpu, desc = CONFIGS[args.config]
    if args.instances:
        per_gpu = args.instances

    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    cl = importlib.import_module(PKG)
    cldist = importlib.import_module(PKG + ".dist")
    _, seed_base = cldist.shard(per_gpu, rank, cl.REFERENCE_SEED)
    sim = cl.ChandyLamportSim(per_gpu, device=local_rank, seed_base=seed_base,
                              fifo_lds_slots=args.fifo_slots)
    sim.read_topology_file(os.path.join(TEST_DATA, top))
    sim.read_events_file(os.path.join(TEST_DATA, events))
    sim.flush()                      # uploads topology/program/delays, first full run
    counters = sim.counters(only_ok=False)
    counters_ok = sim.counters(only_ok=True)
    n_nodes = sim.num_nodes

    for _ in range(args.warmup):
        sim.rerun()
    sim.synchronize()
    sim.kernel_time()                # reset the per-launch HIP-event accumulator

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.rerun()
    sim.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    k_total_ms, k_launches = sim.kernel_time()   # HIP events around each timed launch

    sums = sim.checksums()
    t_max, red = cldist.reduce_results(elapsed, sums.tolist() + [counters_ok["pop_tok"] + counters_ok["pop_mk"]],
                                       "cuda")   # RCCL all-reduce (max time, summed checksums)
    tot = dict(zip(cl.SUM_NAMES, red[:len(cl.SUM_NAMES)]))
    delivered_ok = red[-1]                       # packets of OK instances, all ranks

    per_step = t_max / args.steps
    value = delivered_ok / per_step
    avg_kernel_ms = k_total_ms / max(k_launches, 1)
    alg = b_alg(counters, n_nodes)                  # bytes per launch (this rank)
    achieved = alg / (avg_kernel_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(top, events, per_gpu, args.cpu_baseline_seconds)

    traffic = None
    tr_path = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tr_path):
        with open(tr_path) as f:
            tr = json.load(f)
        if tr.get("instances") == per_gpu and tr.get("fifo_slots") == args.fifo_slots:
            traffic = tr.get("hbm_bytes_per_launch")

    if rank == 0:
        line = {
            "metric": "delivered packets/sec (whole node)",
            "value": value,
            "unit": "packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: reference test_data scenario, per-instance Go math/rand delay streams",
            "config": {"workload": desc, "instances_per_gpu": per_gpu,
                       "instances_total": per_gpu * world, "parallelism": f"instances sharded over {world} GPU(s)",
                       "fifo_lds_slots": args.fifo_slots},
            "packets_per_step": delivered_ok,
            "status": {"ok": tot["ok"], "fatal": tot["fatal"], "other": tot["other"]},
            "checks": {"cut_residual": tot["cut_residual"], "final_residual": tot["final_residual"],
                       "snapshot_hash": tot["snapshot_hash"], "completed": tot["completed"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "kernel": "cl_exec_kernel",
                         "kernel_ms": avg_kernel_ms, "alg_bytes_per_launch": alg},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def b_alg_graph(c, n_nodes):
    """SURVEY.md §8(d) with CounterHash delays: no delay-schedule byte per draw."""
    pops = c["pop_tok"] + c["pop_mk"]
    return 8 * c["push"] + 8 * c["peek"] + 8 * pops + 4 * c["recorded"] + 4 * n_nodes * c["completed"]


def bench_graph(args, rank, world, local_rank):
    import torch
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    clg = importlib.import_module(PKG + ".graph")
    cldist = importlib.import_module(PKG + ".dist")
    cfg = dict(GRAPH_CONFIGS[args.config])
    n = args.graph_nodes or cfg["n"]
    steps = args.graph_steps or cfg["steps"]
    fifo = args.graph_fifo or cfg["fifo"]
    snap_steps = [k for k in cfg["snap_steps"] if k < steps]
    seed = cfg["seed"]
    rs = seed + 1000 * rank           # replica seeds: delays, traffic, snapshot placement
    snap_nodes = [(clg.counter_hash(rs + 3, i, 1) * n) >> 64 for i in range(len(snap_steps))]

    g = clg.GraphSim(device=local_rank, fifo_slots=fifo, max_snapshots=max(len(snap_steps), 1))
    if cfg["kind"] == "regular":
        g.generate_regular(n, cfg["degree"], cfg["tokens"], seed)
    else:
        g.generate_powerlaw(n, cfg["targets"], cfg["exponent"], cfg["ring"], cfg["tokens"], seed)
    g.set_delay_hash(rs + 1)
    g.set_traffic(rs + 2, 1 << 30, steps)
    si = 0
    for k in range(steps):
        while si < len(snap_steps) and snap_steps[si] == k:
            g.start_snapshot_rank(int(snap_nodes[si]))
            si += 1
        g.Tick(1)
    g.flush()                               # allocates, uploads, first full run
    counters = g.counters()
    for _ in range(args.warmup):
        g.rerun()
    g.synchronize()
    g.run_time()                            # reset the HIP-event accumulator

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.rerun()
    g.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    run_ms, runs, ticks = g.run_time()
    sums = g.checksums()
    status = g.status()
    vals = [sums[k] for k in clg.GSUM_NAMES]
    t_max, red = cldist.reduce_results(elapsed, vals, "cuda")
    tot = dict(zip(clg.GSUM_NAMES, red))
    per_step = t_max / args.steps
    value = tot["delivered"] / per_step if tot["ok"] == world else 0.0
    avg_run_ms = run_ms / max(runs, 1)
    alg = b_alg_graph(counters, n)
    achieved = alg / (avg_run_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_graph(g, cfg, n, steps, snap_steps, snap_nodes, rs, args.cpu_baseline_seconds)

    traffic = None
    tr_path = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tr_path):
        with open(tr_path) as f:
            tr = json.load(f)
        if tr.get("nodes") == n and tr.get("steps") == steps:
            traffic = tr.get("hbm_bytes_per_launch")

    if rank == 0:
        line = {
            "metric": "delivered packets/sec (whole node)",
            "value": value,
            "unit": "packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: generated graph, counter-hash traffic and delay streams (seeded per rank)",
            "config": {"workload": cfg["desc"], "nodes": n, "channels": g.num_channels, "ticks": steps,
                       "snapshots": len(snap_steps), "fifo_slots": fifo,
                       "parallelism": f"one replica per GPU, {world} GPU(s)"},
            "packets_per_step": tot["delivered"],
            "status": {"ok_replicas": tot["ok"], "replicas": world, "rank0_status": status},
            "checks": {"completed": tot["completed"], "cut_residual": tot["cut_residual"],
                       "final_residual": tot["final_residual"], "digest": tot["digest"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "graph tick pipeline (k_hostops, k_pick, k_marker, k_scan, k_push)",
                         "kernel_ms": avg_run_ms, "alg_bytes_per_launch": alg},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_graph(g, cfg, n, steps, snap_steps, snap_nodes, rs, budget_s):
    """The CPU oracle (C restatement, one simulation, one thread) on the SAME graph and
    program, timed over the first ticks of the window (about budget_s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    src, dst = g.channels()
    tok = np.full(n, cfg["tokens"], dtype=np.int64)
    width = len(str(n - 1))

    def run(k):
        o = O.OracleSim()
        o.use_counter_hash(rs + 1)
        o.build_graph(tok, src, dst, width)
        ss = np.array([s for s in snap_steps if s < k], dtype=np.int32)
        t = time.perf_counter()
        o.run_program(k, rs + 2, 1 << 30, steps, ss, np.array(snap_nodes[:ss.size], dtype=np.int32))
        secs = time.perf_counter() - t
        c = o.counters()
        return secs, c["pop_tok"] + c["pop_mk"], o.status

    k = min(steps, 8)
    secs, pk, st = run(k)
    while secs < budget_s / 3 and k < steps:   # later ticks cost more (longer logs): grow
        k = min(steps, 2 * k)
        secs, pk, st = run(k)
    return {"value": pk / secs, "unit": "packets/s", "cores": 1, "kind": "port",
            "sample": f"first {k} of {steps} ticks of the same graph and program ({pk} packets, "
                      f"{secs:.1f} s); CPU restatement in C (oracle/cl_oracle.c), one simulation on one "
                      f"thread -- not the Go reference (no Go toolchain in the image)"}


def cpu_baseline(top, events, n_total, budget_s):
    """The CPU oracle (C restatement, one simulation per thread) on the same instances
    (same seeds), repeated in passes until about budget_s of CPU work has run."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = min(16, os.cpu_count() or 1)
    t_text = open(os.path.join(TEST_DATA, top)).read()
    e_text = open(os.path.join(TEST_DATA, events)).read()
    probe = min(n_total, 4096)
    secs, st, _, cnt, _ = O.run_batch(t_text, e_text, probe, threads=threads)
    sample = int(min(n_total, max(probe, probe / max(secs, 1e-6) * budget_s)))
    total_s, total_pkts, passes = 0.0, 0, 0
    while passes == 0 or total_s < budget_s:
        secs, st, _, cnt, _ = O.run_batch(t_text, e_text, sample, threads=threads)
        ok = st == 0
        total_pkts += int((cnt[ok, 2] + cnt[ok, 3]).sum())
        total_s += secs
        passes += 1
    return {"value": total_pkts / total_s, "unit": "packets/s", "cores": threads, "kind": "port",
            "sample": f"{passes} pass(es) over the first {sample} of {n_total} instances (same seeds), "
                      f"{total_s:.1f} s; CPU restatement in C (oracle/cl_oracle.c), one simulation per "
                      f"thread -- not the Go reference (no Go toolchain in the image)"}


if __name__ == "__main__":
    main()
