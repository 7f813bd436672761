#!/usr/bin/env python3
"""Benchmark: delivered packets/s of the batched Chandy-Lamport engine (BASELINE.json).

A step = one pass of the hot path over one batch: every instance runs the whole event
program from the initial topology to the end of the drain (test_common.go:79-140).  The
default batch is the north_star's: BASELINE config 3, 8nodes.top +
8nodes-concurrent-snapshots.events x 2^20 instances, each with its own Go delay stream
(instance i: rand.Seed(REFERENCE_SEED + i)).  Inputs (topology, event program, delay
schedule) are resident in HBM before timing; the timed region is K launches of the exec
kernel.  After timing, the batch checksums of the timed path are compared with the CPU
oracle's values for the same instances (tests/golden/bench_sums.json): "parity".

Multi-GPU: one process per GPU; the fixed 2^20-instance batch is split into disjoint
instance ranges (rank r: instances [r*I/N, (r+1)*I/N), seeds base + global index), so
there is no data-path collective ("scaling": "strong"); RCCL all-reduces the batch
checksums once, after timing.  `bench.py --gpus N` run by hand starts the N ranks itself
(a child torch.distributed.run); under the driver's own torch.distributed.run each rank
checks that WORLD_SIZE equals --gpus.  --config c2 is BASELINE config 2 (10nodes x 65,536);
c4/c5 are the large-graph configs (one simulation per GPU, replicas).

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
    # BASELINE.json configs[2] -- the north_star's batch and the default bench line:
    # 2^20 instances in total, split over the ranks (strong scaling)
    "c3": ("8nodes.top", "8nodes-concurrent-snapshots.events", 1 << 20,
           "8nodes-concurrent x 1,048,576: 8nodes.top + 8nodes-concurrent-snapshots.events, "
           "2^20 instances split over the GPUs, Go delay streams"),
    # BASELINE.json configs[1]: 65,536 replicas (split over the GPUs likewise)
    "c2": ("10nodes.top", "10nodes.events", 65536,
           "10nodes x 65,536: 10nodes.top + 10nodes.events, 65,536 replicas split over the GPUs, "
           "Go delay streams"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)

# BASELINE.json configs[3] and [4]: one large simulation per GPU on the graph engine
# (include/clgraph.h).  Ranks run replicas of the same graph with their own delay,
# traffic and snapshot-placement seeds ("replicas only").
GRAPH_CONFIGS = {
    "c4": dict(kind="regular", n=1 << 20, degree=8, tokens=100, steps=80, snap_steps=[5], fifo=16,
               seed=20240, cpu_full=True,
               desc="random 8-out regular digraph, 2^20 nodes, one snapshot under continuous token "
                    "traffic (p=1/4 per node per tick), 80 ticks"),
    "c5": dict(kind="powerlaw", n=100_000, targets=8, exponent=0.9, ring=True, tokens=100, steps=4100,
               snap_steps=list(range(1, 4097)), fifo=8192, seed=30240, drain=True,
               desc="power-law digraph (8 Zipf(0.9) targets + ring), 100k nodes, 4,096 overlapping "
                    "snapshots (one start per tick) under continuous traffic for 4,100 ticks, then "
                    "readEventsFile's drain until every snapshot completed (+6 ticks)"),
}


def b_alg(c, n_nodes):
    """8 push + 8 peek + 8 pop + 4 recorded + 1 draw + 4 N completed."""
    pops = c["pop_tok"] + c["pop_mk"]
    return 8 * c["push"] + 8 * c["peek"] + 8 * pops + 4 * c["recorded"] + 1 * c["push"] \
        + 4 * n_nodes * c["completed"]


SIMDS = 256 * 4          # MI355X: 256 CUs x 4 SIMD-32 units (MI355X_MICROARCH.md)
CLOCK_HZ = 2.4e9         # max engine clock (MI355X_MICROARCH.md)
VALU_PEAK = SIMDS * CLOCK_HZ / 2   # wave64 VALU instructions/s: one per 2 cycles per SIMD-32
FIXTURE = os.path.join(ROOT, "tests", "golden", "bench_sums.json")
PARITY_KEYS = ("instances", "ok", "fatal", "other", "delivered", "snapshot_hash", "completed",
               "cut_residual", "final_residual")


# Default (steps, warmup) per config: enough untimed launches for the GPU's clocks to settle
# (C2's 0.18 ms launches measured 0.185 ms per kernel over 3 warmup + 30 timed steps and
# 0.176 ms over 300 timed steps) and a timed region of >= 50 ms.
# (timed steps, warmup): enough timed replays that the two stream synchronisations of the timed
# region stay under 1 % of it (C3: 200 x 1.64 ms)
STEP_DEFAULTS = {"c2": (300, 100), "c3": (200, 20)}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: per config, STEP_DEFAULTS)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warmup steps (default: per config)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS) + sorted(GRAPH_CONFIGS))
    ap.add_argument("--graph-nodes", type=int, default=0, help="override the graph size (c4/c5)")
    ap.add_argument("--graph-steps", type=int, default=0, help="override the tick window (c4/c5)")
    ap.add_argument("--graph-fifo", type=int, default=0, help="override FIFO slots per channel (c4/c5)")
    ap.add_argument("--instances", type=int, default=0, help="instances in total (default: the config's batch)")
    ap.add_argument("--fifo-slots", type=int, default=0, help="LDS ring slots per channel (0 = automatic)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fresh", action="store_true", help="skip the fresh-seed first-launch measurement")
    ap.add_argument("--no-collect", action="store_true", help="skip the full-batch CollectSnapshot measurement")
    ap.add_argument("--no-parity", action="store_true",
                    help="graph configs: skip the after-timing parity run (profiler passes that must see one program)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on GPUs; gloo for rehearsals")
    ap.add_argument("--shared-device", action="store_true",
                    help="every rank on cuda:0 (multi-rank rehearsal on a one-GPU box)")
    ap.add_argument("--launch-check", action="store_true",
                    help="test hook: ranks rendezvous over gloo, rank 0 prints the world it saw, no GPU work")
    args = ap.parse_args(argv)
    steps, warmup = STEP_DEFAULTS.get(args.config, (20, 3))
    args.steps = steps if args.steps is None else args.steps
    args.warmup = warmup if args.warmup is None else args.warmup
    return args


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(args, env, argv):
    """How this process runs `--gpus N` (one process per GPU).

    Returns None when this process is a rank already (WORLD_SIZE set and equal to
    --gpus) or the run is single-GPU; else the torch.distributed.run command that starts
    N ranks of this script with the same arguments.  A WORLD_SIZE that differs from
    --gpus is an error (SystemExit, non-zero): the line would report a world it was not
    asked to measure."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to measure a "
                             f"different world than the one asked for")
        return None
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus}")
    if args.gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)


def relaunch(args, argv):
    """`bench.py --gpus N` started by hand (no WORLD_SIZE): start the N ranks as a child
    torch.distributed.run before anything here touches the GPU, let rank 0's JSON line
    through, and return the child's exit code.  None: this process runs the bench."""
    cmd = launch_plan(args, os.environ, argv)
    if cmd is None:
        return None
    if not args.shared_device and not args.launch_check:
        import torch   # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if have < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but {have} visible GPU(s) "
                             f"(--shared-device rehearses N ranks on one GPU)")
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def launch_check(args, rank, world):
    """--launch-check: the rank launch alone (rendezvous + one gloo all-reduce), no GPU."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    t = torch.tensor([rank, 1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_seen": int(t[1]),
                          "rank_sum": int(t[0]), "gpus_arg": args.gpus}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def init_dist(args, world, local_rank):
    import torch
    import torch.distributed as dist
    device = 0 if args.shared_device else local_rank
    if world > 1:
        torch.cuda.set_device(device)
        dist.init_process_group(args.dist_backend, init_method="env://")
    return device


def profile_entry(cfg, instances):
    """The committed rocprofv3 PMC summary (profiles/<round>_<cfg>_pmc.json) of this
    per-GPU batch: (path, summary, scale).  The latest round's profile of exactly this
    many instances, else the latest round's nearest one with its byte and instruction
    counts scaled by the batch ratio (both are per-instance sums; the resident-wave
    count is not scaled)."""
    import glob
    exact, near = None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg}_pmc.json"))):
        with open(path) as f:
            d = json.load(f)
        if d.get("instances") == instances:
            exact = (path, d, 1.0)
        elif d.get("instances") and (near is None or path.split("_")[0] >= near[0].split("_")[0]):
            near = (path, d, instances / d["instances"])
    return exact or near


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    rc = relaunch(args, argv)
    if rc is not None:
        return rc
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        return launch_check(args, rank, world)
    if args.config in GRAPH_CONFIGS:
        return bench_graph(args, rank, world, local_rank)
    top, events, total, desc = CONFIGS[args.config]
    if args.instances:
        total = args.instances
    if total % world:
        raise SystemExit(f"{total} instances do not split over {world} ranks")
    per_rank = total // world

    import torch
    import torch.distributed as dist
    device = init_dist(args, world, local_rank)
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

    cl = importlib.import_module(PKG)
    cldist = importlib.import_module(PKG + ".dist")
    _, seed_base = cldist.shard(per_rank, rank, cl.REFERENCE_SEED)
    sim = cl.ChandyLamportSim(per_rank, device=device, seed_base=seed_base,
                              fifo_lds_slots=args.fifo_slots)
    sim.read_topology_file(os.path.join(TEST_DATA, top))
    sim.read_events_file(os.path.join(TEST_DATA, events))
    sim.flush()                      # uploads topology/program/delays, first full run
    counters = sim.counters(only_ok=False)
    n_nodes = sim.num_nodes

    for _ in range(args.warmup):
        sim.rerun()
    sim.synchronize()
    sim.kernel_time()                # reset the per-launch HIP-event accumulator

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps - 1):
        sim.rerun()
    sim.synchronize()
    t1 = time.perf_counter()
    # The last timed step writes into output planes poisoned just before it (outside the
    # timed region): the parity checksums below can only come from that timed launch.
    sim.poison_outputs()
    sim.synchronize()
    t2 = time.perf_counter()
    sim.rerun()
    sim.synchronize()
    barrier()
    elapsed = (t1 - t0) + (time.perf_counter() - t2)
    k_total_ms, k_launches = sim.kernel_time()   # HIP events around each timed launch

    # checksums of the LAST timed rerun (the timed path itself), all-reduced over ranks
    sums = sim.checksums()
    recorded_ok = sim.counters(only_ok=True)["recorded"]
    collect = collect_all(sim, args) if not args.no_collect else None
    engine = sim.exec_engine()
    spilled, split = sim.replay_split()
    # (cl_jit.cpp launch_lanes: the spilling half runs on the lanes spill kernel when it fills a
    # wave per SIMD, node-parallel otherwise)
    spill_on_lanes = per_rank - split >= 64 * 4 * torch.cuda.get_device_properties(device).multi_processor_count
    replay = {"slot_map": sim.mapped_replays(), "spill_free": sim.spill_free_replays(),
              "spilled_instances": spilled, "split_slot": split}
    fresh = fresh_run(cl, per_rank, device, seed_base + total, top, events, args) if not args.no_fresh else None
    t_max, red = cldist.reduce_results(elapsed, sums.tolist() + [recorded_ok], coll_dev)
    tot = dict(zip(cl.SUM_NAMES, red[:len(cl.SUM_NAMES)]))
    tot["recorded"] = red[len(cl.SUM_NAMES)]
    delivered_ok = tot["delivered"]              # packets of OK instances, all ranks

    parity, parity_note = None, "no fixture for this batch"
    if os.path.exists(FIXTURE):
        with open(FIXTURE) as f:
            fx = json.load(f)
        want = fx["batches"].get(args.config)
        if want and want["instances"] == total and fx["seed_base"] == cl.REFERENCE_SEED:
            w = want["sums"]
            diff = {k: (tot[k], w[k]) for k in PARITY_KEYS + ("recorded",)
                    if (tot[k] - w[k]) % (1 << 64) != 0}
            parity = not diff
            parity_note = "tests/golden/bench_sums.json (CPU oracle over every instance)" + \
                ("" if parity else f"; mismatches {diff}")

    per_step = t_max / args.steps
    value = delivered_ok / per_step
    alg_rank = b_alg(counters, n_nodes)             # bytes per launch (this rank)
    # whole node: algorithmic bytes of every rank's launch over the slowest rank's average
    # kernel time, against N x the HBM peak
    kmax = cldist.reduce_max([k_total_ms / max(k_launches, 1)] +
                             ([fresh["kernel_ms"]] if fresh else []), coll_dev)
    avg_kernel_ms = kmax[0]
    alg = cldist.reduce_results(0.0, [alg_rank], coll_dev)[1][0]
    achieved = alg / (avg_kernel_ms * 1e-3) / 1e9
    if fresh:
        fsum = cldist.reduce_results(0.0, [fresh["delivered"]], coll_dev)[1][0]
        fresh = {"fresh_run_ms": kmax[1], "packets_per_s": fsum / (kmax[1] * 1e-3), "packets": fsum,
                 "seeds": f"rand.Seed(REFERENCE_SEED + {total} + i): a batch of the same size the "
                          f"engine never ran", "note": fresh["note"]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(top, events, total, args.cpu_baseline_seconds)

    traffic, valu, traffic_detail = None, None, None
    prof = profile_entry(args.config, per_rank)
    if prof is not None and args.fifo_slots == 0:
        path, d, scale = prof
        c = d["counters"]
        src = os.path.relpath(path, ROOT) + ("" if scale == 1 else
                                             f" (x{scale:g}: per-GPU batch {per_rank} vs profiled {d['instances']})")
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            # whole node, per launch: every rank moves its share.  The exec kernels' reads are
            # scattered per-instance delay rows, not wide coalesced streams, so the raw count is
            # the HBM traffic (the guide's 2x FETCH factor would overstate it: C3's raw FETCH_SIZE
            # equals the 117 MB schedule); the corrected figure rides along (tools/traffic_model.py)
            traffic = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 * scale * world
            traffic_detail = {"raw": traffic, "fetch_doubled": (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 * scale * world,
                              "write": c["WRITE_SIZE"] * 1024 * scale * world, "used": "raw",
                              "why": "the exec kernels read per-instance delay rows scattered by the slot map, "
                                     "not wide coalesced streams (the guide's 2x FETCH factor applies to those)",
                              "source": src}
        if "SQ_INSTS_VALU" in c:
            rate = c["SQ_INSTS_VALU"] * scale * world / (avg_kernel_ms * 1e-3)
            valu = {"achieved": rate, "peak": VALU_PEAK * world, "unit": "wave64 VALU instr/s",
                    "frac": rate / (VALU_PEAK * world), "insts_per_launch": c["SQ_INSTS_VALU"] * scale * world,
                    "source": src}
            if "SQ_WAVE_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
                # SQ_WAVE_CYCLES counts quad-cycles summed over waves; GRBM over the 8 XCDs
                valu["waves_per_simd"] = 4 * c["SQ_WAVE_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8) / SIMDS
    peak = HBM_PEAK_GBS * world
    hbm_frac = achieved / peak

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
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: reference test_data scenario, per-instance Go math/rand delay streams",
            "config": {"workload": desc, "instances_total": total, "instances_per_gpu": per_rank,
                       "parallelism": f"instances sharded over {world} GPU(s)",
                       "fifo_lds_slots": args.fifo_slots},
            "packets_per_step": delivered_ok,
            "parity": parity,
            "parity_ref": parity_note,
            "status": {"ok": tot["ok"], "fatal": tot["fatal"], "other": tot["other"]},
            "checks": {"cut_residual": tot["cut_residual"], "final_residual": tot["final_residual"],
                       "snapshot_hash": tot["snapshot_hash"], "completed": tot["completed"],
                       "recorded": tot["recorded"]},
            "fresh_run": fresh,
            "collect": collect,
            "replay": dict(replay, note="value is the replay rate: the timed steps re-run the same "
                                        "program and delays, launched through the slot map that the "
                                        "first run's final ticks give (DESIGN.md section 6); fresh_run is "
                                        "the first launch on new seeds, with no map; split replays run "
                                        "slots [0, split_slot) on the spill-free kernel and the instances "
                                        "that spilled in the first run on the spill-capable one, "
                                        "concurrently (section 5), both inside kernel_ms"),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": hbm_frac,
                         "traffic": traffic, "traffic_detail": traffic_detail,
                         "kernel": ("clsnap_lanes_nospill (instance per lane, hipRTC-specialized to the "
                                    "topology)" + ((" + clsnap_lanes_spill" if spill_on_lanes else " + cl_exec_kernel")
                                                   + " on the spilling instances" if split else "")
                                    if engine == cl.ChandyLamportSim.ENGINE_LANES else "cl_exec_kernel"),
                         "kernel_ms": avg_kernel_ms, "alg_bytes_per_launch": alg,
                         "scope": f"whole node: {world} GPU(s), bytes summed over ranks, slowest rank's "
                                  f"average kernel time, peak {world} x {HBM_PEAK_GBS:g} GB/s",
                         "valu": valu,
                         "binding_resource": (
                             "instruction issue per wave: the instance-per-lane kernel runs 3 waves per SIMD "
                             "(168 VGPRs, 13 KB of LDS per wave), each wave bound by its own dependent chains "
                             "(one VALU per 4 cycles at most, the SIMD could take one per 2); neither the B_alg "
                             "HBM fraction nor the VALU issue fraction is near 1 (DESIGN.md sections 5 and 9)"
                             if engine == cl.ChandyLamportSim.ENGINE_LANES else
                             "instruction issue per wave-tick at ~5 resident waves per SIMD (LDS-capped): "
                             "neither the B_alg HBM fraction nor the VALU issue fraction is near 1; "
                             "fewer issued instructions (register pressure, compile-time LDS offsets) "
                             "moved the time, fewer dependent LDS round trips did not; DESIGN.md section 9")},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def collect_all(sim, args):
    """CollectSnapshot (sim.go:134-173) of every snapshot over this rank's whole batch, packed
    on the GPU (cl_collect_snapshot_packed) into host arrays: the reference's {tokenMap,
    messages} for every instance.  Outside `value`.  Device ms = the packing kernels (HIP
    events), wall ms = packing + the PCIe copies into pageable host memory, summed over the
    snapshots (second pass: buffers already sized)."""
    out = None
    for _ in range(2):
        dev, wall, msgs, nbytes = 0.0, 0.0, 0, 0
        for sid in range(sim.num_snapshots):
            t = time.perf_counter()
            tok, done, off, msg = sim.collect_snapshot_packed(sid, out=out)
            wall += time.perf_counter() - t
            if out is None or msg.size > out[3].size:
                out = (tok, np.zeros(done.size, dtype=np.int32), off, np.zeros(max(msg.size, 1024), dtype=np.int32))
            dev += sim.collect_time()
            msgs += int(msg.size)
            nbytes += tok.nbytes + 4 * done.size + off.nbytes + 4 * msg.size
    return {"snapshots": sim.num_snapshots, "instances": sim.n_instances, "messages": msgs,
            "device_ms": dev, "wall_ms": wall * 1e3, "bytes_to_host": nbytes,
            "note": "CollectSnapshot of every snapshot of the whole batch, packed on the GPU into one CSR "
                    "over (instance, channel) per snapshot (cl_collect_snapshot_packed); not in value"}


def fresh_run(cl, n, device, seed_base, top, events, args):
    """One first launch on seeds the engine never ran: a new batch of the same size and
    program (instances seeded seed_base + i), no slot map and no spill probe from a prior
    run -- what a caller with a fresh batch gets.  Warm clocks (it follows the timed
    region).  Returns its kernel time and the packets its OK instances delivered."""
    f = cl.ChandyLamportSim(n, device=device, seed_base=seed_base, fifo_lds_slots=args.fifo_slots)
    f.read_topology_file(os.path.join(TEST_DATA, top))
    f.read_events_file(os.path.join(TEST_DATA, events))
    f.rerun()                    # the first launch of this sim: nothing derived from a prior run
    f.synchronize()
    ms, launches = f.kernel_time()
    sums = dict(zip(cl.SUM_NAMES, f.checksums().tolist()))
    return {"kernel_ms": ms / max(launches, 1), "delivered": sums["delivered"],
            "note": "first launch of a new sim on unseen seeds (HIP events): no replay plan, so the whole "
                    "batch runs unordered on the spill-capable kernel; the same fresh path on the fixture "
                    "seeds is parity-pinned (tests/test_gpu_parity.py test_headline_batch_fresh_path_matches_"
                    "fixture)"}


def b_alg_graph(c, n_nodes):
    """SURVEY.md §8(d) with CounterHash delays: no delay-schedule byte per draw."""
    pops = c["pop_tok"] + c["pop_mk"]
    return 8 * c["push"] + 8 * c["peek"] + 8 * pops + 4 * c["recorded"] + 4 * n_nodes * c["completed"]


def bench_graph(args, rank, world, local_rank):
    import torch
    import torch.distributed as dist
    device = init_dist(args, world, local_rank)
    coll_dev = "cuda" if args.dist_backend == "nccl" else "cpu"

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

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

    g = clg.GraphSim(device=device, fifo_slots=fifo, max_snapshots=max(len(snap_steps), 1),
                     max_drain_ticks=1_000_000)
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
    if cfg.get("drain"):
        g.drain()                           # test_common.go:123-137, on the device
    g.flush()                               # allocates, uploads, first full run
    counters = g.counters()
    for _ in range(args.warmup):
        g.rerun()
    g.synchronize()
    g.run_time()                            # reset the HIP-event accumulator

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps - 1):
        g.rerun()
    g.synchronize()
    t1 = time.perf_counter()
    g.poison_outputs()            # (untimed) the last timed run writes into poisoned planes
    g.synchronize()
    t2 = time.perf_counter()
    g.rerun()
    g.synchronize()
    barrier()
    elapsed = (t1 - t0) + (time.perf_counter() - t2)
    run_ms, runs, ticks = g.run_time()
    (pre_ms, pre_ticks), (drain_ms, drain_ticks) = g.phase_time()   # the last timed run
    sums = g.checksums()
    status = g.status()
    parity, parity_ref = (None, "skipped (--no-parity)") if args.no_parity else \
        graph_parity(args.config, g, rank, n, steps, device)
    vals = [sums[k] for k in clg.GSUM_NAMES]
    t_max, red = cldist.reduce_results(elapsed, vals, coll_dev)
    tot = dict(zip(clg.GSUM_NAMES, red))
    per_step = t_max / args.steps
    value = tot["delivered"] / per_step if tot["ok"] == world else 0.0
    avg_run_ms = run_ms / max(runs, 1)
    alg = b_alg_graph(counters, n)
    achieved = alg / (avg_run_ms * 1e-3) / 1e9

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_graph(g, cfg, n, steps, snap_steps, snap_nodes, rs, args.cpu_baseline_seconds)

    traffic, traffic_detail = None, None
    tr_path = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tr_path):
        with open(tr_path) as f:
            tr = json.load(f)
        if tr.get("nodes") == n and tr.get("steps") == steps and tr.get("drain", False) == bool(cfg.get("drain")):
            traffic = tr.get("hbm_bytes_per_launch")  # raw per kernel unless its reads stream
            traffic_detail = {k: tr.get(k) for k in ("raw_bytes_per_launch", "corrected_bytes_per_launch")}
            traffic_detail["used"] = "per kernel: raw, or fetch-doubled where the reads are wide coalesced streams"
            traffic_detail["source"] = os.path.relpath(tr_path, ROOT)

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
            "config": {"workload": cfg["desc"], "nodes": n, "channels": g.num_channels,
                       "ticks": ticks // max(runs, 1), "traffic_ticks": steps,
                       "snapshots": len(snap_steps), "fifo_slots": fifo,
                       "parallelism": f"one replica per GPU, {world} GPU(s)"},
            "packets_per_step": tot["delivered"],
            "parity": parity,
            "parity_ref": parity_ref,
            "phases": {"traffic": {"ticks": pre_ticks, "ms": pre_ms,
                                   "us_per_tick": 1e3 * pre_ms / max(pre_ticks, 1)},
                       "drain": {"ticks": drain_ticks, "ms": drain_ms,
                                 "us_per_tick": 1e3 * drain_ms / max(drain_ticks, 1)},
                       "note": "rank 0's last timed run, HIP events at the first drain (cl_graph_phase_time)"},
            "status": {"ok_replicas": tot["ok"], "replicas": world, "rank0_status": status},
            "checks": {"completed": tot["completed"], "cut_residual": tot["cut_residual"],
                       "final_residual": tot["final_residual"], "digest": tot["digest"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_detail": traffic_detail,
                         "kernel": "graph tick pipeline (k_hostops, k_pick, k_marker, k_scan, k_push)",
                         "kernel_ms": avg_run_ms, "alg_bytes_per_launch": alg},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


GRAPH_FIXTURE = os.path.join(ROOT, "tests", "golden", "graph_runs.json")


def _mix64(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


def graph_run_summary(g):
    """The exact run summary tests/graphcheck.py run_summary defines (status, time, counters,
    completion ticks, content digest of the completed snapshots, final-token sum and hash),
    from the engine's own results; the fixture holds the CPU oracle's."""
    c = g.counters()
    tok = g.node_tokens_array()
    with np.errstate(over="ignore"):
        h = int(_mix64(tok.astype(np.uint64) ^ np.arange(tok.size, dtype=np.uint64)).sum(dtype=np.uint64))
    return {"status": g.status(), "time": g.time(),
            "counters": {k: c[k] for k in ("push", "peek", "pop_tok", "pop_mk", "recorded", "completed")},
            "ctick": [g.snapshot_tick(s) for s in range(g.num_snapshots)],
            "digest_sum": g.checksums()["digest"] % (1 << 64),
            "final_tokens_sum": int(tok.sum()), "final_tokens_hash": h % (1 << 64)}


def fixture_matches(got, want):
    """Mismatched keys of a run summary against a graph_runs.json summary."""
    w = dict(want)
    w["digest_sum"] = sum(want["digest"]) % (1 << 64)
    w["final_tokens_hash"] = want["final_tokens_hash"] % (1 << 64)
    return {k: (got[k], w[k]) for k in got if got[k] != w[k]}


def graph_parity(cfg, g, rank, n, steps, device):
    """C4: the timed run itself (rank 0's seeds, the default size) against the CPU oracle's
    full-size run of the same program.  C5: the full-size run is far beyond the oracle
    (4e9 deliveries with O(snapshots) recording per token), so the same engine runs the
    20,000-node x 256-snapshot C5-shape program with the drain against its oracle fixture,
    after timing; the full-size run is checked by properties in the line's `checks`."""
    if not os.path.exists(GRAPH_FIXTURE):
        return None, "no fixture"
    with open(GRAPH_FIXTURE) as f:
        runs = json.load(f)["runs"]
    clg = importlib.import_module(PKG + ".graph")
    if cfg == "c4":
        fx = runs.get("c4_full")
        if rank != 0 or not fx or (fx["nodes"], fx["steps"]) != (n, steps):
            return None, "the c4_full fixture is rank 0's default-size program"
        bad = fixture_matches(graph_run_summary(g), fx["summary"])
        return not bad, ("tests/golden/graph_runs.json c4_full: CPU oracle over the same full-size program "
                         "(tools/gen_graph_fixture.py), compared with the last timed run (written into "
                         "poisoned result planes)" + (f"; mismatches {bad}" if bad else ""))
    fx = runs.get("c5_shape_20k_256")
    if not fx:
        return None, "no c5 fixture"
    m, w, k, seed = fx["nodes"], fx["steps"], fx["snapshots"], 21      # tests/graphcheck.py powerlaw_program
    s = clg.GraphSim(device=device, fifo_slots=fx["fifo_slots"], max_snapshots=k, max_drain_ticks=fx["max_drain"])
    s.generate_powerlaw(m, 8, 0.9, True, 100, seed)
    s.set_delay_hash(seed + 2)
    s.set_traffic(seed + 1, 1 << 30, w)
    for step in range(w):
        if 1 <= step <= k:
            s.start_snapshot_rank((clg.counter_hash(seed + 3, step - 1, 1) * m) >> 64)
        s.Tick(1)
    s.drain()
    s.flush()
    bad = fixture_matches(graph_run_summary(s), fx["summary"])
    return not bad, ("tests/golden/graph_runs.json c5_shape_20k_256: the 20,000-node x 256-snapshot C5-shape "
                     "program with the drain on the same engine, after timing, vs the CPU oracle's run; the "
                     "full-size run itself is checked by properties (checks: completed, residuals)"
                     + (f"; mismatches {bad}" if bad else ""))


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

    if cfg.get("drain"):
        return cpu_baseline_drain(O, tok, src, dst, width, steps, snap_steps, snap_nodes, rs, budget_s)
    if cfg.get("cpu_full"):
        # the whole program (C4: 80 ticks, ~25 s of oracle time): the same run the GPU times
        k = steps
        secs, pk, st = run(k)
    else:
        k = min(steps, 8)
        secs, pk, st = run(k)
        while secs < budget_s / 3 and k < steps:   # later ticks cost more (longer logs): grow
            k = min(steps, 2 * k)
            secs, pk, st = run(k)
    what = f"all {steps} ticks" if k == steps else f"first {k} of {steps} ticks"
    return {"value": pk / secs, "unit": "packets/s", "cores": 1, "kind": "port",
            "sample": f"{what} of the same graph and program ({pk} packets, {secs:.1f} s); CPU restatement in "
                      f"C (oracle/cl_oracle.c), one simulation on one thread (the reference simulates one "
                      f"graph on one goroutine) -- not the Go reference (no Go toolchain in the image)"}


def cpu_baseline_drain(O, tok, src, dst, width, steps, snap_steps, snap_nodes, rs, budget_s):
    """C5's two regimes on the CPU oracle, on the SAME graph: a shortened program -- traffic
    and one snapshot start per tick for the first k ticks, as C5 begins -- followed by
    readEventsFile's drain until every snapshot completed (+6 ticks), as C5 ends.  k grows until
    the run takes about budget_s / 3.  The traffic ticks and the drain ticks are timed (and
    their packets counted) separately; `value` is the whole run's rate."""
    def run(k):
        o = O.OracleSim()
        o.use_counter_hash(rs + 1)
        o.build_graph(tok, src, dst, width)
        ss = np.array(snap_steps[:k], dtype=np.int32)
        t0 = time.perf_counter()
        o.run_program(k, rs + 2, 1 << 30, steps, ss, np.array(snap_nodes[:ss.size], dtype=np.int32))
        t1 = time.perf_counter()
        c0 = o.counters()
        ticks0 = o.time
        o.drain(O.MAX_DRAIN_TICKS)
        t2 = time.perf_counter()
        c1 = o.counters()
        p0 = c0["pop_tok"] + c0["pop_mk"]
        p1 = c1["pop_tok"] + c1["pop_mk"]
        return dict(k=k, traffic_s=t1 - t0, drain_s=t2 - t1, traffic_pk=p0, drain_pk=p1 - p0,
                    drain_ticks=o.time - ticks0, status=o.status)

    k = 4
    r = run(k)
    while r["traffic_s"] + r["drain_s"] < budget_s / 3 and k < len(snap_steps):
        k = min(len(snap_steps), 2 * k)
        r = run(k)
    tot_s = r["traffic_s"] + r["drain_s"]
    tot_pk = r["traffic_pk"] + r["drain_pk"]
    return {"value": tot_pk / tot_s, "unit": "packets/s", "cores": 1, "kind": "port",
            "regimes": {"traffic": {"ticks": r["k"], "packets": r["traffic_pk"], "s": r["traffic_s"],
                                    "packets_per_s": r["traffic_pk"] / max(r["traffic_s"], 1e-9)},
                        "drain": {"ticks": r["drain_ticks"], "packets": r["drain_pk"], "s": r["drain_s"],
                                  "packets_per_s": r["drain_pk"] / max(r["drain_s"], 1e-9)}},
            "sample": f"the same 100k-node graph and seeds, shortened program: {r['k']} traffic ticks with one "
                      f"snapshot start per tick (C5 starts one per tick for 4,096 ticks), then readEventsFile's "
                      f"drain until all {r['k']} snapshots completed (+6 ticks; {r['drain_ticks']} drain ticks); "
                      f"{tot_pk} packets in {tot_s:.1f} s, the drain ticks timed separately (regimes); CPU "
                      f"restatement in C (oracle/cl_oracle.c), one simulation on one thread -- not the Go "
                      f"reference (no Go toolchain in the image)"}


def host_cpu():
    """(threads to use, CPU model, logical CPUs of the machine).  The GPU box grants a
    share of its host cores per GPU (OMP_NUM_THREADS there); os.cpu_count() shows the
    whole machine, so the pool is the affinity set capped by that share."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(avail, share) if share > 0 else avail
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return max(threads, 1), model, os.cpu_count()


def cpu_baseline(top, events, n_total, budget_s):
    """The CPU oracle (C restatement, one simulation per thread) over the SAME instance
    set as the timed batch (instances 0..n_total-1, same seeds), with the topology and
    events parsed once outside the timed region; repeated in passes until about
    budget_s of wall time has run."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads, model, ncpu = host_cpu()
    t_text = open(os.path.join(TEST_DATA, top)).read()
    e_text = open(os.path.join(TEST_DATA, events)).read()
    total_s, total_pkts, passes = 0.0, 0, 0
    while passes == 0 or total_s < budget_s:
        secs, st, _, cnt, _ = O.run_batch_prepared(t_text, e_text, n_total, seed_base=O.REFERENCE_SEED,
                                                   threads=threads, want_hash=False)
        ok = st == 0
        total_pkts += int((cnt[ok, 2] + cnt[ok, 3]).sum())
        total_s += secs
        passes += 1
    rate = total_pkts / total_s
    return {"value": rate, "unit": "packets/s", "cores": threads, "kind": "port",
            "cpu_model": model, "host_logical_cpus": ncpu,
            "sample": f"{passes} pass(es) over all {n_total} instances of the timed batch (same seeds), "
                      f"{total_s:.1f} s of simulation wall time on {threads} threads; topology and events "
                      f"parsed once outside the timed region; CPU restatement in C (oracle/cl_oracle.c), "
                      f"one simulation per thread at a time -- not the Go reference (no Go toolchain "
                      f"in the image)",
            "node_host_estimate": {
                "value": rate * NODE_GPUS, "unit": "packets/s", "cores": threads * NODE_GPUS,
                "measured": False,
                "note": f"the whole 8-GPU node's host share, extrapolated linearly from the measured "
                        f"{threads}-thread figure (an upper bound): the GPU box grants {threads} host CPUs "
                        f"per GPU (OMP_NUM_THREADS), and running more threads than that share would take "
                        f"CPU time from other jobs on the machine ({ncpu} logical CPUs)"}}


NODE_GPUS = 8   # MI355X per node (BASELINE.json north_star)


if __name__ == "__main__":
    sys.exit(main() or 0)
