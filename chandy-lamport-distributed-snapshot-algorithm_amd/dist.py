"""Multi-GPU sharding of independent instances (one process per GPU).

Instances are independent simulations, so the path shards with no data-path
collective: rank r owns instances [r * per_rank, (r + 1) * per_rank) and seeds them
base + global index (the reference seeds one run with rand.Seed(seed + 1),
snapshot_test.go:20).  After the timed region the ranks all-reduce a handful of int64
checksums and take the max of their elapsed times -- RCCL over xGMI when the tensors
live on the GPU (backend "nccl"), gloo on CPU in tests.
"""
import torch
import torch.distributed as dist


def shard(per_rank, rank, seed_base):
    """(first global instance, seed of that instance) for this rank."""
    first = rank * per_rank
    return first, seed_base + first


def reduce_results(elapsed_s, sums, device):
    """Max elapsed time and summed int64 checksums over all ranks."""
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    s = torch.tensor([int(v) for v in sums], dtype=torch.int64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(v) for v in s.tolist()]
