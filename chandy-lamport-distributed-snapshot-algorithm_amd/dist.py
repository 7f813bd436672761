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


def reduce_max(values, device):
    """Elementwise max of float values over all ranks."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


# ---- exchange layer of the graph-partitioned mode ---------------------
# One simulation whose nodes are split into rank ranges exchanges, every tick, records
# addressed to the owners of other nodes (deliveries, broadcast-trigger reports, draw
# bases).  Records are fixed-width int64 rows; one all-to-all of counts sizes one
# all-to-all of the rows (RCCL over xGMI for device tensors, gloo for host tensors).

def exchange_rows(rows_by_dest, width, device="cpu"):
    """rows_by_dest[r]: int64 array [k_r, width] for rank r.  Returns the list of the
    arrays every rank addressed to this one, in source-rank order."""
    world = dist.get_world_size()
    counts = torch.tensor([len(r) for r in rows_by_dest], dtype=torch.int64, device=device)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts)
    send = torch.cat([torch.as_tensor(r, dtype=torch.int64).reshape(-1, width) for r in rows_by_dest]).to(device) \
        if any(len(r) for r in rows_by_dest) else torch.zeros((0, width), dtype=torch.int64, device=device)
    rc = recv_counts.tolist()
    recv = torch.empty((sum(rc), width), dtype=torch.int64, device=device)
    dist.all_to_all_single(recv.view(-1), send.reshape(-1).contiguous(),
                           output_split_sizes=[c * width for c in rc],
                           input_split_sizes=[len(r) * width for r in rows_by_dest])
    out, o = [], 0
    host = recv.cpu().numpy()
    for c in rc:
        out.append(host[o:o + c])
        o += c
    return out


def allgather_ints(values, device="cpu"):
    """[world, len(values)] int64: every rank's values."""
    t = torch.tensor([int(v) for v in values], dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out).cpu().numpy()
