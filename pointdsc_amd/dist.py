"""Multi-GPU sharding of independent scan pairs.

Scan pairs are independent forwards (models/PointDSC.py:128-197 has no
cross-pair state), so a job of P pairs is split across W ranks with no
data-path collective.  The split is strided like the reference's
``DistributedSampler(shuffle=False)`` (evaluation/test_KITTI.py:246-251) but
without its padding duplicates: rank r owns pairs r, r+W, r+2W, ...  The only
collectives are at the end: one all-gather of per-pair result rows (the
reference gathers its 14-float stat vectors with an all-reduce,
test_KITTI.py:169-170, and test.py:47-63 gathers files) and a reduce of the
throughput counters.  On MI355X the process group is ``nccl`` (= RCCL over
xGMI) with device tensors; on CPU (tests) ``gloo``.
"""
import torch
import torch.distributed as dist


def world():
    """(rank, world_size) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_indices(n_items, rank, world_size):
    """Pair indices owned by `rank`: strided, no padding, disjoint, covering."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} of world {world_size}")
    return list(range(rank, n_items, world_size))


def shard_count(n_items, rank, world_size):
    return len(range(rank, n_items, world_size))


def gather_rows(rows, n_items, device=None):
    """All-gather each rank's [n_r, C] result rows (rank r holds the rows of
    shard_indices(n_items, r, W) in order) and return the [n_items, C] matrix
    in global pair order on every rank.  One all_gather of equal-sized padded
    blocks (row counts are known from the strided split, so no count
    exchange is needed)."""
    rank, W = world()
    rows = torch.as_tensor(rows)
    if rows.dim() != 2 or rows.shape[0] != shard_count(n_items, rank, W):
        raise ValueError(f"rank {rank}: rows {tuple(rows.shape)} but owns {shard_count(n_items, rank, W)} pairs")
    if not (dist.is_available() and dist.is_initialized()):  # no process group: nothing to gather
        return rows.clone()
    dev = device if device is not None else rows.device
    per = shard_count(n_items, 0, W)  # rank 0 owns the most
    C = rows.shape[1]
    block = torch.zeros((per, C), dtype=rows.dtype, device=dev)
    block[: rows.shape[0]] = rows.to(dev)
    blocks = [torch.empty_like(block) for _ in range(W)]
    dist.all_gather(blocks, block)
    out = torch.empty((n_items, C), dtype=rows.dtype, device=dev)
    for r in range(W):
        n_r = shard_count(n_items, r, W)
        out[r::W] = blocks[r][:n_r]
    return out


def job_throughput(units, seconds, device=None):
    """(total units over all ranks, max seconds over ranks): the whole-job
    rate is their ratio (the slowest rank bounds the job)."""
    rank, W = world()
    if not (dist.is_available() and dist.is_initialized()):
        return float(units), float(seconds)
    dev = device if device is not None else torch.device("cpu")
    u = torch.tensor([float(units)], dtype=torch.float64, device=dev)
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=dev)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(u.item()), float(t.item())
