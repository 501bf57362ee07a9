"""Multi-GPU sharding of a robot batch.

Robots are independent QPs (mpc.py:262-290 couples nothing across robots), so a
node shards the batch into contiguous ranges, one process per GPU, and the only
exchange is the end-of-step gather of the first-step GRFs u0 (48 B/robot) to
every rank -- e.g. back to the simulator that owns the whole batch
(isaacgym_a1.py:161-164).  With the "nccl" backend this is RCCL over xGMI.
"""
import torch
import torch.distributed as dist


def shard(total, rank, world):
    """Contiguous [start, start+count) range of robots owned by `rank`."""
    base, rem = divmod(int(total), int(world))
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def gather_u0(u0_local, total=None, group=None):
    """All-gather per-rank u0 [B_r, 12] into [sum B_r, 12] in rank order.

    Uneven shards are padded to the largest shard for the collective and the
    padding is dropped afterwards.
    """
    world = dist.get_world_size(group)
    if world == 1:
        return u0_local
    if u0_local.is_cuda and dist.get_backend(group) == "gloo":   # gloo is a host backend
        return gather_u0(u0_local.cpu(), total, group).to(u0_local.device)
    b = u0_local.shape[0]
    if total is None:
        counts = [b] * world
    else:
        counts = [shard(total, r, world)[1] for r in range(world)]
    bmax = max(counts)
    if b < bmax:
        pad = torch.zeros((bmax - b, u0_local.shape[1]), dtype=u0_local.dtype, device=u0_local.device)
        u0_local = torch.cat([u0_local, pad])
    out = torch.empty((world * bmax, u0_local.shape[1]), dtype=u0_local.dtype, device=u0_local.device)
    dist.all_gather_into_tensor(out, u0_local.contiguous(), group=group)
    if all(c == bmax for c in counts):
        return out
    return torch.cat([out[r * bmax:r * bmax + counts[r]] for r in range(world)])
