"""Instance sharding across GPUs (BASELINE configs[4]: contiguous blocks of instances per GPU).

The MPCC instances are independent, so the batch shards with no data-path collective; the only
exchange is the gather of the optimal first inputs u0 (what a fleet controller dispatches), one RCCL
all-gather over xGMI per control step (backend "nccl" is RCCL on ROCm; "gloo" for CPU tests).
"""
import torch
import torch.distributed as dist


def shard_bounds(n_total: int, rank: int, world: int):
    """Contiguous shard [start, start + count) of rank among world (the first n % world ranks get one
    more instance)."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("invalid shard request")
    base, rem = divmod(n_total, world)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def check_equal_shards(n_local: int, device=None, group=None) -> None:
    """gather_u0 concatenates equal blocks: raise on every rank unless all ranks hold n_local instances
    (shard_bounds gives unequal blocks when the total is not a multiple of the world size)."""
    t = torch.tensor([n_local, -n_local], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if int(t[0]) != n_local or int(-t[1]) != n_local:
        raise ValueError(f"unequal shards: instances per rank range over [{int(-t[1])}, {int(t[0])}]")


def gather_u0(u_local: torch.Tensor, world: int, out: torch.Tensor = None, group=None) -> torch.Tensor:
    """All-gather equal-size per-rank u0 blocks [B_local, 8] -> [world * B_local, 8] on every rank
    (check the sizes once with check_equal_shards)."""
    if world == 1 and not dist.is_initialized():
        return u_local
    if out is not None and out.shape[0] != world * u_local.shape[0]:
        raise ValueError(f"gather_u0: out has {out.shape[0]} rows, expected {world} x {u_local.shape[0]}")
    if out is None:
        out = torch.empty((world * u_local.shape[0],) + tuple(u_local.shape[1:]), dtype=u_local.dtype,
                          device=u_local.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, u_local.contiguous(), group=group)
    else:
        dist.all_gather_into_tensor(out, u_local.contiguous(), group=group)
    return out


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a scalar over ranks (the bench's elapsed time)."""
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
