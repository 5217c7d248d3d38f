"""Multi-GPU plumbing for the self-play / train loop: one process per GPU,
torch.distributed with backend "nccl" (RCCL over xGMI) on the GPU box, "gloo" in CPU tests.

* self-play shards by episode: episode e is played by rank e mod P with its own
  RandomState(seed(e)); the example lists are gathered on every rank and re-ordered by episode
  index, so the training data is identical for any P (and equal to a 1-rank run);
* the global host RNG streams (`random`, `np.random`) are seeded identically on every rank at
  the start of Coach.learn, so shuffles, batch sampling (np.random.randint,
  Connect4GNN.py:142-143) and arena tie-breaks agree across ranks;
* train: "replicas" (default) -- every rank runs the identical step, no collective: the
  kernels are deterministic (no float atomics), so parameters stay bit-identical, which
  `params_in_sync` checks with one scalar all-reduce; "allreduce" -- the CNN step's 64 rows are
  split over ranks (loss normalised by the global batch) and the flat gradient buffer
  (47,049 floats for Connect4) is summed with one all_reduce before the identical Adam step.
  The GNN step couples all rows through the star's row 0 and its 478.6 MB gradient would cost
  far more on xGMI than the ~20 µs of step compute, so it stays replicated.
"""
import random

import numpy as np
import torch


def dist_ok():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def world_rank():
    if not dist_ok():
        return 1, 0
    import torch.distributed as dist
    return dist.get_world_size(), dist.get_rank()


def my_episodes(num_eps, world, rank):
    """Episodes of this rank: e = rank, rank + P, ... (independent units, no exchange)."""
    return list(range(rank, num_eps, world))


def broadcast_int(x):
    """Rank 0's integer on every rank."""
    if not dist_ok():
        return int(x)
    import torch.distributed as dist
    obj = [int(x)]
    dist.broadcast_object_list(obj, src=0)
    return int(obj[0])


def sync_host_rngs(seed=None):
    """Seed `random` and `np.random` identically on all ranks (rank 0's draw unless given)."""
    if seed is None:
        seed = np.random.randint(0, 2 ** 31 - 1)      # every rank draws: streams stay aligned
    seed = broadcast_int(seed)
    random.seed(seed)
    np.random.seed(seed)
    return seed


def gather_episodes(local):
    """{episode: result} of every rank -> one dict, on every rank."""
    if not dist_ok():
        return dict(local)
    import torch.distributed as dist
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, dict(local))
    out = {}
    for p in parts:
        out.update(p)
    return out


def row_shard(n, world, rank):
    """Contiguous row range [r0, r1) of rank's share of n rows."""
    base, extra = divmod(n, world)
    r0 = rank * base + min(rank, extra)
    return r0, r0 + base + (1 if rank < extra else 0)


def allreduce_sum_(t):
    if dist_ok():
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def params_in_sync(flat):
    """True when this flat parameter buffer is identical on every rank: a position-weighted
    checksum of the raw fp32 bits (int64, wrapping), compared by MIN/MAX all-reduce."""
    if not dist_ok():
        return True
    import torch.distributed as dist
    w = flat.detach().reshape(-1).view(torch.int32).to(torch.int64)
    idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64)
    s = (w * (idx % 65521 + 1)).sum().reshape(1)
    lo, hi = s.clone(), s.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool((lo == hi).item())
