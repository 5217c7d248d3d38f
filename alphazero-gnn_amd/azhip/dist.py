"""Multi-GPU plumbing for the self-play / train loop: one process per GPU,
torch.distributed with backend "nccl" (RCCL over xGMI) on the GPU box, "gloo" in CPU tests.

* self-play shards by episode: episode e is played by rank e mod P with its own
  RandomState(seed(e)); the example lists are gathered on every rank and re-ordered by episode
  index, so the training data is identical for any P (and equal to a 1-rank run);
* the global host RNG streams (`random`, `np.random`) are seeded identically on every rank at
  the start of Coach.learn, so shuffles, batch sampling (np.random.randint,
  Connect4GNN.py:142-143) and arena tie-breaks agree across ranks;
* train (args.train_parallel):
  "replicas" (default) -- every rank runs the identical step, no collective: the kernels are
  deterministic (no float atomics), so parameters stay bit-identical, which `params_in_sync`
  checks with one scalar all-reduce;
  "allreduce" -- data parallel over the sampled rows (azhip/train.py): the CNN step's rows are
  split over ranks (loss normalised by the global batch) and the flat 188 KB gradient is summed
  with one all_reduce; the GNN step uses SURVEY.md §8e's scheme (row-sharded trunk, gathered
  features, the star's row-0 layer stack on every rank, own-row output_transform / heads / loss,
  gradient all_reduce(SUM)) in one of two gradient-exchange forms (args.gnn_grad_sync):
  "row0" (default) broadcasts d loss / d x_L[0] (12.5 KB) so every rank computes the identical
  layer gradients itself and only output_transform's 78.7 MB is all-reduced; "flat" is the
  literal one-bucket all_reduce of the whole 478.6 MB gradient (layer parts from row 0's owner).
  DESIGN.md §5 says why "replicas" stays the default.
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


def broadcast_(t, src=0):
    if dist_ok():
        import torch.distributed as dist
        dist.broadcast(t, src=src)
    return t


def gather_rows(own, n, world, rank):
    """The [n, F] matrix whose rows row_shard(n, world, r) are rank r's `own` rows, on every
    rank.  RCCL: one all_gather_into_tensor of equal-size padded shards.  Other backends (gloo
    cannot all-gather device tensors): an all_reduce(SUM) of a zero matrix holding only this
    rank's rows -- exact, since every element is one rank's value plus zeros."""
    r0, r1 = row_shard(n, world, rank)
    F = own.shape[1]
    if not dist_ok():
        return own.contiguous()
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        m = -(-n // world)
        pad = torch.zeros((m, F), dtype=own.dtype, device=own.device)
        pad[:r1 - r0] = own
        buf = torch.empty((world * m, F), dtype=own.dtype, device=own.device)
        dist.all_gather_into_tensor(buf, pad)
        parts = [buf[r * m:r * m + (row_shard(n, world, r)[1] - row_shard(n, world, r)[0])]
                 for r in range(world)]
        return torch.cat(parts)
    full = torch.zeros((n, F), dtype=own.dtype, device=own.device)
    full[r0:r1] = own
    dist.all_reduce(full, op=dist.ReduceOp.SUM)
    return full


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
