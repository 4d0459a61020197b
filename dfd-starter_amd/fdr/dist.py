"""Multi-GPU sharding of the FD step (DESIGN.md "Multi-GPU").

One process per GPU; the perturbation set is split into contiguous lane slices, one per rank:
  * every rank draws the FULL index list from its own copy of the shared noise table stream, in
    the reference's order (utils/noise_sources.py:44-47), and keeps its slice -- no index exchange;
  * antithetic pairs are never split across ranks (slices are whole directions);
  * the data-path exchange per FD step (z-score, antithetic, the default) is ONE all-reduce of the f64
    moments [A | B | n | r' slots] (2P + 1 + n_lanes doubles: each rank's r' at its global lanes, so the
    sum carries every return for the global z-score, learner/finite_differences.py:43); centred-rank and
    one-sided steps take (1) an all-gather of the per-lane returns (a few KB) and (2) an all-reduce of g
    (P * 8 bytes).  DSGD then runs replicated and bit-identically on every rank.
Backend "nccl" is RCCL on ROCm (xGMI); the same helpers run on gloo for CPU tests.
"""
import os

import torch
import torch.distributed as dist

# FDR_FORCE_COLLECTIVES=1: a process group of ONE rank still takes the sharded exchange (count / reward all-gathers,
# the moments or gradient all-reduce) -- runs the RCCL code path on a one-GPU box (tests/test_gpu_dist_equivalence.py)
FORCE = os.environ.get("FDR_FORCE_COLLECTIVES") == "1"


def active(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or FORCE


def world_rank(group=None):
    if not active(group):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def lane_range(n_dirs, lanes_per_dir, world, rank):
    """Contiguous [lo, hi) lane slice of `rank`; whole directions only, remainder to the low ranks."""
    base, extra = divmod(n_dirs, world)
    d_lo = rank * base + min(rank, extra)
    d_hi = d_lo + base + (1 if rank < extra else 0)
    return d_lo * lanes_per_dir, d_hi * lanes_per_dir


def exchange_counts(n, device, group=None):
    """Every rank's local count (one all-gather of an int64; a host sync) -> list of ints in rank order."""
    ws, _ = world_rank(group)
    if not active(group):
        return [int(n)]
    t = torch.tensor([int(n)], dtype=torch.int64, device=device)
    counts = torch.empty(ws, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(counts, t, group=group)
    return [int(c) for c in counts.tolist()]


def gather_rewards(local, group=None, sizes=None):
    """All-gather per-lane rewards -> (all rewards in rank order, this rank's offset).

    sizes: every rank's lane count, when the caller knows the split (Worker.evaluate's standard
    lane_range split sets FDBatch.rank_lanes): then the exchange is ONE all-gather issued on the
    stream with no host synchronisation.  Without it the counts are exchanged first (a host sync)."""
    ws, rank = world_rank(group)
    if not active(group):
        return local, 0
    if sizes is None:
        n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
        counts = torch.empty(ws, dtype=torch.int64, device=local.device)
        dist.all_gather_into_tensor(counts, n, group=group)
        sizes = counts.tolist()
    sizes = [int(s) for s in sizes]
    if len(sizes) != ws or sizes[rank] != local.numel():
        raise ValueError("gather_rewards: sizes %s do not match this rank's %d lanes" % (sizes, local.numel()))
    m = max(sizes)
    if local.numel() == m:
        buf = local.contiguous()
    else:
        buf = torch.zeros(m, dtype=local.dtype, device=local.device)
        buf[:local.numel()] = local
    out = torch.empty(ws * m, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    if all(s == m for s in sizes):
        return out, rank * m
    return torch.cat([out[k * m:k * m + s] for k, s in enumerate(sizes)]), sum(sizes[:rank])


def allreduce_grad(g, group=None):
    if active(group):
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=group)
    return g
