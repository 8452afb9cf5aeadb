"""Multi-GPU sharding of the TDA operator (one process per GPU).

The reference has no distributed code; the design here
is SURVEY.md 8(e)'s contraction-dimension sharding:

* rank r keeps aux functions P in ``shard_range(naux, r, n)`` and grid points
  in ``shard_range(ngrid, r, n)``; everything else (orbitals, Fock, trial
  vectors, the Davidson subspace) is replicated;
* every rank evaluates the partial sigma_r of ALL trial vectors from its
  shard (J, K and XC are sums over P and over grid points, and the MO
  projections are linear, so sigma = sum_r sigma_r); the one-electron terms
  are added on rank 0 only;
* one all-reduce (sum) of sigma per A.x -- ``torch.distributed`` with the
  ``nccl`` backend, i.e. RCCL over xGMI on MI355X (``gloo`` on CPU in tests).

The Davidson control flow is deterministic given identical inputs, so every
rank runs it redundantly on the all-reduced sigma and stays in lockstep; that
assumption is checked, not trusted: ``lockstep_check`` gathers every rank's
decision data each iteration (heff checksum, Ritz values, residual norms, the
convergence flags, the number of new vectors) and raises on every rank at once when
they differ -- a diverged rank would otherwise leave the others waiting in the next
all-reduce forever.
"""
from __future__ import annotations


def shard_range(n: int, rank: int, nranks: int):
    """Contiguous [lo, hi) slice of n items for this rank (remainder to low ranks)."""
    if nranks < 1 or not (0 <= rank < nranks):
        raise ValueError("bad rank / nranks")
    base, rem = divmod(n, nranks)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def allreduce_sigma(sigma, group=None):
    """Sum of the per-rank partial sigma over the process group.

    A torch tensor is reduced in place (through a host copy when the backend
    is gloo and the tensor lives on the GPU, through a device copy when the
    backend is RCCL and it lives on the host); a NumPy array is left untouched
    and the sum is returned as a new array."""
    import numpy as np
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return sigma
    nccl = dist.get_backend(group) == "nccl"
    if isinstance(sigma, np.ndarray):
        t = torch.tensor(np.asarray(sigma, dtype=np.float64))      # a copy: the input stays as it was
        if nccl:     # RCCL reduces device tensors only
            d = t.to(f"cuda:{torch.cuda.current_device()}")
            dist.all_reduce(d, group=group)
            return d.cpu().numpy()
        dist.all_reduce(t, group=group)
        return t.numpy()
    if not sigma.is_cuda and nccl:
        d = sigma.to(f"cuda:{torch.cuda.current_device()}")
        dist.all_reduce(d, group=group)
        sigma.copy_(d)
        return sigma
    if sigma.is_cuda and dist.get_backend(group) == "gloo":
        h = sigma.cpu()
        dist.all_reduce(h, group=group)
        sigma.copy_(h)
        return sigma
    dist.all_reduce(sigma, group=group)
    return sigma


def agree_min(value: int, group=None, device=None) -> int:
    """The minimum of an integer decision over the process group (the value itself
    outside a multi-rank group).  Used where a rank-local resolution must be made
    collectively, e.g. whether the stored exchange fits (DeviceOperator): ranks that
    stream stored exchange ROWS and ranks that contract an aux WINDOW directly would
    not sum to the operator.  ``device``: the GPU of the caller's operator (RCCL reduces
    device tensors; default the current device)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64)
    if dist.get_backend(group) == "nccl":
        t = t.to(f"cuda:{torch.cuda.current_device() if device is None else int(device)}")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item())


class LockstepError(RuntimeError):
    pass


def group_size(group=None):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def lockstep_check(values, what="", group=None):
    """All-gather ``values`` (a flat float64 vector, same length on every rank) and
    raise ``LockstepError`` on EVERY rank when any rank's copy differs bitwise from
    rank 0's.  A no-op without a process group of size > 1."""
    import numpy as np
    import torch
    import torch.distributed as dist
    n = group_size(group)
    if n <= 1:
        return
    v = torch.as_tensor(np.ascontiguousarray(np.asarray(values, dtype=np.float64).ravel()))
    if dist.get_backend(group) == "nccl":      # RCCL gathers device tensors only
        v = v.to(f"cuda:{torch.cuda.current_device()}")
    out = [torch.empty_like(v) for _ in range(n)]
    dist.all_gather(out, v, group=group)
    ref = out[0].cpu().numpy().view(np.int64)
    bad = [r for r in range(1, n) if not np.array_equal(out[r].cpu().numpy().view(np.int64), ref)]
    if bad:
        raise LockstepError(f"replicated Davidson diverged ({what}): ranks {bad} differ from rank 0")


def require_group(nranks):
    """A driver sharded over nranks > 1 needs the torch.distributed group that
    sums its partial sigma; refuse to run on 1/nranks of the operator."""
    import torch.distributed as dist
    if nranks > 1 and not (dist.is_available() and dist.is_initialized()
                           and dist.get_world_size() == nranks):
        raise ValueError(f"shard over {nranks} ranks needs an initialised torch.distributed "
                         f"group of that size (the partial sigma must be all-reduced)")


class ShardedOperator:
    """sigma = sum_r A_r z: a rank-local DeviceOperator followed by the all-reduce."""

    def __init__(self, mf, kind, rank=None, nranks=None, device=None, presharded=False, **kw):
        import torch
        import torch.distributed as dist
        from .operator import DeviceOperator
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        if nranks is None:
            nranks = dist.get_world_size() if dist.is_initialized() else 1
        if device is None:
            device = torch.cuda.current_device()
        self.rank, self.nranks = rank, nranks
        self.op = DeviceOperator(mf, kind, shard=(rank, nranks), device=device,
                                 presharded=presharded, **kw)
        self.dim = self.op.dim

    def apply(self, zs):
        import torch
        if not (isinstance(zs, torch.Tensor) and zs.is_cuda):
            raise TypeError("ShardedOperator works on device tensors")
        return allreduce_sigma(self.op.apply(zs))

    __call__ = apply
