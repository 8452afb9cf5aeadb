"""CPU, world_size 2 over gloo: the multi-GPU decomposition (aux + grid shards,
one-electron terms on rank 0, all-reduce of sigma) reproduces the full operator.

The arithmetic per rank is the oracle on the rank's slice (no GPU here); the
sharding (``xtddft_amd.parallel.shard_range``) and the collective
(``allreduce_sigma``) are the production code paths used by bench.py and
``ShardedOperator``.
"""
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slice(mf, p, g):
    from xtddft_amd.meanfield import Grid
    m = copy.copy(mf)
    m.cderi = mf.cderi[p[0]:p[1]]
    if mf.cderi_lr is not None:
        m.cderi_lr = mf.cderi_lr[p[0]:p[1]]
    if mf.grids is not None:
        m.grids = Grid(ao=mf.grids.ao[:, g[0]:g[1]], weights=mf.grids.weights[g[0]:g[1]])
        m.fxc = mf.fxc[..., g[0]:g[1]]
        m.fxc_sf = mf.fxc_sf[g[0]:g[1]]
        if mf.fxc_sf_mc is not None:
            m.fxc_sf_mc = mf.fxc_sf_mc[..., g[0]:g[1]]
    return m


def _worker(rank, world, port, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import sf_tda as osf
    from oracle import xtda as oxtda
    from xtddft_amd.parallel import allreduce_sigma, shard_range
    from xtddft_amd.synthetic import make_mf, make_trial_vectors
    mf = make_mf(nao=14, nc=3, no=2, xctype="GGA", hyb=0.2, omega=0.3, alpha=0.6)

    def op(m):
        if kind == "XTDA":
            return oxtda.gen_tda_operation(m)[0]
        return osf.gen_tda_operation_sf(m, -1, method=1 if kind == "SF_DOWN_MC" else 0)[0]
    p = shard_range(mf.naux, rank, world)
    g = shard_range(mf.grids.ngrid, rank, world)
    full = op(mf)
    z = make_trial_vectors(3, (5 * 9 + 3 * 11) if kind == "XTDA" else 5 * 11)
    s = op(_slice(mf, p, g))(z)
    if rank != 0:   # one-electron terms only on rank 0
        s = s - op(_slice(mf, (0, 0), (0, 0)))(z)
    t = torch.from_numpy(np.ascontiguousarray(s))
    allreduce_sigma(t)
    if rank == 0:
        ref = full(z)
        q.put(float(np.abs(t.numpy() - ref).max() / np.abs(ref).max()))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["XTDA", "SF_DOWN", "SF_DOWN_MC"])
def test_sharded_sum_equals_full_operator(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    err = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert err < 1e-13


def _device_mf_host(rank, world):
    """bench.py's synthetic generator (block-seeded; torch CPU generator here) for this
    rank's shard, as host arrays for the oracle."""
    from xtddft_amd.meanfield import Grid
    from xtddft_amd.synthetic import make_device_mf
    m = make_device_mf(nao=14, nc=3, no=2, naux=40, ngrid=3000, torch_device="cpu", shard=(rank, world))
    m.cderi = m.cderi.numpy()
    m.grids = Grid(ao=m.grids.ao.numpy(), weights=m.grids.weights.numpy())
    m.fxc, m.fxc_sf = m.fxc.numpy(), m.fxc_sf.numpy()
    return m


def _worker_lockstep(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import xtda as oxtda
    from xtddft_amd.parallel import LockstepError, agree_min, allreduce_sigma, lockstep_check
    from xtddft_amd.synthetic import make_trial_vectors
    out = {}
    # (a) the shards of the block-seeded generator: partial sigma all-reduced == 1-rank operator
    part = _device_mf_host(rank, world)
    z = make_trial_vectors(3, 5 * 9 + 3 * 11)
    s = oxtda.gen_tda_operation(part)[0](z)
    if rank != 0:   # one-electron terms only on rank 0
        s = s - oxtda.gen_tda_operation(_slice(part, (0, 0), (0, 0)))[0](z)
    t = torch.from_numpy(np.ascontiguousarray(s))
    allreduce_sigma(t)
    ref = oxtda.gen_tda_operation(_device_mf_host(0, 1))[0](z)
    out["shard_err"] = float(np.abs(t.numpy() - ref).max() / np.abs(ref).max())
    # (b) the replicated Davidson's guard: equal decisions pass, a diverged rank raises everywhere
    lockstep_check(np.array([3.0, 1.5, 0.0]), "equal")
    try:
        lockstep_check(np.array([1.0, float(rank)]), "diverged")
        out["raised"] = False
    except LockstepError:
        out["raised"] = True
    # (c) a rank-local resolution made collectively: the stored exchange only if every rank fits
    out["agree"] = (agree_min(1 if rank == 0 else 0), agree_min(1))
    q.put((rank, out))
    dist.destroy_process_group()


def test_block_seeded_shards_and_lockstep_guard():
    """World 2 over gloo: (a) bench's synthetic mean field generated per rank from global
    block seeds sums (partial sigma, all-reduced) to the 1-rank operator, so a sharded run
    solves the N = 1 problem; (b) ``lockstep_check`` passes identical decision data and
    raises LockstepError on EVERY rank when one rank's data differ (no rank left waiting);
    (c) ``agree_min`` gives every rank the same exchange-mode decision (DeviceOperator: the
    stored exchange only when it fits on every rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_lockstep, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert res[0]["shard_err"] < 1e-13
    assert res[0]["raised"] and res[1]["raised"]
    assert res[0]["agree"] == res[1]["agree"] == (0, 1)
