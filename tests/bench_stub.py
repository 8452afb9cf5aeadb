"""CPU stand-in for bench.py's operator factory (launcher / rank-plumbing test).

TEST INFRASTRUCTURE ONLY: selected with XT_BENCH_OPERATOR=bench_stub:make_workload
(tests/test_bench_launch.py).  Each rank evaluates the oracle A.x on ITS shard of
the contraction dimensions, split exactly as DeviceOperator splits them
(``shard_range`` of the aux rows and grid points, one-electron terms on rank 0
only), so the all-reduced sigma equals the full operator -- which ``verify``
checks on rank 0 against the unsharded oracle.
"""
import dataclasses
import time

import numpy as np
import torch

from oracle import xtda as oxtda
from xtddft_amd.meanfield import Grid
from xtddft_amd.parallel import shard_range
from xtddft_amd.synthetic import make_mf


class _StubOp:
    def __init__(self, vind, dim):
        self._vind, self.dim = vind, dim
        self.k_mode, self.k_gib, self.prepare_s = "direct", 0.0, 0.0

    def apply(self, z, out=None):
        s = torch.as_tensor(self._vind(z.numpy()))
        if out is None:
            return s
        out.copy_(s)
        return out

    def set_profile(self, mask):
        pass

    def profile_stats(self):
        return {"oracle_vind": dict(ms=1.0, launches=1, flops=1.0)}

    def last_timings(self):
        return dict(jk_ms=0.0, xc_ms=0.0, local_ms=0.0, total_ms=0.0)


class _Workload:
    def __init__(self, op, mf, full_vind, replicate):
        self.op, self.mf, self.device = op, mf, torch.device("cpu")
        self.t_gen, self.t_op, self.replicate = 0.0, 0.0, replicate
        self._full = full_vind

    def verify(self, z, out):
        ref = self._full(z.numpy())
        return float(np.abs(out.numpy() - ref).max() / np.abs(ref).max())


def make_workload(args, rank, world, local):
    t0 = time.perf_counter()
    mf = make_mf(nao=args.nao, nc=args.nc, no=args.no, naux=args.naux, ngrid=args.ngrid,
                 xctype=args.xc, hyb=args.hyb)
    p0, p1 = shard_range(mf.naux, rank, world)
    g0, g1 = shard_range(mf.grids.ngrid, rank, world)
    part = dataclasses.replace(mf, cderi=mf.cderi[p0:p1],
                               grids=Grid(ao=mf.grids.ao[:, g0:g1], weights=mf.grids.weights[g0:g1]),
                               fxc=mf.fxc[..., g0:g1], fxc_sf=mf.fxc_sf[g0:g1])
    vind_part, _ = oxtda.gen_tda_operation(part)
    if rank == 0:
        vind = vind_part
    else:
        # drop the one-electron terms every partial carries (they are added once, on rank 0)
        zero = dataclasses.replace(part, cderi=np.zeros((1, mf.nao, mf.nao)), fxc=part.fxc * 0.0)
        vind_1e, _ = oxtda.gen_tda_operation(zero)

        def vind(z):
            return vind_part(z) - vind_1e(z)
    full, hdiag = oxtda.gen_tda_operation(mf)
    w = _Workload(_StubOp(vind, hdiag.size), mf, full, replicate=False)
    w.t_gen = time.perf_counter() - t0
    return w
