#!/usr/bin/env python
"""Benchmark: TDA A.x throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config H|C1..C5|C4d]

With ``--gpus N > 1`` outside a torch.distributed launch, this process starts
``torch.distributed.run`` with N ranks (one process per GPU, RCCL over xGMI)
before it touches the GPU and exits with the launcher's status; under
torchrun (WORLD_SIZE set) it runs as one rank.

Workload (default ``H``): the BASELINE headline shape -- synthetic ROKS X-TDA,
nao = 1000, nocc_a/nocc_b = 101/99 (nc 99, no 2, nv 899), naux = 3 nao,
ngrid = 1200 nao, GGA kernel + global hybrid (hyb 0.2), nvec = 20 trial
vectors per A.x.  A "step" is one full A.x on the nvec-vector batch (plus the
all-reduce of sigma when N > 1).  value = matvecs/s = nvec * K / T, T the max
over ranks of the barrier + synchronise bracketed wall time of the K steps.
The other BASELINE.json configs are parity-test shapes (tests/test_gpu_configs.py);
``--config`` prints their lines for DESIGN.md.

Multi-GPU: the grid is sharded over ranks and the DF factor replicated with an
aux window + a row block of the stored exchange per rank (``DeviceOperator``
partition); each rank computes a partial sigma of all vectors, one all-reduce
sums them: fixed total work, "scaling": "strong".

Extra JSON fields: roofline (dominant GEMM class timed live with HIP events on
the library's stream over the timed steps; traffic from this config's committed
rocprofv3 PMC summary), cpu_baseline (the NumPy oracle = the reference's AO
route, timed on this host's cores), converge (wall time of the device Davidson
to nroots with the reference's criteria, including operator construction).

``XT_BENCH_OPERATOR=module:function`` replaces the operator factory (the CPU
launcher test uses a stub from tests/); ``XT_BENCH_BACKEND=gloo`` rehearses the
N-rank path with ranks sharing the visible GPU(s).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6     # MI355X dense FP64 matrix peak (AMD spec); 74.2 measured (tools/mfma_probe.hip)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec
# this round's committed rocprofv3 FETCH / WRITE summary (tools/parse_prof.py): the only one
# roofline.traffic is read from (an older round's bytes would describe older kernels)
ROUND = 6
PMC_SUMMARY = os.path.join(ROOT, "profiles", f"r{ROUND:02d}_pmc_summary.json")

CPU_CONVERGE_AUTO_S = 60.0
WARM_FULL_DIM = 20000        # converge(): a whole untimed warm-up solve below this dimension   # bench's default run times the CPU Davidson only when it is this short

KIND_NAME = {"XTDA": "X-TDA", "SF_UP": "SF-TDA (spin-flip up)", "SF_DOWN": "SF-TDA (spin-flip down)",
             "XSF": "XSF-TDA"}

# BASELINE.json configs as synthetic shapes (SURVEY.md 8 shape table): nao, closed /
# open shells, operator, vectors per A.x (= nroots), hybrid fraction, J/K model.
# C4 (C60- doublet) is ill-posed for spin adaptation (XSF divides by 2S - 1 = 0,
# XSF_TDA.py:1102-1121): C4 is the quartet shape (no = 3, SA = 3, OO compressed),
# C4d the doublet at SA = 0.  C5 is the exact-K path: stored 8-fold ERIs.
CONFIGS = {
    "H": dict(nao=1000, nc=99, no=2, kind="XTDA", nvec=20, nroots=20, hyb=0.2),
    "C1": dict(nao=13, nc=3, no=2, kind="XTDA", nvec=5, nroots=5, hyb=0.2, ngrid=35000),
    "C2": dict(nao=180, nc=33, no=1, kind="XTDA", nvec=20, nroots=20, hyb=0.2),
    "C3": dict(nao=861, nc=91, no=4, kind="SF_UP", nvec=30, nroots=30, hyb=0.5),
    "C4": dict(nao=840, nc=179, no=3, kind="XSF", nvec=40, nroots=40, hyb=0.5, sa=3, remove=True),
    "C4d": dict(nao=840, nc=180, no=1, kind="XSF", nvec=40, nroots=40, hyb=0.5, sa=0, remove=True),
    "C5": dict(nao=152, nc=35, no=2, kind="XTDA", nvec=50, nroots=50, hyb=0.2, jk="ERI8"),
    # C3 with the multicollinear spin-flip kernel (method=1, SF_TDA.py:855-1047)
    "C3mc": dict(nao=861, nc=91, no=4, kind="SF_UP", nvec=30, nroots=30, hyb=0.5, method=1),
}
CONFIG_NAMES = {"H": "headline", "C1": "CH2 triplet / 6-31G", "C2": "naphthalene+ / def2-SVP",
                "C3": "Fe(II)P quintet / def2-TZVP", "C4": "C60-like quartet / def2-SVP",
                "C4d": "C60- doublet / def2-SVP", "C5": "[Cu2O2]2+ triplet / def2-TZVP",
                "C3mc": "Fe(II)P quintet / def2-TZVP, multicollinear kernel"}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="H", choices=sorted(CONFIGS),
                    help="BASELINE.json shape preset (synthetic data of that shape)")
    ap.add_argument("--nao", type=int, default=None)
    # (long names: torch.distributed.run re-parses the script's argv and rejects
    # abbreviations of its own options such as --no / --node-rank)
    ap.add_argument("--nclosed", dest="nc", type=int, default=None)
    ap.add_argument("--nopen", dest="no", type=int, default=None)
    ap.add_argument("--naux", type=int, default=None)
    ap.add_argument("--ngrid", type=int, default=None)
    ap.add_argument("--nvec", type=int, default=None)
    ap.add_argument("--nroots", type=int, default=None)
    ap.add_argument("--xc", default="GGA")
    ap.add_argument("--hyb", type=float, default=None)
    ap.add_argument("--kind", default=None, choices=["XTDA", "SF_UP", "SF_DOWN", "XSF"])
    ap.add_argument("--sa", type=int, default=None, help="XSF spin-adaptation level (XSF_TDA.py SA)")
    ap.add_argument("--jk", default=None, choices=["DF", "ERI8"])
    ap.add_argument("--method", type=int, default=None, choices=[0, 1],
                    help="spin-flip XC kernel: 0 ALDA0, 1 multicollinear (SF / XSF kinds)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-converge", action="store_true")
    ap.add_argument("--converge", action="store_true", help="force the Davidson run (default on; see --no-converge)")
    ap.add_argument("--cpu-converge", default="auto", choices=["auto", "on", "off"],
                    help="time the oracle Davidson to nroots on the host (auto: when the CPU A.x "
                         "rate puts it under CPU_CONVERGE_AUTO_S)")
    ap.add_argument("--k-mode", default="auto", choices=["auto", "direct", "stored"],
                    help="exchange evaluation (xt_set_exchange_mode)")
    args = ap.parse_args(argv)
    preset = dict(sa=0, remove=False, jk="DF", ngrid=None, method=0)
    preset.update(CONFIGS[args.config])
    # a shape overridden on the command line is not the profiled preset: its PMC
    # bytes (roofline.traffic) are unmeasured
    args.custom = any(getattr(args, k, None) is not None
                      for k in ("nao", "nc", "no", "naux", "ngrid", "nvec", "hyb", "kind", "sa", "jk", "method"))
    for k, v in preset.items():
        if getattr(args, k, None) is None:
            setattr(args, k, v)
    args.nv = args.nao - args.nc - args.no
    args.naux = args.naux or 3 * args.nao
    args.ngrid = args.ngrid or 1200 * args.nao
    return args


# ---------------------------------------------------------------------------
# launcher: N ranks under torch.distributed.run, started before any GPU use
# ---------------------------------------------------------------------------
def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------
# the operator under test
# ---------------------------------------------------------------------------
class Workload:
    """What a factory returns: the operator, its mean field, the torch device the
    trial vectors live on, and the setup split (synthetic generation vs operator
    construction = MO transforms + xt_prepare).  ``regen()`` (device workloads) returns
    the operator's input mean field again, bit-identical (same block seeds): what the
    cpu_baseline leg hands the oracle."""

    def __init__(self, op, mf, device, t_gen, t_op, replicate, regen=None):
        self.op, self.mf, self.device = op, mf, device
        self.t_gen, self.t_op, self.replicate = t_gen, t_op, replicate
        self.regen = regen


def _eri8_from_device_factor(cderi):
    """8-fold packed ERIs (mu nu|la si) = sum_P B B from a device DF factor
    (synthetic exact-K input; PySCF 's8' order, ij = i(i+1)/2 + j)."""
    import torch
    nao = cderi.shape[1]
    ii, jj = torch.tril_indices(nao, nao, device=cderi.device)
    b2 = cderi[:, ii, jj]                       # (naux, npair)
    e = b2.T @ b2                               # (npair, npair)
    pi, pj = torch.tril_indices(e.shape[0], e.shape[0], device=cderi.device)
    return e[pi, pj].contiguous()


def device_workload(args, rank, world, local):
    import torch
    from xtddft_amd.operator import DeviceOperator
    from xtddft_amd.synthetic import make_device_mf
    from xtddft_amd.xsf_tda import get_vect
    replicate = world > 1 and args.k_mode != "direct"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gen_kw = dict(nao=args.nao, nc=args.nc, no=args.no, naux=args.naux, ngrid=args.ngrid,
                  xctype=args.xc, hyb=args.hyb, device=local, shard=(rank, world),
                  full_aux=replicate or args.jk == "ERI8", sf_mc=args.method == 1)
    mf = make_device_mf(**gen_kw)
    if args.jk == "ERI8":
        mf.eri = _eri8_from_device_factor(mf.cderi)
        mf.cderi = None
        mf.chol_tol = 0.0
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0
    kw = {}
    if args.kind == "XSF":
        # XSF_TDA.kernel default fglobal = (1 - d_lda) c_x + d_lda, d_lda = 0.3, c_x = hyb
        kw = dict(sa=args.sa, fglobal=0.7 * args.hyb + 0.3, foo=1.0, remove=bool(args.remove))
    t1 = time.perf_counter()
    if args.method == 1:
        kw.update(sf_kernel="mc", mc_kernel=mf.fxc_sf_mc)
    op = DeviceOperator(mf, args.kind, shard=(rank, world), device=local, **kw,
                        presharded="grid" if (replicate or args.jk == "ERI8") else True,
                        k_mode=args.k_mode, replicate_df=replicate)
    if args.kind == "XSF" and args.remove:
        op.set_oo_basis(get_vect(args.no))
    torch.cuda.synchronize()
    t_op = time.perf_counter() - t1
    mf.cderi = None
    mf.eri = None
    mf.grids = None
    mf.fxc = None
    mf.fxc_sf = None
    mf.fxc_sf_mc = None
    torch.cuda.empty_cache()
    return Workload(op, mf, torch.device(f"cuda:{local}"), t_gen, t_op, replicate,
                    regen=lambda: make_device_mf(**gen_kw))


def _factory():
    spec = os.environ.get("XT_BENCH_OPERATOR")
    if not spec:
        return device_workload
    mod, fn = spec.split(":")
    return getattr(importlib.import_module(mod), fn)


# ---------------------------------------------------------------------------
# CPU baseline: the oracle on this host's cores
# ---------------------------------------------------------------------------
def cpu_share():
    """CPUs this process may use: the affinity mask, capped by the cgroup CPU quota
    (cpu.max) when one is set -- on a shared GPU box the quota, not os.cpu_count(),
    is what BLAS threads can actually run on."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                quota, period = f.read().split()[:2]
            if quota != "max":
                n = min(n, max(1, int(float(quota) / float(period))))
        except (OSError, ValueError):
            pass
    return n


def _host_info():
    """CPU model and BLAS build of the host timing the CPU baseline."""
    info = {"host_cpus": os.cpu_count(), "cpu_share": cpu_share()}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["cpu"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        from threadpoolctl import threadpool_info
        info["blas"] = [f"{i.get('internal_api')} {i.get('version')} threads={i.get('num_threads')}"
                        for i in threadpool_info()]
    except Exception:
        pass
    return info


def _oracle_vind(args, mf, with_hdiag=False):
    from oracle import sf_tda as osf
    from oracle import xsf_tda as oxsf
    from oracle import xtda as oxtda
    if args.kind == "XTDA":
        return oxtda.gen_tda_operation(mf)
    if args.kind in ("SF_UP", "SF_DOWN"):
        return osf.gen_tda_operation_sf(mf, 1 if args.kind == "SF_UP" else -1, method=args.method)
    o = oxsf.XSFOracle(mf, SA=args.sa, method=args.method)
    o.re = bool(args.remove)
    if o.re and o.no > 1:
        o.vects = oxsf.get_vect(o.no)
    # the preconditioner's J diagonals are solver setup, not A.x: built only for a solve
    return o.gen_tda_operation_sf(fglobal=0.7 * args.hyb + 0.3, with_hdiag=with_hdiag)


def log(msg):
    """Progress to stderr (long phases must keep writing: the GPU box kills silent runs)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _time_call(f, reps, what=""):
    t0 = time.perf_counter()
    f()                                  # 1 warm-up
    log(f"cpu baseline {what}: warm-up {time.perf_counter() - t0:.2f} s")
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
        log(f"cpu baseline {what}: {ts[-1]:.2f} s")
    return float(np.median(ts))


class _DevSlicer:
    """A device tensor the oracle reads block by block: ``x[key]`` copies that block to
    host memory (the oracle walks the grid in oracle.engines.GRID_BLOCK-point blocks), so
    the full-size grid data never has to fit in host memory at once."""

    def __init__(self, t):
        self.t, self.shape = t, tuple(t.shape)

    def __getitem__(self, key):
        return self.t[key].cpu().numpy()


def oracle_meanfield(args, w):
    """The timed operator's own input data for the oracle: the workload's synthetic mean
    field regenerated bit-identically on the device (``Workload.regen``: same seeds, same
    block generators), the DF factor (or the stored ERIs it defines) copied to host
    memory, the grid data copied too when small, else read from HBM block by block."""
    import dataclasses
    from oracle.engines import eri_full_from_cderi
    from xtddft_amd.meanfield import Grid
    mf = w.regen()
    cd = mf.cderi.cpu().numpy()
    small = 8.0 * 4 * args.ngrid * args.nao < 4e9
    conv = (lambda t: None if t is None else t.cpu().numpy()) if small else \
        (lambda t: None if t is None else _DevSlicer(t))
    grid = Grid(ao=conv(mf.grids.ao), weights=conv(mf.grids.weights))
    out = dataclasses.replace(mf, cderi=cd, grids=grid, fxc=conv(mf.fxc), fxc_sf=conv(mf.fxc_sf),
                              fxc_sf_mc=conv(mf.fxc_sf_mc), extra=dict(mf.extra))
    if args.jk == "ERI8":
        out.extra["eri_full"] = eri_full_from_cderi(cd)
    return out, small


def cpu_baseline(args, w, z0, s0):
    """The oracle's A.x (the reference's AO-route algorithm, NumPy/BLAS) on ALL host
    cores, on the SAME data and the SAME trial vector as the timed device steps.

    Threads: every CPU this process may run on (``cpu_share``: the host's CPUs capped by
    the cgroup quota of a shared GPU box; more BLAS threads than the quota only
    oversubscribe it).  Data: ``oracle_meanfield`` (the timed operator's inputs).  Shapes
    whose grid data fit host memory comfortably are timed 1 warm-up + median of 5; the
    large ones as ONE call at the full naux and ngrid (after a warm-up call on a small
    synthetic problem), the grid streamed from HBM block by block -- nothing extrapolated.
    The exact-K configuration contracts stored 4-index ERIs (the incore mf._eri route).
    Returns (cpu_baseline dict in matvecs/s, verify dict): ``verify.rel_err`` = max |sigma_gpu
    - sigma_oracle| / max |sigma_oracle| for the first vector of the timed batch."""
    from threadpoolctl import threadpool_info, threadpool_limits
    from oracle.engines import GRID_BLOCK
    from xtddft_amd.synthetic import make_mf, make_trial_vectors
    ncpu = cpu_share()
    t_all = time.perf_counter()
    with threadpool_limits(limits=ncpu):
        threads = max([i.get("num_threads", 1) for i in threadpool_info()
                       if i.get("user_api") == "blas"] or [1])
        log(f"cpu baseline on {threads} BLAS threads ({ncpu} CPUs in this process's share, "
            f"{os.cpu_count()} on the host)")
        t0 = time.perf_counter()
        mfo, small = oracle_meanfield(args, w)
        log(f"cpu baseline: the timed operator's data regenerated and staged in {time.perf_counter() - t0:.1f} s")
        vind, _ = _oracle_vind(args, mfo)
        res = {}

        def call():
            res["s"] = vind(z0)
        if small:
            t = _time_call(call, 5, "full size")
            how = f"timed at the full size (naux={args.naux}, ngrid={args.ngrid}), 1 warm-up + median of 5"
        else:
            warm = make_mf(nao=args.nao, nc=args.nc, no=args.no, naux=16, ngrid=2 * GRID_BLOCK,
                           xctype=args.xc, hyb=args.hyb)
            vind_s, hd = _oracle_vind(args, warm)
            t0 = time.perf_counter()
            vind_s(make_trial_vectors(1, hd.size))          # warms BLAS threads and allocators
            log(f"cpu baseline warm-up (naux=16, ngrid={2 * GRID_BLOCK}): {time.perf_counter() - t0:.2f} s")
            log(f"cpu baseline: one call at naux={args.naux}, ngrid={args.ngrid} (grid read from HBM)")
            t0 = time.perf_counter()
            call()
            t = time.perf_counter() - t0
            log(f"cpu baseline naux={args.naux} ngrid={args.ngrid}: {t:.2f} s")
            how = (f"one call timed at the full naux={args.naux} and the full ngrid={args.ngrid} (the grid "
                   f"data read from HBM in {GRID_BLOCK}-point blocks, included), after a warm-up call on "
                   f"a small synthetic problem")
    s_or = np.asarray(res["s"]).reshape(s0.shape)
    err = float(np.abs(s0 - s_or).max() / np.abs(s_or).max())
    log(f"verify: max |sigma_gpu - sigma_oracle| / max |sigma_oracle| = {err:.3e}")
    del mfo
    import torch
    torch.cuda.empty_cache()
    cpu = dict(value=1.0 / t, unit="matvecs/s", cores=int(threads), kind="port",
               sample=(f"oracle {KIND_NAME[args.kind]} vind (NumPy AO route, "
                       f"{'stored 4-index ERI' if args.jk == 'ERI8' else 'DF'} J/K, {args.xc}) on 1 vector "
                       f"at nao={args.nao} on the timed operator's own data: {how}; t_vec = {t:.2f} s"),
               host=_host_info(), sample_wall_s=round(time.perf_counter() - t_all, 1))
    verify = dict(rel_err=err, max_abs_sigma=float(np.abs(s_or).max()),
                  what=("max |sigma_gpu - sigma_oracle| / max |sigma_oracle| on the first vector of the timed "
                        "batch, full naux and ngrid, the oracle (reference AO route) on the same data"),
                  tol=1e-12, ok=bool(err <= 1e-12))
    return cpu, verify


# ---------------------------------------------------------------------------
# Davidson to nroots on the same operator (reference criteria per kind)
# ---------------------------------------------------------------------------
def _solver_setup(args, w, dev):
    """(x0, preconditioner, davidson1 keywords, criteria) of the device solve, per kind."""
    mf, op = w.mf, w.op
    from xtddft_amd.davidson import DiagPrecond
    if args.kind == "XTDA":
        from xtddft_amd.xtda import XTDA
        x = XTDA.__new__(XTDA)
        x.mf, x.X, x.nstates, x.device = mf, True, args.nroots, dev.index
        hdiag = x._hdiag()
        x0 = x.get_init_guess(mf, args.nroots)

        def pickeig(wv, v, nroots, envs):
            idx = np.where(wv > 0.001)[0]
            return wv[idx], v[:, idx], idx
        kw = dict(tol_residual=1e-5, lindep=1e-12, pick=pickeig, max_cycle=100)
        return x0, DiagPrecond(hdiag, 0.0, dev.index), kw, "|de|<1e-12, |r|<1e-5, pick w>1e-3 (XTDA.py:769-777)"
    if args.kind in ("SF_UP", "SF_DOWN"):
        from xtddft_amd.sf_tda import init_guess, sf_hdiag
        isf = 1 if args.kind == "SF_UP" else -1
        x0 = init_guess(mf, args.nroots, isf)
        return (x0, DiagPrecond(sf_hdiag(mf, isf), 1e-3, dev.index), dict(tol=1e-7, lindep=1e-14, max_cycle=3000),
                "tol 1e-7, lindep 1e-14 (SF_TDA.py:392-395)")
    from xtddft_amd.xsf_tda import XSF_TDA, get_vect
    x = XSF_TDA(mf, SA=args.sa, device=dev.index)
    x.re = bool(args.remove)
    x.vects = get_vect(args.no)
    x.nstates = args.nroots
    hdiag = x._build_preconditioner_hdiag(0.7 * args.hyb + 0.3, op)
    if x.re:
        hdiag = x._compress_removed_hdiag(hdiag)
    x0 = x.init_guess(args.nroots, hdiag)
    return (x0, DiagPrecond(hdiag, 1e-3, dev.index), dict(tol=1e-8, lindep=1e-9, max_cycle=1000),
            "tol 1e-8, lindep 1e-9 (XSF_TDA.py:1467-1470)")


def converge(args, w, allreduce, world=1):
    """Wall time of the device Davidson to nroots under the reference's criteria (operator
    construction included).  An untimed solve first loads the solver's kernels (first-launch
    costs are not per-solve work: the whole solve up to WARM_FULL_DIM, 2 iterations above);
    the replicated solver of a sharded operator runs with the lockstep guard."""
    import torch
    from xtddft_amd.davidson import davidson1
    op, dev = w.op, w.device
    x0, pre, kw, crit = _solver_setup(args, w, dev)
    stats = dict(calls=0, vectors=0, s=0.0, allreduce_s=0.0, nvec=[])

    def aop(xt):
        t = time.perf_counter()
        s = op.apply(xt)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        allreduce(s)
        torch.cuda.synchronize()
        stats["calls"] += 1
        stats["vectors"] += int(s.shape[0])
        stats["nvec"].append(int(s.shape[0]))
        stats["s"] += t1 - t
        stats["allreduce_s"] += time.perf_counter() - t1
        return s
    # small operators: the whole solve (seconds at most), so every solver path -- dropped
    # vectors, restarts -- has loaded its kernels; large ones: two iterations
    warm = dict(kw, max_cycle=2) if op.dim > WARM_FULL_DIM else kw
    davidson1(lambda xt: allreduce(op.apply(xt)), x0, pre, nroots=args.nroots, device=dev.index,
              return_device=True, lockstep=world > 1, **warm)
    torch.cuda.synchronize()
    log(f"converging {args.nroots} roots")
    phase_s = {}
    tc = time.perf_counter()
    conv, e, _, icyc = davidson1(aop, x0, pre, nroots=args.nroots, device=dev.index,
                                 return_device=True, lockstep=world > 1, stats=phase_s, **kw)
    torch.cuda.synchronize()
    wall = time.perf_counter() - tc
    hist = {}
    for k in stats["nvec"]:
        hist[k] = hist.get(k, 0) + 1
    host = wall - stats["s"] - stats["allreduce_s"]
    return dict(nroots=args.nroots, wall_s=round(wall + w.t_op, 2), davidson_s=round(wall, 2),
                operator_setup_s=round(w.t_op, 2), iterations=int(icyc) + 1,
                converged=bool(np.all(conv)), ax_calls=stats["calls"], ax_vectors=stats["vectors"],
                ax_s=round(stats["s"], 3), allreduce_s=round(stats["allreduce_s"], 3),
                host_davidson_s=round(host, 4), host_ms_per_iteration=round(1e3 * host / (int(icyc) + 1), 3),
                solver_phase_ms={k: round(1e3 * v, 2) for k, v in phase_s.items()},
                nvec_histogram={str(k): v for k, v in sorted(hist.items())},
                e_min_ha=float(e[0]), e_ha=[float(v) for v in e], criteria=crit,
                warmup=("an untimed " + ("2-iteration solve" if op.dim > WARM_FULL_DIM else "solve")
                        + " first (solver kernels loaded)"))


def cpu_converge(args, w, gpu):
    """The CPU side of wall-to-converge (SURVEY.md 8(d) "both sides"): the oracle Davidson
    (oracle/davidson.py, the reference's davidson1 restated, Davidson.py:21-298) driving the
    oracle vind (the reference's AO route) on the SAME data, x0, preconditioner and criteria
    as the device solve, on every CPU of this process's share.  Operator construction (the
    oracle's Fock / hdiag set-up) is included, as on the device side."""
    from threadpoolctl import threadpool_info, threadpool_limits
    from oracle import davidson as odav
    ncpu = cpu_share()
    with threadpool_limits(limits=ncpu):
        threads = max([i.get("num_threads", 1) for i in threadpool_info()
                       if i.get("user_api") == "blas"] or [1])
        mfo, _ = oracle_meanfield(args, w)
        log(f"cpu converge: {args.nroots} roots, oracle Davidson on {threads} BLAS threads")
        t0 = time.perf_counter()
        calls = dict(n=0, v=0)
        vind, hd = _oracle_vind(args, mfo, with_hdiag=args.kind == "XSF")

        def aop(xt):
            calls["n"] += 1
            calls["v"] += len(xt)
            log(f"cpu converge: A.x call {calls['n']} ({len(xt)} vectors, {time.perf_counter() - t0:.0f} s)")
            return vind(xt)
        x0, pre, kw, crit = _solver_setup(args, w, w.device)
        if args.kind == "XTDA":
            from oracle import xtda as oxtda
            precond, kw = oxtda.get_precond(mfo, hd), dict(kw, pick=oxtda.pickeig)
        else:
            precond = odav.make_diag_precond(hd, 1e-3)
        conv, e, _, icyc = odav.davidson1(aop, x0, precond, nroots=args.nroots, **kw)
        wall = time.perf_counter() - t0
    e = np.asarray(e)
    return dict(converge_wall_s=round(wall, 2), iterations=int(icyc) + 1, converged=bool(np.all(conv)),
                ax_calls=calls["n"], ax_vectors=calls["v"], cores=int(threads), kind="port",
                e_min_ha=float(e[0]), max_abs_de_vs_gpu_ha=float(np.abs(e - np.asarray(gpu["e_ha"])).max()),
                gpu_over_cpu_speedup=round(wall / gpu["wall_s"], 1), criteria=crit,
                sample=("oracle Davidson + oracle vind (NumPy AO route) on the timed operator's own data, "
                        "same x0 / preconditioner / criteria as the device solve, full size"))


# ---------------------------------------------------------------------------
def load_traffic(config, tag_name):
    """(HBM bytes per launch of the tagged kernel, source file) from this round's committed
    rocprofv3 PMC summary; (None, None) when it does not hold this config and class."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    v = d.get(config, {}).get(tag_name, {}).get("hbm_bytes_per_launch")
    return (v, os.path.relpath(PMC_SUMMARY, ROOT)) if v is not None else (None, None)


def roofline_of(args, stats_acc, steps, world=1):
    dom_name, dom = max(stats_acc.items(), key=lambda kv: kv[1]["ms"])
    avg_ms = dom["ms"] / max(1, dom["launches"])
    # the committed PMC summaries are single-GPU runs of the presets
    traffic, source = (None, None) if (args.custom or world > 1) else load_traffic(args.config, dom_name)
    if dom_name == "mo_exchange_stored":
        # HBM-bound: streams the stored exchange matrix once per launch (+ Ze in, sigma in/out)
        occ = args.nc if args.kind == "SF_UP" else args.nc + args.no
        vir = args.nv if args.kind == "SF_UP" else args.no + args.nv
        ov = occ * vir
        nzg = (2 if args.kind == "XTDA" else 1) * args.nvec
        bytes_launch = 8.0 * (ov * ov + 3.0 * nzg * ov)
        gbs = bytes_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        return dict(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(gbs / HBM_PEAK_GBS, 4), traffic=traffic, traffic_source=source, kernel=dom_name,
                    avg_launch_ms=round(avg_ms, 4), bytes_per_launch=bytes_launch,
                    launches_per_step=dom["launches"] / steps)
    flops_fused = dom["flops"] / max(1, dom["launches"])
    # algorithmic flops: 2 G nvec sum_s o_s v_s per XC class -- the
    # library counts the superset block (O x V per channel) and, for the two fused
    # classes, their gradient contraction / operand generation (2 (O + 3) per element)
    flops_launch = flops_fused * strict_factor(args, dom_name)
    achieved = flops_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    fused = flops_fused / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    return dict(bound="mfma", achieved=round(achieved, 3), peak=FP64_PEAK_TFLOPS, unit="TFLOP/s",
                frac=round(achieved / FP64_PEAK_TFLOPS, 4), traffic=traffic, traffic_source=source,
                kernel=dom_name, avg_launch_ms=round(avg_ms, 4),
                flops_per_launch=flops_launch, launches_per_step=dom["launches"] / steps,
                accounting="strict: 2 G nvec sum_s o_s v_s (SURVEY.md 8(d))",
                achieved_fused_accounting=round(fused, 3),
                frac_fused_accounting=round(fused / FP64_PEAK_TFLOPS, 4))


def strict_factor(args, name):
    """Algorithmic / counted flops of an XC class: the actual occupied-virtual pairs
    over the superset block the kernels run (both X-TDA channels as O x V), times
    O / (O + 3) for the fused classes (their 3-FMA contraction / generation counted by
    the library as extra rows)."""
    if name not in ("xc_forward_u", "xc_back_l", "xc_forward_w", "xc_back_m"):
        return 1.0
    if args.kind == "XTDA":
        O, V = args.nc + args.no, args.no + args.nv
        pairs, sup = (args.nc + args.no) * args.nv + args.nc * (args.no + args.nv), 2 * O * V
    elif args.kind == "SF_UP":
        O = args.nc
        pairs = sup = args.nc * args.nv
    else:
        O = args.nc + args.no
        pairs = sup = O * (args.no + args.nv)
    f = pairs / sup
    return f * O / (O + 3) if name in ("xc_forward_w", "xc_back_m") else f


def breakdown(op, z, out, allreduce, sync, stats_acc, steps, rank, world, reps=2):
    """This rank's phase split of one step: device A.x and the sigma all-reduce each
    timed between synchronisations (``reps`` extra steps after the timed region), and
    the live per-class kernel ms of the timed steps."""
    ta = tr = 0.0
    for _ in range(reps):
        sync()
        t0 = time.perf_counter()
        op.apply(z, out)
        sync()
        t1 = time.perf_counter()
        allreduce(out)
        sync()
        ta += t1 - t0
        tr += time.perf_counter() - t1
    return dict(rank=rank, ax_ms=round(1e3 * ta / reps, 3), allreduce_ms=round(1e3 * tr / reps, 3),
                sigma_mb=round(out.numel() * 8 / 1e6, 3), k_mode=getattr(op, "k_mode", None),
                partition=getattr(op, "partition", None),
                kernel_ms={k: round(v["ms"] / steps, 3) for k, v in stats_acc.items() if v["launches"]})


def rank_main(args):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("XT_BENCH_BACKEND", "nccl")
    stub = bool(os.environ.get("XT_BENCH_OPERATOR"))
    use_gpu = not stub
    if use_gpu:
        if backend != "nccl":     # gloo rehearsal: ranks share the visible GPU(s)
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
    # XT_BENCH_FORCE_PG=1: a process group (and its collectives) even at world 1 -- the
    # single-GPU pool's only way to run RCCL itself (two ranks on one GPU are refused)
    pg = world > 1 or os.environ.get("XT_BENCH_FORCE_PG") == "1"
    if world > 1:
        # the host side of a rank (the replicated Davidson's subspace eigh, <= 108^2) is tiny:
        # N ranks x the node's BLAS thread count oversubscribe the host (8 gloo ranks on one
        # box: 0.8-1.5 s of host Davidson per solve against 0.07 s at N = 1)
        try:
            from threadpoolctl import threadpool_limits
            threadpool_limits(limits=2)
        except Exception:
            pass
    if pg:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    if use_gpu:
        from xtddft_amd import build
        if rank == 0:
            build.build()
        if pg:
            dist.barrier()
    from xtddft_amd.parallel import allreduce_sigma

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    log(f"rank {rank}/{world}: building the {args.config} workload")
    w = _factory()(args, rank, world, local)
    op = w.op
    log(f"rank {rank}: generation {w.t_gen:.2f} s, operator construction {w.t_op:.2f} s")
    gen = torch.Generator(device=w.device)
    gen.manual_seed(20261016)
    z = torch.randn((args.nvec, op.dim), dtype=torch.float64, device=w.device, generator=gen)
    z /= z.norm(dim=1, keepdim=True)
    out = torch.empty_like(z)

    def step():
        op.apply(z, out)
        allreduce_sigma(out)

    for _ in range(args.warmup):
        step()
    op.set_profile(0b111110)
    stats_acc = {}
    if pg:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for name, s in op.profile_stats().items():
            a = stats_acc.setdefault(name, dict(ms=0.0, launches=0, flops=0.0, bytes=0.0))
            a["ms"] += s["ms"]; a["launches"] += s["launches"]; a["flops"] += s["flops"]
            a["bytes"] += s.get("bytes", 0.0)
    sync()
    if pg:
        dist.barrier()
    dt = time.perf_counter() - t0
    op.set_profile(0)
    phases = op.last_timings()          # the last timed step's phase split
    z0 = s0 = None
    if use_gpu:                          # the first timed vector and its device sigma (verify)
        z0, s0 = z[:1].cpu().numpy(), out[:1].cpu().numpy()
    # RCCL reduces device tensors only (a host tensor raises under the nccl backend)
    tt = torch.tensor([dt], dtype=torch.float64,
                      device=w.device if (use_gpu and backend == "nccl") else "cpu")
    if pg:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    T = float(tt.item())
    log(f"timed {args.steps} steps: {1e3 * T / args.steps:.2f} ms per step")
    verify = w.verify(z, out) if hasattr(w, "verify") else None   # a workload's own self-check
    # outside the timed region: A is symmetric, so <y, A x> = <A y, x> on the measured
    # operator itself (two 2-vector A.x calls, all-reduced like the timed ones)
    symmetry = None
    if use_gpu:
        import torch
        gs = torch.Generator(device=w.device)
        gs.manual_seed(7)
        xv = torch.randn((2, op.dim), dtype=torch.float64, device=w.device, generator=gs)
        yv = torch.randn((2, op.dim), dtype=torch.float64, device=w.device, generator=gs)
        ax, ay = allreduce_sigma(op.apply(xv)), allreduce_sigma(op.apply(yv))
        lhs, rhs = yv @ ax.T, ay @ xv.T
        symmetry = float((lhs - rhs).abs().max() / lhs.abs().max())
    # per-rank breakdown (outside the timed region: synchronised after each phase)
    mine = breakdown(op, z, out, allreduce_sigma, sync, stats_acc, args.steps, rank, world)
    roofline = roofline_of(args, stats_acc, args.steps, world)
    others = {}
    for k, v in stats_acc.items():
        if not v["launches"]:
            continue
        comp = v["bytes"] / v["launches"]
        hbm = None if (args.custom or world > 1) else load_traffic(args.config, k)[0]
        others[k] = dict(ms_per_step=round(v["ms"] / args.steps, 3),
                         tflops=round(v["flops"] * strict_factor(args, k) / max(v["ms"], 1e-9) / 1e9, 3),
                         tflops_fused_accounting=round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 3),
                         compulsory_bytes_per_launch=comp, hbm_bytes_per_launch=hbm,
                         traffic_ratio=round(hbm / comp, 3) if hbm and comp > 0 else None)
    workload = (f"{KIND_NAME[args.kind]} A.x, nao={args.nao}, nocc_a/nocc_b={args.nc + args.no}/{args.nc}, "
                f"dim={op.dim}, nvec={args.nvec}, {args.jk} naux={args.naux}, ngrid={args.ngrid}, "
                f"xc={args.xc}, hyb={args.hyb}"
                + (", multicollinear kernel (method=1)" if args.method == 1 else "")
                + (f", SA={args.sa}, remove={bool(args.remove)}" if args.kind == "XSF" else "")
                + f" [BASELINE {args.config}: {CONFIG_NAMES[args.config]}]")
    # a gloo rehearsal time-shares the visible GPU(s): n_gpus is the physical count
    ngpu = world if (backend == "nccl" or not use_gpu) else min(world, torch.cuda.device_count())
    result = dict(
        metric="A·x matvecs/sec (nao, nocc×nvir, nvec)",
        value=round(args.nvec * args.steps / T, 4),
        unit="matvecs/s",
        n_gpus=ngpu, steps=args.steps, warmup=args.warmup,
        ms_per_step=round(1e3 * T / args.steps, 3),
        higher_is_better=True, scaling="strong", vs_baseline=None, dtype="f64",
        data=("synthetic (seeded ROKS mean field, DF factor, GGA grid kernel; generated in HBM)"
              if not stub else "STUB operator (launcher test only; not a measurement)"),
        config=dict(workload=workload, nao=args.nao, dim=op.dim, nvec=args.nvec, naux=args.naux,
                    ngrid=args.ngrid, parallelism=(
                        f"grid sharded x{world}; " +
                        ("replicated MO DF factor, aux window + stored-exchange rows"
                         if w.replicate else "aux sharded") + " per rank; all-reduce of sigma")),
        roofline=roofline,
        gemm_classes=others,
        phases_ms_last_step=phases,
        setup_s=dict(synthetic_generation=round(w.t_gen, 2), operator_construction=round(w.t_op, 2),
                     construction_phases={k: round(v, 3) for k, v in getattr(op, "setup_s", {}).items()}),
        exchange=dict(mode=op.k_mode, stored_gib=round(op.k_gib, 2), build_s=round(op.prepare_s, 3)),
    )
    if verify is not None:
        result["verify"] = verify
    if ngpu != world:
        result["rehearsal"] = (f"{world} ranks over {backend} time-sharing {ngpu} GPU(s): a correctness "
                               f"rehearsal of the sharded path, not a {world}-GPU measurement")
    if symmetry is not None:
        result["check"] = dict(symmetry_rel=symmetry,
                               what="max |<y,Ax> - <Ay,x>| / max |<y,Ax>| over 2 x 2 random vectors")
    if rank == 0 and world == 1 and use_gpu and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"], result["verify"] = cpu_baseline(args, w, z0, s0)
        except Exception as e:   # report, never hide
            result["cpu_baseline"] = dict(value=None, error=repr(e))
    if use_gpu and (not args.no_converge or args.converge):
        result["converge"] = converge(args, w, allreduce_sigma, world)
        mine["converge"] = {k: result["converge"][k] for k in ("ax_s", "allreduce_s", "host_davidson_s")}
        cpu = result.get("cpu_baseline") or {}
        est = result["converge"]["ax_vectors"] / cpu["value"] if cpu.get("value") else None
        if rank == 0 and world == 1 and (args.cpu_converge == "on" or (
                args.cpu_converge == "auto" and est is not None and est < CPU_CONVERGE_AUTO_S)):
            try:
                cpu["converge"] = cpu_converge(args, w, result["converge"])
            except Exception as e:   # report, never hide
                cpu["converge"] = dict(error=repr(e))
            result["cpu_baseline"] = cpu
        elif rank == 0 and world == 1 and est is not None:
            cpu["converge"] = dict(skipped=f"estimated {est:.0f} s of CPU A.x (--cpu-converge on runs it)")
    if pg:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        result["ranks"] = ranks
    else:
        result["ranks"] = [mine]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if pg:
        dist.destroy_process_group()
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args, argv)
    return rank_main(args)


if __name__ == "__main__":
    sys.exit(main())
