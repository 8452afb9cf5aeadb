#!/usr/bin/env python
"""Benchmark: X-TDA A.x throughput on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Workload (default): the BASELINE headline shape -- synthetic ROKS X-TDA,
nao = 1000, nocc_a/nocc_b = 101/99 (nc 99, no 2, nv 899), naux = 3 nao,
ngrid = 1200 nao, GGA kernel + global hybrid (hyb 0.2), nvec = 20 trial
vectors per A.x.  A "step" is one full A.x on the 20-vector batch (plus the
RCCL all-reduce of sigma when N > 1).  value = matvecs/s = nvec*K / T where T
is the max over ranks of the barrier+synchronise-bracketed wall time.

Multi-GPU: the DF aux index and the grid are sharded over ranks (each rank
generates and holds only its shard); every rank computes a partial sigma for
all vectors and one all-reduce (torch.distributed / RCCL over xGMI) sums them:
fixed total work, so "scaling": "strong".

Extra JSON fields: roofline (dominant GEMM class timed live with HIP events
on the library's stream over the timed steps), cpu_baseline (the NumPy
oracle = the reference's AO-route algorithm, timed on this host on a bounded
sample and extrapolated), converge (wall time of the device Davidson to
nroots = 20 on the same operator, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6     # MI355X dense FP64 matrix peak (AMD spec); 74.2 measured (tools/mfma_probe.hip)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec


KIND_NAME = {"XTDA": "X-TDA", "SF_UP": "SF-TDA (spin-flip up)", "SF_DOWN": "SF-TDA (spin-flip down)",
             "XSF": "XSF-TDA"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nao", type=int, default=1000)
    ap.add_argument("--nc", type=int, default=99)
    ap.add_argument("--no", type=int, default=2)
    ap.add_argument("--naux", type=int, default=None)
    ap.add_argument("--ngrid", type=int, default=None)
    ap.add_argument("--nvec", type=int, default=20)
    ap.add_argument("--xc", default="GGA")
    ap.add_argument("--hyb", type=float, default=0.2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-converge", action="store_true")
    ap.add_argument("--converge", action="store_true", help="also at N > 1")
    ap.add_argument("--nroots", type=int, default=20)
    ap.add_argument("--k-mode", default="auto", choices=["auto", "direct", "stored"],
                    help="exchange evaluation (xt_set_exchange_mode)")
    ap.add_argument("--kind", default="XTDA", choices=["XTDA", "SF_UP", "SF_DOWN", "XSF"],
                    help="operator (XTDA.py / SF_TDA.py / XSF_TDA.py vind)")
    ap.add_argument("--sa", type=int, default=0, help="XSF spin-adaptation level (XSF_TDA.py SA)")
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="BASELINE.json shape preset (synthetic data of that shape); the default "
                         "bench line is the headline H")
    args = ap.parse_args()
    if args.config:
        for k, v in CONFIGS[args.config].items():
            setattr(args, k, v)
    return args


# BASELINE.json configs as synthetic shapes (SURVEY.md 8 shape table): nao, closed /
# open shells, operator, vectors per A.x (= nroots), hybrid fraction.  C4 is the
# XSF doublet, run at SA = 0 (SA > 0 divides by 2S - 1 = 0, XSF_TDA.py:1102-1121).
CONFIGS = {
    "H": dict(nao=1000, nc=99, no=2, kind="XTDA", nvec=20, nroots=20, hyb=0.2),
    "C2": dict(nao=180, nc=33, no=1, kind="XTDA", nvec=20, nroots=20, hyb=0.2),
    "C3": dict(nao=861, nc=91, no=4, kind="SF_UP", nvec=30, nroots=30, hyb=0.5),
    "C4": dict(nao=840, nc=180, no=1, kind="XSF", nvec=40, nroots=40, hyb=0.5, sa=0),
    "C5": dict(nao=152, nc=35, no=2, kind="XTDA", nvec=50, nroots=50, hyb=0.2),
}


def cpu_baseline(args):
    """Oracle (reference AO-route algorithm, NumPy/BLAS) on this host.

    t(naux, ngrid) per trial vector is linear in both sizes; it is timed at
    three bounded samples of the SAME shape (nao, nc, no) and extrapolated to
    the full naux / ngrid.  Returns matvecs/s.
    """
    from oracle import xtda as oxtda
    from xtddft_amd.synthetic import make_mf, make_trial_vectors
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    naux = args.naux or 3 * args.nao
    ngrid = args.ngrid or 1200 * args.nao
    samples = [(16, 8192), (32, 8192), (16, 16384)]
    times = []
    t_all = time.perf_counter()
    for n, g in samples:
        mf = make_mf(nao=args.nao, nc=args.nc, no=args.no, naux=n, ngrid=g, xctype=args.xc,
                     hyb=args.hyb)
        vind, hdiag = oxtda.gen_tda_operation(mf)
        z = make_trial_vectors(1, hdiag.size)
        vind(z)                        # warm-up (1 warm-up, median of >= 5)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter(); vind(z); ts.append(time.perf_counter() - t0)
        times.append(float(np.median(ts)))
        del mf, vind
    (n1, g1), (n2, _), (_, g3) = samples
    a = (times[1] - times[0]) / (n2 - n1)
    b = (times[2] - times[0]) / (g3 - g1)
    t0 = times[0] - a * n1 - b * g1
    t_vec = t0 + a * naux + b * ngrid
    return dict(value=1.0 / t_vec, unit="matvecs/s", cores=int(cores), kind="port",
                sample=(f"oracle X-TDA vind (NumPy AO route, DF J/K, GGA) on 1 vector at nao={args.nao}, "
                        f"(naux, ngrid) in {samples}, 1 warm-up + median of 5; linear extrapolation to "
                        f"naux={naux}, ngrid={ngrid}: t_vec = {t_vec:.1f} s"),
                host=_host_info(), sample_wall_s=round(time.perf_counter() - t_all, 1))


def _host_info():
    """CPU model and BLAS build of the host timing the CPU baseline."""
    info = {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["cpu"] = line.split(":", 1)[1].strip()
                    break
        info["host_cpus"] = os.cpu_count()
    except Exception:
        pass
    try:
        from threadpoolctl import threadpool_info
        info["blas"] = [f"{i.get('internal_api')} {i.get('version')} threads={i.get('num_threads')}"
                        for i in threadpool_info()]
    except Exception:
        pass
    return info


def load_traffic(tag_name):
    """HBM bytes per launch of the tagged kernel from a committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(tag_name, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("for --gpus N > 1 launch with torch.distributed.run (one process per GPU)")
    # XT_BENCH_BACKEND=gloo rehearses the N-rank path with ranks sharing the visible
    # GPU(s) (tests on a one-GPU box); the real runs use nccl = RCCL over xGMI
    backend = os.environ.get("XT_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    from xtddft_amd import build
    if rank == 0:
        build.build()
    if world > 1:
        dist.barrier()
    from xtddft_amd.synthetic import make_device_mf
    from xtddft_amd.operator import DeviceOperator

    naux = args.naux or 3 * args.nao
    ngrid = args.ngrid or 1200 * args.nao
    nv = args.nao - args.nc - args.no
    t_setup = time.perf_counter()
    # stored exchange over N ranks: the MO factor is replicated and each rank
    # keeps 1/N of the exchange rows (xt_set_partition); direct: aux-sliced factor
    replicate = world > 1 and args.k_mode != "direct"
    mf = make_device_mf(nao=args.nao, nc=args.nc, no=args.no, naux=naux, ngrid=ngrid,
                        xctype=args.xc, hyb=args.hyb, device=local, shard=(rank, world),
                        full_aux=replicate)
    kw = {}
    if args.kind == "XSF":
        # XSF_TDA.kernel default fglobal = (1 - d_lda) c_x + d_lda, d_lda = 0.3, c_x = hyb
        kw = dict(sa=args.sa, fglobal=0.7 * args.hyb + 0.3, foo=1.0, remove=False)
    op = DeviceOperator(mf, args.kind, shard=(rank, world), device=local, **kw,
                        presharded="grid" if replicate else True, k_mode=args.k_mode,
                        replicate_df=replicate)
    mf.cderi = None
    mf.grids = None
    mf.fxc = None
    mf.fxc_sf = None
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    t_setup = time.perf_counter() - t_setup

    gen = torch.Generator(device=f"cuda:{local}")
    gen.manual_seed(20261016)
    z = torch.randn((args.nvec, op.dim), dtype=torch.float64, device=f"cuda:{local}", generator=gen)
    z /= z.norm(dim=1, keepdim=True)
    out = torch.empty_like(z)

    def step():
        op.apply(z, out)
        if world > 1:
            dist.all_reduce(out)

    for _ in range(args.warmup):
        step()
    op.set_profile(0b111110)
    stats_acc = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        for name, s in op.profile_stats().items():
            a = stats_acc.setdefault(name, dict(ms=0.0, launches=0, flops=0.0))
            a["ms"] += s["ms"]; a["launches"] += s["launches"]; a["flops"] += s["flops"]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    op.set_profile(0)
    tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    T = float(tt.item())
    phases = op.last_timings()

    # dominant GEMM class on this rank
    dom_name, dom = max(stats_acc.items(), key=lambda kv: kv[1]["ms"])
    avg_ms = dom["ms"] / max(1, dom["launches"])
    flops_launch = dom["flops"] / max(1, dom["launches"])
    achieved = flops_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    traffic = load_traffic(dom_name)
    if dom_name == "mo_exchange_stored":
        # HBM-bound: streams the stored exchange matrix once per launch (+ Ze in, sigma in/out)
        occ = args.nc if args.kind == "SF_UP" else args.nc + args.no
        vir = nv if args.kind == "SF_UP" else args.no + nv
        ov = occ * vir
        nzg = (2 if args.kind == "XTDA" else 1) * args.nvec
        bytes_launch = 8.0 * (ov * ov + 3.0 * nzg * ov)
        gbs = bytes_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        roofline = dict(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(gbs / HBM_PEAK_GBS, 4), traffic=traffic, kernel=dom_name,
                        avg_launch_ms=round(avg_ms, 4), bytes_per_launch=bytes_launch,
                        launches_per_step=dom["launches"] / args.steps)
    else:
        roofline = dict(bound="mfma", achieved=round(achieved, 3), peak=FP64_PEAK_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / FP64_PEAK_TFLOPS, 4), traffic=traffic,
                        kernel=dom_name, avg_launch_ms=round(avg_ms, 4),
                        flops_per_launch=flops_launch, launches_per_step=dom["launches"] / args.steps)
    others = {k: dict(ms_per_step=round(v["ms"] / args.steps, 3),
                      tflops=round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 3))
              for k, v in stats_acc.items()}

    result = dict(
        metric="A·x matvecs/sec (nao, nocc×nvir, nvec)",
        value=round(args.nvec * args.steps / T, 4),
        unit="matvecs/s",
        n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=round(1e3 * T / args.steps, 3),
        higher_is_better=True, scaling="strong", vs_baseline=None, dtype="f64",
        data="synthetic (seeded ROKS mean field, DF factor, GGA grid kernel; generated in HBM)",
        config=dict(workload=(f"{KIND_NAME[args.kind]} A.x, nao={args.nao}, nocc_a/nocc_b={args.nc + args.no}/{args.nc}, "
                              f"dim={op.dim}, "
                              f"nvec={args.nvec}, naux={naux}, ngrid={ngrid}, xc={args.xc}, hyb={args.hyb}"
                              + (f", SA={args.sa}" if args.kind == "XSF" else "")
                              + (f" [BASELINE {args.config}]" if args.config else "")),
                    nao=args.nao, dim=op.dim, nvec=args.nvec, naux=naux, ngrid=ngrid,
                    parallelism=(f"grid sharded x{world}; " +
                                 ("replicated MO DF factor, aux window + stored-exchange rows"
                                  if replicate else "aux sharded") +
                                 " per rank; RCCL all-reduce of sigma")),
        roofline=roofline,
        gemm_classes=others,
        phases_ms_last_step=phases,
        setup_s=round(t_setup, 2),
        exchange=dict(mode=op.k_mode, stored_gib=round(op.k_gib, 2), build_s=round(op.prepare_s, 3)),
    )

    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.kind == "XTDA":
        try:
            result["cpu_baseline"] = cpu_baseline(args)
        except Exception as e:   # report, never hide
            result["cpu_baseline"] = dict(value=None, error=repr(e))

    if ((world == 1 and not args.no_converge) or args.converge) and args.kind == "XTDA":
        from xtddft_amd.davidson import DiagPrecond, davidson1
        from xtddft_amd.xtda import XTDA
        x = XTDA.__new__(XTDA)
        x.mf, x.X, x.nstates, x.device = mf, True, args.nroots, local
        hdiag = x._hdiag()
        x0 = x.get_init_guess(mf, args.nroots)

        aop_stats = dict(calls=0, vectors=0, s=0.0)

        def aop(xt):
            t = time.perf_counter()
            s = op.apply(xt)
            if world > 1:
                dist.all_reduce(s)
            torch.cuda.synchronize()
            aop_stats["calls"] += 1
            aop_stats["vectors"] += int(s.shape[0])
            aop_stats["s"] += time.perf_counter() - t
            return s

        def pickeig(w, v, nroots, envs):
            idx = np.where(w > 0.001)[0]
            return w[idx], v[:, idx], idx
        torch.cuda.synchronize()
        tc = time.perf_counter()
        conv, e, _, icyc = davidson1(aop, x0, DiagPrecond(hdiag, 0.0, local), tol_residual=1e-5,
                                     lindep=1e-12, nroots=args.nroots, pick=pickeig, max_cycle=100,
                                     device=local, return_device=True)
        torch.cuda.synchronize()
        wall = time.perf_counter() - tc
        result["converge"] = dict(nroots=args.nroots, wall_s=round(wall, 2),
                                  wall_s_incl_exchange_build=round(wall + op.prepare_s, 2),
                                  iterations=int(icyc) + 1, converged=bool(np.all(conv)),
                                  ax_vectors=aop_stats["vectors"], ax_s=round(aop_stats["s"], 2),
                                  e_min_ha=float(e[0]), criteria="|de|<1e-12, |r|<1e-5 (XTDA.py:775)")
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
