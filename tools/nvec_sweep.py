"""A.x time per trial-vector count on the headline operator (Davidson steps with few
new vectors): ms per call and per class (live HIP-event timing) for nvec in --nvecs.

    python tools/nvec_sweep.py [--nvecs 1,2,3,4,6,8,12,16,20] [--reps 3] [--out FILE]
    python tools/nvec_sweep.py --nao 256 --nclosed 24 --nvecs 1,8,20,40,80   (SURVEY 8(d) sweeps)
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nvecs", default="1,2,3,4,5,6,8,10,12,16,20")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", default="H")
    ap.add_argument("--out", default="gpurun_out/nvec_sweep.json")
    ap.add_argument("--nao", type=int, default=None)
    ap.add_argument("--nclosed", type=int, default=None)
    ap.add_argument("--nopen", type=int, default=None)
    a = ap.parse_args()
    import torch
    import bench
    argv = ["--config", a.config]
    for k in ("nao", "nclosed", "nopen"):
        if getattr(a, k) is not None:
            argv += [f"--{k}", str(getattr(a, k))]
    args = bench.parse(argv)
    w = bench.device_workload(args, 0, 1, 0)
    op = w.op
    rows = []
    for nv in [int(x) for x in a.nvecs.split(",")]:
        g = torch.Generator(device="cuda").manual_seed(nv)
        z = torch.randn((nv, op.dim), dtype=torch.float64, device="cuda", generator=g)
        out = torch.empty_like(z)
        op.apply(z, out)
        torch.cuda.synchronize()
        op.set_profile(0b111110)
        cls = {}
        t0 = time.perf_counter()
        for _ in range(a.reps):
            op.apply(z, out)
            for k, v in op.profile_stats().items():
                cls[k] = cls.get(k, 0.0) + v["ms"] / a.reps
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / a.reps
        op.set_profile(0)
        r = dict(nao=args.nao, nc=args.nc, no=args.no, dim=op.dim, ngrid=args.ngrid, naux=args.naux, nvec=nv,
                 ms=round(ms, 3), ms_per_vec=round(ms / nv, 3), matvecs_per_s=round(1e3 * nv / ms, 2),
                 k_mode=getattr(op, "k_mode", None), classes={k: round(v, 3) for k, v in cls.items()})
        rows.append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
