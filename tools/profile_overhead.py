"""A / B of the bench's per-class HIP-event profiling against un-profiled steps.

    python tools/profile_overhead.py --config C5 --steps 20

Times the same workload three ways, alternating, on one GPU: the bench's timed loop
(profiling on, `profile_stats()` read every step), profiling off with one synchronise per
step, and profiling off with one synchronise over all steps.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    args = bench.parse(sys.argv[1:])
    w = bench.device_workload(args, 0, 1, 0)
    op = w.op
    gen = torch.Generator(device=w.device)
    gen.manual_seed(20261016)
    z = torch.randn((args.nvec, op.dim), dtype=torch.float64, device=w.device, generator=gen)
    z /= z.norm(dim=1, keepdim=True)
    out = torch.empty_like(z)
    for _ in range(max(args.warmup, 2)):
        op.apply(z, out)
    torch.cuda.synchronize()

    def run(mode):
        op.set_profile(0b111110 if mode == "profiled" else 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            op.apply(z, out)
            if mode == "profiled":
                op.profile_stats()
            elif mode == "sync":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        op.set_profile(0)
        return 1e3 * (time.perf_counter() - t0) / args.steps

    res = {m: [] for m in ("profiled", "sync", "async")}
    for _ in range(3):
        for m in res:
            res[m].append(run(m))
    for m, v in res.items():
        print(f"{args.config} {m:9s} ms/step " + " ".join(f"{x:.3f}" for x in v), flush=True)


if __name__ == "__main__":
    main()
