"""HBM probe: achievable in-place read + write and read-only / write-only rates on one GPU,
the bound the grid-point kernel (k_xc_point_b, U read and overwritten in place) runs against.

    python tools/stream_probe.py
"""
import torch


def rate(f, nbytes, reps=10):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        f()
    b.record()
    b.synchronize()
    ms = a.elapsed_time(b) / reps
    return ms, nbytes / ms / 1e9


def main():
    n = 5_250_000_000 // 8          # C5's U (both spins) per A.x: 5.25 GB
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    x.fill_(1.0)
    y = torch.empty_like(x)
    for name, f, nb in (("inplace_scale", lambda: x.mul_(1.0000001), 2 * 8 * n),
                        ("copy", lambda: y.copy_(x), 2 * 8 * n),
                        ("fill", lambda: y.fill_(0.5), 8 * n),
                        ("sum", lambda: x.sum(), 8 * n)):
        ms, tb = rate(f, nb)
        print(f"{name:14s} {ms:8.3f} ms  {tb:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
