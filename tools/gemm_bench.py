"""Time xt_dgemm on the headline contraction shapes vs torch.matmul (rocBLAS/hipBLASLt).

Each row: name, M, N, K, transA, transB (op(A) = A^T when set; row-major storage).
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xtddft_amd import _capi, build  # noqa: E402

SHAPES = [
    ("xc_fwd_u    (k,k)", 65536, 4040, 901, 0, 1),
    ("xc_back_l   (m,n)", 4040, 901, 65536, 1, 0),
    ("square4096  (k,n)", 4096, 4096, 4096, 0, 0),
    ("square8192  (k,n)", 8192, 8192, 8192, 0, 0),
]


def main():
    build.build()
    L = _capi.lib()
    st = torch.cuda.current_stream().cuda_stream
    for name, m, n, k, ta, tb in SHAPES:
        a = torch.randn((k, m) if ta else (m, k), dtype=torch.float64, device="cuda")
        b = torch.randn((n, k) if tb else (k, n), dtype=torch.float64, device="cuda")
        c = torch.empty((m, n), dtype=torch.float64, device="cuda")

        def ours():
            _capi.check(L.xt_dgemm(ta, tb, m, n, k, 1.0, a.data_ptr(), a.shape[1], b.data_ptr(), b.shape[1],
                                   0.0, c.data_ptr(), n, ctypes.c_void_p(st)), "dgemm")

        def lib():
            torch.matmul(a.T if ta else a, b.T if tb else b, out=c)
        res = []
        for f in (ours, lib):
            f(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 5
            e0.record()
            for _ in range(reps):
                f()
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res.append((ms, 2.0 * m * n * k / ms / 1e9))
        print(f"{name:24s} M={m:6d} N={n:6d} K={k:7d}  ours {res[0][0]:8.3f} ms {res[0][1]:6.1f} TF/s"
              f"   torch {res[1][0]:8.3f} ms {res[1][1]:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
