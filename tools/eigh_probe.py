"""Host eigh at Davidson subspace sizes on this box's CPU, one thread: SciPy (OpenBLAS)
drivers evr (SciPy's default) / evd against torch's CPU eigh (MKL syevd) -- which host
LAPACK the replicated Davidson step should call (xtddft_amd/davidson.py); and the device
eigh (torch.linalg.eigh on the GPU: rocSOLVER) for comparison."""
import json
import time

import numpy as np
import scipy.linalg
import torch
from threadpoolctl import threadpool_limits


def main():
    torch.set_num_threads(1)
    out = {}
    rng = np.random.default_rng(0)
    with threadpool_limits(limits=1):
        for n in (36, 70, 108, 180, 258):
            a = rng.standard_normal((n, n))
            a = a + a.T
            row = {}
            ad = torch.from_numpy(a).cuda() if torch.cuda.is_available() else None

            def gpu():
                w, v = torch.linalg.eigh(ad)
                torch.cuda.synchronize()
            for name, f in (("scipy_evr", lambda: scipy.linalg.eigh(a)),
                            ("scipy_evd", lambda: scipy.linalg.eigh(a, driver="evd")),
                            ("torch_mkl", lambda: torch.linalg.eigh(torch.from_numpy(a)))) + \
                    ((("gpu_syevd", gpu),) if ad is not None else ()):
                f()
                ts = []
                for _ in range(5):
                    t = time.perf_counter()
                    for _ in range(20):
                        f()
                    ts.append((time.perf_counter() - t) / 20 * 1e3)
                row[name] = round(min(ts), 4)
            out[n] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
