"""Time the 3-index DF integrals and the 4-index ERIs, host McMurchie-Davidson
(qc/ints.py) against the HIP kernel (qc/dints.py, csrc/xt_int.hip), on clusters of
s/p/d "water" molecules (the basis of tests/test_gpu_qc.py::_spd_mol).
python tools/int_bench.py [nmol ...]   (GPU needed for the device columns)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xtddft_amd.qc import M  # noqa: E402
from xtddft_amd.qc.df import aux_mole  # noqa: E402

BASIS = {"O": [[0, [30.0, 0.3], [6.0, 0.7]], [0, [0.9, 1.0]], [1, [5.0, 0.4], [1.1, 0.7]], [2, [1.2, 1.0]]],
         "H": [[0, [3.0, 0.4], [0.5, 0.7]], [1, [0.8, 1.0]]]}


def cluster(nmol):
    atoms = []
    for k in range(nmol):
        o = np.array([3.5 * (k % 3), 3.5 * ((k // 3) % 3), 3.5 * (k // 9)])
        atoms += [("O", o), ("H", o + [1.4, 1.0, 0.2]), ("H", o + [-1.3, 1.1, -0.4])]
    return M(atoms, basis=BASIS, unit="Bohr")


def timed(f):
    t = time.perf_counter()
    r = f()
    return r, time.perf_counter() - t


def main(sizes):
    for nmol in sizes:
        mol = cluster(nmol)
        aux = aux_mole(mol)
        row = dict(nmol=nmol, nao=mol.nao, naux=aux.nao)
        mol.int3c2e(aux, device=0)                     # warm-up (library load, first launch)
        dev3, row["int3c2e_device_s"] = timed(lambda: mol.int3c2e(aux, device=0))
        if nmol <= 4:
            host3, row["int3c2e_host_s"] = timed(lambda: mol.int3c2e(aux))
            row["int3c2e_max_abs_diff"] = float(np.abs(dev3 - host3).max())
        dev4, row["eri_device_s"] = timed(lambda: mol.eri_full(device=0))
        if nmol <= 2:
            host4, row["eri_host_s"] = timed(lambda: mol.eri_full())
            row["eri_max_abs_diff"] = float(np.abs(dev4 - host4).max())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [1, 2, 4, 8])
