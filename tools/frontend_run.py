"""End to end on the device for a >= 300-AO molecule: (HF)_n cluster plus an H atom
(a doublet with a localised open shell), 6-31G + d + f on F (tests/molecules.py
hf_cluster_radical), ROKS B3LYP with exact J/K from
the integral-direct Cholesky factor (no 4-index array), device integrals and AO
values, then X-TDA 20 roots through the device operator and Davidson.

    python tools/frontend_run.py [--n 14] [--nroots 20] [--tol 1e-12] [--out FILE]

Prints one JSON record (stage timings, sizes, roots, residual check) and writes it
to --out.  Run on the GPU box; the committed record lives under profiles/.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--nroots", type=int, default=20)
    ap.add_argument("--tol", type=float, default=1e-12)
    ap.add_argument("--xc", default="b3lyp")
    ap.add_argument("--conv", type=float, default=1e-9)
    ap.add_argument("--out", default="gpurun_out/frontend_run.json")
    a = ap.parse_args()
    import torch
    from molecules import hf_cluster_radical
    from xtddft_amd.qc import ROKS
    from xtddft_amd.xtda import XTDA
    rec = dict(molecule=f"(HF){a.n} + H doublet, 6-31G + d,f on F", xc=a.xc, chol_tol=a.tol)
    t0 = time.perf_counter()
    mol = hf_cluster_radical(a.n)
    rec.update(nao=mol.nao, nshell=len(mol.shells), natm=mol.natm, mole_s=time.perf_counter() - t0)
    mf = ROKS(mol, a.xc)
    mf.conv_tol = a.conv
    mf.max_cycle = 150
    mf.to_device(0).cholesky(a.tol)
    t0 = time.perf_counter()
    mf.build()
    torch.cuda.synchronize()
    rec["build_s"] = time.perf_counter() - t0
    rec["build"] = {k: v for k, v in mf.timings.items()}
    rec["ngrid"] = int(mf.grids.size)
    print("build", json.dumps(rec), flush=True)
    t0 = time.perf_counter()
    mf.kernel()
    torch.cuda.synchronize()
    rec.update(scf_s=time.perf_counter() - t0, scf_converged=bool(mf.converged), e_tot=mf.e_tot)
    print("scf", rec["scf_s"], mf.converged, mf.e_tot, flush=True)
    t0 = time.perf_counter()
    mfield = mf.to_meanfield()
    torch.cuda.synchronize()
    rec["meanfield_s"] = time.perf_counter() - t0
    td = XTDA(None, mfield, nstates=a.nroots)
    t0 = time.perf_counter()
    e = td.kernel()
    torch.cuda.synchronize()
    rec.update(xtda_s=time.perf_counter() - t0, xtda_converged=bool(np.all(td.converged)),
               xtda_iterations=int(td.icyc) if np.isscalar(td.icyc) else td.icyc,
               dim=int(td.operator().dim), k_mode=td.operator().k_mode,
               roots_ha=[float(x) for x in e])
    # independent residual check: |A x - e x| for every root through a fresh A.x
    op = td.operator()
    x = td.v[np.argsort(td.order), :].T          # back to PySCF order
    ax = op.apply(np.ascontiguousarray(x))
    res = np.linalg.norm(ax - np.asarray(e)[:, None] * x, axis=1)
    rec["max_residual"] = float(res.max())
    naux, _ = op.naux()
    rec["naux_cholesky"] = naux
    print(json.dumps(rec), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
