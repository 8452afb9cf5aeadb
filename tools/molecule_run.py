"""A BASELINE-class molecule end to end on the device, checked against the oracle.

    python tools/molecule_run.py --molecule naphthalene+ [--nroots 20] [--out FILE]
    python tools/molecule_run.py --molecule ch2
    python tools/molecule_run.py --molecule naphthalene+ --kind xsf [--sa 0]
    python tools/molecule_run.py --molecule naphthalene+ --kind sfup [--method 1]

* naphthalene+ : C10H8+ doublet, cc-pVDZ (180 AOs: the nao of BASELINE config C2's
  def2-SVP), ROKS B3LYP (the reference's default functional, XTDA.py:1526), X-TDA 20 roots;
* ch2          : CH2 3B1 triplet, 6-31G (13 AOs, BASELINE config C1), ROKS B3LYP, 5 roots.

Pipeline: device integrals and AO values, the integral-direct pivoted Cholesky factor of
the exact ERIs (no DF approximation: the reference's exact J/K), ROKS SCF on the device,
then XTDA(mf).kernel() (device operator + device Davidson, XTDA.py:746-829).  Check: the
device roots against the eigenvalues (w > 1e-3, XTDA.py:769-772) of the oracle's explicit
X-TDA matrix (oracle.xtda.full_diag_matrix, XTDA.py:56-400) on the same mean field, and a
residual |A x - e x| per root through a fresh device A.x.  Writes one JSON record.

--kind xsf: XSF_TDA(mf, SA).kernel() instead (the spin-flip-down, spin-adapted operator of
BASELINE C4 / C4d; ALDA0 kernel, OO block removed for ROKS, XSF_TDA.py:1501-1554), checked
against the lowest eigenvalues of the oracle's explicit XSF matrix (XSF_TDA.get_Amat,
XSF_TDA.py:265-395, oracle.xsf_tda.XSFOracle.get_amat + remove) with the same fglobal.

--kind sfup: SF_TDA(mf, isf=1, method).kernel() (spin-flip up, BASELINE C3's kind; method 1 =
the multicollinear kernel of C3mc, 50 samples as the reference's Davidson path), checked
against the oracle's explicit SF-up matrix (SF_TDA_up.get_Amat, SF_TDA.py:448-560) built on
the same kernel.
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))

# D2h naphthalene (Angstrom), long axis x, the fused C-C bond on the y axis
NAPHTHALENE = """C 0.0000 0.7164 0; C 0.0000 -0.7164 0;
C 1.2431 1.4002 0; C -1.2431 1.4002 0; C 1.2431 -1.4002 0; C -1.2431 -1.4002 0;
C 2.4262 0.7081 0; C -2.4262 0.7081 0; C 2.4262 -0.7081 0; C -2.4262 -0.7081 0;
H 1.2428 2.4878 0; H -1.2428 2.4878 0; H 1.2428 -2.4878 0; H -1.2428 -2.4878 0;
H 3.3700 1.2434 0; H -3.3700 1.2434 0; H 3.3700 -1.2434 0; H -3.3700 -1.2434 0"""
# CH2 3B1: C-H 1.075 A, H-C-H 133.9 degrees
CH2 = "C 0 0 0; H 0 0.98934 -0.42079; H 0 -0.98934 -0.42079"

MOLECULES = {
    "naphthalene+": dict(atom=NAPHTHALENE, basis="cc-pvdz", charge=1, spin=1, nroots=20,
                         label="naphthalene+ doublet / cc-pVDZ (BASELINE C2 class: nao 180)"),
    "ch2": dict(atom=CH2, basis="6-31g", charge=0, spin=2, nroots=5,
                label="CH2 3B1 / 6-31G (BASELINE C1)"),
}


def _rounded(d):
    if isinstance(d, dict):
        return {k: _rounded(v) for k, v in d.items()}
    return round(d, 3) if isinstance(d, float) else d


def _host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--molecule", default="naphthalene+", choices=sorted(MOLECULES))
    ap.add_argument("--nroots", type=int, default=None)
    ap.add_argument("--nstates", type=int, default=None,
                    help="roots the Davidson solves for (>= nroots; the Koopmans guess of the lowest gaps "
                         "may miss a symmetry block, XTDA.py:700-734)")
    ap.add_argument("--kind", default="xtda", choices=("xtda", "xsf", "sfup"))
    ap.add_argument("--method", type=int, default=0, help="spin-flip XC kernel: 0 ALDA0, 1 multicollinear")
    ap.add_argument("--sa", type=int, default=0, help="XSF spin adaptation (doublets: 0)")
    ap.add_argument("--xc", default="b3lyp")
    ap.add_argument("--tol", type=float, default=1e-12, help="Cholesky tolerance of the exact ERIs")
    ap.add_argument("--conv", type=float, default=1e-10)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    spec = MOLECULES[a.molecule]
    nroots = a.nroots or spec["nroots"]
    nstates = max(nroots, a.nstates or nroots)
    import torch
    from xtddft_amd.qc import M, ROKS
    from xtddft_amd.xtda import XTDA
    rec = dict(molecule=spec["label"], kind=a.kind, xc=a.xc, chol_tol=a.tol, nroots=nroots, nstates=nstates)
    t0 = time.perf_counter()
    mol = M(spec["atom"], basis=spec["basis"], charge=spec["charge"], spin=spec["spin"])
    rec.update(nao=mol.nao, natm=mol.natm, nelectron=mol.nelectron)
    mf = ROKS(mol, a.xc)
    mf.conv_tol = a.conv
    mf.max_cycle = 200
    mf.to_device(0).cholesky(a.tol)
    mf.build()
    torch.cuda.synchronize()
    rec["build_s"] = round(time.perf_counter() - t0, 3)
    rec["build_phases_s"] = _rounded(dict(mf.timings))
    rec["ngrid"] = int(mf.grids.size)
    print("build", json.dumps(rec), flush=True)
    t0 = time.perf_counter()
    mf.kernel()
    torch.cuda.synchronize()
    rec.update(scf_s=round(time.perf_counter() - t0, 3), scf_converged=bool(mf.converged), e_tot=mf.e_tot)
    print("scf", rec["scf_s"], mf.converged, mf.e_tot, flush=True)
    t0 = time.perf_counter()
    mfield = mf.to_meanfield()
    torch.cuda.synchronize()
    rec["meanfield_s"] = round(time.perf_counter() - t0, 3)
    if a.kind == "sfup":
        from xtddft_amd.sf_tda import DAVIDSON_SAMPLES, SF_TDA
        td = SF_TDA(mfield, isf=1, method=a.method)
        t0 = time.perf_counter()
        td.kernel(nstates=nstates)
        torch.cuda.synchronize()
        e = np.asarray(td.e)[:nstates]
        rec.update(xtda_s=round(time.perf_counter() - t0, 3), xtda_converged=bool(np.all(td.converged)),
                   method=a.method, roots_ha=[float(x) for x in e])
        print("sfup", rec["xtda_s"], e[:5], flush=True)
    elif a.kind == "xsf":
        from xtddft_amd.xsf_tda import XSF_TDA
        td = XSF_TDA(mfield, SA=a.sa)
        t0 = time.perf_counter()
        td.kernel(nstates=nstates)
        torch.cuda.synchronize()
        e = np.asarray(td.e)
        rec.update(xtda_s=round(time.perf_counter() - t0, 3), xtda_converged=bool(np.all(td.converged)),
                   fglobal=td.fglobal, sa=a.sa, remove=bool(td.re), davidson_iterations=int(td.icyc),
                   roots_ha=[float(x) for x in e])
        print("xsf", rec["xtda_s"], e[:5], flush=True)
    else:
        td = XTDA(None, mfield, nstates=nstates)
        t0 = time.perf_counter()
        e = np.asarray(td.kernel())
        torch.cuda.synchronize()
        op = td.operator()
        rec.update(xtda_s=round(time.perf_counter() - t0, 3), xtda_converged=bool(np.all(td.converged)),
                   operator_setup_s=_rounded(dict(op.setup_s)),
                   dim=int(op.dim), k_mode=op.k_mode, naux_cholesky=op.naux()[0],
                   roots_ha=[float(x) for x in e])
        x = td.v[np.argsort(td.order), :].T          # back to PySCF order
        ax = op.apply(np.ascontiguousarray(x))
        rec["max_residual"] = float(np.linalg.norm(ax - e[:, None] * x, axis=1).max())
        print("xtda", rec["xtda_s"], rec["dim"], e[:5], flush=True)
    if not a.no_oracle:
        import threading
        from oracle import xtda as oxtda
        from xtddft_amd.meanfield import Grid
        t0 = time.perf_counter()
        done = threading.Event()

        def heartbeat():     # the GPU box kills a run that prints nothing for 3 minutes
            while not done.wait(30.0):
                print(f"oracle explicit A: {time.perf_counter() - t0:.0f} s", flush=True)
        threading.Thread(target=heartbeat, daemon=True).start()
        mfo = dataclasses.replace(mfield, cderi=_host(mfield.cderi),
                                  grids=Grid(ao=_host(mfield.grids.ao), weights=_host(mfield.grids.weights)),
                                  fxc=_host(mfield.fxc),
                                  fxc_sf=None if mfield.fxc_sf is None else _host(mfield.fxc_sf))
        if a.kind == "sfup":
            from oracle import sf_tda as osf
            if a.method == 1:        # the kernel the device solve used (pinned on its own, test_qc.py)
                mfo.fxc_sf_mc = _host(mfield.extra[("fxc_sf_mc", DAVIDSON_SAMPLES)])
            A = osf.amat_up(mfo, method=a.method)
            rec["dim"] = int(A.shape[0])
        elif a.kind == "xsf":
            from oracle import xsf_tda as oxsf
            o = oxsf.XSFOracle(mfo, SA=a.sa)
            A = o.get_amat(foo=1.0, fglobal=oxsf.default_fglobal(mfo))
            if o.re:
                A = o.remove(A)
            rec["dim"] = int(A.shape[0])
        else:
            A = oxtda.full_diag_matrix(mfo)
        rec["oracle_symmetry"] = float(np.abs(A - A.T).max() / np.abs(A).max())
        wall = np.linalg.eigvalsh(0.5 * (A + A.T))
        if a.kind == "xtda":
            wall = wall[wall > 1e-3]
        w = wall[:nroots]
        rec["oracle_s"] = round(time.perf_counter() - t0, 1)
        rec["oracle_roots_ha"] = [float(v) for v in w]
        # the lowest nroots of the device solve against the lowest nroots of the spectrum, and
        # every device root against its nearest exact eigenvalue
        rec["max_abs_diff_ha"] = float(np.abs(e[:nroots] - w).max())
        rec["max_abs_diff_nearest_ha"] = float(np.abs(e[:, None] - wall[None, :]).min(axis=1).max())
        done.set()
        print("oracle", rec["oracle_s"], rec["max_abs_diff_ha"], flush=True)
    suffix = "" if a.kind == "xtda" else f"_{a.kind}" + (f"_mc" if a.method == 1 else "")
    out = a.out or f"gpurun_out/molecule_{a.molecule.replace('+', 'p')}{suffix}.json"
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
