"""A BASELINE-class molecule end to end on the device, checked against the oracle.

    python tools/molecule_run.py --molecule naphthalene+ [--nroots 20] [--out FILE]
    python tools/molecule_run.py --molecule ch2
    python tools/molecule_run.py --molecule naphthalene+ --kind xsf [--sa 0]
    python tools/molecule_run.py --molecule naphthalene+ --kind sfup [--method 1]

* naphthalene+ : C10H8+ doublet, cc-pVDZ (180 AOs: the nao of BASELINE config C2's
  def2-SVP), ROKS B3LYP (the reference's default functional, XTDA.py:1526), X-TDA 20 roots;
* ch2          : CH2 3B1 triplet, 6-31G (13 AOs, BASELINE config C1), ROKS B3LYP, 5 roots;
* porphyrin    : free-base porphyrin C20H14N4 (the reference's own geometry, xtddft/utils/atom.py:313,
  Bohr), triplet, cc-pVDZ (406 AOs), ROKS BHandHLYP, SF-TDA up 30 roots (BASELINE C3's kind);
* c60-         : C60 anion doublet on the analytic truncated icosahedron (90 bonds of 1.43 A),
  cc-pVDZ (840 AOs = BASELINE C4's def2-SVP count), ROKS BHandHLYP, XSF-TDA SA = 0, 40 roots
  (BASELINE C4d's operator kind).

Large molecules (dim above --explicit-max) cannot be checked through an explicit A; they are
checked by (i) the device sigma = A z of one random vector against the oracle's AO-route vind
(XTDA.py:615-690 / SF_TDA.py:224-243 / XSF_TDA.py:1131-1276) on the SAME mean field (the same
Cholesky factor, grid and kernel, copied to host memory), and (ii) every converged root's
residual |A x - e x| through a fresh device A.x.  The exact ERIs are factorised to the stated
Cholesky tolerance (--tol; the molecule's default), which both sides share.

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

# free-base porphyrin, xtddft/utils/atom.py:313-351 (TPSS-D3/def2-TZVP geometry, Bohr)
PORPHYRIN = """C -8.03864054980912 1.28355565610347 0; C -8.03864054980912 -1.28355565610347 0;
C -5.39342598970294 -2.05504973592643 0; C -4.61107220150279 -4.57965767758428 0;
N -3.82524921858544 0 0; C -5.39342598970294 2.05504973592643 0;
C -4.61107220150279 4.57965767758428 0; C -2.13573683447591 5.47424067772668 0;
N 0 3.99808810865002 0; C -1.29753280957893 8.05049347032883 0;
C 2.13573683447591 5.47424067772668 0; C 1.29753280957893 8.05049347032883 0;
C 4.61107220150279 4.57965767758428 0; C 5.39342598970294 2.05504973592643 0;
C 8.03864054980912 1.28355565610347 0; N 3.82524921858544 0 0;
C 5.39342598970294 -2.05504973592643 0; C 8.03864054980912 -1.28355565610347 0;
C 4.61107220150279 -4.57965767758428 0; C 2.13573683447591 -5.47424067772668 0;
C 1.29753280957893 -8.05049347032883 0; N 0 -3.99808810865002 0;
C -1.29753280957893 -8.05049347032883 0; C -2.13573683447591 -5.47424067772668 0;
H 9.64345627077377 2.55368984858905 0; H 9.64345627077377 -2.55368984858905 0;
H 6.08263565411431 -6.01054939209590 0; H 2.54767382892794 -9.66722194409625 0;
H -2.54767382892794 -9.66722194409625 0; H 0 -2.07347199362234 0;
H -6.08263565411431 -6.01054939209590 0; H -9.64345627077377 2.55368984858905 0;
H -9.64345627077377 -2.55368984858905 0; H -6.08263565411431 6.01054939209590 0;
H 0 2.07347199362234 0; H 2.54767382892794 9.66722194409625 0;
H -2.54767382892794 9.66722194409625 0; H 6.08263565411431 6.01054939209590 0"""


def c60_geometry(bond: float = 1.43) -> str:
    """Truncated icosahedron with every edge ``bond`` Angstrom: the 60 even (cyclic)
    permutations of (0, +-1, +-3 phi), (+-1, +-(2 + phi), +-2 phi), (+-phi, +-2, +-(2 phi + 1))
    of the edge-2 solid, scaled."""
    import itertools
    phi = (1 + 5 ** 0.5) / 2
    pts = set()
    for b in ((0.0, 1.0, 3 * phi), (1.0, 2 + phi, 2 * phi), (phi, 2.0, 2 * phi + 1)):
        for cyc in ((0, 1, 2), (1, 2, 0), (2, 0, 1)):
            for sg in itertools.product((1, -1), repeat=3):
                pts.add(tuple(round(sg[k] * b[cyc[k]], 12) + 0.0 for k in range(3)))
    xyz = np.array(sorted(pts)) * (bond / 2.0)
    assert xyz.shape == (60, 3)
    return "; ".join(f"C {x:.12f} {y:.12f} {z:.12f}" for x, y, z in xyz)


MOLECULES = {
    "naphthalene+": dict(atom=NAPHTHALENE, basis="cc-pvdz", charge=1, spin=1, nroots=20,
                         label="naphthalene+ doublet / cc-pVDZ (BASELINE C2 class: nao 180)"),
    "ch2": dict(atom=CH2, basis="6-31g", charge=0, spin=2, nroots=5,
                label="CH2 3B1 / 6-31G (BASELINE C1)"),
    "porphyrin": dict(atom=PORPHYRIN, unit="Bohr", basis="cc-pvdz", charge=0, spin=2, nroots=30,
                      kind="sfup", xc="bhandhlyp", tol=1e-8,
                      label="free-base porphyrin triplet / cc-pVDZ (atom.py:313; BASELINE C3 class: SF-up)"),
    "c60-": dict(atom=None, basis="cc-pvdz", charge=-1, spin=1, nroots=40, kind="xsf", sa=0,
                 xc="bhandhlyp", tol=1e-8,
                 label="C60- doublet / cc-pVDZ (nao 840 = BASELINE C4's; XSF-TDA SA = 0, C4d's kind)"),
}


def _rounded(d):
    if isinstance(d, dict):
        return {k: (v if k == "tol" else _rounded(v)) for k, v in d.items()}
    return round(d, 3) if isinstance(d, float) else d


def _host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


class _DevSlicer:
    """A device tensor the oracle reads block by block (x[key] copies that block to host)."""

    def __init__(self, t):
        self.t, self.shape = t, tuple(t.shape)

    def __getitem__(self, key):
        return self.t[key].cpu().numpy()


def _cpus():
    """CPUs this process may use (affinity mask capped by the cgroup quota, as bench.cpu_share)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(p))))
    except (OSError, ValueError):
        pass
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--molecule", default="naphthalene+", choices=sorted(MOLECULES))
    ap.add_argument("--nroots", type=int, default=None)
    ap.add_argument("--nstates", type=int, default=None,
                    help="roots the Davidson solves for (>= nroots; the Koopmans guess of the lowest gaps "
                         "may miss a symmetry block, XTDA.py:700-734)")
    ap.add_argument("--kind", default=None, choices=("xtda", "xsf", "sfup"))
    ap.add_argument("--method", type=int, default=0, help="spin-flip XC kernel: 0 ALDA0, 1 multicollinear")
    ap.add_argument("--sa", type=int, default=None, help="XSF spin adaptation (doublets: 0)")
    ap.add_argument("--xc", default=None)
    ap.add_argument("--tol", type=float, default=None, help="Cholesky tolerance of the exact ERIs")
    ap.add_argument("--conv", type=float, default=1e-10)
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--explicit-max", type=int, default=12000,
                    help="largest dim checked through the oracle's explicit A; above it, sigma parity")
    ap.add_argument("--scf-only", action="store_true")
    ap.add_argument("--factor-host", default="auto", choices=("auto", "on", "off"),
                    help="after the SCF, keep the AO Cholesky factor in host memory instead of HBM "
                         "(auto: nao >= 600), so the operator's stored exchange fits beside its MO factor")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    spec = MOLECULES[a.molecule]
    a.kind = a.kind or spec.get("kind", "xtda")
    a.sa = spec.get("sa", 0) if a.sa is None else a.sa
    a.xc = a.xc or spec.get("xc", "b3lyp")
    a.tol = a.tol or spec.get("tol", 1e-12)
    atom = spec["atom"] if spec["atom"] is not None else c60_geometry()
    nroots = a.nroots or spec["nroots"]
    nstates = max(nroots, a.nstates or nroots)
    import torch
    from xtddft_amd.qc import M, ROKS
    from xtddft_amd.xtda import XTDA
    import threading
    t_start = time.perf_counter()
    phase = {"name": "start"}
    stop = threading.Event()

    def heartbeat():     # the GPU box kills a run that prints nothing for 3 minutes
        while not stop.wait(30.0):
            print(f"[{time.perf_counter() - t_start:.0f} s] {phase['name']} ...", flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    rec = dict(molecule=spec["label"], kind=a.kind, xc=a.xc, chol_tol=a.tol, nroots=nroots, nstates=nstates)
    t0 = time.perf_counter()
    phase["name"] = "molecule + one-electron integrals + Cholesky + grid"
    mol = M(atom, basis=spec["basis"], charge=spec["charge"], spin=spec["spin"], unit=spec.get("unit", "Angstrom"))
    rec.update(nao=mol.nao, natm=mol.natm, nelectron=mol.nelectron)
    mf = ROKS(mol, a.xc)
    mf.conv_tol = a.conv
    mf.max_cycle = 200
    mf.verbose = 1
    mf.to_device(0).cholesky(a.tol)
    mf.build()
    torch.cuda.synchronize()
    rec["build_s"] = round(time.perf_counter() - t0, 3)
    rec["build_phases_s"] = _rounded(dict(mf.timings))
    rec["ngrid"] = int(mf.grids.size)
    rec["gpu_mem_gib_after_build"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)
    print("build", json.dumps(rec), flush=True)
    phase["name"] = "SCF"
    t0 = time.perf_counter()
    mf.kernel()
    torch.cuda.synchronize()
    rec.update(scf_s=round(time.perf_counter() - t0, 3), scf_converged=bool(mf.converged), e_tot=mf.e_tot)
    print("scf", rec["scf_s"], mf.converged, mf.e_tot, flush=True)
    rec["homo_lumo_ha"] = [float(x) for x in mf.mo_energy[mol.nelec[1] - 1:mol.nelec[0] + 1]]
    if a.scf_only:
        _write(a, rec)
        return
    phase["name"] = "mean field (kernels on the grid)"
    t0 = time.perf_counter()
    mfield = mf.to_meanfield()
    torch.cuda.synchronize()
    rec["meanfield_s"] = round(time.perf_counter() - t0, 3)
    if a.factor_host == "on" or (a.factor_host == "auto" and mol.nao >= 600):
        # the operator transforms the AO factor to its MO factor once (xt_set_jk_df stages host
        # input in chunks); the SCF's HBM copy (54 GB for C60 at tol 1e-8) would otherwise keep
        # the stored MO exchange out of HBM (the auto rule takes the free memory)
        mfield.cderi = mfield.cderi.cpu() if hasattr(mfield.cderi, "cpu") else mfield.cderi
        mf.cderi_exact = None
        mf.device_engine = None
        torch.cuda.empty_cache()
        rec["factor_in_host_memory"] = True
    phase["name"] = f"{a.kind} solve"
    if a.kind == "sfup":
        from xtddft_amd.sf_tda import DAVIDSON_SAMPLES, SF_TDA
        td = SF_TDA(mfield, isf=1, method=a.method)
        t0 = time.perf_counter()
        td.kernel(nstates=nstates)
        torch.cuda.synchronize()
        e = np.asarray(td.e)[:nstates]
        op = td._op
        rec.update(xtda_s=round(time.perf_counter() - t0, 3), xtda_converged=bool(np.all(td.converged)),
                   method=a.method, dim=int(op.dim), k_mode=op.k_mode, roots_ha=[float(x) for x in e])
        x = np.ascontiguousarray(np.asarray(td.v)[:, :nstates].T)
        rec["max_residual"] = float(np.linalg.norm(op.apply_full(x) - e[:, None] * x, axis=1).max())
        print("sfup", rec["xtda_s"], e[:5], flush=True)
    elif a.kind == "xsf":
        from xtddft_amd.xsf_tda import XSF_TDA
        td = XSF_TDA(mfield, SA=a.sa)
        t0 = time.perf_counter()
        td.kernel(nstates=nstates)
        torch.cuda.synchronize()
        e = np.asarray(td.e)
        op = td._op
        rec.update(xtda_s=round(time.perf_counter() - t0, 3), xtda_converged=bool(np.all(td.converged)),
                   fglobal=td.fglobal, sa=a.sa, remove=bool(td.re), davidson_iterations=int(td.icyc),
                   dim=int(op.dim), k_mode=op.k_mode, roots_ha=[float(x) for x in e])
        x = np.ascontiguousarray(np.asarray(td.v)[:, :nstates].T)
        rec["max_residual"] = float(np.linalg.norm(op.apply_full(x) - e[:, None] * x, axis=1).max())
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
    stop.set()
    if not a.no_oracle:
        from xtddft_amd.meanfield import Grid
        t0 = time.perf_counter()
        phase["name"] = "oracle"
        stop.clear()
        threading.Thread(target=heartbeat, daemon=True).start()
        big = rec["dim"] > a.explicit_max
        ng = int(mfield.grids.weights.shape[0])
        # the grid AO values stay in HBM for large molecules: the oracle reads them block by block
        ao = mfield.grids.ao
        if big and hasattr(ao, "cpu"):
            # ALDA0 spin flip reads AO values only; X-TDA and the multicollinear kernel need gradients
            ao = _DevSlicer(ao[:1] if (a.kind != "xtda" and a.method == 0) else ao)
        else:
            ao = _host(ao)
        mfo = dataclasses.replace(mfield, cderi=_host(mfield.cderi),
                                  grids=Grid(ao=ao, weights=_host(mfield.grids.weights)),
                                  fxc=_host(mfield.fxc),
                                  fxc_sf=None if mfield.fxc_sf is None else _host(mfield.fxc_sf),
                                  extra=dict(mfield.extra))
        if a.kind == "sfup" and a.method == 1:   # the kernel the device solve used (pinned, test_qc.py)
            mfo.fxc_sf_mc = _host(mfield.extra[("fxc_sf_mc", DAVIDSON_SAMPLES)])
        if big:
            # sigma parity of one random vector on the same mean field (AO route, reference algorithm)
            from threadpoolctl import threadpool_limits
            z = np.random.default_rng(20261018).standard_normal((1, rec["dim"]))
            z /= np.linalg.norm(z)
            s_dev = np.asarray(op.apply_full(z) if a.kind != "xtda" else op.apply(z))
            if a.kind == "sfup":
                from oracle import sf_tda as osf
                vind = osf.gen_tda_operation_sf(mfo, 1, method=a.method)[0]
            elif a.kind == "xsf":
                from oracle import xsf_tda as oxsf
                o = oxsf.XSFOracle(mfo, SA=a.sa)
                o.re = bool(td.re)
                vind = o.gen_tda_operation_sf(foo=1.0, fglobal=td.fglobal, with_hdiag=False)[0]
            else:
                from oracle import xtda as oxtda
                vind = oxtda.gen_tda_operation(mfo)[0]
            with threadpool_limits(limits=_cpus()):
                s_or = np.asarray(vind(z)).reshape(s_dev.shape)
            rec["verify"] = dict(rel_err=float(np.abs(s_dev - s_or).max() / np.abs(s_or).max()),
                                 max_abs_sigma=float(np.abs(s_or).max()), cpus=_cpus(), ngrid=ng,
                                 what="max |sigma_gpu - sigma_oracle| / max |sigma_oracle|, one random unit "
                                      "vector, oracle AO route on the same mean field", tol=1e-12)
            rec["oracle_s"] = round(time.perf_counter() - t0, 1)
            print("oracle sigma", rec["oracle_s"], rec["verify"]["rel_err"], flush=True)
        else:
            if a.kind == "sfup":
                from oracle import sf_tda as osf
                A = osf.amat_up(mfo, method=a.method)
            elif a.kind == "xsf":
                from oracle import xsf_tda as oxsf
                o = oxsf.XSFOracle(mfo, SA=a.sa)
                A = o.get_amat(foo=1.0, fglobal=oxsf.default_fglobal(mfo))
                if o.re:
                    A = o.remove(A)
            else:
                from oracle import xtda as oxtda
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
            print("oracle", rec["oracle_s"], rec["max_abs_diff_ha"], flush=True)
        stop.set()
    rec["total_s"] = round(time.perf_counter() - t_start, 1)
    _write(a, rec)


def _write(a, rec):
    suffix = "" if a.kind == "xtda" else f"_{a.kind}" + (f"_mc" if a.method == 1 else "")
    out = a.out or f"gpurun_out/molecule_{a.molecule.replace('+', 'p')}{suffix}.json"
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
