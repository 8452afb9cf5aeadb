"""Generate the golden fixtures in tests/golden/ with the CPU oracle.

    python tests/golden/make_golden.py

Each fixture holds the full synthetic inputs (so it does not depend on RNG
reproducibility), trial vectors, the oracle's sigma = A z and the lowest
eigenvalues of the oracle's explicit A (reference code path full_diag /
get_Amat).  The reference itself cannot run here, so these
are oracle pins, not reference outputs -- see DESIGN.md "Oracle".
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from xtddft_amd.synthetic import make_mf, make_trial_vectors  # noqa: E402
from oracle import sf_tda, xsf_tda, xtda  # noqa: E402
from golden_io import save  # noqa: E402

CASES = {
    "xtda_ro_gga": dict(kind="XTDA", mf=dict(nao=16, nc=4, no=2, naux=48, ngrid=320, xctype="GGA", hyb=0.2)),
    "xtda_ro_lda_rsh": dict(kind="XTDA", mf=dict(nao=16, nc=4, no=2, naux=48, ngrid=320, xctype="LDA",
                                               hyb=0.19, omega=0.33, alpha=0.65)),
    "xtda_ro_hf_no1": dict(kind="XTDA", mf=dict(nao=14, nc=4, no=1, naux=42, xctype="HF")),
    "utda_u_gga": dict(kind="UTDA", mf=dict(nao=16, nc=4, no=2, naux=48, ngrid=320, xctype="GGA", hyb=0.2,
                                           kind="U")),
    "sf_down_ro_gga": dict(kind="SF_DOWN", mf=dict(nao=16, nc=4, no=2, naux=48, ngrid=320, xctype="GGA",
                                                  hyb=0.5)),
    "sf_up_u_lda": dict(kind="SF_UP", mf=dict(nao=16, nc=4, no=2, naux=48, ngrid=320, xctype="LDA", hyb=0.5,
                                             kind="U")),
    "xsf_ro_sa3_no3": dict(kind="XSF", mf=dict(nao=18, nc=4, no=3, naux=54, ngrid=360, xctype="GGA",
                                              hyb=0.5)),
}


def operator(kind, mf):
    if kind in ("XTDA", "UTDA"):
        vind, hdiag = xtda.gen_tda_operation(mf)
    elif kind == "SF_DOWN":
        vind, hdiag = sf_tda.gen_tda_operation_sf(mf, -1)
    elif kind == "SF_UP":
        vind, hdiag = sf_tda.gen_tda_operation_sf(mf, 1)
    else:
        o = xsf_tda.XSFOracle(mf, SA=3)
        vind, hdiag = o.gen_tda_operation_sf(foo=1.0, fglobal=xsf_tda.default_fglobal(mf))
    return vind, hdiag


def main():
    for name, case in CASES.items():
        mf = make_mf(**case["mf"])
        vind, hdiag = operator(case["kind"], mf)
        z = make_trial_vectors(5, hdiag.size, seed=11)
        sigma = vind(z)
        a = vind(np.eye(hdiag.size)).T
        e = np.linalg.eigvalsh(0.5 * (a + a.T))[:6]
        save(name, mf, in_z=z, out_sigma=sigma, out_hdiag=hdiag, out_eig=e,
             in_kind=np.array(case["kind"]))
        print(name, hdiag.size, e[:3])


if __name__ == "__main__":
    main()
