"""Index utilities and unit constants (reference ``xtddft/utils``).

* ``order_pyscf2my`` -- permutation from PySCF's X-TDA vector order
  ``[za (nocc_a x nvir_a) | zb (nocc_b x nvir_b)]`` (zb rows = [CO(i,.)|CV(i,.)])
  to the reference's "my order" CV(0), OV(0), CO(0), CV(1) (utils.py:44-64).
  Built in closed form rather than by repeated insert/delete.
* ``so2st`` / ``st2so`` -- spin-orbital <-> spin-tensor rotation of the CV
  blocks (utils.py:67-122).
* ``HA2EV`` etc. -- ``unit.py`` constants (ORCA's 27.2113834, unit.py:8) and
  the 27.21138505 factor XSF_TDA.kernel uses (XSF_TDA.py:1554).
"""
from __future__ import annotations

import numpy as np

HA2EV = 27.2113834
HA2EV_XSF = 27.21138505
EVXNM = 1239.84193


def order_pyscf2my(nc: int, no: int, nv: int) -> np.ndarray:
    """my_vector = pyscf_vector[order]."""
    na = (nc + no) * nv
    alpha = np.arange(na)
    base = na + np.arange(nc)[:, None] * (no + nv)
    co = (base + np.arange(no)[None, :]).ravel()
    cv = (base + no + np.arange(nv)[None, :]).ravel()
    return np.concatenate([alpha, co, cv]).astype(np.int64)


def order_sf_down(nc: int, no: int, nv: int) -> np.ndarray:
    """Spin-flip-down vector order: PySCF's (occ_a x vir_b) row-major layout ->
    the reference's cv|co|ov|oo blocks, block_vector = pyscf_vector[order]
    (``deal_v_davidson``, SF_TDA.py:304-345; the explicit A of
    SF_TDA_down.get_Amat is assembled in the same block order, SF_TDA.py:746-801)."""
    vir = no + nv
    rows_c = np.arange(nc)[:, None] * vir
    rows_o = (nc + np.arange(no))[:, None] * vir
    cv = (rows_c + no + np.arange(nv)[None, :]).ravel()
    co = (rows_c + np.arange(no)[None, :]).ravel()
    ov = (rows_o + no + np.arange(nv)[None, :]).ravel()
    oo = (rows_o + np.arange(no)[None, :]).ravel()
    return np.concatenate([cv, co, ov, oo]).astype(np.int64)


def so2st(eigvec, nc, no, nv):
    """Spin-orbital -> spin-tensor basis for vectors stacked as columns."""
    cva = eigvec[:nc * nv]
    ova = eigvec[nc * nv:(nc + no) * nv]
    cob = eigvec[(nc + no) * nv:(nc + no) * nv + no * nc]
    cvb = eigvec[(nc + no) * nv + no * nc:]
    r = np.sqrt(2) / 2
    return np.concatenate((r * (cva + cvb), ova, cob, r * (cva - cvb)), axis=0)


def st2so(eigvec, nc, no, nv):
    cv0 = eigvec[:nc * nv]
    ov0 = eigvec[nc * nv:(nc + no) * nv]
    co0 = eigvec[(nc + no) * nv:(nc + no) * nv + no * nc]
    cv1 = eigvec[(nc + no) * nv + no * nc:]
    return np.concatenate(((cv0 + cv1) / np.sqrt(2), ov0, co0, (cv0 - cv1) / np.sqrt(2)), axis=0)


NLC_SF_WARNING = ('NLC functional found in DFT object.  Its second derivative is not available. '
                  'Its contribution is not included in the response function.')


def nlc_check(mf, davidson_xtda=False):
    """The reference's treatment of a VV10 (NLC) functional: the X-TDA / U-TDA Davidson
    response adds ``get_vnlc_resp`` (XTDA.py:515-517), which is not built here, so that path
    refuses; every other path (explicit X-TDA A, XTDA.py:166-169; SF-TDA, SF_TDA.py:490-493,
    669-672, 869-872; XSF-TDA through the same kernels) leaves it out with this warning."""
    if not getattr(mf, "nlc", False):
        return
    if davidson_xtda:
        raise NotImplementedError("the VV10 (NLC) response term of the X-TDA Davidson path "
                                  "(XTDA.py:515-517, pyscf.hessian.rks.get_vnlc_resp) is not built; "
                                  "use_Davidson=False runs the explicit A, which leaves it out as the "
                                  "reference does")
    import warnings
    warnings.warn(NLC_SF_WARNING, RuntimeWarning, stacklevel=3)
