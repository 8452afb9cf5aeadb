"""GPU: the molecular front end on the device.

The SCF's J/K and XC through the library's GEMM engine with the DF factor and
the grid in HBM (``qc.device.DeviceEngine``) against the host SCF: energies to
1e-9 Ha, the cached TDA kernels (fxc, ALDA0 fxc_ab) to round-off; and a
density-fitted mean field driving the device XSF-TDA to the reference's stored
roots within the DF error.
"""
import numpy as np
import pytest

from molecules import HF_IRREP_NELEC, hf_mol, reference_outputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch(hiplib):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _scf(kind, device, df=False, conv=1e-10):
    from xtddft_amd.qc import ROKS, UKS
    mf = (ROKS if kind == "ROKS" else UKS)(hf_mol(), "bhandhlyp")
    mf.irrep_nelec = dict(HF_IRREP_NELEC)
    mf.conv_tol = conv
    if df:
        mf.density_fit()
    if device:
        mf.to_device(0)
    mf.kernel()
    assert mf.converged
    return mf


@pytest.mark.parametrize("kind", ["ROKS", "UKS"])
def test_device_scf_equals_host(torch, kind):
    host, dev = _scf(kind, False), _scf(kind, True)
    assert dev.device_engine is not None
    assert abs(dev.e_tot - host.e_tot) < 1e-9
    assert abs(dev.e_tot - reference_outputs()[f"{kind.lower()}_bhandhlyp_e_tot"]) < 1e-8
    mh, md = host.to_meanfield(), dev.to_meanfield()
    assert np.abs(md.fxc - mh.fxc).max() < 1e-10 * np.abs(mh.fxc).max()
    assert np.abs(md.fxc_sf - mh.fxc_sf).max() < 1e-10 * np.abs(mh.fxc_sf).max()


def test_density_fitted_device_scf_and_xsf(torch):
    """DF mean field built on the device (no 4-index ERIs anywhere) drives the
    device XSF-TDA; roots within the DF error (~1e-4 Ha) of the reference's."""
    from molecules import HA2EV_XSF
    from xtddft_amd.xsf_tda import XSF_TDA
    host, dev = _scf("ROKS", False, df=True), _scf("ROKS", True, df=True)
    assert abs(dev.e_tot - host.e_tot) < 1e-9
    mf = dev.to_meanfield()
    assert mf.eri is None and mf.jk_mode == "DF"
    ref = reference_outputs()
    e, _ = XSF_TDA(mf).kernel(nstates=10, fglobal=ref["xsf_roks_alda0_fglobal"])
    assert np.abs(np.asarray(e) / HA2EV_XSF - np.asarray(ref["xsf_roks_alda0_ev"]) / HA2EV_XSF).max() < 5e-4


def _spd_mol():
    from xtddft_amd.qc import M
    basis = {"O": [[0, [30.0, 0.3], [6.0, 0.7]], [0, [0.9, 1.0]], [1, [5.0, 0.4], [1.1, 0.7]],
                   [2, [1.2, 1.0]]],
             "H": [[0, [3.0, 0.4], [0.5, 0.7]], [1, [0.8, 1.0]]]}
    atoms = [("O", (0.0, 0.0, 0.1)), ("H", (1.4, 1.0, 0.2)), ("H", (-1.3, 1.1, -0.4))]
    return M(atoms, basis=basis, unit="Bohr")


@pytest.mark.parametrize("omega", [0.0, 0.33])
@pytest.mark.parametrize("which", ["hf_631g", "spd"])
def test_device_int3c2e_equals_host(torch, which, omega):
    """The HIP 3-index integrals (csrc/xt_int.hip) against the host McMurchie-Davidson
    routine (qc/ints.py eri3c, itself checked against the 4-index routine):
    HF / 6-31G with its even-tempered auxiliary basis (aux l <= 3) and an s/p/d
    molecule (aux l <= 5; exponents up to 30 put the Boys argument on both sides of
    the series / asymptotic switch at T = 30).  Tolerance 1e-12 of the largest
    integral (FP64 round-off of a different summation order).  omega = 0.33: the
    long-range operator erf(omega r12)/r12."""
    from xtddft_amd.qc.df import aux_mole
    mol = hf_mol() if which == "hf_631g" else _spd_mol()
    aux = aux_mole(mol)
    host = mol.int3c2e(aux, omega=omega)
    dev = mol.int3c2e(aux, device=0, omega=omega)
    assert dev.shape == host.shape
    assert np.abs(dev - host).max() < 1e-12 * np.abs(host).max()


def test_density_fitted_scf_with_device_integrals(torch):
    """mf.density_fit() + mf.to_device(0): the DF factor's 3-index integrals come from
    the GPU; the SCF energy equals the host DF SCF to 1e-10 Ha."""
    host = _scf("ROKS", False, df=True)
    dev = _scf("ROKS", True, df=True)
    assert dev.with_df.device == 0
    assert abs(dev.e_tot - host.e_tot) < 1e-10


@pytest.mark.parametrize("omega", [0.0, 0.33])
@pytest.mark.parametrize("which", ["hf_631g", "spd"])
def test_device_eri_full_equals_host(torch, which, omega):
    """The 4-index ERIs through the same HIP kernel with the ket given as shell pairs
    (ket Hermite order up to 4, L <= 8) against the host routine, all 8 symmetry
    copies; tolerance 1e-12 of the largest integral."""
    mol = hf_mol() if which == "hf_631g" else _spd_mol()
    host = mol.eri_full(omega=omega)
    dev = mol.eri_full(device=0, omega=omega)
    assert np.abs(dev - host).max() < 1e-12 * np.abs(host).max()
    assert np.abs(dev - dev.transpose(2, 3, 0, 1)).max() == 0.0
