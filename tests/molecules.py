"""Real-molecule mean fields for parity against the reference's stored outputs.

The molecules are the ones the reference's example notebooks ran (see
``tests/golden/extract_reference_outputs.py``); the SCF runs here through
``xtddft_amd.qc`` (integrals, PySCF-default grid, BHandHLYP, ROKS/UKS with
``irrep_nelec``) and is cached per process.
"""
import json
import os
from functools import lru_cache

from xtddft_amd.qc import M, ROKS, UKS

HERE = os.path.dirname(os.path.abspath(__file__))
HA2EV_XSF = 27.21138505          # XSF_TDA.py:1554

HF_GEOM = "F 0 0 0; H 0 0 1.0"   # example/XSF_TDA.ipynb cell 1
HF_IRREP_NELEC = {"A1": (4, 2), "B1": (1, 1), "B2": (1, 1)}


@lru_cache(maxsize=None)
def reference_outputs():
    with open(os.path.join(HERE, "golden", "reference_outputs.json")) as f:
        return json.load(f)


@lru_cache(maxsize=None)
def hf_mol():
    return M(HF_GEOM, basis="6-31G", charge=0, spin=2, symmetry="C2v")


@lru_cache(maxsize=None)
def hf_scf(kind: str):
    """Converged SCF object: 'ROKS' / 'UKS' with the notebook's irrep_nelec,
    'ROKS_AUFBAU' = example/spin up.ipynb (H 0 0 0; F 0 0 1.0, no constraint)."""
    if kind == "ROKS_AUFBAU":
        mol = M("H 0 0 0; F 0 0 1.0", basis="6-31G", spin=2, symmetry="C2v")
        mf = ROKS(mol, "bhandhlyp")
    else:
        mf = (ROKS if kind == "ROKS" else UKS)(hf_mol(), "bhandhlyp")
        mf.irrep_nelec = dict(HF_IRREP_NELEC)
    mf.conv_tol = 1e-11
    mf.kernel()
    assert mf.converged
    return mf


@lru_cache(maxsize=None)
def hf_meanfield(kind: str):
    return hf_scf(kind).to_meanfield()
