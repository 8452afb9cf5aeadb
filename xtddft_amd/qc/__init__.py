"""Molecular front end for the TDA hot path.

The reference builds every operator from a PySCF ``mol`` / ``mf`` pair
(``gto.M``, ``dft.ROKS`` / ``dft.UKS``, ``mf.kernel()``).  PySCF is not part of
this framework, so this subpackage provides what those calls produce for the
hot path, from scratch:

* ``gto``   -- ``Mole`` (atoms, Gaussian basis, spherical AOs normalised as in
  libcint), one-electron integrals (S, T, V, dipole) and 4-index ERIs by the
  McMurchie-Davidson scheme (``ints``).
* ``grid``  -- PySCF-default DFT grids: Treutler-Ahlrichs M4 radial grids,
  Lebedev angular grids, NWChem pruning, Becke partitioning with Treutler
  radii adjustment; AO values and gradients on the grid.
* ``xc``    -- Slater / B88 exchange, VWN5 / LYP correlation and the hybrids
  built from them (BHandHLYP, B3LYP), with first and second functional
  derivatives in PySCF's ``eval_xc_eff`` layout (autograd, float64).
* ``scf``   -- ROKS / UKS (and ROHF / UHF) SCF with optional ``irrep_nelec``
  occupation constraints, producing the ``MeanField`` the TDA drivers consume
  (``mo_coeff``, ``mo_occ``, ``mo_energy``, KS and pure-HF potentials, the
  stored ERIs, the grid and the cached XC kernels).

This is host-side input preparation (what PySCF does in the reference); the
hot path itself (A.x and the Davidson solver) runs in the HIP library.
"""
from .gto import Mole, M
from .scf import ROKS, UKS, ROHF, UHF

__all__ = ["Mole", "M", "ROKS", "UKS", "ROHF", "UHF"]
