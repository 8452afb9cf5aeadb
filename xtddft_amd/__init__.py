"""xtddft_amd -- MI355X-native TDA response hot path of XTDDFT.

Reference-compatible entry points (PySCF-style operator API):

* ``XTDA(mol, mf, ...)``                (xtddft/XTDA.py)
* ``SF_TDA(mf, isf, davidson, method)`` (xtddft/SF_TDA.py) and
  ``gen_tda_operation_sf``, ``init_guess``, ``davidson_process``
* ``XSF_TDA(mf, SA, ...)``              (xtddft/XSF_TDA.py)
* ``davidson1``                         (xtddft/utils/Davidson.py)

The arithmetic runs in the HIP library ``_lib/libxtddft_amd.so`` (C ABI in
``include/xtddft_amd.h``); there is no CPU fallback.
"""
from .meanfield import Grid, MeanField, Mole
from .utils import HA2EV, HA2EV_XSF, order_pyscf2my, so2st, st2so

__all__ = ["Grid", "MeanField", "Mole", "HA2EV", "HA2EV_XSF", "order_pyscf2my", "so2st", "st2so",
           "XTDA", "SF_TDA", "SF_TDA_up", "SF_TDA_down", "XSF_TDA", "davidson1", "DeviceOperator"]


def __getattr__(name):   # lazy: importing the package must not require a GPU
    if name == "XTDA":
        from .xtda import XTDA
        return XTDA
    if name in ("SF_TDA", "SF_TDA_up", "SF_TDA_down"):
        from . import sf_tda
        return getattr(sf_tda, name)
    if name == "XSF_TDA":
        from .xsf_tda import XSF_TDA
        return XSF_TDA
    if name == "davidson1":
        from .davidson import davidson1
        return davidson1
    if name == "DeviceOperator":
        from .operator import DeviceOperator
        return DeviceOperator
    raise AttributeError(name)
