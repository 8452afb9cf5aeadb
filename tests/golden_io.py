"""Save / load golden fixtures: full MeanField inputs + trial vectors + oracle outputs."""
import os

import numpy as np

from xtddft_amd.meanfield import Grid, MeanField, Mole

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

ARRAYS = ["mo_coeff", "mo_occ", "mo_energy", "h1e", "veff", "veff_hf", "cderi", "cderi_lr",
          "fxc", "fxc_sf"]


def save(name, mf, **extra):
    d = {k: getattr(mf, k) for k in ARRAYS if getattr(mf, k) is not None}
    if mf.grids is not None:
        d["grid_ao"] = mf.grids.ao
        d["grid_w"] = mf.grids.weights
    d["scalars"] = np.array([mf.mol.nao, mf.mol.spin, mf.omega, mf.alpha, mf.hyb])
    d["xctype"] = np.array(mf.xctype)
    d.update(extra)
    np.savez_compressed(os.path.join(GOLDEN, name + ".npz"), **d)


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    nao, spin, omega, alpha, hyb = z["scalars"]
    grids = Grid(ao=z["grid_ao"], weights=z["grid_w"]) if "grid_ao" in z else None
    mf = MeanField(mol=Mole(nao=int(nao), spin=int(spin)), mo_coeff=z["mo_coeff"],
                   mo_occ=z["mo_occ"], mo_energy=z["mo_energy"], h1e=z["h1e"], veff=z["veff"],
                   veff_hf=z["veff_hf"], cderi=z["cderi"], grids=grids,
                   fxc=z["fxc"] if "fxc" in z else None, fxc_sf=z["fxc_sf"] if "fxc_sf" in z else None,
                   cderi_lr=z["cderi_lr"] if "cderi_lr" in z else None, xctype=str(z["xctype"]),
                   omega=float(omega), alpha=float(alpha), hyb=float(hyb))
    extra = {k: z[k] for k in z.files if k.startswith("out_") or k.startswith("in_")}
    return mf, extra


def list_cases():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))
