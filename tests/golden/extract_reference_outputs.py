"""Extract the reference's own stored results into ``reference_outputs.json``.

Run in the build container (``/root/reference`` exists only there):

    python tests/golden/extract_reference_outputs.py

Sources (PySCF 2.12.1 / libxc 7.0.0 runs recorded by the reference authors):

* ``example/XSF_TDA.ipynb`` cell 1  -- HF molecule (F 0 0 0; H 0 0 1.0 A), 6-31G,
  spin 2, C2v, ``irrep_nelec {'A1':(4,2),'B1':(1,1),'B2':(1,1)}``, ROKS/BHandHLYP:
  nuclear repulsion, cond(S), per-atom pruned grid sizes, total grid count,
  converged SCF energy, final Roothaan orbital energies.
* cell 2 -- XSF-TDA (ALDA0, SA=3, remove=True) 10 roots in eV.
* cell 3 -- XSF-TDA with the multicollinear kernel (``method=1``, 60 collinear
  samples; the BHandHLYP fit makes fglobal = 0) 10 roots in eV, and the printed
  fglobal.
* cell 5 / 6 -- the same molecule with UKS: SCF energy, USF-TDA (XSF_TDA on a
  UKS mf: SA=0, no OO compression) 10 roots in eV and the Delta<S^2> list.
* cell 7 -- USF-TDA with the multicollinear kernel: 10 roots, Delta<S^2> list.
* ``example/spin up.ipynb`` cell 1 -- H 0 0 0; F 0 0 1.0 A ROKS/BHandHLYP aufbau
  triplet SCF energy.
* ``example/TDA.ipynb`` (PySCF 2.11.0 / libxc 7.0.0), B3LYP / cc-pVDZ,
  conv_tol 1e-11: cell 2 -- N2 RKS (shell / primitive / AO counts, nuclear
  repulsion, total grid count, SCF energy, closed-shell TDA singlet roots: the
  4-decimal table and the 5-decimal "Excited state N  x eV" lines of tda.analyze());
  cell 4 -- CH2O+ (``atom.ch2o_vacuum``) UKS: SCF energy and the U-TDA table
  (energy eV, oscillator strength, Delta<S^2>, 12 roots); cell 6 -- the same
  cation with ROKS: SCF energy and the X-TDA table (``XTDA.kernel``, the
  headline operator kind).

Only numbers are extracted (the fixture is data); no reference code is copied.
"""
from __future__ import annotations

import json
import os
import re

import numpy as np

REF = "/root/reference/example"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_outputs.json")


def _outputs(cell):
    texts = []
    for o in cell.get("outputs", []):
        t = "".join(o.get("text", ""))
        if not t and "data" in o:
            t = "".join(o["data"].get("text/plain", ""))
        texts.append(t)
    return texts


def _floats(s):
    return [float(x) for x in re.findall(r"[-+]?\d+\.\d+(?:e[-+]?\d+)?", s)]


def _bracket_after(text, key):
    i = text.index(key)
    j = text.index("[", i)
    k = text.index("]", j)
    return text[j + 1:k]


def main():
    nb = json.load(open(os.path.join(REF, "XSF_TDA.ipynb")))
    cells = nb["cells"]
    out = {"source": "reference example notebooks (PySCF 2.12.1, libxc 7.0.0)"}

    log = "\n".join(_outputs(cells[1]))
    out["hf_631g_nuclear_repulsion"] = float(re.search(r"nuclear repulsion = ([-\d.]+)", log).group(1))
    out["hf_631g_cond_S"] = float(re.search(r"cond\(S\) = ([-\d.]+)", log).group(1))
    out["hf_631g_grid_ang_F"] = [int(x) for x in _bracket_after(log, "atom F rad-grids").split()]
    out["hf_631g_grid_ang_H"] = [int(x) for x in _bracket_after(log, "atom H rad-grids").split()]
    out["hf_631g_tot_grids_padded"] = int(re.search(r"tot grids = (\d+)", log).group(1))
    out["hf_631g_padding"] = int(re.search(r"Padding (\d+) grids", log).group(1))
    out["roks_bhandhlyp_e_tot"] = float(re.search(r"converged SCF energy = ([-\d.]+)", log).group(1))
    roothaan = log.rsplit("Roothaan mo_energy =", 1)[1]
    out["roks_bhandhlyp_mo_energy_last_cycle"] = _floats(roothaan[:roothaan.index("]")])

    xsf = "\n".join(_outputs(cells[2]))
    out["xsf_roks_alda0_fglobal"] = float(re.search(r"fglobal ([-\d.]+)", xsf).group(1))
    # the eigenvalue list is the bracket after the "Converged [True ...]" line
    out["xsf_roks_alda0_ev"] = _floats(xsf[xsf.index("]", xsf.index("Converged")) + 1:].split("]")[0])
    mc = "\n".join(_outputs(cells[3]))
    out["xsf_roks_mc_fglobal"] = float(re.search(r"fglobal ([-\d.]+)", mc).group(1))
    out["xsf_roks_mc_ev"] = _floats(mc[mc.index("]", mc.index("Converged")) + 1:].split("]")[0])
    log5 = "\n".join(_outputs(cells[5]))
    out["uks_bhandhlyp_e_tot"] = float(_floats(_outputs(cells[5])[-1])[0])
    s2 = re.findall(r"multiplicity <S\^2> = ([\d.]+)", log5)
    out["uks_bhandhlyp_s2_last_printed"] = float(s2[-1])
    usf = "\n".join(_outputs(cells[6]))
    out["usf_uks_alda0_ev"] = _floats(usf[usf.index("]", usf.index("Converged")) + 1:].split("]")[0])
    tail = _outputs(cells[6])[-1]
    out["usf_uks_alda0_delta_s2"] = _floats(tail[:tail.index("]")])
    umc = "\n".join(_outputs(cells[7]))
    out["usf_uks_mc_ev"] = _floats(umc[umc.index("]", umc.index("Converged")) + 1:].split("]")[0])
    tail = _outputs(cells[7])[-1]
    out["usf_uks_mc_delta_s2"] = _floats(tail[:tail.index("]")])

    nb2 = json.load(open(os.path.join(REF, "spin up.ipynb")))
    up = "\n".join(_outputs(nb2["cells"][1]))
    out["roks_aufbau_hf_e_tot"] = float(re.search(r"converged SCF energy = ([-\d.]+)", up).group(1))

    nb3 = json.load(open(os.path.join(REF, "TDA.ipynb")))
    for cell, tag, head in ((2, "n2_rks_b3lyp", "TDA result is"),
                            (4, "ch2o_uks_b3lyp", "UTDA result is"),
                            (6, "ch2o_roks_b3lyp", "my XTDA result is")):
        log = "\n".join(_outputs(nb3["cells"][cell]))
        out[f"{tag}_counts"] = [int(re.search(rf"{k} = (\d+)", log).group(1))
                                for k in ("number of shells", "number of NR pGTOs",
                                          "number of NR cGTOs")]
        out[f"{tag}_nuclear_repulsion"] = float(re.search(r"nuclear repulsion = ([-\d.]+)", log).group(1))
        out[f"{tag}_tot_grids"] = int(re.search(r"tot grids = (\d+)", log).group(1))
        out[f"{tag}_e_tot"] = float(re.search(r"converged SCF energy = ([-\d.]+)", log).group(1))
        rows = []
        for line in log[log.index(head):].splitlines()[2:]:
            f = line.split()
            if len(f) < 5 or not f[0].isdigit():
                break
            rows.append([float(x) for x in f[1:]])
        rows = np.array(rows)
        out[f"{tag}_td_ev"] = rows[:, 0].tolist()
        if cell == 2:   # TDA.analyze prints every root again with 5 decimals (TDA.py:283)
            out[f"{tag}_td_ev5"] = [float(x) for x in re.findall(r"Excited state\s+\d+\s+([-\d.]+) eV", log)]
            assert len(out[f"{tag}_td_ev5"]) == 12
        out[f"{tag}_td_osc"] = rows[:, 2].tolist()
        if rows.shape[1] > 4:
            out[f"{tag}_td_delta_s2"] = rows[:, 4].tolist()
        if cell == 6:   # xtda.analyze(): the spin-tensor (so2st) CI coefficients above 0.1
            states = []
            for line in log[log.index("D1 "):].splitlines():
                f = line.split()
                if f and re.fullmatch(r"D\d+", f[0]):
                    states.append([])
                elif len(f) >= 6 and f[0] in ("CV(0)", "OV(0)", "CO(0)", "CV(1)") and f[2] == "->":
                    states[-1].append([f[0], int(f[1]), int(f[3]), float(f[5])])
            out[f"{tag}_analyze"] = states
    assert len(out["ch2o_roks_b3lyp_td_ev"]) == 12 and len(out["ch2o_uks_b3lyp_td_ev"]) == 12
    assert len(out["ch2o_roks_b3lyp_analyze"]) == 12

    assert len(out["xsf_roks_alda0_ev"]) == 10 and len(out["usf_uks_alda0_ev"]) == 10
    assert len(out["xsf_roks_mc_ev"]) == 10 and len(out["usf_uks_mc_ev"]) == 10
    assert len(out["usf_uks_mc_delta_s2"]) == 10
    assert len(out["hf_631g_grid_ang_F"]) == 75 and len(out["hf_631g_grid_ang_H"]) == 50
    json.dump(out, open(OUT, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    np.set_printoptions(precision=12)
    main()
