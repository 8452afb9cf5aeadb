"""Basis-set data (PySCF internal format: ``[[l, [exp, c], [exp, c], ...], ...]``).

Only data that the reference itself records is embedded: the 6-31G shells of
F and H exactly as PySCF 2.12.1 printed them in the reference's example run
(``example/XSF_TDA.ipynb``, cell 1 output, "[INPUT] ---- BASIS SET ----").
Any other basis is passed to ``Mole`` as a dict in the same format, or as
NWChem-format text through ``parse_nwchem`` (PySCF ``gto.basis.parse``).
"""
from __future__ import annotations

_631G = {
    "F": [
        [0, [7001.71309, 0.0018196169], [1051.36609, 0.0139160796], [239.28569, 0.0684053245],
         [67.3974453, 0.23318576], [21.5199573, 0.471267439], [7.4031013, 0.356618546]],
        [0, [20.8479528, -0.108506975], [4.80830834, -0.146451658], [1.34406986, 1.12868858]],
        [0, [0.358151393, 1.0]],
        [1, [20.8479528, 0.0716287243], [4.80830834, 0.345912103], [1.34406986, 0.722469957]],
        [1, [0.358151393, 1.0]],
    ],
    "H": [
        [0, [18.731137, 0.0334946], [2.8253937, 0.23472695], [0.6401217, 0.81375733]],
        [0, [0.1612778, 1.0]],
    ],
}

# 6-31G carbon (Hehre, Ditchfield, Pople, J. Chem. Phys. 56, 2257 (1972); the EMSL / NWChem
# values PySCF ships) -- not printed by any reference run: BASELINE config C1 (CH2 3B1 /
# 6-31G) is checked device against oracle (tools/molecule_run.py), not against the reference.
_631G["C"] = [
    [0, [3047.5249, 0.0018347], [457.36951, 0.0140373], [103.94869, 0.0688426],
     [29.210155, 0.2321844], [9.286663, 0.4679413], [3.163927, 0.3623120]],
    [0, [7.8682724, -0.1193324], [1.8812885, -0.1608542], [0.5442493, 1.1434564]],
    [0, [0.1687144, 1.0]],
    [1, [7.8682724, 0.0689991], [1.8812885, 0.3164240], [0.5442493, 0.7443083]],
    [1, [0.1687144, 1.0]],
]

# STO-3G hydrogen (zeta = 1.24), the Szabo-Ostlund textbook H2 basis used by the
# integral unit tests.
_STO3G = {
    "H": [[0, [3.42525091, 0.15432897], [0.62391373, 0.53532814], [0.16885540, 0.44463454]]],
}

# cc-pVDZ of H, C, N, O: Dunning, J. Chem. Phys. 90, 1007 (1989), in the segmented
# layout of the EMSL / NWChem library file that PySCF ships (the most diffuse s and p
# primitives appear only as their own uncontracted shells, which spans the same space
# as the original general contraction).  The layout is fixed by the shell / primitive
# counts the reference printed ("number of shells = 16", "number of NR pGTOs = 66",
# "number of NR cGTOs = 38" for CH2O+, 10 / 52 / 28 for N2; example/TDA.ipynb cells
# 2, 4, 6), and the numbers by the reference's printed SCF energies, which the front
# end reproduces to 1e-9 Ha (tests/test_qc.py::test_cc_pvdz_scf_energies).
_CCPVDZ = {
    "H": [
        [0, [13.01, 0.019685], [1.962, 0.137977], [0.4446, 0.478148]],
        [0, [0.122, 1.0]],
        [1, [0.727, 1.0]],
    ],
    "C": [
        [0, [6665.0, 0.000692, -0.000146], [1000.0, 0.005329, -0.001154],
         [228.0, 0.027077, -0.005725], [64.71, 0.101718, -0.023312],
         [21.06, 0.27474, -0.063955], [7.495, 0.448564, -0.149981],
         [2.797, 0.285074, -0.127262], [0.5215, 0.015204, 0.544529]],
        [0, [0.1596, 1.0]],
        [1, [9.439, 0.038109], [2.002, 0.20948], [0.5456, 0.508557]],
        [1, [0.1517, 1.0]],
        [2, [0.55, 1.0]],
    ],
    "N": [
        [0, [9046.0, 0.0007, -0.000153], [1357.0, 0.005389, -0.001208],
         [309.3, 0.027406, -0.005992], [87.73, 0.103207, -0.024544],
         [28.56, 0.278723, -0.067459], [10.21, 0.44854, -0.158078],
         [3.838, 0.278238, -0.121831], [0.7466, 0.01544, 0.549003]],
        [0, [0.2248, 1.0]],
        [1, [13.55, 0.039919], [2.917, 0.217169], [0.7973, 0.510319]],
        [1, [0.2185, 1.0]],
        [2, [0.817, 1.0]],
    ],
    "O": [
        [0, [11720.0, 0.00071, -0.00016], [1759.0, 0.00547, -0.001263],
         [400.8, 0.027837, -0.006267], [113.7, 0.1048, -0.025716],
         [37.03, 0.283062, -0.070924], [13.27, 0.448719, -0.165411],
         [5.025, 0.270952, -0.116955], [1.013, 0.015458, 0.557368]],
        [0, [0.3023, 1.0]],
        [1, [17.7, 0.043018], [3.854, 0.228913], [1.046, 0.508728]],
        [1, [0.2753, 1.0]],
        [2, [1.185, 1.0]],
    ],
}

BASIS = {"6-31g": _631G, "sto-3g": _STO3G, "sto3g": _STO3G, "cc-pvdz": _CCPVDZ}


def load(name_or_dict, symbol: str):
    """Shells of element ``symbol`` for a basis name or a {symbol: shells} dict."""
    if isinstance(name_or_dict, dict):
        if symbol in name_or_dict:
            shells = name_or_dict[symbol]
        else:
            raise KeyError(f"basis dict has no entry for {symbol}")
        if isinstance(shells, str):
            return load(shells, symbol)
        return shells
    key = str(name_or_dict).lower().replace("_", "-")
    if key not in BASIS:
        raise KeyError(f"basis {name_or_dict!r} is not embedded; pass the shells as a dict "
                       f"(embedded: {sorted(BASIS)})")
    table = BASIS[key]
    if symbol not in table:
        raise KeyError(f"basis {name_or_dict!r} has no data for {symbol} here")
    return table[symbol]


_L = {"S": 0, "P": 1, "D": 2, "F": 3, "G": 4, "H": 5}


def parse_nwchem(text: str, symbol: str | None = None):
    """NWChem-format basis text -> {element: shells} (PySCF ``gto.basis.parse``).

    Each block starts with ``<Element> <L>`` (L in S P D F G H, or ``SP`` for a
    shared-exponent s+p pair) followed by rows ``exponent c1 [c2 ...]``; lines
    starting with ``#`` and ``BASIS`` / ``END`` markers are ignored.  With
    ``symbol`` the shells of that element are returned directly."""
    out: dict = {}
    cur = None
    for raw in text.splitlines():
        line = raw.split("#")[0].strip()
        if not line or line.upper().startswith(("BASIS", "END")):
            continue
        f = line.split()
        if f[0][0].isalpha():
            el = f[0].capitalize()
            lab = f[1].upper()
            if lab == "SP":
                cur = (el, "SP", [[0], [1]])
                out.setdefault(el, []).extend(cur[2])
            else:
                shell = [_L[lab]]
                cur = (el, lab, [shell])
                out.setdefault(el, []).append(shell)
            continue
        if cur is None:
            raise ValueError(f"basis data before a shell header: {raw!r}")
        vals = [float(x.replace("D", "E").replace("d", "e")) for x in f]
        if cur[1] == "SP":
            cur[2][0].append([vals[0], vals[1]])
            cur[2][1].append([vals[0], vals[2]])
        else:
            cur[2][0].append(vals)
    if symbol is not None:
        return out[symbol.capitalize()]
    return out
