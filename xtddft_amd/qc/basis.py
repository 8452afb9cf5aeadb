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

# STO-3G hydrogen (zeta = 1.24), the Szabo-Ostlund textbook H2 basis used by the
# integral unit tests.
_STO3G = {
    "H": [[0, [3.42525091, 0.15432897], [0.62391373, 0.53532814], [0.16885540, 0.44463454]]],
}

BASIS = {"6-31g": _631G, "sto-3g": _STO3G, "sto3g": _STO3G}


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
