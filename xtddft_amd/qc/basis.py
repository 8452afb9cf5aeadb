"""Basis-set data (PySCF internal format: ``[[l, [exp, c], [exp, c], ...], ...]``).

Only data that the reference itself records is embedded: the 6-31G shells of
F and H exactly as PySCF 2.12.1 printed them in the reference's example run
(``example/XSF_TDA.ipynb``, cell 1 output, "[INPUT] ---- BASIS SET ----").
Any other basis is passed to ``Mole`` as a dict in the same format.
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
