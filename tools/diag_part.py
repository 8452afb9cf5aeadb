import sys, numpy as np
sys.path.insert(0, '.')
from xtddft_amd.synthetic import make_mf, make_trial_vectors
from xtddft_amd.operator import DeviceOperator
from oracle import xtda as oxtda
def rel(a, b): return np.abs(a - b).max() / np.abs(b).max()
for (nao, nc, no) in [(130, 99, 2), (80, 46, 2)]:
    mf = make_mf(nao=nao, nc=nc, no=no, xctype="GGA", hyb=0.25, ngrid=3000)
    vind, hdiag = oxtda.gen_tda_operation(mf)
    z = make_trial_vectors(4, hdiag.size)
    ref = vind(z)
    full = DeviceOperator(mf, "XTDA", k_mode="stored")
    print(nao, nc, no, 'full', rel(full.apply(z), ref), flush=True)
    for n in (2, 3, 4, 5, 8):
        for rep in (True, False):
            parts = [DeviceOperator(mf, "XTDA", k_mode="stored", shard=(r, n), replicate_df=rep) for r in range(n)]
            s = sum(p.apply(z) for p in parts)
            print(nao, 'n', n, 'replicate_df', rep, 'rows', [getattr(p, "partition", {}).get("exchange_rows") for p in parts], 'aux', [getattr(p, "partition", {}).get("aux") for p in parts], 'naux', [p.naux()[0] for p in parts], 'rel', rel(s, ref), flush=True)
            del parts
