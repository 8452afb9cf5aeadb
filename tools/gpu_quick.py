import numpy as np, sys, time
sys.path.insert(0, '/root/repo')
from xtddft_amd import build; build.build()
from xtddft_amd.synthetic import make_mf, make_trial_vectors
from xtddft_amd.operator import DeviceOperator
from oracle import xtda, sf_tda, xsf_tda
def rel(a, b): return np.abs(a-b).max() / max(1e-300, np.abs(b).max())
for kind, xct, om in [('RO','GGA',0.0),('RO','LDA',0.0),('RO','HF',0.0),('RO','GGA',0.33),('U','GGA',0.0),('U','LDA',0.33)]:
    mf = make_mf(nao=26, nc=5, no=2, xctype=xct, kind=kind, omega=om, alpha=0.65 if om else 0.0, hyb=0.19 if om else 0.2)
    vind, hdiag = xtda.gen_tda_operation(mf)
    z = make_trial_vectors(7, hdiag.size)
    op = DeviceOperator(mf, 'XTDA' if kind=='RO' else 'UTDA')
    s = op.apply(z); r = vind(z)
    print('XTDA' if kind=='RO' else 'UTDA', kind, xct, om, 'rel err', rel(s, r), flush=True)
for kind in ['RO','U']:
  for xct in ['GGA','HF']:
    mf = make_mf(nao=26, nc=5, no=2, xctype=xct, kind=kind, hyb=0.5)
    for isf, name in [(-1,'SF_DOWN'),(1,'SF_UP')]:
        vind, hdiag = sf_tda.gen_tda_operation_sf(mf, isf)
        z = make_trial_vectors(5, hdiag.size)
        op = DeviceOperator(mf, name)
        print(name, kind, xct, 'rel err', rel(op.apply(z), vind(z)), flush=True)
for SA in [0,1,2,3]:
  for no in [2,3]:
    mf = make_mf(nao=26, nc=5, no=no, xctype='GGA', hyb=0.5)
    o = xsf_tda.XSFOracle(mf, SA=SA)
    fg = xsf_tda.default_fglobal(mf)
    vind, hdiag = o.gen_tda_operation_sf(fglobal=fg)
    z = make_trial_vectors(4, hdiag.size)
    op = DeviceOperator(mf, 'XSF', sa=SA, fglobal=fg, foo=1.0, remove=o.re)
    if o.re: op.set_oo_basis(o.vects)
    print('XSF SA', SA, 'no', no, 'rel err', rel(op.apply(z), vind(z)), flush=True)
