"""Quick end-to-end check of the reference-style API on the GPU vs the oracle."""
import sys, time
import numpy as np
sys.path.insert(0, '/root/repo')
from xtddft_amd import build; build.build()
from xtddft_amd.synthetic import make_mf
from xtddft_amd import XTDA, SF_TDA, XSF_TDA
from oracle import xtda as oxtda, davidson as odav, xsf_tda as oxsf, sf_tda as osf

mf = make_mf(nao=40, nc=8, no=2, xctype='GGA', hyb=0.2)
t = time.time(); x = XTDA(mf.mol, mf, nstates=8); e = x.kernel(); t1 = time.time() - t
vind, hdiag = oxtda.gen_tda_operation(mf)
w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
print('XTDA davidson', x.converged.all(), x.icyc, 'max|e-eigh|', np.abs(e - w[:8]).max(), f'{t1:.2f}s', flush=True)
x2 = XTDA(mf.mol, mf, nstates=8, use_Davidson=False); e2 = x2.kernel()
print('XTDA full_diag max|e-eigh|', np.abs(e2 - w[:8]).max(), 'dS2', x2.dS2[:3], flush=True)

mfu = make_mf(nao=40, nc=8, no=2, xctype='LDA', hyb=0.2, kind='U')
xu = XTDA(mfu.mol, mfu, nstates=6); eu = xu.kernel()
vind, hdiag = oxtda.gen_tda_operation(mfu)
w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
print('UTDA davidson', xu.converged.all(), 'max|e-eigh|', np.abs(eu - w[:6]).max(), flush=True)

for isf in (-1, 1):
    s = SF_TDA(mf, isf=isf); es, vs = s.kernel(nstates=5)
    vind, hdiag = osf.gen_tda_operation_sf(mf, isf)
    w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
    print('SF', isf, s.converged.all(), 'max|e-eigh| (eV)', np.abs(es - w[:5] * 27.2113834).max(), flush=True)

mf3 = make_mf(nao=40, nc=8, no=3, xctype='GGA', hyb=0.5)
xs = XSF_TDA(mf3); ex, vx = xs.kernel(nstates=6)
o = oxsf.XSFOracle(mf3); vind, hdiag = o.gen_tda_operation_sf()
w = np.linalg.eigvalsh(vind(np.eye(hdiag.size)).T)
print('XSF', xs.converged.all(), 'max|e-eigh| (eV)', np.abs(ex - w[:6] * 27.21138505).max(), flush=True)
hd_o = hdiag
print('XSF hdiag parity', np.abs(xs.gen_tda_operation_sf(fglobal=xs.fglobal)[1] - hd_o).max(), flush=True)
