"""GPU: parity at the BASELINE configurations' FULL sizes against the oracle on the
same data.

The synthetic mean field of a bench configuration is generated in HBM (block-seeded,
``make_device_mf``), the device operator is built from it exactly as ``bench.py``
builds the timed one, and ONE trial vector's sigma is compared with the oracle's
AO-route vind (XTDA.py:615-690, SF_TDA.py:224-243, XSF_TDA.py:1131-1276) evaluated on
the same data regenerated bit-identically and streamed from HBM block by block
(``bench.oracle_meanfield``).  These are the code paths only full sizes reach: the
multi-chunk XC grid loop, the stored-exchange K-split chosen for fill, the ragged
edge tiles of V, the real O.  Tolerance: 1e-12 relative max-norm.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config", ["C2", "C3", "C4", "C4d", "C5", "C3mc", "H"])
def test_full_size_sigma_matches_oracle_on_same_data(hiplib, config):
    """Every BASELINE configuration and the headline (H: ~1 min of oracle on 16 CPUs)."""
    import torch
    import bench
    from threadpoolctl import threadpool_limits
    args = bench.parse(["--config", config])
    w = bench.device_workload(args, 0, 1, 0)
    g = torch.Generator(device=w.device)
    g.manual_seed(20261016)
    z = torch.randn((1, w.op.dim), dtype=torch.float64, device=w.device, generator=g)
    z /= z.norm(dim=1, keepdim=True)
    s_dev = w.op.apply(z).cpu().numpy()
    with threadpool_limits(limits=bench.cpu_share()):
        mfo, _ = bench.oracle_meanfield(args, w)
        vind, _ = bench._oracle_vind(args, mfo)
        s_or = vind(z.cpu().numpy())
    err = np.abs(s_dev - s_or).max() / np.abs(s_or).max()
    assert err < 1e-12, err
