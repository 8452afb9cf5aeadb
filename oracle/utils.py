"""Index utilities, literal restatement.  TEST INFRASTRUCTURE ONLY.

``order_pyscf2my`` follows utils.py:44-64 step by step (insert/delete loop)
so tests can check the product's closed-form permutation against it.
"""
import numpy as np


def order_pyscf2my(nc, no, nv):
    order = np.indices(((nc + no) * nv + nc * (no + nv),)).squeeze(axis=0)
    for oi in range(nc):
        for noi in range(no):
            order = np.insert(order, (nc + no) * nv + no * oi + noi,
                              (nc + no) * nv + oi * nv + no * oi + noi)
            order = np.delete(order, (nc + no) * nv + oi * nv + no * oi + noi + 1)
    return order
