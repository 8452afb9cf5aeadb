"""Device TDA operator: owns one ``xt_ctx`` and evaluates sigma = A z on the GPU.

This is the object behind every ``vind`` the reference API hands out
(``XTDA.gen_vind``, ``SF_TDA.gen_tda_operation_sf``,
``XSF_TDA.gen_tda_operation_sf``).  Inputs may be NumPy arrays (host) or
``torch`` CUDA tensors (device); trial vectors keep their kind on return.

Sharding (multi-GPU, one process per GPU): ``shard=(rank, nranks)`` keeps
1/nranks of the grid points on this rank and adds the one-electron terms on
rank 0 only, so the per-rank sigma are partial sums that
``xtddft_amd.parallel.allreduce_sigma`` combines.  The DF
factor is either sliced by aux index (``replicate_df=False``: each rank holds
1/nranks of P) or replicated with an aux *window* plus a row block of the
stored exchange matrix (``xt_set_partition``; the default unless the exchange
is forced direct), so the stored exchange is split over the ranks too.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi
from .meanfield import MeanField


def _torch():
    try:
        import torch
        return torch
    except Exception:   # pragma: no cover
        return None


def _is_device(x) -> bool:
    t = _torch()
    return t is not None and isinstance(x, t.Tensor) and x.is_cuda


def _ptr(x):
    """(address, ptr_kind, keepalive) for a numpy array or CUDA tensor."""
    if x is None:
        return None, _capi.XT_PTR_HOST, None
    if _is_device(x):
        x = x.contiguous()
        if x.dtype != _torch().float64:
            raise TypeError("device arrays must be float64")
        return x.data_ptr(), _capi.XT_PTR_DEVICE, x
    a = np.ascontiguousarray(x, dtype=np.float64)
    return a.ctypes.data, _capi.XT_PTR_HOST, a


def _split(n, rank, nranks):
    base, rem = divmod(n, nranks)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shape_info(mf: MeanField, kind: str):
    info = mf.shape_info()
    nc, no, nv = info["nc"], info["no"], info["nv"]
    if kind in ("XTDA", "UTDA"):
        dim = (nc + no) * nv + nc * (no + nv)
    elif kind == "SF_DOWN":
        dim = (nc + no) * (no + nv)
    elif kind == "SF_UP":
        dim = nc * nv
    else:
        dim = None
    return nc, no, nv, dim


class DeviceOperator:
    def __init__(self, mf: MeanField, kind: str, *, sa: int = 0, foo: float = 1.0,
                 fglobal: float = 0.0, remove: bool = False, shard=(0, 1), device: int = 0,
                 stream=None, presharded=False, k_mode: str = "auto",
                 k_max_gib: float = 0.0, replicate_df=None, sf_kernel: str = "alda0", mc_kernel=None,
                 group=None):
        """sf_kernel: spin-flip XC kernel of the SF / XSF kinds -- 'alda0' (method 0,
        mf.fxc_sf) or 'mc' (method 1: the multicollinear kernel ``mc_kernel`` (nk, nk, ngrid),
        ``xtddft_amd.mcol.sf_mc_kernel``).
        presharded: True -- mf.cderi / mf.grids hold only this rank's slices;
        "grid" -- only mf.grids is this rank's slice (mf.cderi is whole).
        k_mode: exchange evaluation ('auto' | 'direct' | 'stored', see
        xt_set_exchange_mode); k_max_gib caps the stored matrix in auto mode.
        replicate_df: keep the whole factor on every rank and partition by aux
        window + exchange rows (default: k_mode != 'direct').  With replicate_df, k_mode
        'auto' and an initialised process group, construction is a collective: the ranks
        agree on stored vs direct exchange (the minimum of their fits over ``group``, default
        the WORLD group), so every rank of that group must construct its operator; an
        operator without an exchange matrix to store skips the agreement."""
        L = _capi.lib()
        self.mf, self.kind = mf, kind
        if sf_kernel not in _capi.SF_KERNEL:
            raise ValueError(f"sf_kernel must be one of {sorted(_capi.SF_KERNEL)}")
        self.sf_kernel = sf_kernel if kind in ("SF_DOWN", "SF_UP", "XSF") else "alda0"
        self.mc_kernel = mc_kernel
        if self.sf_kernel == "mc" and mf.xctype != "HF" and mc_kernel is None:
            raise ValueError("sf_kernel='mc' needs the multicollinear kernel (mc_kernel)")
        rank, nranks = shard
        nc, no, nv, _ = shape_info(mf, kind)
        nmo = nc + no + nv
        self.nc, self.no, self.nv = nc, no, nv
        naux = mf.naux
        ngrid = mf.grids.ngrid if (mf.grids is not None and mf.xctype != "HF") else 0
        self.shard = (rank, nranks)
        self.device = int(device)
        if replicate_df is None:
            replicate_df = k_mode != "direct" and presharded is not True
        self.replicate_df = bool(replicate_df) and nranks > 1
        if presharded is True:
            self.aux_range, self.grid_range = (0, naux), (0, ngrid)
        else:
            self.aux_range = (0, naux) if (self.replicate_df or presharded == "grid") \
                else _split(naux, rank, nranks)
            self.grid_range = (0, ngrid) if presharded == "grid" else _split(ngrid, rank, nranks)
        d = _capi.XtDesc()
        d.kind = _capi.KIND[kind]
        d.restricted = 1 if mf.is_rohf else 0
        d.nao, d.nmo = mf.nao, nmo
        d.nc, d.no, d.nv = nc, no, nv
        d.naux = self.aux_range[1] - self.aux_range[0]
        d.ngrid = self.grid_range[1] - self.grid_range[0]
        d.xctype = _capi.XC[mf.xctype]
        d.hyb, d.alpha, d.omega = mf.hyb, mf.alpha, mf.omega
        d.si = 0.5 * mf.mol.spin if kind != "XSF" else no / 2.0
        d.sa, d.foo, d.fglobal = sa, foo, fglobal
        d.remove = 1 if remove else 0
        d.add_local = 1 if rank == 0 else 0
        d.device = device
        d.sf_kernel = _capi.SF_KERNEL[self.sf_kernel]
        self.desc = d
        h = ctypes.c_void_p()
        _capi.check(L.xt_create(ctypes.byref(d), ctypes.byref(h)), "xt_create")
        self._h = h
        self._L = L
        if stream is None and _torch() is not None and _torch().cuda.is_available():
            stream = _torch().cuda.current_stream(device).cuda_stream
        self.stream = stream
        _capi.check(L.xt_set_stream(h, ctypes.c_void_p(stream or 0)), "xt_set_stream")
        self.dim = L.xt_dim(h)
        self.setup_s = {}
        self._setup()
        if self.replicate_df:
            self._set_partition(kind, nc, no)
        _capi.check(L.xt_set_exchange_mode(h, _capi.K_MODE[k_mode], float(k_max_gib)),
                    "xt_set_exchange_mode")
        if self.replicate_df and k_mode == "auto":
            # the auto rule reads this GPU's free HBM: the ranks agree (store only if every
            # rank's rows fit) before anything is built -- stored rows on one rank and a
            # direct aux window on another do not sum to the operator
            fits, gib = ctypes.c_int(), ctypes.c_double()
            _capi.check(L.xt_exchange_plan(h, ctypes.byref(fits), ctypes.byref(gib)), "xt_exchange_plan")
            if gib.value > 0:    # same descriptors on every rank: all skip or none does
                from .parallel import agree_min
                k_mode = "stored" if agree_min(fits.value, group, device=self.device) else "direct"
                _capi.check(L.xt_set_exchange_mode(h, _capi.K_MODE[k_mode], float(k_max_gib)),
                            "xt_set_exchange_mode")
        self.prepare()
        self.setup_s["prepare"] = self.prepare_s

    def _set_partition(self, kind, nc, no):
        """Aux window and exchange row block of this rank (xt_set_partition)."""
        rank, nranks = self.shard
        naux_local, _ = self.naux()
        p0, p1 = _split(naux_local, rank, nranks)
        occ = nc if kind == "SF_UP" else nc + no
        i0, i1 = _split(occ, rank, nranks)
        _capi.check(self._L.xt_set_partition(self._h, p0, p1, i0, i1), "xt_set_partition")
        self.partition = dict(aux=(p0, p1), exchange_rows=(i0, i1))

    def prepare(self):
        """Build the once-per-solve device data (stored exchange matrix when chosen)."""
        import time
        m, g = ctypes.c_int(), ctypes.c_double()
        t0 = time.perf_counter()
        _capi.check(self._L.xt_prepare(self._h, ctypes.byref(m), ctypes.byref(g)), "xt_prepare")
        self.prepare_s = time.perf_counter() - t0     # xt_prepare synchronises the stream
        self.k_mode = _capi.K_MODE_NAME[m.value]
        self.k_gib = g.value
        return self.k_mode

    # -------------------------------------------------------------- setup
    def _sync(self):
        t = _torch()
        if t is not None and t.cuda.is_available():
            t.cuda.synchronize(self.desc.device)

    def _lap(self, name, t0):
        """Setup phase timer (the phases enqueue device work: synchronised at each lap)."""
        import time
        self._sync()
        t1 = time.perf_counter()
        self.setup_s[name] = self.setup_s.get(name, 0.0) + (t1 - t0)
        return t1

    def _setup(self):
        import time
        L, h, mf = self._L, self._h, self.mf
        t = time.perf_counter()
        if mf.is_rohf:
            ca = mf.mo_coeff; cb = None
        else:
            ca, cb = mf.mo_coeff[0], mf.mo_coeff[1]
        pa, ka, ra = _ptr(ca)
        pb, _, rb = _ptr(cb)
        _capi.check(L.xt_set_orbitals(h, pa, pb, ka), "xt_set_orbitals")
        t = self._lap("orbitals", t)
        fa, fb = mf.fock_mo()
        fah, fbh = mf.fock_mo_hf()
        ptrs = [_ptr(x) for x in (fa, fb, fah, fbh)]
        _capi.check(L.xt_set_fock_mo(h, *[p[0] for p in ptrs], _capi.XT_PTR_HOST), "xt_set_fock_mo")
        if not mf.is_rohf:
            e = [_ptr(mf.mo_energy[0]), _ptr(mf.mo_energy[1])]
            _capi.check(L.xt_set_orbital_energies(h, e[0][0], e[1][0], _capi.XT_PTR_HOST),
                        "xt_set_orbital_energies")
        t = self._lap("fock_mo", t)
        p0, p1 = self.aux_range
        if mf.jk_mode == "ERI8":
            # stored ERIs: factorised on the device; this rank keeps its block
            # of Cholesky vectors (aux sharding) or all of them
            # (replicated factor, partitioned by window)
            rank, nranks = self.shard if not self.replicate_df else (0, 1)
            for which, eri in ((0, mf.eri), (1, mf.eri_lr if mf.omega != 0 else None)):
                if eri is None:
                    continue
                pe, ke, re_ = _ptr(eri)
                _capi.check(L.xt_set_jk_eri8(h, pe, which, float(mf.chol_tol), rank, nranks, ke),
                            "xt_set_jk_eri8")
        elif p1 > p0:
            pc, kc, rc = _ptr(mf.cderi[p0:p1])
            _capi.check(L.xt_set_jk_df(h, pc, 0, kc), "xt_set_jk_df")
            if mf.cderi_lr is not None and mf.omega != 0:
                pl, kl, rl = _ptr(mf.cderi_lr[p0:p1])
                _capi.check(L.xt_set_jk_df(h, pl, 1, kl), "xt_set_jk_df(lr)")
        t = self._lap("jk_factor", t)
        g0, g1 = self.grid_range
        if g1 > g0:
            grids = mf.grids
            sf = self.kind in ("SF_DOWN", "SF_UP", "XSF")
            w = grids.weights[g0:g1]
            if sf and self.sf_kernel == "mc":       # multicollinear: GGA-shaped one-channel kernel
                ao = grids.ao[:(1 if mf.xctype == "LDA" else 4), g0:g1]
                kern = self.mc_kernel[..., g0:g1]
            elif sf:                                # ALDA0: density only
                ao = grids.ao[:1, g0:g1]
                kern = mf.fxc_sf[g0:g1]
            else:
                ao = grids.ao[:, g0:g1]
                kern = mf.fxc[..., g0:g1]
            if _is_device(ao):       # AO values resident in HBM (device eval_ao): kernel data follows
                torch = _torch()
                w, kern = (x if _is_device(x) else torch.as_tensor(np.ascontiguousarray(x), device=ao.device)
                           for x in (w, kern))
            pao, kao, rao = _ptr(ao)
            pw, kw, rw = _ptr(w)
            pk, kk, rk = _ptr(kern)
            if not (kao == kw == kk):
                raise TypeError("grid arrays must all be host or all device")
            _capi.check(L.xt_set_grid(h, pao, pw, pk, kao), "xt_set_grid")
        self._lap("grid", t)

    def naux(self):
        """(DF / Cholesky functions on this rank, full Cholesky rank of an ERI8 factorisation)."""
        a, r = ctypes.c_int(), ctypes.c_int()
        _capi.check(self._L.xt_naux(self._h, ctypes.byref(a), ctypes.byref(r)), "xt_naux")
        return a.value, r.value

    def set_oo_basis(self, vects):
        p, k, r = _ptr(vects)
        _capi.check(self._L.xt_set_oo_basis(self._h, p, k), "xt_set_oo_basis")

    # -------------------------------------------------------------- hot path
    def apply(self, zs, out=None):
        """sigma = A z for zs of shape (nz, dim) (NumPy or CUDA tensor)."""
        if _is_device(zs):
            torch = _torch()
            # the C ABI takes raw FP64 pointers on this context's device: refuse anything
            # else here rather than let the kernels read or write past a buffer
            if zs.dtype != torch.float64:
                raise TypeError(f"trial vectors must be float64, got {zs.dtype}")
            if zs.device.index != self.device:
                raise ValueError(f"trial vectors on cuda:{zs.device.index}, operator on cuda:{self.device}")
            z = zs.contiguous()
            if z.dim() == 1:
                z = z[None]
            if z.dim() != 2 or z.shape[1] != self.dim:
                raise ValueError(f"trial vectors have shape {tuple(z.shape)}, expected (nz, {self.dim})")
            nz = z.shape[0]
            if out is None:
                out = torch.empty_like(z)
            elif (out.dtype != torch.float64 or not out.is_cuda or out.device.index != self.device
                  or tuple(out.shape) != tuple(z.shape) or not out.is_contiguous()):
                raise ValueError(f"out must be a contiguous float64 tensor of shape {tuple(z.shape)} "
                                 f"on cuda:{self.device}")
            if nz == 0:
                return out
            _capi.check(self._L.xt_apply(self._h, nz, z.data_ptr(), out.data_ptr(),
                                         _capi.XT_PTR_DEVICE), "xt_apply")
            return out
        if out is not None:
            raise ValueError("out is for device tensors; host arrays return a new array")
        z = np.ascontiguousarray(np.asarray(zs, dtype=np.float64))
        if z.ndim == 1:
            z = z[None]
        if z.ndim != 2 or z.shape[1] != self.dim:
            raise ValueError(f"trial vectors have shape {z.shape}, expected (nz, {self.dim})")
        out = np.empty_like(z)
        if z.shape[0] == 0:
            return out
        _capi.check(self._L.xt_apply(self._h, z.shape[0], z.ctypes.data, out.ctypes.data,
                                     _capi.XT_PTR_HOST), "xt_apply")
        return out

    __call__ = apply

    def apply_full(self, zs):
        """The whole operator: this rank's partial sigma all-reduced over the
        process group when the operator is sharded (what the drivers' vind
        returns; ``apply`` is the rank-partial sum)."""
        out = self.apply(zs)
        if self.shard[1] > 1:
            from .parallel import allreduce_sigma, require_group
            require_group(self.shard[1])
            out = allreduce_sigma(out)
        return out

    def last_timings(self):
        buf = (ctypes.c_double * 4)()
        _capi.check(self._L.xt_last_timings(self._h, ctypes.cast(buf, ctypes.c_void_p)), "timings")
        return dict(jk_ms=buf[0], xc_ms=buf[1], local_ms=buf[2], total_ms=buf[3])

    PROFILE_TAGS = {1: "df_exchange_contract", 2: "xc_forward_u", 3: "xc_back_l",
                    4: "xc_forward_w", 5: "xc_back_m"}

    def set_profile(self, mask: int = 0b111110):
        """Time GEMM classes live with HIP events (bit t = tag t, see PROFILE_TAGS)."""
        _capi.check(self._L.xt_set_profile(self._h, int(mask)), "xt_set_profile")

    def profile_stats(self):
        out = {}
        names = dict(self.PROFILE_TAGS)
        if getattr(self, "k_mode", "direct") == "stored":
            names[1] = "mo_exchange_stored"
        for tag, name in names.items():
            buf = (ctypes.c_double * 3)()
            _capi.check(self._L.xt_profile_stats(self._h, tag, ctypes.cast(buf, ctypes.c_void_p)), "stats")
            nbytes = ctypes.c_double(0.0)
            _capi.check(self._L.xt_profile_bytes(self._h, tag, ctypes.byref(nbytes)), "bytes")
            out[name] = dict(tag=tag, ms=buf[0], launches=int(buf[1]), flops=buf[2], bytes=nbytes.value)
        return out

    def xsf_j_diagonals(self):
        """XSF preconditioner J diagonals over this rank's aux rows, summed over
        the group when sharded."""
        co = np.empty((self.nc, self.no))
        ov = np.empty((self.no, self.nv))
        _capi.check(self._L.xt_xsf_j_diagonals(self._h, co.ctypes.data, ov.ctypes.data,
                                               _capi.XT_PTR_HOST), "xt_xsf_j_diagonals")
        if self.shard[1] > 1:
            from .parallel import allreduce_sigma, require_group
            require_group(self.shard[1])
            both = allreduce_sigma(np.concatenate([co.ravel(), ov.ravel()]))
            co, ov = both[:co.size].reshape(co.shape), both[co.size:].reshape(ov.shape)
        return co, ov

    def close(self):
        if getattr(self, "_h", None):
            self._L.xt_destroy(self._h)
            self._h = None

    def __del__(self):   # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
