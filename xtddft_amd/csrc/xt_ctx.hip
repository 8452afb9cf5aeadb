// xt_ctx: device-resident TDA operator and its C ABI (include/xtddft_amd.h).
//
// The reference forms AO transition densities, calls PySCF get_jk and
// nr_uks_fxc on them and projects back (XTDA.py:615-690).  Here the same
// operator is evaluated in the MO basis, with every tensor transformed once
// at setup and kept resident in HBM:
//
//   Bmo[P,p,q] = (C^T B_P C)_pq       DF factor in the MO basis
//   Phi[c,g,p] = (ao_c(g) C)_p        MO values / gradients on the grid
//
// and per xt_apply (nz trial vectors, one spin channel Ze = (nz, O, V)):
//   J   gamma[x,P] = sum_ch <Bmo[P,occ,vir], Ze_ch[x]>;  sigma += gamma . Bmo[:,occ,vir]
//   K   sigma[x] -= c_K sum_P Bmo[P,occ,occ] Ze[x] Bmo[P,vir,vir]          (sandwich)
//   XC  U_c = PhiV^c Ze^T ; rho1/wv/S on the grid (k_xc_*) ; sigma += S_c^T PhiV^c
//   1e  Fock (and Delta-A) MO products, or the orbital-energy diagonal (UTDA)
// all as strided FP64-MFMA GEMMs (xt_gemm.hip).  Algebraically identical to
// the reference's AO route (the projections are linear), different summation
// order: parity is to FP64 round-off, see tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>
#include <utility>
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../include/xtddft_amd.h"
#include "xt_internal.h"
#include "xt_kernels.h"

using namespace xt;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) { g_err = msg; return code; }
#define HIPCHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) \
    return fail(XT_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); } while (0)
#define RET(x) do { int _r = (x); if (_r) return _r; } while (0)

struct DevBuf {
  double* p = nullptr;
  size_t n = 0;   // doubles
  int ensure(size_t count) {
    if (count <= n) return 0;
    if (p) (void)hipFree(p);
    p = nullptr; n = 0;
    if (hipMalloc(&p, count * sizeof(double)) != hipSuccess) {
      p = nullptr;
      return fail(XT_ERR_OOM, "hipMalloc failed for " + std::to_string(count * 8) + " bytes");
    }
    n = count;
    return 0;
  }
  void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

// function-local scratch: freed on every return path
struct TmpBuf : DevBuf {
  ~TmpBuf() { release(); }
  void swap(DevBuf& o) { std::swap(p, o.p); std::swap(n, o.n); }
};

struct xt_ctx {
  xt_desc d;
  hipStream_t st = nullptr;
  int nbasis = 1;            // MO bases: 1 restricted, 2 unrestricted
  int ncomp = 1;                 // MO planes on the grid: value (+ 3 gradients for GGA / MGGA)
  int nkc = 1;                   // kernel components: 1 LDA, 4 GGA, 5 MGGA (+ tau)
  int nchan = 2;             // spin channels in the trial vector
  int O = 0, V = 0, v0 = 0;  // superset occupied / virtual dims, vir MO offset
  int occ_basis[2] = {0, 0}, vir_basis[2] = {0, 0};
  double ck = 0.0, ck_lr = 0.0;
  bool has_orb = false, has_df = false, has_lr = false, has_grid = false, has_fock = false, has_eps = false;
  bool has_vects = false;    // XSF OO basis set (empty for a doublet: no^2 - 1 = 0)
  DevBuf C, Bmo, Bmo_lr, Phi, kern, F, eps, vects;
  DevBuf ze, acc, kx, zr, tbuf, ubuf, gam, gam2, ws, stage, stage2, zin, sout, trace;
  DevBuf zp, accT, wbuf, taubuf;
  hipEvent_t ev[5];
  double timings[4] = {0, 0, 0, 0};
  // live per-kernel timing of tagged GEMM classes (bench roofline); mask bit t = tag t
  int prof_mask = 0;
  std::vector<hipEvent_t> pev;     // pairs
  std::vector<int> pev_tag;
  int pev_used = 0;
  double prof_flops[6] = {0, 0, 0, 0, 0, 0};
  double prof_bytes[6] = {0, 0, 0, 0, 0, 0};   // compulsory HBM bytes (operands once)
  double prof_ms[6] = {0, 0, 0, 0, 0, 0};
  int prof_launches[6] = {0, 0, 0, 0, 0, 0};
  int chol_rank = 0;         // full Cholesky rank of the last xt_set_jk_eri8
  // exchange evaluation (xt_set_exchange_mode): stored MO exchange matrix per channel group
  int kmode = XT_K_AUTO;
  double k_max_bytes = 0.0;  // auto-mode cap (0: free HBM minus a reserve)
  int k_resolved = -1;       // -1 undecided, 0 direct (DF sandwich), 1 stored
  bool kx_valid = false;
  DevBuf Kx;
  // rank partition (xt_set_partition): aux window for J / direct exchange / XSF
  // Delta-A over the resident factor, and the occupied rows of the stored exchange
  int win_p0 = 0, win_np = -1;   // -1: all aux rows
  bool m_kernel = true;          // XC M-backward through xt_xcm.hip (XT_M_KERNEL=0: the engine's mode 2)
  int w_kernel = 2;              // XC rho-forward: 1 xt_xcw.hip, 0 the engine's mode 1, 2 by size (XT_W_KERNEL)
  int kr0 = 0, kr1 = -1;         // -1: all O rows
  bool trimmed = false;          // the MO factor holds only this rank's aux window (xt_prepare)
  int naux_full = 0;             // desc naux before the trim
};

// a factor setter after a trim starts over with the full aux count (both factors must be set again)
static void untrim(xt_ctx* c) {
  if (!c->trimmed) return;
  c->d.naux = c->naux_full;
  c->Bmo.release(); c->Bmo_lr.release();
  c->has_df = c->has_lr = false;
  c->trimmed = false;
}

static int dim_of(const xt_desc& d) {
  const int nc = d.nc, no = d.no, nv = d.nv;
  switch (d.kind) {
    case XT_KIND_XTDA: case XT_KIND_UTDA: return (nc + no) * nv + nc * (no + nv);
    case XT_KIND_SF_DOWN: return (nc + no) * (no + nv);
    case XT_KIND_SF_UP: return nc * nv;
    case XT_KIND_XSF: return (nc + no) * (no + nv) - (d.remove ? 1 : 0);
  }
  return 0;
}

static int to_device(xt_ctx* c, DevBuf& dst, const double* src, size_t count, int ptr_kind) {
  RET(dst.ensure(count));
  HIPCHK(hipMemcpyAsync(dst.p, src, count * sizeof(double),
                        ptr_kind == XT_PTR_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice, c->st));
  return 0;
}

// live timing of a tagged launch class (xt_set_profile): an event pair around it
static int prof_begin(xt_ctx* c, int tag, double flops, double bytes, bool* on) {
  *on = tag > 0 && tag < 6 && ((c->prof_mask >> tag) & 1);
  if (!*on) return 0;
  if ((int)c->pev.size() < c->pev_used + 2) {
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b));
    c->pev.push_back(a); c->pev.push_back(b);
    c->pev_tag.push_back(0); c->pev_tag.push_back(0);
  }
  c->pev_tag[c->pev_used] = tag;
  HIPCHK(hipEventRecord(c->pev[c->pev_used], c->st));
  c->prof_flops[tag] += flops;
  c->prof_bytes[tag] += bytes;
  return 0;
}

static int prof_end(xt_ctx* c, int tag, bool on) {
  if (!on) return 0;
  HIPCHK(hipEventRecord(c->pev[c->pev_used + 1], c->st));
  c->pev_used += 2;
  c->prof_launches[tag] += 1;
  return 0;
}

static int gemm(xt_ctx* c, const GemmDesc& g) {
  bool prof = false;
  const double nr = g.R > 0 ? g.R : 1, nb = (double)(g.nb1 > 0 ? g.nb1 : 1) * (g.nb2 > 0 ? g.nb2 : 1);
  // compulsory bytes: A and B read once, C written once (read too when beta != 0)
  const double bytes = g.bytes > 0 ? g.bytes
                                   : 8.0 * nb * (nr * ((double)g.M * g.K + (double)g.K * g.N) +
                                                 (g.beta != 0.0 ? 2.0 : 1.0) * g.M * (double)g.N);
  RET(prof_begin(c, g.tag, g.flops > 0 ? g.flops : 2.0 * g.M * (double)g.N * g.K * nr * nb, bytes, &prof));
  size_t need = dgemm_workspace_bytes(g);
  if (need > 0) {
    size_t cap = (size_t)512 << 20;   // 512 MiB split-K workspace cap
    size_t want = need < cap ? need : cap;
    if (c->ws.n * sizeof(double) < want) RET(c->ws.ensure(want / sizeof(double) + 1));
  }
  int r = dgemm(g, c->st, c->ws.p, c->ws.n * sizeof(double));
  if (r) return fail(r, "dgemm launch failed");
  return prof_end(c, g.tag, prof);
}

extern "C" {

int xt_set_profile(xt_ctx* c, int mask) {
  if (!c) return fail(XT_ERR_ARG, "null ctx");
  c->prof_mask = mask;
  return 0;
}

// device ms, launches and algorithmic flops of GEMM class `tag` in the last
// xt_apply (one launch = one GEMM call including its split-K reduce)
int xt_profile_stats(const xt_ctx* c, int tag, double* out3) {
  if (!c || !out3 || tag < 1 || tag > 5) return fail(XT_ERR_ARG, "bad argument");
  out3[0] = c->prof_ms[tag]; out3[1] = c->prof_launches[tag]; out3[2] = c->prof_flops[tag];
  return 0;
}

// compulsory HBM bytes of GEMM class `tag` in the last xt_apply (every operand
// read once, the output written once): the denominator of a traffic ratio
int xt_profile_bytes(const xt_ctx* c, int tag, double* bytes) {
  if (!c || !bytes || tag < 1 || tag > 5) return fail(XT_ERR_ARG, "bad argument");
  *bytes = c->prof_bytes[tag];
  return 0;
}


int xt_abi_version(void) { return XT_ABI_VERSION; }
const char* xt_last_error(void) { return g_err.c_str(); }

int xt_create(const xt_desc* desc, xt_ctx** out) {
  if (!desc || !out) return fail(XT_ERR_ARG, "null argument");
  const xt_desc& d = *desc;
  if (d.nao <= 0 || d.nmo <= 0 || d.nc < 0 || d.no < 0 || d.nv <= 0 || d.nc + d.no + d.nv != d.nmo)
    return fail(XT_ERR_ARG, "inconsistent orbital dimensions (need nc+no+nv == nmo)");
  if (d.kind < XT_KIND_XTDA || d.kind > XT_KIND_XSF) return fail(XT_ERR_ARG, "unknown kind");
  if (d.kind == XT_KIND_XTDA && !d.restricted) return fail(XT_ERR_ARG, "XTDA needs a ROKS reference");
  if (d.kind == XT_KIND_UTDA && d.restricted) return fail(XT_ERR_ARG, "UTDA needs a UKS reference");
  if (d.kind == XT_KIND_XTDA && d.si <= 0) return fail(XT_ERR_ARG, "XTDA needs spin > 0");
  if (d.kind == XT_KIND_XSF && d.sa > 0 && (d.no < 2 || !d.restricted))
    return fail(XT_ERR_ARG, "XSF spin adaptation needs ROKS with no >= 2 (2S-1 > 0)");
  if (d.kind == XT_KIND_XSF && d.remove && d.no < 1)
    return fail(XT_ERR_ARG, "XSF OO compression needs an open shell");
  if (d.xctype < XT_XC_NONE || d.xctype > XT_XC_MGGA) return fail(XT_ERR_ARG, "bad xctype");
  const bool sf = (d.kind == XT_KIND_SF_DOWN || d.kind == XT_KIND_SF_UP || d.kind == XT_KIND_XSF);
  if (sf && d.sf_kernel != XT_SF_ALDA0 && d.sf_kernel != XT_SF_MC) return fail(XT_ERR_ARG, "bad sf_kernel");
  // spin flip: ALDA0 uses densities only, the grid needs ao[0] only (SF_TDA.py:73-80); the
  // multicollinear kernel is GGA / MGGA-shaped over (s, grad s[, tau_s]) (SF_TDA.py:997-1041)
  const bool dens_only = sf && d.sf_kernel == XT_SF_ALDA0;
  HIPCHK(hipSetDevice(d.device));
  xt_ctx* c = new xt_ctx();
  c->d = d;
  c->nbasis = d.restricted ? 1 : 2;
  c->ncomp = ((d.xctype == XT_XC_GGA || d.xctype == XT_XC_MGGA) && !dens_only) ? 4 : 1;
  c->nkc = (d.xctype == XT_XC_MGGA && !dens_only) ? 5 : c->ncomp;
  const int nb = d.restricted ? 0 : 1;   // beta basis index
  if (d.kind == XT_KIND_XTDA || d.kind == XT_KIND_UTDA) {
    c->nchan = 2; c->O = d.nc + d.no; c->V = d.no + d.nv; c->v0 = d.nc;
    c->occ_basis[0] = 0; c->vir_basis[0] = 0; c->occ_basis[1] = nb; c->vir_basis[1] = nb;
  } else if (d.kind == XT_KIND_SF_UP) {
    c->nchan = 1; c->O = d.nc; c->V = d.nv; c->v0 = d.nc + d.no;
    c->occ_basis[0] = nb; c->vir_basis[0] = 0;
  } else {
    c->nchan = 1; c->O = d.nc + d.no; c->V = d.no + d.nv; c->v0 = d.nc;
    c->occ_basis[0] = 0; c->vir_basis[0] = nb;
  }
  // exchange coefficients (XTDA.py:522-539 ; SF_TDA.py:273-277)
  const bool hf = (d.xctype == XT_XC_NONE);
  const double hyb = hf ? 1.0 : d.hyb;
  c->ck = hyb; c->ck_lr = 0.0;
  if (!hf && d.omega != 0.0) {
    if (sf) c->ck_lr = d.alpha - d.hyb;
    else if (d.alpha == 0.0) c->ck_lr = -d.hyb;
    else if (d.hyb == 0.0) { c->ck = 0.0; c->ck_lr = d.alpha; }
    else c->ck_lr = d.alpha - d.hyb;
  }
  for (int i = 0; i < 5; ++i) (void)hipEventCreate(&c->ev[i]);
  {
    // the only environment knobs, read here once per context: which XC kernels run the
    // fused classes outside their automatic ranges (tests/test_gpu_variants.py).
    // Defaults: dedicated M-backward for O <= 128, rho-forward for O > 64 and the
    // small-O rho-forward for O <= 48 (from 8 trial pairs), the engine's fused modes
    // otherwise (where they win or the dedicated kernels do not fit).  XT_W_KERNEL: 0 the
    // engine, 1 the O > 64 kernel, 3 the small-O kernel wherever they fit
    const char* em = getenv("XT_M_KERNEL");
    c->m_kernel = !(em && atoi(em) == 0);
    const char* ew = getenv("XT_W_KERNEL");
    c->w_kernel = ew ? (atoi(ew) == 0 ? 0 : atoi(ew) == 3 ? 3 : 1) : 2;
  }
  *out = c;
  return 0;
}

int xt_destroy(xt_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->d.device);
  DevBuf* bufs[] = {&c->C, &c->Bmo, &c->Bmo_lr, &c->Phi, &c->kern, &c->F, &c->eps, &c->vects,
                    &c->ze, &c->acc, &c->kx, &c->zr, &c->tbuf, &c->ubuf, &c->gam, &c->gam2, &c->ws,
                    &c->stage, &c->stage2, &c->zin, &c->sout, &c->trace, &c->zp, &c->accT, &c->wbuf, &c->taubuf,
                    &c->Kx};
  for (DevBuf* b : bufs) b->release();
  for (int i = 0; i < 5; ++i) (void)hipEventDestroy(c->ev[i]);
  for (hipEvent_t e : c->pev) (void)hipEventDestroy(e);
  delete c;
  return 0;
}

int xt_set_stream(xt_ctx* c, void* s) {
  if (!c) return fail(XT_ERR_ARG, "null ctx");
  c->st = (hipStream_t)s;
  return 0;
}

int xt_dim(const xt_ctx* c) { return c ? dim_of(c->d) : 0; }

int xt_last_timings(const xt_ctx* c, double* out4) {
  if (!c || !out4) return fail(XT_ERR_ARG, "null argument");
  for (int i = 0; i < 4; ++i) out4[i] = c->timings[i];
  return 0;
}

int xt_set_orbitals(xt_ctx* c, const double* ca, const double* cb, int ptr_kind) {
  if (!c || !ca) return fail(XT_ERR_ARG, "null argument");
  (void)hipSetDevice(c->d.device);
  const size_t nn = (size_t)c->d.nao * c->d.nmo;
  RET(c->C.ensure(nn * c->nbasis));
  const hipMemcpyKind k = ptr_kind == XT_PTR_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  HIPCHK(hipMemcpyAsync(c->C.p, ca, nn * 8, k, c->st));
  if (c->nbasis == 2) {
    if (!cb) return fail(XT_ERR_ARG, "UKS needs beta orbitals");
    HIPCHK(hipMemcpyAsync(c->C.p + nn, cb, nn * 8, k, c->st));
  }
  c->has_orb = true;
  c->kx_valid = false;
  return 0;
}

int xt_set_fock_mo(xt_ctx* c, const double* fa, const double* fb, const double* fa_hf,
                   const double* fb_hf, int ptr_kind) {
  if (!c || !fa || !fb) return fail(XT_ERR_ARG, "null argument");
  (void)hipSetDevice(c->d.device);
  const size_t mm = (size_t)c->d.nmo * c->d.nmo;
  // F layout: [fa, fb, fa_hf, fb_hf, fs = (fb_hf - fa_hf)/2, dF = fb_hf - fa_hf]
  RET(c->F.ensure(6 * mm));
  const hipMemcpyKind k = ptr_kind == XT_PTR_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  HIPCHK(hipMemcpyAsync(c->F.p, fa, mm * 8, k, c->st));
  HIPCHK(hipMemcpyAsync(c->F.p + mm, fb, mm * 8, k, c->st));
  const double* srcs[2] = {fa_hf ? fa_hf : fa, fb_hf ? fb_hf : fb};
  HIPCHK(hipMemcpyAsync(c->F.p + 2 * mm, srcs[0], mm * 8, k, c->st));
  HIPCHK(hipMemcpyAsync(c->F.p + 3 * mm, srcs[1], mm * 8, k, c->st));
  // fs and dF via a tiny GEMM-free host round trip is avoided: use geam-like GEMM with identity?
  // simpler: stage on host (nmo^2 is small)
  std::vector<double> a(mm), b(mm), s(mm), df(mm);
  HIPCHK(hipMemcpyAsync(a.data(), c->F.p + 2 * mm, mm * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipMemcpyAsync(b.data(), c->F.p + 3 * mm, mm * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  for (size_t i = 0; i < mm; ++i) { df[i] = b[i] - a[i]; s[i] = 0.5 * df[i]; }
  HIPCHK(hipMemcpy(c->F.p + 4 * mm, s.data(), mm * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(c->F.p + 5 * mm, df.data(), mm * 8, hipMemcpyHostToDevice));
  c->has_fock = true;
  return 0;
}

int xt_set_orbital_energies(xt_ctx* c, const double* ea, const double* eb, int ptr_kind) {
  if (!c || !ea || !eb) return fail(XT_ERR_ARG, "null argument");
  (void)hipSetDevice(c->d.device);
  const size_t n = c->d.nmo;
  RET(c->eps.ensure(2 * n));
  const hipMemcpyKind k = ptr_kind == XT_PTR_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  HIPCHK(hipMemcpyAsync(c->eps.p, ea, n * 8, k, c->st));
  HIPCHK(hipMemcpyAsync(c->eps.p + n, eb, n * 8, k, c->st));
  c->has_eps = true;
  return 0;
}

// Bmo[b][P] = C_b^T B_P C_b, chunked over P so host inputs stream through HBM.
// AO factor rows (np x nao x nao) -> MO factor Bmo[b][P] = C_b^T B_P C_b for
// P < np, rows np..naux_rows of each basis block zeroed (dst holds
// nbasis x naux_rows x nmo x nmo).
static int df_to_mo(xt_ctx* c, const double* cderi, int np_total, DevBuf& dst, int naux_rows, int ptr_kind) {
  const int nao = c->d.nao, nmo = c->d.nmo;
  const size_t mm = (size_t)nmo * nmo, aa = (size_t)nao * nao;
  RET(dst.ensure(mm * (size_t)naux_rows * c->nbasis));
  if (naux_rows > np_total)
    for (int b = 0; b < c->nbasis; ++b)
      HIPCHK(hipMemsetAsync(dst.p + ((size_t)b * naux_rows + np_total) * mm, 0,
                            (size_t)(naux_rows - np_total) * mm * 8, c->st));
  if (np_total <= 0) return 0;
  const size_t budget = (size_t)2 << 30;   // bytes per staging buffer
  int pc = (int)(budget / (8 * (aa > mm ? aa : mm)));
  if (pc < 1) pc = 1;
  if (pc > np_total) pc = np_total;
  RET(c->stage2.ensure((size_t)pc * nao * nmo));
  if (ptr_kind == XT_PTR_HOST) RET(c->stage.ensure((size_t)pc * aa));
  for (int p0 = 0; p0 < np_total; p0 += pc) {
    const int np = (p0 + pc <= np_total) ? pc : np_total - p0;
    const double* src = cderi + (size_t)p0 * aa;
    if (ptr_kind == XT_PTR_HOST) {
      HIPCHK(hipMemcpyAsync(c->stage.p, src, (size_t)np * aa * 8, hipMemcpyHostToDevice, c->st));
      src = c->stage.p;
    }
    for (int b = 0; b < c->nbasis; ++b) {
      const double* Cb = c->C.p + (size_t)b * nao * nmo;
      GemmDesc g1;   // T_P = B_P C  (nao x nmo)
      g1.M = nao; g1.N = nmo; g1.K = nao; g1.nb1 = np;
      g1.A = src; g1.sAm = nao; g1.sAk = 1; g1.sAb1 = (long)aa;
      g1.B = Cb; g1.sBk = nmo; g1.sBn = 1;
      g1.C = c->stage2.p; g1.ldc = nmo; g1.sCb1 = (long)nao * nmo;
      RET(gemm(c, g1));
      GemmDesc g2;   // Bmo_P = C^T T_P
      g2.M = nmo; g2.N = nmo; g2.K = nao; g2.nb1 = np;
      g2.A = Cb; g2.sAm = 1; g2.sAk = nmo;
      g2.B = c->stage2.p; g2.sBk = nmo; g2.sBn = 1; g2.sBb1 = (long)nao * nmo;
      g2.C = dst.p + ((size_t)b * naux_rows + p0) * mm; g2.ldc = nmo; g2.sCb1 = (long)mm;
      RET(gemm(c, g2));
    }
  }
  return 0;
}

int xt_set_jk_df(xt_ctx* c, const double* cderi, int which, int ptr_kind) {
  if (!c || !cderi) return fail(XT_ERR_ARG, "null argument");
  if (which != 0 && which != 1) return fail(XT_ERR_ARG, "which must be 0 (full range) or 1 (long range)");
  if (!c->has_orb) return fail(XT_ERR_STATE, "xt_set_orbitals must precede xt_set_jk_df");
  (void)hipSetDevice(c->d.device);
  untrim(c);
  DevBuf& dst = which == 0 ? c->Bmo : c->Bmo_lr;
  RET(df_to_mo(c, cderi, c->d.naux, dst, c->d.naux, ptr_kind));
  HIPCHK(hipStreamSynchronize(c->st));
  c->stage.release(); c->stage2.release();
  if (which == 0) c->has_df = true; else c->has_lr = true;
  c->kx_valid = false; c->k_resolved = -1;
  c->win_p0 = 0; c->win_np = -1;
  return 0;
}

// Re-lay an MO factor (nbasis blocks of old_rows x mm) with new_rows >= old_rows
// rows per block, the extra rows zero.
static int grow_factor(xt_ctx* c, DevBuf& B, int old_rows, int new_rows) {
  const size_t mm = (size_t)c->d.nmo * c->d.nmo;
  TmpBuf nb;
  RET(nb.ensure((size_t)c->nbasis * new_rows * mm));
  HIPCHK(hipMemsetAsync(nb.p, 0, nb.n * 8, c->st));
  for (int b = 0; b < c->nbasis; ++b)
    if (old_rows > 0)
      HIPCHK(hipMemcpyAsync(nb.p + (size_t)b * new_rows * mm, B.p + (size_t)b * old_rows * mm,
                            (size_t)old_rows * mm * 8, hipMemcpyDeviceToDevice, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  nb.swap(B);   // B takes the new rows, nb frees the old ones
  return 0;
}

int xt_set_jk_eri8(xt_ctx* c, const double* eri, int which, double tol, int p_rank, int p_count, int ptr_kind) {
  if (!c || !eri) return fail(XT_ERR_ARG, "null argument");
  if (which != 0 && which != 1) return fail(XT_ERR_ARG, "which must be 0 (full range) or 1 (long range)");
  if (p_count < 1 || p_rank < 0 || p_rank >= p_count) return fail(XT_ERR_ARG, "bad shard (p_rank, p_count)");
  if (!c->has_orb) return fail(XT_ERR_STATE, "xt_set_orbitals must precede xt_set_jk_eri8");
  (void)hipSetDevice(c->d.device);
  untrim(c);
  const int nao = c->d.nao;
  const long npair = (long)nao * (nao + 1) / 2;
  const size_t n8 = (size_t)npair * (npair + 1) / 2;
  const double* e = eri;
  TmpBuf ebuf, d, Lt, piv, Bao;
  if (ptr_kind == XT_PTR_HOST) {
    RET(ebuf.ensure(n8));
    HIPCHK(hipMemcpyAsync(ebuf.p, eri, n8 * 8, hipMemcpyHostToDevice, c->st));
    e = ebuf.p;
  }
  RET(d.ensure(npair));
  RET(piv.ensure(2));
  eri_diag(c->st, npair, e, d.p);
  long cap = 8L * nao < npair ? 8L * nao : npair;
  RET(Lt.ensure((size_t)cap * npair));
  double thr = tol;
  int rank = 0;
  for (; rank < npair; ++rank) {
    argmax(c->st, npair, d.p, piv.p);
    double hv[2];
    HIPCHK(hipMemcpyAsync(hv, piv.p, 16, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (rank == 0 && thr <= 0.0) thr = 1e-13 * hv[0];
    if (!(hv[0] > thr)) break;
    if (rank == cap) {   // grow the vector store
      const long ncap = 2 * cap < npair ? 2 * cap : npair;
      TmpBuf nl;
      RET(nl.ensure((size_t)ncap * npair));
      HIPCHK(hipMemcpyAsync(nl.p, Lt.p, (size_t)cap * npair * 8, hipMemcpyDeviceToDevice, c->st));
      HIPCHK(hipStreamSynchronize(c->st));
      nl.swap(Lt);
      cap = ncap;
    }
    chol_step(c->st, npair, rank, (long)hv[1], hv[0], e, Lt.p, npair, d.p);
  }
  ebuf.release(); d.release(); piv.release();
  // this rank's contiguous block of Cholesky vectors
  const int base = rank / p_count, rem = rank % p_count;
  const int lo = p_rank * base + (p_rank < rem ? p_rank : rem);
  const int np = base + (p_rank < rem ? 1 : 0);
  if (np > 0) {
    RET(Bao.ensure((size_t)np * nao * nao));
    chol_unpack(c->st, np, lo, nao, Lt.p, npair, Bao.p);
  }
  // common naux for the full-range and long-range factors (zero-padded)
  const bool other_set = which == 0 ? c->has_lr : c->has_df;
  int rows = np;
  if (other_set) {
    if (c->d.naux > rows) rows = c->d.naux;
    else if (c->d.naux < rows) RET(grow_factor(c, which == 0 ? c->Bmo_lr : c->Bmo, c->d.naux, rows));
  }
  DevBuf& dst = which == 0 ? c->Bmo : c->Bmo_lr;
  dst.release();
  RET(df_to_mo(c, Bao.p, np, dst, rows, XT_PTR_DEVICE));
  HIPCHK(hipStreamSynchronize(c->st));
  Bao.release(); Lt.release(); c->stage.release(); c->stage2.release();
  c->d.naux = rows;
  c->chol_rank = rank;
  if (which == 0) c->has_df = true; else c->has_lr = true;
  c->kx_valid = false; c->k_resolved = -1;
  c->win_p0 = 0; c->win_np = -1;
  return 0;
}

int xt_naux(const xt_ctx* c, int* naux_local, int* chol_rank) {
  if (!c) return fail(XT_ERR_ARG, "null argument");
  if (naux_local) *naux_local = c->d.naux;
  if (chol_rank) *chol_rank = c->chol_rank;
  return 0;
}

int xt_set_grid(xt_ctx* c, const double* ao, const double* w, const double* kernel, int ptr_kind) {
  if (!c || !ao || !w || !kernel) return fail(XT_ERR_ARG, "null argument");
  if (!c->has_orb) return fail(XT_ERR_STATE, "xt_set_orbitals must precede xt_set_grid");
  (void)hipSetDevice(c->d.device);
  const int nao = c->d.nao, nmo = c->d.nmo, ng = c->d.ngrid;
  const bool sf = (c->d.kind == XT_KIND_SF_DOWN || c->d.kind == XT_KIND_SF_UP || c->d.kind == XT_KIND_XSF);
  // input ao carries c->ncomp components (1 for the density-only ALDA0 spin-flip kernel)
  const int ncomp = c->ncomp;
  // + zeroed slack rows after the last plane (fused XC kernels read whole K-tiles)
  const size_t phi_used = (size_t)c->nbasis * ncomp * ng * nmo;
  RET(c->Phi.ensure(phi_used + (size_t)XC_GRID_SLACK * nmo));
  HIPCHK(hipMemsetAsync(c->Phi.p + phi_used, 0, (c->Phi.n - phi_used) * sizeof(double), c->st));
  const size_t gchunk_max = ((size_t)1 << 30) / (8 * (size_t)nao);
  const int gc = (int)(gchunk_max < (size_t)ng ? gchunk_max : ng);
  if (ptr_kind == XT_PTR_HOST) RET(c->stage.ensure((size_t)gc * nao));
  for (int comp = 0; comp < ncomp; ++comp) {
    for (int g0 = 0; g0 < ng; g0 += gc) {
      const int n = (g0 + gc <= ng) ? gc : ng - g0;
      const double* src = ao + ((size_t)comp * ng + g0) * nao;
      if (ptr_kind == XT_PTR_HOST) {
        HIPCHK(hipMemcpyAsync(c->stage.p, src, (size_t)n * nao * 8, hipMemcpyHostToDevice, c->st));
        src = c->stage.p;
      }
      for (int b = 0; b < c->nbasis; ++b) {
        GemmDesc g;
        g.M = n; g.N = nmo; g.K = nao;
        g.A = src; g.sAm = nao; g.sAk = 1;
        g.B = c->C.p + (size_t)b * nao * nmo; g.sBk = nmo; g.sBn = 1;
        g.C = c->Phi.p + (((size_t)b * ncomp + comp) * ng + g0) * nmo; g.ldc = nmo;
        RET(gemm(c, g));
      }
    }
  }
  if (sf && c->d.sf_kernel == XT_SF_ALDA0) {
    RET(to_device(c, c->kern, kernel, (size_t)ng, ptr_kind));   // already weighted
  } else {
    // UKS fxc (2, nk, 2, nk) x w, or the multicollinear spin-flip kernel (nk, nk) x 2 w
    const size_t n4 = (size_t)(sf ? 1 : 4) * c->nkc * c->nkc;
    RET(to_device(c, c->kern, kernel, n4 * ng, ptr_kind));
    RET(c->stage2.ensure(ng));
    const hipMemcpyKind k = ptr_kind == XT_PTR_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    HIPCHK(hipMemcpyAsync(c->stage2.p, w, (size_t)ng * 8, k, c->st));
    weight_fxc(c->st, (long)n4, ng, sf ? 2.0 : 1.0, c->stage2.p, c->kern.p);
  }
  HIPCHK(hipStreamSynchronize(c->st));
  c->stage.release(); c->stage2.release();
  c->has_grid = true;
  return 0;
}

int xt_set_oo_basis(xt_ctx* c, const double* vects, int ptr_kind) {
  if (!c || (!vects && c->d.no > 1)) return fail(XT_ERR_ARG, "null argument");
  (void)hipSetDevice(c->d.device);
  const size_t n = (size_t)c->d.no * c->d.no * (c->d.no * c->d.no - 1);
  if (n > 0) RET(to_device(c, c->vects, vects, n, ptr_kind));
  c->has_vects = true;
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// building blocks
// ---------------------------------------------------------------------------
// aux rows this context contracts over (its window of the resident factor)
static inline int naux_w(const xt_ctx* c) { return c->win_np < 0 ? c->d.naux : c->win_np; }
// basis block of an MO factor, full rows / from the window start
static inline const double* bmo_full(const xt_ctx* c, const DevBuf& B, int basis) {
  return B.p + (size_t)basis * c->d.naux * c->d.nmo * c->d.nmo;
}
static inline const double* bmo_of(xt_ctx* c, const DevBuf& B, int basis) {
  return bmo_full(c, B, basis) + (size_t)c->win_p0 * c->d.nmo * c->d.nmo;
}
static inline int krow0(const xt_ctx* c) { return c->kr0; }
static inline int krow1(const xt_ctx* c) { return c->kr1 < 0 ? c->O : c->kr1; }

// S[x] += coef * sum_P Bo[P, ry0:+nry, rx0:+nrx] Z[x] Bv[P, cx0:+ncx, cy0:+ncy]
// Z[x] at Z + x*svZ with row stride ldZ; S[x] at S + x*svS, row stride ldS.
static int sandwich(xt_ctx* c, const double* Bo, const double* Bv, int nz,
                    int ry0, int nry, int rx0, int nrx, int cx0, int ncx, int cy0, int ncy,
                    const double* Z, long ldZ, long svZ, double* S, long ldS, long svS, double coef) {
  if (nry <= 0 || nrx <= 0 || ncx <= 0 || ncy <= 0 || coef == 0.0) return 0;
  const int naux = naux_w(c), nmo = c->d.nmo;
  if (naux <= 0) return 0;
  const long mm = (long)nmo * nmo;
  const double left = 2.0 * nry * nrx * (double)nz * ncx + 2.0 * nry * (double)nz * ncx * ncy;
  const double right = 2.0 * (double)nz * nrx * ncx * ncy + 2.0 * nry * nrx * (double)nz * ncy;
  const size_t budget = (size_t)3 << 30;
  if (left <= right) {
    // T[P] (nry, nz, ncx) = Bo[P,rows] . Zr ; out(nry,nz,ncy) += T . Bv[P,cols]
    const size_t per = (size_t)nry * nz * ncx;
    int pc = (int)(budget / (8 * per)); if (pc < 1) pc = 1; if (pc > naux) pc = naux;
    RET(c->tbuf.ensure((size_t)pc * per));
    RET(c->zr.ensure((size_t)nrx * nz * ncx));
    RET(c->kx.ensure((size_t)nry * nz * ncy));
    // Zr[i][x][a] = Z[x][i][a]   (gather via GEMM-free copy: treat as batched strided copy)
    for (int x = 0; x < nz; ++x)
      HIPCHK(hipMemcpy2DAsync(c->zr.p + (size_t)x * ncx, (size_t)nz * ncx * 8, Z + x * svZ, ldZ * 8,
                              (size_t)ncx * 8, nrx, hipMemcpyDeviceToDevice, c->st));
    for (int p0 = 0; p0 < naux; p0 += pc) {
      const int np = (p0 + pc <= naux) ? pc : naux - p0;
      GemmDesc g1;
      g1.M = nry; g1.N = nz * ncx; g1.K = nrx; g1.nb1 = np;
      g1.A = Bo + p0 * mm + (long)ry0 * nmo + rx0; g1.sAm = nmo; g1.sAk = 1; g1.sAb1 = mm;
      g1.B = c->zr.p; g1.sBk = (long)nz * ncx; g1.sBn = 1;
      g1.C = c->tbuf.p; g1.ldc = (long)nz * ncx; g1.sCb1 = (long)per;
      RET(gemm(c, g1));
      GemmDesc g2;
      g2.M = nry * nz; g2.N = ncy; g2.K = ncx; g2.R = np;
      g2.A = c->tbuf.p; g2.sAm = ncx; g2.sAk = 1; g2.sAr = (long)per;
      g2.B = Bv + p0 * mm + (long)cx0 * nmo + cy0; g2.sBk = nmo; g2.sBn = 1; g2.sBr = mm;
      g2.C = c->kx.p; g2.ldc = ncy;
      g2.alpha = 1.0; g2.beta = (p0 == 0) ? 0.0 : 1.0;
      g2.tag = 1;
      RET(gemm(c, g2));
    }
    // S[x][j][b] += coef * kx[j][x][b]
    permute_add_strided(c->st, nz, nry, ncy, coef, c->kx.p, S, ldS, svS);
  } else {
    // W[P][x] (nrx, ncy) = Z[x] . Bv[P,cols] ; S[x] += coef * sum_P Bo[P,rows] W[P][x]
    const size_t per = (size_t)nz * nrx * ncy;
    int pc = (int)(budget / (8 * per)); if (pc < 1) pc = 1; if (pc > naux) pc = naux;
    RET(c->tbuf.ensure((size_t)pc * per));
    for (int p0 = 0; p0 < naux; p0 += pc) {
      const int np = (p0 + pc <= naux) ? pc : naux - p0;
      GemmDesc g1;
      g1.M = nrx; g1.N = ncy; g1.K = ncx; g1.nb1 = np; g1.nb2 = nz;
      g1.A = Z; g1.sAm = ldZ; g1.sAk = 1; g1.sAb1 = 0; g1.sAb2 = svZ;
      g1.B = Bv + p0 * mm + (long)cx0 * nmo + cy0; g1.sBk = nmo; g1.sBn = 1; g1.sBb1 = mm;
      g1.C = c->tbuf.p; g1.ldc = ncy; g1.sCb1 = (long)per; g1.sCb2 = (long)nrx * ncy;
      RET(gemm(c, g1));
      GemmDesc g2;
      g2.M = nry; g2.N = ncy; g2.K = nrx; g2.R = np; g2.nb1 = nz;
      g2.A = Bo + p0 * mm + (long)ry0 * nmo + rx0; g2.sAm = nmo; g2.sAk = 1; g2.sAr = mm;
      g2.B = c->tbuf.p; g2.sBk = ncy; g2.sBn = 1; g2.sBr = (long)per; g2.sBb1 = (long)nrx * ncy;
      g2.C = S; g2.ldc = ldS; g2.sCb1 = svS;
      g2.alpha = coef; g2.beta = 1.0;
      RET(gemm(c, g2));
    }
  }
  return 0;
}

// gamma[x,P] (+)= sum_{i,a} Z[x][i][a] Bmo[P][r0+i][c0+a]
static int coulomb_gamma(xt_ctx* c, const double* B, int nz, int r0, int nr, int c0, int ncl,
                         const double* Z, long ldZ, long svZ, double* gam, double beta) {
  const int nmo = c->d.nmo;
  GemmDesc g;
  g.M = nz; g.N = naux_w(c); g.K = ncl; g.R = nr;
  g.A = Z; g.sAm = svZ; g.sAk = 1; g.sAr = ldZ;
  g.B = B + (long)r0 * nmo + c0; g.sBn = (long)nmo * nmo; g.sBk = 1; g.sBr = nmo;
  g.C = gam; g.ldc = naux_w(c); g.beta = beta;
  return gemm(c, g);
}

// S[x][i][a] += coef * sum_P gamma[x,P] Bmo[P][r0+i][c0+a]
static int coulomb_project(xt_ctx* c, const double* B, int nz, int r0, int nr, int c0, int ncl,
                           const double* gam, double* S, long ldS, long svS, double coef) {
  const int nmo = c->d.nmo;
  GemmDesc g;
  g.M = nz; g.N = ncl; g.K = naux_w(c); g.nb1 = nr;
  g.A = gam; g.sAm = naux_w(c); g.sAk = 1;
  g.B = B + (long)r0 * nmo + c0; g.sBk = (long)nmo * nmo; g.sBn = 1; g.sBb1 = nmo;
  g.C = S; g.ldc = svS; g.sCb1 = ldS;
  g.alpha = coef; g.beta = 1.0;
  return gemm(c, g);
}

// S[x] += alpha * Z[x] . F[fr0:, fc0:]   (Z: nr x K rows; F block K x ncl, row-major in nmo)
static int right_mo(xt_ctx* c, int nz, int nr, int K, int ncl, const double* Z, long ldZ, long svZ,
                    const double* F, long sFk, long sFn, double* S, long ldS, long svS, double alpha) {
  if (nr <= 0 || K <= 0 || ncl <= 0 || alpha == 0.0) return 0;
  GemmDesc g;
  g.M = nr; g.N = ncl; g.K = K; g.nb1 = nz;
  g.A = Z; g.sAm = ldZ; g.sAk = 1; g.sAb1 = svZ;
  g.B = F; g.sBk = sFk; g.sBn = sFn;
  g.C = S; g.ldc = ldS; g.sCb1 = svS;
  g.alpha = alpha; g.beta = 1.0;
  return gemm(c, g);
}

// S[x] += alpha * F . Z[x]   (F block nr x K with strides (sFm, sFk))
static int left_mo(xt_ctx* c, int nz, int nr, int K, int ncl, const double* F, long sFm, long sFk,
                   const double* Z, long ldZ, long svZ, double* S, long ldS, long svS, double alpha) {
  if (nr <= 0 || K <= 0 || ncl <= 0 || alpha == 0.0) return 0;
  GemmDesc g;
  g.M = nr; g.N = ncl; g.K = K; g.nb1 = nz;
  g.A = F; g.sAm = sFm; g.sAk = sFk;
  g.B = Z; g.sBk = ldZ; g.sBn = 1; g.sBb1 = svZ;
  g.C = S; g.ldc = ldS; g.sCb1 = svS;
  g.alpha = alpha; g.beta = 1.0;
  return gemm(c, g);
}

// ---------------------------------------------------------------------------
// Channel groups.  Spin channels that share one MO basis are contracted
// together (ROKS X-TDA: both channels form one group of 2*nz "vectors"; UKS:
// one group per channel; SF/XSF: one channel).  Per group (channels ch0..ch0+nch-1,
// nzg = nch*nz rows):
//   Ze   : (nzg, O, V) rows of c->ze starting at channel ch0
//   Zp   : (O, nzg, V)  permuted copy for contractions over the occupied index
//   accT : (O, nzg, V)  results of those contractions (exchange, XC back-2),
//          permute-added into acc at the end of xt_apply
// ---------------------------------------------------------------------------
struct Group { int ch0, nch, ob, vb; };

static int channel_groups(const xt_ctx* c, Group* g) {
  if (c->nchan == 2 && c->occ_basis[0] == c->occ_basis[1] && c->vir_basis[0] == c->vir_basis[1]) {
    g[0] = {0, 2, c->occ_basis[0], c->vir_basis[0]};
    return 1;
  }
  for (int ch = 0; ch < c->nchan; ++ch) g[ch] = {ch, 1, c->occ_basis[ch], c->vir_basis[ch]};
  return c->nchan;
}

// accT_g[(j,x)][b] += coef * sum_P sum_{i,a} B[P][j][i] Zp_g[i][x][a] B[P][v0+a][v0+b]
static int exchange_main(xt_ctx* c, int nz, const DevBuf& B, double coef) {
  if (coef == 0.0) return 0;
  const int O = c->O, V = c->V, nmo = c->d.nmo, naux = naux_w(c);
  const long mm = (long)nmo * nmo, chs = (long)nz * O * V;
  if (naux <= 0) return 0;
  Group gr[2];
  const int ngr = channel_groups(c, gr);
  for (int q = 0; q < ngr; ++q) {
    const int nzg = gr[q].nch * nz;
    const size_t per = (size_t)O * nzg * V;
    int pc = (int)(((size_t)3 << 30) / (8 * per));
    if (pc < 1) pc = 1;
    if (pc > naux) pc = naux;
    RET(c->tbuf.ensure((size_t)pc * per));
    const double* Bo = bmo_of(c, B, gr[q].ob);
    const double* Bv = bmo_of(c, B, gr[q].vb);
    const double* zp = c->zp.p + gr[q].ch0 * chs;
    double* at = c->accT.p + gr[q].ch0 * chs;
    for (int p0 = 0; p0 < naux; p0 += pc) {
      const int np = (p0 + pc <= naux) ? pc : naux - p0;
      GemmDesc g1;   // T[P] (O, nzg*V) = B[P][occ][occ] . Zp
      g1.M = O; g1.N = nzg * V; g1.K = O; g1.nb1 = np;
      g1.A = Bo + p0 * mm; g1.sAm = nmo; g1.sAk = 1; g1.sAb1 = mm;
      g1.B = zp; g1.sBk = (long)nzg * V; g1.sBn = 1;
      g1.C = c->tbuf.p; g1.ldc = (long)nzg * V; g1.sCb1 = (long)per;
      RET(gemm(c, g1));
      GemmDesc g2;   // accT[(j,x)][b] += coef * sum_{P,a} T[P][(j,x)][a] B[P][v0+a][v0+b]
      g2.M = O * nzg; g2.N = V; g2.K = V; g2.R = np;
      g2.A = c->tbuf.p; g2.sAm = V; g2.sAk = 1; g2.sAr = (long)per;
      g2.B = Bv + p0 * mm + (long)c->v0 * nmo + c->v0; g2.sBk = nmo; g2.sBn = 1; g2.sBr = mm;
      g2.C = at; g2.ldc = V;
      g2.alpha = coef; g2.beta = 1.0;
      g2.tag = 1;
      RET(gemm(c, g2));
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Stored MO exchange (XT_K_STORED).  Per channel group g (occupied basis ob,
// virtual basis vb) the exchange kernel of the sandwich above, contracted over
// P once per solve and kept in HBM:
//   Kx_g[(i,a),(j,b)] = ck sum_P Bo[P][i][j] Bv[P][v0+a][v0+b] + ck_lr (same, long range)
// (symmetric under (i,a) <-> (j,b); (O V)^2 doubles per group).  Per A.x the
// exchange is then one skinny GEMM  acc_g[x][(j,b)] -= sum_(i,a) Ze_g[x][(i,a)] Kx_g[(i,a),(j,b)],
// streaming Kx once (HBM-bound, 2 nzg flops per 8 bytes) instead of the
// 2 naux nzg O V^2 flops of the DF sandwich.  The reference makes the same
// trade when PySCF keeps the ERIs incore (mf._eri, max_memory) rather than
// running integral-direct J/K.
// ---------------------------------------------------------------------------
// row stride of the stored exchange: O V rounded up to 8 doubles (64 B) so every
// row starts 16-B aligned for the streaming kernel's wide loads
static size_t kx_ld(const xt_ctx* c) {
  const size_t ov = (size_t)c->O * c->V;
  return (ov + 7) & ~(size_t)7;
}

static size_t kx_doubles(const xt_ctx* c) {
  Group gr[2];
  const int ngr = channel_groups(c, gr);
  return (size_t)(krow1(c) - krow0(c)) * c->V * kx_ld(c) * (size_t)ngr;
}

static bool has_exchange(const xt_ctx* c) {
  return (c->ck != 0.0 || c->ck_lr != 0.0) && c->d.naux > 0;
}

extern "C" int xt_set_partition(xt_ctx* c, int p0, int p1, int i0, int i1) {
  if (!c) return fail(XT_ERR_ARG, "null ctx");
  if (c->trimmed) return fail(XT_ERR_STATE, "the MO factor was trimmed to this rank's aux window; set it again");
  if (p0 < 0 || p1 < p0 || p1 > c->d.naux) return fail(XT_ERR_ARG, "aux window outside [0, naux]");
  if (i0 < 0 || i1 < i0 || i1 > c->O) return fail(XT_ERR_ARG, "exchange rows outside [0, O]");
  c->win_p0 = p0; c->win_np = p1 - p0;
  c->kr0 = i0; c->kr1 = i1;
  c->kx_valid = false; c->k_resolved = -1;
  return 0;
}

static int resolve_kmode(xt_ctx* c) {
  if (c->k_resolved >= 0) return 0;
  if (!has_exchange(c) || c->kmode == XT_K_DIRECT) { c->k_resolved = 0; return 0; }
  if (c->kmode == XT_K_STORED) { c->k_resolved = 1; return 0; }
  const size_t need = kx_doubles(c) * 8;
  size_t cap;
  if (c->k_max_bytes > 0) {
    cap = (size_t)c->k_max_bytes;
  } else {
    size_t fr = 0, tot = 0;
    HIPCHK(hipMemGetInfo(&fr, &tot));
    fr += c->Kx.n * 8;                       // an existing matrix would be reused
    size_t reserve = tot / 10;
    if (reserve < ((size_t)24 << 30)) reserve = (size_t)24 << 30;   // XC chunks, Davidson subspace
    cap = fr > reserve ? fr - reserve : 0;
  }
  c->k_resolved = need <= cap ? 1 : 0;
  return 0;
}

// occupied rows per stored-exchange build GEMM (the fold of the symmetric build, build_kx)
constexpr int KX_FOLD = 8;

static int build_kx(xt_ctx* c) {
  if (c->trimmed) return fail(XT_ERR_STATE, "the stored exchange needs every aux row: set the factor again");
  const int O = c->O, V = c->V, nmo = c->d.nmo, naux = c->d.naux;
  const long mm = (long)nmo * nmo;
  const size_t ov = (size_t)O * V, ld = kx_ld(c);
  const int i0 = krow0(c), i1 = krow1(c);
  const size_t blk = (size_t)(i1 - i0) * V * ld;   // this context's rows of one group
  Group gr[2];
  const int ngr = channel_groups(c, gr);
  if (blk == 0) { c->kx_valid = true; return 0; }
  // + zeroed slack rows after the last group (the streaming kernel's tail loads)
  RET(c->Kx.ensure(blk * ngr + (size_t)SKINNY_B_SLACK * ld));
  HIPCHK(hipMemsetAsync(c->Kx.p, 0, c->Kx.n * 8, c->st));
  for (int q = 0; q < ngr; ++q) {
    double* K = c->Kx.p + (size_t)q * blk - (size_t)i0 * V * ld;   // row (i,a) at (i V + a) ld
    for (int pass = 0; pass < 2; ++pass) {
      const double coef = pass ? c->ck_lr : c->ck;
      if (coef == 0.0) continue;
      const DevBuf& B = pass ? c->Bmo_lr : c->Bmo;
      const double* Bo = bmo_full(c, B, gr[q].ob);   // all aux rows: Kx sums over every P
      const double* Bv = bmo_full(c, B, gr[q].vb) + (long)c->v0 * nmo + c->v0;
      // batch a: Kx[(i,a)][(j,b)] += coef sum_P Bo[P][i][j] Bv[P][a][b] with rows (i, j) of
      // a chunk of KX_FOLD occupied i in one GEMM (two-level rows: i strides nmo in Bo and
      // V ld in Kx, j strides 1 and V).  Kx is symmetric under (i,a) <-> (j,b), so a chunk
      // [ci, ce) computes only j >= ci (and the j < i0 outside this context's rows); the
      // blocks (i, j) with i0 <= j < ci are transposes of blocks built by earlier chunks
      // and are mirrored afterwards: ~54 % of the full build's flops at O = 101.
      for (int ci = i0; ci < i1; ci += KX_FOLD) {
        const int ce = ci + KX_FOLD < i1 ? ci + KX_FOLD : i1;
        const int jr[2][2] = {{0, i0}, {ci, O}};
        for (int r = 0; r < 2; ++r) {
          const int j0 = jr[r][0], j1 = jr[r][1];
          if (j1 <= j0) continue;
          GemmDesc g;
          g.M = (ce - ci) * (j1 - j0); g.N = V; g.K = naux; g.nb1 = V;
          g.rdiv = j1 - j0; g.sAm_hi = nmo; g.sC_hi = (long)V * ld;
          g.A = Bo + (long)ci * nmo + j0; g.sAm = 1; g.sAk = mm; g.sAb1 = 0;
          g.B = Bv; g.sBk = mm; g.sBn = 1; g.sBb1 = nmo;
          g.C = K + (size_t)ci * V * ld + (size_t)j0 * V; g.ldc = V; g.sCb1 = (long)ld;
          g.alpha = coef; g.beta = 1.0;
          RET(gemm(c, g));
        }
      }
    }
    kx_mirror(c->st, O, V, (long)ld, i0, i1, KX_FOLD, K);
    HIPCHK(hipGetLastError());   // a rejected mirror launch would leave zero blocks in Kx
  }
  HIPCHK(hipStreamSynchronize(c->st));
  c->kx_valid = true;
  return 0;
}

// Per group: acc_g[x][(j,b)] -= sum_{(i,a), i in [i0,i1)} Ze_g[x][(i,a)] Kx_g[(i,a)][(j,b)].
// Up to SKINNY_MAX_M rows (2 nz <= 48: the headline's 40) the skinny streaming kernel
// (xt_exch.hip) reads Kx once with wide loads straight into the MFMA operands;
// more rows take the generic tile, which also reads Kx once.
static int exchange_stored(xt_ctx* c, int nz) {
  const size_t ov = (size_t)c->O * c->V, ld = kx_ld(c);
  const long chs = (long)nz * ov;
  const int i0 = krow0(c), i1 = krow1(c);
  const size_t blk = (size_t)(i1 - i0) * c->V * ld;
  if (blk == 0) return 0;
  Group gr[2];
  const int ngr = channel_groups(c, gr);
  for (int q = 0; q < ngr; ++q) {
    const int M = gr[q].nch * nz, K = (i1 - i0) * c->V;
    const double* A = c->ze.p + gr[q].ch0 * chs + (long)i0 * c->V;
    const double* B = c->Kx.p + (size_t)q * blk;
    double* C = c->acc.p + gr[q].ch0 * chs;
    if (M <= SKINNY_MAX_M) {
      bool prof = false;
      RET(prof_begin(c, 1, 2.0 * M * (double)ov * K, 8.0 * ((double)ov * K + (double)M * K + 2.0 * M * (double)ov), &prof));
      const size_t need = skinny_workspace_bytes(M, (int)ov, K);
      if (c->ws.n * sizeof(double) < need) RET(c->ws.ensure(need / sizeof(double) + 1));
      const int r = skinny_gemm(M, (int)ov, K, -1.0, A, (long)ov, B, (long)ld, 1.0, C, (long)ov,
                                c->ws.p, c->ws.n * sizeof(double), c->st);
      if (r) return fail(r, "skinny exchange launch failed");
      RET(prof_end(c, 1, prof));
      continue;
    }
    GemmDesc g;
    g.M = M; g.N = (int)ov; g.K = K;
    g.A = A; g.sAm = (long)ov; g.sAk = 1;
    g.B = B; g.sBk = (long)ld; g.sBn = 1;
    g.C = C; g.ldc = (long)ov;
    g.alpha = -1.0; g.beta = 1.0;
    g.tag = 1;
    RET(gemm(c, g));
  }
  return 0;
}

// XSF with spin adaptation SA >= 2 through the stored matrix: the main exchange
// (-Kx z) and the twelve Delta-A exchange projections (XSF_TDA.py:1175-1274, the
// direct sandwiches of xsf_delta_a) are all sub-blocks of Kx applied to the four
// source blocks of z, so ONE stream of Kx with the four blocks as 4 nz rows gives
// every term; a 4 x 4 weight table (source block, target block) combines them.
// Kx carries c_K: the Delta-A coefficients (on sum_P B B) are divided by it.
static bool xsf_fused_k(const xt_ctx* c) {
  const xt_desc& d = c->d;
  return d.kind == XT_KIND_XSF && d.sa > 1 && c->k_resolved == 1 && c->ck != 0.0 && c->ck_lr == 0.0 &&
         c->nchan == 1;
}

static int exchange_stored_xsf(xt_ctx* c, int nz) {
  const xt_desc& d = c->d;
  const int O = c->O, V = c->V, nc = d.nc, no = d.no;
  const size_t ov = (size_t)O * V, ld = kx_ld(c);
  const int i0 = krow0(c), i1 = krow1(c);
  const size_t blk = (size_t)(i1 - i0) * V * ld;
  if (blk == 0) return 0;
  const int K = (i1 - i0) * V;
  const int zmax = SKINNY_MAX_M / 4;           // trial vectors per Kx stream
  // coefficient table (xsf_delta_a's sandwich coefficients / c_K), source X -> target Y
  const double si = no / 2.0, fg = d.fglobal, ff = fg * d.foo, tsm1 = 2 * si - 1;
  const double f1 = sqrt((2 * si + 1) / (2 * si)) - 1;
  const double f2 = sqrt((2 * si + 1) / (2 * si - 1));
  const double f3 = sqrt((2 * si) / (2 * si - 1)) - 1;
  enum { CV = 0, CO = 1, OV = 2, OO = 3 };
  double dk[4][4] = {};
  dk[CO][CV] = dk[CV][CO] = dk[OV][CV] = dk[CV][OV] = -fg * f1;   // cv_co, co_cv, cv_ov, ov_cv
  dk[OV][CO] = dk[CO][OV] = -fg / tsm1;                           // co_ov, ov_co
  if (d.sa > 2) {
    dk[OO][CV] = dk[CV][OO] = -ff * (f2 - 1);                     // cv_oo, oo_cv
    dk[OO][CO] = dk[CO][OO] = dk[OO][OV] = dk[OV][OO] = -ff * f3; // co_oo, oo_co, ov_oo, oo_ov
  }
  W16 w;
  for (int X = 0; X < 4; ++X)
    for (int Y = 0; Y < 4; ++Y) w.w[4 * X + Y] = -1.0 + dk[X][Y] / c->ck;   // main exchange: -Kx z
  for (int z0 = 0; z0 < nz; z0 += zmax) {
    const int nzb = nz - z0 < zmax ? nz - z0 : zmax, M = 4 * nzb;
    RET(c->zr.ensure((size_t)M * ov));
    RET(c->tbuf.ensure((size_t)M * ov));
    xsf_split4(c->st, nzb, O, V, nc, no, c->ze.p + (size_t)z0 * ov, c->zr.p);
    bool prof = false;
    RET(prof_begin(c, 1, 2.0 * M * (double)ov * K, 8.0 * ((double)ov * K + (double)M * K + 2.0 * M * (double)ov),
                   &prof));
    const size_t need = skinny_workspace_bytes(M, (int)ov, K);
    if (c->ws.n * sizeof(double) < need) RET(c->ws.ensure(need / sizeof(double) + 1));
    const int r = skinny_gemm(M, (int)ov, K, 1.0, c->zr.p + (long)i0 * V, (long)ov, c->Kx.p, (long)ld, 0.0,
                              c->tbuf.p, (long)ov, c->ws.p, c->ws.n * sizeof(double), c->st);
    if (r) return fail(r, "skinny exchange launch failed");
    RET(prof_end(c, 1, prof));
    xsf_combine4(c->st, nzb, O, V, nc, no, w, c->tbuf.p, c->acc.p + (size_t)z0 * ov);
  }
  return 0;
}

extern "C" int xt_set_exchange_mode(xt_ctx* c, int mode, double max_gib) {
  if (!c) return fail(XT_ERR_ARG, "null ctx");
  if (mode < XT_K_AUTO || mode > XT_K_STORED) return fail(XT_ERR_ARG, "bad exchange mode");
  c->kmode = mode;
  c->k_max_bytes = max_gib > 0 ? max_gib * (double)((size_t)1 << 30) : 0.0;
  c->k_resolved = -1;
  if (mode == XT_K_DIRECT) { c->Kx.release(); c->kx_valid = false; }
  return 0;
}

extern "C" int xt_exchange_plan(xt_ctx* c, int* stored, double* k_gib) {
  if (!c) return fail(XT_ERR_ARG, "null ctx");
  (void)hipSetDevice(c->d.device);
  RET(resolve_kmode(c));
  if (stored) *stored = c->k_resolved == 1 ? 1 : 0;
  if (k_gib) *k_gib = has_exchange(c) ? kx_doubles(c) * 8.0 / (double)((size_t)1 << 30) : 0.0;
  return 0;
}

// Once a partitioned context holds its rows of the stored exchange, only the aux window
// [win_p0, win_p0 + win_np) of the MO factor is ever read again (J, the XSF Delta-A, the
// preconditioner diagonals): the other rows are dropped, so a replicated factor costs
// naux / N rows per rank instead of naux (24 GB -> 3 GB at the headline, N = 8).
static int trim_factor(xt_ctx* c) {
  const size_t mm = (size_t)c->d.nmo * c->d.nmo;
  const int np = c->win_np, p0 = c->win_p0, naux = c->d.naux;
  DevBuf* bufs[2] = {&c->Bmo, &c->Bmo_lr};
  for (DevBuf* B : bufs) {
    if (!B->p) continue;
    TmpBuf nb;
    RET(nb.ensure((size_t)c->nbasis * np * mm));
    for (int b = 0; b < c->nbasis; ++b)
      HIPCHK(hipMemcpyAsync(nb.p + (size_t)b * np * mm, B->p + ((size_t)b * naux + p0) * mm, (size_t)np * mm * 8,
                            hipMemcpyDeviceToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    nb.swap(*B);   // B takes the window, nb frees the full factor
  }
  c->naux_full = naux;
  c->d.naux = np;
  c->win_p0 = 0; c->win_np = -1;
  c->trimmed = true;
  return 0;
}

extern "C" int xt_prepare(xt_ctx* c, int* k_mode, double* k_gib) {
  if (!c) return fail(XT_ERR_ARG, "null ctx");
  (void)hipSetDevice(c->d.device);
  if (has_exchange(c) && !c->has_df) return fail(XT_ERR_STATE, "DF factor not set");
  RET(resolve_kmode(c));
  if (c->k_resolved == 1 && !c->kx_valid) RET(build_kx(c));
  if (c->k_resolved == 1 && c->kx_valid && c->win_np > 0 && c->win_np < c->d.naux) RET(trim_factor(c));
  if (k_mode) *k_mode = c->k_resolved == 1 ? XT_K_STORED : XT_K_DIRECT;
  if (k_gib) *k_gib = c->k_resolved == 1 ? kx_doubles(c) * 8.0 / (double)((size_t)1 << 30) : 0.0;
  return 0;
}

// ---------------------------------------------------------------------------
// XC response over the grid (chunks of G points), W route (see k_xc_uks_w):
//   F1  U = PhiV0 Ze^T                              (GEMM, tag 2)
//   F2' rhoW[g][xg][c] = sum_a (PhiO0 Zp)[g,xg,a] dPhiV_c[g,a]
//                                                   (fused GEMM mode 1, tag 4: W never stored)
//   point kernel: rho = U-part + rhoW; wv; U <- L; rhoW <- wv[1..3]
//   B1  acc += L^T PhiV0                            (GEMM, tag 3)
//   B2' accT += PhiO0^T M, M[g,xg,a] = sum_c wv_c dPhiV_c[g,a] generated on the fly
//                                                   (fused GEMM mode 2, tag 5: M never stored)
// LDA / ALDA0: F1, point kernel, B1.
// ---------------------------------------------------------------------------
static int xc_response(xt_ctx* c, int nz) {
  const int O = c->O, V = c->V, nmo = c->d.nmo, ng = c->d.ngrid, nc = c->ncomp;
  const int nch = c->nchan;
  const bool gga = (nc == 4);
  const bool mgga = (c->nkc == 5);
  const long chs = (long)nz * O * V;
  Group gr[2];
  const int ngr = channel_groups(c, gr);
  const size_t per_g = (size_t)nch * nz * O * (mgga ? 4 : 1) + (gga ? (size_t)nch * nz * 3 : 0);
  size_t G = ((size_t)8 << 30) / (8 * per_g);
  if (G > (size_t)ng) G = ng;
  if (G < 64) G = 64 < (size_t)ng ? 64 : ng;
  RET(c->ubuf.ensure((size_t)nch * nz * O * G));
  if (gga) RET(c->wbuf.ensure((size_t)nch * nz * 3 * (G + XC_GRID_SLACK)));
  // MGGA: three tau planes T_c = dPhiV_c Ze^T laid out like U (forward), then the tau
  // potential's back operands 1/2 wv_tau dPhiO_c (point kernel)
  if (mgga) RET(c->taubuf.ensure((size_t)3 * nch * nz * O * G));
  const long compP = (long)ng * nmo;
  const long basP = (long)nc * compP;
  const int nab = (V + 15) / 16;
  for (int g0 = 0; g0 < ng; g0 += (int)G) {
    const int n = (g0 + (int)G <= ng) ? (int)G : ng - g0;
    double* Ug[2]; double* Rg[2]; long ldU[2], ldR[2];
    for (int q = 0; q < ngr; ++q) {
      const int nzg = gr[q].nch * nz;
      Ug[q] = c->ubuf.p + (long)gr[q].ch0 * nz * O * n;  ldU[q] = (long)nzg * O;
      // each group's wv block is followed by XC_GRID_SLACK zero rows (the M-backward
      // kernel's last K-tile reads them instead of masking rows past n)
      Rg[q] = gga ? c->wbuf.p + (long)gr[q].ch0 * nz * 3 * (n + XC_GRID_SLACK) : nullptr;  ldR[q] = (long)nzg * 3;
      if (gga && hipMemsetAsync(Rg[q] + (long)n * ldR[q], 0, sizeof(double) * XC_GRID_SLACK * ldR[q], c->st) !=
                     hipSuccess)
        return fail(XT_ERR_HIP, "wv slack memset failed");
      const double* PV = c->Phi.p + gr[q].vb * basP + (long)g0 * nmo + c->v0;
      const double* PO = c->Phi.p + gr[q].ob * basP + (long)g0 * nmo;
      GemmDesc f1;   // U[g][(x,i)] = sum_a PhiV0[g][a] Ze[(x,i)][a]
      f1.M = n; f1.N = nzg * O; f1.K = V;
      f1.A = PV; f1.sAm = nmo; f1.sAk = 1;
      f1.B = c->ze.p + gr[q].ch0 * chs; f1.sBn = V; f1.sBk = 1;
      f1.C = Ug[q]; f1.ldc = ldU[q];
      f1.tag = 2;
      RET(gemm(c, f1));
      if (mgga) {
        const long tcs = (long)nch * nz * O * n;
        for (int cc = 1; cc < 4; ++cc) {   // T_c[g][(x,i)] = sum_a dPhiV_c[g][a] Ze[(x,i)][a]
          GemmDesc ft = f1;
          ft.A = PV + cc * compP;
          ft.C = c->taubuf.p + (cc - 1) * tcs + (long)gr[q].ch0 * nz * O * n;
          RET(gemm(c, ft));
        }
      }
      // the dedicated kernel pays off from ~5 occupied 16-row blocks up (O = 101: 168.6 vs
      // 173.1 ms/step; O = 91, C3mc: 75.2 vs 87.0; O = 34 / 37: 18 % / 15 % slower than the
      // engine's mode 1, and the small-O kernel takes O <= 48)
      const bool w_ded = c->w_kernel == 1 || (c->w_kernel == 2 && O > 64);
      const bool w_small = (c->w_kernel == 3 || (c->w_kernel == 2 && nzg >= 8)) &&
                           xc_rho_ws_lds_bytes(O) <= 160 * 1024;
      if (gga && w_small) {
        // small-O kernel (xt_xcws.hip): every pair of a 64-point block, weights staged once
        bool prof = false;
        RET(prof_begin(c, 4, 2.0 * nzg * V * (double)n * (O + 3),
                       8.0 * ((double)nzg * O * V + (double)n * O + 3.0 * n * V + 3.0 * n * nzg), &prof));
        const int r = xc_rho_ws(O, nzg, V, n, PO, nmo, c->zp.p + gr[q].ch0 * chs, (long)nzg * V, V,
                                PV + compP, compP, nmo, Rg[q], ldR[q], c->st);
        if (r) return fail(r, "xc_rho_ws launch failed");
        RET(prof_end(c, 4, prof));
      } else if (gga && w_ded && xc_rho_w_lds_bytes(O) <= 160 * 1024) {
        // dedicated kernel (xt_xcw.hip); tag 4 timing
        bool prof = false;
        // flops: the T = PhiO^T Zp GEMM (2 O per T element) + the fused gradient
        // contraction rhoW = sum_a dPhiV_c T (3 FMAs per T element)
        RET(prof_begin(c, 4, 2.0 * nzg * V * (double)n * (O + 3),
                       8.0 * ((double)nzg * O * V + (double)n * O + 3.0 * n * V + 3.0 * n * nzg), &prof));
        const int r = xc_rho_w(O, nzg, V, n, PO, nmo, c->zp.p + gr[q].ch0 * chs, (long)nzg * V, V,
                               PV + compP, compP, nmo, Rg[q], ldR[q], c->st);
        if (r) return fail(r, "xc_rho_w launch failed");
        RET(prof_end(c, 4, prof));
      } else if (gga) {
        GemmDesc f2;   // rhoW[g][xg][c] = sum_a sum_i PhiO0[g][i] Zp[i][xg][a] dPhiV_c[g][a]
        f2.M = 16 * nzg; f2.N = n; f2.K = O; f2.R = nab;
        f2.A = c->zp.p + gr[q].ch0 * chs; f2.sAm = 1; f2.sAk = (long)nzg * V; f2.sAr = 16;
        f2.B = PO; f2.sBk = 1; f2.sBn = nmo;
        f2.fz.mode = 1; f2.fz.ablk = V; f2.fz.V = V; f2.fz.nx = nzg;
        f2.fz.w = PV + compP; f2.fz.wc = compP; f2.fz.wg = nmo;
        f2.fz.rho = Rg[q]; f2.fz.rg = ldR[q];
        f2.tag = 4;
        f2.flops = 2.0 * nzg * V * (double)n * (O + 3);   // GEMM + fused contraction
        // Zp, PhiO0, dPhiV_{x,y,z} in; rhoW out
        f2.bytes = 8.0 * ((double)nzg * O * V + (double)n * O + 3.0 * n * V + 3.0 * n * nzg);
        RET(gemm(c, f2));
      }
    }
    if (nch == 2) {
      // spin s -> (group, row offset inside the group)
      double* Us[2]; double* Rs[2]; long lus[2], lrs[2];
      for (int s = 0; s < 2; ++s) {
        const int q = (ngr == 1) ? 0 : s;
        const int off = (ngr == 1) ? s : 0;
        Us[s] = Ug[q] + (long)off * nz * O; lus[s] = ldU[q];
        Rs[s] = gga ? Rg[q] + (long)off * nz * 3 : nullptr; lrs[s] = ldR[q];
      }
      if (mgga) {
        double* Ts[2];
        for (int s = 0; s < 2; ++s) Ts[s] = c->taubuf.p + (Us[s] - c->ubuf.p);   // same layout as U
        xc_uks_mgga(c->st, 2, n, g0, ng, nz, O, nmo, compP, c->Phi.p + c->occ_basis[0] * basP,
                    c->Phi.p + c->occ_basis[1] * basP, c->kern.p, Us[0], lus[0], Us[1], lus[1], Ts[0], Ts[1],
                    (long)nch * nz * O * n, Rs[0], lrs[0], Rs[1], lrs[1]);
      } else {
        xc_uks_w(c->st, 2, nc, n, g0, ng, nz, O, nmo, compP,
                 c->Phi.p + c->occ_basis[0] * basP, c->Phi.p + c->occ_basis[1] * basP,
                 c->kern.p, Us[0], lus[0], Us[1], lus[1], Rs[0], lrs[0], Rs[1], lrs[1]);
      }
    } else if (mgga) {   // one spin-flip channel, multicollinear (rho, grad rho, tau) kernel
      xc_uks_mgga(c->st, 1, n, g0, ng, nz, O, nmo, compP, c->Phi.p + c->occ_basis[0] * basP, nullptr, c->kern.p,
                  Ug[0], ldU[0], nullptr, 0, c->taubuf.p, nullptr, (long)nz * O * n, Rg[0], ldR[0], nullptr, 0);
    } else if (gga) {    // one spin-flip channel, multicollinear (rho, grad rho) kernel
      xc_uks_w(c->st, 1, nc, n, g0, ng, nz, O, nmo, compP, c->Phi.p + c->occ_basis[0] * basP, nullptr, c->kern.p,
               Ug[0], ldU[0], nullptr, 0, Rg[0], ldR[0], nullptr, 0);
    } else {             // ALDA0, or the multicollinear LDA kernel (2 w f_ss: scalar)
      xc_sf(c->st, n, g0, nz, O, nmo, c->Phi.p + c->occ_basis[0] * basP, c->kern.p, Ug[0]);
    }
    for (int q = 0; q < ngr; ++q) {
      const int nzg = gr[q].nch * nz;
      const double* PV = c->Phi.p + gr[q].vb * basP + (long)g0 * nmo + c->v0;
      const double* PO = c->Phi.p + gr[q].ob * basP + (long)g0 * nmo;
      GemmDesc b1;   // acc[(x,i)][a] += sum_g L[g][(x,i)] PhiV0[g][a]
      b1.M = nzg * O; b1.N = V; b1.K = n;
      b1.A = Ug[q]; b1.sAm = 1; b1.sAk = ldU[q];
      b1.B = PV; b1.sBk = nmo; b1.sBn = 1;
      b1.C = c->acc.p + gr[q].ch0 * chs; b1.ldc = V; b1.beta = 1.0;
      b1.tag = 3;
      RET(gemm(c, b1));
      if (mgga) {
        const long tcs = (long)nch * nz * O * n;
        for (int cc = 1; cc < 4; ++cc) {   // acc[(x,i)][a] += sum_g (1/2 wv_tau dPhiO_c)[g][(x,i)] dPhiV_c[g][a]
          GemmDesc bt = b1;
          bt.A = c->taubuf.p + (cc - 1) * tcs + (long)gr[q].ch0 * nz * O * n;
          bt.B = PV + cc * compP;
          RET(gemm(c, bt));
        }
      }
      if (gga) {
        if (O <= 128 && c->m_kernel) {
          // dedicated kernel (xt_xcm.hip); tag 5 timing around it and its reduce
          bool prof = false;
          // flops: the PhiO^T M GEMM (2 O per M element) + generating M = sum_c wv_c
          // dPhiV_c (3 FMAs per M element)
          RET(prof_begin(c, 5, 2.0 * (O + 3) * (double)nzg * V * n,
                         8.0 * ((double)n * O + 3.0 * n * V + 3.0 * n * nzg + 2.0 * O * (double)nzg * V), &prof));
          const size_t need = xc_back_m_workspace_bytes(O, nzg, V, n);
          if (c->ws.n * sizeof(double) < need) RET(c->ws.ensure(need / sizeof(double) + 1));
          const int r = xc_back_m(O, nzg, V, n, PO, nmo, PV + compP, compP, nmo, Rg[q], ldR[q],
                                  c->accT.p + gr[q].ch0 * chs, (long)nzg * V, c->ws.p, c->ws.n * sizeof(double),
                                  c->st);
          if (r) return fail(r, "xc_back_m launch failed");
          RET(prof_end(c, 5, prof));
          continue;
        }
        GemmDesc b2;   // accT[i][(xg,a)] += sum_g PhiO0[g][i] sum_c wv_c[g][xg] dPhiV_c[g][a]
        b2.M = O; b2.N = xc_m_cols(nzg, V, xc_m_bn()); b2.K = n;
        b2.A = PO; b2.sAm = 1; b2.sAk = nmo;
        b2.fz.mode = 2; b2.fz.V = V; b2.fz.nx = nzg; b2.fz.mbn = xc_m_bn();
        b2.fz.w = PV + compP; b2.fz.wc = compP; b2.fz.wg = nmo;
        b2.fz.rho = Rg[q]; b2.fz.rg = ldR[q];
        b2.C = c->accT.p + gr[q].ch0 * chs; b2.ldc = (long)nzg * V; b2.beta = 1.0;
        b2.tag = 5;
        b2.flops = 2.0 * (O + 3) * (double)nzg * V * n;   // GEMM + generated operand
        // PhiO0, dPhiV_{x,y,z}, wv in; accT read + written
        b2.bytes = 8.0 * ((double)n * O + 3.0 * n * V + 3.0 * n * nzg + 2.0 * O * (double)nzg * V);
        RET(gemm(c, b2));
      }
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// XSF spin-adaptation Delta-A (XSF_TDA.py:1175-1274), ROKS only
// full-space blocks: rows [0,nc) core / [nc,O) open ; cols [0,no) open / [no,V) virtual
// ---------------------------------------------------------------------------
static int xsf_delta_a(xt_ctx* c, int nz, bool skip_k) {
  const xt_desc& d = c->d;
  const int nc = d.nc, no = d.no, nv = d.nv, O = c->O, V = c->V, nmo = d.nmo;
  const long ld = V, sv = (long)O * V, mm = (long)nmo * nmo;
  const double si = no / 2.0;
  const double fg = d.fglobal, foo = d.foo;
  const double f1 = sqrt((2 * si + 1) / (2 * si)) - 1;
  const double f2 = sqrt((2 * si + 1) / (2 * si - 1));
  const double f3 = sqrt((2 * si) / (2 * si - 1)) - 1;
  const double f4 = 1 / sqrt(2 * si * (2 * si - 1));
  const double tsm1 = 2 * si - 1;
  const double* Z = c->ze.p;
  double* S = c->acc.p;
  // block pointers in the full space
  const double* Zcv = Z + no;            double* Scv = S + no;
  const double* Zco = Z;                 double* Sco = S;
  const double* Zov = Z + nc * ld + no;  double* Sov = S + nc * ld + no;
  const double* Zoo = Z + nc * ld;       double* Soo = S + nc * ld;
  const double* FAh = c->F.p + 2 * mm;
  const double* FBh = c->F.p + 3 * mm;
  const double* FS = c->F.p + 4 * mm;
  // MO offsets
  const int mc = 0, mo_ = nc, mv = nc + no;
  const bool loc = d.add_local != 0;
  if (loc) {
    // SA >= 1 one-electron parts
    RET(right_mo(c, nz, nc, nv, nv, Zcv, ld, sv, FS + (long)mv * nmo + mv, nmo, 1, Scv, ld, sv, fg / si));
    RET(left_mo(c, nz, nc, nc, nv, FS + (long)mc * nmo + mc, 1, nmo, Zcv, ld, sv, Scv, ld, sv, fg / si));
    RET(left_mo(c, nz, nc, nc, no, FS, 1, nmo, Zco, ld, sv, Sco, ld, sv, fg * 2.0 / tsm1));
    RET(right_mo(c, nz, no, nv, nv, Zov, ld, sv, FS + (long)mv * nmo + mv, nmo, 1, Sov, ld, sv, fg * 2.0 / tsm1));
  }
  const double* B = bmo_of(c, c->Bmo, 0);
  // J parts: gamma_co, gamma_ov
  RET(c->gam.ensure((size_t)nz * naux_w(c) + 1));
  RET(c->gam2.ensure((size_t)nz * naux_w(c) + 1));
  RET(coulomb_gamma(c, B, nz, mc, nc, mo_, no, Zco, ld, sv, c->gam.p, 0.0));
  RET(coulomb_gamma(c, B, nz, mo_, no, mv, nv, Zov, ld, sv, c->gam2.p, 0.0));
  RET(coulomb_project(c, B, nz, mc, nc, mo_, no, c->gam.p, Sco, ld, sv, -fg / tsm1));
  RET(coulomb_project(c, B, nz, mo_, no, mv, nv, c->gam2.p, Sov, ld, sv, -fg / tsm1));
  if (d.sa > 1) {
    RET(coulomb_project(c, B, nz, mc, nc, mo_, no, c->gam2.p, Sco, ld, sv, fg / tsm1));   // co_ov_j
    RET(coulomb_project(c, B, nz, mo_, no, mv, nv, c->gam.p, Sov, ld, sv, fg / tsm1));   // ov_co_j
    if (loc) {
      // fB_vo = FBh[mv+a][mo_+v] ; fA_oc = FAh[mo_+v][mc+i]
      RET(right_mo(c, nz, nc, no, nv, Zco, ld, sv, FBh + (long)mv * nmo + mo_, 1, nmo, Scv, ld, sv, fg * f1));
      RET(right_mo(c, nz, nc, nv, no, Zcv, ld, sv, FBh + (long)mv * nmo + mo_, nmo, 1, Sco, ld, sv, fg * f1));
      RET(left_mo(c, nz, nc, no, nv, FAh + (long)mo_ * nmo + mc, 1, nmo, Zov, ld, sv, Scv, ld, sv, -fg * f1));
      RET(left_mo(c, nz, no, nc, nv, FAh + (long)mo_ * nmo + mc, nmo, 1, Zcv, ld, sv, Sov, ld, sv, -fg * f1));
    }
    // K parts: S_Y += coef * sum_P B[rowsY,rowsX] Z_X B[colsX,colsY]
    // (skip_k: applied through the stored exchange matrix, exchange_stored_xsf)
    // blocks: cv (rows mc:nc, cols mv:nv) co (mc:nc, mo_:no) ov (mo_:no, mv:nv) oo (mo_:no, mo_:no)
    if (!skip_k) {
    RET(sandwich(c, B, B, nz, mc, nc, mc, nc, mo_, no, mv, nv, Zco, ld, sv, Scv, ld, sv, -fg * f1));   // cv_co_k
    RET(sandwich(c, B, B, nz, mc, nc, mc, nc, mv, nv, mo_, no, Zcv, ld, sv, Sco, ld, sv, -fg * f1));   // co_cv_k
    RET(sandwich(c, B, B, nz, mc, nc, mo_, no, mv, nv, mv, nv, Zov, ld, sv, Scv, ld, sv, -fg * f1));   // cv_ov_k
    RET(sandwich(c, B, B, nz, mo_, no, mc, nc, mv, nv, mv, nv, Zcv, ld, sv, Sov, ld, sv, -fg * f1));   // ov_cv_k
    RET(sandwich(c, B, B, nz, mc, nc, mo_, no, mv, nv, mo_, no, Zov, ld, sv, Sco, ld, sv, -fg / tsm1)); // co_ov_k
    RET(sandwich(c, B, B, nz, mo_, no, mc, nc, mo_, no, mv, nv, Zco, ld, sv, Sov, ld, sv, -fg / tsm1)); // ov_co_k
    }
  }
  if (d.sa > 2) {
    const double ff = fg * foo;
    if (!skip_k) {
    RET(sandwich(c, B, B, nz, mc, nc, mo_, no, mo_, no, mv, nv, Zoo, ld, sv, Scv, ld, sv, -ff * (f2 - 1)));  // cv_oo_k
    RET(sandwich(c, B, B, nz, mo_, no, mc, nc, mv, nv, mo_, no, Zcv, ld, sv, Soo, ld, sv, -ff * (f2 - 1)));  // oo_cv_k
    RET(sandwich(c, B, B, nz, mc, nc, mo_, no, mo_, no, mo_, no, Zoo, ld, sv, Sco, ld, sv, -ff * f3));       // co_oo_k
    RET(sandwich(c, B, B, nz, mo_, no, mc, nc, mo_, no, mo_, no, Zco, ld, sv, Soo, ld, sv, -ff * f3));       // oo_co_k
    RET(sandwich(c, B, B, nz, mc + nc, no, mo_, no, mo_, no, mv, nv, Zoo, ld, sv, Sov, ld, sv, -ff * f3));   // ov_oo_k
    RET(sandwich(c, B, B, nz, mo_, no, mo_, no, mv, nv, mo_, no, Zov, ld, sv, Soo, ld, sv, -ff * f3));       // oo_ov_k
    }
    if (loc) {
      // fA_co = FAh[mc+i][mo_+w] ; fB_vo = FBh[mv+a][mo_+v]
      RET(left_mo(c, nz, nc, no, no, FAh + (long)mc * nmo + mo_, nmo, 1, Zoo, ld, sv, Sco, ld, sv, -ff * f3));
      RET(left_mo(c, nz, no, nc, no, FAh + (long)mc * nmo + mo_, 1, nmo, Zco, ld, sv, Soo, ld, sv, -ff * f3));
      RET(right_mo(c, nz, no, no, nv, Zoo, ld, sv, FBh + (long)mv * nmo + mo_, 1, nmo, Sov, ld, sv, ff * f3));
      RET(right_mo(c, nz, no, nv, no, Zov, ld, sv, FBh + (long)mv * nmo + mo_, nmo, 1, Soo, ld, sv, ff * f3));
      // trace / rank-one terms (XSF_TDA.py:1237-1269: 'xvv', 'vw,..' contractions)
      xsf_rank1(c->st, nz, nc, no, nv, nmo, ff * (f2 / si), ff * f4, Z, FS, FAh, FBh, S);
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// the hot path
// ---------------------------------------------------------------------------
extern "C" int xt_apply(xt_ctx* c, int nz, const double* z, double* sigma, int ptr_kind) {
  if (!c || !z || !sigma) return fail(XT_ERR_ARG, "null argument");
  if (nz <= 0) return 0;
  const xt_desc& d = c->d;
  if (!c->has_orb) return fail(XT_ERR_STATE, "orbitals not set");
  if (!c->has_df && (d.naux > 0)) return fail(XT_ERR_STATE, "DF factor not set");
  if (d.omega != 0.0 && c->ck_lr != 0.0 && !c->has_lr && d.naux > 0)
    return fail(XT_ERR_STATE, "range-separated exchange needs the long-range DF factor");
  if (d.xctype != XT_XC_NONE && d.ngrid > 0 && !c->has_grid) return fail(XT_ERR_STATE, "grid not set");
  const bool xsf = d.kind == XT_KIND_XSF;
  const bool sf = d.kind == XT_KIND_SF_DOWN || d.kind == XT_KIND_SF_UP || xsf;
  if (d.add_local && d.kind != XT_KIND_UTDA && !c->has_fock) return fail(XT_ERR_STATE, "Fock matrices not set");
  if (d.add_local && d.kind == XT_KIND_UTDA && !c->has_eps) return fail(XT_ERR_STATE, "orbital energies not set");
  if (xsf && d.remove && !c->has_vects) return fail(XT_ERR_STATE, "OO basis not set");
  (void)hipSetDevice(d.device);
  const int O = c->O, V = c->V, nmo = d.nmo, nch = c->nchan;
  const long chs = (long)nz * O * V;
  const long mm = (long)nmo * nmo;
  const int dim = dim_of(d);

  const double* zd = z;
  double* sd = sigma;
  if (ptr_kind == XT_PTR_HOST) {
    RET(c->zin.ensure((size_t)nz * dim));
    RET(c->sout.ensure((size_t)nz * dim));
    HIPCHK(hipMemcpyAsync(c->zin.p, z, (size_t)nz * dim * 8, hipMemcpyHostToDevice, c->st));
    zd = c->zin.p; sd = c->sout.p;
  }
  RET(c->ze.ensure(nch * chs));
  RET(c->acc.ensure(nch * chs));
  c->pev_used = 0;
  for (int t = 0; t < 6; ++t) { c->prof_flops[t] = 0.0; c->prof_bytes[t] = 0.0; c->prof_ms[t] = 0.0; c->prof_launches[t] = 0; }
  HIPCHK(hipEventRecord(c->ev[0], c->st));
  // ---- embed trial vectors -------------------------------------------------
  if (d.kind == XT_KIND_XTDA || d.kind == XT_KIND_UTDA) embed_xtda(c->st, nz, d.nc, d.no, d.nv, zd, c->ze.p);
  else if (xsf) xsf_assemble(c->st, nz, d.nc, d.no, d.nv, d.remove, c->vects.p, zd, c->ze.p);
  else HIPCHK(hipMemcpyAsync(c->ze.p, zd, chs * 8, hipMemcpyDeviceToDevice, c->st));
  HIPCHK(hipMemsetAsync(c->acc.p, 0, nch * chs * 8, c->st));
  // Zp gets zeroed slack: the fused rho-forward kernels read whole a-tiles (up to 31
  // columns past the last channel's V, weighted by zero) and whole 8-row occupied
  // blocks (up to 7 rows of nch nz V past O, multiplied by zero PhiO rows)
  const long zslack = 8L * nch * nz * V + 64;
  RET(c->zp.ensure(nch * chs + zslack));
  HIPCHK(hipMemsetAsync(c->zp.p + nch * chs, 0, zslack * 8, c->st));
  RET(c->accT.ensure(nch * chs));
  HIPCHK(hipMemsetAsync(c->accT.p, 0, nch * chs * 8, c->st));
  Group grp[2];
  const int ngrp = channel_groups(c, grp);
  for (int q = 0; q < ngrp; ++q)   // Zp_g (O, nzg, V) = permuted Ze_g
    permute_xi(c->st, grp[q].nch * nz, O, V, c->ze.p + grp[q].ch0 * chs, c->zp.p + grp[q].ch0 * chs);

  // ---- one-electron terms (rank-local) --------------------------------------
  if (d.add_local) {
    if (d.kind == XT_KIND_UTDA) {
      ediag(c->st, nz, O, V, nmo, c->v0, c->eps.p, c->ze.p, c->acc.p);
    } else {
      for (int ch = 0; ch < nch; ++ch) {
        // channel Fock matrices: XTDA alpha/beta ; SF-down/XSF vir=FB occ=FA ; SF-up vir=FA occ=FB
        const double* Fv; const double* Fo;
        if (d.kind == XT_KIND_XTDA) { Fv = Fo = c->F.p + ch * mm; }
        else if (d.kind == XT_KIND_SF_UP) { Fv = c->F.p; Fo = c->F.p + mm; }
        else { Fv = c->F.p + mm; Fo = c->F.p; }
        RET(right_mo(c, nz, O, V, V, c->ze.p + ch * chs, V, (long)O * V, Fv + (long)c->v0 * nmo + c->v0,
                     nmo, 1, c->acc.p + ch * chs, V, (long)O * V, 1.0));
        RET(left_mo(c, nz, O, O, V, Fo, nmo, 1, c->ze.p + ch * chs, V, (long)O * V,
                    c->acc.p + ch * chs, V, (long)O * V, -1.0));
      }
      if (d.kind == XT_KIND_XTDA) {
        // spin-adaptation Delta-A on the CV blocks (XTDA.py:636-684)
        const double si = d.si;
        const double cp = 0.5 * (1 - sqrt((si + 1) / si) + 1 / (2 * si));
        const double cm = 0.5 * (-1 + sqrt((si + 1) / si) + 1 / (2 * si));
        const double cx = 0.5 / (2 * si);
        const int nc = d.nc, no = d.no, nv = d.nv;
        const double* dF = c->F.p + 5 * mm;           // fb_hf - fa_hf
        const double* dv = dF + (long)(nc + no) * nmo + (nc + no);
        const double* dov = dF;                       // core-core block
        const long sv = (long)O * V;
        for (int src = 0; src < 2; ++src) {
          const double* Zs = c->ze.p + src * chs + no;      // CV block of channel src
          for (int dst = 0; dst < 2; ++dst) {
            double* Sd = c->acc.p + dst * chs + no;
            double av, ao;
            if (src == dst) { av = (dst == 0) ? cp : cm; ao = (dst == 0) ? cm : cp; }
            else { av = -cx; ao = -cx; }
            RET(right_mo(c, nz, nc, nv, nv, Zs, V, sv, dv, nmo, 1, Sd, V, sv, av));
            RET(left_mo(c, nz, nc, nc, nv, dov, nmo, 1, Zs, V, sv, Sd, V, sv, ao));
          }
        }
      }
    }
  }
  HIPCHK(hipEventRecord(c->ev[1], c->st));

  // ---- Coulomb / exchange ----------------------------------------------------
  const bool has_k = (c->ck != 0.0 || c->ck_lr != 0.0);
  bool xsf_k_done = false;   // Delta-A exchange already applied through the stored matrix
  if (d.naux > 0) {
    if (!sf && naux_w(c) > 0) {   // J (spin-conserving only)
      RET(c->gam.ensure((size_t)nz * naux_w(c)));
      for (int ch = 0; ch < nch; ++ch)
        RET(coulomb_gamma(c, bmo_of(c, c->Bmo, c->occ_basis[ch]), nz, 0, O, c->v0, V,
                          c->ze.p + ch * chs, V, (long)O * V, c->gam.p, ch == 0 ? 0.0 : 1.0));
      for (int ch = 0; ch < nch; ++ch)
        RET(coulomb_project(c, bmo_of(c, c->Bmo, c->occ_basis[ch]), nz, 0, O, c->v0, V, c->gam.p,
                            c->acc.p + ch * chs, V, (long)O * V, 1.0));
    }
    if (has_k) {
      RET(resolve_kmode(c));
      if (c->k_resolved == 1) {
        if (!c->kx_valid) RET(build_kx(c));
        if (xsf_fused_k(c)) {
          RET(exchange_stored_xsf(c, nz));
          xsf_k_done = true;
        } else {
          RET(exchange_stored(c, nz));
        }
      } else {
        RET(exchange_main(c, nz, c->Bmo, -c->ck));
        if (c->ck_lr != 0.0) RET(exchange_main(c, nz, c->Bmo_lr, -c->ck_lr));
      }
    }
    if (xsf && d.sa > 0 && naux_w(c) > 0) RET(xsf_delta_a(c, nz, xsf_k_done));
  }
  HIPCHK(hipEventRecord(c->ev[2], c->st));

  // ---- XC ----------------------------------------------------------------------
  if (d.xctype != XT_XC_NONE && d.ngrid > 0) RET(xc_response(c, nz));
  for (int q = 0; q < ngrp; ++q)   // acc_g += accT_g (left-contraction results)
    permute_add(c->st, grp[q].nch * nz, O, V, 1.0, c->accT.p + grp[q].ch0 * chs, c->acc.p + grp[q].ch0 * chs);
  HIPCHK(hipEventRecord(c->ev[3], c->st));

  // ---- extract -----------------------------------------------------------------
  if (d.kind == XT_KIND_XTDA || d.kind == XT_KIND_UTDA) extract_xtda(c->st, nz, d.nc, d.no, d.nv, c->acc.p, nullptr, sd);
  else if (xsf) xsf_extract(c->st, nz, d.nc, d.no, d.nv, d.remove, c->vects.p, c->acc.p, sd);
  else HIPCHK(hipMemcpyAsync(sd, c->acc.p, chs * 8, hipMemcpyDeviceToDevice, c->st));
  HIPCHK(hipEventRecord(c->ev[4], c->st));
  if (ptr_kind == XT_PTR_HOST)
    HIPCHK(hipMemcpyAsync(sigma, c->sout.p, (size_t)nz * dim * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipEventSynchronize(c->ev[4]));
  float t01, t12, t23, t04;
  (void)hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  (void)hipEventElapsedTime(&t12, c->ev[1], c->ev[2]);
  (void)hipEventElapsedTime(&t23, c->ev[2], c->ev[3]);
  (void)hipEventElapsedTime(&t04, c->ev[0], c->ev[4]);
  c->timings[0] = t12; c->timings[1] = t23; c->timings[2] = t01; c->timings[3] = t04;
  for (int i = 0; i < c->pev_used; i += 2) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->pev[i], c->pev[i + 1]);
    c->prof_ms[c->pev_tag[i]] += ms;
  }
  if (ptr_kind == XT_PTR_HOST) HIPCHK(hipStreamSynchronize(c->st));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(XT_ERR_HIP, std::string("kernel error: ") + hipGetErrorString(e));
  return 0;
}

extern "C" int xt_xsf_j_diagonals(xt_ctx* c, double* co_j, double* ov_j, int ptr_kind) {
  if (!c || !co_j || !ov_j) return fail(XT_ERR_ARG, "null argument");
  if (!c->has_df) return fail(XT_ERR_STATE, "DF factor not set");
  (void)hipSetDevice(c->d.device);
  const int nc = c->d.nc, no = c->d.no, nv = c->d.nv;
  RET(c->trace.ensure((size_t)nc * no + (size_t)no * nv));
  // over this context's aux window (xt_set_partition): partial sums over ranks add up
  xsf_jdiag(c->st, naux_w(c), c->d.nmo, nc, no, nv, bmo_of(c, c->Bmo, 0), c->trace.p, c->trace.p + (size_t)nc * no);
  const hipMemcpyKind k = ptr_kind == XT_PTR_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  HIPCHK(hipMemcpyAsync(co_j, c->trace.p, (size_t)nc * no * 8, k, c->st));
  HIPCHK(hipMemcpyAsync(ov_j, c->trace.p + (size_t)nc * no, (size_t)no * nv * 8, k, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return 0;
}

// ---------------------------------------------------------------------------
// device linear algebra for the Davidson solver
// ---------------------------------------------------------------------------
static int run_desc(const GemmDesc& g, void* stream);

extern "C" int xt_dgemm(int transa, int transb, int m, int n, int k, double alpha,
                        const double* a, long lda, const double* b, long ldb, double beta,
                        double* cc, long ldc, void* stream) {
  GemmDesc g;
  g.M = m; g.N = n; g.K = k;
  g.A = a; if (transa) { g.sAm = 1; g.sAk = lda; } else { g.sAm = lda; g.sAk = 1; }
  g.B = b; if (transb) { g.sBk = 1; g.sBn = ldb; } else { g.sBk = ldb; g.sBn = 1; }
  g.C = cc; g.ldc = ldc; g.alpha = alpha; g.beta = beta;
  return run_desc(g, stream);
}

extern "C" int xt_dgemm_strided(int m, int n, int k, int r, int nbatch, double alpha,
                                const double* a, long sAm, long sAk, long sAr, long sAb,
                                const double* b, long sBk, long sBn, long sBr, long sBb, double beta,
                                double* cc, long ldc, long sCb, void* stream) {
  if (m < 0 || n < 0 || k < 0 || r < 1 || nbatch < 1) return fail(XT_ERR_ARG, "xt_dgemm_strided: bad sizes");
  if (sAm != 1 && sAk != 1) return fail(XT_ERR_ARG, "xt_dgemm_strided: A needs a unit m or k stride");
  if (sBn != 1 && sBk != 1) return fail(XT_ERR_ARG, "xt_dgemm_strided: B needs a unit k or n stride");
  if (sAm < 0 || sAk < 0 || sAr < 0 || sAb < 0 || sBk < 0 || sBn < 0 || sBr < 0 || sBb < 0 || sCb < 0)
    return fail(XT_ERR_ARG, "xt_dgemm_strided: negative stride");
  if (ldc < n) return fail(XT_ERR_ARG, "xt_dgemm_strided: ldc < n");
  if ((long)m * n > 0 && (!cc || (k > 0 && (!a || !b))))
    return fail(XT_ERR_ARG, "xt_dgemm_strided: null operand");
  GemmDesc g;
  g.M = m; g.N = n; g.K = k; g.R = r; g.nb1 = nbatch;
  g.A = a; g.sAm = sAm; g.sAk = sAk; g.sAr = sAr; g.sAb1 = sAb;
  g.B = b; g.sBk = sBk; g.sBn = sBn; g.sBr = sBr; g.sBb1 = sBb;
  g.C = cc; g.ldc = ldc; g.sCb1 = sCb; g.alpha = alpha; g.beta = beta;
  return run_desc(g, stream);
}

static int run_desc(const GemmDesc& g, void* stream) {
  // split-K workspace per HIP device (the caller's current device owns the
  // stream and the operands)
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  static thread_local std::vector<DevBuf> ws_dev;
  if ((int)ws_dev.size() <= dev) ws_dev.resize(dev + 1);
  DevBuf& ws = ws_dev[dev];
  size_t need = dgemm_workspace_bytes(g);
  if (need > 0) {
    size_t cap = (size_t)256 << 20;
    RET(ws.ensure((need < cap ? need : cap) / 8 + 1));
  }
  int r = dgemm(g, (hipStream_t)stream, ws.p, ws.n * 8);
  if (r) return fail(r, "dgemm launch failed");
  return 0;
}

extern "C" int xt_precond(int nrow, int dim, const double* diag, const double* e, double shift,
                          const double* r, double* out, void* stream) {
  precond((hipStream_t)stream, nrow, dim, diag, e, shift, r, out);
  return hipGetLastError() == hipSuccess ? 0 : fail(XT_ERR_HIP, "precond launch failed");
}
extern "C" int xt_row_norms2(int nrow, int dim, const double* x, double* out, void* stream) {
  row_norms2((hipStream_t)stream, nrow, dim, x, out);
  return hipGetLastError() == hipSuccess ? 0 : fail(XT_ERR_HIP, "row_norms2 launch failed");
}
extern "C" int xt_row_scale(int nrow, int dim, double* x, const double* s, void* stream) {
  row_scale((hipStream_t)stream, nrow, dim, x, s);
  return hipGetLastError() == hipSuccess ? 0 : fail(XT_ERR_HIP, "row_scale launch failed");
}

extern "C" int xt_int3c2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab,
                               int naux_shells, const int* aux_info, const double* aux_prim, const double* ek,
                               int lmax_orb, int lmax_aux, double omega, double* out, long ldo,
                               void* stream) {
  return xt_int2e_cart(npair, pair_info, pair_prim, eab, naux_shells, aux_info, aux_prim, ek, lmax_orb, lmax_aux,
                       omega, nullptr, nullptr, 0.0, 0, out, ldo, stream);
}

extern "C" int xt_int2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab,
                             int nket, const int* ket_info, const double* ket_prim, const double* ek,
                             int lmax_orb, int lket, double omega, const double* q_bra, const double* q_ket,
                             double q_thr, int diag, double* out, long ldo, void* stream) {
  if (npair < 0 || nket < 0 || ldo < 0) return fail(XT_ERR_ARG, "xt_int2e_cart: negative size");
  if (lmax_orb < 0 || lket < 0 || lmax_orb > kIntMaxLOrb || 2 * lmax_orb + lket > kIntMaxL)
    return fail(XT_ERR_ARG, "xt_int2e_cart: orbital shells up to f and 2 l_orb + l_ket <= 13");
  if (omega < 0.0) return fail(XT_ERR_ARG, "xt_int2e_cart: omega < 0");
  if ((q_bra == nullptr) != (q_ket == nullptr)) return fail(XT_ERR_ARG, "xt_int2e_cart: give both bounds or none");
  if (diag && nket != npair) return fail(XT_ERR_ARG, "xt_int2e_cart: diag needs the ket table = the bra table");
  const int r = int2e_cart(npair, pair_info, pair_prim, eab, nket, ket_info, ket_prim, ek, lmax_orb, lket, omega,
                           q_bra, q_ket, q_thr, diag, out, ldo, (hipStream_t)stream);
  return r ? fail(r, "int2e launch failed") : 0;
}

extern "C" int xt_eval_ao(int ngrid, const double* coords, int nshell, const int* shell_info,
                          const double* shell_data, const double* sph, const double* ao_norm, int deriv,
                          double* out, long ldo, long comp_stride, void* stream) {
  if (ngrid < 0 || nshell < 0 || ldo < 0 || comp_stride < 0) return fail(XT_ERR_ARG, "xt_eval_ao: negative size");
  if (deriv != 0 && deriv != 1) return fail(XT_ERR_ARG, "xt_eval_ao: deriv must be 0 or 1");
  const int r = eval_ao(ngrid, coords, nshell, shell_info, shell_data, sph, ao_norm, deriv, out, ldo, comp_stride,
                        (hipStream_t)stream);
  return r ? fail(r, "eval_ao launch failed") : 0;
}
