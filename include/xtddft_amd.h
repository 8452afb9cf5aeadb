/* xtddft_amd -- MI355X-native TDA response hot path (C ABI).
 *
 * Drop-in boundary for the Davidson/TDA operator of
 * Quantum-Chemistry-Group-BNU/XTDDFT.  Each entry point names the reference
 * interface it replaces (file:line relative to the reference root).  All
 * arrays are FP64, row-major, caller-owned; setters copy into device memory
 * owned by the context.  `ptr_kind` is XT_PTR_HOST or XT_PTR_DEVICE.
 * Every call returns 0 on success or a negative XT_ERR_* code; the message of
 * the last failure is available from xt_last_error().
 */
#ifndef XTDDFT_AMD_H
#define XTDDFT_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

#define XT_ABI_VERSION 7

#define XT_PTR_HOST 0
#define XT_PTR_DEVICE 1

/* operator kinds */
#define XT_KIND_XTDA 0     /* spin-adapted X-TDA on ROKS        (XTDA.py:558-692, self.X)   */
#define XT_KIND_UTDA 1     /* unrestricted TDA on UKS          (XTDA.py:685-687)            */
#define XT_KIND_SF_DOWN 2  /* spin-flip down  (SF_TDA.py:162-244, isf=-1)                   */
#define XT_KIND_SF_UP 3    /* spin-flip up    (SF_TDA.py:162-244, isf=+1)                   */
#define XT_KIND_XSF 4      /* spin-adapted spin-flip down (XSF_TDA.py:1029-1277)           */

/* exchange-correlation kernel types */
#define XT_XC_NONE 0       /* pure Hartree-Fock response (XTDA.py:546-554)                 */
#define XT_XC_LDA 1
#define XT_XC_GGA 2
#define XT_XC_MGGA 3       /* meta-GGA: (rho, grad rho, tau) kernel, XTDA.py:239-276 / nr_uks_fxc   */

/* spin-flip XC kernels (SF_DOWN / SF_UP / XSF; the reference's `method`) */
#define XT_SF_ALDA0 0      /* method 0: collinear-limit ALDA0, density only (SF_TDA.py:39-160)     */
#define XT_SF_MC 1         /* method 1: multicollinear kernel over (s, grad s[, tau_s])            */
                           /*   (_gen_uhf_tda_response_sf / nr_uks_fxc_sf_tda_mc, SF_TDA.py:855-1047) */

typedef struct xt_ctx xt_ctx;

typedef struct xt_desc {
  int kind;          /* XT_KIND_* */
  int restricted;    /* 1: ROKS (one MO basis), 0: UKS (alpha/beta bases) */
  int nao, nmo;
  int nc, no, nv;    /* closed / open / virtual counts (utils.get_cov, utils.py:6-41) */
  int naux;          /* DF functions held by THIS context (a shard when distributed) */
  int ngrid;         /* grid points held by THIS context */
  int xctype;        /* XT_XC_* */
  double hyb;        /* rsh_and_hybrid_coeff (XTDA.py:501) */
  double alpha;
  double omega;      /* != 0: long-range factor set with xt_set_jk_df(which=1) */
  double si;         /* spin/2 (XTDA.py:613); XSF uses no/2 (XSF_TDA.py:1061) */
  int sa;            /* XSF spin-adaptation level 0..3 (XSF_TDA.py:148-152) */
  double foo, fglobal; /* XSF scale factors (XSF_TDA.py:1501-1518) */
  int remove;        /* XSF: compress the OO block by one vector (XSF_TDA.py:397-414) */
  int add_local;     /* 1: add the rank-local one-electron terms (Fock, Delta-A Fock
                        parts); set on exactly one rank of a sharded operator */
  int device;        /* HIP device ordinal */
  int sf_kernel;     /* spin-flip kinds: XT_SF_ALDA0 or XT_SF_MC (ignored otherwise) */
} xt_desc;

/* lifetime ------------------------------------------------------------- */
int xt_create(const xt_desc* desc, xt_ctx** out);
int xt_destroy(xt_ctx* ctx);
int xt_set_stream(xt_ctx* ctx, void* hip_stream);
const char* xt_last_error(void);
int xt_abi_version(void);
/* SHA-256 prefix of the sources, headers and flags the library was built from
   (xtddft_amd/build.py source_hash); the Python loader refuses a library whose
   id differs from its tree. */
const char* xt_build_id(void);

/* one-time setup (what the reference builds once per solve) ------------ */
/* MO coefficients (nao x nmo); c_beta ignored when restricted.
   Replaces mf.mo_coeff consumption in _gen_tda_operation (XTDA.py:565-586). */
int xt_set_orbitals(xt_ctx* ctx, const double* c_alpha, const double* c_beta, int ptr_kind);
/* KS and pure-HF Fock matrices in the MO basis (nmo x nmo each), or the orbital
   energies for UTDA via xt_set_orbital_energies.
   Replaces mf.get_veff/get_hcore + scf.ROHF(mol).get_veff (XTDA.py:588-613,
   XSF_TDA.py:1070-1114). */
int xt_set_fock_mo(xt_ctx* ctx, const double* fa, const double* fb,
                   const double* fa_hf, const double* fb_hf, int ptr_kind);
int xt_set_orbital_energies(xt_ctx* ctx, const double* e_a, const double* e_b, int ptr_kind);
/* Density-fitting factor B[P,mu,nu] (naux x nao x nao) defining
   (mu nu|la si) = sum_P B B.  which = 0: full-range Coulomb, 1: long-range.
   Replaces mf.get_jk / get_j / get_k (XTDA.py:518-543, SF_TDA.py:273-281,
   XSF_TDA.py:996) -- the AO->MO transform is done once here on the device. */
int xt_set_jk_df(xt_ctx* ctx, const double* cderi, int which, int ptr_kind);
/* Stored 4-index ERIs instead of a DF factor (jk_mode ERI8): PySCF 8-fold
   packed order ('s8', ao2mo.restore(8, ...)): pair index ij = i(i+1)/2 + j
   (i >= j), npair = nao(nao+1)/2, (ij|kl) stored at ij(ij+1)/2 + kl (ij >= kl).
   Factorised on the device by pivoted Cholesky, (mu nu|la si) = sum_P L_P L_P,
   down to a largest residual diagonal <= tol (tol <= 0: 1e-13 x the largest
   diagonal), i.e. exact to that tolerance; the Cholesky vectors then drive the
   same MO-route J/K engine as xt_set_jk_df.  The context keeps the vectors of
   the contiguous block p_rank of p_count (multi-GPU aux sharding; 0, 1 for
   all) and takes that count as its naux (xt_naux); a long-range set (which = 1)
   of a different rank is zero-padded to a common naux.
   Replaces the incore mf._eri consumed by PySCF get_jk / get_k(omega=)
   (XTDA.py:518-543, SF_TDA.py:273-281, XSF_TDA.py:857,996). */
int xt_set_jk_eri8(xt_ctx* ctx, const double* eri_s8, int which, double tol,
                   int p_rank, int p_count, int ptr_kind);
/* DF / Cholesky functions held by this context (desc.naux, or the rank
   found by xt_set_jk_eri8) and the full Cholesky rank of the last
   xt_set_jk_eri8 (before sharding). */
int xt_naux(const xt_ctx* ctx, int* naux_local, int* chol_rank);
/* AO values on the grid (ncomp x ngrid x nao; ncomp = 1 LDA / 4 GGA and MGGA;
   spin-flip ALDA0: 1), weights (ngrid) and the kernel: UKS fxc (2 x nk x 2 x nk x ngrid,
   un-weighted; nk = 1 LDA, 4 GGA, 5 MGGA with tau = 1/2 sum |grad phi|^2 last) for
   XTDA/UTDA; for SF/XSF the weighted ALDA0 kernel (ngrid), or with XT_SF_MC the
   un-weighted multicollinear kernel fxc_sf (nk x nk x ngrid, the output of mcfun's
   eval_xc_eff_sf; the library applies the reference's factor 2 and the weights).
   Replaces ni.cache_xc_kernel / cache_xc_kernel_sf / cache_xc_kernel_sf_mc
   (XTDA.py:504, SF_TDA.py:39-88, 942-974) and the per-call grid loop of ni.nr_uks_fxc /
   nr_uks_fxc_sf_tda / nr_uks_fxc_sf_tda_mc (XTDA.py:514, SF_TDA.py:90-160, 976-1047). */
int xt_set_grid(xt_ctx* ctx, const double* ao, const double* weights,
                const double* kernel, int ptr_kind);
/* XSF only: OO compression basis vects (no^2 x (no^2-1)) (XSF_TDA.py:397-414). */
int xt_set_oo_basis(xt_ctx* ctx, const double* vects, int ptr_kind);

/* exchange evaluation: the K part of get_jk / get_k (XTDA.py:518-543,
   SF_TDA.py:273-281, XSF_TDA.py:996).  XT_K_DIRECT contracts the MO DF factor
   per A.x (cost 2 naux nz O V^2); XT_K_STORED builds once per solve the MO
   exchange matrix Kx[(i,a),(j,b)] = sum_P B_P[i,j] B_P[a,b] (x the hybrid
   coefficients) and keeps it in HBM ((O V)^2 doubles per MO basis), making the
   per-A.x exchange one HBM-streaming GEMM -- PySCF's incore-vs-direct choice
   (mf._eri kept when it fits max_memory).  XT_K_AUTO (default) stores when
   the matrix fits max_gib (<= 0: free HBM minus a reserve).  The XSF Delta-A
   exchange blocks always run direct. */
#define XT_K_AUTO 0
#define XT_K_DIRECT 1
#define XT_K_STORED 2
int xt_set_exchange_mode(xt_ctx* ctx, int mode, double max_gib);
/* Build what is built once per solve (the stored exchange matrix when the
   mode resolves to it; xt_apply would otherwise build it on first use) and
   report the resolved mode and its HBM footprint (GiB).  A partitioned context
   (xt_set_partition with a proper aux window) that stores the exchange then drops
   the MO-factor rows outside its window (every later use reads only the window):
   xt_naux reports the window; re-partitioning or a stored-exchange rebuild needs
   the factor set again. */
int xt_prepare(xt_ctx* ctx, int* k_mode, double* k_gib);
/* What XT_K_AUTO resolves to on this context (*stored = 1 / 0) and the stored
   matrix's footprint (GiB; 0 for an operator without exchange), without building
   anything.  The resolution depends
   on this GPU's free HBM, so the ranks of a partitioned operator must agree
   before they build: a rank that streams its stored ROWS and a rank that
   contracts its aux WINDOW directly do not sum to the operator.  The host side
   takes the minimum over ranks and sets the mode explicitly
   (xtddft_amd/operator.py).  Same fit rule as xt_prepare. */
int xt_exchange_plan(xt_ctx* ctx, int* stored, double* k_gib);

/* Rank partition of a sharded operator (one process per GPU):
   the context keeps the whole MO factor but contracts J, the direct exchange
   and the XSF Delta-A only over aux rows [p0, p1), and stores / applies only
   the exchange rows whose occupied index is in [i0, i1) (superset O index).
   Over ranks with disjoint windows and row blocks the partial sigma sum to
   the full operator.  Defaults: all rows.  Call after the factor is set. */
int xt_set_partition(xt_ctx* ctx, int p0, int p1, int i0, int i1);

/* the hot path --------------------------------------------------------- */
/* sigma = A z for nz trial vectors, row-major (nz x dim) in the reference's
   vector order (PySCF order for XTDA/UTDA/SF; cv|co|ov|oo for XSF, OO
   compressed when remove).  Replaces the vind closures (XTDA.py:615-690,
   SF_TDA.py:224-243, XSF_TDA.py:1131-1276). */
int xt_apply(xt_ctx* ctx, int nz, const double* z, double* sigma, int ptr_kind);
int xt_dim(const xt_ctx* ctx);
/* per-phase device timings of the last xt_apply (ms): jk, xc, local, total */
int xt_last_timings(const xt_ctx* ctx, double* out4);

/* live timing of GEMM classes with HIP events on the context's stream (mask bit t:
   t = 1 exchange contraction (stored or direct), 2 XC forward U, 3 XC back L,
   4 XC forward W (fused rho), 5 XC back M (fused generated operand); 0 = off);
   xt_profile_stats(tag): {device ms summed over the launches of the last xt_apply,
   number of launches, algorithmic flops} */
int xt_set_profile(xt_ctx* ctx, int tag);
int xt_profile_stats(const xt_ctx* ctx, int tag, double* out3);
/* compulsory HBM bytes of class `tag` in the last xt_apply (each operand once) */
int xt_profile_bytes(const xt_ctx* ctx, int tag, double* bytes);

/* XSF preconditioner J diagonals (XSF_TDA.py:859-913): co_j (nc x no), ov_j (no x nv). */
int xt_xsf_j_diagonals(xt_ctx* ctx, double* co_j, double* ov_j, int ptr_kind);

/* device linear algebra used by the Davidson solver (Davidson.py:21-298) ---- */
/* C = alpha * op(A) op(B) + beta * C on device pointers (strided, batched);
   trans flags: 0 = as stored row-major, 1 = transposed. */
int xt_dgemm(int transa, int transb, int m, int n, int k, double alpha,
             const double* a, long lda, const double* b, long ldb, double beta,
             double* c, long ldc, void* hip_stream);
/* C[b] = alpha * sum_r A[b,r] B[b,r] + beta * C[b] with explicit strides: A(m, k) at
   a + b sAb + r sAr + m sAm + k sAk (sAm or sAk = 1), B(k, n) likewise (sBk or sBn = 1),
   C row-major with ldc, batch stride sCb.  The strided, reduce-indexed contraction the
   MO transforms and J/K builds run (lib.einsum over the DF index behind get_jk,
   XTDA.py:518-543); exposed so every engine layout is testable. */
int xt_dgemm_strided(int m, int n, int k, int r, int nbatch, double alpha,
                     const double* a, long sAm, long sAk, long sAr, long sAb,
                     const double* b, long sBk, long sBn, long sBr, long sBb, double beta,
                     double* c, long ldc, long sCb, void* hip_stream);
/* y = (x - e*w) / clamp(d - (e - shift)) row-wise; diag preconditioner
   (XTDA.py:736-744, PySCF make_diag_precond). nrow vectors of length dim. */
int xt_precond(int nrow, int dim, const double* diag, const double* e, double shift,
               const double* r, double* out, void* hip_stream);
/* out[i] = sum_j x[i,j]^2 for nrow rows. */
int xt_row_norms2(int nrow, int dim, const double* x, double* out, void* hip_stream);
/* x[i,:] *= s[i] */
int xt_row_scale(int nrow, int dim, double* x, const double* s, void* hip_stream);

/* mean-field front end ------------------------------ */
/* 3-index Coulomb integrals (ab|c) over contracted Cartesian Gaussians by
   McMurchie-Davidson (replaces libcint int3c2e behind PySCF df.incore.aux_e2,
   the DF factor whose get_jk XTDA.py:518-543 calls and whose MO transform
   stands in for ao2mo.general, XTDA.py:120).  Device pointers, launched on
   `hip_stream`; `out` is accumulated into (zero it first).
     pair_info[8k+0..5]  la, lb, npp, first row of pair_prim, offset in eab, first output row
     pair_prim[4q+0..3]  p, Px, Py, Pz of primitive pair q
     eab                 per pair [a][b][t][q]: Hermite coefficients x contraction coefficients
     aux_info[8j+0..5]   lc, nprim, first row of aux_prim, offset in ek, first output column, nc
     aux_prim[4r+0..3]   exponent, Cx, Cy, Cz
     ek                  per aux shell [c][u][r]: one-centre Hermite coefficients x coefficients
     out[(row0 + a*ncart(lb) + b) * ldo + col0 + c] += (ab|c)
   The ket may be a shell pair (4-index (ab|cd), the stored-ERI path of `jk_mode`
   ERI8 / PySCF mol.intor('int2e')): lc = l_c + l_d, nc = ncart(l_c) ncart(l_d),
   its primitive pairs in aux_prim and its pair Hermite coefficients in ek.
   lmax_orb <= 3 (f), 2 lmax_orb + lmax_aux <= 13 (lmax_aux: the ket's Hermite order).
   omega > 0: the long-range operator erf(omega r12)/r12 (PySCF mol.with_range_coulomb,
   the cderi_lr / eri_lr factors of range-separated hybrids, XTDA.py:501,527-539); 0: 1/r12. */
int xt_int3c2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab,
                    int naux_shells, const int* aux_info, const double* aux_prim, const double* ek,
                    int lmax_orb, int lmax_aux, double omega, double* out, long ldo, void* hip_stream);
/* The same integrals with Schwarz screening and a diagonal mode -- the exact ERIs of
   the direct-SCF mean field (PySCF's default mf, whose get_jk XTDA.py:518-543 calls
   and whose ERIs ao2mo.general transforms, XTDA.py:120) without the 4-index array:
   the integral-direct pivoted Cholesky of xtddft_amd/qc/dchol.py evaluates the
   diagonal (ab|ab) (diag = 1: one block per bra pair with ket = the same table
   entry, nket == npair) and the pivot columns (all pairs | chosen pairs) through it.
   q_bra / q_ket (device, per table entry; both or neither): blocks with
   q_bra[k] q_ket[j] < q_thr are skipped (left zero). */
int xt_int2e_cart(int npair, const int* pair_info, const double* pair_prim, const double* eab,
                  int nket, const int* ket_info, const double* ket_prim, const double* ek,
                  int lmax_orb, int lket, double omega, const double* q_bra, const double* q_ket,
                  double q_thr, int diag, double* out, long ldo, void* hip_stream);
/* AO values (deriv 0) or values and gradients (deriv 1) of normalised spherical
   AOs on grid points (PySCF mol.eval_ao / ni.block_loop, SF_TDA.py:63-68, the AO
   input of cache_xc_kernel / nr_uks_fxc, XTDA.py:504,514), device pointers:
     coords[3g + 0..2]      grid point (Bohr)
     shell_info[8s + 0..3]  l (<= 4), nprim, offset in shell_data, first AO
     shell_data[off ..]     nprim exponents, nprim coefficients (x radial norms), centre
     sph                    solid-harmonic tables of l = 0..4 ((2l+1) x ncart(l) each,
                            concatenated, libcint order)
     ao_norm[ao]            AO normalisation
     out[c * comp_stride + g * ldo + ao], c = value (, d/dx, d/dy, d/dz). */
int xt_eval_ao(int ngrid, const double* coords, int nshell, const int* shell_info,
               const double* shell_data, const double* sph, const double* ao_norm, int deriv,
               double* out, long ldo, long comp_stride, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif
