#pragma once
#include <hip/hip_runtime.h>

namespace xt {
void embed_xtda(hipStream_t st, int nz, int nc, int no, int nv, const double* z, double* ze);
void extract_xtda(hipStream_t st, int nz, int nc, int no, int nv, const double* acc, const double* kx, double* out);
void extract_one(hipStream_t st, int nz, int O, int V, const double* acc, const double* kx, double* out);
void permute_xi(hipStream_t st, int nz, int O, int V, const double* src, double* dst);
void permute_add(hipStream_t st, int nz, int O, int V, double alpha, const double* src, double* dst);
void permute_add_strided(hipStream_t st, int nz, int nry, int ncy, double alpha, const double* src,
                         double* dst, long ldS, long svS);
void xsf_rank1(hipStream_t st, int nz, int nc, int no, int nv, int nmo, double a2, double a4,
               const double* ze, const double* fs, const double* fa, const double* fb, double* acc);
void ediag(hipStream_t st, int nz, int O, int V, int nmo, int v0, const double* eps, const double* ze, double* acc);
void xc_uks(hipStream_t st, int ncomp, int G, int g0, int ngrid, int nz, int O, int nmo,
            const double* phi0, const double* phi1, const double* wfxc, double* U);
// ns = 2: both spin channels of the UKS response (kernel (2, nk, 2, nk, ngrid)); ns = 1: one
// spin-flip channel with the multicollinear kernel (nk, nk, ngrid); U1 / R1 / pO1 unused
void xc_uks_w(hipStream_t st, int ns, int ncomp, int G, int g0, int ngrid, int nz, int O, int nmo, long compP,
              const double* pO0, const double* pO1, const double* wfxc, double* U0, long ldU0,
              double* U1, long ldU1, double* R0, long ldR0, double* R1, long ldR1);
void xc_sf(hipStream_t st, int G, int g0, int nz, int O, int nmo, const double* phio, const double* fsf, double* U);
void weight_fxc(hipStream_t st, long n4, int ngrid, double scale, const double* w, double* f);
// meta-GGA point kernel: GGA terms + tau (T_s[c] planes tcs apart, same leading dims as U)
void xc_uks_mgga(hipStream_t st, int ns, int G, int g0, int ngrid, int nz, int O, int nmo, long compP,
                 const double* pO0, const double* pO1, const double* wfxc, double* U0, long ldU0, double* U1,
                 long ldU1, double* T0, double* T1, long tcs, double* R0, long ldR0, double* R1, long ldR1);
void xsf_assemble(hipStream_t st, int nz, int nc, int no, int nv, int remove, const double* vects, const double* z, double* ze);
// XSF exchange through the stored matrix: the trial vectors split into their four
// spin-adaptation source blocks (cv, co, ov, oo), and the per-block results combined
// with a 4 x 4 weight table w16[source][target]
void xsf_split4(hipStream_t st, int nz, int O, int V, int nc, int no, const double* ze, double* zb);
struct W16 { double w[16]; };   // w[4 source + target]
void xsf_combine4(hipStream_t st, int nz, int O, int V, int nc, int no, const W16& w16, const double* yb,
                  double* acc);
void xsf_extract(hipStream_t st, int nz, int nc, int no, int nv, int remove, const double* vects, const double* full, double* out);
void xsf_jdiag(hipStream_t st, int naux, int nmo, int nc, int no, int nv, const double* bmo, double* co_j, double* ov_j);
// stored exchange: blocks (i, j), i0 <= j < i0 + fold floor((i - i0) / fold), of K (row (i,a) at
// (i V + a) ld, column (j,b) at j V + b) set to the transposes of blocks (j, i)
void kx_mirror(hipStream_t st, int O, int V, long ld, int i0, int i1, int fold, double* K);
void precond(hipStream_t st, int nrow, int dim, const double* diag, const double* e, double shift, const double* r, double* out);
void row_norms2(hipStream_t st, int nrow, int dim, const double* x, double* out);
void row_scale(hipStream_t st, int nrow, int dim, double* x, const double* s);
// pivoted Cholesky of packed 8-fold ERIs (xt_chol.hip)
void eri_diag(hipStream_t st, long npair, const double* eri, double* d);
void argmax(hipStream_t st, long n, const double* d, double* out2);
void chol_step(hipStream_t st, long npair, int k, long p, double dp, const double* eri, double* Lt, long ldL,
               double* d);
void chol_unpack(hipStream_t st, int np, int p0, int nao, const double* Lt, long ldL, double* B);
}  // namespace xt
