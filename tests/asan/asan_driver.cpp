// Host-side AddressSanitizer check of the C ABI (include/xtddft_amd.h), built with
// tools/asan_host.sh (every csrc/*.hip with -Xarch_host -fsanitize=address).  Runs on a
// machine without a GPU: it drives the argument validation and error-reporting paths of
// the entry points -- every rejected call must return a negative code and leave a
// readable message in xt_last_error -- under ASan (heap / stack / global overflows,
// use-after-free in the error-string handling and descriptor checks).
#include <cstdio>
#include <cstring>
#include "../../include/xtddft_amd.h"

static int failures = 0;
static void expect_err(int rc, const char* what) {
  const char* msg = xt_last_error();
  if (rc >= 0 || msg == nullptr || std::strlen(msg) == 0) {
    std::printf("FAIL %s: rc %d msg '%s'\n", what, rc, msg ? msg : "(null)");
    ++failures;
  }
}

int main() {
  if (xt_abi_version() <= 0) { std::printf("FAIL abi\n"); return 1; }
  if (!xt_build_id() || std::strlen(xt_build_id()) == 0) { std::printf("FAIL build id\n"); return 1; }
  xt_ctx* h = nullptr;
  expect_err(xt_create(nullptr, &h), "create null desc");
  xt_desc d;
  std::memset(&d, 0, sizeof(d));
  expect_err(xt_create(&d, &h), "create empty desc");
  d.kind = XT_KIND_XTDA; d.restricted = 1; d.nao = 10; d.nmo = 10; d.nc = 3; d.no = 2; d.nv = 4;
  expect_err(xt_create(&d, &h), "create nc+no+nv != nmo");
  d.nv = 5; d.si = 0.0;
  expect_err(xt_create(&d, &h), "create XTDA with zero spin");
  d.si = 1.0; d.restricted = 0;
  expect_err(xt_create(&d, &h), "create XTDA on UKS");
  d.kind = 99;
  expect_err(xt_create(&d, &h), "create unknown kind");
  d.kind = XT_KIND_XSF; d.restricted = 1; d.sa = 2; d.no = 1; d.nc = 4;
  expect_err(xt_create(&d, &h), "create XSF SA>0 with one open shell");
  d.kind = XT_KIND_XTDA; d.sa = 0; d.xctype = 17;
  expect_err(xt_create(&d, &h), "create bad xctype");
  d.kind = XT_KIND_SF_DOWN; d.xctype = XT_XC_GGA; d.no = 2; d.nc = 3; d.sf_kernel = 5;
  expect_err(xt_create(&d, &h), "create bad sf_kernel");
  d.sf_kernel = XT_SF_ALDA0;
  // null-context calls of every setter / query
  double buf[8] = {0};
  expect_err(xt_set_orbitals(nullptr, buf, buf, XT_PTR_HOST), "set_orbitals null");
  expect_err(xt_set_fock_mo(nullptr, buf, buf, buf, buf, XT_PTR_HOST), "set_fock_mo null");
  expect_err(xt_set_jk_df(nullptr, buf, 0, XT_PTR_HOST), "set_jk_df null");
  expect_err(xt_set_grid(nullptr, buf, buf, buf, XT_PTR_HOST), "set_grid null");
  expect_err(xt_apply(nullptr, 1, buf, buf, XT_PTR_HOST), "apply null");
  expect_err(xt_set_exchange_mode(nullptr, XT_K_AUTO, 0.0), "exchange_mode null");
  expect_err(xt_exchange_plan(nullptr, nullptr, nullptr), "exchange_plan null");
  expect_err(xt_set_profile(nullptr, 1), "profile null");
  expect_err(xt_profile_stats(nullptr, 1, buf), "profile_stats null");
  expect_err(xt_profile_bytes(nullptr, 9, buf), "profile_bytes bad tag");
  // device kernels: argument checks run before any HIP call
  expect_err(xt_dgemm_strided(-1, 4, 4, 1, 1, 1.0, buf, 1, 4, 0, 0, buf, 4, 1, 0, 0, 0.0, buf, 4, 0, nullptr),
             "dgemm_strided negative m");
  expect_err(xt_dgemm_strided(4, 4, 4, 1, 1, 1.0, buf, 2, 4, 0, 0, buf, 4, 1, 0, 0, 0.0, buf, 4, 0, nullptr),
             "dgemm_strided A without a unit stride");
  expect_err(xt_dgemm_strided(4, 4, 4, 1, 1, 1.0, buf, 4, 1, 0, 0, buf, 4, 1, 0, 0, 0.0, buf, 3, 0, nullptr),
             "dgemm_strided ldc < n");
  expect_err(xt_dgemm_strided(4, 4, 4, 1, 1, 1.0, nullptr, 4, 1, 0, 0, buf, 4, 1, 0, 0, 0.0, buf, 4, 0, nullptr),
             "dgemm_strided null A");
  expect_err(xt_dgemm_strided(4, 4, 4, 2, 1, 1.0, buf, 4, 1, -16, 0, buf, 4, 1, 16, 0, 0.0, buf, 4, 0, nullptr),
             "dgemm_strided negative stride");
  expect_err(xt_int2e_cart(-1, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, 0, 0.0, nullptr,
                           nullptr, 0.0, 0, nullptr, 0, nullptr), "int2e negative npair");
  expect_err(xt_int2e_cart(1, nullptr, nullptr, nullptr, 1, nullptr, nullptr, nullptr, 4, 0, 0.0, nullptr,
                           nullptr, 0.0, 0, nullptr, 0, nullptr), "int2e orbital l > 3");
  expect_err(xt_eval_ao(10, nullptr, 1, nullptr, nullptr, nullptr, nullptr, 2, nullptr, 0, 0, nullptr),
             "eval_ao deriv 2");
  std::printf(failures ? "asan driver: %d failures\n" : "asan driver: ok\n", failures);
  return failures ? 1 : 0;
}
