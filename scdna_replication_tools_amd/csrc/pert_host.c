/* pert_host.c -- host (CPU) helpers of the tau initialiser's exact path (tau_init.py).
 *
 * The reference's per-cell guess_times (pert_model.py:364-457) fits
 * sklearn.mixture.GaussianMixture in fp32; tau_init.exact_gmm_means restates that EM op for
 * op.  Its E step is elementwise (numpy, on each cell's distinct values); this file is its
 * M step and lower bound, the part that walks all L bins of every cell, written in C so
 * the tau initialiser's threads run it without the GIL:
 *
 *   resp = resp_u[inv]                          gather of the distinct-value rows
 *   nk   = resp.sum(axis=0) + 10 eps            numpy adds the rows in order
 *   mu   = np.dot(resp.T, X) / nk               the same cblas_sgemv call numpy makes
 *   cov  = np.dot(resp[:, k] * diff.T, diff) / nk[k] + reg_covar    the same cblas_sdot
 *   lb   = np.mean(lpn_u[inv])                  numpy's pairwise float32 sum, then
 *                                               float64 division by the count
 *
 * Every fp32 operation is the one numpy / OpenBLAS performs, in the same order: the BLAS
 * routines are numpy's own (their addresses are passed in by the caller), the reductions
 * follow numpy's loops (add.reduce over a contiguous row: pairwise with 8 accumulators and
 * blocks of 128; along axis 0: one add per row), and the file is compiled without
 * contraction (-ffp-contract=off) or reassociation.  tests/test_tau_init.py checks the
 * results against sklearn bit for bit.
 */
#include <stdint.h>

typedef void (*pert_sgemv_fn)(int order, int trans, int64_t m, int64_t n, float alpha, const float* a,
                              int64_t lda, const float* x, int64_t incx, float beta, float* y, int64_t incy);
typedef float (*pert_sdot_fn)(int64_t n, const float* x, int64_t incx, const float* y, int64_t incy);

enum { kColMajor = 102, kNoTrans = 111 };

/* numpy's float32 add.reduce of a contiguous run (loops_utils.h pairwise sum) */
static float pairwise(const float* a, int64_t n) {
  if (n < 8) {
    float res = -0.0f;
    for (int64_t i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= 128) {
    float r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i;
    for (i = 8; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise(a, n2) + pairwise(a + n2, n - n2);
}

float pert_host_pairwise_sum(const float* a, int64_t n) { return pairwise(a, n); }

/* "pert_host src=<hash>": the hash of the sources and flags this binary was built from
 * (build.py build_host passes it in); tau_init refuses a library whose hash differs. */
#ifndef PERT_HOST_SRC
#define PERT_HOST_SRC "unknown"
#endif
const char* pert_host_version(void) { return "pert_host src=" PERT_HOST_SRC; }

/* One M step and lower bound for the cells ``rows`` (m of them) of an EM chunk.
 *   resp_u  (m, U, 2)  responsibilities of each cell's distinct values (E step output)
 *   lpn_u   (m, U)     their log p(x) (NULL: no lower bound, the initial M step)
 *   inv     (n, L)     distinct-value index of every bin of every cell of the chunk
 *   X       (n, L)     the standardized fp32 profiles
 * outputs per cell j: nk[2j..], means[2j..], cov[2j..] (reg_covar added), lb[j].
 * scratch: 4 L floats.  Returns 0. */
int pert_host_em_mstep(int64_t m, int64_t L, int64_t U, const int64_t* rows, const float* resp_u,
                       const float* lpn_u, const int64_t* inv, const float* X, void* sgemv_ptr, void* sdot_ptr,
                       float* nk, float* means, float* cov, float* lb, float* scratch) {
  const pert_sgemv_fn sgemv = (pert_sgemv_fn)sgemv_ptr;
  const pert_sdot_fn sdot = (pert_sdot_fn)sdot_ptr;
  const float eps10 = 10.0f * 1.1920928955078125e-07f;   /* 10 * np.finfo(np.float32).eps */
  const float reg_covar = (float)1e-6;
  float* r = scratch;              /* (L, 2) */
  float* diff = scratch + 2 * L;   /* (L) */
  float* prod = scratch + 3 * L;   /* (L) */
  for (int64_t j = 0; j < m; ++j) {
    const int64_t c = rows[j];
    const int64_t* iv = inv + c * L;
    const float* x = X + c * L;
    const float* ru = resp_u + j * U * 2;
    for (int64_t l = 0; l < L; ++l) {
      r[2 * l] = ru[2 * iv[l]];
      r[2 * l + 1] = ru[2 * iv[l] + 1];
    }
    float n0 = r[0], n1 = r[1];
    for (int64_t l = 1; l < L; ++l) {
      n0 += r[2 * l];
      n1 += r[2 * l + 1];
    }
    n0 += eps10;
    n1 += eps10;
    float dots[2];
    sgemv(kColMajor, kNoTrans, 2, L, 1.0f, r, 2, x, 1, 0.0f, dots, 1);   /* np.dot(resp.T, X) */
    const float mu[2] = {dots[0] / n0, dots[1] / n1};
    const float nkk[2] = {n0, n1};
    for (int k = 0; k < 2; ++k) {
      for (int64_t l = 0; l < L; ++l) {
        diff[l] = x[l] - mu[k];
        prod[l] = r[2 * l + k] * diff[l];
      }
      const float d = sdot(L, prod, 1, diff, 1);
      const float cv = d / nkk[k];
      cov[2 * j + k] = cv + reg_covar;
    }
    nk[2 * j] = n0;
    nk[2 * j + 1] = n1;
    means[2 * j] = mu[0];
    means[2 * j + 1] = mu[1];
    if (lpn_u != 0) {
      const float* lu = lpn_u + j * U;
      for (int64_t l = 0; l < L; ++l) diff[l] = lu[iv[l]];
      lb[j] = (float)((double)pairwise(diff, L) / (double)L);
    }
  }
  return 0;
}
