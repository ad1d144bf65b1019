// tau_kernels.hip -- gfx950 kernel of the tau initialiser's batched pass (tau_init.py).
//
// Reference: pert_model.py:364-375 (manhattan_binarization's standardisation and its
// 2-component GaussianMixture, random_state=0, whose initialisation is one k-means run,
// sklearn cluster/_kmeans.py _kmeans_plusplus + _kmeans_single_lloyd, then EM,
// mixture/_base.py fit_predict), called per cell by guess_times (:426-457).
//
// The Python restatement of this stage (tau_init._kmeans_em, one tensor program over all
// cells) is an iterative loop of ~20 small launches per Lloyd / EM iteration, up to 300 + 100
// iterations: launch-bound on the GPU (a C1-sized fit spent 1.1 s there).  Here the whole
// stage is ONE launch: one 256-thread workgroup per (cell, tie direction) runs k-means++ ->
// Lloyd -> (alternative Lloyd runs where a k-means++ draw sat on a rounding boundary) -> EM
// to its own stopping iteration, in fp64, with the same decisions and the same rounding-
// margin flags as the tensor program (the flagged cells are then recomputed exactly on the
// host, tau_init.exact_fractions).  Every reduction is a fixed-order block sum, so reruns are
// bit-identical.  The profile is read from the fp32 CN-normalised reads [N][L] (one
// contiguous row per cell; the fp64 standardised values are recomputed from it on each pass
// instead of being stored, 4 B per bin per pass, L2/MALL resident at genome length).

#include "../../include/pert_hip.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace {

constexpr int kT = 256;                 // threads per workgroup
constexpr int kTW = kT / 64;            // waves per workgroup
constexpr double kLog2Pi = 1.8378770664093454836;
constexpr double kEps10 = 10.0 * 2.220446049250313e-16;   // 10 * finfo(float64).eps

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Fixed-order block sums of NV values; every thread receives the sums.
template <int NV>
__device__ __forceinline__ void block_sums(double (&v)[NV], double* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();                      // earlier readers of sm are done
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) sm[k * kTW + w] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double t = 0.0;
#pragma unroll
    for (int ww = 0; ww < kTW; ++ww) t += sm[k * kTW + ww];
    v[k] = t;
  }
}

__device__ __forceinline__ int block_min_i(int v, int* smi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
  __syncthreads();
  if (lane == 0) smi[w] = v;
  __syncthreads();
  int t = smi[0];
#pragma unroll
  for (int ww = 1; ww < kTW; ++ww) t = min(t, smi[ww]);
  return t;
}

struct Cell {
  const float* x;      // the cell's CN-normalised reads, [L]
  int L;
  double mean, sd;     // standardisation (pert_model.py:367)
  double mX;           // mean of the standardised profile (KMeans centres its data first)
  __device__ __forceinline__ double X(int i) const { return ((double)x[i] - mean) / sd; }
  __device__ __forceinline__ double Xc(int i) const { return X(i) - mX; }
};

// sklearn's label rule for 2 centres: centre 1 where ||c1||^2 - 2 x c1 < ||c0||^2 - 2 x c0.
// Points within `tie` (relative to the magnitude of the compared values) of the decision go
// to centre 1 (tie > 0) or centre 0 (tie < 0): integer read counts put whole groups of
// identical values exactly on a decision, where rounding decides (tau_init._assign).
__device__ __forceinline__ int assign2(double X, double c0, double c1, double tie) {
  const double d1 = c1 * c1 - 2.0 * X * c1;
  const double d0 = c0 * c0 - 2.0 * X * c0;
  if (tie == 0.0) return d1 < d0 ? 1 : 0;
  const double scale = c0 * c0 + c1 * c1 + 2.0 * fabs(X) * (fabs(c0) + fabs(c1));
  return (d1 - d0 < tie * scale) ? 1 : 0;
}

// Lloyd's k-means for 2 centres (sklearn _kmeans_single_lloyd: at most max_iter iterations,
// stop on unchanged labels (strict convergence) or a centre shift <= tol, then the final
// re-assignment) -- tau_init._lloyd for one cell.  lab_old: the cell's scratch row; out: the
// final labels.  Sets *fragile when the shift test is within `fragile_rel` of tol.
__device__ void lloyd(const Cell& c, double c0, double c1, double tol, double sumXc, double tie,
                      double fragile_rel, int max_iter, int8_t* lab_old, int8_t* out, bool* fragile,
                      double* sm) {
  const int L = c.L;
  for (int i = threadIdx.x; i < L; i += kT) lab_old[i] = -1;
  bool strict = false;
  for (int it = 0; it < max_iter; ++it) {
    double acc[3] = {0.0, 0.0, 0.0};            // w1, s1, changed labels
    for (int i = threadIdx.x; i < L; i += kT) {
      const double X = c.Xc(i);
      const int l = assign2(X, c0, c1, tie);
      acc[0] += (double)l;
      acc[1] += l ? X : 0.0;
      acc[2] += (l != lab_old[i]) ? 1.0 : 0.0;
      lab_old[i] = (int8_t)l;
    }
    block_sums<3>(acc, sm);
    const double w1 = acc[0], w0 = (double)L - w1;
    const double s1 = acc[1], s0 = sumXc - s1;
    const double n0 = w0 > 0.0 ? s0 / fmax(w0, 1.0) : c0;
    const double n1 = w1 > 0.0 ? s1 / fmax(w1, 1.0) : c1;
    const double shift = (n0 - c0) * (n0 - c0) + (n1 - c1) * (n1 - c1);
    const bool same = acc[2] == 0.0;
    if (!same && fabs(shift - tol) <= fragile_rel * tol) *fragile = true;
    c0 = n0;
    c1 = n1;
    if (same) {
      strict = true;
      break;
    }
    if (shift <= tol) break;
  }
  for (int i = threadIdx.x; i < L; i += kT) out[i] = strict ? lab_old[i] : (int8_t)assign2(c.Xc(i), c0, c1, tie);
}

// Inclusive prefix sums of one 256-element chunk: returns this thread's cumulative value
// (carry + the chunk's elements up to and including this thread's), *total the carry plus
// the whole chunk -- both sums in one fixed order.
__device__ __forceinline__ double chunk_scan(double v, double carry, double* total, double* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double t = __shfl_up(v, off, 64);
    if (lane >= off) v += t;
  }
  __syncthreads();
  if (lane == 63) sm[w] = v;
  __syncthreads();
  double pre = carry;
  for (int ww = 0; ww < w; ++ww) pre += sm[ww];
  double tot = carry;
#pragma unroll
  for (int ww = 0; ww < kTW; ++ww) tot += sm[ww];
  *total = tot;
  return pre + v;
}

// Order-preserving map of a double onto uint64 (radix select) and back.
__device__ __forceinline__ uint64_t okey(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double ikey(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// Order statistics rank[0..3] (0-based) of the standardised profile by 8-bit radix select,
// MSB first (8 passes, one 256-bin integer histogram per target in LDS: deterministic).
__device__ void select4(const Cell& c, const int (&rank)[4], double (&out)[4], uint32_t* hist, uint64_t* s_pref,
                        long long* s_k) {
  const int L = c.L;
  if (threadIdx.x < 4) {
    s_pref[threadIdx.x] = 0;
    s_k[threadIdx.x] = rank[threadIdx.x];
  }
  for (int pass = 0; pass < 8; ++pass) {
    const int shift = 56 - 8 * pass;
    for (int i = threadIdx.x; i < 4 * 256; i += kT) hist[i] = 0;
    __syncthreads();
    uint64_t pref[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pref[j] = s_pref[j];
    for (int i = threadIdx.x; i < L; i += kT) {
      const uint64_t key = okey(c.X(i));
      const uint32_t dig = (uint32_t)(key >> shift) & 255u;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (pass == 0 || (key >> (shift + 8)) == (pref[j] >> (shift + 8))) atomicAdd(&hist[j * 256 + dig], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      const int j = threadIdx.x;
      long long cum = 0;
      for (int d = 0; d < 256; ++d) {
        const long long h = hist[j * 256 + d];
        if (cum + h > s_k[j]) {
          s_pref[j] = pref[j] | ((uint64_t)d << shift);
          s_k[j] -= cum;
          break;
        }
        cum += h;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) out[j] = ikey(s_pref[j]);
}

// first index i in [0, 100) with th[i] >= v (th ascending), i.e. #{i : th[i] < v}
__device__ __forceinline__ int count_below(const double* th, double v) {
  int lo = 0, hi = 100;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (th[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}
// #{i : th[i] <= v}
__device__ __forceinline__ int count_le(const double* th, double v) {
  int lo = 0, hi = 100;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (th[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

constexpr double kFix = 4294967296.0;     // 2^32: fixed-point scale of the scan's LDS histograms

__global__ __launch_bounds__(kT) void tau_binarize_kernel(int L, int N, const float* __restrict__ norm,
                                                             pert_tau_params p, int8_t* __restrict__ labels,
                                                             int8_t* __restrict__ scratch,
                                                             double* __restrict__ means,
                                                             int32_t* __restrict__ flags,
                                                             double* __restrict__ frac_out,
                                                             double* __restrict__ minor_out) {
  __shared__ double sm[8 * kTW];
  __shared__ double sval[4];
  __shared__ int smi[kTW];
  __shared__ uint32_t s_hist[4 * 256];
  __shared__ uint64_t s_pref[4];
  __shared__ long long s_k[4];
  __shared__ double s_th[100];
  __shared__ unsigned long long s_h0[101], s_h1[101];
  __shared__ int s_hn[101], s_e[101];
  __shared__ double s_d[100];
  __shared__ int s_cnt[100], s_near[100];
  const int n = blockIdx.x, run = blockIdx.y;
  if (n >= N) return;
  const double tie = run == 0 ? p.tie : -p.tie;
  const size_t row = ((size_t)run * N + n) * (size_t)L;
  int8_t* lab1 = labels + row;
  int8_t* lab_old = scratch + row;
  Cell c;
  c.x = norm + (size_t)n * L;
  c.L = L;
  const double invL = 1.0 / (double)L;

  // ---- standardisation (X - mean) / std (population std), and the k-means tolerance
  {
    double a[1] = {0.0};
    for (int i = threadIdx.x; i < L; i += kT) a[0] += (double)c.x[i];
    block_sums<1>(a, sm);
    c.mean = a[0] / (double)L;
    double q[1] = {0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double d = (double)c.x[i] - c.mean;
      q[0] += d * d;
    }
    block_sums<1>(q, sm);
    c.sd = sqrt(q[0] / (double)L);
    c.mX = 0.0;
    double s[1] = {0.0};
    for (int i = threadIdx.x; i < L; i += kT) s[0] += c.X(i);
    block_sums<1>(s, sm);
    c.mX = s[0] / (double)L;
  }
  double sumXc, tol;
  {
    double s[1] = {0.0};
    for (int i = threadIdx.x; i < L; i += kT) s[0] += c.Xc(i);
    block_sums<1>(s, sm);
    sumXc = s[0];
    const double m = sumXc / (double)L;
    double q[1] = {0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double d = c.Xc(i) - m;
      q[0] += d * d;
    }
    block_sums<1>(q, sm);
    tol = q[0] / (double)L * 1e-4;            // KMeans tolerance: mean variance x 1e-4
  }

  // ---- k-means++ for 2 centres (tau_init._kmeans_pp): first centre from the data-free
  // RandomState(0) draw, two local trials at u * potential on the cumulative sum
  const int first = min(max(p.first, 0), L - 1);
  const double cen0 = c.Xc(first);
  double pot;
  {
    double a[1] = {0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double d = c.Xc(i) - cen0;
      a[0] += d * d;
    }
    block_sums<1>(a, sm);
    pot = a[0];
  }
  const double rv[2] = {p.u[0] * pot, p.u[1] * pot};
  int cand[2] = {-1, -1};
  double cum_at[2] = {0.0, 0.0}, cum_prev[2] = {0.0, 0.0};
  {
    double carry = 0.0;
    for (int base = 0; base < L && (cand[0] < 0 || cand[1] < 0); base += kT) {
      const int i = base + threadIdx.x;
      double v = 0.0;
      if (i < L) {
        const double d = c.Xc(i) - cen0;
        v = d * d;
      }
      double total;
      const double cum = chunk_scan(v, carry, &total, sm);
      const bool last = base + kT >= L;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (cand[t] >= 0) continue;                                   // uniform
        const int hit = block_min_i((i < L && cum >= rv[t]) ? i : 0x7fffffff, smi);
        if (hit == 0x7fffffff && !last) continue;                     // uniform
        const int ci = hit != 0x7fffffff ? hit : L - 1;               // searchsorted, clamped
        __syncthreads();
        if (i == ci) sval[0] = cum;
        if (i == ci - 1) sval[1] = cum;
        __syncthreads();
        cand[t] = ci;
        cum_at[t] = sval[0];
        cum_prev[t] = ci == base ? carry : sval[1];
      }
      carry = total;
    }
  }
  const double xc[2] = {c.Xc(cand[0]), c.Xc(cand[1])};
  double pots[2] = {0.0, 0.0};
  for (int i = threadIdx.x; i < L; i += kT) {
    const double X = c.Xc(i);
    const double d0 = (X - cen0) * (X - cen0);
    pots[0] += fmin(d0, (X - xc[0]) * (X - xc[0]));
    pots[1] += fmin(d0, (X - xc[1]) * (X - xc[1]));
  }
  block_sums<2>(pots, sm);
  const double cen1 = pots[1] < pots[0] ? xc[1] : xc[0];               // first minimum
  bool frag_pp = false;
  for (int t = 0; t < 2; ++t) {
    if (fabs(cum_at[t] - rv[t]) <= p.pp_margin * pot) frag_pp = true;
    if (cand[t] > 0 && fabs(cum_prev[t] - rv[t]) <= p.pp_margin * pot) frag_pp = true;
  }
  if (xc[0] != xc[1] && fabs(pots[0] - pots[1]) <= p.pp_margin * fmax(fabs(pots[0]), fabs(pots[1])))
    frag_pp = true;

  bool fragile = false;
  lloyd(c, cen0, cen1, tol, sumXc, tie, p.fragile, p.lloyd_max_iter, lab_old, lab1, &fragile, sm);
  if (frag_pp) {
    // the partition is still certain when Lloyd ends in the same labels from every second
    // centre the reference could have drawn: either trial's candidate and its neighbours
    bool same_all = true;
    for (int a = 0; a < 6; ++a) {
      const int t = a & 1, off = a / 2 - 1;                           // (cand-1, cand, cand+1) x trials
      const int ia = min(max(cand[t] + off, 0), L - 1);
      bool fr_a = false;
      lloyd(c, cen0, c.Xc(ia), tol, sumXc, tie, p.fragile, p.lloyd_max_iter, lab_old, lab_old, &fr_a, sm);
      double d[1] = {0.0};
      for (int i = threadIdx.x; i < L; i += kT) d[0] += (lab_old[i] != lab1[i]) ? 1.0 : 0.0;
      block_sums<1>(d, sm);
      same_all = same_all && d[0] == 0.0 && !fr_a;
    }
    if (same_all) frag_pp = false;
  }

  // ---- EM of the 2-component 1-D mixture from the k-means labels (tau_init._gmm_means;
  // sklearn fit_predict: at most em_max_iter iterations, |lower-bound change| < em_tol)
  double w0, w1, mu0, mu1, var0, var1;
  {
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double X = c.X(i);
      const double r1 = (double)lab1[i], r0 = 1.0 - r1;
      a[0] += r0;
      a[1] += r1;
      a[2] += r0 * X;
      a[3] += r1 * X;
    }
    block_sums<4>(a, sm);
    const double nk0 = a[0] + kEps10, nk1 = a[1] + kEps10;
    mu0 = a[2] / nk0;
    mu1 = a[3] / nk1;
    double q[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double X = c.X(i);
      const double r1 = (double)lab1[i], r0 = 1.0 - r1;
      q[0] += r0 * (X - mu0) * (X - mu0);
      q[1] += r1 * (X - mu1) * (X - mu1);
    }
    block_sums<2>(q, sm);
    var0 = q[0] / nk0 + p.reg_covar;
    var1 = q[1] / nk1 + p.reg_covar;
    w0 = nk0 * invL;
    w1 = nk1 * invL;
    const double ws = w0 + w1;
    w0 /= ws;
    w1 /= ws;
  }
  double lb = -INFINITY;
  for (int it = 0; it < p.em_max_iter; ++it) {
    const double pr0 = 1.0 / sqrt(var0), pr1 = 1.0 / sqrt(var1);
    const double lp0 = log(pr0), lp1 = log(pr1), lw0 = log(w0), lw1 = log(w1);
    double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double X = c.X(i);
      const double y0 = (X - mu0) * pr0, y1 = (X - mu1) * pr1;
      const double l0 = (-0.5 * (kLog2Pi + y0 * y0) + lp0) + lw0, l1 = (-0.5 * (kLog2Pi + y1 * y1) + lp1) + lw1;
      const double m = fmax(l0, l1);
      const double lpn = m + log(exp(l0 - m) + exp(l1 - m));
      const double r0 = exp(l0 - lpn), r1 = exp(l1 - lpn);
      a[0] += r0;
      a[1] += r1;
      a[2] += r0 * X;
      a[3] += r1 * X;
      a[4] += lpn;
    }
    block_sums<5>(a, sm);
    const double nk0 = a[0] + kEps10, nk1 = a[1] + kEps10;
    const double m0 = a[2] / nk0, m1 = a[3] / nk1;
    double q[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double X = c.X(i);
      const double y0 = (X - mu0) * pr0, y1 = (X - mu1) * pr1;
      const double l0 = (-0.5 * (kLog2Pi + y0 * y0) + lp0) + lw0, l1 = (-0.5 * (kLog2Pi + y1 * y1) + lp1) + lw1;
      const double m = fmax(l0, l1);
      const double lpn = m + log(exp(l0 - m) + exp(l1 - m));
      const double r0 = exp(l0 - lpn), r1 = exp(l1 - lpn);
      q[0] += r0 * (X - m0) * (X - m0);
      q[1] += r1 * (X - m1) * (X - m1);
    }
    block_sums<2>(q, sm);
    double nw0 = nk0 * invL, nw1 = nk1 * invL;
    const double ws = nw0 + nw1;
    w0 = nw0 / ws;
    w1 = nw1 / ws;
    mu0 = m0;
    mu1 = m1;
    var0 = q[0] / nk0 + p.reg_covar;
    var1 = q[1] / nk1 + p.reg_covar;
    const double lb2 = a[4] * invL;
    const double change = lb2 - lb;
    lb = lb2;
    if (fabs(fabs(change) - p.em_tol) <= p.em_margin) fragile = true;
    if (fabs(change) < p.em_tol) break;
  }
  // ---- levels (pert_model.py:377-400; tau_init._levels_scan): the GMM means, or percentiles of
  // the profile chosen by its skew when the means are closer than MEAN_GAP_THRESH
  double b0 = fmin(mu0, mu1), b1 = fmax(mu0, mu1);
  const double gap = fabs(mu0 - mu1);
  if (fabs(gap - p.mean_gap) <= p.fragile_abs) fragile = true;
  if (gap < p.mean_gap) {
    double m[2] = {0.0, 0.0};
    for (int i = threadIdx.x; i < L; i += kT) {
      const double xc = c.Xc(i);
      m[0] += xc * xc;
      m[1] += xc * xc * xc;
    }
    block_sums<2>(m, sm);
    const double m2 = m[0] / (double)L, m3 = m[1] / (double)L;
    const double sk = m3 / pow(m2, 1.5);
    if (fabs(sk - p.early_skew) <= p.fragile_abs || fabs(sk - p.late_skew) <= p.fragile_abs) fragile = true;
    const bool early = sk > p.early_skew, late = !early && sk < p.late_skew;
    const int qa = early ? 2 : (late ? 0 : 1), qb = early ? 4 : (late ? 2 : 3);   // (50, 95) / (5, 50) / (25, 75)
    const int rank[4] = {p.q_lo[qa], p.q_hi[qa], p.q_lo[qb], p.q_hi[qb]};
    double v[4];
    select4(c, rank, v, s_hist, s_pref, s_k);
    // np.percentile 'linear' with numpy's two-sided lerp (tau_init._percentiles)
    const double ta = p.q_t[qa], tb = p.q_t[qb];
    const double da = v[1] - v[0], dbq = v[3] - v[2];
    b0 = ta >= 0.5 ? v[1] - da * (1.0 - ta) : v[0] + da * ta;
    b1 = tb >= 0.5 ? v[3] - dbq * (1.0 - tb) : v[2] + dbq * tb;
  }

  // ---- the 100-threshold scan (:402-423) with the rounding margins of tau_init._levels_scan.
  // Threshold i binarises x to b1 iff x > th[i]; with c(x) = #{i : th[i] < x} the distance
  // d(th[i]) = sum_{c(x) <= i} |x - b0| + sum_{c(x) > i} |x - b1| is a prefix sum over a
  // 101-bin histogram of c(x) (fixed-point integer atomics: order-independent), and so are the
  // counts above each threshold and the points within the margin window of each threshold.
  for (int i = threadIdx.x; i < 101; i += kT) {
    s_h0[i] = 0;
    s_h1[i] = 0;
    s_hn[i] = 0;
    s_e[i] = 0;
  }
  if (threadIdx.x < 100) s_th[threadIdx.x] = threadIdx.x == 99 ? b1 : b0 + threadIdx.x * ((b1 - b0) / 99.0);
  __syncthreads();
  const double dbm = p.level_margin * fmax(fabs(b0), fabs(b1));
  const double win = 2.0 * dbm + 1e-6;
  double tmax = 0.0;
  for (int i = threadIdx.x; i < L; i += kT) {
    const double x = c.X(i);
    const double e0 = fabs(x - b0), e1 = fabs(x - b1);
    tmax = fmax(tmax, fmax(e0, e1));
    const int cx = count_below(s_th, x);
    atomicAdd(&s_h0[cx], (unsigned long long)(long long)llrint(e0 * kFix));
    atomicAdd(&s_h1[cx], (unsigned long long)(long long)llrint(e1 * kFix));
    atomicAdd(&s_hn[cx], 1);
    const int lo = count_below(s_th, x - win), hi = count_le(s_th, x + win);   // |x - th[i]| <= win
    if (lo < hi) {
      atomicAdd(&s_e[lo], 1);
      if (hi < 100) atomicAdd(&s_e[hi], -1);
    }
  }
  {
    double tm[1] = {tmax};
    // block max through the sum helper's LDS: wave max, then the 4 waves
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tm[0] = fmax(tm[0], __shfl_xor(tm[0], off, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = tm[0];
    __syncthreads();
    tmax = fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
  }
  if (threadIdx.x == 0) {
    long long h0 = 0, h1t = 0, h1 = 0;
    int hn = 0, hnt = 0, e = 0;
    for (int k = 0; k < 101; ++k) {
      h1t += (long long)s_h1[k];
      hnt += s_hn[k];
    }
    for (int i = 0; i < 100; ++i) {
      h0 += (long long)s_h0[i];
      h1 += (long long)s_h1[i];
      hn += s_hn[i];
      e += s_e[i];
      s_d[i] = (double)(h0 + (h1t - h1)) / kFix;
      s_cnt[i] = hnt - hn;
      s_near[i] = e;
    }
    int bi = 0;
    for (int i = 1; i < 100; ++i)
      if (s_d[i] < s_d[bi]) bi = i;                                   // first minimum
    smi[0] = bi;
  }
  __syncthreads();
  const int bi = smi[0];
  const double dmin = s_d[bi];
  const double near_best = (double)s_near[bi];
  bool scan = false;
  if (threadIdx.x < 100) {
    const int i = threadIdx.x;
    const double dcnt = fabs((double)(s_cnt[i] - s_cnt[bi]));
    const double nr = (double)s_near[i];
    const double noise = p.eps32 * (dcnt * 56.0 * 16.0 * tmax + (log2(dcnt + 1.0) + 2.0) * dmin);
    const double mid = b0 + b1;
    const double flip = fabs(mid - 2.0 * s_th[i]) + 4.0 * dbm;
    const double flip_b = fabs(mid - 2.0 * s_th[bi]) + 4.0 * dbm;
    const double slack = 2.0 * dcnt * dbm + nr * flip + near_best * flip_b + noise;
    scan = (dcnt > 0.0 || nr > 0.0) && (s_d[i] - dmin <= slack);
  }
  const int any_scan = block_min_i(scan ? 0 : 1, smi) == 0;

  if (threadIdx.x == 0) {
    const size_t o = (size_t)run * N + n;
    means[2 * o] = mu0;
    means[2 * o + 1] = mu1;
    flags[o] = (fragile ? 1 : 0) | (frag_pp ? 2 : 0) | (any_scan ? 4 : 0);
    frac_out[o] = (double)s_cnt[bi] / (double)L;
    minor_out[o] = near_best;
  }
}

}  // namespace

extern "C" int pert_tau_binarize(int32_t L, int32_t N, const float* norm, const pert_tau_params* p,
                                 int8_t* labels, int8_t* scratch, double* means, int32_t* flags, double* frac,
                                 double* minor, hipStream_t stream) {
  if (L < 2 || N < 1 || !norm || !p || !labels || !scratch || !means || !flags || !frac || !minor) return PERT_E_ARG;
  if (p->first < 0 || p->first >= L || p->lloyd_max_iter < 1 || p->em_max_iter < 1) return PERT_E_ARG;
  for (int j = 0; j < 5; ++j)
    if (p->q_lo[j] < 0 || p->q_lo[j] >= L || p->q_hi[j] < 0 || p->q_hi[j] >= L) return PERT_E_ARG;
  hipLaunchKernelGGL(tau_binarize_kernel, dim3(N, 2), dim3(kT), 0, stream, L, N, norm, *p, labels, scratch,
                     means, flags, frac, minor);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? PERT_OK : PERT_E_HIP_BASE + (int)e;
}
