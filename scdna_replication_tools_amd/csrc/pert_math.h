// pert_math.h -- per (bin, cell) arithmetic of the PERT log joint, shared by the
// gfx950 kernels (pert_kernels.hip) and the host self-test entry points.
//
// Everything here restates reference scdna_replication_tools/pert_model.py:607-646
// plus the torch.distributions log densities Pyro wraps:
//
//   s(c, r) = log pi~_c + log Bern(r | phi) + NB'(chi = c (1 + r))
//   NB'(chi) = delta_chi log(1 - lam) + Lambda(delta_chi, x)
//   Lambda(d, x) = lgamma(d + x) - lgamma(d) - (x log x - x)
//
// The chi-independent remainder of the NB log density, x log(lam) - lgamma(1 + x)
// + (x log x - x), is parameter independent in steps 2/3 and is added on the host
// once (kappa(x) in DESIGN.md).  Subtracting x log x - x from lgamma(d + x) keeps
// every per-state score O(100) instead of O(x log x), so the fp32 differences
// that decide the responsibilities stay accurate.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define PERT_HD __host__ __device__ __forceinline__

namespace pert {

constexpr float kLn2 = 0.693147180559945309f;
constexpr float kLog2e = 1.442695040888963407f;
constexpr float kEps32 = 1.1920928955078125e-07f;   // torch.finfo(float32).eps (clamp_probs)
constexpr float kTiny32 = 1.1754943508222875e-38f;  // torch.finfo(float32).tiny (_clipped_sigmoid)
constexpr float kHalfLog2Pi = 0.918938533204672742f;
constexpr float kLogEps32 = -15.942385152878742f;    // log(eps)
constexpr float kLog1mEps32 = -1.1920929665620896e-07f;  // log(1 - eps)

// ----------------------------------------------------------------- primitives
// v_log_f32 / v_exp_f32 / v_rcp_f32 on the device; libm on the host self-test.
PERT_HD float flog(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_logf(x) * kLn2;
#else
  return logf(x);
#endif
}
PERT_HD float __builtin_amdgcn_logf_or_log2(float x) {   // log2(x): v_log_f32 / libm
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_logf(x);
#else
  return log2f(x);
#endif
}
PERT_HD float fexp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_exp2f(x * kLog2e);
#else
  return expf(x);
#endif
}
PERT_HD float fexp2(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_exp2f(x);
#else
  return exp2f(x);
#endif
}
PERT_HD float fmed3(float v, float lo, float hi) {   // clamp v to [lo, hi] (v_med3_f32)
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_fmed3f(v, lo, hi);
#else
  return fminf(fmaxf(v, lo), hi);
#endif
}
PERT_HD float frcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}

// every active lane of the wave (the predicate itself on the host self-test)
PERT_HD bool wave_all(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __all(p) != 0;
#else
  return p;
#endif
}

// log1p(q) for q >= 0 given inv_u ~= 1/(1+q): the rounding error of 1+q is added
// back (q - ((1+q) - 1)) / (1+q) -- exact to a few ulp of the result.
PERT_HD float log1p_corr(float q, float inv_u) {
  float u = 1.0f + q;
  return flog(u) + (q - (u - 1.0f)) * inv_u;
}

// Stirling remainder S(z) = 1/(12 z) - 1/(360 z^3) + 1/(1260 z^5): truncation error below
// 1/(1680 z^7), 2.7e-7 at z = 3 (kAsymMin); the digamma series below (to 1/(252 z^6)) below
// 1/(240 z^8), 6.4e-7 at z = 3.  Over d in [3, 3.5] and every x the series' error in the terms
// the kernels use is 1e-7 (Lambda) / 1.4e-6 (Psi) of the accuracy test's scale (5e-6 / 2e-5
// allowed; at z = 5 it was 2e-9 / 4e-8).  Round 6 lowered the threshold from 5 (shift 4) to
// 3 (shift 2): at 20 kb bins (C5: D = u omega (1-lam)/lam ~ 0.7) most chains of a wave run the
// shift, and now with half its factors, fewer chains need it and more chain pairs run packed.
#ifndef PERT_SHIFT_N
#define PERT_SHIFT_N 2             // (A/B builds: -DPERT_SHIFT_N=4 is round 5's threshold 5 / shift 4)
#endif
#ifndef PERT_PACKED_SHIFT
#define PERT_PACKED_SHIFT 0
#endif
constexpr int kShiftN = PERT_SHIFT_N;   // 1 <= d < kAsymMin is shifted by kShiftN (d + kShiftN >= kAsymMin)
constexpr float kAsymMin = 1.0f + kShiftN;   // asymptotic series used for arguments >= kAsymMin
constexpr float kShift = (float)kShiftN;
PERT_HD float stirling_rem(float rz) {
  float rz2 = rz * rz;
  return rz * (0.0833333333333333333f - rz2 * (0.00277777777777777778f - rz2 * 0.000793650793650793651f));
}

// Lambda(d, x) = lgamma(d+x) - lgamma(d) - (x log x - x)  and  Psi(d, x) = digamma(d+x) - digamma(d)
// for d >= 1, x >= 0 (x integer valued as in pert_model.py:163-166; any x >= 0 works).
// invx = 1/x (0 when x == 0).
//   d >= kAsymMin: asymptotic series on both arguments in cancellation-free form
//     (d - 1/2) log1p(x/d) + x log1p(d/x) + S(d+x) - S(d)
//   d <  kAsymMin: shift d by kShift with the recurrences (nb_shift)
//     lgamma(y) = lgamma(y + 4) - log prod_{i<4} (y + i),  digamma(y) = digamma(y + 4) - sum 1/(y + i).
PERT_HD void nb_lgdiff_asym(float d, float x, float invx, float& lam, float& psi) {
  // d >= kAsymMin (no branches)
  const float r = frcp(d);
  const float zs = d + x;
  const float rz = frcp(zs);
  const float l1 = log1p_corr(x * r, d * rz);         // log1p(x/d)
  const float l2 = log1p_corr(d * invx, x * rz);      // log1p(d/x); 0 when x == 0
  lam = (d - 0.5f) * l1 + x * l2 + (stirling_rem(rz) - stirling_rem(r));
  const float r2 = r * r, rz2 = rz * rz;
  const float r4 = r2 * r2, rz4 = rz2 * rz2;
  psi = l1 - 0.5f * (rz - r) - 0.0833333333333333333f * (rz2 - r2)
        + 0.00833333333333333333f * (rz4 - r4) - 0.00396825396825396825f * (rz4 * rz2 - r4 * r2);
}

// nb_lgdiff_asym for d = chi D >= kAsymMin with the per-(bin, cell) invariants hoisted out of
// the chi loop: r = 1/d = (1/D)(1/chi) (one v_rcp per cell.bin instead of per chi) and
// log1p(d/x) = log1p(x/d) + log(d/x), log(d/x) = log(chi) + (log D - log x) (no second
// v_log per chi).  ldxc = log(d/x) (any finite value when x == 0: it is multiplied by x).
PERT_HD void nb_lgdiff_asym_hoisted(float d, float r, float x, float ldxc, float& lam, float& psi) {
  const float zs = d + x;
  const float rz = frcp(zs);
  const float l1 = log1p_corr(x * r, d * rz);         // log1p(x/d)
  const float l2 = l1 + ldxc;                         // log1p(d/x)
  lam = (d - 0.5f) * l1 + x * l2 + (stirling_rem(rz) - stirling_rem(r));
  const float r2 = r * r, rz2 = rz * rz;
  const float r4 = r2 * r2, rz4 = rz2 * rz2;
  psi = l1 - 0.5f * (rz - r) - 0.0833333333333333333f * (rz2 - r2)
        + 0.00833333333333333333f * (rz4 - r4) - 0.00396825396825396825f * (rz4 * rz2 - r4 * r2);
}

// Two chi chains at once in packed fp32 (v_pk_fma/mul/add_f32: two lanes' worth of work per
// VALU issue; the transcendentals stay per element): nb_lgdiff_asym_hoisted for chi = (c.x,
// c.y), with NB'(chi) = d log(1-lam) + Lambda and Bc = chi (log(1-lam) + Psi) folded in.
typedef float pf2 __attribute__((ext_vector_type(2)));
PERT_HD void nb_asym_pair(pf2 chi, pf2 rchi, pf2 lchi, float D, float rD, float x, float ldx, float log1m_lam,
                          pf2& nchi, pf2& bc) {
  const pf2 d = chi * D;
  const pf2 r = rchi * rD;                            // 1/d
  const pf2 zs = d + x;
  const pf2 rz = {frcp(zs.x), frcp(zs.y)};
  const pf2 q = r * x;                                // x/d
  const pf2 iu = d * rz;                              // 1/(1 + x/d)
  const pf2 u = q + 1.0f;
  const pf2 lu = pf2{__builtin_amdgcn_logf_or_log2(u.x), __builtin_amdgcn_logf_or_log2(u.y)} * kLn2;
  const pf2 l1 = lu + (q - (u - 1.0f)) * iu;          // log1p(x/d), log1p_corr
  const pf2 l2 = l1 + (lchi + ldx);                   // log1p(d/x)
  const pf2 r2 = r * r, rz2 = rz * rz;
  const pf2 sr = r * (0.0833333333333333333f - r2 * (0.00277777777777777778f - r2 * 0.000793650793650793651f));
  const pf2 srz = rz * (0.0833333333333333333f - rz2 * (0.00277777777777777778f - rz2 * 0.000793650793650793651f));
  const pf2 lam = (d - 0.5f) * l1 + x * l2 + (srz - sr);
  const pf2 r4 = r2 * r2, rz4 = rz2 * rz2;
  const pf2 psi = l1 - 0.5f * (rz - r) - 0.0833333333333333333f * (rz2 - r2)
                  + 0.00833333333333333333f * (rz4 - r4) - 0.00396825396825396825f * (rz4 * rz2 - r4 * r2);
  nchi = d * log1m_lam + lam;
  bc = chi * (psi + log1m_lam);
}

// nb_asym_pair without the hoisted per-(bin, cell) invariants: each chain's own 1/d and
// log1p(d/x) (as nb_lgdiff_asym), the series in packed fp32 -- for chain pairs of the
// low-coverage regime whose deltas are all >= kAsymMin (no extra values live across chains).
PERT_HD void nb_asym_pair_direct(pf2 chi, float D, float x, float invx, float log1m_lam, pf2& nchi, pf2& bc) {
  const pf2 d = chi * D;
  const pf2 r = {frcp(d.x), frcp(d.y)};
  const pf2 zs = d + x;
  const pf2 rz = {frcp(zs.x), frcp(zs.y)};
  const pf2 q = r * x;                                // x/d
  const pf2 iu = d * rz;                              // 1/(1 + x/d)
  const pf2 u = q + 1.0f;
  const pf2 lu = pf2{__builtin_amdgcn_logf_or_log2(u.x), __builtin_amdgcn_logf_or_log2(u.y)} * kLn2;
  const pf2 l1 = lu + (q - (u - 1.0f)) * iu;          // log1p(x/d)
  const pf2 q2 = d * invx;                            // d/x (0 when x == 0)
  const pf2 u2 = q2 + 1.0f;
  const pf2 lu2 = pf2{__builtin_amdgcn_logf_or_log2(u2.x), __builtin_amdgcn_logf_or_log2(u2.y)} * kLn2;
  const pf2 l2 = lu2 + (q2 - (u2 - 1.0f)) * (rz * x); // log1p(d/x)
  const pf2 r2 = r * r, rz2 = rz * rz;
  const pf2 sr = r * (0.0833333333333333333f - r2 * (0.00277777777777777778f - r2 * 0.000793650793650793651f));
  const pf2 srz = rz * (0.0833333333333333333f - rz2 * (0.00277777777777777778f - rz2 * 0.000793650793650793651f));
  const pf2 lam = (d - 0.5f) * l1 + x * l2 + (srz - sr);
  const pf2 r4 = r2 * r2, rz4 = rz2 * rz2;
  const pf2 psi = l1 - 0.5f * (rz - r) - 0.0833333333333333333f * (rz2 - r2)
                  + 0.00833333333333333333f * (rz4 - r4) - 0.00396825396825396825f * (rz4 * rz2 - r4 * r2);
  nchi = d * log1m_lam + lam;
  bc = chi * (psi + log1m_lam);
}

// nb_asym_pair_direct for a chain pair whose deltas are >= 1 on every lane but below kAsymMin on
// some (low coverage): per element, d < kAsymMin is shifted by kShiftN = 2 in closed form --
// A = d (d + 1), A' = 2 d + 1, B = (d + x)(d + x + 1), B' = 2 (d + x) + 1 (nb_shift's products for
// two factors) -- the series evaluated at the shifted argument, the corrections -log(B / A) and
// A'/A - B'/B added where shifted (zero where x == 0, as nb_shift), all in packed fp32
// (PERT_PACKED_SHIFT; 2 v_rcp + 1 v_log per shifted element as nb_shift, no divergent branch).
// Measured in round 6 and off: it compiles to the same 168 VGPRs, and is correct (GPU parity,
// edge, configs and chain suites green with it), but C5's step is 0.7 % and its 250-cell
// shard's 2 % slower (profiles/r06ab) -- every lane of the pair pays the shift's products and
// logarithm, where the per-chain path skips them on the lanes already past the threshold.
PERT_HD void nb_shift_pair_direct(pf2 chi, float D, float x, float invx, float log1m_lam, pf2& nchi, pf2& bc) {
  const pf2 d = chi * D;
  const bool s0 = d.x < kAsymMin, s1 = d.y < kAsymMin;
  const pf2 ds = {s0 ? d.x + kShift : d.x, s1 ? d.y + kShift : d.y};
  // the series at ds (nb_asym_pair_direct's arithmetic)
  const pf2 r = {frcp(ds.x), frcp(ds.y)};
  const pf2 zs = ds + x;
  const pf2 rz = {frcp(zs.x), frcp(zs.y)};
  const pf2 q = r * x;
  const pf2 iu = ds * rz;
  const pf2 u = q + 1.0f;
  const pf2 lu = pf2{__builtin_amdgcn_logf_or_log2(u.x), __builtin_amdgcn_logf_or_log2(u.y)} * kLn2;
  const pf2 l1 = lu + (q - (u - 1.0f)) * iu;
  const pf2 q2 = ds * invx;
  const pf2 u2 = q2 + 1.0f;
  const pf2 lu2 = pf2{__builtin_amdgcn_logf_or_log2(u2.x), __builtin_amdgcn_logf_or_log2(u2.y)} * kLn2;
  const pf2 l2 = lu2 + (q2 - (u2 - 1.0f)) * (rz * x);
  const pf2 r2 = r * r, rz2 = rz * rz;
  const pf2 sr = r * (0.0833333333333333333f - r2 * (0.00277777777777777778f - r2 * 0.000793650793650793651f));
  const pf2 srz = rz * (0.0833333333333333333f - rz2 * (0.00277777777777777778f - rz2 * 0.000793650793650793651f));
  pf2 lam = (ds - 0.5f) * l1 + x * l2 + (srz - sr);
  const pf2 r4 = r2 * r2, rz4 = rz2 * rz2;
  pf2 psi = l1 - 0.5f * (rz - r) - 0.0833333333333333333f * (rz2 - r2)
            + 0.00833333333333333333f * (rz4 - r4) - 0.00396825396825396825f * (rz4 * rz2 - r4 * r2);
  // the shift's corrections at d (2 factors)
  const pf2 A = d * (d + 1.0f), Ap = 2.0f * d + 1.0f;
  const pf2 b = d + x;
  const pf2 B = b * (b + 1.0f), Bp = 2.0f * b + 1.0f;
  const pf2 rA = {frcp(A.x), frcp(A.y)}, rB = {frcp(B.x), frcp(B.y)};
  const pf2 BA = B * rA;
  const pf2 cl = pf2{__builtin_amdgcn_logf_or_log2(BA.x), __builtin_amdgcn_logf_or_log2(BA.y)} * -kLn2;
  const pf2 cp = Ap * rA - Bp * rB;
  const bool xp = x > 0.0f;
  lam += pf2{(s0 && xp) ? cl.x : 0.0f, (s1 && xp) ? cl.y : 0.0f};
  psi += pf2{(s0 && xp) ? cp.x : 0.0f, (s1 && xp) ? cp.y : 0.0f};
  nchi = d * log1m_lam + lam;
  bc = chi * (psi + log1m_lam);
}

// 1 <= d < kAsymMin: shift by exactly kShiftN = 2 (d + 2 >= 3 for every d >= 1, so no per-lane
// shift count) with the products A = prod_{i<2} (d+i), B = prod_{i<2} (d+x+i) and their
// d-derivatives carried along (one fma + one mul per factor, no per-factor reciprocal):
//   lgamma(d+x) - lgamma(d) = [lgamma(d+2+x) - lgamma(d+2)] - log(B / A)
//   psi(d+x) - psi(d)       = [psi(d+2+x) - psi(d+2)] - B'/B + A'/A
// B / A <= (1 + x)^2, so nothing overflows for any count x < 1e19, and x = 0 gives exactly zero
// corrections (2 v_rcp + 1 v_log per shifted argument).
PERT_HD void nb_shift(float d, float x, float& corr_l, float& corr_p) {
  float A = 1.0f, Ap = 0.0f, B = 1.0f, Bp = 0.0f;
#pragma unroll
  for (int i = 0; i < kShiftN; ++i) {
    const float a = d + (float)i;
    const float b = a + x;
    Ap = Ap * a + A;
    A *= a;
    Bp = Bp * b + B;
    B *= b;
  }
  const float rA = frcp(A);
  corr_l = -flog(B * rA);
  corr_p = Ap * rA - Bp * frcp(B);
  // x = 0: B = A, so both corrections are exactly 0 (fma contraction would leave ~1 ulp)
  corr_l = x > 0.0f ? corr_l : 0.0f;
  corr_p = x > 0.0f ? corr_p : 0.0f;
}

PERT_HD void nb_lgdiff(float d, float x, float invx, float& lam, float& psi) {
  float corr_l = 0.0f, corr_p = 0.0f;
  if (d < kAsymMin) {
    nb_shift(d, x, corr_l, corr_p);
    d += kShift;
  }
  nb_lgdiff_asym(d, x, invx, lam, psi);
  lam += corr_l;
  psi += corr_p;
}

// Lambda(1, x) = lgamma(1 + x) - (x log x - x): parameter free (delta clamped to 1).
// x >= 8: 1/2 log(2 pi x) + S(x); small integer x: exact table; otherwise the shift path.
PERT_HD float lambda_delta1(float x, float invx) {
  if (x >= 8.0f) return kHalfLog2Pi + 0.5f * flog(x) + stirling_rem(invx);
  const float xi = floorf(x);
  if (xi == x) {
    // lgamma(1 + k) - (k log k - k), k = 0..7 (select chain: no indexed local array)
    float v = 0.0f;
    v = (xi == 1.0f) ? 1.000000000e+00f : v;
    v = (xi == 2.0f) ? 1.306852819e+00f : v;
    v = (xi == 3.0f) ? 1.495922603e+00f : v;
    v = (xi == 4.0f) ? 1.632876386e+00f : v;
    v = (xi == 5.0f) ? 1.740302181e+00f : v;
    v = (xi == 6.0f) ? 1.828694397e+00f : v;
    v = (xi == 7.0f) ? 1.903790318e+00f : v;
    return v;
  }
  float lam, psi;
  nb_lgdiff(1.0f, x, invx, lam, psi);
  return lam;
}

// log(k) for k = 0..31 (k = 0 unused)
constexpr float kLogInt[32] = {
    0.0f, 0.0f, 0.693147180559945f, 1.098612288668110f, 1.386294361119891f, 1.609437912434100f,
    1.791759469228055f, 1.945910149055313f, 2.079441541679836f, 2.197224577336220f, 2.302585092994046f,
    2.397895272798371f, 2.484906649788000f, 2.564949357461537f, 2.639057329615259f, 2.708050201102210f,
    2.772588722239781f, 2.833213344056216f, 2.890371757896165f, 2.944438979166440f, 2.995732273553991f,
    3.044522437723423f, 3.091042453358316f, 3.135494215929150f, 3.178053830347946f, 3.218875824868201f,
    3.258096538021482f, 3.295836866004329f, 3.332204510175204f, 3.367295829986474f, 3.401197381662155f,
    3.433987204485146f};

// Number of CN states P is a compile-time constant of every kernel; chi = c (1 + r)
// takes the values 0..P-1 (r = 0) and the even values 0..2P-2 (r = 1).
template <int P>
PERT_HD constexpr bool chi_needed(int chi) { return chi < P || (chi % 2) == 0; }

// ----------------------------------------------------------------- enumerated cell.bin
// One (bin, cell) of the step-2/3 enumerated log joint: forward, responsibilities
// and the analytic backward.  Split in two so a kernel can
// keep few arrays live: enum_forward needs only the pi logits z; enum_tail adds
// the Dirichlet terms once eta (em1 = eta - 1, S1 = sum em1) is at hand.
template <int P>
struct EnumFwd {
  float E;        // logsumexp_{c,r} s(c, r)                        (pert_model.py:607-646, B.1)
  float gD;       // dE/dD, D = u omega (1-lam)/lam                 (delta = chi D, mask delta >= 1)
  float gt;       // dE/dt / a, t = tau - rho                        (masked where phi clamped)
  float zmax;     // max_k z_k
  float lse1p;    // log1p(sum_{k != argmax} exp(z_k - zmax)) -> log pi_k = z_k - zmax - lse1p
  float sgm;      // sum_k gamma^cn_k [pi_k unclamped]
  float pi[P];    // softmax(z)
  float gcm[P];   // gamma^cn_k [pi_k unclamped]
  int argmax;     // r * P + c of the joint MAP state               (infer_discrete, B.7)
  int jmax;       // first argmax_k z_k (torch max, SoftmaxTransform)
  float om;       // 1 - pi_jmax summed from the other states (not rounded through pi_jmax ~ 1)
};

// d(-ELBO)/dz of the argmax logit as minus the sum of the other logits' (a softmax gradient
// sums to zero over the states):
//   sum_{k != jmax} (W_k + gcm_k) - (S1 + sgm) (1 - pi_jmax),   W = eta - 1, S1 = sum W,
// with 1 - pi_jmax = om summed from the other states.  This is the value the reference's fp32
// autograd delivers through SoftmaxTransform's max subtraction (transforms.py:951-954: the
// gradient of the max term lands on the argmax logit and cancels the rounding of the direct
// path), and it stays accurate where fp32 pi_jmax has rounded to 1: the per-element form
// pi_k (S1 + sgm) - W_k - gcm_k quantises W (1 - pi_jmax) to multiples of W eps32 there and
// stops the prior's pull on a saturated state (tools/stop_probe.py: a fit with that form
// stops 27 iterations later than the reference's on the genome-length fixture).
template <int P>
PERT_HD float jmax_grad(int jmax, const float (&em)[P + 1], const float* gcm, float sgm, float om) {
  float wj = 0.0f, gj = 0.0f;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    wj = (k == jmax) ? em[k] : wj;
    gj = (k == jmax) ? gcm[k] : gj;
  }
  const float S1 = em[P];
  return ((S1 - wj) + (sgm - gj)) - (S1 + sgm) * om;
}

template <int P, bool WANT_GRAD, bool WANT_ARGMAX>
PERT_HD void enum_forward(float x, float invx, const float (&z)[P], float log1m_lam, float D,
                          float phi_raw, EnumFwd<P>& o) {
  // Bernoulli(phi) with the in-place clamps of pert_model.py:622-623
  float phic = phi_raw;
  bool mphi = true;
  if (phic < 0.001f) { phic = 0.001f; mphi = false; }
  if (phic > 0.999f) { phic = 0.999f; mphi = false; }
  const float lphi = flog(phic);
  const float l1mphi = flog(1.0f - phic);

  // pi = softmax(z) (SoftmaxTransform, transforms.py:951-954) and the Categorical log
  // pmf log(clamp_probs(pi)) (categorical.py:67-71, utils.py clamp_probs)
  float m = z[0];
  int jmax = 0;
#pragma unroll
  for (int k = 1; k < P; ++k) { if (z[k] > m) { m = z[k]; jmax = k; } }
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    o.pi[k] = (k == jmax) ? 1.0f : fexp(z[k] - m);
    t += (k == jmax) ? 0.0f : o.pi[k];
  }
  const float inv1t = frcp(1.0f + t);
  const float lse1p = log1p_corr(t, inv1t);
  o.zmax = m;
  o.lse1p = lse1p;
  o.jmax = jmax;
  o.om = t * inv1t;
  // joint scores s(c, r): r-major like the oracle's (2, P) layout
  float s[2 * P];
  uint32_t mk = 0;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const float e = o.pi[k];
    const float pk = e * inv1t;
    o.pi[k] = pk;
    const float om = (k == jmax) ? t * inv1t : 1.0f - pk;
    const bool hi = om < kEps32;
    const bool lo = pk < kEps32;
    mk |= (hi || lo) ? 0u : (1u << k);
    const float lc = hi ? kLog1mEps32 : (lo ? kLogEps32 : (z[k] - m) - lse1p);
    s[k] = lc + l1mphi;
    s[P + k] = lc + lphi;
  }

  // negative-binomial part per distinct chi, folded straight into the scores
  const float n_clamped = log1m_lam + lambda_delta1(x, invx);   // delta == 1 (chi == 0 or chi D < 1)
  float Bc[2 * P - 1];
  s[0] += n_clamped;
  s[P] += n_clamped;
  Bc[0] = 0.0f;
  if (D >= kAsymMin) {
    // every delta = chi D >= kAsymMin: straight-line asymptotic series, no clamp, no shift --
    // one basic block, so the 2P-2 independent chains interleave (ILP)
    const float rD = frcp(D);
    const float ldx = x > 0.0f ? flog(D) - flog(x) : 0.0f;
#pragma unroll
    for (int chi = 1; chi < 2 * P - 1; ++chi) {
      if (!chi_needed<P>(chi)) continue;
      const float d = (float)chi * D;
      float lam, psi;
      nb_lgdiff_asym_hoisted(d, rD * (1.0f / (float)chi), x, ldx + kLogInt[chi], lam, psi);
      const float nchi = d * log1m_lam + lam;
      Bc[chi] = (float)chi * (log1m_lam + psi);
      if (chi < P) s[chi] += nchi;
      if ((chi % 2) == 0) s[P + chi / 2] += nchi;
    }
  } else {
#pragma unroll
    for (int chi = 1; chi < 2 * P - 1; ++chi) {
      if (!chi_needed<P>(chi)) continue;
      const float d = (float)chi * D;
      float nchi;
      if (d < 1.0f) {
        nchi = n_clamped;
        Bc[chi] = 0.0f;
      } else {
        float lam, psi;
        nb_lgdiff(d, x, invx, lam, psi);
        nchi = d * log1m_lam + lam;
        Bc[chi] = (float)chi * (log1m_lam + psi);
      }
      if (chi < P) s[chi] += nchi;
      if ((chi % 2) == 0) s[P + chi / 2] += nchi;
    }
  }

  float smax = -INFINITY;
  int amax = 0;
#pragma unroll
  for (int i = 0; i < 2 * P; ++i) { if (s[i] > smax) { smax = s[i]; amax = i; } }
  if (WANT_ARGMAX) o.argmax = amax;
  if (!WANT_GRAD) { o.E = smax; return; }
  float se = 0.0f;
#pragma unroll
  for (int i = 0; i < 2 * P; ++i) { s[i] = fexp(s[i] - smax); se += s[i]; }
  const float inv_se = frcp(se);
  o.E = smax + flog(se);

  float gD = 0.0f, g1 = 0.0f, sgm = 0.0f;
#pragma unroll
  for (int c = 0; c < P; ++c) {
    const float g0c = s[c] * inv_se, g1c = s[P + c] * inv_se;
    gD += g0c * Bc[c] + g1c * Bc[2 * c];
    g1 += g1c;
    const float gm = ((mk >> c) & 1u) ? g0c + g1c : 0.0f;
    o.gcm[c] = gm;
    sgm += gm;
  }
  o.gD = gD;
  o.gt = mphi ? (g1 - phic) : 0.0f;
  o.sgm = sgm;
}

// ----------------------------------------------------------------- enumerated cell.bin, online form
// The same per-(bin, cell) arithmetic as enum_forward, arranged for the streamed pass
// (enum3_kernel) so that no per-state array is ever live: the log pi~ part of every score is
// formed first (from z), then the chi chains of the NB part run in groups of G and each
// group's scores are folded into a running logsumexp at once,
//   M <- max(M, max_group s),  acc <- acc exp(M_old - M) + sum_group exp(s - M),
// for acc = (sum e, sum e Bc, sum_{r=1} e, e per cn state); the scores and the per-chi delta
// derivatives Bc = chi (log(1-lam) + Psi) die with their group.  M ends as the exact max of
// the 2P scores (the logsumexp offset of pert_model.py's enumeration), so E = M + log(sum e)
// differs from enum_forward by rounding only.  The chains of a group interleave; a
// scheduling barrier between groups bounds the live temporaries (three waves per SIMD).

template <int I, int N, class F>
PERT_HD void pert_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    pert_static_for<I + 1, N>(f);
  }
}

template <int P>
struct ChiList {                 // the chi values the 2P states use, increasing
  int v[2 * P - 1];
  int n;
  constexpr ChiList() : v{}, n(0) {
    for (int chi = 0; chi < 2 * P - 1; ++chi)
      if (chi_needed<P>(chi)) v[n++] = chi;
  }
  // does a chain among the first `upto` touch cn state c (as (c, 0) or (c, 1))?
  constexpr bool touches(int upto, int c) const {
    for (int i = 0; i < upto && i < n; ++i)
      if (v[i] == c || v[i] == 2 * c) return true;
    return false;
  }
};

template <int P>
struct EnumOnline {
  float E;        // logsumexp_{c,r} s(c, r)
  float gD;       // dE/dD
  float gt;       // dE/dt / a (masked where phi clamped)
  float zmax;     // max_k z_k
  float zmaxS;    // zmax log2(e)
  float lse1p;    // log sum_k exp(z_k - zmax): log pi_k = z_k - zmax - lse1p
  float inv1t;    // 1 / sum_k exp(z_k - zmax): pi_k = exp(z_k - zmax) inv1t
  float sgm;      // sum_k gcm_k
  float gcm[P];   // gamma^cn_k [pi_k unclamped]
  int argmax;     // r * P + c of the joint MAP state (first maximum)
};

// ---- the Dirichlet site's VALUE as the reference's fp32 arithmetic forms it
// (torch.distributions.Dirichlet.log_prob: xlogy(eta - 1, pi).sum(-1) + lgamma(eta.sum(-1))
//  - lgamma(eta).sum(-1), per (bin, cell) element, fp32).  Two roundings matter for the loss
// record the stopping rule reads:
//  * pi_jmax is fl(1 / s), s = the fp32 row sum of exp(z - max) with exp(0) = 1 for the argmax,
//    so near saturation log pi_jmax moves in steps of ~2^-24 (and is 0 once s rounds to 1);
//  * lgamma(sum eta) ~ 1.3e7 for the weight-1e6 priors (ulp 1): the element's value is rounded
//    to that grid before any sum, and where thousands of elements' logits move in lockstep
//    (late iterations) the reference's loss falls in steps of ~3.5e5 (tools/stop_probe.py).
// The kernels add q = fl(xs + A) - A per element (A = the row's fp32 lgamma(sum eta), the eta
// table's last column; 0 keeps xs unrounded) and the host the rows' fp32 lgamma(sum eta) -
// sum lgamma(eta) (EtaCodebook.dirichlet_normaliser "torch32"): fl(fl(xs + A) - B) = q + (A - B)
// exactly (both differences are exact: Sterbenz).

// torch's CPU order for the fp32 sum of a contiguous row of P values (reduce over the last
// dim; tests/test_dirichlet_value.py pins it): elements 8 .. P-1 first, then 0 .. 7, one
// rounding per addition, for 9 <= P <= 15; 4 .. 0 .. 3 for P = 5; sequential otherwise (the
// sequential order is exact for P <= 4 and P = 8, approximate for P = 6, 7, 16).
template <int P>
PERT_HD constexpr int torch_row_sum_index(int i) {
  constexpr int split = (P >= 9 && P <= 15) ? 8 : (P == 5 ? 4 : 0);
  return i < P - split ? split + i : i - (P - split);
}

// log of the reference's fp32 pi_jmax = fl(exp(0) / s) (SoftmaxTransform, transforms.py:951-954)
// from s, the row sum in torch's order.  Where the rounding of pi matters -- the saturated
// elements, whose logits move in lockstep -- s = 1 + ds with ds a few 2^-23 and fl(1 / s) is
// exactly 1 - ds (for ds < 2^-13 the ds^2 term is below half an ulp of 1 - ds), so
// log pi = log(1 - ds) by its series (|error| < ds^5 / 5); above, -log(s), which differs from
// log(fl(1 / s)) by the quotient's rounding only (<= 2^-24 relative, no lockstep there).
PERT_HD float ref_log_pi_from_sum(float s) {
  const float ds = s - 1.0f;                           // exact (s in [1, P])
  return ds < 1.220703125e-4f ? -ds * (1.0f + ds * (0.5f + ds * (0.33333334f + 0.25f * ds))) : -flog(s);
}

template <int P>
PERT_HD float ref_log_pi_jmax(const float (&z)[P], float zmax, int jmax) {
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int k = torch_row_sum_index<P>(i);
    s += (k == jmax) ? 1.0f : fexp(z[k] - zmax);
  }
  return ref_log_pi_from_sum(s);
}

// q = fl(xs + A) - A: xs rounded to the grid of the row's fp32 lgamma(sum eta) (A = 0: xs)
PERT_HD float dir_site_round(float xs, float A) {
  float t = xs + A;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(t));                          // keep the two roundings apart
#endif
  return t - A;
}

// The argmax logit (first maximum, as torch's max) and 1 - pi_jmax summed from the other
// states (jmax_grad), from the logits and the EnumOnline summary -- evaluated where the
// gradient is formed (the passes' tails), so neither is live through the NB chains.
// lpj: the reference's fp32 log pi_jmax (ref_log_pi_from_sum), from the same exponentials.
template <int P>
PERT_HD void enum_jmax(const float (&z)[P], const EnumOnline<P>& o, int& jmax, float& om, float& lpj) {
  float m = z[0];
  jmax = 0;
#pragma unroll
  for (int k = 1; k < P; ++k) {
    jmax = z[k] > m ? k : jmax;
    m = fmaxf(m, z[k]);
  }
  // the exponentials are enum_pi's (shared with the tail's pi_k): 2^(z_k log2e - fl(m log2e)),
  // i.e. torch's exp(z_k - m) scaled by c = 2^d, d = m log2e - fl(m log2e) (|d| < 2^-20); the
  // argmax adds exactly 1 to the row sum, as torch's exp(0)
  float t = 0.0f, s = 0.0f;
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int k = torch_row_sum_index<P>(i);
    const float e = fexp2(fmaf(z[k], kLog2e, -o.zmaxS));
    t += (k == jmax) ? 0.0f : e;
    s += (k == jmax) ? 1.0f : e;
  }
  // 1 - pi_jmax = the other states' pi_k summed: t = c S and inv1t = 1 / (c (1 + S)) carry the
  // same scale c (enum_online's total includes the argmax's 2^d), so t inv1t = S / (1 + S) and
  // the argmax logit's gradient is minus the sum of the others' (enum_pi gives e_k inv1t), as
  // in enum_forward (the lpj row sum s, unscaled, is the reference's own)
  om = t * o.inv1t;
  lpj = ref_log_pi_from_sum(s);
}

// pi_k from the EnumOnline summary (the exponential enum_online summed)
template <int P>
PERT_HD float enum_pi(const EnumOnline<P>& o, float zk, int k) {
  (void)k;
  return fexp2(fmaf(zk, kLog2e, -o.zmaxS)) * o.inv1t;
}

template <int P, int G, bool WANT_GRAD, bool WANT_ARGMAX>
PERT_HD void enum_online(float x, float invx, const float (&z)[P], float log1m_lam, float D, float phi_raw,
                         EnumOnline<P>& o) {
  // Bernoulli(phi) with the in-place clamps of pert_model.py:622-623
  float phic = phi_raw;
  bool mphi = true;
  if (phic < 0.001f) { phic = 0.001f; mphi = false; }
  if (phic > 0.999f) { phic = 0.999f; mphi = false; }
  const float lphi = flog(phic);
  const float l1mphi = flog(1.0f - phic);
  // pi = softmax(z) (transforms.py:951-954) and log(clamp_probs(pi)) (categorical.py:67-71):
  // log pi_k = z_k - m - log(sum_j exp(z_j - m)), clamped to [log eps, log(1 - eps)] (one
  // v_med3); the gradient mask bit is set where the clamp did not bind
  float m = z[0];
#pragma unroll
  for (int k = 1; k < P; ++k) m = fmaxf(m, z[k]);
  const float mS = m * kLog2e;
  float tot = 0.0f;
#pragma unroll
  for (int k = 0; k < P; ++k) tot += fexp2(fmaf(z[k], kLog2e, -mS));
  const float inv_tot = frcp(tot);
  const float lse = flog(tot);
  float lc[P];
  uint32_t mk = 0;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const float l = (z[k] - m) - lse;
    const float c = fmed3(l, kLogEps32, kLog1mEps32);
    mk |= (c == l) ? (1u << k) : 0u;
    lc[k] = c;
  }
  o.zmax = m;
  o.zmaxS = mS;
  o.lse1p = lse;
  o.inv1t = inv_tot;

  const float n_clamped = log1m_lam + lambda_delta1(x, invx);   // delta == 1 (chi == 0 or chi D < 1)
  float M = -INFINITY, se = 0.0f, seB = 0.0f, g1 = 0.0f, best = -INFINITY;
  int bi = 0;
  if (WANT_GRAD) {
#pragma unroll
    for (int c = 0; c < P; ++c) o.gcm[c] = 0.0f;
  }
  constexpr ChiList<P> CL{};
  constexpr int NG = (CL.n + G - 1) / G;

  auto run = [&](auto asym_c) {
    constexpr bool ASYM = decltype(asym_c)::value;
    float rD = 0.0f, ldx = 0.0f;
    if (ASYM) {
      rD = frcp(D);
      ldx = x > 0.0f ? flog(D) - flog(x) : 0.0f;
    }
    pert_static_for<0, NG>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
#if defined(__HIP_DEVICE_COMPILE__)
      if (g > 0) __builtin_amdgcn_sched_barrier(0);
#endif
      // the group's NB parts; on the asymptotic path two chains per packed-fp32 evaluation
      float nn[G], bb[G];
      bool pdone[(G + 1) / 2];                              // (low coverage) pair taken packed
      if constexpr (!ASYM) {
        pert_static_for<0, (G + 1) / 2>([&](auto pc) {
          constexpr int j0 = 2 * decltype(pc)::value, j1 = j0 + 1;
          constexpr int i0 = g * G + j0, i1 = g * G + j1;
          constexpr bool h0 = i0 < CL.n, h1 = j1 < G && i1 < CL.n;
          constexpr int c0 = h0 ? CL.v[i0] : 1, c1 = h1 ? CL.v[i1] : 1;
          pdone[decltype(pc)::value] = false;
          if constexpr (h0 && h1 && c0 != 0) {
            if (wave_all((float)c0 * D >= kAsymMin)) {     // both chains past the shift on every lane
              pf2 n2, b2;
              nb_asym_pair_direct(pf2{(float)c0, (float)c1}, D, x, invx, log1m_lam, n2, b2);
              nn[j0] = n2.x;
              bb[j0] = b2.x;
              nn[j1] = n2.y;
              bb[j1] = b2.y;
              pdone[decltype(pc)::value] = true;
            }
#if PERT_PACKED_SHIFT
            else if (wave_all((float)c0 * D >= 1.0f)) {   // no clamp on any lane: shifted where needed
              pf2 n2, b2;
              nb_shift_pair_direct(pf2{(float)c0, (float)c1}, D, x, invx, log1m_lam, n2, b2);
              nn[j0] = n2.x;
              bb[j0] = b2.x;
              nn[j1] = n2.y;
              bb[j1] = b2.y;
              pdone[decltype(pc)::value] = true;
            }
#endif
          }
        });
      }
      if constexpr (ASYM) {
        pert_static_for<0, (G + 1) / 2>([&](auto pc) {
          constexpr int j0 = 2 * decltype(pc)::value, j1 = j0 + 1;
          constexpr int i0 = g * G + j0, i1 = g * G + j1;
          constexpr bool h0 = i0 < CL.n, h1 = j1 < G && i1 < CL.n;
          constexpr int c0 = h0 ? CL.v[i0] : 1, c1 = h1 ? CL.v[i1] : 1;
          if constexpr (h0 && h1 && c0 != 0) {
            pf2 n2, b2;
            nb_asym_pair(pf2{(float)c0, (float)c1}, pf2{1.0f / (float)c0, 1.0f / (float)c1},
                         pf2{kLogInt[c0], kLogInt[c1]}, D, rD, x, ldx, log1m_lam, n2, b2);
            nn[j0] = n2.x;
            bb[j0] = b2.x;
            nn[j1] = n2.y;
            bb[j1] = b2.y;
          }
        });
      }
      pert_static_for<0, G>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int idx = g * G + j;
        constexpr int jp = j - j % 2;                          // pair head
        constexpr bool pairable = jp + 1 < G && g * G + jp + 1 < CL.n && CL.v[g * G + jp] != 0;
        constexpr bool paired = ASYM && pairable;
        if constexpr (!ASYM && pairable && idx < CL.n) {
          if (pdone[j / 2]) return;                          // (wave-uniform)
        }
        if constexpr (idx < CL.n && !paired) {
          constexpr int chi = CL.v[idx];
          if constexpr (chi == 0) {
            nn[j] = n_clamped;
            bb[j] = 0.0f;
          } else {
            const float d = (float)chi * D;
            float lam, psi;
            if constexpr (ASYM) {
              nb_lgdiff_asym_hoisted(d, rD * (1.0f / (float)chi), x, ldx + kLogInt[chi], lam, psi);
              nn[j] = d * log1m_lam + lam;
              bb[j] = (float)chi * (log1m_lam + psi);
            } else {
              if (d < 1.0f) {
                nn[j] = n_clamped;
                bb[j] = 0.0f;
              } else {
                nb_lgdiff(d, x, invx, lam, psi);
                nn[j] = d * log1m_lam + lam;
                bb[j] = (float)chi * (log1m_lam + psi);
              }
            }
          }
        }
      });
      // the group's scores: chain chi feeds (chi, 0) when chi < P and (chi / 2, 1) when even
      float sg[2 * G];
      float mg = -INFINITY;
      pert_static_for<0, G>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int idx = g * G + j;
        if constexpr (idx < CL.n) {
          constexpr int chi = CL.v[idx];
          if constexpr (chi < P) {
            sg[2 * j] = nn[j] + lc[chi] + l1mphi;
            mg = fmaxf(mg, sg[2 * j]);
            if (WANT_ARGMAX && (sg[2 * j] > best || (sg[2 * j] == best && chi < bi))) { best = sg[2 * j]; bi = chi; }
          }
          if constexpr (chi % 2 == 0) {
            sg[2 * j + 1] = nn[j] + lc[chi / 2] + lphi;
            mg = fmaxf(mg, sg[2 * j + 1]);
            if (WANT_ARGMAX && (sg[2 * j + 1] > best || (sg[2 * j + 1] == best && P + chi / 2 < bi))) {
              best = sg[2 * j + 1];
              bi = P + chi / 2;
            }
          }
        }
      });
      if (!WANT_GRAD) {
        M = fmaxf(M, mg);
        return;
      }
      float Mn = mg;
      if constexpr (g > 0) {
        Mn = fmaxf(M, mg);
        const float sc = fexp(M - Mn);
        se *= sc;
        seB *= sc;
        g1 *= sc;
        pert_static_for<0, P>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          if constexpr (CL.touches(g * G, c)) o.gcm[c] *= sc;
        });
      }
      M = Mn;
      const float ML = M * kLog2e;
      pert_static_for<0, G>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int idx = g * G + j;
        if constexpr (idx < CL.n) {
          constexpr int chi = CL.v[idx];
          float ej = 0.0f;
          if constexpr (chi < P) {
            const float e = fexp2(fmaf(sg[2 * j], kLog2e, -ML));
            ej += e;
            o.gcm[chi] += e;
          }
          if constexpr (chi % 2 == 0) {
            const float e = fexp2(fmaf(sg[2 * j + 1], kLog2e, -ML));
            ej += e;
            g1 += e;
            o.gcm[chi / 2] += e;
          }
          se += ej;
          seB += ej * bb[j];
        }
      });
    });
  };
  if (D >= kAsymMin) run(std::true_type{});
  else run(std::false_type{});

  if (WANT_ARGMAX) o.argmax = bi;
  if (!WANT_GRAD) {
    o.E = M;
    return;
  }
  const float inv_se = frcp(se);
  o.E = M + flog(se);
  o.gD = seB * inv_se;
  o.gt = mphi ? (g1 * inv_se - phic) : 0.0f;
  float sgm = 0.0f;
#pragma unroll
  for (int c = 0; c < P; ++c) {
    const float gm = ((mk >> c) & 1u) ? o.gcm[c] * inv_se : 0.0f;
    o.gcm[c] = gm;
    sgm += gm;
  }
  o.sgm = sgm;
}

// Dirichlet(eta) variable part sum_k (eta_k - 1) log pi_k and d(E + dirv)/dz_k, the
// (eta_k - 1) - pi_k S1 term in the cancellation-free form of SURVEY.md Appendix C.
template <int P>
PERT_HD float enum_tail(const EnumFwd<P>& o, const float (&z)[P], const float (&em1)[P], float S1,
                        float (&gz)[P]) {
  float dirv = 0.0f;
  float em[P + 1];
  const float lpj = ref_log_pi_jmax<P>(z, o.zmax, o.jmax);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    dirv += em1[k] * ((k == o.jmax) ? lpj : (z[k] - o.zmax) - o.lse1p);
    gz[k] = em1[k] - o.pi[k] * S1 + o.gcm[k] - o.pi[k] * o.sgm;
    em[k] = em1[k];
  }
  em[P] = S1;
  const float gj = -jmax_grad<P>(o.jmax, em, o.gcm, o.sgm, o.om);
#pragma unroll
  for (int k = 0; k < P; ++k) gz[k] = (k == o.jmax) ? gj : gz[k];
  return dirv;
}

template <int P>
struct EnumOut {
  float E, dirv, gD, gt;
  float gz[P];
  int argmax;
};

template <int P, bool WANT_GRAD, bool WANT_ARGMAX>
PERT_HD void enum_cellbin(float x, float invx, const float (&em1)[P], float S1, const float (&z)[P],
                          float log1m_lam, float D, float phi_raw, EnumOut<P>& out) {
  EnumFwd<P> o;
  enum_forward<P, WANT_GRAD, WANT_ARGMAX>(x, invx, z, log1m_lam, D, phi_raw, o);
  out.E = o.E;
  out.argmax = WANT_ARGMAX ? o.argmax : 0;
  if (WANT_GRAD) {
    out.gD = o.gD;
    out.gt = o.gt;
    out.dirv = enum_tail<P>(o, z, em1, S1, out.gz);
  }
}

// ----------------------------------------------------------------- observed cell.bin (step 1)
// NB + Bernoulli terms with cn / rep observed (pert_model.py:724-729, JitTrace_ELBO).
struct ObsOut {
  float ll;      // delta log(1-lam) + Lambda(delta, x) + log Bern(rep | phi)
  float gD;      // d ll / dD            (chi (log(1-lam) + Psi) masked on delta >= 1)
  float dsum;    // delta (clamped value) -- d/dlam of delta log(1-lam) is -delta/(1-lam)
  float gdd;     // (log(1-lam) + Psi) delta, masked -- enters d/dlam through ddelta/dlam
  float gt;      // d ll / dt / a
};

PERT_HD void obs_cellbin(float x, float invx, float cn, float rep, float log1m_lam, float D,
                         float phi_raw, ObsOut& o) {
  float phic = phi_raw;
  bool mphi = true;
  if (phic < 0.001f) { phic = 0.001f; mphi = false; }
  if (phic > 0.999f) { phic = 0.999f; mphi = false; }
  o.ll = rep > 0.5f ? flog(phic) : flog(1.0f - phic);
  o.gt = mphi ? (rep - phic) : 0.0f;
  const float chi = cn * (1.0f + rep);
  float d = chi * D;
  float lam, psi;
  if (d < 1.0f) {
    nb_lgdiff(1.0f, x, invx, lam, psi);
    o.ll += log1m_lam + lam;
    o.gD = 0.0f;
    o.gdd = 0.0f;
    o.dsum = 1.0f;
  } else {
    nb_lgdiff(d, x, invx, lam, psi);
    o.ll += d * log1m_lam + lam;
    const float g = log1m_lam + psi;
    o.gD = chi * g;
    o.gdd = d * g;
    o.dsum = d;
  }
}

// Step 1 in pair mode (pert_hip.h): the two copies of one G1/2 cell.bin -- rep 0 and rep 1,
// chi = (cn, 2 cn), each copy with its own D = u omega (1-lam)/lam and phi -- together in packed
// fp32 (v_pk_fma / mul / add_f32: both copies per VALU issue; transcendentals stay per element).
// The same terms as obs_cellbin for each copy.  Where both copies have delta >= kAsymMin (every
// copy with cn > 0 at 500 kb coverage) the asymptotic series runs packed; any other pair takes
// obs_cellbin per copy (clamped / shifted delta).
struct ObsPairOut {
  pf2 ll, gD, dsum, gdd, gt;
};

PERT_HD void obs_pair_cellbin(float x, float invx, float cn, float log1m_lam, pf2 D, pf2 phi, ObsPairOut& o) {
  const pf2 chi = {cn, 2.0f * cn};
  const pf2 d = chi * D;
  pf2 ll, gD, dsum, gdd, gt;
  if (d.x >= kAsymMin && d.y >= kAsymMin) {
    // Bernoulli(phi) of rep 0 / rep 1 with the clamps of pert_model.py:622-623
    const pf2 phic = {fmed3(phi.x, 0.001f, 0.999f), fmed3(phi.y, 0.001f, 0.999f)};
    const pf2 lb = pf2{__builtin_amdgcn_logf_or_log2(1.0f - phic.x), __builtin_amdgcn_logf_or_log2(phic.y)} * kLn2;
    gt = pf2{phic.x == phi.x ? -phic.x : 0.0f, phic.y == phi.y ? 1.0f - phic.y : 0.0f};
    const pf2 r = {frcp(d.x), frcp(d.y)};
    const pf2 zs = d + x;
    const pf2 rz = {frcp(zs.x), frcp(zs.y)};
    const pf2 q = r * x;                                // x/d
    const pf2 iu = d * rz;                              // 1/(1 + x/d)
    const pf2 u = q + 1.0f;
    const pf2 lu = pf2{__builtin_amdgcn_logf_or_log2(u.x), __builtin_amdgcn_logf_or_log2(u.y)} * kLn2;
    const pf2 l1 = lu + (q - (u - 1.0f)) * iu;          // log1p(x/d), log1p_corr
    // log1p(d/x), direct (the hoisted log1p(x/d) + log(d/x) cancels where x >> d); 0 when x == 0
    const pf2 q2 = d * invx;
    const pf2 u2 = q2 + 1.0f;
    const pf2 lu2 = pf2{__builtin_amdgcn_logf_or_log2(u2.x), __builtin_amdgcn_logf_or_log2(u2.y)} * kLn2;
    const pf2 l2 = lu2 + (q2 - (u2 - 1.0f)) * (rz * x);
    const pf2 r2 = r * r, rz2 = rz * rz;
    const pf2 sr = r * (0.0833333333333333333f - r2 * (0.00277777777777777778f - r2 * 0.000793650793650793651f));
    const pf2 srz = rz * (0.0833333333333333333f - rz2 * (0.00277777777777777778f - rz2 * 0.000793650793650793651f));
    const pf2 lam = (d - 0.5f) * l1 + x * l2 + (srz - sr);
    const pf2 r4 = r2 * r2, rz4 = rz2 * rz2;
    const pf2 psi = l1 - 0.5f * (rz - r) - 0.0833333333333333333f * (rz2 - r2)
                    + 0.00833333333333333333f * (rz4 - r4) - 0.00396825396825396825f * (rz4 * rz2 - r4 * r2);
    const pf2 g = psi + log1m_lam;
    ll = lb + (d * log1m_lam + lam);
    gD = chi * g;
    gdd = d * g;
    dsum = d;
  } else {
    ObsOut a;
    obs_cellbin(x, invx, cn, 0.0f, log1m_lam, D.x, phi.x, a);
    const float ll0 = a.ll, gD0 = a.gD, ds0 = a.dsum, gdd0 = a.gdd, gt0 = a.gt;
    obs_cellbin(x, invx, cn, 1.0f, log1m_lam, D.y, phi.y, a);
    ll = pf2{ll0, a.ll};
    gD = pf2{gD0, a.gD};
    dsum = pf2{ds0, a.dsum};
    gdd = pf2{gdd0, a.gdd};
    gt = pf2{gt0, a.gt};
  }
  o.ll = ll;
  o.gD = gD;
  o.dsum = dsum;
  o.gdd = gdd;
  o.gt = gt;
}

// ----------------------------------------------------------------- transforms
// _clipped_sigmoid (torch/distributions/transforms.py:629-631); *mask = 0 where clipped.
PERT_HD float clipped_sigmoid(float zz, float* dmask) {
  float s = frcp(1.0f + fexp(-zz));
  float ds = s * (1.0f - s);
  if (s < kTiny32) { s = kTiny32; ds = 0.0f; }
  if (s > 1.0f - kEps32) { s = 1.0f - kEps32; ds = 0.0f; }
  *dmask = ds;
  return s;
}

}  // namespace pert
