// pert_kernels.hip -- gfx950 kernels of the PERT SVI hot path + the C ABI of include/pert_hip.h.
//
// One SVI step of reference pert_model.py (svi_s.step at :801, svi.step at :743,
// svi_s2.step at :868) becomes:
//   enum3_kernel (default) / enum_dma_kernel (variant 0) / obs_kernel (step 1)
//                              one pass over every (bin, cell): forward, analytic backward,
//                              fused Adam on the (L, P, N) pi logits, reduction partials
//   finalize_kernel            per-cell sums + u / betas / tau priors (:589-603),
//                              per-bin sums for rho (:572-574), and in its last block
//                              the global sums (loss, a, beta_stds, lambda, beta_means)
//   adam_kernel                Adam on the packed non-pi params
// All reductions are fixed-order (no float atomics), so a rerun is bit-identical.
//
// Work decomposition of the enumerated passes: one wave per workgroup = 64 cells (one per
// lane) x LT bins (obs_kernel: 256 cells x LT bins).  Lanes walk their bins in order;
// per-cell partial sums stay in registers, per-bin sums are wave shuffles.  Every HBM access
// of the (L, N) / (L, P, N) tensors is a contiguous wave access (cells are the fastest axis).

#include "../../include/pert_hip.h"
#include "pert_math.h"

#include <math.h>
#include <stddef.h>
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>

namespace {

using namespace pert;

constexpr int kBlock = PERT_BLOCK;
constexpr int kWaves = kBlock / 64;
constexpr int kDefaultLT = 32;
constexpr int kMaxLT = 64;
#ifndef PERT_ENUM3_ORDER
#define PERT_ENUM3_ORDER 2
#endif
// variant 3's workgroup -> (cell tile, bin tile) order (the dispatcher deals consecutive
// workgroup ids round robin over the 8 XCDs): 0 cell tiles fastest, 1 bin tiles fastest,
// 2 / 3 XCD-aware -- XCD k runs a contiguous eighth of the tiles in bin- / cell-fastest order.
// 2 (default): each XCD streams its own contiguous run of the tile-major z / m / v arrays, bins
// of a cell tile in order; interleaved A/B on one box (profiles/r05f_tile_order_ab.log): C4
// pass 3.444-3.455 vs 3.478-3.481 ms and its pattern ceiling 3.34 vs 3.43 ms, the 1,250-cell
// shard's pass 0.464-0.467 vs 0.468-0.471 ms (order 1 alone: +5 % there, order 3: no gain)
constexpr int kEnum3Order = PERT_ENUM3_ORDER;
constexpr int kShortLT3 = 12;                    // variant 3's tile length on multi-round launches
constexpr int kLongLT3 = 18;                     // ... and on launches of 8 rounds or more
constexpr int kEtaLdsFloats = 1024;   // eta tables up to 4 KB are staged in LDS
// eta table row: eta_k - 1 (k < P), S1 = sum_k (eta_k - 1), A = fp32 lgamma(sum eta) (the grid
// the reference's fp32 Dirichlet value is rounded to; 0: unrounded) -- include/pert_hip.h
__host__ __device__ constexpr int kTabRow(int P) { return P + 2; }
constexpr int kBlkSlots = 4;      // loss, d/da, sum delta, sum gdd (step 1)
constexpr float kHalfLog2PiF = 0.918938533204672742f;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block-wide fixed-order sum; every thread gets the result.
__device__ __forceinline__ double block_sum_d(double v, double* sm) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum_d(v);
  __syncthreads();
  if (lane == 0) sm[wave] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) t += sm[w];
  return t;
}

__device__ __forceinline__ float gamma_lp_a(float a) {
  // Gamma(2, 0.2).log_prob(a) = xlogy(2, 0.2) + xlogy(1, a) - 0.2 a - lgamma(2)   (pert_model.py:553)
  return 2.0f * logf(0.2f) + logf(a) - 0.2f * a;
}

// Device-side SVI loop (include/pert_hip.h): a launch of iteration st.step is a no-op once
// an earlier iteration has stopped the fit.  The flag is written by pert_adam of the stopping
// iteration (a previous launch), so a plain load at kernel start sees it.
__device__ __forceinline__ bool loop_stopped(const pert_state& st) {
  if (st.loop_ctl == nullptr) return false;
  const int s = *(volatile const int32_t*)st.loop_ctl;
  return s >= 0 && s < st.step;
}

// ------------------------------------------------------------------------------------------
// Enumerated pass, LDS-DMA streamed (default).  One wave per workgroup = 64 cells x LT bins.
// Per bin the wave's inputs are contiguous runs in HBM (x 256 B, eta code 128 B, pi logits
// and Adam moments P*256 B each in the wave-tiled layout) and are copied HBM -> LDS by
// global_load_lds (no VGPRs): the inputs of bin l+1 and the Adam moments of bin l are
// in flight while bin l computes.  LDS-DMA completion is ordered for the issuing wave
// by its own vmcnt only (no workgroup barrier is needed with one wave), and hipcc does
// not wait for it on its own, so every wait below is explicit and counted.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// Cache policy of the streamed traffic: every byte of the pi state, reads and eta codes is
// touched once per pass, so the HBM -> LDS copies are non-temporal (aux = 2, `nt`) and so are
// the pi-state stores.  Both together: -1.8 % kernel at C4, -1.6 % at 1,250 cells (A/B on one
// box, two interleaved rounds); either alone is within noise.
#ifndef PERT_DMA_AUX
#define PERT_DMA_AUX 2
#endif
#ifndef PERT_NT_STORE
#define PERT_NT_STORE 1
#endif
// cache policy of enum3's streamed z / m / v (g) stores (gfx950 CPol bits: 1 sc0, 2 nt, 16 sc1);
// A/B knob: 2 = nt (default), 19 = sc0 sc1 nt (written through: no dirty L2 lines left for the
// end-of-kernel release)
#ifndef PERT_STORE_CPOL
#define PERT_STORE_CPOL 2
#endif
__device__ __forceinline__ void store_stream(float* p, float v) {
#if PERT_NT_STORE
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

template <int BYTES>
__device__ __forceinline__ void dma_run(const void* gsrc, float* ldst, int lane) {
  // a contiguous run of BYTES (multiple of 128) -> the same bytes at ldst
  const char* g = (const char*)gsrc;
  constexpr int n16 = BYTES / 1024;
  constexpr int rem = BYTES % 1024;
#pragma unroll
  for (int i = 0; i < n16; ++i)
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g + i * 1024 + lane * 16), (lds_ptr_t)(ldst + i * 256), 16, 0, PERT_DMA_AUX);
  if constexpr (rem >= 256) {
#pragma unroll
    for (int i = 0; i < rem / 256; ++i)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g + n16 * 1024 + i * 256 + lane * 4),
                                       (lds_ptr_t)(ldst + n16 * 256 + i * 64), 4, 0, PERT_DMA_AUX);
  }
  if constexpr (rem % 256 == 128) {
    // 128-B tail: 4-B pieces on half the wave (sub-dword LDS-DMA is not lane-packed)
    if (lane < 32)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(g + BYTES - 128 + lane * 4), (lds_ptr_t)(ldst + (BYTES - 128) / 4), 4, 0, PERT_DMA_AUX);
  }
}

template <int BYTES>
constexpr int dma_count() { return BYTES / 1024 + (BYTES % 1024) / 256 + ((BYTES % 256) == 128 ? 1 : 0); }

// the DMA pass's per-(bin, cell) arithmetic: 1 = enum_online + the packed tail (as enum3_kernel),
// 0 = enum_forward + the scalar tail (A/B knob)
#ifndef PERT_V0_ONLINE
#define PERT_V0_ONLINE 1
#endif
#ifndef PERT_ENUM3_GROUP
#define PERT_ENUM3_GROUP 6
#endif
constexpr int kEnum3Group = PERT_ENUM3_GROUP;   // chi chains interleaved per group (enum_online)

template <int P, int MODE, int K1T>
__global__ void __launch_bounds__(64, 2) enum_dma_kernel(pert_problem pr, pert_state st, pert_adam_hparams hp) {
  constexpr bool kDecode = MODE == PERT_MODE_DECODE;
  constexpr bool kStep = MODE == PERT_MODE_STEP;
  constexpr int ZF = P * 64;                 // floats of one P-plane run
  constexpr int SF = ZF + 64 + 32;           // stage: z, x, code (64 x u16)
  constexpr int kStores = kStep ? 3 * P : (kDecode ? 2 : P);   // VMEM stores per iteration
  if (kStep && loop_stopped(st)) return;
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
  // one dynamic LDS array (16-B aligned base, cdna_hip_programming.md G17):
  //   [stage 0 | stage 1 | m | v (STEP)] [per-bin rho partials: LT] [per-bin rho, gcf: LT x (K1+1)]
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* s_binp = lds + 2 * SF + (kStep ? 2 * ZF : 0);

  const int lane = threadIdx.x;
  const int N = pr.N, K1 = (K1T == PERT_MAX_K1) ? pr.K1 : K1T, ldn = pr.ldn;
  const int wt = blockIdx.x;
  const int n = wt * 64 + lane;
  const bool valid = n < N;
  const int LT = st.bins_per_tile;
  const int l0 = blockIdx.y * LT;
  const int l1 = min(pr.L, l0 + LT);
  const bool frozen = pr.kind == PERT_KIND_STEP3;
  const pert_layout lay = st.lay;
  const size_t bin_stride = (size_t)P * 64;                  // floats per bin of a wave tile
  const size_t toff = (size_t)wt * pr.L * P * 64;

  const float* __restrict__ params = st.params;
  float* s_bc = s_binp + LT;
  // the eta table (n_codes x (P+1)) is staged in LDS when it is small (every builder but a
  // large composite prior): the tail's per-lane row gather is then an LDS read, not a
  // dependent global load after the forward pass
  float* s_tab = s_bc + LT * (K1 + 1);
  const bool etal = !kDecode && pr.n_codes * kTabRow(P) <= kEtaLdsFloats;
  // Tile prologue: every load below is unconditional (clamped index, masked store), so each
  // group is one round trip instead of one guarded load + wait per loop trip.
  if (etal) {
    const int nt = pr.n_codes * kTabRow(P);
    float tv[kEtaLdsFloats / 64];
#pragma unroll
    for (int r = 0; r < kEtaLdsFloats / 64; ++r) tv[r] = pr.eta_table[min(lane + 64 * r, nt - 1)];
#pragma unroll
    for (int r = 0; r < kEtaLdsFloats / 64; ++r)
      if (lane + 64 * r < nt) s_tab[lane + 64 * r] = tv[r];
  }
  // per-bin constants of the tile: constrained rho (one bin per lane, LT <= 64) and the
  // GC features (a contiguous run of nb * K1 floats of gcf)
  {
    const int nb = l1 - l0;
    const int lr = l0 + min(lane, nb - 1);
    const float zr = frozen ? pr.rho_fixed[lr] : params[lay.off_rho + lr];
    const int ng = nb * K1;
    const float* gsrc = pr.gcf + (size_t)l0 * K1;
    float gv[PERT_MAX_K1];
#pragma unroll
    for (int r = 0; r < PERT_MAX_K1; ++r) gv[r] = gsrc[min(lane + 64 * r, ng - 1)];
    if (lane < nb) {
      float dm;
      s_bc[lane * (K1 + 1)] = frozen ? zr : clipped_sigmoid(zr, &dm);
    }
#pragma unroll
    for (int r = 0; r < PERT_MAX_K1; ++r) {
      const int i = lane + 64 * r;
      if (i < ng) {
        const int lb = i / K1, j = i - lb * K1;
        s_bc[lb * (K1 + 1) + 1 + j] = gv[r];
      }
    }
  }
  const float a_val = frozen ? pr.a_fixed : fexp(params[lay.off_a]);
  const float c0 = (1.0f - pr.lamb) / pr.lamb;
  float u = 0.0f, tau = 0.5f;
  float beta[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) beta[k] = 0.0f;
  if (valid) {
    u = st.params[lay.off_u + n];
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) beta[k] = st.params[lay.off_beta + k * N + n];
    float dm;
    tau = clipped_sigmoid(st.params[lay.off_tau + n], &dm);
  }
  const float ucc = u * c0;
  float acc[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) acc[k] = 0.0f;
  float accT = 0.0f, loss = 0.0f, ga = 0.0f;

  auto issue_stage = [&](int l, int buf) {
    float* sb = lds + buf * SF;
    dma_run<P * 256>(st.z_pi + (size_t)l * bin_stride + toff, sb, lane);
    dma_run<256>(pr.reads + (size_t)l * ldn + wt * 64, sb + ZF, lane);
    dma_run<128>(pr.eta_code + (size_t)l * ldn + wt * 64, sb + ZF + 64, lane);
  };
  if (l0 < l1) issue_stage(l0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // variant 2 = diagnostic build of the same kernel: wave timeline stamps (s_memrealtime,
  // 100 MHz) at entry, after the first stage landed and at exit, into the g_pi buffer
  // (unused in STEP mode) -- tools/wave_timeline.py.
  const bool stamps = kStep && st.variant == 2 && st.g_pi != nullptr;
  unsigned long long* dbg = (unsigned long long*)st.g_pi + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4;
  if (stamps && lane == 0) dbg[1] = __builtin_amdgcn_s_memrealtime();
  // Issue priority falls with the wave's progress through its tile (3, 2, 1, 0 by quarters).
  // Arbitration between ready waves of a SIMD is by priority, then age, so at equal priority
  // the older of the two resident waves runs ahead and the younger finishes its tile alone,
  // latency-bound (tools/wave_timeline.py: exits bimodal at 340 / 590 us on a one-round
  // 1,250-cell launch).  Favouring the wave that is behind closes the gap (exit spread
  // 340-590 -> 440-530 us; -3.4 % kernel at 1,250 cells, -0.9 % at 10 k).
  const int nbt = l1 - l0;
  __builtin_amdgcn_s_setprio(3);
  for (int l = l0; l < l1; ++l) {
    const int buf = (l - l0) & 1;
    {
      const int q4 = 4 * (l - l0);
      if (q4 >= nbt && q4 - 4 < nbt) __builtin_amdgcn_s_setprio(2);
      if (q4 >= 2 * nbt && q4 - 4 < 2 * nbt) __builtin_amdgcn_s_setprio(1);
      if (q4 >= 3 * nbt && q4 - 4 < 3 * nbt) __builtin_amdgcn_s_setprio(0);
    }
    // stage(l) was issued one iteration ago; only this wave's stores of bin l-1
    // (kStores, unconditional) may be younger than it
    if (l > l0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kStores) : "memory");
    const float* sb = lds + buf * SF;
    float z[P];
#pragma unroll
    for (int k = 0; k < P; ++k) z[k] = sb[k * 64 + lane];
    const float x = sb[ZF + lane];
    const uint32_t code = ((const uint16_t*)(sb + ZF + 64))[lane];
    // per-bin constants, read before this iteration's DMAs are issued (hipcc waits for
    // every outstanding LDS-DMA before the first LDS read that follows one)
    const float* bcl = s_bc + (l - l0) * (K1 + 1);
    const float rho = bcl[0];
    float g[K1T];
#pragma unroll
    for (int k = 0; k < K1T; ++k) g[k] = (k < K1) ? bcl[1 + k] : 0.0f;
    const size_t tile = (size_t)l * bin_stride + toff;
    if (kStep) {
      dma_run<P * 256>(st.m_pi + tile, lds + 2 * SF, lane);
      dma_run<P * 256>(st.v_pi + tile, lds + 2 * SF + ZF, lane);
    }
    if (l + 1 < l1) issue_stage(l + 1, buf ^ 1);

    const float invx = x > 0.0f ? frcp(x) : 0.0f;
    float dot = 0.0f;
#pragma unroll
    for (int k = 0; k < K1T; ++k) dot += beta[k] * g[k];
    const float omega = fexp(dot);                         // pert_model.py:633
    const float D = ucc * omega;                           // :636-640 (delta = chi D)
    const float t = tau - rho;                             // :616
    const float phi = frcp(1.0f + fexp(-a_val * t));       // :619
#if PERT_V0_ONLINE
    EnumOnline<P> o;
    enum_online<P, kEnum3Group, !kDecode, kDecode>(x, invx, z, pr.log1m_lam, D, phi, o);
#else
    EnumFwd<P> o;
    enum_forward<P, !kDecode, kDecode>(x, invx, z, pr.log1m_lam, D, phi, o);
#endif
    float gtv = 0.0f;
    if (kDecode) {
      st.cn_out[(size_t)l * ldn + n] = (uint8_t)(o.argmax % P);
      st.rep_out[(size_t)l * ldn + n] = (uint8_t)(o.argmax / P);
    } else {
      // Everything the tail needs is re-read from LDS after this point (the asm is a
      // compiler memory barrier, so the pi logits are not kept live through the NB work).
      // (the register operand pins the wait after the whole forward pass)
      if (kStep) asm volatile("s_waitcnt vmcnt(0)" :: "v"(o.E), "v"(o.sgm) : "memory");   // m, v of bin l landed
      else asm volatile("" :: "v"(o.E), "v"(o.sgm) : "memory");
      float zt[P];
#pragma unroll
      for (int k = 0; k < P; ++k) zt[k] = sb[k * 64 + lane];
      float em1[P], S1, Arow;
      if (etal) {
        const float* row = s_tab + code * kTabRow(P);
#pragma unroll
        for (int k = 0; k < P; ++k) em1[k] = row[k];
        S1 = row[P];
        Arow = row[P + 1];
      } else {
        const float* row = pr.eta_table + (size_t)code * kTabRow(P);
#pragma unroll
        for (int k = 0; k < P; ++k) em1[k] = row[k];
        S1 = row[P];
        Arow = row[P + 1];
      }
#if PERT_V0_ONLINE
      // the gradient and Adam of the logits in plane pairs, packed fp32 (as enum3_kernel)
      const float S1s = S1 + o.sgm;
      int jmax;
      float om;
      float lpj;                                            // the reference's fp32 log pi_jmax
      enum_jmax<P>(zt, o, jmax, om, lpj);
      const float tom = S1s * om;                           // (S1 + sgm)(1 - pi_jmax), jmax_grad
      pf2 dirv2 = {0.0f, 0.0f};
      const float* mb = lds + 2 * SF;
      float* zo = st.z_pi + tile + lane;
      float* mo = st.m_pi + tile + lane;
      float* vo = st.v_pi + tile + lane;
      float* gp = st.g_pi + tile + lane;
      pert_static_for<0, (P + 1) / 2>([&](auto pc) {
        constexpr int k0 = 2 * decltype(pc)::value;
        constexpr int k1 = k0 + 1 < P ? k0 + 1 : k0;
        const pf2 zz = {zt[k0], zt[k1]};
        const pf2 e1 = {em1[k0], k1 != k0 ? em1[k1] : 0.0f};
        const pf2 pk = pf2{enum_pi(o, zt[k0], k0), enum_pi(o, zt[k1], k1)};
        dirv2 += e1 * ((zz - o.zmax) - o.lse1p);
        const pf2 gc = pf2{o.gcm[k0], o.gcm[k1]};
        pf2 gl = pk * S1s - e1 - gc;                                  // d(-ELBO)/dz
        const pf2 gj = ((S1 - e1) + (o.sgm - gc)) - tom;              // the argmax logit (jmax_grad)
        gl = pf2{k0 == jmax ? gj.x : gl.x, k1 == jmax ? gj.y : gl.y};
        if (kStep) {
          const pf2 m0 = {mb[k0 * 64 + lane], mb[k1 * 64 + lane]};
          const pf2 v0 = {mb[ZF + k0 * 64 + lane], mb[ZF + k1 * 64 + lane]};
          const pf2 m1 = m0 * hp.beta1 + gl * (1.0f - hp.beta1);
          const pf2 v1 = v0 * hp.beta2 + (gl * gl) * (1.0f - hp.beta2);
          const pf2 den = pf2{__builtin_amdgcn_sqrtf(v1.x), __builtin_amdgcn_sqrtf(v1.y)} * hp.inv_bc2_sqrt + hp.eps;
          const pf2 zn = zz - (m1 * hp.step_size) * pf2{frcp(den.x), frcp(den.y)};
          const float zn0 = zn.x, zn1 = zn.y, m10 = m1.x, m11 = m1.y, v10 = v1.x, v11 = v1.y;
          store_stream(zo + k0 * 64, zn0);
          store_stream(mo + k0 * 64, m10);
          store_stream(vo + k0 * 64, v10);
          if constexpr (k1 != k0) {
            store_stream(zo + k1 * 64, zn1);
            store_stream(mo + k1 * 64, m11);
            store_stream(vo + k1 * 64, v11);
          }
        } else {
          const float g0 = gl.x, g1 = gl.y;
          gp[k0 * 64] = g0;
          if constexpr (k1 != k0) gp[k1 * 64] = g1;
        }
      });
      float wj = 0.0f;
#pragma unroll
      for (int k = 0; k < P; ++k) wj = (k == jmax) ? em1[k] : wj;
      const float dirv = dir_site_round((dirv2.x + dirv2.y) + wj * (lpj + o.lse1p), Arow);
      if (valid) {
        loss += o.E + dirv;
        gtv = o.gt;
        accT += a_val * o.gt;
        ga += t * o.gt;
        const float ge = o.gD * omega;
#pragma unroll
        for (int k = 0; k < K1T; ++k) acc[k] += ge * g[k];
      }
#else
      float gz[P];
      const float dirv = dir_site_round(enum_tail<P>(o, zt, em1, S1, gz), Arow);
      if (valid) {
        loss += o.E + dirv;
        gtv = o.gt;
        accT += a_val * o.gt;
        ga += t * o.gt;
        const float ge = o.gD * omega;
#pragma unroll
        for (int k = 0; k < K1T; ++k) acc[k] += ge * g[k];
      }
      if (kStep) {
        const float* mb = lds + 2 * SF;
        float* zo = st.z_pi + tile + lane;
        float* mo = st.m_pi + tile + lane;
        float* vo = st.v_pi + tile + lane;
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const float gl = -gz[k];                          // d(-ELBO)/dz
          const float m1 = hp.beta1 * mb[k * 64 + lane] + (1.0f - hp.beta1) * gl;
          const float v1 = hp.beta2 * mb[ZF + k * 64 + lane] + (1.0f - hp.beta2) * gl * gl;
          const float denom = __builtin_sqrtf(v1) * hp.inv_bc2_sqrt + hp.eps;
          store_stream(zo + k * 64, zt[k] - hp.step_size * m1 * frcp(denom));
          store_stream(mo + k * 64, m1);
          store_stream(vo + k * 64, v1);
        }
      } else {
        float* gp = st.g_pi + tile + lane;
#pragma unroll
        for (int k = 0; k < P; ++k) gp[k * 64] = -gz[k];
      }
#endif
    }
    if (!kDecode && !frozen) {
      const float ws = wave_sum(gtv);
      if (lane == 0) s_binp[l - l0] = ws;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (stamps && lane == 0) {
    dbg[0] = t_entry;
    dbg[2] = __builtin_amdgcn_s_memrealtime();
    unsigned int hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    dbg[3] = ((unsigned long long)xcc << 32) | hw;
  }
  if (kDecode) return;
  __syncthreads();
  if (!frozen) {
    for (int i = lane; i < l1 - l0; i += 64) st.bin_part[(size_t)wt * pr.L + l0 + i] = s_binp[i];
  }
  if (valid) {
    float* cp = st.cell_part + (size_t)blockIdx.y * (K1 + 1) * N + n;
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) cp[(size_t)k * N] = acc[k];
    cp[(size_t)K1 * N] = accT;
  }
  // the wave's ELBO and d/da sums: blk_part[bt][ldn/64] (read by the finalize block of
  // this cell tile)
  const double bl = wave_sum_d((double)loss);
  const double bga = wave_sum_d((double)ga);
  if (lane == 0) {
    double* bp = st.blk_part + ((size_t)blockIdx.y * (ldn / 64) + wt) * kBlkSlots;
    bp[0] = bl;
    bp[1] = bga;
  }
}

// ------------------------------------------------------------------------------------------
// Enumerated pass, three waves per SIMD (variant 3).  One wave per workgroup = 64 cells x LT
// bins, like enum_dma_kernel, restructured for occupancy: <= 168 VGPRs and <= 13 KB of LDS
// per wave (12 resident waves per CU instead of 8).
//  * every streamed array has ONE LDS buffer, refilled by LDS-DMA (buffer_load ... lds, one
//    voffset VGPR, the bin offset in an SGPR, the pieces as immediate offsets) as soon as the
//    wave has read it into registers: at the top of bin l, after reading x, the eta code and
//    the pi logits of bin l, the copies of x, code, logits of bin l+1 and of the Adam moments
//    of bin l (read in bin l's tail) are issued.  Each buffer is its own __shared__ object,
//    so the compiler's LDS-DMA tracking waits (counted vmcnt) only for the copy a read needs;
//  * the per-(bin, cell) arithmetic is enum_online (pert_math.h): the scores are folded into a
//    running logsumexp group by group, so no per-state array is live; the tail recomputes
//    pi_k from z and reads the eta row element by element.
// every supported P (a P=13-only build, -DPERT_ONLY_P13, is for quick A/B timing tools only)
#ifdef PERT_ONLY_P13
#define PERT_ALL_P_CASES PERT_CASE(13)
#else
#define PERT_ALL_P_CASES                                                                        \
  PERT_CASE(2) PERT_CASE(3) PERT_CASE(4) PERT_CASE(5) PERT_CASE(6) PERT_CASE(7) PERT_CASE(8)    \
  PERT_CASE(9) PERT_CASE(10) PERT_CASE(11) PERT_CASE(12) PERT_CASE(13) PERT_CASE(14)            \
  PERT_CASE(15) PERT_CASE(16)
#endif


#ifndef PERT_ENUM3_WAVES
#define PERT_ENUM3_WAVES 3
#endif
#ifndef PERT_ENUM3_PRIO
#define PERT_ENUM3_PRIO 1            // issue priority falls by quarters of the tile (0: none)
#endif
constexpr int kEnum3TabFloats = 256;            // eta table staged in LDS up to this size
constexpr unsigned kRsrcWord3 = 0x00020000;     // raw buffer resource, gfx9 data format

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, (int)kRsrcWord3);
}

// copy a contiguous run of BYTES (multiple of 128) at rsrc + soff into the LDS buffer dst.
// Each piece advances the LDS pointer (M0) and the SGPR offset together and keeps the
// instruction's immediate offset at 0: the immediate would be added to the LDS address as
// well as to the global one, and M0 + immediate is not what the pieces want.
template <int BYTES>
__device__ __forceinline__ void dma_buf(__amdgpu_buffer_rsrc_t rs, uint32_t soff, float* dst, int lane) {
  constexpr int n16 = BYTES / 1024;
  constexpr int rem = BYTES % 1024;
  static_assert(BYTES % 128 == 0, "runs are whole half-waves of dwords");
  // cast once from the shared object (folds to a constant M0 per piece); offsetting the
  // generic pointer would keep a null check per piece
  typedef __attribute__((address_space(3))) float* lds_f32_t;
  const lds_f32_t d = (lds_f32_t)dst;
  pert_static_for<0, n16>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(d + i * 256), 16, lane * 16, soff + i * 1024, 0,
                                             PERT_DMA_AUX);
  });
  pert_static_for<0, rem / 256>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(d + n16 * 256 + i * 64), 4, lane * 4,
                                             soff + n16 * 1024 + i * 256, 0, PERT_DMA_AUX);
  });
  if constexpr (rem % 256 == 128) {
    if (lane < 32)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(d + (BYTES - 128) / 4), 4, lane * 4,
                                               soff + BYTES - 128, 0, PERT_DMA_AUX);
  }
}

// Cross-workgroup data of the fused step (partials, level-1 rows, counters) is written and
// read with agent-scope relaxed atomics, i.e. `sc1` stores and loads that are coherent across
// the XCDs' separate L2s on their own.  Publishing is then only "s_waitcnt vmcnt(0)" before
// the counter RMW -- an agent-scope __threadfence() would write back and invalidate the whole
// L2 of the XCD, once per workgroup (18 k per launch at C4: it doubled the pass).
template <class T>
__device__ __forceinline__ void st_coh(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_coh(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ unsigned int arrive(unsigned int* c, unsigned int v) {
  return __hip_atomic_fetch_add(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// plane k of a bin: bin and plane offsets in an SGPR (a per-plane voffset would hold a
// loop-invariant VGPR per plane for the whole pass)
template <int K>
__device__ __forceinline__ void store_nt(__amdgpu_buffer_rsrc_t rs, float v, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs, voff, soff + K * 256,
                                        PERT_NT_STORE ? PERT_STORE_CPOL : 0);
}

// (cell tile, bin tile) of this workgroup of a variant-3 launch (grid from enum3_grid)
__device__ __forceinline__ bool enum3_tile(int n_ct, int n_bt, int& wt, int& bt) {
  if constexpr (kEnum3Order == 0) {
    wt = blockIdx.x;
    bt = blockIdx.y;
    return true;
  } else if constexpr (kEnum3Order == 1) {
    wt = blockIdx.y;
    bt = blockIdx.x;
    return true;
  } else {
    const int T = n_ct * n_bt, per = (T + 7) / 8;
    const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
    if (w >= T) return false;
    constexpr bool bin_fast = kEnum3Order == 2;
    wt = bin_fast ? w / n_bt : w % n_ct;
    bt = bin_fast ? w % n_bt : w / n_ct;
    return true;
  }
}

template <int K1T>
__device__ void enum3_fused_tail(const pert_problem& pr, const pert_state& st, const pert_adam_hparams& hp, int wt,
                                 int by, int lane, bool update_shared);

// fuse (STEP mode): 0 = partials only (pert_finalize + pert_adam follow), 1 = reductions and the
// cell sites' Adam folded in (all-reduce + pert_adam_shared follow), 2 = everything folded in
template <int P, int MODE, int K1T>
__global__ void __launch_bounds__(64, PERT_ENUM3_WAVES) enum3_kernel(pert_problem pr, pert_state st, pert_adam_hparams hp,
                                                      int fuse) {
  constexpr bool kDecode = MODE == PERT_MODE_DECODE;
  constexpr bool kStep = MODE == PERT_MODE_STEP;
  constexpr int ZF = P * 64;
  if (kStep && loop_stopped(st)) return;
  __shared__ __attribute__((aligned(16))) float s_z[ZF];
  __shared__ __attribute__((aligned(16))) float s_m[kStep ? ZF : 4];
  __shared__ __attribute__((aligned(16))) float s_v[kStep ? ZF : 4];
  __shared__ __attribute__((aligned(16))) float s_xc[96];          // x (64 floats), code (64 x u16)
  __shared__ float s_bc[kMaxLT * (K1T + 1)];                        // per bin: rho, gcf[K1]
  __shared__ float s_tab[kDecode ? 1 : kEnum3TabFloats];

  const int lane = threadIdx.x;
#ifdef PERT_ENUM3_STAMPS
  // diagnostic build only (tools/wave_timeline.py): s_memrealtime at entry, first bin, exit
  unsigned long long* dbg = (unsigned long long*)st.g_pi + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4;
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
#endif
  const int N = pr.N, K1 = (K1T == PERT_MAX_K1) ? pr.K1 : K1T, ldn = pr.ldn;
  const int LT = st.bins_per_tile;
  int wt, bt;
  if (!enum3_tile((N + 63) / 64, (pr.L + LT - 1) / LT, wt, bt)) return;   // (the grid's round-up)
  const int n = wt * 64 + lane;
  const bool valid = n < N;
  const int l0 = bt * LT;
  const int l1 = min(pr.L, l0 + LT);
  const int nb = l1 - l0;
  const bool frozen = pr.kind == PERT_KIND_STEP3;
  const pert_layout lay = st.lay;
  const float* __restrict__ params = st.params;

  // streamed arrays of this tile as buffer resources (bin offsets < 2^32 within a tile)
  const size_t tile0 = ((size_t)wt * pr.L + l0) * P * 64;          // floats
  const uint32_t zbytes = (uint32_t)(nb * P * 256);
  const __amdgpu_buffer_rsrc_t rz = make_rsrc(st.z_pi + tile0, zbytes);
  const __amdgpu_buffer_rsrc_t rm = make_rsrc(kStep ? st.m_pi + tile0 : st.z_pi + tile0, zbytes);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(kStep ? st.v_pi + tile0 : st.z_pi + tile0, zbytes);
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(MODE == PERT_MODE_GRAD ? st.g_pi + tile0 : st.z_pi + tile0, zbytes);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(pr.reads + (size_t)l0 * ldn + wt * 64, (uint32_t)(nb * ldn * 4));
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(pr.eta_code + (size_t)l0 * ldn + wt * 64, (uint32_t)(nb * ldn * 2));

#define E3_DMA_X(lb_) dma_buf<256>(rx, (uint32_t)((lb_) * ldn * 4), s_xc, lane)
#define E3_DMA_C(lb_) dma_buf<128>(rc, (uint32_t)((lb_) * ldn * 2), s_xc + 64, lane)
#define E3_DMA_Z(off_) dma_buf<P * 256>(rz, (off_), s_z, lane)
#define E3_DMA_M(off_) dma_buf<P * 256>(rm, (off_), s_m, lane)
#define E3_DMA_V(off_) dma_buf<P * 256>(rv, (off_), s_v, lane)
  // first stage in flight before the prologue's parameter loads
  E3_DMA_X(0);
  E3_DMA_C(0);
  E3_DMA_Z(0u);

  // ---- tile prologue: eta table (when small), per-bin rho and GC features, cell parameters
  const int ntab = pr.n_codes * kTabRow(P);
  const bool etal = !kDecode && ntab <= kEnum3TabFloats;
  if (!kDecode && etal) {
    for (int i = lane; i < ntab; i += 64) s_tab[i] = pr.eta_table[i];
  }
  {
    const int lr = l0 + min(lane, nb - 1);
    const float zr = frozen ? pr.rho_fixed[lr] : params[lay.off_rho + lr];
    const int ng = nb * K1;
    const float* gsrc = pr.gcf + (size_t)l0 * K1;
    float gv[PERT_MAX_K1];
#pragma unroll
    for (int r = 0; r < PERT_MAX_K1; ++r) gv[r] = gsrc[min(lane + 64 * r, ng - 1)];
    if (lane < nb) {
      float dm;
      s_bc[lane * (K1 + 1)] = frozen ? zr : clipped_sigmoid(zr, &dm);
    }
#pragma unroll
    for (int r = 0; r < PERT_MAX_K1; ++r) {
      const int i = lane + 64 * r;
      if (i < ng) {
        const int lb = i / K1, j = i - lb * K1;
        s_bc[lb * (K1 + 1) + 1 + j] = gv[r];
      }
    }
  }
  const float a_val = frozen ? pr.a_fixed : fexp(params[lay.off_a]);
  const float c0 = (1.0f - pr.lamb) / pr.lamb;
  const float log1m_lam = pr.log1m_lam;
  float u = 0.0f, tau = 0.5f;
  float beta[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) beta[k] = 0.0f;
  if (valid) {
    u = params[lay.off_u + n];
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) beta[k] = params[lay.off_beta + k * N + n];
    float dm;
    tau = clipped_sigmoid(params[lay.off_tau + n], &dm);
  }
  const float ucc = u * c0;
  float acc[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) acc[k] = 0.0f;
  float sgt = 0.0f, loss = 0.0f, ga = 0.0f;
  const uint32_t voff = lane * 4;
  // the tile's partials: coherent (sc1) stores when another workgroup of this launch reads them
  const bool coh = kStep && fuse;

#if PERT_ENUM3_PRIO
  __builtin_amdgcn_s_setprio(3);
#endif
  for (int l = l0; l < l1; ++l) {
    const int lb = l - l0;
#if PERT_ENUM3_PRIO
    {
      const int q4 = 4 * lb;
      if (q4 >= nb && q4 - 4 < nb) __builtin_amdgcn_s_setprio(2);
      if (q4 >= 2 * nb && q4 - 4 < 2 * nb) __builtin_amdgcn_s_setprio(1);
      if (q4 >= 3 * nb && q4 - 4 < 3 * nb) __builtin_amdgcn_s_setprio(0);
    }
#endif
    // ---- x, eta code and pi logits of bin l into registers; then the copies of bin l+1 and
    // this bin's Adam moments are issued (they land during the NB chains)
#ifdef PERT_ENUM3_STAMPS
    if (kStep && lb == 0 && lane == 0) dbg[1] = __builtin_amdgcn_s_memrealtime();
#endif
    const float x = s_xc[lane];
    const uint32_t code = ((const uint16_t*)(s_xc + 64))[lane];
    float z[P];
#pragma unroll
    for (int k = 0; k < P; ++k) z[k] = s_z[k * 64 + lane];
    const float* bcl = s_bc + lb * (K1 + 1);
    const float rho = bcl[0];
    float dot = 0.0f;
#pragma unroll
    for (int k = 0; k < K1T; ++k) dot += (k < K1) ? beta[k] * bcl[1 + k] : 0.0f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // reads done before the buffers refill
    const uint32_t zoff = (uint32_t)(lb * P * 256);
    if (l + 1 < l1) {
      E3_DMA_X(lb + 1);
      E3_DMA_C(lb + 1);
      E3_DMA_Z(zoff + P * 256);
    }
    if (kStep) {
      E3_DMA_M(zoff);
      E3_DMA_V(zoff);
    }

    const float invx = x > 0.0f ? frcp(x) : 0.0f;
    const float omega = fexp(dot);                         // pert_model.py:633
    const float D = ucc * omega;                           // :636-640 (delta = chi D)
    const float t = tau - rho;                             // :616
    const float phi = frcp(1.0f + fexp(-a_val * t));       // :619
    EnumOnline<P> o;
    enum_online<P, kEnum3Group, !kDecode, kDecode>(x, invx, z, log1m_lam, D, phi, o);

    // The copies of bin l+1 (issued at the top of this bin) land in the buffers the next
    // iteration reads first, with no wait of their own: hipcc's LDS-DMA tracking does not carry
    // them across the loop's back edge (ROCm 7.2: no vmcnt before those reads in the GRAD and
    // DECODE instances; the STEP instance's wait for this bin's Adam moments covered them).
    // Wait here, after the NB chains have covered their latency and before this bin's stores,
    // so the wait never includes a store (the register operands pin it after the forward pass).
    if (kDecode) asm volatile("s_waitcnt vmcnt(0)" :: "v"(o.E), "v"(o.argmax) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" :: "v"(o.E), "v"(o.sgm), "v"(o.gt) : "memory");
    float gtv = 0.0f;
    if (kDecode) {
      st.cn_out[(size_t)l * ldn + n] = (uint8_t)(o.argmax % P);
      st.rep_out[(size_t)l * ldn + n] = (uint8_t)(o.argmax / P);
    } else {
      // ---- tail: Dirichlet term, gradient and fused Adam (or the gradient) of the logits, one
      // plane at a time; the eta row from the LDS copy or from global memory (two copies of
      // the tail under a wave-uniform branch: one pointer for both would be a flat address)
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_sched_barrier(0);
#endif
      float dirv = 0.0f;
      auto tail = [&](const auto* row) {
        // the eta row read per plane pair (an array of it live through the planes would cost the
        // registers the argmax logit's two values need)
        const float S1 = row[P];
        const float S1s = S1 + o.sgm;
        int jmax;
        float om;
        float lpj;                                          // the reference's fp32 log pi_jmax
        enum_jmax<P>(z, o, jmax, om, lpj);
        const float tom = S1s * om;                         // (S1 + sgm)(1 - pi_jmax), jmax_grad
        // planes in pairs, packed fp32 (the exponential, square root and reciprocal per element)
        pf2 dirv2 = {0.0f, 0.0f};
        pert_static_for<0, (P + 1) / 2>([&](auto pc) {
          constexpr int k0 = 2 * decltype(pc)::value;
          constexpr int k1 = k0 + 1 < P ? k0 + 1 : k0;        // odd P: the last pair repeats plane k0
          const pf2 zz = {z[k0], z[k1]};
          const pf2 e1 = {row[k0], k1 != k0 ? row[k1] : 0.0f};
          const pf2 pk = pf2{enum_pi(o, z[k0], k0), enum_pi(o, z[k1], k1)};
          dirv2 += e1 * ((zz - o.zmax) - o.lse1p);
          const pf2 gc = pf2{o.gcm[k0], o.gcm[k1]};
          pf2 gl = pk * S1s - e1 - gc;                                  // d(-ELBO)/dz
          // the argmax logit: jmax_grad, evaluated at the plane that holds it
          const pf2 gj = ((S1 - e1) + (o.sgm - gc)) - tom;
          gl = pf2{k0 == jmax ? gj.x : gl.x, k1 == jmax ? gj.y : gl.y};
          if (kStep) {
            const pf2 m0 = {s_m[k0 * 64 + lane], s_m[k1 * 64 + lane]};
            const pf2 v0 = {s_v[k0 * 64 + lane], s_v[k1 * 64 + lane]};
            const pf2 m1 = m0 * hp.beta1 + gl * (1.0f - hp.beta1);
            const pf2 v1 = v0 * hp.beta2 + (gl * gl) * (1.0f - hp.beta2);
            const pf2 den = pf2{__builtin_amdgcn_sqrtf(v1.x), __builtin_amdgcn_sqrtf(v1.y)} * hp.inv_bc2_sqrt + hp.eps;
            const pf2 zn = zz - (m1 * hp.step_size) * pf2{frcp(den.x), frcp(den.y)};
            store_nt<k0>(rz, zn.x, voff, zoff);
            store_nt<k0>(rm, m1.x, voff, zoff);
            store_nt<k0>(rv, v1.x, voff, zoff);
            if constexpr (k1 != k0) {
              store_nt<k1>(rz, zn.y, voff, zoff);
              store_nt<k1>(rm, m1.y, voff, zoff);
              store_nt<k1>(rv, v1.y, voff, zoff);
            }
          } else {
            // through plain floats: __builtin_bit_cast of a vector element (gl.y) compiles to
            // the bits of element 0 here (hipcc / ROCm 7.2)
            const float g0 = gl.x, g1 = gl.y;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, g0), rg, voff, zoff + k0 * 256, 0);
            if constexpr (k1 != k0)
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, g1), rg, voff, zoff + k1 * 256, 0);
          }
        });
        // the argmax plane's log pi as the reference's fp32 value (its term above used -lse1p),
        // then the site value's fp32 rounding
        dirv = dir_site_round((dirv2.x + dirv2.y) + row[jmax] * (lpj + o.lse1p), row[P + 1]);
      };
      if (etal) tail(s_tab + code * kTabRow(P));
      else tail(pr.eta_table + (size_t)code * kTabRow(P));
      if (valid) {
        loss += o.E + dirv;
        gtv = o.gt;
        sgt += o.gt;
        ga += t * o.gt;
        const float ge = o.gD * omega;
#pragma unroll
        for (int k = 0; k < K1T; ++k)
          if (k < K1) acc[k] += ge * bcl[1 + k];
      }
    }
    if (!kDecode && !frozen) {
      // the bin's rho partial of this wave tile, stored by lane 0 (the LDS a staging row would
      // take holds the eta table's rounding column instead)
      const float ws = wave_sum(gtv);
      if (lane == 0) {
        float* q = st.bin_part + (size_t)wt * pr.L + l;
        if (coh) st_coh(q, ws);
        else *q = ws;
      }
    }
  }
  if (kDecode) return;
  if (valid) {
    float* cp = st.cell_part + (size_t)bt * (K1 + 1) * N + n;
#pragma unroll
    for (int k = 0; k < K1T; ++k) {
      if (k >= K1) continue;
      if (coh) st_coh(cp + (size_t)k * N, acc[k]);
      else cp[(size_t)k * N] = acc[k];
    }
    if (coh) st_coh(cp + (size_t)K1 * N, a_val * sgt);
    else cp[(size_t)K1 * N] = a_val * sgt;
  }
  const double bl = wave_sum_d((double)loss);
  const double bga = wave_sum_d((double)ga);
  if (lane == 0) {
    double* bp = st.blk_part + ((size_t)bt * (ldn / 64) + wt) * kBlkSlots;
    if (coh) {
      st_coh(bp, bl);
      st_coh(bp + 1, bga);
    } else {
      bp[0] = bl;
      bp[1] = bga;
    }
  }
  if (kStep && fuse) enum3_fused_tail<K1T>(pr, st, hp, wt, bt, lane, fuse == 2);
#ifdef PERT_ENUM3_STAMPS
  if (kStep && lane == 0) {
    dbg[0] = t_entry;
    dbg[2] = __builtin_amdgcn_s_memrealtime();
    unsigned int hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    dbg[3] = ((unsigned long long)xcc << 32) | hw;
  }
#endif
}

// ------------------------------------------------------------------------------------------
// Observed pass (step 1): cn, rep conditioned (pert_model.py:724-729).
__global__ void __launch_bounds__(kBlock) obs_kernel(pert_problem pr, pert_state st) {
  if (loop_stopped(st)) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = pr.N, K1 = pr.K1;
  const int n = blockIdx.x * kBlock + tid;
  const bool valid = n < N;
  const int LT = st.bins_per_tile;
  const int l0 = blockIdx.y * LT;
  const int l1 = min(pr.L, l0 + LT);
  const pert_layout lay = st.lay;

  __shared__ float s_bin[kWaves][kMaxLT];
  __shared__ double s_red[kWaves];

  const float a_val = fexp(st.params[lay.off_a]);
  float dml;
  const float lam = 0.001f + 0.998f * clipped_sigmoid(st.params[lay.off_lam], &dml);
  const float c0 = (1.0f - lam) / lam;
  const float log1m_lam = logf(1.0f - lam);

  float u = 0.0f, tau = 0.5f;
  float beta[PERT_MAX_K1];
#pragma unroll
  for (int k = 0; k < PERT_MAX_K1; ++k) beta[k] = 0.0f;
  if (valid) {
    u = st.params[lay.off_u + n];
#pragma unroll
    for (int k = 0; k < PERT_MAX_K1; ++k)
      if (k < K1) beta[k] = st.params[lay.off_beta + k * N + n];
    float dm;
    tau = clipped_sigmoid(st.params[lay.off_tau + n], &dm);
  }
  const float ucc = u * c0;
  float acc[PERT_MAX_K1];
#pragma unroll
  for (int k = 0; k < PERT_MAX_K1; ++k) acc[k] = 0.0f;
  float accT = 0.0f, loss = 0.0f, ga = 0.0f, dsum = 0.0f, gdd = 0.0f;

  // Per-bin constants of the tile (constrained rho, GC features) staged in LDS once: read per
  // bin they would be scalar-cache loads whose latency every bin waits for.
  __shared__ float s_bc[kMaxLT * (PERT_MAX_K1 + 1)];
  for (int i = tid; i < (l1 - l0) * (K1 + 1); i += kBlock) {
    const int lb = i / (K1 + 1), j = i - lb * (K1 + 1);
    float dm;
    s_bc[i] = j == 0 ? clipped_sigmoid(st.params[lay.off_rho + l0 + lb], &dm) : pr.gcf[(l0 + lb) * K1 + j - 1];
  }
  __syncthreads();

  // Register software pipeline in groups of kObsU bins: the reads and observed states of the
  // next group are loaded while the current group computes.  One bin of step-1 work (~150
  // VALU) is far shorter than an HBM round trip under load, so the loads run kObsU bins
  // ahead.  Rows are padded to ldn (every launched lane may load; only valid lanes add).
  constexpr int kObsU = 4;
  const float* __restrict__ reads = pr.reads;
  const uint8_t* __restrict__ cno = pr.cn_obs;
  const uint8_t* __restrict__ repo = pr.rep_obs;
  float xq[kObsU];
  uint32_t cq[kObsU], rq[kObsU];
  auto load_group = [&](int lg) {
#pragma unroll
    for (int u = 0; u < kObsU; ++u) {
      const int l = min(lg + u, l1 - 1);
      const size_t ln = (size_t)l * pr.ldn + n;
      xq[u] = reads[ln];
      cq[u] = cno[ln];
      rq[u] = repo[ln];
    }
  };
  if (l0 < l1) load_group(l0);

  for (int lg = l0; lg < l1; lg += kObsU) {
    float xg[kObsU], cg[kObsU], rg[kObsU];
#pragma unroll
    for (int u = 0; u < kObsU; ++u) { xg[u] = xq[u]; cg[u] = (float)cq[u]; rg[u] = (float)rq[u]; }
    if (lg + kObsU < l1) load_group(lg + kObsU);
#pragma unroll
    for (int u = 0; u < kObsU; ++u) {
      const int l = lg + u;
      if (l >= l1) break;
      const float x = xg[u], cnf = cg[u], repf = rg[u];
      const float* bcl = s_bc + (l - l0) * (K1 + 1);
      const float rho = bcl[0];
      float g[PERT_MAX_K1];
#pragma unroll
      for (int k = 0; k < PERT_MAX_K1; ++k) g[k] = (k < K1) ? bcl[1 + k] : 0.0f;
      float gt = 0.0f;
      if (valid) {
        const float invx = x > 0.0f ? frcp(x) : 0.0f;
        float dot = 0.0f;
#pragma unroll
        for (int k = 0; k < PERT_MAX_K1; ++k) dot += beta[k] * g[k];
        const float omega = fexp(dot);
        const float D = ucc * omega;
        const float t = tau - rho;
        const float phi = 1.0f / (1.0f + fexp(-a_val * t));
        ObsOut o;
        obs_cellbin(x, invx, cnf, repf, log1m_lam, D, phi, o);
        loss += o.ll;
        gt = o.gt;
        accT += a_val * o.gt;
        ga += t * o.gt;
        dsum += o.dsum;
        gdd += o.gdd;
        const float ge = o.gD * omega;
#pragma unroll
        for (int k = 0; k < PERT_MAX_K1; ++k) acc[k] += ge * g[k];
      }
      const float ws = wave_sum(gt);
      if (lane == 0) s_bin[wave][l - l0] = ws;
    }
  }
  __syncthreads();
  if (tid < l1 - l0) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += s_bin[w][tid];
    st.bin_part[(size_t)blockIdx.x * pr.L + l0 + tid] = s;
  }
  if (valid) {
    float* cp = st.cell_part + (size_t)blockIdx.y * (K1 + 1) * N + n;
#pragma unroll
    for (int k = 0; k < PERT_MAX_K1; ++k)
      if (k < K1) cp[(size_t)k * N] = acc[k];
    cp[(size_t)K1 * N] = accT;
  }
  const double bl = block_sum_d((double)loss, s_red);
  const double bga = block_sum_d((double)ga, s_red);
  const double bds = block_sum_d((double)dsum, s_red);
  const double bgd = block_sum_d((double)gdd, s_red);
  if (tid == 0) {
    double* bp = st.blk_part + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kBlkSlots;
    bp[0] = bl;
    bp[1] = bga;
    bp[2] = bds;
    bp[3] = bgd;
  }
}

// ------------------------------------------------------------------------------------------
// Observed pass over PAIRS (step 1's training set, pert_model.py:228-251: every G1/2 cell twice,
// rep 0 then rep 1, with the same reads and CN).  Pair mode (include/pert_hip.h): rep_obs is
// NULL, cells [0, N/2) are the rep-0 copies and [N/2, N) the rep-1 copies, reads / cn_obs hold
// the N/2 columns once.  One lane = one pair: the two copies' NB chains share the loads (5 B
// per pair and bin instead of 12) and are independent, so each lane carries two dependency
// chains -- the single-cell pass (obs_kernel) is latency-bound at ~0.3 VALU issue with its
// waves waiting on their own chain 63 % of the time (profiles/r03b_s1).  One wave per
// workgroup, no barrier in the bin loop; per-bin rho sums by a wave reduction, staged in LDS
// and stored once per tile.
constexpr int kMaxLTObs = 512;       // the pair pass's LDS (per-bin constants) is sized by its tile
constexpr int kPlanMaxLTObs = 128;   // longest tile the step-1 planner considers
inline size_t obs_pair_lds_bytes(int K1T, int lt) { return sizeof(float) * (size_t)lt * (K1T + 2); }

template <int K1T>
__global__ void __launch_bounds__(64) obs_pair_kernel(pert_problem pr, pert_state st) {
  if (loop_stopped(st)) return;
  const int lane = threadIdx.x;
  const int N = pr.N, NG = pr.N >> 1;
  const int K1 = (K1T == PERT_MAX_K1) ? pr.K1 : K1T;
  const int g = blockIdx.x * 64 + lane;
  const bool valid = g < NG;
  const int LT = st.bins_per_tile;
  const int l0 = blockIdx.y * LT;
  const int l1 = min(pr.L, l0 + LT);
  const pert_layout lay = st.lay;

  // dynamic LDS (obs_pair_lds_bytes): per bin of the tile rho and the GC features, then the
  // per-bin rho sums
  extern __shared__ float obs_lds[];
  float* s_bc = obs_lds;
  float* s_bin = obs_lds + (size_t)st.bins_per_tile * (K1T + 1);
  // per-bin constants of the tile (constrained rho, GC features), requested first
  for (int i = lane; i < (l1 - l0) * (K1 + 1); i += 64) {
    const int lb = i / (K1 + 1), j = i - lb * (K1 + 1);
    float dm;
    s_bc[lb * (K1T + 1) + j] =
        j == 0 ? clipped_sigmoid(st.params[lay.off_rho + l0 + lb], &dm) : pr.gcf[(l0 + lb) * K1 + j - 1];
  }
  const float a_val = fexp(st.params[lay.off_a]);
  float dml;
  const float lam = 0.001f + 0.998f * clipped_sigmoid(st.params[lay.off_lam], &dml);
  const float c0 = (1.0f - lam) / lam;
  const float log1m_lam = logf(1.0f - lam);

  // the pair's parameters as packed (rep-0 copy, rep-1 copy) values
  pf2 ucc = {0.0f, 0.0f}, tau = {0.5f, 0.5f}, beta[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) beta[k] = pf2{0.0f, 0.0f};
  if (valid) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int n = g + r * NG;
      const float uc = st.params[lay.off_u + n] * c0;
      float dm;
      const float tr = clipped_sigmoid(st.params[lay.off_tau + n], &dm);
      if (r == 0) { ucc.x = uc; tau.x = tr; } else { ucc.y = uc; tau.y = tr; }
#pragma unroll
      for (int k = 0; k < K1T; ++k) {
        const float b = (k < K1) ? st.params[lay.off_beta + k * N + n] : 0.0f;
        if (r == 0) beta[k].x = b; else beta[k].y = b;
      }
    }
  }
  pf2 acc[K1T], accT = {0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < K1T; ++k) acc[k] = pf2{0.0f, 0.0f};
  pf2 loss2 = {0.0f, 0.0f}, ga2 = {0.0f, 0.0f}, dsum2 = {0.0f, 0.0f}, gdd2 = {0.0f, 0.0f};
  const float vmask = valid ? 1.0f : 0.0f;
  __syncthreads();                                   // s_bc written by the wave's lanes

  // register software pipeline: the reads and CN of the next kObsU bins are in flight while
  // the current ones compute (rows padded to ldn: every lane may load)
  constexpr int kObsU = 4;
  const float* __restrict__ reads = pr.reads;
  const uint8_t* __restrict__ cno = pr.cn_obs;
  const size_t col = (size_t)(valid ? g : 0);
  float xq[kObsU];
  uint32_t cq[kObsU];
  auto load_group = [&](int lg) {
#pragma unroll
    for (int u = 0; u < kObsU; ++u) {
      const size_t ln = (size_t)min(lg + u, l1 - 1) * pr.ldn + col;
      xq[u] = reads[ln];
      cq[u] = cno[ln];
    }
  };
  if (l0 < l1) load_group(l0);
  for (int lg = l0; lg < l1; lg += kObsU) {
    float xg[kObsU], cg[kObsU];
#pragma unroll
    for (int u = 0; u < kObsU; ++u) { xg[u] = xq[u]; cg[u] = (float)cq[u]; }
    if (lg + kObsU < l1) load_group(lg + kObsU);
    float gts[kObsU];
#pragma unroll
    for (int u = 0; u < kObsU; ++u) {
      gts[u] = 0.0f;
      const int l = lg + u;
      if (l >= l1) continue;
      const float x = xg[u], cnf = cg[u];
      const float* bcl = s_bc + (l - l0) * (K1T + 1);
      const float rho = bcl[0];
      pf2 dot = {0.0f, 0.0f};
      float gf[K1T];
#pragma unroll
      for (int k = 0; k < K1T; ++k) {
        gf[k] = (k < K1) ? bcl[1 + k] : 0.0f;
        dot += beta[k] * gf[k];
      }
      const float invx = x > 0.0f ? frcp(x) : 0.0f;
      const pf2 omega = {fexp(dot.x), fexp(dot.y)};
      const pf2 t = tau - rho;
      const pf2 at = t * (-a_val);
      const pf2 phi = {frcp(1.0f + fexp(at.x)), frcp(1.0f + fexp(at.y))};
      ObsPairOut o;
      obs_pair_cellbin(x, invx, cnf, log1m_lam, ucc * omega, phi, o);
      const pf2 gt = o.gt * vmask;
      loss2 += o.ll * vmask;
      accT += gt * a_val;
      ga2 += t * gt;
      dsum2 += o.dsum * vmask;
      gdd2 += o.gdd * vmask;
      const pf2 ge = o.gD * omega * vmask;
#pragma unroll
      for (int k = 0; k < K1T; ++k) acc[k] += ge * gf[k];
      gts[u] = gt.x + gt.y;
    }
    // the per-bin rho sums of the kObsU bins over the wave's 64 lanes: a butterfly that halves
    // the values per lane at each exchange (2 + 1 + 4 shuffles for 4 bins, not 4 x 6)
    static_assert(kObsU == 4, "butterfly written for 4 bins");
    const bool hi32 = (lane & 32) != 0, hi16 = (lane & 16) != 0;
    float a0 = hi32 ? gts[2] : gts[0], a1 = hi32 ? gts[3] : gts[1];      // keep
    float b0 = hi32 ? gts[0] : gts[2], b1 = hi32 ? gts[1] : gts[3];      // send
    a0 += __shfl_xor(b0, 32, 64);
    a1 += __shfl_xor(b1, 32, 64);
    float c = hi16 ? a1 : a0;
    c += __shfl_xor(hi16 ? a0 : a1, 16, 64);
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    // lane (hi32, hi16) holds bin lg + 2 hi32 + hi16
    if ((lane & 15) == 0) {
      const int lb = lg + (hi32 ? 2 : 0) + (hi16 ? 1 : 0);
      if (lb < l1) s_bin[lb - l0] = c;
    }
  }
  float acc_out[2][K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) { acc_out[0][k] = acc[k].x; acc_out[1][k] = acc[k].y; }
  const float accT_out[2] = {accT.x, accT.y};
  const float loss = loss2.x + loss2.y, ga = ga2.x + ga2.y, dsum = dsum2.x + dsum2.y, gdd = gdd2.x + gdd2.y;
  __syncthreads();
  for (int i = lane; i < l1 - l0; i += 64) st.bin_part[(size_t)blockIdx.x * pr.L + l0 + i] = s_bin[i];
  if (valid) {
    float* cp = st.cell_part + (size_t)blockIdx.y * (K1 + 1) * N;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int n = g + r * NG;
#pragma unroll
      for (int k = 0; k < K1T; ++k)
        if (k < K1) cp[(size_t)k * N + n] = acc_out[r][k];
      cp[(size_t)K1 * N + n] = accT_out[r];
    }
  }
  const double bl = wave_sum_d((double)loss);
  const double bga = wave_sum_d((double)ga);
  const double bds = wave_sum_d((double)dsum);
  const double bgd = wave_sum_d((double)gdd);
  if (lane == 0) {
    double* bp = st.blk_part + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kBlkSlots;
    bp[0] = bl;
    bp[1] = bga;
    bp[2] = bds;
    bp[3] = bgd;
  }
}

// Adam of one packed parameter (torch.optim.Adam; the adam_kernel arithmetic)
__device__ __forceinline__ void adam_one(const pert_state& st, const pert_adam_hparams& hp, int i, float g) {
  float mm = st.adam_m[i], vv = st.adam_v[i];
  mm = hp.beta1 * mm + (1.0f - hp.beta1) * g;
  vv = hp.beta2 * vv + (1.0f - hp.beta2) * g * g;
  const float denom = sqrtf(vv) * hp.inv_bc2_sqrt + hp.eps;
  st.params[i] -= hp.step_size * mm / denom;
  st.adam_m[i] = mm;
  st.adam_v[i] = vv;
}

// ------------------------------------------------------------------------------------------
// Per-cell and per-bin reductions + priors of the non-enumerated sites + the global sums,
// one launch.  1024-thread workgroups = 64 items (lanes) x 16 groups (waves).  Blocks
// [0, n_cblk) take 64 cells each: group g sums the per-cell partials [n_bt][CS][N] of bin
// tiles g, g+16, ... (independent loads, kFinU tiles in flight per thread), the 16 group
// sums are added in fixed order through LDS, and wave 0 applies the priors.  Blocks
// [n_cblk, n_cblk+n_lblk) take 64 bins each and sum bin_part [n_ct][L] the same way.  Every
// item is reduced in one memory round trip, so the launch stays short when a small shard
// has many bin tiles.  The last block to finish (arrival counter after the cell-block
// partials, zeroed again by that block) adds the global sums -- the former separate
// single-workgroup launch, now in the tail of this one.
//
// The pass partials: per cell and bin tile the K1 GC-feature sums and the tau sum
// (cell_part [n_bt][K1+1][N]); the enumerated passes store each wave's ELBO and d/da sums
// in blk_part [n_bt][ldn/64] (summed by the cell block of that tile), the observed pass
// (step 1) each workgroup's ELBO / d/da / lambda sums (summed by the last block).
constexpr int kFinBlock = 1024;
constexpr int kFinG = kFinBlock / 64;
#ifndef PERT_FIN_U
#define PERT_FIN_U 4
#endif
#ifndef PERT_FIN_COH
#define PERT_FIN_COH 1
#endif
__host__ __device__ constexpr int fin_slots(int n_libs, int K1) { return 2 * n_libs * K1 + 2; }

// bin tiles per level-0 group: about sqrt(n_bt), so both levels stay short (C4: 13 x 14,
// C5 at LT 32: 66 x 65)
__device__ __forceinline__ int fused_g1(int n_bt) {
  int g = 8;
  while (g * g < n_bt) ++g;
  return g;
}
__device__ __forceinline__ int fused_n_g1(int n_bt) { const int g = fused_g1(n_bt); return (n_bt + g - 1) / g; }

// s[k] += sum_{j < n} p[j rs + k ps] for k < np, in j order; 4-8 rows x NP planes of loads in
// flight per round trip (clamped indices, masked values: no guarded loads); coherent loads
template <int NP>
__device__ __forceinline__ void sum_rows(const float* __restrict__ p, size_t rs, size_t ps, int np, int n,
                                         double (&s)[NP]) {
  constexpr int R = NP >= 6 ? 4 : 8;                        // rows per round trip
  for (int j0 = 0; j0 < n; j0 += R) {
    float v[R][NP];
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const int j = j0 + u;
        const float x = ld_coh(p + (size_t)min(j, n - 1) * rs + (size_t)min(k, np - 1) * ps);
        v[u][k] = (j < n && k < np) ? x : 0.0f;
      }
#pragma unroll
    for (int u = 0; u < R; ++u)
#pragma unroll
      for (int k = 0; k < NP; ++k) s[k] += (double)v[u][k];
  }
}

// counters after finalize's arrival counter in cellblk_part: [n_ct][n_g1] group, [n_ct]
// level-1, [n_bt] bin, [1] global
__device__ __forceinline__ unsigned int* fused_counters(const pert_problem& pr, const pert_state& st) {
  const int n_cblk = (pr.N + 63) / 64;
  return reinterpret_cast<unsigned int*>(st.cellblk_part + (size_t)n_cblk * fin_slots(pr.n_libs, pr.K1) + 1);
}

__device__ __forceinline__ bool wave_flag(bool v) {
  return __builtin_amdgcn_readfirstlane((int)v) != 0;
}

// ---- per-bin: d(-ELBO)/dz_rho   (rho ~ Beta(1,1) has zero log density, :574)
__device__ __forceinline__ void fin_bins(const pert_problem& pr, const pert_state& st, int lb, int n_ct,
                                         bool stopped, double (*s_g)[64]) {
  constexpr int kFinU = 4;
  const int tid = threadIdx.x, lane = tid & 63, grp = tid >> 6;
  const int L = pr.L;
  const pert_layout lay = st.lay;
  const int l = lb * 64 + lane;
  const bool on = l < L && pr.kind != PERT_KIND_STEP3;
  // wave 0's parameters, loaded before the partials so the two round trips overlap
  float a_z = 0.0f, rho_z = 0.0f;
  if (grp == 0 && on) {
    a_z = st.params[lay.off_a];
    rho_z = st.params[lay.off_rho + l];
  }
  double s = 0.0;
  if (on) {
    const float* __restrict__ bp = st.bin_part;
    for (int c0 = grp; c0 < n_ct; c0 += kFinG * kFinU) {
      float v[kFinU];
#pragma unroll
      for (int u = 0; u < kFinU; ++u) {
        // clamped index, masked value: the loads stay unconditional, so they are all in
        // flight together (a guarded load compiles to a branch with its own wait)
        const int ct = c0 + u * kFinG;
        const float x = bp[(size_t)min(ct, n_ct - 1) * L + l];
        v[u] = ct < n_ct ? x : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kFinU; ++u) s += (double)v[u];
    }
  }
  s_g[grp][lane] = s;
  __syncthreads();
  if (stopped || grp != 0 || l >= L) return;
  if (pr.kind == PERT_KIND_STEP3) { st.grad_shared[lay.off_rho + l] = 0.0; return; }
  double tot = 0.0;
#pragma unroll
  for (int g = 0; g < kFinG; ++g) tot += s_g[g][lane];
  const float a_val = fexp(a_z);
  float dmask;
  clipped_sigmoid(rho_z, &dmask);
  // dE/drho = -a sum_n gt ;  loss gradient = +a sum gt * drho/dz
  st.grad_shared[lay.off_rho + l] = (double)a_val * tot * (double)dmask;
}

// fin_bins with one wave per 64 bins (a workgroup takes 1024 bins): for a long genome over
// few cell tiles (C5: 136 k bins x 32 tiles), where 64-bin workgroups of 16 waves loaded one
// or two rows per wave in ~2,100 workgroups.  The same sums in the same order: the 16
// interleaved groups of cell tiles (ct = g, g + 16, ...) each summed in tile order, then the
// groups in order -- bit for bit fin_bins' result.
__device__ __forceinline__ void fin_bins_wide(const pert_problem& pr, const pert_state& st, int lb, int n_ct,
                                              bool stopped) {
  const int tid = threadIdx.x;
  const int L = pr.L;
  const pert_layout lay = st.lay;
  const int l = lb * kFinBlock + tid;
  if (l >= L || stopped) return;
  if (pr.kind == PERT_KIND_STEP3) { st.grad_shared[lay.off_rho + l] = 0.0; return; }
  const float a_z = st.params[lay.off_a];
  const float rho_z = st.params[lay.off_rho + l];
  const float* __restrict__ bp = st.bin_part + l;
  double tot = 0.0;
  for (int g = 0; g < kFinG; ++g) {
    // group g's tiles g, g + 16, ... in order, 4 loads in flight (fin_bins' kFinU rounds)
    double sg = 0.0;
    for (int c0 = g; c0 < n_ct; c0 += kFinG * 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int ct = c0 + u * kFinG;
        const float x = bp[(size_t)min(ct, n_ct - 1) * L];
        v[u] = ct < n_ct ? x : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) sg += (double)v[u];
    }
    tot += sg;
  }
  const float a_val = fexp(a_z);
  float dmask;
  clipped_sigmoid(rho_z, &dmask);
  st.grad_shared[lay.off_rho + l] = (double)a_val * tot * (double)dmask;
}

// ---- per-cell: the u / beta / tau priors (pert_model.py:585, :597-603) on top of the pass's
// data sums T[k] (k < K1: sum_l gD omega g_k; k = K1: sum_l a gt) -> the ELBO's derivatives
// for the cell's sites and its prior log density; dzbs / dbm: the cell's terms of the
// per-library beta_stds (z = log) and beta_means derivatives.
template <int K1T>
struct CellGrads {
  float dU, dTauZ;
  float dB[K1T], dzbs[K1T], dbm[K1T];
  double lp;
};

template <int K1T, int KCS>
__device__ __forceinline__ void cell_grads(int K1, bool step1, float c0, float u, float tau_z, float mean_x,
                                           float ploidy, const float (&bz)[K1T], const float (&lbsd)[K1T],
                                           const float (&lbmn)[K1T], const double (&T)[KCS], CellGrads<K1T>& o) {
  double Ak[K1T], Tt = 0.0;
#pragma unroll
  for (int k = 0; k < K1T; ++k) Ak[k] = 0.0;
#pragma unroll
  for (int k = 0; k < KCS; ++k) {
    if (k < K1) Ak[k] = T[k];
    if (k == K1) Tt = T[k];
  }
  float dtau_dz;
  const float tau = clipped_sigmoid(tau_z, &dtau_dz);
  // data terms: dE/du = c0 sum_l gD omega (intercept column of gcf is 1), dE/dbeta_k = u c0 sum gD omega g_k
  float dU = c0 * (float)Ak[K1 - 1];
  float dTau = (float)Tt;
#pragma unroll
  for (int k = 0; k < K1T; ++k) o.dB[k] = (k < K1) ? u * c0 * (float)Ak[k] : 0.0f;
  double lp = 0.0;
  // u ~ Normal(mu, mu/10), mu = mean(x) / ((1 + tau) ploidy)   (:597-600)
  const float mu = mean_x / ((1.0f + tau) * ploidy);
  const float sg = mu / 10.0f;
  const float w = (u - mu) / sg;
  lp += (double)(-0.5f * w * w - logf(sg) - kHalfLog2PiF);
  dU += -w / sg;
  const float dmu = w / sg + 0.1f * w * w / sg - 0.1f / sg;
  dTau += dmu * (-mu / (1.0f + tau));
  // betas ~ Normal(beta_means[lib], beta_stds[lib]).to_event(1)   (:603)
#pragma unroll
  for (int k = 0; k < K1T; ++k) {
    o.dzbs[k] = 0.0f;
    o.dbm[k] = 0.0f;
    if (k >= K1) continue;
    const float bsd = fexp(lbsd[k]);
    const float wk = (bz[k] - lbmn[k]) / bsd;
    lp += (double)(-0.5f * wk * wk - logf(bsd) - kHalfLog2PiF);
    o.dB[k] += -wk / bsd;
    o.dzbs[k] = wk * wk - 1.0f;          // d/dz_bstds (z = log beta_stds)
    o.dbm[k] = wk / bsd;                 // d/dbeta_means (step 1)
  }
  if (step1) {
    // tau ~ Beta(1.5, 1.5)  (:585): 0.5 log tau + 0.5 log(1-tau) + lgamma(3) - 2 lgamma(1.5)
    lp += (double)(0.5f * logf(tau) + 0.5f * logf(1.0f - tau) + 0.69314718055994531f
                   - 2.0f * (-0.12078223763524522f));
    dTau += 0.5f / tau - 0.5f / (1.0f - tau);
  }
  o.dU = dU;
  o.dTauZ = dTau * dtau_dz;
  o.lp = lp;
}

// ---- per-cell: data sums over bin tiles + u / beta / tau priors -> grad_cell, and the
// block's per-library beta_stds / beta_means sums, ELBO and d/da into cellblk_part.
// Everything wave 0 needs besides the sums (its cells' parameters, the per-library prior
// table in LDS, the tile's ELBO / d/da partials) is requested before the partial loop.
// PART (the split finalize of a sharded step, pert_finalize_shared / pert_finalize_cells):
//   kFinAll    both halves (pert_finalize);
//   kFinShared only what the shared block needs -- the priors' per-library / ELBO terms
//              (parameters only) and the tile's ELBO / d/da partials -- into cellblk_part;
//   kFinCells  only the per-cell data sums + priors -> grad_cell, while the shared block is
//              all-reduced (Adam then runs once both are done).
constexpr int kFinAll = 0, kFinShared = 1, kFinCells = 2;

// Groups (n_cg > 1): a cell block's bin tiles are split over n_cg workgroups of tpg tiles
// (a genome of 20 kb bins has ~10^4 tiles: one workgroup per 64 cells walking them all left
// the launch to 32 CUs at C5); each group's per-cell sums and ELBO / d/da sums go to a level-1
// row (the rows after the bin tiles' in cell_part / blk_part, as pert_enum_step's), and the
// group that arrives last adds the rows in group order and applies the priors.  n_cg == 1 is
// the single-workgroup reduction, bit for bit.  (fin_groups: only few cell blocks over many
// tiles are split -- at C4, 157 blocks of 303 tiles, three groups made the launch 37 -> 52 us)

template <int K1T, int PART = kFinAll>
__device__ __forceinline__ void fin_cells(const pert_problem& pr, const pert_state& st, int cb, int n_bt,
                                          bool stopped, double (*s_g)[64], int grp_c = 0, int n_cg = 1, int tpg = 0) {
  constexpr int kCS = K1T + 1;
  constexpr int kFinU = K1T <= 5 ? PERT_FIN_U : 1;   // bin tiles in flight per thread
  const int tid = threadIdx.x, lane = tid & 63, grp = tid >> 6;
  const int N = pr.N, K1 = (K1T == PERT_MAX_K1) ? pr.K1 : K1T, nl = pr.n_libs;
  const pert_layout lay = st.lay;
  const bool step1 = pr.kind == PERT_KIND_STEP1;
  const int CS = K1 + 1;
  const int n = cb * 64 + lane;
  const bool in_range = n < N;
  __shared__ double s_cs[kCS][kFinG][64];
  // wave 0: its cells' parameters and their libraries' prior rows (beta_stds constrained,
  // beta_means), gathered per lane -- any number of libraries
  float u = 0.0f, tau_z = 0.0f, mean_x = 1.0f, ploidy = 1.0f;
  int lib = 0;
  float bz[K1T], lbsd[K1T], lbmn[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) { bz[k] = 0.0f; lbsd[k] = 1.0f; lbmn[k] = 0.0f; }
  if (grp == 0 && in_range) {
    u = st.params[lay.off_u + n];
    tau_z = st.params[lay.off_tau + n];
    lib = pr.libs[n];
    mean_x = pr.mean_reads[n];
    ploidy = pr.ploidy[n];
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) {
        bz[k] = st.params[lay.off_beta + k * N + n];
        lbsd[k] = st.params[lay.off_bstds + lib * K1 + k];
        lbmn[k] = step1 ? st.params[lay.off_bmeans + lib * K1 + k] : pr.beta_means[lib * K1 + k];
      }
  }
  // this group's bin tiles [t0, t1) (all of them when n_cg == 1)
  const int t0 = n_cg > 1 ? grp_c * tpg : 0;
  const int t1 = n_cg > 1 ? min(n_bt, t0 + tpg) : n_bt;
  // the enumerated pass's ELBO / d/da sums of this cell tile, one bin tile per thread
  double wl = 0.0, wa = 0.0;
  const size_t bstride = (size_t)(pr.ldn / 64) * kBlkSlots;
  if (PART != kFinCells && !step1 && tid < t1 - t0) {
    const double* bp = st.blk_part + (size_t)(t0 + tid) * bstride + (size_t)cb * kBlkSlots;
    wl = bp[0];
    wa = bp[1];
  }
  double A[kCS];
#pragma unroll
  for (int k = 0; k < kCS; ++k) A[k] = 0.0;
  if (PART != kFinShared && in_range) {
    const float* __restrict__ cp = st.cell_part;
    const size_t tstride = (size_t)CS * N;
    for (int b0 = t0 + grp; b0 < t1; b0 += kFinG * kFinU) {
      float v[kFinU][kCS];
#pragma unroll
      for (int u = 0; u < kFinU; ++u) {
        const int bt = b0 + u * kFinG;
        const float* row = cp + (size_t)min(bt, t1 - 1) * tstride + n;   // clamped, see fin_bins
#pragma unroll
        for (int k = 0; k < kCS; ++k) {
          const float x = row[(size_t)min(k, CS - 1) * N];
          v[u][k] = (bt < t1 && k < CS) ? x : 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < kFinU; ++u)
#pragma unroll
        for (int k = 0; k < kCS; ++k) A[k] += (double)v[u][k];
    }
  }
  if (PART != kFinCells && !step1) {
    for (int bt = t0 + tid + kFinBlock; bt < t1; bt += kFinBlock) {
      const double* bp = st.blk_part + (size_t)bt * bstride + (size_t)cb * kBlkSlots;
      wl += bp[0];
      wa += bp[1];
    }
  }
  // fixed-order sums of the 16 groups: every slot through LDS in one round
#pragma unroll
  for (int k = 0; k < kCS; ++k)
    if (k < CS) s_cs[k][grp][lane] = A[k];
  wl = wave_sum_d(wl);
  wa = wave_sum_d(wa);
  if (lane == 0) { s_g[grp][0] = wl; s_g[grp][1] = wa; }
  __syncthreads();
  if (stopped || grp != 0) return;
  double T[kCS];
#pragma unroll
  for (int k = 0; k < kCS; ++k) {
    double t = 0.0;
    if (k < CS) {
#pragma unroll 4
      for (int g = 0; g < kFinG; ++g) t += s_cs[k][g][lane];
    }
    T[k] = t;
  }
  double tile_l = 0.0, tile_a = 0.0;
#pragma unroll
  for (int g = 0; g < kFinG; ++g) { tile_l += s_g[g][0]; tile_a += s_g[g][1]; }
  if (n_cg > 1) {
    // level 1: this group's rows out (coherent stores), then count the group in; the last
    // group of the cell block adds every group's rows in group order
    const size_t tstride = (size_t)CS * N;
    const bool blk = PART != kFinCells && !step1;
    const size_t l1_stride = (size_t)(pr.ldn / 64) * kBlkSlots;
    double* blk1 = st.blk_part + (size_t)n_bt * l1_stride + (size_t)cb * kBlkSlots;
    float* lvl1 = st.cell_part + (size_t)n_bt * tstride + n;
    if (PART != kFinShared && in_range) {
      float* dst = lvl1 + (size_t)grp_c * tstride;
#pragma unroll
      for (int k = 0; k < kCS; ++k)
        if (k < CS) st_coh(dst + (size_t)k * N, (float)T[k]);
    }
    if (blk && lane == 0) {
      st_coh(blk1 + (size_t)grp_c * l1_stride, tile_l);
      st_coh(blk1 + (size_t)grp_c * l1_stride + 1, tile_a);
    }
    publish_wait();
    unsigned int* ctr = fused_counters(pr, st) + cb;        // (idle outside pert_enum_step)
    bool last = false;
    if (lane == 0) last = arrive(ctr, 1u) == (unsigned)(n_cg - 1);
    if (!wave_flag(last)) return;
    if (lane == 0) st_coh(ctr, 0u);
#pragma unroll
    for (int k = 0; k < kCS; ++k) T[k] = 0.0;
    if (PART != kFinShared && in_range) sum_rows<kCS>(lvl1, tstride, (size_t)N, CS, n_cg, T);
    tile_l = tile_a = 0.0;
    if (blk) {
      for (int g = lane; g < n_cg; g += 64) {
        tile_l += ld_coh(blk1 + (size_t)g * l1_stride);
        tile_a += ld_coh(blk1 + (size_t)g * l1_stride + 1);
      }
      tile_l = wave_sum_d(tile_l);
      tile_a = wave_sum_d(tile_a);
    }
  }

  const bool valid = in_range;
  float lam = pr.lamb;
  if (step1) {
    float dml;
    lam = 0.001f + 0.998f * clipped_sigmoid(st.params[lay.off_lam], &dml);
  }
  CellGrads<K1T> cg;
  cell_grads<K1T>(K1, step1, (1.0f - lam) / lam, u, tau_z, mean_x, ploidy, bz, lbsd, lbmn, T, cg);
  if (PART != kFinShared && valid) {
    float* gc = st.grad_cell - lay.n_shared;
    gc[lay.off_u + n] = -cg.dU;
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) gc[lay.off_beta + k * N + n] = -cg.dB[k];
    gc[lay.off_tau + n] = -cg.dTauZ;
  }
  if (PART == kFinCells) return;                           // (the shared half wrote the slots)
  const double lp = valid ? cg.lp : 0.0;
  float dzbs[K1T], dbm[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) {
    dzbs[k] = cg.dzbs[k];
    dbm[k] = cg.dbm[k];
  }
  // per-library sums for beta_stds (and beta_means in step 1), the ELBO and d/da:
  // wave 0 holds every value, one wave reduction per slot, fixed order
  const int nslot = fin_slots(nl, K1);
  double* out = st.cellblk_part + (size_t)cb * nslot;
  for (int sl = 0; sl < nslot; ++sl) {
    double val;
    if (sl < 2 * nl * K1) {
      const int half = sl / (nl * K1), r = sl - half * nl * K1;
      const int li = r / K1, k = r - li * K1;
      const bool mine = valid && lib == li && (half == 0 || step1);
      float fv = 0.0f;
#pragma unroll
      for (int kk = 0; kk < K1T; ++kk)
        if (kk == k) fv = half == 0 ? dzbs[kk] : dbm[kk];
      val = mine ? (double)fv : 0.0;
    } else {
      val = sl == 2 * nl * K1 ? lp : 0.0;
    }
    val = wave_sum_d(val);
    const double v = val + (sl == 2 * nl * K1 ? tile_l : (sl == 2 * nl * K1 + 1 ? tile_a : 0.0));
#if PERT_FIN_COH
    if (lane == 0) st_coh(out + sl, v);                    // read by this launch's last block
#else
    if (lane == 0) out[sl] = v;
#endif
  }
}

// ---- global sums (the last block): loss, a, beta_stds, lambda, beta_means; fixed order
__device__ void fin_global(const pert_problem& pr, const pert_state& st, int n_blk, int n_cblk) {
  const int tid = threadIdx.x;
  const int K1 = pr.K1, nl = pr.n_libs;
  const pert_layout lay = st.lay;
  const int kind = pr.kind;
  constexpr int kSW = kFinBlock / 64;
  __shared__ double s_red4[kSW][kBlkSlots];
  __shared__ double s_tail[2];
  const int lane = tid & 63, wave = tid >> 6;
  // (1) the observed pass's workgroup partials (step 1; none for the enumerated passes):
  //     all 1024 threads, double4 per workgroup, one LDS round
  //     (kGU partials per thread in flight per round trip: clamped index, masked value; the
  //     same per-thread order as one at a time)
  constexpr int kGU = 8;
  double v[kBlkSlots] = {0.0, 0.0, 0.0, 0.0};
  const double4* bp4 = reinterpret_cast<const double4*>(st.blk_part);
  for (int b0 = tid; b0 < n_blk; b0 += kFinBlock * kGU) {
    double4 q[kGU];
#pragma unroll
    for (int u = 0; u < kGU; ++u) q[u] = bp4[min(b0 + u * kFinBlock, n_blk - 1)];
#pragma unroll
    for (int u = 0; u < kGU; ++u) {
      if (b0 + u * kFinBlock < n_blk) { v[0] += q[u].x; v[1] += q[u].y; v[2] += q[u].z; v[3] += q[u].w; }
    }
  }
#pragma unroll
  for (int j = 0; j < kBlkSlots; ++j) v[j] = wave_sum_d(v[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < kBlkSlots; ++j) s_red4[wave][j] = v[j];
  }
  // (2) the cell-block partials: one wave per slot (fixed order), any number of libraries.
  //     The per-library slots go straight to their gradients; the ELBO and d/da sums to LDS.
  const int nslot = fin_slots(nl, K1);
  const int nlk = nl * K1;
  for (int sl = wave; sl < nslot; sl += kSW) {
    double acc = 0.0;
    for (int b0 = lane; b0 < n_cblk; b0 += 64 * kGU) {
      double q[kGU];
#pragma unroll
      for (int u = 0; u < kGU; ++u) {
        const double* slot = st.cellblk_part + (size_t)min(b0 + 64 * u, n_cblk - 1) * nslot + sl;
#if PERT_FIN_COH
        q[u] = ld_coh(slot);
#else
        q[u] = *slot;
#endif
      }
#pragma unroll
      for (int u = 0; u < kGU; ++u)
        if (b0 + 64 * u < n_cblk) acc += q[u];
    }
    acc = wave_sum_d(acc);
    if (lane == 0) {
      if (sl < nlk) {
        st.grad_shared[lay.off_bstds + sl] = -acc;
      } else if (sl < 2 * nlk) {
        const int j = sl - nlk;
        if (kind == PERT_KIND_STEP1) {
          const double bm = st.params[lay.off_bmeans + j];
          // beta_means ~ N(0, 1) (:560): prior gradient -bm added once (root)
          st.grad_shared[lay.off_bmeans + j] = -(acc + (pr.is_root ? -bm : 0.0));
        } else {
          st.grad_shared[lay.off_bmeans + j] = 0.0;
        }
      } else {
        s_tail[sl - 2 * nlk] = acc;
      }
    }
  }
  __syncthreads();
  if (tid != 0) return;
  double tot[kBlkSlots];
#pragma unroll
  for (int j = 0; j < kBlkSlots; ++j) {
    double t = 0.0;
    for (int w = 0; w < kSW; ++w) t += s_red4[w][j];
    tot[j] = t;
  }
  double elbo = tot[0] + s_tail[0];
  tot[1] += s_tail[1];
  // global sites
  if (kind != PERT_KIND_STEP3) {
    const double a = exp((double)st.params[lay.off_a]);
    double dza = a * tot[1];                               // dE/dz_a = a dE/da (data part)
    if (pr.is_root) {
      dza += 1.0 - 0.2 * a;                                // Gamma(2, 0.2) prior through a = exp(z)
      elbo += (double)gamma_lp_a((float)a);
    }
    st.grad_shared[lay.off_a] = -dza;
  } else {
    st.grad_shared[lay.off_a] = 0.0;
    if (pr.is_root) elbo += (double)gamma_lp_a(pr.a_fixed);   // observed a (:847)
  }
  if (kind == PERT_KIND_STEP1) {
    float dml;
    const float s = clipped_sigmoid(st.params[lay.off_lam], &dml);
    const double lam = 0.001 + 0.998 * (double)s;
    // d/dlam of sum[delta log(1-lam) + x log lam] with delta = chi u omega (1-lam)/lam
    const double dlam = -tot[2] / (1.0 - lam) + (double)pr.sum_reads / lam - tot[3] / (lam * (1.0 - lam));
    st.grad_shared[lay.off_lam] = -dlam * 0.998 * (double)dml;
    elbo += (double)pr.sum_reads * log(lam);
    if (pr.is_root) {
      double bmlp = 0.0;
      for (int j = 0; j < nl * K1; ++j) {
        const double bm = st.params[lay.off_bmeans + j];
        bmlp += -0.5 * bm * bm - 0.91893853320467274;
      }
      elbo += bmlp;
    }
  } else {
    st.grad_shared[lay.off_lam] = 0.0;
    if (pr.is_root) {                                      // observed beta_means (:785)
      double bmlp = 0.0;
      for (int j = 0; j < nl * K1; ++j) {
        const double bm = pr.beta_means[j];
        bmlp += -0.5 * bm * bm - 0.91893853320467274;
      }
      elbo += bmlp;
    }
  }
  st.grad_shared[lay.n_shared] = -elbo;                     // local loss (host adds constants)
}

template <int K1T, int PART>
__global__ void __launch_bounds__(kFinBlock) finalize_kernel(pert_problem pr, pert_state st, int n_cblk,
                                                             int n_bt, int n_ct, int n_blk, int n_cg, int tpg,
                                                             int bins_wide) {
  // the device loop's stop flag is read first but tested only before the first store, so
  // its round trip overlaps the partial loads (a stopped launch writes nothing)
  const bool stopped = loop_stopped(st);
  __shared__ double s_g[kFinG][64];
  __shared__ int s_last;
  const int tid = threadIdx.x;
  const int n_cgb = n_cblk * n_cg;                         // cell-group blocks first, then bin blocks
  if ((int)blockIdx.x >= n_cgb) {
    if (bins_wide) fin_bins_wide(pr, st, blockIdx.x - n_cgb, n_ct, stopped);
    else fin_bins(pr, st, blockIdx.x - n_cgb, n_ct, stopped, s_g);
  } else {
    fin_cells<K1T, PART>(pr, st, blockIdx.x / n_cg, n_bt, stopped, s_g, blockIdx.x % n_cg, n_cg, tpg);
  }
  if (stopped || PART == kFinCells) return;                // (the cell half has no global sums)
  // Wave 0 wrote this block's outputs: publish them, then count the block in.  The last block
  // to arrive runs the global sums, then re-arms the counter for the next launch.  (PERT_FIN_COH:
  // the only outputs the last block reads, the cell blocks' slots, are coherent sc1 stores, so
  // publishing is a vmcnt wait -- as pert_enum_step's hand-offs -- not an agent-scope fence,
  // which writes back the XCD's L2 once per workgroup: round 6 measured the shared half of a
  // 1,250-cell finalize at 14-15 of its 19-22 us.)
#if PERT_FIN_COH
  if (tid < 64) publish_wait();
#else
  if (tid < 64) __threadfence();
#endif
  __syncthreads();
  unsigned int* arrivals = reinterpret_cast<unsigned int*>(
      st.cellblk_part + (size_t)n_cblk * fin_slots(pr.n_libs, pr.K1));
  if (tid == 0) s_last = atomicAdd(arrivals, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
#if !PERT_FIN_COH
  __threadfence();
#endif
  fin_global(pr, st, n_blk, n_cblk);
  if (tid == 0) atomicExch(arrivals, 0u);
}

// Loss of iteration st.step and the reference's stopping rule, evaluated by one thread after
// the all-reduce (pert_model.py:742-758 / :800-816 / :867-883):
//   losses.append(loss)
//   if i >= min_iter: stop if |max(losses[-10:-1]) - min(losses[-10:-1])| / |losses[0] - losses[-1]| < rel_tol
//   if isnan(loss): stop
// The loss is accumulated in fp64 and recorded as the fp32 value the reference appends
// (``float(loss)`` of its fp32 ELBO tensor); the rule itself runs in fp64 on those values,
// as Python's floats do, so the stopping iteration is the host's.
// (The reference raises on an empty window (min_iter = 0 at i = 0) or a zero denominator;
// here those iterations simply do not stop.)
__device__ void loop_record(const pert_state& st) {
  const int t = st.step;
  const double loss = (double)(float)(st.grad_shared[st.lay.n_shared] - st.loss_const -
                                      (st.loss_offset != nullptr ? st.loss_offset[t] : 0.0));
  double* rec = st.loop_rec;
  int reason = 0;
  if (t >= st.min_iter) {
    const int lo = t - 9 > 0 ? t - 9 : 0;
    if (t - 1 >= lo) {
      double mx = rec[2 * lo], mn = mx;
      for (int j = lo + 1; j <= t - 1; ++j) {
        const double v = rec[2 * j];
        mx = v > mx ? v : mx;
        mn = v < mn ? v : mn;
      }
      const double diff = fabs(mx - mn) / fabs(rec[0] - loss);
      if (diff < st.rel_tol) reason = 1;
    }
  }
  if (reason == 0 && loss != loss) reason = 2;
  rec[2 * t] = loss;
  rec[2 * t + 1] = reason ? (double)t : -1.0;
  if (reason) {
    st.loop_ctl[1] = reason;
    st.loop_ctl[0] = t;
  }
}

// ------------------------------------------------------------------------------------------
// The reductions of an enumerated STEP pass folded into the pass itself (pert_enum_step):
// every workgroup (64 cells x LT bins, one wave) publishes its partials and counts itself in;
//  * per cell tile, bin tiles are counted in groups of ~sqrt(n_bt): the last of a group sums the
//    group's per-cell partials into a level-1 row, and the last level-1 row of the cell tile
//    sums those, applies the u / beta / tau priors and runs Adam on the tile's cell sites at
//    once (nothing reads them again in this launch) -- the finalize + adam of the unfused
//    sequence for that tile, overlapped with the rest of the pass;
//  * per bin tile, the last cell tile to arrive sums the tile's rho partials over the cell
//    tiles (and with update_shared, runs Adam on those rho);
//  * the last of those finalizers adds the global sums (beta_stds, a, the loss) and, with
//    update_shared (a single rank: no all-reduce between the sums and Adam), records the
//    loss for the device loop and runs Adam on a and beta_stds.
// Sums are in fixed order (level 0 in bin-tile order within the group, level 1 in group
// order, cell tiles in order), so the result does not depend on arrival order.  Everything
// one workgroup hands to another goes through coherent (sc1) stores and loads, published by
// a vmcnt wait before the counter RMW (st_coh / ld_coh below); every counter is re-armed by
// the workgroup that consumed it.

template <int K1T>
__device__ void fused_cell_tile(const pert_problem& pr, const pert_state& st, const pert_adam_hparams& hp, int wt,
                                int n_bt, int n_g1, int lane) {
  constexpr int kCS = K1T + 1;
  const int N = pr.N, K1 = (K1T == PERT_MAX_K1) ? pr.K1 : K1T, nl = pr.n_libs, CS = K1 + 1;
  const pert_layout lay = st.lay;
  const int n = wt * 64 + lane;
  const bool valid = n < N;
  const int ldn = pr.ldn;
  const size_t tstride = (size_t)CS * N;
  const float* lvl1 = st.cell_part + (size_t)n_bt * tstride;
  const double* blk1 = st.blk_part + (size_t)n_bt * (ldn / 64) * kBlkSlots;
  // the cell parameters and library prior rows first (their round trip overlaps the sums)
  float u = 0.0f, tau_z = 0.0f, mean_x = 1.0f, ploidy = 1.0f;
  int lib = 0;
  float bz[K1T], lbsd[K1T], lbmn[K1T];
#pragma unroll
  for (int k = 0; k < K1T; ++k) { bz[k] = 0.0f; lbsd[k] = 1.0f; lbmn[k] = 0.0f; }
  if (valid) {
    u = st.params[lay.off_u + n];
    tau_z = st.params[lay.off_tau + n];
    lib = pr.libs[n];
    mean_x = pr.mean_reads[n];
    ploidy = pr.ploidy[n];
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) {
        bz[k] = st.params[lay.off_beta + k * N + n];
        lbsd[k] = st.params[lay.off_bstds + lib * K1 + k];
        lbmn[k] = pr.beta_means[lib * K1 + k];
      }
  }
  double T[kCS];
#pragma unroll
  for (int k = 0; k < kCS; ++k) T[k] = 0.0;
  if (valid) sum_rows<kCS>(lvl1 + n, tstride, (size_t)N, CS, n_g1, T);
  // the tile's ELBO / d/da sums over its level-1 rows: lane g holds row g, fixed-order tree
  double wl = 0.0, wa = 0.0;
  for (int g = lane; g < n_g1; g += 64) {
    const double* bp = blk1 + ((size_t)g * (ldn / 64) + wt) * kBlkSlots;
    wl += ld_coh(bp);
    wa += ld_coh(bp + 1);
  }
  wl = wave_sum_d(wl);
  wa = wave_sum_d(wa);

  CellGrads<K1T> cg;
  cell_grads<K1T>(K1, false, (1.0f - pr.lamb) / pr.lamb, u, tau_z, mean_x, ploidy, bz, lbsd, lbmn, T, cg);
  if (valid) {
    adam_one(st, hp, lay.off_u + n, -cg.dU);
#pragma unroll
    for (int k = 0; k < K1T; ++k)
      if (k < K1) adam_one(st, hp, lay.off_beta + k * N + n, -cg.dB[k]);
    adam_one(st, hp, lay.off_tau + n, -cg.dTauZ);
  }
  // per-library beta_stds sums, the ELBO (priors + the tile's data terms) and d/da
  const int nslot = fin_slots(nl, K1);
  double* out = st.cellblk_part + (size_t)wt * nslot;
  for (int sl = 0; sl < nslot; ++sl) {
    double val = 0.0;
    if (sl < nl * K1) {
      const int li = sl / K1, k = sl - li * K1;
      float fv = 0.0f;
#pragma unroll
      for (int kk = 0; kk < K1T; ++kk)
        if (kk == k) fv = cg.dzbs[kk];
      val = (valid && lib == li) ? (double)fv : 0.0;
    } else if (sl == 2 * nl * K1) {
      val = valid ? cg.lp : 0.0;
    }
    if (sl >= nl * K1 && sl < 2 * nl * K1) continue;      // beta_means: observed in steps 2/3
    val = wave_sum_d(val);
    if (lane == 0) st_coh(out + sl, val + (sl == 2 * nl * K1 ? wl : (sl == 2 * nl * K1 + 1 ? wa : 0.0)));
  }
}

__device__ void fused_bin_tile(const pert_problem& pr, const pert_state& st, const pert_adam_hparams& hp, int by,
                               int n_ct, bool update_shared, int lane) {
  const int L = pr.L, LT = st.bins_per_tile;
  const pert_layout lay = st.lay;
  // lanes = parts x LT: part q sums the cell tiles [q c, (q+1) c) of bin by*LT + lane % LT
  const int parts = 64 / LT;
  const int lb = lane % LT, q = lane / LT;
  const int l = by * LT + lb;
  const bool on = q < parts && l < L && pr.kind != PERT_KIND_STEP3;
  const int chunk = (n_ct + parts - 1) / parts;
  const int c0 = min(n_ct, q * chunk), c1 = min(n_ct, c0 + chunk);
  double part[1] = {0.0};
  if (on) sum_rows<1>(st.bin_part + (size_t)c0 * L + l, (size_t)L, 0, 1, c1 - c0, part);
  double tot = part[0];
  for (int r = 1; r < parts; ++r) {                        // parts added in order
    const double o = __shfl(part[0], lb + r * LT, 64);
    tot += o;
  }
  if (q != 0 || l >= L) return;
  if (pr.kind == PERT_KIND_STEP3) {
    st.grad_shared[lay.off_rho + l] = 0.0;
    return;
  }
  float dmask;
  clipped_sigmoid(st.params[lay.off_rho + l], &dmask);
  const double g = (double)fexp(st.params[lay.off_a]) * tot * (double)dmask;   // see fin_bins
  st.grad_shared[lay.off_rho + l] = g;
  if (update_shared) adam_one(st, hp, lay.off_rho + l, (float)g);
}

__device__ void fused_global(const pert_problem& pr, const pert_state& st, const pert_adam_hparams& hp, int n_ct,
                             bool update_shared, int lane) {
  const int K1 = pr.K1, nl = pr.n_libs, nlk = nl * K1;
  const pert_layout lay = st.lay;
  const int nslot = fin_slots(nl, K1);
  double elbo = 0.0, da = 0.0;
  // the beta_stds slots [0, nlk) and the ELBO / d/da slots [2 nlk, 2 nlk + 2), 8 at a time,
  // 4 cell tiles per lane in flight
  for (int s0 = 0; s0 < nslot; s0 += 8) {
    double acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.0;
    for (int b0 = lane; b0 < n_ct; b0 += 256) {
      double v[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int b = b0 + 64 * u, sl = s0 + j;
          const double x = ld_coh(st.cellblk_part + (size_t)min(b, n_ct - 1) * nslot + min(sl, nslot - 1));
          v[u][j] = (b < n_ct && sl < nslot && (sl < nlk || sl >= 2 * nlk)) ? x : 0.0;
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[u][j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int sl = s0 + j;
      if (sl >= nslot || (sl >= nlk && sl < 2 * nlk)) continue;
      const double a = wave_sum_d(acc[j]);
      if (sl < nlk) {
        if (lane == 0) st.grad_shared[lay.off_bstds + sl] = -a;
      } else if (sl == 2 * nlk) {
        elbo = a;
      } else {
        da = a;
      }
    }
  }
  if (lane != 0) return;
  for (int j = 0; j < nlk; ++j) st.grad_shared[lay.off_bmeans + j] = 0.0;
  st.grad_shared[lay.off_lam] = 0.0;
  if (pr.kind != PERT_KIND_STEP3) {
    const double a = exp((double)st.params[lay.off_a]);
    double dza = a * da;                                   // dE/dz_a = a dE/da (data part)
    if (pr.is_root) {
      dza += 1.0 - 0.2 * a;                                // Gamma(2, 0.2) prior through a = exp(z)
      elbo += (double)gamma_lp_a((float)a);
    }
    st.grad_shared[lay.off_a] = -dza;
  } else {
    st.grad_shared[lay.off_a] = 0.0;
    if (pr.is_root) elbo += (double)gamma_lp_a(pr.a_fixed);   // observed a (:847)
  }
  if (pr.is_root) {                                        // observed beta_means (:785)
    double bmlp = 0.0;
    for (int j = 0; j < nlk; ++j) {
      const double bm = pr.beta_means[j];
      bmlp += -0.5 * bm * bm - 0.91893853320467274;
    }
    elbo += bmlp;
  }
  st.grad_shared[lay.n_shared] = -elbo;                     // local loss (host adds constants)
  if (!update_shared) return;
  if (st.loop_ctl != nullptr) loop_record(st);
  if (pr.kind != PERT_KIND_STEP3) adam_one(st, hp, lay.off_a, (float)st.grad_shared[lay.off_a]);
  for (int j = 0; j < nlk; ++j) adam_one(st, hp, lay.off_bstds + j, (float)st.grad_shared[lay.off_bstds + j]);
}

template <int K1T>
__device__ void enum3_fused_tail(const pert_problem& pr, const pert_state& st, const pert_adam_hparams& hp, int wt,
                                 int by, int lane, bool update_shared) {
  const int LT = st.bins_per_tile;
  const int n_bt = (pr.L + LT - 1) / LT;
  const int n_ct = (pr.N + 63) / 64;
  const int n_g1 = fused_n_g1(n_bt);
  unsigned int* ctr = fused_counters(pr, st);
  unsigned int* c_grp = ctr;                               // [n_ct][n_g1]
  unsigned int* c_lv1 = ctr + (size_t)n_ct * n_g1;         // [n_ct]
  unsigned int* c_bin = c_lv1 + n_ct;                      // [n_bt]
  unsigned int* c_glob = c_bin + n_bt;                     // [1]
  const int G1 = fused_g1(n_bt);
  const int g = by / G1;
  const int gsz = min(G1, n_bt - g * G1);
  publish_wait();                                          // this workgroup's partials are out
  bool last_g = false, last_b = false;
  if (lane == 0) {
    last_g = arrive(&c_grp[(size_t)wt * n_g1 + g], 1u) == (unsigned)(gsz - 1);
    last_b = arrive(&c_bin[by], 1u) == (unsigned)(n_ct - 1);
  }
  last_g = wave_flag(last_g);
  last_b = wave_flag(last_b);
  unsigned int n_arr = 0;
  if (last_g) {
    if (lane == 0) st_coh(&c_grp[(size_t)wt * n_g1 + g], 0u);
    // level 0 -> level 1: the group's per-cell partial rows (fixed order) and its tiles'
    // ELBO / d/da partials
    const int N = pr.N, K1 = (K1T == PERT_MAX_K1) ? pr.K1 : K1T, CS = K1 + 1;
    const int n = wt * 64 + lane;
    const size_t tstride = (size_t)CS * N;
    const int b0 = g * G1;
    if (n < N) {
      double S[K1T + 1];
#pragma unroll
      for (int k = 0; k <= K1T; ++k) S[k] = 0.0;
      sum_rows<K1T + 1>(st.cell_part + (size_t)b0 * tstride + n, tstride, (size_t)N, CS, gsz, S);
      float* dst = st.cell_part + (size_t)(n_bt + g) * tstride + n;
#pragma unroll
      for (int k = 0; k <= K1T; ++k)
        if (k < CS) st_coh(dst + (size_t)k * N, (float)S[k]);
    }
    {
      const int ldn = pr.ldn;
      double wl = 0.0, wa = 0.0;
      for (int j = lane; j < gsz; j += 64) {
        const double* bp = st.blk_part + ((size_t)(b0 + j) * (ldn / 64) + wt) * kBlkSlots;
        wl += ld_coh(bp);
        wa += ld_coh(bp + 1);
      }
      wl = wave_sum_d(wl);
      wa = wave_sum_d(wa);
      if (lane == 0) {
        double* d1 = st.blk_part + ((size_t)(n_bt + g) * (ldn / 64) + wt) * kBlkSlots;
        st_coh(d1, wl);
        st_coh(d1 + 1, wa);
      }
    }
    publish_wait();                                        // the level-1 row is out
    bool last_c = false;
    if (lane == 0) last_c = arrive(&c_lv1[wt], 1u) == (unsigned)(n_g1 - 1);
    last_c = wave_flag(last_c);
    if (last_c) {
      if (lane == 0) st_coh(&c_lv1[wt], 0u);
      fused_cell_tile<K1T>(pr, st, hp, wt, n_bt, n_g1, lane);
      n_arr += 1;
    }
  }
  if (last_b) {
    if (lane == 0) st_coh(&c_bin[by], 0u);
    fused_bin_tile(pr, st, hp, by, n_ct, update_shared, lane);
    n_arr += 1;
  }
  if (n_arr == 0) return;
  publish_wait();                                          // the finalizer's outputs are out
  bool last = false;
  if (lane == 0) last = arrive(c_glob, n_arr) + n_arr == (unsigned)(n_ct + n_bt);
  last = wave_flag(last);
  if (!last) return;
  if (lane == 0) st_coh(c_glob, 0u);
  fused_global(pr, st, hp, n_ct, update_shared, lane);
}

// Adam on the packed params (torch.optim.Adam, pyro.optim.Adam wrapper; one state per param).
__global__ void __launch_bounds__(kBlock) adam_kernel(pert_problem pr, pert_state st,
                                                      pert_adam_hparams hp, int n_limit) {
  if (loop_stopped(st)) return;
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const pert_layout lay = st.lay;
  if (st.loop_ctl != nullptr && i == 0) loop_record(st);
  if (i >= n_limit) return;
  const int kind = pr.kind;
  bool active = true;
  if (i < lay.off_a + 1 && kind == PERT_KIND_STEP3) active = false;                   // rho, a
  if (i >= lay.off_lam && i < lay.off_lam + 1 && kind != PERT_KIND_STEP1) active = false;
  if (i >= lay.off_bmeans && i < lay.n_shared && kind != PERT_KIND_STEP1) active = false;
  if (!active) return;
  const float g = i < lay.n_shared ? (float)st.grad_shared[i] : st.grad_cell[i - lay.n_shared];
  float mm = st.adam_m[i], vv = st.adam_v[i];
  mm = hp.beta1 * mm + (1.0f - hp.beta1) * g;
  vv = hp.beta2 * vv + (1.0f - hp.beta2) * g * g;
  const float denom = sqrtf(vv) * hp.inv_bc2_sqrt + hp.eps;
  st.params[i] -= hp.step_size * mm / denom;
  st.adam_m[i] = mm;
  st.adam_v[i] = vv;
}

// Pattern ceiling (diagnostic): the STEP pass's HBM streams with no arithmetic -- per 64-cell
// wave tile and bin, x and the eta code read, the P planes of z, m, v read and written back
// unchanged (the values pass through an opaque register move, so the stores are not folded
// away and the state is bit-identical afterwards).  Same grid and tile length as the pass:
// its time is what this access pattern costs in HBM on the box it runs on.
template <int P>
__global__ void __launch_bounds__(64) stream_ceiling_kernel(pert_problem pr, pert_state st) {
  const int lane = threadIdx.x, ldn = pr.ldn;
  const int LT = st.bins_per_tile;
  int wt, bt;                                                   // the three-wave pass's tile order
  if (!enum3_tile((pr.N + 63) / 64, (pr.L + LT - 1) / LT, wt, bt)) return;
  const int l0 = bt * LT, l1 = min(pr.L, l0 + LT);
  const size_t t0 = (size_t)wt * pr.L * P * 64 + lane;
  float zr[P], mr[P], vr[P];
  float xr = 0.0f;
  uint32_t cr = 0;
  auto load = [&](int l) {
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      zr[k] = __builtin_nontemporal_load(st.z_pi + o + k * 64);
      mr[k] = __builtin_nontemporal_load(st.m_pi + o + k * 64);
      vr[k] = __builtin_nontemporal_load(st.v_pi + o + k * 64);
    }
    xr = pr.reads[(size_t)l * ldn + wt * 64 + lane];
    cr = pr.eta_code[(size_t)l * ldn + wt * 64 + lane];
  };
  float acc = 0.0f;
  load(l0);
  for (int l = l0; l < l1; ++l) {
    float zc[P], mc[P], vc[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
      zc[k] = zr[k];
      mc[k] = mr[k];
      vc[k] = vr[k];
    }
    acc += xr + (float)cr;
    if (l + 1 < l1) load(l + 1);
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      asm volatile("" : "+v"(zc[k]), "+v"(mc[k]), "+v"(vc[k]));
      __builtin_nontemporal_store(zc[k], st.z_pi + o + k * 64);
      __builtin_nontemporal_store(mc[k], st.m_pi + o + k * 64);
      __builtin_nontemporal_store(vc[k], st.v_pi + o + k * 64);
    }
  }
  asm volatile("" ::"v"(acc));
}

// Device self-test of nb_lgdiff (accuracy of the special functions on gfx950).
__global__ void nb_selftest_kernel(int64_t n, const float* d, const float* x, float* lam, float* psi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float xi = x[i];
  float l, p;
  nb_lgdiff(d[i], xi, xi > 0.0f ? 1.0f / xi : 0.0f, l, p);
  lam[i] = l;
  psi[i] = p;
}

int hip_status(hipError_t e) { return e == hipSuccess ? PERT_OK : PERT_E_HIP_BASE + (int)e; }

int tile_bins(const pert_state* st) {
  int lt = st->bins_per_tile > 0 ? st->bins_per_tile : kDefaultLT;
  return lt > kMaxLT ? kMaxLT : lt;
}

// step 1 in pair mode (include/pert_hip.h): rep_obs NULL, the N/2 stored columns read twice
bool pair_mode(const pert_problem* p) { return p->kind == PERT_KIND_STEP1 && p->rep_obs == nullptr; }

// cell tiles of the observed pass: 256-cell workgroups, or 64-pair waves in pair mode
int obs_cell_tiles(const pert_problem* pr) { return pair_mode(pr) ? (pr->N / 2 + 63) / 64 : pr->ldn / kBlock; }


// the tile length a launch of this problem uses (the pair pass allows longer tiles)
int tile_bins(const pert_problem* p, const pert_state* st) {
  if (!pair_mode(p)) return tile_bins(st);
  const int lt = st->bins_per_tile > 0 ? st->bins_per_tile : kDefaultLT;
  return lt > kMaxLTObs ? kMaxLTObs : lt;
}

bool problem_ok(const pert_problem* p) {
  return p && p->L > 0 && p->N > 0 && p->ldn % PERT_BLOCK == 0 &&
         (pair_mode(p) ? (p->N % 2 == 0 && p->ldn >= p->N / 2) : p->ldn >= p->N) &&
         p->K1 >= 1 && p->K1 <= PERT_MAX_K1 && p->n_libs >= 1 &&
         p->P >= PERT_MIN_P && p->P <= PERT_MAX_P && p->reads && p->gcf && p->libs && p->mean_reads &&
         p->ploidy;
}

size_t dma_lds_bytes(int P, int mode, const pert_state& st, const pert_problem& pr) {
  const int ZF = P * 64, SF = ZF + 96;
  const int lt = st.bins_per_tile;
  const int tab = (mode != PERT_MODE_DECODE && pr.n_codes * kTabRow(P) <= kEtaLdsFloats) ? pr.n_codes * kTabRow(P) : 0;
  return sizeof(float) * (size_t)(2 * SF + (mode == PERT_MODE_STEP ? 2 * ZF : 0) + lt + lt * (pr.K1 + 1) + tab);
}

// cell tiles launched (64 cells each): only tiles holding at least one real cell (the padding
// of ldn up to a multiple of 256 is never visited)
int enum_cell_tiles(const pert_problem* pr, const pert_state* st) {
  (void)st;
  return (pr->N + 63) / 64;
}

// the grid of a variant-3 launch (and of its pattern-ceiling kernel) in kEnum3Order
dim3 enum3_grid(const pert_problem* pr, const pert_state* st, int lt) {
  const unsigned n_ct = (unsigned)enum_cell_tiles(pr, st), n_bt = (unsigned)((pr->L + lt - 1) / lt);
  if (kEnum3Order == 0) return dim3(n_ct, n_bt);
  if (kEnum3Order == 1) return dim3(n_bt, n_ct);
  return dim3((n_ct * n_bt + 7) / 8 * 8);
}

// the enumerated-pass variants this library carries: 0 (LDS-DMA, two waves per SIMD),
// 2 (its wave-timeline diagnostic build) and 3 (three waves per SIMD, the default)
bool variant_ok(int v) { return v == 0 || v == 2 || v == 3; }

template <int MODE>
int launch_enum_mode(int P, dim3 grid, const pert_problem& pr, const pert_state& st,
                     const pert_adam_hparams& hp, hipStream_t s, int fuse = 0) {
  const bool v3 = st.variant == 3;
  switch (P) {
#define PERT_CASE(PP)                                                                             \
  case PP:                                                                                        \
    if (v3 && pr.K1 == 5)                                                                         \
      hipLaunchKernelGGL((enum3_kernel<PP, MODE, 5>), grid, dim3(64), 0, s, pr, st, hp, fuse);    \
    else if (v3)                                                                                  \
      hipLaunchKernelGGL((enum3_kernel<PP, MODE, PERT_MAX_K1>), grid, dim3(64), 0, s, pr, st, hp, fuse); \
    else if (pr.K1 == 5)                                                                          \
      hipLaunchKernelGGL((enum_dma_kernel<PP, MODE, 5>), grid, dim3(64), dma_lds_bytes(PP, MODE, st, pr), s, pr, st, hp); \
    else                                                                                          \
      hipLaunchKernelGGL((enum_dma_kernel<PP, MODE, PERT_MAX_K1>), grid, dim3(64), dma_lds_bytes(PP, MODE, st, pr), s, pr, st, hp); \
    break;
    PERT_ALL_P_CASES
#undef PERT_CASE
    default: return PERT_E_UNSUPPORTED_P;
  }
  return hip_status(hipGetLastError());
}

// Resident one-wave workgroups per CU of the STEP-mode LDS-DMA pass at tile length lt.
template <int P>
int dma_step_occupancy(const pert_problem& pr, int lt, int variant) {
  pert_state tmp{};
  tmp.bins_per_tile = lt;
  const size_t lds = dma_lds_bytes(P, PERT_MODE_STEP, tmp, pr);
  int nb = 0;
  hipError_t e;
  if (variant == 3 && pr.K1 == 5)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, enum3_kernel<P, PERT_MODE_STEP, 5>, 64, 0);
  else if (variant == 3)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, enum3_kernel<P, PERT_MODE_STEP, PERT_MAX_K1>, 64, 0);
  else if (pr.K1 == 5)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, enum_dma_kernel<P, PERT_MODE_STEP, 5>, 64, lds);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, enum_dma_kernel<P, PERT_MODE_STEP, PERT_MAX_K1>, 64, lds);
  return e == hipSuccess ? nb : 0;
}

int step_occupancy(const pert_problem& pr, int lt, int variant) {
  switch (pr.P) {
#define PERT_CASE(PP) case PP: return dma_step_occupancy<PP>(pr, lt, variant);
    PERT_ALL_P_CASES
#undef PERT_CASE
    default: return 0;
  }
}

template <int P>
int selftest_enum_host(int64_t n, const float* x, const float* em1, const float* S1, const float* z,
                       float log1m_lam, const float* D, const float* phi, float* E, float* dirv,
                       float* gD, float* gt, float* gz, int32_t* amax) {
  for (int64_t i = 0; i < n; ++i) {
    float e[P], zz[P];
    for (int k = 0; k < P; ++k) { e[k] = em1[i * P + k]; zz[k] = z[i * P + k]; }
    EnumOut<P> o;
    const float xi = x[i];
    enum_cellbin<P, true, true>(xi, xi > 0.0f ? 1.0f / xi : 0.0f, e, S1[i], zz, log1m_lam, D[i], phi[i], o);
    E[i] = o.E; dirv[i] = o.dirv; gD[i] = o.gD; gt[i] = o.gt; amax[i] = o.argmax;
    for (int k = 0; k < P; ++k) gz[i * P + k] = o.gz[k];
  }
  return PERT_OK;
}

// the three-wave pass's arithmetic on the host: enum_online's forward summary, then the tail's
// pi-logit gradient as enum3_kernel forms it (enum_jmax for the argmax logit), returned as
// d(E + dirv)/dz (the sign of enum_tail's gz)
template <int P>
int selftest_online_host(int64_t n, const float* x, const float* em1, const float* S1, const float* z,
                         float log1m_lam, const float* D, const float* phi, float* E, float* gz) {
  for (int64_t i = 0; i < n; ++i) {
    float e[P], zz[P];
    for (int k = 0; k < P; ++k) { e[k] = em1[i * P + k]; zz[k] = z[i * P + k]; }
    const float xi = x[i];
    EnumOnline<P> o;
    enum_online<P, kEnum3Group, true, false>(xi, xi > 0.0f ? 1.0f / xi : 0.0f, zz, log1m_lam, D[i], phi[i], o);
    E[i] = o.E;
    int jmax;
    float om, lpj;
    enum_jmax<P>(zz, o, jmax, om, lpj);
    const float S1s = S1[i] + o.sgm;
    const float tom = S1s * om;
    for (int k = 0; k < P; ++k) {
      const float gl = enum_pi(o, zz[k], k) * S1s - e[k] - o.gcm[k];
      const float gj = ((S1[i] - e[k]) + (o.sgm - o.gcm[k])) - tom;
      gz[i * P + k] = -(k == jmax ? gj : gl);
    }
  }
  return PERT_OK;
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

// pert_version() ("... src=<hash>", the SHA-256 prefix of every source of the library) is
// compiled by build.py into a one-line object of its own, so a change to one source
// recompiles only that source's object.

int pert_make_layout(int32_t L, int32_t N, int32_t K1, int32_t n_libs, pert_layout* o) {
  if (!o || L <= 0 || N <= 0 || K1 < 1 || K1 > PERT_MAX_K1 || n_libs < 1) return PERT_E_ARG;
  o->off_rho = 0;
  o->off_a = L;
  o->off_lam = L + 1;
  o->off_bstds = L + 2;
  o->off_bmeans = L + 2 + n_libs * K1;
  o->n_shared = L + 2 + 2 * n_libs * K1;
  o->off_u = o->n_shared;
  o->off_beta = o->off_u + N;
  o->off_tau = o->off_beta + K1 * N;
  o->n_params = o->off_tau + N;
  return PERT_OK;
}

int pert_workspace_sizes(int32_t kind, int32_t L, int32_t N, int32_t K1, int32_t n_libs,
                         int32_t bins_per_tile, int64_t* n_cell_part, int64_t* n_bin_part,
                         int64_t* n_blk_part, int64_t* n_cellblk_part) {
  (void)kind;
  if (L <= 0 || N <= 0 || K1 < 1 || K1 > PERT_MAX_K1 || n_libs < 1) return PERT_E_ARG;
  pert_state tmp;
  tmp.bins_per_tile = bins_per_tile;
  const int lt = tile_bins(&tmp);
  const int64_t ldn = (N + kBlock - 1) / kBlock * kBlock;
  const int64_t n_bt = (L + lt - 1) / lt, n_ct = ldn / 64;     // sized for the 64-cell tiles
  int64_t g1 = 8;
  while (g1 * g1 < n_bt) ++g1;
  const int64_t n_g1 = (n_bt + g1 - 1) / g1;                    // pert_enum_step's level-1 rows
  if (n_cell_part) *n_cell_part = (n_bt + n_g1) * (K1 + 1) * (int64_t)N;
  if (n_bin_part) *n_bin_part = n_ct * (int64_t)L;
  if (n_blk_part) *n_blk_part = (n_bt + n_g1) * n_ct * kBlkSlots;
  // the cell-block partials, then one element whose first 4 bytes are the finalize
  // launch's arrival counter, then pert_enum_step's arrival counters (uint32: n_ct x n_g1
  // group, n_ct level-1, n_bt bin, 1 global); zero-initialised by the caller, re-armed by
  // every launch
  const int64_t n_ctr = n_ct * n_g1 + n_ct + n_bt + 1;
  if (n_cellblk_part) *n_cellblk_part = ((N + 63) / 64) * (int64_t)fin_slots(n_libs, K1) + 1 + (n_ctr + 1) / 2;
  return PERT_OK;
}

int pert_auto_bins_per_tile(const pert_problem* prob, int32_t variant, int32_t* out) {
  if (!prob || !out || prob->L <= 0 || prob->ldn <= 0 || prob->P < PERT_MIN_P || prob->P > PERT_MAX_P ||
      prob->K1 < 1 || prob->K1 > PERT_MAX_K1)
    return PERT_E_ARG;
  if (!variant_ok(variant)) return PERT_E_ARG;
  *out = kDefaultLT;
  if (prob->kind == PERT_KIND_STEP1 && !pair_mode(prob)) return PERT_OK;
  int dev = 0, ncu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return hip_status(e);
  if (prob->kind == PERT_KIND_STEP1) {
    // pair pass: one-wave tiles of 64 pairs x lt bins.  Each tile also writes (and finalize
    // reads) 2 (K1 + 1) partial floats per pair, against 5 B per pair and bin of input, so
    // longer tiles cut traffic; but the launch takes ceil(tiles / slots) rounds and a last
    // round that fills few slots idles most of the chip.  Least (rounds + 1/8) x (lt + 8),
    // the 8 being the partials' cost in bins, over lt in [32, kPlanMaxLTObs].
    int nb = 0;
    const int K1T = prob->K1 == 5 ? 5 : PERT_MAX_K1;
    if (prob->K1 == 5)
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, obs_pair_kernel<5>, 64,
                                                       obs_pair_lds_bytes(K1T, kPlanMaxLTObs));
    else
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, obs_pair_kernel<PERT_MAX_K1>, 64,
                                                       obs_pair_lds_bytes(K1T, kPlanMaxLTObs));
    if (e != hipSuccess) return hip_status(e);
    const long slots = (long)ncu * (nb > 0 ? nb : 16);
    const long n_ct = obs_cell_tiles(prob);
    long best = -1;
    for (int lt = kPlanMaxLTObs; lt >= 32; --lt) {
      const long tiles = n_ct * ((prob->L + lt - 1) / lt);
      const long rounds = (tiles + slots - 1) / slots;
      const long cost = (8 * rounds + 1) * (lt + 8);
      if (best < 0 || cost < best) { best = cost; *out = lt; }
    }
    return PERT_OK;
  }
  // Each resident wave runs one tile (a prologue of about kTilePrologue bins plus lt bins);
  // the pass takes ceil(tiles / slots) such rounds, and the last round ends with a tail in
  // which the slowest waves finish their tiles: wave exits spread over about 1/8 of a tile
  // (tools/wave_timeline.py, one-round launch: exits 453-551 us for 56-bin tiles).  Pick
  // the lt with the least predicted time (in 1/8 bins), the longer tile on a tie.  At 1,250
  // cells this takes two rounds of 27 bins over one of 54 (-3 % kernel, tools/lt_sweep.sh).
  constexpr int kTilePrologue = 2;
  const long n_ct = (prob->N + 63) / 64;
  if (variant == 3) {
    // The three-wave pass streams at 0.95-0.99 of its own HBM pattern ceiling with short
    // tiles whenever the launch runs several rounds (12 bins: 2,500-10,000 cells; the
    // cell-tile x bin-tile sweep of profiles/r02q, r02r).  A shard small enough that ONE
    // round of longer tiles leaves some slots free (1,250 cells, the per-rank shard of an
    // 8-GPU run) does better that way (0.87 vs 0.86 at 12 bins): each wave pays one tile
    // prologue and the round has no tail of late tiles.  Take the shortest such tile from 36
    // bins up that leaves a third of the slots free, else 12 (1,250 cells: 54 bins, 2,020
    // tiles, 1.0-1.7 % shorter steps than 42 bins / 85 % of the slots in two interleaved
    // leases, profiles/r04f_lt_ab.log, r04n_sweep.log).
    // A shard far smaller still (a few cell tiles: the C1 stand-in, the 64-cell genome-length
    // chain) leaves the chip idle at any tile length, and a lone wave's bin costs ~6 us of
    // latency (profiles/r04s: 209 us for 36-bin tiles of 400 cells x 271 bins), so shorter
    // tiles win until the partial rows the reductions read over the bin tiles (64 per round
    // trip, ~2 us each) catch up: least 6 (lt + 2) + 2 ceil(n_bt / 64) over the tile lengths
    // from 4 bins up that fit, the longer tile on a tie.
    const int occ = step_occupancy(*prob, kShortLT3, 3);
    const long slots = (long)ncu * (occ > 0 ? occ : 8);
    long best_cost = -1;
    int best = 0;
    for (int lt = 4; lt <= kMaxLT; ++lt) {
      const long n_bt = (prob->L + lt - 1) / lt;
      const long tiles = n_ct * n_bt;
      if (3 * tiles > 2 * slots) continue;
      const long cost = 6 * (lt + 2) + 2 * ((n_bt + 63) / 64);
      if (best_cost < 0 || cost <= best_cost) { best_cost = cost; best = lt; }
    }
    if (best > 0) {
      *out = best;
      return PERT_OK;
    }
    // many rounds (10 k cells: 15 rounds at 18 bins) -> 18 bins: the same kernel as 12 and a
    // third fewer per-cell partials for finalize (step -1 %, profiles/r02u); fewer -> 12
    const long tiles18 = n_ct * ((prob->L + kLongLT3 - 1) / kLongLT3);
    *out = tiles18 >= 8 * slots ? kLongLT3 : kShortLT3;
    return PERT_OK;
  }
  long best = -1;
  int best_lt = kDefaultLT;
  for (int lt = kMaxLT; lt >= 8; --lt) {
    const int occ = step_occupancy(*prob, lt, variant);
    if (occ <= 0) continue;
    const long slots = (long)ncu * occ;
    const long tiles = n_ct * ((prob->L + lt - 1) / lt);
    const long rounds = (tiles + slots - 1) / slots;
    const long cost = (8 * rounds + 1) * (lt + kTilePrologue);
    if (best < 0 || cost < best) { best = cost; best_lt = lt; }
  }
  *out = best_lt;
  return PERT_OK;
}

int pert_enum_pass(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                   int32_t mode, hipStream_t stream) {
  if (!problem_ok(prob) || !st || !hp || !variant_ok(st->variant)) return PERT_E_ARG;
  if (prob->kind != PERT_KIND_STEP2 && prob->kind != PERT_KIND_STEP3) return PERT_E_ARG;
  if (!prob->eta_code || !prob->eta_table || prob->n_codes < 1 || !st->z_pi) return PERT_E_ARG;
  if (prob->kind == PERT_KIND_STEP3 && !prob->rho_fixed) return PERT_E_ARG;
  if (mode == PERT_MODE_STEP && (!st->m_pi || !st->v_pi)) return PERT_E_ARG;
  if (mode == PERT_MODE_GRAD && !st->g_pi) return PERT_E_ARG;
  if (mode == PERT_MODE_DECODE && (!st->cn_out || !st->rep_out)) return PERT_E_ARG;
  if (mode != PERT_MODE_DECODE &&
      (!st->cell_part || !st->bin_part || !st->blk_part || !st->params))
    return PERT_E_ARG;
  pert_state s2 = *st;
  s2.bins_per_tile = tile_bins(st);
  const dim3 grid = st->variant == 3 ? enum3_grid(prob, st, s2.bins_per_tile)
                                     : dim3(enum_cell_tiles(prob, st), (prob->L + s2.bins_per_tile - 1) / s2.bins_per_tile);
  switch (mode) {
    case PERT_MODE_STEP: return launch_enum_mode<PERT_MODE_STEP>(prob->P, grid, *prob, s2, *hp, stream);
    case PERT_MODE_GRAD: return launch_enum_mode<PERT_MODE_GRAD>(prob->P, grid, *prob, s2, *hp, stream);
    case PERT_MODE_DECODE: return launch_enum_mode<PERT_MODE_DECODE>(prob->P, grid, *prob, s2, *hp, stream);
    default: return PERT_E_ARG;
  }
}

int pert_enum_step(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, int32_t update_shared,
                   hipStream_t stream) {
  if (!problem_ok(prob) || !st || !hp) return PERT_E_ARG;
  if (prob->kind != PERT_KIND_STEP2 && prob->kind != PERT_KIND_STEP3) return PERT_E_ARG;
  if (st->variant != 3) return PERT_E_ARG;                          // the three-wave pass only
  if (!prob->eta_code || !prob->eta_table || prob->n_codes < 1 || !st->z_pi || !st->m_pi || !st->v_pi)
    return PERT_E_ARG;
  if (prob->kind == PERT_KIND_STEP3 && !prob->rho_fixed) return PERT_E_ARG;
  if (!st->cell_part || !st->bin_part || !st->blk_part || !st->cellblk_part || !st->params || !st->adam_m ||
      !st->adam_v || !st->grad_shared)
    return PERT_E_ARG;
  pert_state s2 = *st;
  s2.bins_per_tile = tile_bins(st);
  const dim3 grid = enum3_grid(prob, st, s2.bins_per_tile);
  return launch_enum_mode<PERT_MODE_STEP>(prob->P, grid, *prob, s2, *hp, stream, update_shared ? 2 : 1);
}

int pert_adam_shared(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, hipStream_t stream) {
  if (!prob || !st || !hp || !st->params || !st->adam_m || !st->adam_v || !st->grad_shared) return PERT_E_ARG;
  const int n = st->lay.n_shared;
  hipLaunchKernelGGL(adam_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, *prob, *st, *hp, n);
  return hip_status(hipGetLastError());
}

int pert_obs_pass(const pert_problem* prob, pert_state* st, hipStream_t stream) {
  if (!problem_ok(prob) || !st || prob->kind != PERT_KIND_STEP1) return PERT_E_ARG;
  if (!prob->cn_obs || !st->cell_part || !st->bin_part || !st->blk_part) return PERT_E_ARG;
  pert_state s2 = *st;
  s2.bins_per_tile = tile_bins(prob, st);
  const dim3 grid(obs_cell_tiles(prob), (prob->L + s2.bins_per_tile - 1) / s2.bins_per_tile);
  if (!pair_mode(prob))
    hipLaunchKernelGGL(obs_kernel, grid, dim3(kBlock), 0, stream, *prob, s2);
  else if (prob->K1 == 5)
    hipLaunchKernelGGL(obs_pair_kernel<5>, grid, dim3(64), obs_pair_lds_bytes(5, s2.bins_per_tile), stream, *prob, s2);
  else
    hipLaunchKernelGGL(obs_pair_kernel<PERT_MAX_K1>, grid, dim3(64),
                       obs_pair_lds_bytes(PERT_MAX_K1, s2.bins_per_tile), stream, *prob, s2);
  return hip_status(hipGetLastError());
}

}  // extern "C"

namespace {

template <int PART>
int launch_finalize(const pert_problem* prob, pert_state* st, hipStream_t stream) {
  pert_state s2 = *st;
  s2.bins_per_tile = tile_bins(prob, st);
  const int lt = s2.bins_per_tile;
  const int n_ct = prob->kind == PERT_KIND_STEP1 ? obs_cell_tiles(prob) : enum_cell_tiles(prob, st);
  const int n_bt = (prob->L + lt - 1) / lt;
  const int n_lblk = PART == kFinCells ? 0 : (prob->L + 63) / 64;
  const int n_cblk = (prob->N + 63) / 64;
  const int n_blk = prob->kind == PERT_KIND_STEP1 ? n_bt * n_ct : 0;   // observed pass only
  // bin-tile groups of the per-cell reduction (fin_cells), as many as the workspace's level-1
  // rows allow (pert_workspace_sizes: n_bt + n_g1 rows at the state's tile length)
  // only few cell blocks over many tiles are split: about one workgroup per CU in all, groups
  // of at least 256 tiles (C5 2,000 cells: 8 groups; its 250-cell shard: 30; C4: none)
  int n_cg = 1, tpg = n_bt;
  static const int forced = [] {                 // PERT_FIN_GROUPS=<n>: a fixed group count (A/B runs)
    const char* e = getenv("PERT_FIN_GROUPS");
    return e ? atoi(e) : 0;
  }();
  if (PART != kFinShared && forced > 1 && n_bt >= 2 * forced) {
    const int64_t n_bt_ws = (prob->L + tile_bins(st) - 1) / tile_bins(st);
    int64_t g1 = 8;
    while (g1 * g1 < n_bt_ws) ++g1;
    const int64_t rows = n_bt_ws + (n_bt_ws + g1 - 1) / g1 - n_bt;
    const int64_t cg = std::max<int64_t>(1, std::min<int64_t>(forced, rows));
    tpg = (int)((n_bt + cg - 1) / cg);
    n_cg = (int)((n_bt + tpg - 1) / tpg);
  } else if (PART != kFinShared && forced == 0 && n_cblk < 128 && n_bt >= 1024) {
    const int64_t n_bt_ws = (prob->L + tile_bins(st) - 1) / tile_bins(st);
    int64_t g1 = 8;
    while (g1 * g1 < n_bt_ws) ++g1;
    const int64_t rows = n_bt_ws + (n_bt_ws + g1 - 1) / g1 - n_bt;
    const int64_t want = std::min<int64_t>((256 + n_cblk - 1) / n_cblk, (n_bt + 255) / 256);
    const int64_t cg = std::max<int64_t>(1, std::min<int64_t>(want, rows));
    tpg = (int)((n_bt + cg - 1) / cg);
    n_cg = (int)((n_bt + tpg - 1) / tpg);
  }
  // the bin blocks: 1,024 bins each when the genome is long against the cell tiles
  const int bins_wide = (PART != kFinCells && n_lblk > 512 && n_ct <= 64) ? 1 : 0;
  const int n_bblk = bins_wide ? (prob->L + kFinBlock - 1) / kFinBlock : n_lblk;
  const dim3 grid(n_cblk * n_cg + n_bblk);
  if (prob->K1 == 5)
    hipLaunchKernelGGL((finalize_kernel<5, PART>), grid, dim3(kFinBlock), 0, stream, *prob, s2,
                       n_cblk, n_bt, n_ct, n_blk, n_cg, tpg, bins_wide);
  else
    hipLaunchKernelGGL((finalize_kernel<PERT_MAX_K1, PART>), grid, dim3(kFinBlock), 0, stream,
                       *prob, s2, n_cblk, n_bt, n_ct, n_blk, n_cg, tpg, bins_wide);
  return hip_status(hipGetLastError());
}

}  // namespace

extern "C" {

int pert_finalize(const pert_problem* prob, pert_state* st, hipStream_t stream) {
  if (!problem_ok(prob) || !st || !st->grad_shared || !st->grad_cell || !st->cellblk_part) return PERT_E_ARG;
  return launch_finalize<kFinAll>(prob, st, stream);
}

int pert_finalize_shared(const pert_problem* prob, pert_state* st, hipStream_t stream) {
  if (!problem_ok(prob) || !st || !st->grad_shared || !st->cellblk_part) return PERT_E_ARG;
  return launch_finalize<kFinShared>(prob, st, stream);
}

int pert_finalize_cells(const pert_problem* prob, pert_state* st, hipStream_t stream) {
  if (!problem_ok(prob) || !st || !st->grad_cell || !st->cell_part) return PERT_E_ARG;
  return launch_finalize<kFinCells>(prob, st, stream);
}

int pert_adam(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, hipStream_t stream) {
  if (!prob || !st || !hp || !st->params || !st->adam_m || !st->adam_v) return PERT_E_ARG;
  const int n = st->lay.n_params;
  hipLaunchKernelGGL(adam_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, *prob, *st, *hp, n);
  return hip_status(hipGetLastError());
}

}  // extern "C"

namespace {

// n SVI steps from loop iteration iter0; comm != NULL: one rank of a sharded fit (the shard's
// shared-block sums into grad_local, summed over the ranks into st->grad_shared before Adam)
int svi_steps(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, const float* step_size,
              const float* inv_bc2_sqrt, int32_t iter0, int32_t n, int32_t one_launch, pert_comm* comm,
              double* grad_local, hipEvent_t* pass_events, hipStream_t stream) {
  if (!problem_ok(prob) || !st || !hp || !step_size || !inv_bc2_sqrt || n < 0 || iter0 < 0) return PERT_E_ARG;
  if (comm && (!grad_local || !st->grad_shared || grad_local == st->grad_shared)) return PERT_E_ARG;
  const bool enumerated = prob->kind == PERT_KIND_STEP2 || prob->kind == PERT_KIND_STEP3;
  if (one_launch && (!enumerated || st->variant != 3)) return PERT_E_ARG;
  pert_state s = *st;
  pert_state s_loc = *st;                      // the reductions' view: grad_shared -> grad_local
  if (comm) s_loc.grad_shared = grad_local;
  pert_adam_hparams h = *hp;
  const int64_t n_sum = (int64_t)st->lay.n_shared + 1;
  int rc = PERT_OK;
  auto mark = [&](int32_t i, int which) {
    if (pass_events && pass_events[2 * i + which] && rc == PERT_OK)
      rc = hip_status(hipEventRecord(pass_events[2 * i + which], stream));
  };
  auto all_reduce = [&]() {
    if (rc == PERT_OK) rc = pert_comm_allreduce_sum_f64(comm, grad_local, st->grad_shared, n_sum, stream);
  };
  for (int32_t i = 0; i < n && rc == PERT_OK; ++i) {
    s.step = s_loc.step = iter0 + i;           // the loop record's iteration index
    h.step_size = step_size[i];
    h.inv_bc2_sqrt = inv_bc2_sqrt[i];
    mark(i, 0);
    if (one_launch) {
      if (rc == PERT_OK) rc = pert_enum_step(prob, comm ? &s_loc : &s, &h, comm ? 0 : 1, stream);
      mark(i, 1);
      if (comm) {
        all_reduce();
        if (rc == PERT_OK) rc = pert_adam_shared(prob, &s, &h, stream);
      }
      continue;
    }
    if (rc == PERT_OK)
      rc = enumerated ? pert_enum_pass(prob, &s, &h, PERT_MODE_STEP, stream) : pert_obs_pass(prob, &s, stream);
    mark(i, 1);
    if (comm && pert_comm_overlap(comm)) {
      // the split step: the shared block's sums first, its all-reduce on the comm's side
      // stream while this stream runs the per-cell sums, then Adam (and the loss record) once
      // both are done
      if (rc == PERT_OK) rc = pert_finalize_shared(prob, &s_loc, stream);
      if (rc == PERT_OK) rc = pert_comm_allreduce_async(comm, grad_local, st->grad_shared, n_sum, stream);
      if (rc == PERT_OK) rc = pert_finalize_cells(prob, &s, stream);
      if (rc == PERT_OK) rc = pert_comm_join(comm, stream);
      if (rc == PERT_OK) rc = pert_adam(prob, &s, &h, stream);
      continue;
    }
    if (rc == PERT_OK) rc = pert_finalize(prob, comm ? &s_loc : &s, stream);
    if (comm) all_reduce();
    if (rc == PERT_OK) rc = pert_adam(prob, &s, &h, stream);
  }
  return rc;
}

// The loop's chunk events come from a per-process pool (per device) instead of being created
// and destroyed by every call: a fit makes one call per step, a bench or test many.
struct EventPool {
  std::mutex mu;
  std::vector<std::pair<int, hipEvent_t>> free_list;
};
EventPool& event_pool() {
  static EventPool* p = new EventPool;          // (never destroyed: events outlive static teardown)
  return *p;
}

int take_events(int n, hipEvent_t* ev, int* taken) {
  int dev = 0;
  int rc = hip_status(hipGetDevice(&dev));
  *taken = 0;
  EventPool& pool = event_pool();
  {
    std::lock_guard<std::mutex> lock(pool.mu);
    for (size_t i = pool.free_list.size(); i-- > 0 && *taken < n;)
      if (pool.free_list[i].first == dev) {
        ev[(*taken)++] = pool.free_list[i].second;
        pool.free_list.erase(pool.free_list.begin() + i);
      }
  }
  for (; *taken < n && rc == PERT_OK; ++*taken)
    rc = hip_status(hipEventCreateWithFlags(&ev[*taken], hipEventDisableTiming | hipEventBlockingSync));
  return rc;
}

void give_events(int n, const hipEvent_t* ev) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  EventPool& pool = event_pool();
  std::lock_guard<std::mutex> lock(pool.mu);
  for (int k = 0; k < n; ++k) pool.free_list.emplace_back(dev, ev[k]);
}

int svi_run(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, const float* step_size,
            const float* inv_bc2_sqrt, int32_t n_iter, int32_t chunk, int32_t depth, int32_t one_launch,
            pert_comm* comm, double* grad_local, hipEvent_t* pass_events, double* host_rec, int32_t* n_launched,
            hipStream_t stream) {
  if (!st || !st->loop_ctl || !st->loop_rec || !host_rec || !n_launched || n_iter < 0 || chunk < 1 || depth < 1)
    return PERT_E_ARG;
  *n_launched = 0;
  if (n_iter == 0) return PERT_OK;
  const int n_chunks = (n_iter + chunk - 1) / chunk;
  const int ring = depth + 1;
  hipEvent_t ev[65];
  if (ring > 64) return PERT_E_ARG;
  int made = 0;
  int rc = take_events(ring + 1, ev, &made);
  int waited = 0;                              // chunks whose records have been looked at
  bool stop_seen = false;
  int c = 0;
  // a chunk's records are at host_rec[2 j] (loss) and host_rec[2 j + 1] (>= 0: stopped at j).
  // Which chunks are looked at, and when, depends only on the chunk index: the ranks of a
  // sharded fit (identical, all-reduced loss records) stop queueing after the same chunk.
  // Sharded, a wait polls the communicator (a peer's abort, RCCL's async error, a deadline)
  // instead of blocking, so a failed rank cannot leave the others waiting forever.
  auto look = [&](int k) {
    rc = rc == PERT_OK ? pert_comm_wait_event(comm, ev[k % ring], 0) : rc;
    const int j1 = (k + 1) * chunk < n_iter ? (k + 1) * chunk : n_iter;
    for (int j = k * chunk; j < j1 && rc == PERT_OK; ++j)
      if (host_rec[2 * j + 1] >= 0.0) stop_seen = true;
  };
  for (; c < n_chunks && rc == PERT_OK && !stop_seen; ++c) {
    if (c - waited >= ring - 1) look(waited++);          // the ring's oldest chunk is done
    if (stop_seen || rc != PERT_OK) break;
    const int j0 = c * chunk, n = (j0 + chunk < n_iter ? j0 + chunk : n_iter) - j0;
    rc = svi_steps(prob, st, hp, step_size + j0, inv_bc2_sqrt + j0, j0, n, one_launch, comm, grad_local,
                   pass_events ? pass_events + 2 * j0 : nullptr, stream);
    if (rc == PERT_OK)
      rc = hip_status(hipMemcpyAsync(host_rec + 2 * j0, st->loop_rec + 2 * j0, sizeof(double) * 2 * n,
                                     hipMemcpyDeviceToHost, stream));
    if (rc == PERT_OK) rc = hip_status(hipEventRecord(ev[c % ring], stream));
    if (rc == PERT_OK) *n_launched = j0 + n;
  }
  // every queued launch and copy, the last ones polled for rather than slept on (a blocking
  // wait's wake-up was 35-120 us of every call's fixed cost, profiles/r06e); sharded, under the
  // watchdog -- a failure on this rank raises the abort word the peers poll and stops this
  // rank's own collectives
  if (rc == PERT_OK && made == ring + 1) {
    if (c >= 2 && waited < c - 1) rc = pert_comm_wait_event(comm, ev[(c - 2) % ring], 0);   // all but the last chunk
    if (rc == PERT_OK) rc = hip_status(hipEventRecord(ev[ring], stream));
    if (rc == PERT_OK) rc = pert_comm_wait_event(comm, ev[ring], 1);
  }
  if (comm && rc != PERT_OK) (void)pert_comm_abort(comm, rc);
  const hipError_t e = hipStreamSynchronize(stream);     // (drained: returns at once)
  if (rc == PERT_OK) rc = hip_status(e);
  give_events(made, ev);
  return rc;
}

}  // namespace

extern "C" {

int pert_svi_steps(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, const float* step_size,
                   const float* inv_bc2_sqrt, int32_t iter0, int32_t n, int32_t one_launch, hipEvent_t* pass_events,
                   hipStream_t stream) {
  return svi_steps(prob, st, hp, step_size, inv_bc2_sqrt, iter0, n, one_launch, nullptr, nullptr, pass_events, stream);
}

int pert_svi_run(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp, const float* step_size,
                 const float* inv_bc2_sqrt, int32_t n_iter, int32_t chunk, int32_t depth, int32_t one_launch,
                 hipEvent_t* pass_events, double* host_rec, int32_t* n_launched, hipStream_t stream) {
  return svi_run(prob, st, hp, step_size, inv_bc2_sqrt, n_iter, chunk, depth, one_launch, nullptr, nullptr,
                 pass_events, host_rec, n_launched, stream);
}

int pert_svi_steps_sharded(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                           const float* step_size, const float* inv_bc2_sqrt, int32_t iter0, int32_t n,
                           int32_t one_launch, pert_comm* comm, double* grad_local, hipEvent_t* pass_events,
                           hipStream_t stream) {
  if (!comm) return PERT_E_ARG;
  return svi_steps(prob, st, hp, step_size, inv_bc2_sqrt, iter0, n, one_launch, comm, grad_local, pass_events, stream);
}

int pert_svi_run_sharded(const pert_problem* prob, pert_state* st, const pert_adam_hparams* hp,
                         const float* step_size, const float* inv_bc2_sqrt, int32_t n_iter, int32_t chunk,
                         int32_t depth, int32_t one_launch, pert_comm* comm, double* grad_local,
                         hipEvent_t* pass_events, double* host_rec, int32_t* n_launched, hipStream_t stream) {
  if (!comm) return PERT_E_ARG;
  return svi_run(prob, st, hp, step_size, inv_bc2_sqrt, n_iter, chunk, depth, one_launch, comm, grad_local,
                 pass_events, host_rec, n_launched, stream);
}

int pert_stream_ceiling(const pert_problem* prob, pert_state* st, hipStream_t stream) {
  if (!problem_ok(prob) || !st || !st->z_pi || !st->m_pi || !st->v_pi || !prob->eta_code) return PERT_E_ARG;
  if (prob->kind != PERT_KIND_STEP2 && prob->kind != PERT_KIND_STEP3) return PERT_E_ARG;
  pert_state s2 = *st;
  s2.bins_per_tile = tile_bins(st);
  const dim3 grid = enum3_grid(prob, st, s2.bins_per_tile);
  switch (prob->P) {
#define PERT_CASE(PP)                                                                          \
  case PP:                                                                                     \
    hipLaunchKernelGGL(stream_ceiling_kernel<PP>, grid, dim3(64), 0, stream, *prob, s2);     \
    return hip_status(hipGetLastError());
    PERT_ALL_P_CASES
#undef PERT_CASE
    default: return PERT_E_UNSUPPORTED_P;
  }
}

int pert_selftest_nb_lgdiff_host(int64_t n, const float* d, const float* x, float* lam, float* psi) {
  for (int64_t i = 0; i < n; ++i) {
    const float xi = x[i];
    nb_lgdiff(d[i], xi, xi > 0.0f ? 1.0f / xi : 0.0f, lam[i], psi[i]);
  }
  return PERT_OK;
}

int pert_selftest_nb_lgdiff_device(int64_t n, const float* d, const float* x, float* lam, float* psi,
                                   hipStream_t stream) {
  if (n <= 0) return PERT_OK;
  hipLaunchKernelGGL(nb_selftest_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, d, x,
                     lam, psi);
  return hip_status(hipGetLastError());
}

int pert_selftest_enum_cellbin_host(int32_t P, int64_t n, const float* x, const float* em1,
                                    const float* S1, const float* z, float log1m_lam, const float* D,
                                    const float* phi, float* E, float* dirv, float* gD, float* gt,
                                    float* gz, int32_t* amax) {
  switch (P) {
#define PERT_CASE(PP) \
  case PP: return selftest_enum_host<PP>(n, x, em1, S1, z, log1m_lam, D, phi, E, dirv, gD, gt, gz, amax);
    PERT_ALL_P_CASES
#undef PERT_CASE
    default: return PERT_E_UNSUPPORTED_P;
  }
}

int pert_selftest_enum_online_host(int32_t P, int64_t n, const float* x, const float* em1, const float* S1,
                                   const float* z, float log1m_lam, const float* D, const float* phi, float* E,
                                   float* gz) {
  switch (P) {
#define PERT_CASE(PP) \
  case PP: return selftest_online_host<PP>(n, x, em1, S1, z, log1m_lam, D, phi, E, gz);
    PERT_ALL_P_CASES
#undef PERT_CASE
    default: return PERT_E_UNSUPPORTED_P;
  }
}

}  // extern "C"
