// Bytes-in-flight probe for the enumerated pass's access pattern (diagnostic, not product code).
//
// The step-2 pass streams per 64-cell wave tile and bin: x (256 B) + eta code (128 B) read, and
// the pi logits z, Adam moments m, v (P x 256 B each) read and written back in place; each wave
// keeps ONE bin of loads in flight ahead of the bin it works on.  A small shard (1,250 cells, the
// per-rank work of C4 on 8 GPUs) launches one round of ~2,000 such waves, a 10 k-cell shard keeps
// ~3,000 resident: if the pattern is latency-bound (Little's law) the small shard's ceiling sits
// below the large one's.  This probe runs the same streams with no arithmetic at lookahead depth
// D = 1..3 bins (register buffers) and at a chosen number of resident waves per CU (LDS padding),
// so the ceiling can be read as a function of bytes in flight.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/depth_probe.hip -o tools/depth_probe
//   ./depth_probe [cells=1250] [bins=5451] [LT=54] [waves_per_cu=12] [iters=20] [spread=1] [swap=0]
// spread: cell tiles placed spread x a tile apart (the footprint of a spread x larger shard);
// subset (9th argument, > 0): only that many cell tiles launched over the whole allocation.
// layout (10th: 0 three hipMallocs, 1 one allocation, 2 three hipDeviceMallocContiguous ones, 3 one
// contiguous allocation) with pads m-z / v-m (11th / 12th, KB, layouts 1 and 3); alloc_cells
// (13th): allocations sized for that many cells.
// work (8th argument, > 0): the load-schedule experiment instead -- that many VALU operations per
// bin between the loads and the stores, m / v loaded in the bin that uses them or a bin ahead.
// swap: the workgroup -> tile order: 0 cell tiles fastest (the pass's), 1 bin tiles fastest,
// 2 / 3 XCD-aware (XCD k gets a contiguous eighth of the tiles, bin- / cell-fastest).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int P = 13;

template <int D>
__global__ void __launch_bounds__(64) depth_stream(const float* __restrict__ x, const uint16_t* __restrict__ code,
                                                   float* z, float* m, float* v, int L, int ldn, int LT, int spread,
                                                   int swap, int n_ct, float* sink) {
  extern __shared__ float pad[];                  // occupancy cap: dynamic LDS per workgroup
  const int lane = threadIdx.x;
  if (lane == 0 && LT < 0) pad[0] = 0.0f;
  // tile of this workgroup (1-D grid of n_ct x n_bt; the dispatcher deals consecutive ids round
  // robin over the 8 XCDs): 0 cell tiles fastest, 1 bin tiles fastest, 2 / 3 XCD-aware -- XCD k
  // runs a contiguous 1/8 of the tiles in bin-fastest (2) / cell-fastest (3) order
  const int n_bt = (L + LT - 1) / LT, T = n_ct * n_bt;
  int w = blockIdx.x;
  if (swap >= 2) {
    const int per = (T + 7) / 8, xcd = w % 8, slot = w / 8;
    w = xcd * per + slot;
    if (w >= T) return;
  }
  const bool bin_fast = swap == 1 || swap == 2;
  const int wt = bin_fast ? w / n_bt : w % n_ct, bt = bin_fast ? w % n_bt : w / n_ct;

  const int l0 = bt * LT, l1 = min(L, l0 + LT);
  const size_t t0 = ((size_t)wt * spread * L) * P * 64 + lane;     // spread: tiles apart by spread x a tile
  float zr[D][P], mr[D][P], vr[D][P], xr[D];
  uint32_t cr[D];
  float acc = 0.0f;
  auto load = [&](auto dd, int l) {
    constexpr int d = decltype(dd)::value;
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      zr[d][k] = __builtin_nontemporal_load(z + o + k * 64);
      mr[d][k] = __builtin_nontemporal_load(m + o + k * 64);
      vr[d][k] = __builtin_nontemporal_load(v + o + k * 64);
    }
    xr[d] = x[(size_t)l * ldn + wt * 64 + lane];
    cr[d] = code[(size_t)l * ldn + wt * 64 + lane];
  };
  auto each = [&](auto f) {
    [&]<int... I>(std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>{}), ...); }
    (std::make_integer_sequence<int, D>{});
  };
  each([&](auto dd) {
    if (l0 + decltype(dd)::value < l1) load(dd, l0 + decltype(dd)::value);
  });
  for (int l = l0; l < l1; l += D) {
    each([&](auto dd) {
      constexpr int d = decltype(dd)::value;
      const int lc = l + d;
      if (lc < l1) {
        float zc[P], mc[P], vc[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
          zc[k] = zr[d][k];
          mc[k] = mr[d][k];
          vc[k] = vr[d][k];
        }
        acc += xr[d] + (float)cr[d];
        if (lc + D < l1) load(dd, lc + D);
        const size_t o = t0 + (size_t)lc * P * 64;
#pragma unroll
        for (int k = 0; k < P; ++k) {
          asm volatile("" : "+v"(zc[k]), "+v"(mc[k]), "+v"(vc[k]));
          __builtin_nontemporal_store(zc[k], z + o + k * 64);
          __builtin_nontemporal_store(mc[k], m + o + k * 64);
          __builtin_nontemporal_store(vc[k], v + o + k * 64);
        }
      }
    });
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// The pass's load schedule with arithmetic in between: per bin, `work` VALU operations (four
// independent fma chains on the bin's z values) between the issue of the next loads and the
// stores.  mv_ahead 0: as enum3_kernel -- x, code, z of bin l+1 and m, v of bin l issued at the top
// of bin l, m and v consumed after the arithmetic; 1: m, v of bin l+1 issued a bin ahead as well.
template <int MV_AHEAD>
__global__ void __launch_bounds__(64) work_stream(const float* __restrict__ x, const uint16_t* __restrict__ code,
                                                  float* z, float* m, float* v, int L, int ldn, int LT, int n_ct,
                                                  int work, float* sink) {
  extern __shared__ float pad[];
  const int lane = threadIdx.x;
  if (lane == 0 && LT < 0) pad[0] = 0.0f;
  const int n_bt = (L + LT - 1) / LT, T = n_ct * n_bt, per = (T + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (w >= T) return;
  const int wt = w / n_bt, bt = w % n_bt;
  const int l0 = bt * LT, l1 = min(L, l0 + LT);
  const size_t t0 = ((size_t)wt * L) * P * 64 + lane;
  float zr[P], mr[P], vr[P], xr = 0.0f;
  uint32_t cr = 0;
  auto load_zxc = [&](int l) {
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) zr[k] = __builtin_nontemporal_load(z + o + k * 64);
    xr = x[(size_t)l * ldn + wt * 64 + lane];
    cr = code[(size_t)l * ldn + wt * 64 + lane];
  };
  auto load_mv = [&](int l) {
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      mr[k] = __builtin_nontemporal_load(m + o + k * 64);
      vr[k] = __builtin_nontemporal_load(v + o + k * 64);
    }
  };
  float acc0 = 0.0f, acc1 = 0.0f, acc2 = 0.0f, acc3 = 0.0f;
  load_zxc(l0);
  if (MV_AHEAD) load_mv(l0);
  for (int l = l0; l < l1; ++l) {
    float zc[P], mc[P], vc[P];
#pragma unroll
    for (int k = 0; k < P; ++k) zc[k] = zr[k];
    float xc = xr + (float)cr;
    if (MV_AHEAD) {
#pragma unroll
      for (int k = 0; k < P; ++k) { mc[k] = mr[k]; vc[k] = vr[k]; }
    }
    if (l + 1 < l1) {
      load_zxc(l + 1);
      if (MV_AHEAD) load_mv(l + 1);
    }
    if (!MV_AHEAD) load_mv(l);
    for (int i = 0; i < work; i += 8) {                  // (constant register indices only)
      acc0 = __builtin_fmaf(acc0, 0.999f, zc[0]);
      acc1 = __builtin_fmaf(acc1, 0.998f, zc[1]);
      acc2 = __builtin_fmaf(acc2, 0.997f, zc[2]);
      acc3 = __builtin_fmaf(acc3, 0.996f, xc);
      acc0 = __builtin_fmaf(acc0, 0.995f, zc[3]);
      acc1 = __builtin_fmaf(acc1, 0.994f, zc[4]);
      acc2 = __builtin_fmaf(acc2, 0.993f, zc[5]);
      acc3 = __builtin_fmaf(acc3, 0.992f, zc[6]);
    }
    if (!MV_AHEAD) {
#pragma unroll
      for (int k = 0; k < P; ++k) { mc[k] = mr[k]; vc[k] = vr[k]; }
    }
    const size_t o = t0 + (size_t)l * P * 64;
    const float g = (acc0 + acc1) * 1e-30f + (acc2 + acc3) * 1e-30f;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      __builtin_nontemporal_store(zc[k] + g, z + o + k * 64);
      __builtin_nontemporal_store(mc[k] + g, m + o + k * 64);
      __builtin_nontemporal_store(vc[k] + g, v + o + k * 64);
    }
  }
  if (acc0 + acc1 + acc2 + acc3 == 12345.678f) sink[0] = acc0;
}

template <class F>
static float time_ms(F f, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / iters;
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 1250;
  const int L = argc > 2 ? atoi(argv[2]) : 5451;
  const int LT = argc > 3 ? atoi(argv[3]) : 54;
  const int wpc = argc > 4 ? atoi(argv[4]) : 12;
  const int iters = argc > 5 ? atoi(argv[5]) : 20;
  const int spread = argc > 6 ? atoi(argv[6]) : 1;
  const int swap = argc > 7 ? atoi(argv[7]) : 0;
  if (N <= 0 || L <= 0 || LT <= 0 || wpc <= 0 || wpc > 32 || spread < 1 || spread > 16) return 2;
  const int ldn = (N + 255) / 256 * 256;
  const int nwt = (N + 63) / 64;
  // alloc_cells (13th argument): size the z / m / v allocations for that many cells (>= N), the
  // tiles of the N cells at their start
  const int alloc_cells = argc > 13 ? atoi(argv[13]) : N;
  const size_t nz_used = (size_t)(ldn / 64) * spread * L * P * 64;
  const size_t nz = alloc_cells > N ? (size_t)((alloc_cells + 255) / 256 * 4) * spread * L * P * 64 : nz_used;
  float *z, *m, *v, *x, *sink;
  uint16_t* code;
  // layout (10th-12th arguments): 0 = three hipMallocs (as the shard's torch tensors get them);
  // 1 = one allocation, m at z + nz + pad_m KB, v at m + nz + pad_v KB
  const int layout = argc > 10 ? atoi(argv[10]) : 0;
  const size_t pad_m = (argc > 11 ? (size_t)atoll(argv[11]) : 0) * 256;   // KB -> floats
  const size_t pad_v = (argc > 12 ? (size_t)atoll(argv[12]) : 0) * 256;
  float* big = nullptr;
  if (layout == 1 || layout == 3) {
    if (layout == 1) CK(hipMalloc(&big, (3 * nz + pad_m + pad_v) * 4));
    else CK(hipExtMallocWithFlags((void**)&big, (3 * nz + pad_m + pad_v) * 4, hipDeviceMallocContiguous));
    z = big;
    m = z + nz + pad_m;
    v = m + nz + pad_v;
  } else if (layout == 2) {                    // three physically contiguous allocations
    CK(hipExtMallocWithFlags((void**)&z, nz * 4, hipDeviceMallocContiguous));
    CK(hipExtMallocWithFlags((void**)&m, nz * 4, hipDeviceMallocContiguous));
    CK(hipExtMallocWithFlags((void**)&v, nz * 4, hipDeviceMallocContiguous));
  } else {
    CK(hipMalloc(&z, nz * 4));
    CK(hipMalloc(&m, nz * 4));
    CK(hipMalloc(&v, nz * 4));
  }
  CK(hipMalloc(&x, (size_t)L * ldn * 4));
  CK(hipMalloc(&code, (size_t)L * ldn * 2));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(z, 0, nz * 4));
  CK(hipMemset(m, 0, nz * 4));
  CK(hipMemset(v, 0, nz * 4));
  CK(hipMemset(x, 0, (size_t)L * ldn * 4));
  CK(hipMemset(code, 0, (size_t)L * ldn * 2));
  const double bytes = (double)nwt * 64 * L * (6.0 + 24.0 * P);   // the launched tiles' bytes
  const int nbt = (L + LT - 1) / LT;
  const int T = nwt * nbt;
  const dim3 grid(swap >= 2 ? (T + 7) / 8 * 8 : T);
  const size_t lds = (size_t)(160 * 1024) / wpc - 256;
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int occ[3] = {0, 0, 0};
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0], depth_stream<1>, 64, lds));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1], depth_stream<2>, 64, lds));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[2], depth_stream<3>, 64, lds));
  const float t1 = time_ms([&] { depth_stream<1><<<grid, 64, lds>>>(x, code, z, m, v, L, ldn, LT, spread, swap, nwt, sink); }, iters);
  const float t2 = time_ms([&] { depth_stream<2><<<grid, 64, lds>>>(x, code, z, m, v, L, ldn, LT, spread, swap, nwt, sink); }, iters);
  const float t3 = time_ms([&] { depth_stream<3><<<grid, 64, lds>>>(x, code, z, m, v, L, ldn, LT, spread, swap, nwt, sink); }, iters);
  const int work = argc > 8 ? atoi(argv[8]) : 0;
  // subset (9th argument, > 0): launch only the first `subset` cell tiles of the allocation (a
  // small launch over a large footprint)
  const int subset = argc > 9 ? atoi(argv[9]) : 0;
  if (subset > 0 && subset < nwt) {
    const int ns = subset, Ts = ns * nbt;
    const double bytes_s = (double)ns * 64 * L * (6.0 + 24.0 * P);
    const dim3 gs(swap >= 2 ? (Ts + 7) / 8 * 8 : Ts);
    const float ts = time_ms([&] { depth_stream<1><<<gs, 64, lds>>>(x, code, z, m, v, L, ldn, LT, spread, swap, ns, sink); }, iters);
    const float tf = time_ms([&] { depth_stream<1><<<grid, 64, lds>>>(x, code, z, m, v, L, ldn, LT, spread, swap, nwt, sink); }, iters);
    printf("subset: %d of %d cell tiles (cells %d, LT %d, order %d): %.4f ms %.3f TB/s | all %d tiles %.4f ms %.3f TB/s"
           " [z %p m-z %td B v-m %td B]\n", ns, nwt, N, LT, swap, ts, bytes_s / ts / 1e9, nwt, tf, bytes / tf / 1e9,
           (void*)z, (char*)m - (char*)z, (char*)v - (char*)m);
    return 0;
  }
  // sets (14th argument, > 1): allocate that many z / m / v sets in one process (each held while
  // the next is made) and time depth 1 on each: do some placements stream fast and others not?
  // watch (15th argument, > 0): time the same set that many times, 20 ms apart (no new
  // allocations): does one placement's speed change over time?
  const int watch = argc > 15 ? atoi(argv[15]) : 0;
  if (watch > 0) {
    for (int w = 0; w < watch; ++w) {
      const float tw = time_ms([&] { depth_stream<1><<<grid, 64, lds>>>(x, code, z, m, v, L, ldn, LT, spread, swap, nwt, sink); }, 3);
      printf("watch %d t=%d ms: %.4f ms %.3f TB/s\n", w, w * 20, tw, bytes / tw / 1e9);
      fflush(stdout);
      usleep(20000);
    }
    return 0;
  }
  const int sets = argc > 14 ? atoi(argv[14]) : 1;
  if (sets > 1) {
    printf("set 0 [z %p]: %.4f ms %.3f TB/s\n", (void*)z, t1, bytes / t1 / 1e9);
    for (int si = 1; si < sets; ++si) {
      float *z2, *m2, *v2;
      if (layout == 2) {
        CK(hipExtMallocWithFlags((void**)&z2, nz * 4, hipDeviceMallocContiguous));
        CK(hipExtMallocWithFlags((void**)&m2, nz * 4, hipDeviceMallocContiguous));
        CK(hipExtMallocWithFlags((void**)&v2, nz * 4, hipDeviceMallocContiguous));
      } else {
        CK(hipMalloc(&z2, nz * 4));
        CK(hipMalloc(&m2, nz * 4));
        CK(hipMalloc(&v2, nz * 4));
      }
      CK(hipMemset(z2, 0, nz * 4));
      CK(hipMemset(m2, 0, nz * 4));
      CK(hipMemset(v2, 0, nz * 4));
      const float ts = time_ms([&] { depth_stream<1><<<grid, 64, lds>>>(x, code, z2, m2, v2, L, ldn, LT, spread, swap, nwt, sink); }, iters);
      printf("set %d [z %p]: %.4f ms %.3f TB/s\n", si, (void*)z2, ts, bytes / ts / 1e9);
      fflush(stdout);
    }
    return 0;
  }
  if (work > 0) {                         // the schedule experiment (work_stream), order 2
    const dim3 g1((nwt * nbt + 7) / 8 * 8);
    const float a0 = time_ms([&] { work_stream<0><<<g1, 64, lds>>>(x, code, z, m, v, L, ldn, LT, nwt, work, sink); }, iters);
    const float a1 = time_ms([&] { work_stream<1><<<g1, 64, lds>>>(x, code, z, m, v, L, ldn, LT, nwt, work, sink); }, iters);
    int o0 = 0, o1 = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o0, work_stream<0>, 64, lds));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o1, work_stream<1>, 64, lds));
    printf("work %d cells %d LT %d: m/v same bin %.4f ms %.3f TB/s | m/v a bin ahead %.4f ms %.3f TB/s (occupancy %d/%d)\n",
           work, N, LT, a0, bytes / a0 / 1e9, a1, bytes / a1 / 1e9, o0, o1);
    return 0;
  }
  printf("[z %p m-z %td B v-m %td B] ", (void*)z, (char*)m - (char*)z, (char*)v - (char*)m);
  printf("spread %d swap %d cells %d bins %d LT %d tiles %d (%.2f rounds of %d x %d slots): depth1 %.4f ms %.3f TB/s | depth2 %.4f ms "
         "%.3f TB/s | depth3 %.4f ms %.3f TB/s (occupancy %d/%d/%d)\n",
         spread, swap, N, L, LT, nwt * nbt, (double)nwt * nbt / ((double)ncu * occ[0]), ncu, occ[0], t1, bytes / t1 / 1e9, t2,
         bytes / t2 / 1e9, t3, bytes / t3 / 1e9, occ[0], occ[1], occ[2]);
  return 0;
}
