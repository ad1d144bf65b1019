// Memory-ceiling probe for the enumerated pass's access pattern (diagnostic, not product code).
//
// The step-2 pass streams, per 64-cell wave tile and bin: x (256 B) + eta code (128 B) read, and
// the pi logits z, Adam moments m, v (P x 256 B each) read and written back in place.  This
// program runs the same streams with no arithmetic beyond a dependent fma per element, so its
// time is the HBM ceiling for THIS pattern (read/write mix, per-wave contiguous runs, stream
// count) -- to compare with the 6.3 TB/s of a plain float4 copy.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_probe.hip -o tools/stream_probe
//   ./stream_probe [cells=10000] [bins=5451] [LT=48] [iters=20]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int P = 13;

// (1) the pass's pattern with register loads: bin l+1's loads issued before bin l's stores.
//   swap: blockIdx.x walks the bin tiles (consecutive workgroups = neighbouring regions)
//   inter: z, m, v of one (tile, bin) interleaved as [3][P][64] (one run per bin, 3x longer)
__global__ void __launch_bounds__(64) tile_stream(const float* __restrict__ x, const uint16_t* __restrict__ code,
                                                         float* z, float* m, float* v, int L, int ldn, int LT,
                                                         int swap, int inter, float* sink) {
  extern __shared__ float pad[];                  // occupancy cap: dynamic LDS per workgroup
  const int lane = threadIdx.x;
  if (lane == 0 && LT < 0) pad[0] = 0.0f;
  const int wt = swap ? blockIdx.y : blockIdx.x;
  const int bt = swap ? blockIdx.x : blockIdx.y;
  const int l0 = bt * LT, l1 = min(L, l0 + LT);
  const size_t t0 = ((size_t)wt * L) * P * 64 * (inter ? 3 : 1) + lane;
  const size_t bstride = (size_t)P * 64 * (inter ? 3 : 1);
  float* zb = z;
  float* mb = inter ? z + P * 64 : m;
  float* vb = inter ? z + 2 * P * 64 : v;
  float acc = 0.0f;
  float zr[P], mr[P], vr[P], xr;
  uint16_t cr;
  auto load = [&](int l) {
    const size_t o = t0 + (size_t)l * bstride;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      zr[k] = __builtin_nontemporal_load(zb + o + k * 64);
      mr[k] = __builtin_nontemporal_load(mb + o + k * 64);
      vr[k] = __builtin_nontemporal_load(vb + o + k * 64);
    }
    xr = x[(size_t)l * ldn + wt * 64 + lane];
    cr = code[(size_t)l * ldn + wt * 64 + lane];
  };
  load(l0);
  for (int l = l0; l < l1; ++l) {
    float zc[P], mc[P], vc[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
      zc[k] = zr[k];
      mc[k] = mr[k];
      vc[k] = vr[k];
    }
    const float xc = xr + (float)cr;
    if (l + 1 < l1) load(l + 1);
    const size_t o = t0 + (size_t)l * bstride;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const float g = __builtin_fmaf(zc[k], xc, mc[k]);
      acc += g;
      __builtin_nontemporal_store(zc[k] - 1e-30f * g, zb + o + k * 64);
      __builtin_nontemporal_store(mc[k] * 0.8f + 0.2f * g, mb + o + k * 64);
      __builtin_nontemporal_store(vc[k] * 0.99f + 0.01f * g * g, vb + o + k * 64);
    }
  }
  if (acc == 12345.678f) sink[0] = acc;
}

// (2) the same bytes as six flat arrays, grid-stride float4 (read-modify-write in place)
__global__ void __launch_bounds__(256) flat_rmw(float4* z, float4* m, float4* v, const float4* x, size_t n4, size_t nx4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = z[i], b = m[i], c = v[i];
    a.x += 1e-30f * b.x; a.y += 1e-30f * b.y; a.z += 1e-30f * b.z; a.w += 1e-30f * b.w;
    b.x *= 0.8f; b.y *= 0.8f; b.z *= 0.8f; b.w *= 0.8f;
    c.x *= 0.99f; c.y *= 0.99f; c.z *= 0.99f; c.w *= 0.99f;
    z[i] = a; m[i] = b; v[i] = c;
  }
}

// (2b) read-only and write-only sweeps of z, m, v (float4, 4 in flight per thread)
typedef float vf4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) read3(const vf4* __restrict__ z, const vf4* __restrict__ m,
                                             const vf4* __restrict__ v, size_t n4, float* sink) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  float acc = 0.0f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const vf4 a = __builtin_nontemporal_load(z + i), b = __builtin_nontemporal_load(m + i),
                 c = __builtin_nontemporal_load(v + i);
    acc += a.x + b.y + c.z + a.w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}
__global__ void __launch_bounds__(256) write3(vf4* z, vf4* m, vf4* v, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const vf4 q = {1.0f, 2.0f, 3.0f, 4.0f};
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    __builtin_nontemporal_store(q, z + i);
    __builtin_nontemporal_store(q, m + i);
    __builtin_nontemporal_store(q, v + i);
  }
}

// (3) plain float4 copy a -> b
__global__ void __launch_bounds__(256) copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) b[i] = a[i];
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
  const int N = argc > 1 ? atoi(argv[1]) : 10000;
  const int L = argc > 2 ? atoi(argv[2]) : 5451;
  const int LT = argc > 3 ? atoi(argv[3]) : 48;
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  const int ldn = (N + 255) / 256 * 256;
  const int nwt = (N + 63) / 64;
  const size_t nz = (size_t)(ldn / 64) * L * P * 64;
  float *z, *m, *v, *x, *sink;
  uint16_t* code;
  CK(hipMalloc(&z, nz * 4 * 3));
  CK(hipMalloc(&m, nz * 4));
  CK(hipMalloc(&v, nz * 4));
  CK(hipMalloc(&x, (size_t)L * ldn * 4));
  CK(hipMalloc(&code, (size_t)L * ldn * 2));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(z, 0, nz * 4 * 3));
  CK(hipMemset(m, 0, nz * 4));
  CK(hipMemset(v, 0, nz * 4));
  CK(hipMemset(x, 0, (size_t)L * ldn * 4));
  CK(hipMemset(code, 0, (size_t)L * ldn * 2));
  const double bytes_pattern = (double)nwt * 64 * L * (6.0 + 24.0 * P);   // real cells' tiles
  const double bytes_alg = (double)N * L * (6.0 + 24.0 * P);
  printf("cells %d bins %d: tile bytes %.3f GB (algorithmic %.3f GB)\n", N, L, bytes_pattern / 1e9, bytes_alg / 1e9);
  // placement of m and v relative to z (one allocation): m = z + nz + dm, v = m + nz + dv floats
  float* big;
  const size_t slack = (size_t)64 << 20;                       // floats (256 MB)
  CK(hipMalloc(&big, (3 * nz + 2 * slack) * 4));
  CK(hipMemset(big, 0, (3 * nz + 2 * slack) * 4));
  const size_t pads[][2] = {{0, 0}, {64, 128}, {1024, 2048}, {16384, 32768}, {262144, 524288},
                            {(1 << 20) + 64, (1 << 21) + 128}, {(size_t)3 << 19, (size_t)5 << 19},
                            {(size_t)1 << 24, (size_t)1 << 25}, {((size_t)1 << 22) + 4096, ((size_t)1 << 23) + 8192}};
  const int nbt = (L + LT - 1) / LT;
  dim3 grid(nwt, nbt);
  const size_t lds = (160 * 1024) / 8 - 256;
  for (auto& pd : pads) {
    float* zz = big;
    float* mm = zz + nz + pd[0];
    float* vv = mm + nz + pd[1];
    float t = time_ms([&] { tile_stream<<<grid, 64, lds>>>(x, code, zz, mm, vv, L, ldn, LT, 0, 0, sink); }, iters);
    printf("pad m +%9zu B, v +%9zu B (m-z %12zu B): LT %d %.4f ms %.3f TB/s\n", pd[0] * 4, pd[1] * 4,
           (size_t)(mm - zz) * 4, LT, t, bytes_pattern / t / 1e9);
  }
  {  // the separate allocations as the extension gets them
    float t = time_ms([&] { tile_stream<<<grid, 64, lds>>>(x, code, z, m, v, L, ldn, LT, 0, 0, sink); }, iters);
    printf("separate hipMalloc z/m/v (m-z %td B, v-m %td B): %.4f ms %.3f TB/s\n", (char*)m - (char*)z,
           (char*)v - (char*)m, t, bytes_pattern / t / 1e9);
  }
  CK(hipFree(big));
  const size_t n4 = nz / 4, nx4 = (size_t)L * ldn / 4;
  float tf = time_ms([&] { flat_rmw<<<256 * 16, 256>>>((float4*)z, (float4*)m, (float4*)v, (float4*)x, n4, nx4); }, iters);
  printf("flat_rmw z/m/v float4: %.4f ms  %.3f TB/s\n", tf, 24.0 * nz / tf / 1e9);
  float tc = time_ms([&] { copy4<<<256 * 16, 256>>>((float4*)z, (float4*)m, n4); }, iters);
  printf("copy4 z->m: %.4f ms  %.3f TB/s\n", tc, 8.0 * nz / tc / 1e9);
  for (int g : {1024, 4096, 16384}) {
    float tr = time_ms([&] { read3<<<g, 256>>>((vf4*)z, (vf4*)m, (vf4*)v, n4, sink); }, iters);
    float tw = time_ms([&] { write3<<<g, 256>>>((vf4*)z, (vf4*)m, (vf4*)v, n4); }, iters);
    float tcc = time_ms([&] { copy4<<<g, 256>>>((float4*)z, (float4*)m, n4); }, iters);
    printf("grid %5d: read3 %.3f TB/s  write3 %.3f TB/s  copy4 %.3f TB/s\n", g, 12.0 * nz / tr / 1e9,
           12.0 * nz / tw / 1e9, 8.0 * nz / tcc / 1e9);
  }
  return 0;
}
