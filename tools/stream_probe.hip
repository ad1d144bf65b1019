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

// (1) the pass's pattern with register loads: bin l+1's loads issued before bin l's stores
template <int WAVES>
__global__ void __launch_bounds__(64, WAVES) tile_stream(const float* __restrict__ x, const uint16_t* __restrict__ code,
                                                         float* z, float* m, float* v, int L, int ldn, int LT,
                                                         float* sink) {
  const int lane = threadIdx.x, wt = blockIdx.x;
  const int l0 = blockIdx.y * LT, l1 = min(L, l0 + LT);
  const size_t t0 = ((size_t)wt * L) * P * 64 + lane;
  float acc = 0.0f;
  float zr[P], mr[P], vr[P], xr;
  uint16_t cr;
  auto load = [&](int l) {
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      zr[k] = __builtin_nontemporal_load(z + o + k * 64);
      mr[k] = __builtin_nontemporal_load(m + o + k * 64);
      vr[k] = __builtin_nontemporal_load(v + o + k * 64);
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
    const size_t o = t0 + (size_t)l * P * 64;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const float g = __builtin_fmaf(zc[k], xc, mc[k]);
      acc += g;
      __builtin_nontemporal_store(zc[k] - 1e-30f * g, z + o + k * 64);
      __builtin_nontemporal_store(mc[k] * 0.8f + 0.2f * g, m + o + k * 64);
      __builtin_nontemporal_store(vc[k] * 0.99f + 0.01f * g * g, v + o + k * 64);
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
  CK(hipMalloc(&z, nz * 4));
  CK(hipMalloc(&m, nz * 4));
  CK(hipMalloc(&v, nz * 4));
  CK(hipMalloc(&x, (size_t)L * ldn * 4));
  CK(hipMalloc(&code, (size_t)L * ldn * 2));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(z, 0, nz * 4));
  CK(hipMemset(m, 0, nz * 4));
  CK(hipMemset(v, 0, nz * 4));
  CK(hipMemset(x, 0, (size_t)L * ldn * 4));
  CK(hipMemset(code, 0, (size_t)L * ldn * 2));
  const double bytes_pattern = (double)nwt * 64 * L * (6.0 + 24.0 * P);   // real cells' tiles
  const double bytes_alg = (double)N * L * (6.0 + 24.0 * P);
  dim3 grid(nwt, (L + LT - 1) / LT);
  printf("cells %d bins %d LT %d: tile bytes %.3f GB (algorithmic %.3f GB)\n", N, L, LT, bytes_pattern / 1e9,
         bytes_alg / 1e9);
  float t2 = time_ms([&] { tile_stream<2><<<grid, 64>>>(x, code, z, m, v, L, ldn, LT, sink); }, iters);
  float t3 = time_ms([&] { tile_stream<3><<<grid, 64>>>(x, code, z, m, v, L, ldn, LT, sink); }, iters);
  float t4 = time_ms([&] { tile_stream<4><<<grid, 64>>>(x, code, z, m, v, L, ldn, LT, sink); }, iters);
  printf("tile_stream 2 waves/SIMD: %.4f ms  %.3f TB/s (tiles)\n", t2, bytes_pattern / t2 / 1e9);
  printf("tile_stream 3 waves/SIMD: %.4f ms  %.3f TB/s\n", t3, bytes_pattern / t3 / 1e9);
  printf("tile_stream 4 waves/SIMD: %.4f ms  %.3f TB/s\n", t4, bytes_pattern / t4 / 1e9);
  const size_t n4 = nz / 4, nx4 = (size_t)L * ldn / 4;
  float tf = time_ms([&] { flat_rmw<<<256 * 16, 256>>>((float4*)z, (float4*)m, (float4*)v, (float4*)x, n4, nx4); }, iters);
  printf("flat_rmw z/m/v float4: %.4f ms  %.3f TB/s\n", tf, 24.0 * nz / tf / 1e9);
  float tc = time_ms([&] { copy4<<<256 * 16, 256>>>((float4*)z, (float4*)m, n4); }, iters);
  printf("copy4 z->m: %.4f ms  %.3f TB/s\n", tc, 8.0 * nz / tc / 1e9);
  return 0;
}
