// Microbenchmark of HBM stream-kernel variants on MI355X (tools/ only; the
// winner goes into kube_gpu_stats_amd/ops/hip/load_kernels.hip).
//   hipcc --offload-arch=gfx950 -O3 -o stream_variants tools/stream_variants.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

using f4 = __attribute__((ext_vector_type(4))) float;
#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::printf("{\"error\":\"%s line %d\"}\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void triad_gs(const f4* __restrict__ a, const f4* __restrict__ b, f4* __restrict__ c,
                                                float s, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * 256;
  size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = NTL ? __builtin_nontemporal_load(a + i + u * stride) : a[i + u * stride];
      y[u] = NTL ? __builtin_nontemporal_load(b + i + u * stride) : b[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(x[u] + s * y[u], c + i + u * stride);
      else c[i + u * stride] = x[u] + s * y[u];
    }
  }
  for (; i < n; i += stride) c[i] = a[i] + s * b[i];
}

// contiguous chunk per block, U float4 per thread per trip
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void triad_chunk(const f4* __restrict__ a, const f4* __restrict__ b,
                                                   f4* __restrict__ c, float s, size_t n) {
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = static_cast<size_t>(blockIdx.x) * per;
  const size_t hi = lo + per < n ? lo + per : n;
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * 256 < hi; i += U * 256) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u] = NTL ? __builtin_nontemporal_load(a + i + u * 256) : a[i + u * 256];
      y[u] = NTL ? __builtin_nontemporal_load(b + i + u * 256) : b[i + u * 256];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(x[u] + s * y[u], c + i + u * 256);
      else c[i + u * 256] = x[u] + s * y[u];
    }
  }
  for (; i < hi; i += 256) c[i] = a[i] + s * b[i];
}

template <class K>
float run(K k, int blocks, const f4* a, const f4* b, f4* c, size_t n, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, a, b, c, 1.5f, n);
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, a, b, c, 1.5f, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const size_t bytes_per = 2ull << 30;  // 2 GiB per array, 6 GiB total ≫ 256 MiB Infinity Cache
  const size_t n = bytes_per / sizeof(f4);
  f4 *a, *b, *c;
  CK(hipMalloc(&a, bytes_per));
  CK(hipMalloc(&b, bytes_per));
  CK(hipMalloc(&c, bytes_per));
  CK(hipMemset(a, 0, bytes_per));
  CK(hipMemset(b, 0, bytes_per));
  const int grids[] = {1024, 2048, 4096, 8192, 16384};
  std::printf("[\n");
  bool first = true;
  auto rep = [&](const char* name, int g, float ms) {
    std::printf("%s{\"variant\":\"%s\",\"blocks\":%d,\"ms\":%.4f,\"TBps\":%.3f}\n", first ? "" : ",", name, g, ms,
                3.0 * bytes_per / (ms * 1e-3) / 1e12);
    first = false;
  };
  for (int g : grids) {
    rep("gs_u4_ntl", g, run(triad_gs<4, true, false>, g, a, b, c, n, 10));
    rep("gs_u4_plain", g, run(triad_gs<4, false, false>, g, a, b, c, n, 10));
    rep("gs_u4_nts", g, run(triad_gs<4, false, true>, g, a, b, c, n, 10));
    rep("gs_u8_plain", g, run(triad_gs<8, false, false>, g, a, b, c, n, 10));
    rep("gs_u2_plain", g, run(triad_gs<2, false, false>, g, a, b, c, n, 10));
    rep("chunk_u4_plain", g, run(triad_chunk<4, false, false>, g, a, b, c, n, 10));
    rep("chunk_u8_plain", g, run(triad_chunk<8, false, false>, g, a, b, c, n, 10));
    rep("chunk_u4_ntl_nts", g, run(triad_chunk<4, true, true>, g, a, b, c, n, 10));
  }
  std::printf("]\n");
  CK(hipDeviceSynchronize());
  return 0;
}
