// Synthetic GPU load for the overhead benchmark.
//
// Three calibrated gfx950 kernels whose throughput is the yardstick for the
// exporter's GPU-time overhead (sampler on vs off, same device):
//
//  * mfma_bf16  — matrix-core bound: every wave keeps four independent
//                 v_mfma_f32_16x16x32_bf16 accumulators busy on register-resident
//                 fragments (16 cycles/MFMA/SIMD issue rate, MI355X_MICROARCH.md
//                 cycle table), computing C = iters · (A·B) for a 16×64 tile so the
//                 result is checkable against torch.
//  * triad_f32  — HBM bound: c = a + s·b with 16-byte (float4) accesses,
//                 grid sized to ≫256 CUs, nontemporal loads (once-read stream).
//  * copy_f32   — float4 copy; with a peer-device source pointer this is the
//                 xGMI peer-read load (hipDeviceEnablePeerAccess first).
//
// C ABI only (loaded with ctypes by kube_gpu_stats_amd/ops/load.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x4 = __attribute__((ext_vector_type(4))) float;  // also the 16-byte stream unit

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves, one per SIMD of the CU

thread_local char g_err[256];

// A: [16][32] bf16 row-major, B: [32][64] bf16 row-major, C: [nwaves][16][64] f32.
__global__ __launch_bounds__(kBlock) void mfma_bf16_kernel(const unsigned short* __restrict__ A,
                                                           const unsigned short* __restrict__ B,
                                                           float* __restrict__ C, int iters) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = (blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int r = lane & 15;          // A row / B column within a 16-wide tile
  const int kb = (lane >> 4) * 8;   // k base of this lane's 8 elements

  bf16x8 a, b[4];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = static_cast<short>(A[r * 32 + kb + j]);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) b[t][j] = static_cast<short>(B[(kb + j) * 64 + t * 16 + r]);

  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[t], acc[t], 0, 0, 0);
  }

  // C/D map for 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + reg.
  float* out = C + static_cast<size_t>(wave) * 16 * 64;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[((lane >> 4) * 4 + i) * 64 + t * 16 + (lane & 15)] = acc[t][i];
}

__global__ __launch_bounds__(kBlock) void triad_f32_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                           f32x4* __restrict__ c, float s, size_t n4) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) {
    const f32x4 x = __builtin_nontemporal_load(a + i);
    const f32x4 y = __builtin_nontemporal_load(b + i);
    c[i] = x + s * y;
  }
}

__global__ __launch_bounds__(kBlock) void copy_f32_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                          size_t n4) {
  const size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
  for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride)
    dst[i] = __builtin_nontemporal_load(src + i);
}

int check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  std::snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
  return -1;
}

}  // namespace

extern "C" {

const char* kgs_load_last_error() { return g_err; }

int kgs_load_block_size() { return kBlock; }

// C must hold nblocks * 4 waves * 16 * 64 floats.
int kgs_load_mfma_bf16(const void* A, const void* B, float* C, int nblocks, int iters, void* stream) {
  if (nblocks <= 0 || iters < 0) return check(hipErrorInvalidValue, "mfma_bf16 args");
  hipLaunchKernelGGL(mfma_bf16_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B), C, iters);
  return check(hipGetLastError(), "mfma_bf16 launch");
}

// n must be a multiple of 4 and pointers 16-byte aligned.
int kgs_load_triad_f32(const float* a, const float* b, float* c, float s, size_t n, int nblocks, void* stream) {
  if ((n & 3) || nblocks <= 0) return check(hipErrorInvalidValue, "triad_f32 args");
  hipLaunchKernelGGL(triad_f32_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b),
                     reinterpret_cast<f32x4*>(c), s, n / 4);
  return check(hipGetLastError(), "triad_f32 launch");
}

int kgs_load_copy_f32(const float* src, float* dst, size_t n, int nblocks, void* stream) {
  if ((n & 3) || nblocks <= 0) return check(hipErrorInvalidValue, "copy_f32 args");
  hipLaunchKernelGGL(copy_f32_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(src), reinterpret_cast<f32x4*>(dst), n / 4);
  return check(hipGetLastError(), "copy_f32 launch");
}

int kgs_load_enable_peer(int dev, int peer) {
  int can = 0;
  if (check(hipDeviceCanAccessPeer(&can, dev, peer), "hipDeviceCanAccessPeer")) return -1;
  if (!can) return check(hipErrorPeerAccessUnsupported, "peer access unsupported");
  int cur = 0;
  if (check(hipGetDevice(&cur), "hipGetDevice") || check(hipSetDevice(dev), "hipSetDevice")) return -1;
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (check(hipSetDevice(cur), "hipSetDevice")) return -1;
  if (e == hipErrorPeerAccessAlreadyEnabled) return 0;
  return check(e, "hipDeviceEnablePeerAccess");
}

}  // extern "C"
