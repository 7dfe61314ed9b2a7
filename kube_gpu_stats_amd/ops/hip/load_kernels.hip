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
//  * copy_f32   — float4 copy; with a peer-device source or destination pointer
//                 this is the xGMI peer load (hipDeviceEnablePeerAccess first).
//  * gather64 / reread — HBM-model validation patterns: random 64 B lines over
//                 a large buffer, and repeated sweeps of a cache-resident one.
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
//
// The iteration loop is one inline-asm block: with the builtin, hipcc rotates
// the four accumulators through AGPR copies every trip (≈20 v_accvgpr moves per
// 4 MFMAs, half of peak measured on MI355X).  Here each accumulator is pinned
// ("+a"), MFMA→MFMA accumulate chains need no wait states, the loop counter is
// SALU work that issues beside the matrix pipe, and the block ends with 20 wait
// states before the compiler's first read of the accumulators
// (cdna_hip_programming.md §5.7 item 2).
//
// xcc_mask: a workgroup runs the loop only if bit <its XCC> is set, read from the
// hardware (HW_REG_XCC_ID) rather than assumed from blockIdx — this is how the
// per-XCD counter tests load exactly the XCDs they name.  xcc_out (optional)
// receives each workgroup's XCC id.
__global__ __launch_bounds__(kBlock) void mfma_bf16_kernel(const unsigned short* __restrict__ A,
                                                           const unsigned short* __restrict__ B,
                                                           float* __restrict__ C, int iters, unsigned xcc_mask,
                                                           int* __restrict__ xcc_out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = (blockIdx.x * kBlock + threadIdx.x) / kWave;
  const int r = lane & 15;          // A row / B column within a 16-wide tile
  const int kb = (lane >> 4) * 8;   // k base of this lane's 8 elements
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 0xF;
  if (xcc_out && threadIdx.x == 0) xcc_out[blockIdx.x] = static_cast<int>(xcc);

  bf16x8 a, b0, b1, b2, b3;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<short>(A[r * 32 + kb + j]);
    b0[j] = static_cast<short>(B[(kb + j) * 64 + r]);
    b1[j] = static_cast<short>(B[(kb + j) * 64 + 16 + r]);
    b2[j] = static_cast<short>(B[(kb + j) * 64 + 32 + r]);
    b3[j] = static_cast<short>(B[(kb + j) * 64 + 48 + r]);
  }
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, c2 = c0, c3 = c0;
  int n = ((xcc_mask >> xcc) & 1u) ? iters : 0;
  if (n > 0) {
    asm volatile(
        "s_nop 4\n"
        "1:\n\t"
        "v_mfma_f32_16x16x32_bf16 %0, %5, %6, %0\n\t"
        "v_mfma_f32_16x16x32_bf16 %1, %5, %7, %1\n\t"
        "v_mfma_f32_16x16x32_bf16 %2, %5, %8, %2\n\t"
        "v_mfma_f32_16x16x32_bf16 %3, %5, %9, %3\n\t"
        "s_sub_u32 %4, %4, 1\n\t"
        "s_cmp_lg_u32 %4, 0\n\t"
        "s_cbranch_scc1 1b\n\t"
        "s_nop 15\n\t"
        "s_nop 3"
        : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3), "+s"(n)
        : "v"(a), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
        : "scc");
  }

  // C/D map for 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + reg.
  float* out = C + static_cast<size_t>(wave) * 16 * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* row = out + ((lane >> 4) * 4 + i) * 64 + (lane & 15);
    row[0] = c0[i];
    row[16] = c1[i];
    row[32] = c2[i];
    row[48] = c3[i];
  }
}

// Four independent 16-byte loads per operand in flight per lane per trip.
// NT: nontemporal loads (once-read stream) vs default cache policy.
template <bool NT>
__device__ inline f32x4 ld(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__device__ inline void st(f32x4 v, f32x4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Each block streams one contiguous chunk (4 × 16 B per lane in flight per
// operand, 1 KiB per wave-instruction) instead of a grid-stride walk: measured on
// MI355X over 6 GiB, 5.6-5.7 TB/s vs 4.6-5.0 TB/s for the grid-stride forms
// (tools/stream_variants.hip → profiles/r1/stream_variants.json); once-touched
// data goes nontemporal both ways so it does not churn L2 / Infinity Cache.
template <bool NT>
__global__ __launch_bounds__(kBlock) void triad_f32_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                           f32x4* __restrict__ c, float s, size_t n4) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t lo = static_cast<size_t>(blockIdx.x) * per;
  const size_t hi = lo + per < n4 ? lo + per : n4;
  size_t i = lo + threadIdx.x;
  for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
    f32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x[u] = ld<NT>(a + i + u * kBlock);
      y[u] = ld<NT>(b + i + u * kBlock);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) st<NT>(x[u] + s * y[u], c + i + u * kBlock);
  }
  for (; i < hi; i += kBlock) st<NT>(ld<NT>(a + i) + s * ld<NT>(b + i), c + i);
}

// Triad on the XCDs in xcc_mask only (HW_REG_XCC_ID), for the per-XCD
// vector-memory counter test; workgroups elsewhere return at once.
__global__ __launch_bounds__(kBlock) void triad_xcc_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                           f32x4* __restrict__ c, float s, size_t n4,
                                                           unsigned xcc_mask) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (!((xcc_mask >> (xcc & 0xF)) & 1u)) return;
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t lo = static_cast<size_t>(blockIdx.x) * per;
  const size_t hi = lo + per < n4 ? lo + per : n4;
  for (size_t i = lo + threadIdx.x; i < hi; i += kBlock) st<true>(ld<true>(a + i) + s * ld<true>(b + i), c + i);
}

__global__ __launch_bounds__(kBlock) void copy_f32_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                          size_t n4) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t lo = static_cast<size_t>(blockIdx.x) * per;
  const size_t hi = lo + per < n4 ? lo + per : n4;
  size_t i = lo + threadIdx.x;
  for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
    f32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = ld<true>(src + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < 4; ++u) st<true>(x[u], dst + i + u * kBlock);
  }
  for (; i < hi; i += kBlock) st<true>(ld<true>(src + i), dst + i);
}

// Random 64-byte gather (HBM-model validation, profiles/umc_calib.md): thread t
// reads `per_thread` 64 B lines (four 16-byte loads each) chosen by a 32-bit LCG
// seeded with t, line = (x >> shift) & (nlines - 1) over a power-of-two number of
// lines, and writes the sum of the floats it read.  Every lane of a wave hits a
// different line, so each wave-load is 64 independent 64 B requests over the whole
// buffer: the small-granularity, TLB- and row-hostile end of HBM traffic, where
// memory-controller activity and requested bytes can part ways.  The LCG is
// replayed in torch for the numerics check (tests/test_gpu.py).
__global__ __launch_bounds__(kBlock) void gather64_kernel(const f32x4* __restrict__ src, uint32_t nlines_mask,
                                                          int shift, int per_thread, uint32_t seed,
                                                          float* __restrict__ out) {
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  uint32_t x = seed ^ (t * 2654435761u);
  float acc = 0.f;
  for (int j = 0; j < per_thread; ++j) {
    x = x * 1664525u + 1013904223u;
    const f32x4* p = src + static_cast<size_t>((x >> shift) & nlines_mask) * 4;
    f32x4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
    f32x4 v = (v0 + v1) + (v2 + v3);
    acc += (v[0] + v[1]) + (v[2] + v[3]);
  }
  out[t] = acc;
}

// Cache-resident re-read (HBM-model validation): `passes` sweeps over a small
// buffer (≤ 128 MiB: MI355X's L2 is 4 MiB per XCD and the Infinity Cache / MALL
// 256 MiB), default cache policy, thread t summing src4[t], src4[t + T], ... each
// pass.  Requested bytes are passes × size; HBM sees the first touch (and what
// the caches evict), so the UMC-activity model should read far below the request.
__global__ __launch_bounds__(kBlock) void reread_kernel(const f32x4* __restrict__ src, size_t n4, int passes,
                                                        float* __restrict__ out) {
  const size_t T = static_cast<size_t>(gridDim.x) * kBlock;
  const size_t t = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  float acc = 0.f;
  for (int p = 0; p < passes; ++p) {
    asm volatile("" ::: "memory");  // every pass reloads (no hoisting across passes)
    f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = t; i < n4; i += T) s4 += src[i];
    acc += (s4[0] + s4[1]) + (s4[2] + s4[3]);
  }
  out[t] = acc;
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
int kgs_load_mfma_bf16_xcc(const void* A, const void* B, float* C, int nblocks, int iters, unsigned xcc_mask,
                           int* xcc_out, void* stream) {
  if (nblocks <= 0 || iters < 0) return check(hipErrorInvalidValue, "mfma_bf16 args");
  hipLaunchKernelGGL(mfma_bf16_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     static_cast<const unsigned short*>(A), static_cast<const unsigned short*>(B), C, iters,
                     xcc_mask, xcc_out);
  return check(hipGetLastError(), "mfma_bf16 launch");
}

int kgs_load_mfma_bf16(const void* A, const void* B, float* C, int nblocks, int iters, void* stream) {
  return kgs_load_mfma_bf16_xcc(A, B, C, nblocks, iters, 0xFFFFu, nullptr, stream);
}

// n must be a multiple of 4 and pointers 16-byte aligned.
int kgs_load_triad_f32_ex(const float* a, const float* b, float* c, float s, size_t n, int nblocks, int nt,
                          void* stream) {
  if ((n & 3) || nblocks <= 0) return check(hipErrorInvalidValue, "triad_f32 args");
  if (nt)
    hipLaunchKernelGGL(triad_f32_kernel<true>, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b),
                       reinterpret_cast<f32x4*>(c), s, n / 4);
  else
    hipLaunchKernelGGL(triad_f32_kernel<false>, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b),
                       reinterpret_cast<f32x4*>(c), s, n / 4);
  return check(hipGetLastError(), "triad_f32 launch");
}

int kgs_load_triad_f32(const float* a, const float* b, float* c, float s, size_t n, int nblocks, void* stream) {
  return kgs_load_triad_f32_ex(a, b, c, s, n, nblocks, 1, stream);
}

int kgs_load_triad_f32_xcc(const float* a, const float* b, float* c, float s, size_t n, int nblocks,
                           unsigned xcc_mask, void* stream) {
  if ((n & 3) || nblocks <= 0) return check(hipErrorInvalidValue, "triad_f32_xcc args");
  hipLaunchKernelGGL(triad_xcc_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b), reinterpret_cast<f32x4*>(c),
                     s, n / 4, xcc_mask);
  return check(hipGetLastError(), "triad_f32_xcc launch");
}

int kgs_load_copy_f32(const float* src, float* dst, size_t n, int nblocks, void* stream) {
  if ((n & 3) || nblocks <= 0) return check(hipErrorInvalidValue, "copy_f32 args");
  hipLaunchKernelGGL(copy_f32_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(src), reinterpret_cast<f32x4*>(dst), n / 4);
  return check(hipGetLastError(), "copy_f32 launch");
}

// nlines must be a power of two (64 B lines), shift = 32 - log2(nlines) ... any
// shift in [0, 31]: the line index is (x >> shift) & (nlines - 1).  out: nblocks*256.
int kgs_load_gather64(const float* src, uint32_t nlines, int shift, int per_thread, uint32_t seed, int nblocks,
                      float* out, void* stream) {
  if (nlines == 0 || (nlines & (nlines - 1)) || shift < 0 || shift > 31 || per_thread <= 0 || nblocks <= 0)
    return check(hipErrorInvalidValue, "gather64 args");
  hipLaunchKernelGGL(gather64_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(src), nlines - 1, shift, per_thread, seed, out);
  return check(hipGetLastError(), "gather64 launch");
}

// n must be a multiple of 4; out: nblocks*256 floats.
int kgs_load_reread(const float* src, size_t n, int passes, int nblocks, float* out, void* stream) {
  if ((n & 3) || passes <= 0 || nblocks <= 0) return check(hipErrorInvalidValue, "reread args");
  hipLaunchKernelGGL(reread_kernel, dim3(nblocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(src), n / 4, passes, out);
  return check(hipGetLastError(), "reread launch");
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
