// mb_rw.hip — can the run prefix's tuple writes hide under its reads? (tools only, not the product)
// A 4 GiB read stream (16 waves per CU, 16-B loads into registers, xor-reduced) plus 207 MB of 16-B streaming
// stores (config 4's INDEX tuples: 4 GiB / 332 B x 16 B), either after each wave's reads (the product's
// uni_post_fill shape: a dense sweep per workgroup at its end) or interleaved (one 1 KiB chunk per wave every
// kEvery loop rounds). Back-to-back launches, average time from events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_rw tools/microbench/mb_rw.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// kMode 0: reads only; 1: reads, then the workgroup's slice of writes; 2: writes interleaved every kEvery rounds;
// 3: writes first, then reads; 4: odd workgroups write first, even ones last; 5: as 1 with plain stores;
// 6: the writes alone
template <int kMode, int kEvery>
__global__ __launch_bounds__(1024) void k_rw(const uint4* __restrict__ in, uint64_t n16, uint4* out, uint64_t m16,
                                             uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool first = kMode == 3 || (kMode == 4 && (blockIdx.x & 1));
  const uint64_t nw = (uint64_t)gridDim.x * 16, gw = (uint64_t)blockIdx.x * 16 + wave;
  // reads: wave gw takes rounds of 8 KiB (8 loads of 1 KiB per wave), rounds interleaved over the waves
  const uint64_t rounds = n16 / 512;
  // writes: the workgroup's slice, dealt over its waves in 1 KiB chunks
  const uint64_t per_wg = (m16 + gridDim.x - 1) / gridDim.x;
  const uint64_t w_lo = (uint64_t)blockIdx.x * per_wg, w_hi = w_lo + per_wg < m16 ? w_lo + per_wg : m16;
  uint64_t wc = w_lo + (uint64_t)wave * 64;   // this wave's next chunk
  uint32_t acc = 0, it = 0;
  if (first) {
    for (; wc < w_hi; wc += 16 * 64) {
      const uint64_t i = wc + lane;
      if (i < w_hi) {
        const u32x4 t = {(uint32_t)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(out + i));
      }
    }
  }
  for (uint64_t r = gw; kMode != 6 && r < rounds; r += nw) {
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + r * 512 + k * 64 + lane));
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= x[k][0] ^ x[k][1] ^ x[k][2] ^ x[k][3];
    if (kMode == 2 && ++it == kEvery) {
      it = 0;
      if (wc < w_hi) {
        const uint64_t i = wc + lane;
        if (i < w_hi) {
          const u32x4 t = {(uint32_t)i, 1u, 2u, 3u};
          __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(out + i));
        }
        wc += 16 * 64;
      }
    }
  }
  if (kMode >= 1 && !first) {
    for (; wc < w_hi; wc += 16 * 64) {
      const uint64_t i = wc + lane;
      if (i < w_hi) {
        const u32x4 t = {(uint32_t)i, 1u, 2u, 3u};
        if (kMode == 5) *reinterpret_cast<u32x4*>(out + i) = t;   // plain store (write-back L2)
        else __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(out + i));
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int kMode, int kEvery>
double run(const uint4* in, uint64_t n16, uint4* out, uint64_t m16, uint32_t* sink, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_rw<kMode, kEvery>), dim3(grid), dim3(1024), 0, 0, in, n16, out, m16, sink);
  CK(hipEventRecord(a, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_rw<kMode, kEvery>), dim3(grid), dim3(1024), 0, 0, in, n16, out, m16, sink);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / it;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t nb = 4ull << 30, mb = nb / 332 * 16;
  uint4 *in, *out;
  uint32_t* sink;
  CK(hipMalloc(&in, nb));
  CK(hipMalloc(&out, mb + 4096));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(in, 1, nb));
  const uint64_t n16 = nb / 16, m16 = mb / 16;
  std::printf("reads 4 GiB, writes %.1f MB, grid %d x 1024\n", mb / 1e6, ncu);
  const double r0 = run<0, 1>(in, n16, out, m16, sink, ncu);
  std::printf("reads only          %.4f ms (%.0f GB/s)\n", r0, nb / r0 / 1e6);
  const double r1 = run<1, 1>(in, n16, out, m16, sink, ncu);
  std::printf("reads then writes   %.4f ms\n", r1);
  std::printf("reads then plain writes %.4f ms\n", run<5, 1>(in, n16, out, m16, sink, ncu));
  const double w6 = run<6, 1>(in, n16, out, m16, sink, ncu);
  std::printf("writes alone        %.4f ms (%.0f GB/s)\n", w6, mb / w6 / 1e6);
  const double w6b = run<6, 1>(in, n16, out, m16, sink, 4 * ncu);
  std::printf("writes alone, 4 workgroups per CU %.4f ms (%.0f GB/s)\n", w6b, mb / w6b / 1e6);
  std::printf("writes then reads   %.4f ms\n", run<3, 1>(in, n16, out, m16, sink, ncu));
  std::printf("half first, half last %.4f ms\n", run<4, 1>(in, n16, out, m16, sink, ncu));
  std::printf("reads only (again) %.4f ms, reads then writes (again) %.4f ms\n", run<0, 1>(in, n16, out, m16, sink, ncu),
              run<1, 1>(in, n16, out, m16, sink, ncu));
  std::printf("interleaved every 1 %.4f ms\n", run<2, 1>(in, n16, out, m16, sink, ncu));
  std::printf("interleaved every 2 %.4f ms\n", run<2, 2>(in, n16, out, m16, sink, ncu));
  std::printf("interleaved every 3 %.4f ms\n", run<2, 3>(in, n16, out, m16, sink, ncu));
  std::printf("interleaved every 4 %.4f ms\n", run<2, 4>(in, n16, out, m16, sink, ncu));
  return 0;
}
