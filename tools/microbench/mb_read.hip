// mb_read.hip — streaming-read ceiling variants on a 4 GiB device buffer (tools only, not the product).
// Each variant XOR-reduces every 16-B word once, so the compiler keeps every load; the rate is
// bytes / kernel time (HIP events over 10 launches after one warm-up).
//   plain4   : grid-stride, 4 x 16-B loads in flight per lane (the product's ldb_read_ceiling today)
//   plain8   : the same with 8 in flight
//   nt8      : 8 in flight, nontemporal loads
//   chunk    : each wave sweeps its own contiguous chunk, 8 x 1 KiB wave-loads in flight
//   dma      : global_load_lds_dwordx4 into a per-wave LDS ring (8 x 1 KiB slots), read back by ds_read_b128
// Build: hipcc --offload-arch=gfx950 -O3 -o mb_read tools/microbench/mb_read.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_plain(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t acc = 0;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        typedef unsigned int v4 __attribute__((ext_vector_type(4)));
        const v4 v = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p + i + u * stride));
        x[u] = make_uint4(v[0], v[1], v[2], v[3]);
      } else {
        x[u] = p[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
  }
  for (; i < n16; i += stride) {
    const uint4 x = p[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

// each wave owns a contiguous chunk of the buffer (8 wave-loads of 1 KiB in flight)
__global__ __launch_bounds__(256) void k_chunk(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t per = (n16 / 64 + waves - 1) / waves * 64;   // 16-B words per wave, a multiple of 64
  const uint64_t a = w * per, b = a + per < n16 ? a + per : n16;
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  uint64_t i = a + lane;
  for (; i + 7 * 64 < b; i += 8 * 64) {
    uint4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = p[i + u * 64];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
  }
  for (; i < b; i += 64) {
    const uint4 x = p[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

// LDS-DMA ring: each wave sweeps its own contiguous chunk through 8 slots of 1 KiB; slot k is
// refilled as soon as it was read back
__global__ __launch_bounds__(256) void k_dma(const uint8_t* __restrict__ p, uint64_t nbytes, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][8][1024];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t)gridDim.x * 4;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + wave;
  const uint64_t nk = nbytes / 1024;   // whole KiB pieces
  const uint64_t per = (nk + waves - 1) / waves;
  const uint64_t a = w * per, b = a + per < nk ? a + per : nk;
  const uint32_t base = (uint32_t)(uintptr_t)&ring[wave][0][0];
  uint32_t acc = 0;
  uint64_t k = a;
  for (int s = 0; s < 8 && k + s < b; ++s) glds16(p + (k + s) * 1024 + lane * 16, base + s * 1024);
  for (; k < b; ++k) {
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    if (b - k < 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int s = (int)((k - a) & 7);
    const uint4 x = *reinterpret_cast<const uint4*>(&ring[wave][s][lane * 16]);
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (k + 8 < b) glds16(p + (k + 8) * 1024 + lane * 16, base + s * 1024);
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

int main() {
  const uint64_t nbytes = 4ull << 30, n16 = nbytes / 16;
  uint8_t* d = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&d, nbytes));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(d, 0x5A, nbytes));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%-8s %8.3f ms  %7.1f GB/s\n", name, ms / 10, nbytes / (ms / 10 * 1e-3) / 1e9);
  };
  for (int g : {4, 8, 16}) {
    std::printf("grid %d blocks/CU of 256 threads\n", g);
    const unsigned grid = ncu * g;
    run("plain4", [&] { hipLaunchKernelGGL((k_plain<4, false>), dim3(grid), dim3(256), 0, 0, (const uint4*)d, n16, sink); });
    run("plain8", [&] { hipLaunchKernelGGL((k_plain<8, false>), dim3(grid), dim3(256), 0, 0, (const uint4*)d, n16, sink); });
    run("nt8", [&] { hipLaunchKernelGGL((k_plain<8, true>), dim3(grid), dim3(256), 0, 0, (const uint4*)d, n16, sink); });
    run("chunk", [&] { hipLaunchKernelGGL(k_chunk, dim3(grid), dim3(256), 0, 0, (const uint4*)d, n16, sink); });
    run("dma", [&] { hipLaunchKernelGGL(k_dma, dim3(grid), dim3(256), 0, 0, (const uint8_t*)d, nbytes, sink); });
  }
  CK(hipFree(d));
  CK(hipFree(sink));
  return 0;
}
