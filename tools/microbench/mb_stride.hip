// mb_stride.hip — load-pattern study for the sweep tier (tools only, not the product). Each wave streams
// 16-KiB batches of a 1 GiB buffer into registers, 16 rows of 16 B per lane, and xor-reduces them. Lane l
// owns S contiguous bytes of each of 16384 / (64 S) quarters (S = 16: every row instruction is one
// coalesced 1-KiB read; S = 256: each lane reads its own 256-B window, 64 lines per instruction).
// 16 waves per workgroup, one workgroup per CU (the product's LDS budget is emulated with a 120-KiB
// shared array). Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_stride tools/microbench/mb_stride.hip
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

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int S, int LDSK, int QB = 4>
__global__ __launch_bounds__(1024) void k_stride(const uint8_t* img, uint64_t nbatch, uint32_t* sink) {
  __shared__ uint32_t pad[LDSK ? LDSK * 256 : 1];
  if (LDSK) pad[threadIdx.x] = threadIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int R = S / 16;             // rows per lane per quarter
  constexpr int Q = QB * 4096 / (64 * S);   // quarters per batch (QB KiB-quarters in flight per wave)
  uint32_t acc = 0;
  const uint64_t gw = (uint64_t)blockIdx.x * 16 + wave, nw = (uint64_t)gridDim.x * 16;
  const uint64_t per = (nbatch + nw - 1) / nw;
  for (uint64_t b = gw * per; b < (gw + 1) * per && b < nbatch; ++b) {
    const __amdgpu_buffer_rsrc_t rs = rsrc(img + b * (QB * 4096), QB * 4096);
    uint32_t d[64];
#pragma unroll
    for (int t = 0; t < Q; ++t)
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const v4u32 q = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(t * 64 * S + lane * S + 16 * k), 0, 0);
        d[4 * (t * R + k)] = q[0]; d[4 * (t * R + k) + 1] = q[1]; d[4 * (t * R + k) + 2] = q[2]; d[4 * (t * R + k) + 3] = q[3];
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < QB * 16; ++i) acc = (acc << 1 | acc >> 31) ^ d[i];
  }
  if (LDSK) acc ^= pad[(threadIdx.x + 1) & 1023];
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int S, int LDSK, int QB = 4>
double run(const uint8_t* img, uint64_t bytes, uint32_t* sink, int ncu) {
  const uint64_t nb = bytes / (QB * 4096);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_stride<S, LDSK, QB>), dim3(ncu), dim3(1024), 0, 0, img, nb, sink);
  CK(hipEventRecord(a, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL((k_stride<S, LDSK, QB>), dim3(ncu), dim3(1024), 0, 0, img, nb, sink);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return bytes / (ms / it * 1e-3) / 1e9;
}

int main() {
  const uint64_t bytes = 1ull << 30;
  uint8_t* img;
  uint32_t* sink;
  CK(hipMalloc(&img, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(img, 0x5A, bytes));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  std::printf("stride 64, 1 quarter (4 KiB) per wave in flight: %.0f GB/s\n", run<64, 120, 1>(img, bytes, sink, ncu));
  std::printf("stride 64, 2 quarters (8 KiB): %.0f GB/s\n", run<64, 120, 2>(img, bytes, sink, ncu));
  std::printf("stride 64, 3 quarters (12 KiB): %.0f GB/s\n", run<64, 120, 3>(img, bytes, sink, ncu));
  std::printf("stride 16: %.0f GB/s\n", run<16, 120>(img, bytes, sink, ncu));
  std::printf("stride 32: %.0f GB/s\n", run<32, 120>(img, bytes, sink, ncu));
  std::printf("stride 64: %.0f GB/s\n", run<64, 120>(img, bytes, sink, ncu));
  std::printf("stride 128: %.0f GB/s\n", run<128, 120>(img, bytes, sink, ncu));
  std::printf("stride 256: %.0f GB/s\n", run<256, 120>(img, bytes, sink, ncu));
  std::printf("stride 16, 2 wg/CU: %.0f GB/s\n", run<16, 0>(img, bytes, sink, 2 * ncu));
  std::printf("stride 64, 2 wg/CU: %.0f GB/s\n", run<64, 0>(img, bytes, sink, 2 * ncu));
  return 0;
}
