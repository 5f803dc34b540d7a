// mb_launch.hip — what a launch that exits at once costs (tools only, not the product). A scan whose run
// prefix covers the file still enqueues the tail kernels, and each leaves at its first instruction after
// reading the done word; their cost is the dispatch of their workgroups. Chains of N such kernels are timed
// back to back with events, per grid / block / LDS shape, and after a 256 MiB streaming-store kernel (the
// run prefix's INDEX sweep leaves that much behind it).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_launch tools/microbench/mb_launch.hip
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

constexpr uint64_t kMagic = 0xD0E5CA11D0E5CA11ull;

template <int LDSW>
__global__ void k_noop(const uint64_t* done, uint32_t* sink) {
  __shared__ uint32_t pad[LDSW ? LDSW : 1];
  if (*done == kMagic) return;
  if (LDSW) pad[threadIdx.x % (LDSW ? LDSW : 1)] = threadIdx.x;
  __syncthreads();
  if (LDSW && pad[(threadIdx.x + 1) % (LDSW ? LDSW : 1)] == 0xFFFFFFFFu) sink[0] = 1;
}

// the product's tail kernels' properties, one at a time: a 480-B kernarg struct by value, a private
// segment (scratch), 128 VGPRs, a large body behind the exit
struct Big {
  const uint64_t* done;
  uint32_t* sink;
  uint64_t pad[58];
};
template <int kV>
__global__ __launch_bounds__(256) void k_prop(Big b) {
  if (*b.done == kMagic) return;
  if (kV == 1) {   // scratch: a dynamically indexed private array
    volatile uint32_t a[36];
    for (int i = 0; i < 36; ++i) a[i] = threadIdx.x + i + (uint32_t)b.pad[i];
    b.sink[0] = a[(threadIdx.x + b.pad[40]) % 36];
  } else if (kV == 2) {   // a large body
    uint32_t x = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 6000; ++i) x = (x * 2654435761u) ^ (x >> 13) ^ (uint32_t)i;
    b.sink[0] = x;
  } else {
    b.sink[0] = (uint32_t)b.pad[threadIdx.x % 58];
  }
}
template <int kV>
double chain_prop(int grid, int n, int reps, const uint64_t* done, uint32_t* sink, uint4* big, uint64_t n16);

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(1024) void k_stream_store(uint4* out, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 t = {(uint32_t)i, 1u, 2u, 3u};
    __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(out + i));
  }
}

template <int LDSW>
double chain(int grid, int block, int n, int reps, const uint64_t* done, uint32_t* sink, uint4* big, uint64_t n16,
             bool heavy) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_noop<LDSW>, dim3(grid), dim3(block), 0, 0, done, sink);
  CK(hipDeviceSynchronize());
  double tot = 0;
  for (int r = 0; r < reps; ++r) {
    if (heavy) hipLaunchKernelGGL(k_stream_store, dim3(512), dim3(1024), 0, 0, big, n16);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_noop<LDSW>, dim3(grid), dim3(block), 0, 0, done, sink);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return tot / reps / n * 1000.0;   // us per launch
}

template <int kV>
double chain_prop(int grid, int n, int reps, const uint64_t* done, uint32_t* sink, uint4* big, uint64_t n16) {
  Big bb{};
  bb.done = done;
  bb.sink = sink;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_prop<kV>, dim3(grid), dim3(256), 0, 0, bb);
  CK(hipDeviceSynchronize());
  double tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipLaunchKernelGGL(k_stream_store, dim3(512), dim3(1024), 0, 0, big, n16);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_prop<kV>, dim3(grid), dim3(256), 0, 0, bb);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  return tot / reps / n * 1000.0;
}

int main() {
  uint64_t* done;
  uint32_t* sink;
  uint4* big;
  const uint64_t n16 = (256ull << 20) / 16;
  CK(hipMalloc(&done, 8));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&big, n16 * 16));
  CK(hipMemcpy(done, &kMagic, 8, hipMemcpyHostToDevice));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("CUs %d\n", ncu);
  struct Cfg {
    int grid, block, ldsw;
  };
  const Cfg cfgs[] = {{1, 64, 0},          {8, 64, 0},          {64, 256, 0},          {256, 256, 0},
                      {256, 1024, 0},      {256, 1024, 33792},  {512, 1024, 16384},    {1024, 256, 0},
                      {1024, 256, 7168},   {3277, 256, 0},      {6554, 256, 0}};
  for (int g : {256, 1024}) {
    std::printf("kernarg 480 B        grid %4d chain 7: %6.2f us/launch\n", g, chain_prop<0>(g, 7, 200, done, sink, big, n16));
    std::printf("kernarg 480 + scratch grid %4d chain 7: %6.2f us/launch\n", g, chain_prop<1>(g, 7, 200, done, sink, big, n16));
    std::printf("kernarg 480 + big body grid %4d chain 7: %6.2f us/launch\n", g, chain_prop<2>(g, 7, 200, done, sink, big, n16));
  }
  for (const Cfg& c : cfgs) {
    for (int heavy = 0; heavy < 2; ++heavy) {
      double us = 0;
      for (int n : {1, 7}) {
        switch (c.ldsw) {
          case 0: us = chain<0>(c.grid, c.block, n, 200, done, sink, big, n16, heavy); break;
          case 33792: us = chain<33792>(c.grid, c.block, n, 200, done, sink, big, n16, heavy); break;
          case 16384: us = chain<16384>(c.grid, c.block, n, 200, done, sink, big, n16, heavy); break;
          case 7168: us = chain<7168>(c.grid, c.block, n, 200, done, sink, big, n16, heavy); break;
        }
        std::printf("grid %5d block %4d lds %6d B heavy %d chain %d: %6.2f us/launch\n", c.grid, c.block, c.ldsw * 4,
                    heavy, n, us);
      }
    }
  }
  return 0;
}
