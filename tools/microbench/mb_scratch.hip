// mb_scratch.hip — what a kernel's private (scratch) segment costs per launch (tools only, not the product).
// k_sweep_fin went from 82 to 34 us at 64 MiB when its 224 B/lane of scratch (a noinline helper taking the
// kernel arguments by reference) went away. Here: a kernel that does nearly nothing, with S bytes/lane of
// forced scratch (a dynamically indexed private array), at the grids the scan uses; back-to-back launches
// on one stream, average time per launch from events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_scratch tools/microbench/mb_scratch.hip
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

template <int W>
__global__ void k_priv(uint32_t* sink, uint32_t sel) {
  if (W == 0) {
    if (sel == 0xFFFFFFFFu) sink[threadIdx.x] = sel;
    return;
  }
  volatile uint32_t a[W > 0 ? W : 1];   // volatile: kept in scratch at every size
#pragma unroll
  for (int i = 0; i < W; ++i) a[i] = threadIdx.x * (i + 1);
  const uint32_t v = a[(threadIdx.x ^ sel) % W];
  if (v == 0xFFFFFFFFu) sink[threadIdx.x] = v;
}

template <int W>
double per_launch_us(uint32_t* sink, int grid, int block) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_priv<W>, dim3(grid), dim3(block), 0, 0, sink, 7u);
  CK(hipEventRecord(a, 0));
  const int it = 200;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(k_priv<W>, dim3(grid), dim3(block), 0, 0, sink, (uint32_t)i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms * 1e3 / it;
}

int main() {
  uint32_t* sink;
  CK(hipMalloc(&sink, 1 << 16));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const int grids[][2] = {{ncu, 1024}, {4 * ncu, 256}, {8 * ncu, 256}, {16 * ncu, 256}, {2 * ncu, 1024}};
  for (const auto& g : grids) {
    std::printf("grid %5d x %4d: scratch 0 B %.2f us, 4 B %.2f, 16 B %.2f us, 32 B %.2f us, 64 B %.2f us, 144 B %.2f us, "
                "224 B %.2f us\n", g[0], g[1], per_launch_us<0>(sink, g[0], g[1]), per_launch_us<1>(sink, g[0], g[1]),
                per_launch_us<4>(sink, g[0], g[1]), per_launch_us<8>(sink, g[0], g[1]),
                per_launch_us<16>(sink, g[0], g[1]), per_launch_us<36>(sink, g[0], g[1]),
                per_launch_us<56>(sink, g[0], g[1]));
  }
  return 0;
}
