// mb_atomic.hip — what k_sweep's phase protocol costs (tools only, not the product): one workgroup per CU,
// thread 0 of each does N device-scope atomicAdds on ONE word (the tickets and done counters), with or without
// an agent-scope release fence before each, or on a word of its own; a plain kernel of the same grid beside it.
// Back-to-back launches, average time per launch from events.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_atomic tools/microbench/mb_atomic.hip
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

// kMode: 0 nothing, 1 N atomics on one word, 2 N (fence release + atomic) on one word, 3 N atomics on own words
template <int kMode>
__global__ __launch_bounds__(1024) void k_atom(uint32_t* w, int n, uint32_t* sink) {
  __shared__ uint32_t s;
  uint32_t acc = 0;
  for (int i = 0; i < n; ++i) {
    __syncthreads();
    if (threadIdx.x == 0) {
      if (kMode == 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (kMode == 1 || kMode == 2) s = atomicAdd(&w[i & 7], 1u);
      if (kMode == 3) s = atomicAdd(&w[64 + 64 * blockIdx.x + (i & 7)], 1u);
      if (kMode == 0) s = i;
    }
    __syncthreads();
    acc += s;
  }
  if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

template <int kMode>
double run(uint32_t* w, int grid, int n, uint32_t* sink) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_atom<kMode>, dim3(grid), dim3(1024), 0, 0, w, n, sink);
  CK(hipEventRecord(a, 0));
  const int it = 200;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(k_atom<kMode>, dim3(grid), dim3(1024), 0, 0, w, n, sink);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / it;
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *w, *sink;
  CK(hipMalloc(&w, 4 * (64 + 64 * 4096)));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(w, 0, 4 * (64 + 64 * 4096)));
  for (int n : {1, 3, 6, 12}) {
    std::printf("grid %d, %2d rounds: plain %6.2f us, one word %6.2f us, fence+one word %6.2f us, own words %6.2f us\n", ncu,
                n, run<0>(w, ncu, n, sink), run<1>(w, ncu, n, sink), run<2>(w, ncu, n, sink), run<3>(w, ncu, n, sink));
  }
  return 0;
}
