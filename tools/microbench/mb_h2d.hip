// mb_h2d.hip — host-to-device ceilings for the e2e path (tools only).
//   memcpy_pinned    : one hipMemcpyAsync of 1 GiB from page-locked host memory (SDMA)
//   memcpy_chunks_Sn : 64 MiB chunks round-robin over n streams
//   memcpy_pageable  : one hipMemcpy from pageable memory
//   kcopy            : a kernel reading the page-locked buffer through its device mapping (PCIe reads
//                      issued by the CUs) and writing HBM
//   kread            : the same reads, XOR-reduced (no HBM write)
// Build: hipcc --offload-arch=gfx950 -O3 -o mb_h2d tools/microbench/mb_h2d.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ src, uint64_t n16, uint32_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t acc = 0;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

int main() {
  const uint64_t nbytes = 1ull << 30, n16 = nbytes / 16;
  uint8_t *h_pin = nullptr, *d = nullptr, *d_map = nullptr;
  uint32_t* sink = nullptr;
  CK(hipHostMalloc(&h_pin, nbytes, hipHostMallocMapped));
  std::memset(h_pin, 0x5A, nbytes);
  CK(hipHostGetDevicePointer((void**)&d_map, h_pin, 0));
  std::vector<uint8_t> h_page(nbytes, 0x5A);
  CK(hipMalloc(&d, nbytes));
  CK(hipMalloc(&sink, 1 << 20));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  hipStream_t st[8];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](const char* name, int reps, auto body) {
    body();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) body();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%-22s %8.2f ms  %6.1f GB/s\n", name, ms / reps, nbytes / (ms / reps * 1e-3) / 1e9);
  };
  timed("memcpy_pinned", 5, [&] { CK(hipMemcpyAsync(d, h_pin, nbytes, hipMemcpyHostToDevice, st[0])); CK(hipStreamSynchronize(st[0])); });
  for (int ns : {2, 4, 8}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "memcpy_chunks_S%d", ns);
    timed(nm, 5, [&] {
      const uint64_t ch = 64ull << 20;
      for (uint64_t o = 0, k = 0; o < nbytes; o += ch, ++k)
        CK(hipMemcpyAsync(d + o, h_pin + o, ch, hipMemcpyHostToDevice, st[k % ns]));
      for (int i = 0; i < ns; ++i) CK(hipStreamSynchronize(st[i]));
    });
  }
  timed("memcpy_pageable", 3, [&] { CK(hipMemcpy(d, h_page.data(), nbytes, hipMemcpyHostToDevice)); });
  for (int g : {1, 2, 4, 8}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "kcopy_%dblk_per_cu", g);
    timed(nm, 3, [&] { hipLaunchKernelGGL(k_copy, dim3(ncu * g), dim3(256), 0, st[0], (const uint4*)d_map, (uint4*)d, n16); CK(hipStreamSynchronize(st[0])); });
    std::snprintf(nm, sizeof nm, "kread_%dblk_per_cu", g);
    timed(nm, 3, [&] { hipLaunchKernelGGL(k_read, dim3(ncu * g), dim3(256), 0, st[0], (const uint4*)d_map, n16, sink); CK(hipStreamSynchronize(st[0])); });
  }
  CK(hipHostFree(h_pin));
  CK(hipFree(d));
  return 0;
}
