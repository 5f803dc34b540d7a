// mb_valu.hip — issue cost of the integer VALU instructions the sweep tier is made of (tools only, not the
// product). 16 waves per CU (4 per SIMD), each running 8 independent chains of one instruction kind; the
// time per instruction per SIMD is (kernel cycles) / (instructions per SIMD). Kinds: v_xor_b32, v_add_u32,
// v_perm_b32, v_alignbyte_b32, v_bitop3_b32 (xor of three), v_lshl_or_b32, v_bfe_u32, v_mul_lo_u32,
// v_mov_b32_dpp (row_shr:1), v_cndmask.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_valu tools/microbench/mb_valu.hip
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

constexpr int kIters = 4096;

template <int K>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b) {
  if constexpr (K == 0) return a ^ b;
  else if constexpr (K == 1) return a + b;
  else if constexpr (K == 2) return __builtin_amdgcn_perm(a, b, 0x05040100u);
  else if constexpr (K == 3) return __builtin_amdgcn_alignbyte(a, b, 1);
  else if constexpr (K == 4) return __builtin_amdgcn_bitop3_b32(a, b, a >> 3, 0x96);
  else if constexpr (K == 5) return (a << 3) | b;
  else if constexpr (K == 6) return __builtin_amdgcn_ubfe(a, b & 31u, 8);
  else if constexpr (K == 7) return a * b;
  else if constexpr (K == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x111, 0xF, 0xF, false) ^ b;
  else if constexpr (K == 9) return (a & 1u) ? b : a;
  else if constexpr (K == 10) {   // byte 1 of a <- byte 0 of b, the rest of a kept (SDWA, VOP1)
    asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(a) : "v"(b));
    return a;
  } else if constexpr (K == 11) {   // a ^ (b >> 16) (SDWA, VOP2)
    uint32_t d;
    asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "=v"(d) : "v"(a), "v"(b));
    return d;
  } else if constexpr (K == 12) {   // (byte 1 of b) << 2, xor a
    uint32_t d;
    asm volatile("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(d) : "v"(b));
    return a ^ d;
  } else return a ^ b ^ 0x5A5A5A5Au;
}

template <int K>
__global__ __launch_bounds__(1024) void k_valu(uint32_t* sink, uint32_t seed) {
  uint32_t c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = threadIdx.x * 0x9E3779B9u + j + seed;
  const uint32_t b = seed ^ threadIdx.x;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = op<K>(c[j], c[(j + 3) & 7] ^ b);
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= c[j];
  if (x == 0x12345678u) sink[threadIdx.x] = x;
}

template <int K>
double cycles_per_inst(uint32_t* sink, int ncu, double ghz) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_valu<K>, dim3(ncu), dim3(1024), 0, 0, sink, 1u);
  CK(hipEventRecord(a, 0));
  const int it = 10;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(k_valu<K>, dim3(ncu), dim3(1024), 0, 0, sink, (uint32_t)i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double cyc = ms / it * 1e-3 * ghz * 1e9;
  const double inst_per_simd = 4.0 * kIters * 8;   // 4 waves per SIMD, 8 chains
  return cyc / inst_per_simd;
}

int main() {
  uint32_t* sink;
  CK(hipMalloc(&sink, 1 << 16));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const double ghz = prop.clockRate / 1e6;
  std::printf("CUs %d, clock %.2f GHz (cycles per wave64 instruction per SIMD, 4 waves per SIMD)\n", ncu, ghz);
  std::printf("v_xor_b32       %.2f\n", cycles_per_inst<0>(sink, ncu, ghz));
  std::printf("v_add_u32       %.2f\n", cycles_per_inst<1>(sink, ncu, ghz));
  std::printf("v_perm_b32      %.2f\n", cycles_per_inst<2>(sink, ncu, ghz));
  std::printf("v_alignbyte_b32 %.2f\n", cycles_per_inst<3>(sink, ncu, ghz));
  std::printf("v_bitop3 (+lshr)%.2f\n", cycles_per_inst<4>(sink, ncu, ghz));
  std::printf("v_lshl_or_b32   %.2f\n", cycles_per_inst<5>(sink, ncu, ghz));
  std::printf("v_bfe_u32       %.2f\n", cycles_per_inst<6>(sink, ncu, ghz));
  std::printf("v_mul_lo_u32    %.2f\n", cycles_per_inst<7>(sink, ncu, ghz));
  std::printf("dpp mov + xor   %.2f\n", cycles_per_inst<8>(sink, ncu, ghz));
  std::printf("v_cndmask (+and)%.2f\n", cycles_per_inst<9>(sink, ncu, ghz));
  std::printf("v_mov_b32_sdwa preserve (+xor) %.2f\n", cycles_per_inst<10>(sink, ncu, ghz));
  std::printf("v_xor_b32_sdwa WORD_1 (+xor)   %.2f\n", cycles_per_inst<11>(sink, ncu, ghz));
  std::printf("v_lshlrev_b32_sdwa BYTE_1 (+2 xor) %.2f\n", cycles_per_inst<12>(sink, ncu, ghz));
  std::printf("xor3 of VGPR,VGPR,literal      %.2f\n", cycles_per_inst<13>(sink, ncu, ghz));
  return 0;
}
