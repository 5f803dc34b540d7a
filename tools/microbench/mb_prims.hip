// Primitive micro-benchmarks for the log-scan design on gfx950 (MI355X).
// Measures, on one 1 GiB device buffer:
//   (1) coalesced dwordx4 read-reduce      -> practical HBM-read ceiling
//   (2) per-lane streaming reads           -> each lane reads its own S-byte range
//   (3) per-lane streaming + CRC32 slicing-by-4 with LDS tables replicated R times
//   (4) workgroup-staged (coalesced -> LDS) + per-lane CRC over LDS ranges
// Build: hipcc --offload-arch=gfx950 -O3 mb_prims.hip -o mb_prims
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

static uint32_t T[8][256];
static void make_tables() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    T[0][i] = c;
  }
  for (int j = 1; j < 8; ++j)
    for (int i = 0; i < 256; ++i) T[j][i] = (T[j - 1][i] >> 8) ^ T[0][T[j - 1][i] & 0xff];
}
static uint32_t crc_ref(const uint8_t* p, size_t n, uint32_t c) {
  for (size_t i = 0; i < n; ++i) c = T[0][(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c;
}

// ---- (1) coalesced read-reduce
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, size_t n16, unsigned* out) {
  unsigned acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// ---- (2) per-lane streaming: lane g reads [g*S, (g+1)*S) 16B at a time, UNROLL pieces per step
template <int S, int UNROLL>
__global__ __launch_bounds__(256) void k_lane_stream(const uint8_t* __restrict__ p, size_t nranges, unsigned* out) {
  size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nranges) return;
  const uint4* q = reinterpret_cast<const uint4*>(p + g * S);
  unsigned acc = 0;
  for (int i = 0; i < S / 16; i += UNROLL) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = q[i + u];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// ---- (3) per-lane streaming + CRC slicing-by-4, LDS tables replicated R times
template <int R>
__device__ __forceinline__ uint32_t s4(const uint32_t* __restrict__ lt, uint32_t c, uint32_t lanec) {
  // lt layout: dword index ((j*256 + i) * R + copy)
  uint32_t a = lt[((3 * 256 + (c & 0xff)) * R) + lanec];
  uint32_t b = lt[((2 * 256 + ((c >> 8) & 0xff)) * R) + lanec];
  uint32_t d = lt[((1 * 256 + ((c >> 16) & 0xff)) * R) + lanec];
  uint32_t e = lt[((0 * 256 + (c >> 24)) * R) + lanec];
  return __builtin_amdgcn_bitop3_b32(a, b, d, 0x96) ^ e;
}

template <int S, int R>
__global__ __launch_bounds__(256) void k_lane_crc(const uint8_t* __restrict__ p, size_t nranges,
                                                  const uint32_t* __restrict__ gtab, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lt[];
  for (int i = threadIdx.x; i < 4 * 256 * R; i += blockDim.x) {
    int copy = i % R, ji = i / R;
    lt[i] = gtab[ji];
    (void)copy;
  }
  __syncthreads();
  size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nranges) return;
  uint32_t lanec = threadIdx.x % R;
  const uint4* q = reinterpret_cast<const uint4*>(p + g * S);
  uint32_t c = 0xFFFFFFFFu;
  for (int i = 0; i < S / 16; i += 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = q[i + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c = s4<R>(lt, c ^ v[u].x, lanec);
      c = s4<R>(lt, c ^ v[u].y, lanec);
      c = s4<R>(lt, c ^ v[u].z, lanec);
      c = s4<R>(lt, c ^ v[u].w, lanec);
    }
  }
  out[g] = c;
}

// ---- (4) WG-staged: block stages W=256*S bytes coalesced into LDS (padded lane stride S+16),
// then each lane CRCs its S bytes from LDS. Tables replicated R times.
template <int S, int R>
__global__ __launch_bounds__(256) void k_staged_crc(const uint8_t* __restrict__ p, size_t nblocks,
                                                    const uint32_t* __restrict__ gtab, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lt[];
  uint8_t* stage = reinterpret_cast<uint8_t*>(lt + 4 * 256 * R);
  constexpr int LS = S + 16;  // padded lane stride in bytes
  for (int i = threadIdx.x; i < 4 * 256 * R; i += blockDim.x) lt[i] = gtab[i / R];
  uint32_t lanec = threadIdx.x % R;
  for (size_t blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(p + blk * (size_t)(256 * S));
    __syncthreads();
    // coalesced: piece k (16 B) of the block -> lane (k*16)/S, offset (k*16)%S
#pragma unroll 4
    for (int k = threadIdx.x; k < 256 * S / 16; k += 256) {
      uint4 v = src[k];
      int byte = k * 16;
      *reinterpret_cast<uint4*>(stage + (byte / S) * LS + (byte % S)) = v;
    }
    __syncthreads();
    const uint4* mine = reinterpret_cast<const uint4*>(stage + threadIdx.x * LS);
    uint32_t c = 0xFFFFFFFFu;
#pragma unroll 2
    for (int i = 0; i < S / 16; ++i) {
      uint4 v = mine[i];
      c = s4<R>(lt, c ^ v.x, lanec);
      c = s4<R>(lt, c ^ v.y, lanec);
      c = s4<R>(lt, c ^ v.z, lanec);
      c = s4<R>(lt, c ^ v.w, lanec);
    }
    out[blk * 256 + threadIdx.x] = c;
  }
}


// ---- (5) per-wave LDS-DMA pipeline: each wave streams regions of 64*S bytes into its own NB-deep
// ring (global_load_lds_dwordx4, lane-linear), then each lane CRCs its S-byte slice from LDS.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory"); }

template <int S, int NB, int WPB, int R>
__global__ __launch_bounds__(64 * WPB) void k_wave_pipe(const uint8_t* __restrict__ p, size_t nregions,
                                                       const uint32_t* __restrict__ gtab, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* lt = reinterpret_cast<uint32_t*>(smem);
  constexpr int REG = 64 * S;
  constexpr int G = S / 16;
  constexpr int TAB = 4 * 256 * R * 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < 4 * 256 * R; i += blockDim.x) lt[i] = gtab[i / R];
  __syncthreads();
  const uint32_t lanec = lane % R;
  const uint32_t wbase = (uint32_t)(uintptr_t)(smem + TAB + wave * NB * REG);  // LDS byte address
  const size_t gw = (size_t)blockIdx.x * WPB + wave, nw = (size_t)gridDim.x * WPB;
  const size_t count = gw < nregions ? (nregions - gw + nw - 1) / nw : 0;
  auto issue = [&](size_t i) {
    const uint8_t* src = p + (gw + i * nw) * (size_t)REG + lane * 16;
    uint32_t dst = wbase + (uint32_t)((i % NB) * REG);
#pragma unroll
    for (int k = 0; k < G; ++k) glds16(src + k * 1024, dst + k * 1024);
  };
  for (int b = 0; b < NB - 1; ++b) if ((size_t)b < count) issue(b);
  uint32_t acc = 0;
  for (size_t i = 0; i < count; ++i) {
    if (i + NB - 2 < count) wait_vm<(NB - 2) * G>(); else wait_vm<0>();
    const uint4* mine = reinterpret_cast<const uint4*>(smem + TAB + wave * NB * REG + (i % NB) * REG + lane * S);
    uint32_t c = 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < S / 16; ++q) {
      uint4 v = mine[q];
      c = s4<R>(lt, c ^ v.x, lanec);
      c = s4<R>(lt, c ^ v.y, lanec);
      c = s4<R>(lt, c ^ v.z, lanec);
      c = s4<R>(lt, c ^ v.w, lanec);
    }
    acc ^= c;
    if (i == 0 && gw == 0 && lane == 0) out[1] = c;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + NB - 1 < count) issue(i + NB - 1);
  }
  if (acc == 0x12345678u) out[0] = acc;
}


// ---- (6) wave pipeline with slicing-by-SL (4/8/16) and optional no-CRC (SL=0) ceiling.
template <int R, int NT>
__device__ __forceinline__ uint32_t lk(const uint32_t* __restrict__ lt, int j, uint32_t byte, uint32_t lanec) {
  return lt[((j * 256 + byte) * R) + lanec];
}
template <int SL, int R>
__device__ __forceinline__ uint32_t crc_block16(const uint32_t* __restrict__ lt, uint32_t c, uint4 v, uint32_t lanec) {
  if constexpr (SL == 0) {
    return c ^ v.x ^ v.y ^ v.z ^ v.w;
  } else if constexpr (SL == 4) {
    c = s4<R>(lt, c ^ v.x, lanec); c = s4<R>(lt, c ^ v.y, lanec);
    c = s4<R>(lt, c ^ v.z, lanec); c = s4<R>(lt, c ^ v.w, lanec);
    return c;
  } else if constexpr (SL == 8) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t a = c ^ w[2 * h], b = w[2 * h + 1];
      c = lk<R, 8>(lt, 7, a & 0xff, lanec) ^ lk<R, 8>(lt, 6, (a >> 8) & 0xff, lanec) ^
          lk<R, 8>(lt, 5, (a >> 16) & 0xff, lanec) ^ lk<R, 8>(lt, 4, a >> 24, lanec) ^
          lk<R, 8>(lt, 3, b & 0xff, lanec) ^ lk<R, 8>(lt, 2, (b >> 8) & 0xff, lanec) ^
          lk<R, 8>(lt, 1, (b >> 16) & 0xff, lanec) ^ lk<R, 8>(lt, 0, b >> 24, lanec);
    }
    return c;
  } else {
    uint32_t a = c ^ v.x;
    return lk<R, 16>(lt, 15, a & 0xff, lanec) ^ lk<R, 16>(lt, 14, (a >> 8) & 0xff, lanec) ^
           lk<R, 16>(lt, 13, (a >> 16) & 0xff, lanec) ^ lk<R, 16>(lt, 12, a >> 24, lanec) ^
           lk<R, 16>(lt, 11, v.y & 0xff, lanec) ^ lk<R, 16>(lt, 10, (v.y >> 8) & 0xff, lanec) ^
           lk<R, 16>(lt, 9, (v.y >> 16) & 0xff, lanec) ^ lk<R, 16>(lt, 8, v.y >> 24, lanec) ^
           lk<R, 16>(lt, 7, v.z & 0xff, lanec) ^ lk<R, 16>(lt, 6, (v.z >> 8) & 0xff, lanec) ^
           lk<R, 16>(lt, 5, (v.z >> 16) & 0xff, lanec) ^ lk<R, 16>(lt, 4, v.z >> 24, lanec) ^
           lk<R, 16>(lt, 3, v.w & 0xff, lanec) ^ lk<R, 16>(lt, 2, (v.w >> 8) & 0xff, lanec) ^
           lk<R, 16>(lt, 1, (v.w >> 16) & 0xff, lanec) ^ lk<R, 16>(lt, 0, v.w >> 24, lanec);
  }
}
template <int S, int NB, int WPB, int R, int SL>
__global__ __launch_bounds__(64 * WPB) void k_wave_sl(const uint8_t* __restrict__ p, size_t nregions,
                                                    const uint32_t* __restrict__ gtab, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* lt = reinterpret_cast<uint32_t*>(smem);
  constexpr int NT = SL == 0 ? 1 : (SL < 4 ? 4 : SL);
  constexpr int REG = 64 * S;
  constexpr int G = S / 16;
  constexpr int TAB = NT * 256 * R * 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < NT * 256 * R; i += blockDim.x) lt[i] = gtab[i / R];
  __syncthreads();
  const uint32_t lanec = lane % R;
  const uint32_t wbase = (uint32_t)(uintptr_t)(smem + TAB + wave * NB * REG);
  const size_t gw = (size_t)blockIdx.x * WPB + wave, nw = (size_t)gridDim.x * WPB;
  const size_t count = gw < nregions ? (nregions - gw + nw - 1) / nw : 0;
  auto issue = [&](size_t i) {
    const uint8_t* src = p + (gw + i * nw) * (size_t)REG + lane * 16;
    uint32_t dst = wbase + (uint32_t)((i % NB) * REG);
#pragma unroll
    for (int k = 0; k < G; ++k) glds16(src + k * 1024, dst + k * 1024);
  };
  for (int b = 0; b < NB - 1; ++b) if ((size_t)b < count) issue(b);
  uint32_t acc = 0;
  for (size_t i = 0; i < count; ++i) {
    if (i + NB - 2 < count) wait_vm<(NB - 2) * G>(); else wait_vm<0>();
    const uint4* mine = reinterpret_cast<const uint4*>(smem + TAB + wave * NB * REG + (i % NB) * REG + lane * S);
    uint32_t c = 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < S / 16; ++q) c = crc_block16<SL, R>(lt, c, mine[q], lanec);
    acc ^= c;
    if (i == 0 && gw == 0 && lane == 0) out[1] = c;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + NB - 1 < count) issue(i + NB - 1);
  }
  if (acc == 0x12345678u) out[0] = acc;
}


// ---- (7) slicing-by-1 with 32-way replicated (bank-private) table + ILP chains per lane.
// Table layout: dword (i*32 + copy), copy = lane&31 -> every lane always hits its own bank.
// ILP=2: slice split in halves, combined with a shift-by-(S/2) table set Z (4x256 dwords, unreplicated).
__device__ __forceinline__ uint32_t step1(const uint32_t* __restrict__ lt, uint32_t c, uint32_t lb) {
  uint32_t a = ((c & 0xffu) << 7) | lb;
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(lt) + a) ^ (c >> 8);
}
template <int S, int NB, int WPB, int ILP>
__global__ __launch_bounds__(64 * WPB) void k_wave_b1(const uint8_t* __restrict__ p, size_t nregions,
                                                    const uint32_t* __restrict__ gtab, const uint32_t* __restrict__ gz,
                                                    uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* lt = reinterpret_cast<uint32_t*>(smem);
  uint32_t* zt = lt + 256 * 32;
  constexpr int REG = 64 * S;
  constexpr int G = S / 16;
  constexpr int TAB = 256 * 32 * 4 + 4 * 256 * 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < 256 * 32; i += blockDim.x) lt[i] = gtab[i >> 5];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) zt[i] = gz[i];
  __syncthreads();
  const uint32_t lb = (lane & 31) * 4;
  const uint32_t wbase = (uint32_t)(uintptr_t)(smem + TAB + wave * NB * REG);
  const size_t gw = (size_t)blockIdx.x * WPB + wave, nw = (size_t)gridDim.x * WPB;
  const size_t count = gw < nregions ? (nregions - gw + nw - 1) / nw : 0;
  auto issue = [&](size_t i) {
    const uint8_t* src = p + (gw + i * nw) * (size_t)REG + lane * 16;
    uint32_t dst = wbase + (uint32_t)((i % NB) * REG);
#pragma unroll
    for (int k = 0; k < G; ++k) glds16(src + k * 1024, dst + k * 1024);
  };
  for (int b = 0; b < NB - 1; ++b) if ((size_t)b < count) issue(b);
  uint32_t acc = 0;
  for (size_t i = 0; i < count; ++i) {
    if (i + NB - 2 < count) wait_vm<(NB - 2) * G>(); else wait_vm<0>();
    const uint32_t* mine = reinterpret_cast<const uint32_t*>(smem + TAB + wave * NB * REG + (i % NB) * REG + lane * S);
    uint32_t c;
    if constexpr (ILP == 1) {
      c = 0xFFFFFFFFu;
#pragma unroll
      for (int q = 0; q < S / 4; ++q) {
        c ^= mine[q];
        c = step1(lt, c, lb); c = step1(lt, c, lb); c = step1(lt, c, lb); c = step1(lt, c, lb);
      }
    } else {
      uint32_t ca = 0xFFFFFFFFu, cb = 0;
      constexpr int H = S / 8;  // dwords per half
#pragma unroll
      for (int q = 0; q < H; ++q) {
        ca ^= mine[q]; cb ^= mine[H + q];
        ca = step1(lt, ca, lb); cb = step1(lt, cb, lb);
        ca = step1(lt, ca, lb); cb = step1(lt, cb, lb);
        ca = step1(lt, ca, lb); cb = step1(lt, cb, lb);
        ca = step1(lt, ca, lb); cb = step1(lt, cb, lb);
      }
      c = zt[ca & 0xff] ^ zt[256 + ((ca >> 8) & 0xff)] ^ zt[512 + ((ca >> 16) & 0xff)] ^ zt[768 + (ca >> 24)] ^ cb;
    }
    acc ^= c;
    if (i == 0 && gw == 0 && lane == 0) out[1] = c;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + NB - 1 < count) issue(i + NB - 1);
  }
  if (acc == 0x12345678u) out[0] = acc;
}


// ---- (8) slicing-by-16 with 6-bit chunks looked up by ds_bpermute (tables live in VGPRs: lane v holds
// entry v of each of the 22 chunk tables). No LDS bank conflicts: bpermute uses the LDS crossbar only.
// Chunk k covers message bits [6k, 6k+6) of the 128-bit block (bit 0 = LSB of first byte); chunk 21 = 2 bits.
__device__ __forceinline__ uint32_t bperm(uint32_t addr, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)v);
}
__device__ __forceinline__ uint32_t chunk_addr(const uint32_t w[4], int k) {
  // returns a value whose bits [7:2] are message bits [6k, 6k+6)
  const int s = 6 * k;
  const int d = s >> 5, o = s & 31;
  if (o == 0) return w[d] << 2;
  if (o == 1) return w[d] << 1;
  if (o + 6 <= 32 || d == 3) return w[d] >> (o - 2);
  return __builtin_amdgcn_alignbit(w[d + 1], w[d], o - 2);
}
template <int S, int NB, int WPB, int ILP>
__global__ __launch_bounds__(64 * WPB) void k_wave_bp(const uint8_t* __restrict__ p, size_t nregions,
                                                    const uint32_t* __restrict__ gchunk, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int REG = 64 * S;
  constexpr int G = S / 16;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t tb[22];
#pragma unroll
  for (int k = 0; k < 22; ++k) tb[k] = gchunk[k * 64 + lane];
  const uint32_t wbase = (uint32_t)(uintptr_t)(smem + wave * NB * REG);
  const size_t gw = (size_t)blockIdx.x * WPB + wave, nw = (size_t)gridDim.x * WPB;
  const size_t count = gw < nregions ? (nregions - gw + nw - 1) / nw : 0;
  auto issue = [&](size_t i) {
    const uint8_t* src = p + (gw + i * nw) * (size_t)REG + lane * 16;
    uint32_t dst = wbase + (uint32_t)((i % NB) * REG);
#pragma unroll
    for (int k = 0; k < G; ++k) glds16(src + k * 1024, dst + k * 1024);
  };
  auto blk = [&](uint32_t c, uint4 v) -> uint32_t {
    uint32_t w[4] = {c ^ v.x, v.y, v.z, v.w};
    uint32_t r[22];
#pragma unroll
    for (int k = 0; k < 22; ++k) r[k] = bperm(chunk_addr(w, k), tb[k]);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 22; k += 2) x = __builtin_amdgcn_bitop3_b32(x, r[k], r[k + 1], 0x96);
    return x;
  };
  for (int b = 0; b < NB - 1; ++b) if ((size_t)b < count) issue(b);
  uint32_t acc = 0;
  for (size_t i = 0; i < count; ++i) {
    if (i + NB - 2 < count) wait_vm<(NB - 2) * G>(); else wait_vm<0>();
    const uint4* mine = reinterpret_cast<const uint4*>(smem + wave * NB * REG + (i % NB) * REG + lane * S);
    uint32_t c;
    if constexpr (ILP == 1) {
      c = 0xFFFFFFFFu;
#pragma unroll
      for (int q = 0; q < S / 16; ++q) c = blk(c, mine[q]);
    } else {
      // two independent halves; combine not modelled (timing only): xor
      uint32_t ca = 0xFFFFFFFFu, cb = 0;
      constexpr int H = S / 32;
#pragma unroll
      for (int q = 0; q < H; ++q) { ca = blk(ca, mine[q]); cb = blk(cb, mine[H + q]); }
      c = ca ^ cb;
    }
    acc ^= c;
    if (i == 0 && gw == 0 && lane == 0) out[1] = c;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + NB - 1 < count) issue(i + NB - 1);
  }
  if (acc == 0x12345678u) out[0] = acc;
}


// ---- (9) slicing-by-SB (4 or 8 bytes) with 11/11/10-bit chunks per dword (0.75 lookups per byte).
// LDS table (p,q) for dword position p in [0,SB/4), chunk q in {0,1,2}: 2048/2048/1024 entries.
template <int SB> struct Tab11 {
  static constexpr int PER_DW = 2048 + 2048 + 1024;   // dwords per dword-position
  static constexpr int DWORDS = PER_DW * (SB / 4);
};
__device__ __forceinline__ uint32_t lds_ld(const uint8_t* base, uint32_t byteoff) {
  return *reinterpret_cast<const uint32_t*>(base + byteoff);
}
template <int SB>
__device__ __forceinline__ uint32_t blk11(const uint8_t* __restrict__ lt, uint32_t c, const uint32_t* w) {
  uint32_t x = 0;
#pragma unroll
  for (int p = 0; p < SB / 4; ++p) {
    uint32_t d = (p == 0) ? (c ^ w[0]) : w[p];
    const uint8_t* tb = lt + p * Tab11<SB>::PER_DW * 4;
    uint32_t a = lds_ld(tb, (d << 2) & 0x1ffcu);
    uint32_t b = lds_ld(tb + 2048 * 4, (d >> 9) & 0x1ffcu);
    uint32_t e = lds_ld(tb + 4096 * 4, (d >> 20) & 0xffcu);
    x = __builtin_amdgcn_bitop3_b32(x, a, b, 0x96) ^ e;
  }
  return x;
}
template <int S, int NB, int WPB, int SB, int ILP>
__global__ __launch_bounds__(64 * WPB) void k_wave_11(const uint8_t* __restrict__ p, size_t nregions,
                                                    const uint32_t* __restrict__ gtab, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int REG = 64 * S;
  constexpr int G = S / 16;
  constexpr int TAB = Tab11<SB>::DWORDS * 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int i = threadIdx.x; i < Tab11<SB>::DWORDS; i += blockDim.x) reinterpret_cast<uint32_t*>(smem)[i] = gtab[i];
  __syncthreads();
  const uint32_t wbase = (uint32_t)(uintptr_t)(smem + TAB + wave * NB * REG);
  const size_t gw = (size_t)blockIdx.x * WPB + wave, nw = (size_t)gridDim.x * WPB;
  const size_t count = gw < nregions ? (nregions - gw + nw - 1) / nw : 0;
  auto issue = [&](size_t i) {
    const uint8_t* src = p + (gw + i * nw) * (size_t)REG + lane * 16;
    uint32_t dst = wbase + (uint32_t)((i % NB) * REG);
#pragma unroll
    for (int k = 0; k < G; ++k) glds16(src + k * 1024, dst + k * 1024);
  };
  for (int b = 0; b < NB - 1; ++b) if ((size_t)b < count) issue(b);
  uint32_t acc = 0;
  for (size_t i = 0; i < count; ++i) {
    if (i + NB - 2 < count) wait_vm<(NB - 2) * G>(); else wait_vm<0>();
    const uint32_t* mine = reinterpret_cast<const uint32_t*>(smem + TAB + wave * NB * REG + (i % NB) * REG + lane * S);
    uint32_t c;
    if constexpr (ILP == 1) {
      c = 0xFFFFFFFFu;
#pragma unroll
      for (int q = 0; q < S / SB; ++q) c = blk11<SB>(smem, c, mine + q * (SB / 4));
    } else {
      uint32_t ca = 0xFFFFFFFFu, cb = 0;
      constexpr int H = S / (2 * SB);
#pragma unroll
      for (int q = 0; q < H; ++q) { ca = blk11<SB>(smem, ca, mine + q * (SB / 4)); cb = blk11<SB>(smem, cb, mine + (H + q) * (SB / 4)); }
      c = ca ^ cb;
    }
    acc ^= c;
    if (i == 0 && gw == 0 && lane == 0) out[1] = c;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + NB - 1 < count) issue(i + NB - 1);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
static float timeit(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  make_tables();
  const size_t N = 1ull << 30;
  uint8_t* d; unsigned* dout; uint32_t* dtab;
  CK(hipMalloc(&d, N));
  CK(hipMalloc(&dout, (N / 64) * 4));
  CK(hipMalloc(&dtab, 4 * 256 * 4));
  std::vector<uint8_t> h(N);
  uint64_t s = 1;
  for (size_t i = 0; i < N; i += 8) { s = s * 6364136223846793005ull + 1442695040888963407ull; memcpy(&h[i], &s, 8); }
  CK(hipMemcpy(d, h.data(), N, hipMemcpyHostToDevice));
  std::vector<uint32_t> tabs(4 * 256);
  for (int j = 0; j < 4; ++j) for (int i = 0; i < 256; ++i) tabs[j * 256 + i] = T[j][i];
  CK(hipMemcpy(dtab, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
  int iters = 20;
  auto report = [&](const char* name, float ms) {
    printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms, N / (ms * 1e-3) / 1e9);
  };
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64]; snprintf(nm, sizeof nm, "read dwordx4 grid=%d", grid);
    report(nm, timeit([&] { k_read<<<grid, 256>>>((const uint4*)d, N / 16, dout); }, iters));
  }
#define LS_(S, U) { size_t nr = N / S; char nm[64]; snprintf(nm, sizeof nm, "lane-stream S=%d unroll=%d", S, U); \
    report(nm, timeit([&] { k_lane_stream<S, U><<<(nr + 255) / 256, 256>>>(d, nr, dout); }, iters)); }
#define LC_(S, R) { size_t nr = N / S; char nm[64]; snprintf(nm, sizeof nm, "lane-crc S=%d R=%d", S, R); \
    size_t lds = 4 * 256 * R * 4; CK(hipFuncSetAttribute((const void*)k_lane_crc<S, R>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_lane_crc<S, R><<<(nr + 255) / 256, 256, lds>>>(d, nr, dtab, dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (o[0] != want) printf("  MISMATCH %08x vs %08x\n", o[0], want); }
#define SC_(S, R, G) { size_t nb = N / (256 * S); char nm[64]; snprintf(nm, sizeof nm, "staged-crc S=%d R=%d grid=%d", S, R, G); \
    size_t lds = 4 * 256 * R * 4 + 256 * (S + 16); CK(hipFuncSetAttribute((const void*)k_staged_crc<S, R>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_staged_crc<S, R><<<G, 256, lds>>>(d, nb, dtab, dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (o[0] != want) printf("  MISMATCH %08x vs %08x\n", o[0], want); }

#define WP_(S, NB, WPB, R, G) { constexpr int REG = 64 * S; size_t nr = N / REG; char nm[80]; \
    snprintf(nm, sizeof nm, "wave-pipe S=%d NB=%d WPB=%d R=%d grid=%d", S, NB, WPB, R, G); \
    size_t lds = 4 * 256 * R * 4 + WPB * NB * REG; \
    CK(hipFuncSetAttribute((const void*)k_wave_pipe<S, NB, WPB, R>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_wave_pipe<S, NB, WPB, R><<<G, 64 * WPB, lds>>>(d, nr, dtab, dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (o[1] != want) printf("  MISMATCH %08x vs %08x\n", o[1], want); }

  { std::vector<uint32_t> t16(16 * 256); static uint32_t TT[16][256];
    for (int i = 0; i < 256; ++i) TT[0][i] = T[0][i];
    for (int j = 1; j < 16; ++j) for (int i = 0; i < 256; ++i) TT[j][i] = (TT[j-1][i] >> 8) ^ TT[0][TT[j-1][i] & 0xff];
    for (int j = 0; j < 16; ++j) for (int i = 0; i < 256; ++i) t16[j * 256 + i] = TT[j][i];
    CK(hipFree(dtab)); CK(hipMalloc(&dtab, 16 * 256 * 4)); CK(hipMemcpy(dtab, t16.data(), 16 * 256 * 4, hipMemcpyHostToDevice)); }
#define WS_(S, NB, WPB, R, SL, G) { constexpr int REG = 64 * S; size_t nr = N / REG; char nm[80]; \
    constexpr int NT = SL == 0 ? 1 : SL; \
    snprintf(nm, sizeof nm, "wave-sl S=%d NB=%d WPB=%d R=%d SL=%d grid=%d", S, NB, WPB, R, SL, G); \
    size_t lds = NT * 256 * R * 4 + WPB * NB * REG; \
    CK(hipFuncSetAttribute((const void*)k_wave_sl<S, NB, WPB, R, SL>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_wave_sl<S, NB, WPB, R, SL><<<G, 64 * WPB, lds>>>(d, nr, dtab, dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (SL && o[1] != want) printf("  MISMATCH %08x vs %08x\n", o[1], want); }
  WS_(80, 3, 4, 1, 0, 512) WS_(144, 3, 4, 1, 0, 256) WS_(80, 2, 4, 1, 0, 1024)
  
  WS_(80, 3, 4, 1, 16, 512) WS_(80, 3, 4, 2, 16, 512) 
  WS_(80, 3, 8, 1, 16, 256)

  uint32_t* dz; CK(hipMalloc(&dz, 4096));
#define WB_(S, NB, WPB, ILP, G) { constexpr int REG = 64 * S; size_t nr = N / REG; char nm[80]; \
    { std::vector<uint32_t> z(1024); for (int q = 0; q < 4; ++q) for (int b = 0; b < 256; ++b) { \
        uint32_t c = (uint32_t)b << (8 * q); for (int k = 0; k < S / 2; ++k) c = T[0][c & 0xff] ^ (c >> 8); z[q * 256 + b] = c; } \
      CK(hipMemcpy(dz, z.data(), 4096, hipMemcpyHostToDevice)); } \
    snprintf(nm, sizeof nm, "wave-b1 S=%d NB=%d WPB=%d ILP=%d grid=%d", S, NB, WPB, ILP, G); \
    size_t lds = 256 * 32 * 4 + 4096 + WPB * NB * REG; \
    CK(hipFuncSetAttribute((const void*)k_wave_b1<S, NB, WPB, ILP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_wave_b1<S, NB, WPB, ILP><<<G, 64 * WPB, lds>>>(d, nr, dtab, dz, dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (o[1] != want) printf("  MISMATCH %08x vs %08x\n", o[1], want); }

  uint32_t* dch; CK(hipMalloc(&dch, 22 * 64 * 4));
  { // chunk tables: lin(i) = register after processing a 16-byte message with only bit i set, from 0
    std::vector<uint32_t> lin(128);
    for (int i = 0; i < 128; ++i) { uint8_t m[16] = {0}; m[i >> 3] = (uint8_t)(1u << (i & 7)); lin[i] = crc_ref(m, 16, 0); }
    std::vector<uint32_t> ch(22 * 64, 0);
    for (int k = 0; k < 22; ++k) for (int v = 0; v < 64; ++v) { uint32_t x = 0;
      for (int b = 0; b < 6; ++b) if ((v >> b) & 1) { int bit = 6 * k + b; if (bit < 128) x ^= lin[bit]; } ch[k * 64 + v] = x; }
    CK(hipMemcpy(dch, ch.data(), ch.size() * 4, hipMemcpyHostToDevice)); }
#define WBP_(S, NB, WPB, ILP, G) { constexpr int REG = 64 * S; size_t nr = N / REG; char nm[80]; \
    snprintf(nm, sizeof nm, "wave-bperm S=%d NB=%d WPB=%d ILP=%d grid=%d", S, NB, WPB, ILP, G); \
    size_t lds = WPB * NB * REG; \
    CK(hipFuncSetAttribute((const void*)k_wave_bp<S, NB, WPB, ILP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_wave_bp<S, NB, WPB, ILP><<<G, 64 * WPB, lds>>>(d, nr, dch, dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (ILP == 1 && o[1] != want) printf("  MISMATCH %08x vs %08x\n", o[1], want); }

  uint32_t* d11[2];
  for (int sbi = 0; sbi < 2; ++sbi) { int SBv = sbi ? 8 : 4;
    std::vector<uint32_t> lin(SBv * 8);
    for (int i = 0; i < SBv * 8; ++i) { uint8_t m[8] = {0}; m[i >> 3] = (uint8_t)(1u << (i & 7)); lin[i] = crc_ref(m, SBv, 0); }
    int perdw = 5120; std::vector<uint32_t> t((SBv / 4) * perdw, 0);
    for (int pp = 0; pp < SBv / 4; ++pp) {
      int offs[3] = {0, 11, 22}, widths[3] = {11, 11, 10}, base[3] = {0, 2048, 4096};
      for (int q = 0; q < 3; ++q) for (int v = 0; v < (1 << widths[q]); ++v) { uint32_t x = 0;
        for (int b = 0; b < widths[q]; ++b) if ((v >> b) & 1) x ^= lin[32 * pp + offs[q] + b];
        t[pp * perdw + base[q] + v] = x; } }
    CK(hipMalloc(&d11[sbi], t.size() * 4)); CK(hipMemcpy(d11[sbi], t.data(), t.size() * 4, hipMemcpyHostToDevice)); }
#define W11_(S, NB, WPB, SB, ILP, G) { constexpr int REG = 64 * S; size_t nr = N / REG; char nm[80]; \
    snprintf(nm, sizeof nm, "wave-11b S=%d NB=%d WPB=%d SB=%d ILP=%d grid=%d", S, NB, WPB, SB, ILP, G); \
    size_t lds = Tab11<SB>::DWORDS * 4 + WPB * NB * REG; \
    CK(hipFuncSetAttribute((const void*)k_wave_11<S, NB, WPB, SB, ILP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(nm, timeit([&] { k_wave_11<S, NB, WPB, SB, ILP><<<G, 64 * WPB, lds>>>(d, nr, d11[SB == 8], dout); }, iters)); \
    std::vector<uint32_t> o(4); CK(hipMemcpy(o.data(), dout, 16, hipMemcpyDeviceToHost)); \
    uint32_t want = crc_ref(h.data(), S, 0xFFFFFFFFu); if (ILP == 1 && o[1] != want) printf("  MISMATCH %08x vs %08x\n", o[1], want); }
  W11_(80, 3, 4, 4, 1, 512) W11_(80, 3, 4, 4, 2, 512) W11_(48, 3, 4, 4, 1, 512) W11_(48, 4, 4, 4, 2, 512)
  W11_(80, 3, 8, 4, 2, 256) W11_(80, 3, 8, 8, 1, 256) W11_(80, 2, 8, 8, 1, 256) W11_(48, 3, 8, 8, 1, 256)
  W11_(112, 2, 4, 4, 2, 512) W11_(64, 3, 4, 4, 2, 512) W11_(32, 4, 4, 4, 1, 512) W11_(32, 4, 8, 4, 1, 256)
  CK(hipFree(d)); CK(hipFree(dout)); CK(hipFree(dtab));
  return 0;
}
