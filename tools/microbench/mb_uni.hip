// mb_uni.hip — design study for the run-prefix kernel (k_uniform) at BASELINE config 4 (tools only,
// not the product). A 4 GiB image of 332-B entries (CRC span [x + 4, x + 332), stored crc at x) is
// verified entry by entry by each variant; every variant writes the same 16-B tuple per entry
// {x lo, x hi, ok, raw register}, and its output is compared with the reference kernel's.
//
// Geometry as the product: G = 4 lanes per entry, P = 88-byte windows, t = 24 lead bytes masked on
// lane 0, 16 entries per wave batch, batches dealt grid-stride over the waves of the grid.
//
// Variants (LD x CR x waves per workgroup):
//   LD gather : each lane loads its own window as 6 dword-aligned 16-B rows (the product's pattern)
//   LD trans  : the wave's bytes as 6 coalesced non-temporal 1-KiB rows, written to LDS, windows read back
//   LD dma    : global_load_lds_dwordx4 (nt) of the same 6 rows straight into LDS, windows read back
//               (db: two buffers per wave, the next batch's DMA issued before this batch's CRC)
//   CR old    : 8-byte steps on shared 11/11/10-bit tables (the product's crc_step8; bank conflicts)
//   CR lp2    : 2-byte slicing on lane-private byte tables: row i = 256 B, dwords [0,32) T16[i] and
//               [32,64) T8[i] replicated, lane l reads its copy (bank = l mod 32: conflict-free);
//               the address (byte << 8 | 4 (l mod 32)) is one v_perm_b32, the xors v_bitop3
//   CR xor    : no CRC (xor of the words) — the memory path alone (results wrong by design)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mb_uni tools/microbench/mb_uni.hip
#include <hip/hip_runtime.h>

#include <cstdint>
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

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kSz = 332, kL = 328, kG = 4, kP = 88, kT = 24, kE = 16;
constexpr uint64_t kPad = 4096;   // readable zero bytes before and after the image

static uint32_t step_bits(uint32_t x, uint64_t n) {
  for (uint64_t k = 0; k < n; ++k) x = (x >> 1) ^ (kPoly & (0u - (x & 1u)));
  return x;
}

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0, (int)bytes, 0x00020000);
}
template <int POL>
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, POL);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) { return __builtin_amdgcn_alignbyte(hi, lo, sh); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}

enum { LD_GATHER = 0, LD_TRANS = 1, LD_DMA = 2 };
enum { CR_OLD = 0, CR_LP2 = 1, CR_XOR = 2 };

constexpr int kOldWords = 5120;
constexpr uint32_t kCombBytes = 3 * 4096;
constexpr uint32_t kStage = 6144;

template <int CR>
constexpr uint32_t crtab_bytes() { return CR == CR_OLD ? kOldWords * 4 : (CR == CR_LP2 ? 65536 : 0); }
template <int LD, int CR, int NW, int DB>
constexpr uint32_t lds_bytes() { return crtab_bytes<CR>() + kCombBytes + (LD == LD_GATHER ? 0 : NW * kStage * (DB > 1 ? DB : 1)); }

// 8-byte step on the shared 11/11/10-bit tables (ldb_engine.h crc_step8)
__device__ __forceinline__ uint32_t step_old(const uint32_t* tab, uint32_t reg, uint32_t w0, uint32_t w1) {
  const uint32_t x = reg ^ w0;
  const uint32_t y = tab[x & 0x7FFu] ^ tab[2048 + ((x >> 11) & 0x7FFu)] ^ tab[4096 + (x >> 22)] ^ w1;
  return tab[y & 0x7FFu] ^ tab[2048 + ((y >> 11) & 0x7FFu)] ^ tab[4096 + (y >> 22)];
}
// 4-byte step on the lane-private 2-byte slicing tables (LDS address 0)
__device__ __forceinline__ uint32_t lpread(const uint8_t* lds, uint32_t a) { return *reinterpret_cast<const uint32_t*>(lds + a); }
__device__ __forceinline__ uint32_t step_lp2(const uint8_t* lds, uint32_t lb, uint32_t reg, uint32_t w) {
  const uint32_t x = reg ^ w;
  const uint32_t y = xor3(x >> 16, lpread(lds, __builtin_amdgcn_perm(x, lb, 0x0C0C0400u)),
                          lpread(lds, __builtin_amdgcn_perm(x, lb, 0x0C0C0500u) + 128));
  return xor3(y >> 16, lpread(lds, __builtin_amdgcn_perm(y, lb, 0x0C0C0400u)),
              lpread(lds, __builtin_amdgcn_perm(y, lb, 0x0C0C0500u) + 128));
}

template <int LD, int CR, int NW, int DB, bool NOST = false>
__global__ __launch_bounds__(64 * NW) void k_var(const uint8_t* __restrict__ img, uint64_t nent, uint4* __restrict__ out,
                                                  const uint32_t* __restrict__ gold, const uint32_t* __restrict__ glp2,
                                                  const uint32_t* __restrict__ gcomb, uint32_t KL, uint32_t hdr0,
                                                  uint32_t hdr1) {
  constexpr uint32_t kTab = crtab_bytes<CR>(), kComb = kTab, kStg = kComb + kCombBytes;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[lds_bytes<LD, CR, NW, DB>()];
  {
    const uint4* src = reinterpret_cast<const uint4*>(CR == CR_OLD ? gold : glp2);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < kTab / 16; i += blockDim.x) dst[i] = src[i];
    const uint4* cs = reinterpret_cast<const uint4*>(gcomb);
    uint4* cd = reinterpret_cast<uint4*>(lds + kComb);
    for (uint32_t i = threadIdx.x; i < kCombBytes / 16; i += blockDim.x) cd[i] = cs[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t j = lane & 3u, grp = lane >> 2;
  const uint32_t lb = (uint32_t)(lane & 31) * 4u;
  const uint32_t* tab = reinterpret_cast<const uint32_t*>(lds);
  const uint32_t* comb = reinterpret_cast<const uint32_t*>(lds + kComb) + (j == 3 ? 0 : (2 - j) * 1024);
  const uint64_t nbatch = (nent + kE - 1) / kE;
  const uint64_t bstride = (uint64_t)gridDim.x * NW;
  uint8_t* stg0 = lds + kStg + (uint32_t)wave * kStage * (DB > 1 ? DB : 1);
  const uint32_t stg0_a = (uint32_t)(uintptr_t)stg0;
  int cur = 0;
  auto issue_dma = [&](uint64_t b, int slot) {
    const uint64_t x0 = b * kE * kSz;
    const int64_t base = ((int64_t)x0 - 20) & ~15ll;
#pragma unroll
    for (int r = 0; r < 6; ++r) glds16(img + base + 1024 * r + 16 * lane, stg0_a + slot * kStage + 1024 * r);
  };
  uint64_t b = (uint64_t)blockIdx.x * NW + wave;
  if (LD == LD_DMA && DB > 1)
    for (int k = 0; k < DB - 1; ++k) issue_dma(min(b + k * bstride, nbatch - 1), k);
  for (; b < nbatch; b += bstride) {
    const uint64_t e = b * kE + grp;
    const uint64_t x = e * kSz;
    const uint64_t x0 = b * kE * kSz;
    uint32_t d[24];
    uint32_t sh, crc_st, h0, h1;
    if (LD == LD_GATHER) {
      const int64_t base = (int64_t)x0 - 512;
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
      const uint32_t hx = (uint32_t)(x - base);
      uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
      if (j == 3) { q0 = ld16<0>(rs, hx & ~3u); q1 = ld16<0>(rs, (hx & ~3u) + 16); }
      const uint32_t ws = hx + 4 - kT + j * kP;
      sh = ws & 3u;
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        const uint4 q = ld16<0>(rs, (ws & ~3u) + 16 * r);
        d[4 * r] = q.x; d[4 * r + 1] = q.y; d[4 * r + 2] = q.z; d[4 * r + 3] = q.w;
      }
      __builtin_amdgcn_sched_barrier(0);   // every row load in flight before the first use
      const uint32_t hs = hx & 3u;
      crc_st = funnel(q0.y, q0.x, hs);
      h0 = funnel(q0.z, q0.y, hs);
      h1 = funnel(q0.w, q0.z, hs);
      (void)q1;
    } else {
      const int64_t base = ((int64_t)x0 - 20) & ~15ll;
      uint8_t* stg = stg0 + (DB > 1 ? cur * kStage : 0);
      if (LD == LD_TRANS) {
        const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
        uint4 q[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) q[r] = ld16<2>(rs, 1024 * r + 16 * lane);
#pragma unroll
        for (int r = 0; r < 6; ++r) *reinterpret_cast<uint4*>(stg + 1024 * r + 16 * lane) = q[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
        if (DB > 1) {   // ring of DB slots: batch b + (DB - 1) s goes to the slot the last batch freed
          issue_dma(min(b + (DB - 1) * bstride, nbatch - 1), (cur + DB - 1) % DB);
          if (DB == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          else if (DB == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
        } else {
          issue_dma(b, 0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      const uint32_t hx = (uint32_t)((int64_t)x - base);
      const uint32_t ws = hx + 4 - kT + j * kP;
      sh = ws & 3u;
      const uint32_t* w32 = reinterpret_cast<const uint32_t*>(stg + (ws & ~3u));
#pragma unroll
      for (int i = 0; i < 24; ++i) d[i] = w32[i];
      const uint32_t* h32 = reinterpret_cast<const uint32_t*>(stg + (hx & ~3u));
      const uint32_t hs = hx & 3u;
      uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
      if (j == 3) { a0 = h32[0]; a1 = h32[1]; a2 = h32[2]; a3 = h32[3]; }
      crc_st = funnel(a1, a0, hs);
      h0 = funnel(a2, a1, hs);
      h1 = funnel(a3, a2, hs);
      if (LD == LD_DMA && DB > 1) cur = (cur + 1) % DB;
    }
    // lane j's window: 11 steps of 8 bytes from register 0, lane 0's first 24 bytes masked (3 steps)
    uint32_t reg = 0;
#pragma unroll
    for (int k = 0; k < 11; ++k) {
      uint32_t w0 = funnel(d[2 * k + 1], d[2 * k], sh), w1 = funnel(d[2 * k + 2], d[2 * k + 1], sh);
      if (k < 3) {
        w0 = j == 0 ? 0u : w0;
        w1 = j == 0 ? 0u : w1;
      }
      if (CR == CR_OLD) reg = step_old(tab, reg, w0, w1);
      else if (CR == CR_LP2) reg = step_lp2(lds, lb, step_lp2(lds, lb, reg, w0), w1);
      else reg ^= w0 ^ w1;
    }
    // combine: lane j shifts by (3 - j) P bytes, the group xor-reduces (quad permutes)
    uint32_t z = reg;
    if (CR != CR_XOR) {
      const uint32_t s = comb[reg & 0xFFu] ^ comb[256 + ((reg >> 8) & 0xFFu)] ^ comb[512 + ((reg >> 16) & 0xFFu)] ^
                         comb[768 + (reg >> 24)];
      z = j == 3 ? reg : s;
    }
    z ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)z, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    z ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)z, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    if (j == 3 && e < nent) {
      const uint32_t ok = ((z ^ KL) == ~crc_st) && h0 == hdr0 && h1 == hdr1;
      if (!NOST) out[e] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), ok, z);
      else if (!ok) out[e].z = 0;   // failures only (rare): the run's tuples are written by a dense sweep
    }
  }
}

// ---------------------------------------------------------------- software-pipelined variants
// Each wave keeps NB batches of rows in flight in registers. gather: a lane's own window rows (the
// product's pattern), reloaded for batch b + NB s once the CRC consumed them. trans: the wave's bytes as
// 6 coalesced nt 1-KiB rows; on arrival they go to the wave's LDS stage and the registers are reloaded at
// once, then the lanes read their windows back (ds_read2_b32). Lane 0 of a group holds the stored crc and
// header words in its window (bytes 20..32) and checks the group's combined register.
template <int LD>
__device__ __forceinline__ void pipe_load(const uint8_t* img, uint64_t b, uint64_t nbatch, int lane, uint32_t j, uint32_t grp,
                                          uint4 (&q)[6]) {
  if (b >= nbatch) b = nbatch - 1;   // keep the instruction count uniform; results unused
  const uint64_t x0 = b * kE * kSz;
  if (LD == LD_GATHER) {
    const int64_t base = (int64_t)x0 - 512;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
    const uint32_t ws = (uint32_t)(512 + grp * kSz) + 4 - kT + j * kP;
#pragma unroll
    for (int r = 0; r < 6; ++r) q[r] = ld16<0>(rs, (ws & ~3u) + 16 * r);
  } else {
    const int64_t base = ((int64_t)x0 - 20) & ~15ll;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
#pragma unroll
    for (int r = 0; r < 6; ++r) q[r] = ld16<2>(rs, 1024 * r + 16 * lane);
  }
}

template <int LD, int CR, int NW, int NB>
constexpr uint32_t pipe_lds() { return crtab_bytes<CR>() + kCombBytes + (LD == LD_GATHER ? 0 : NW * kStage); }

template <int LD, int CR, int NW, int NB>
__global__ __launch_bounds__(64 * NW) void k_pipe(const uint8_t* __restrict__ img, uint64_t nent, uint4* __restrict__ out,
                                                   const uint32_t* __restrict__ gold, const uint32_t* __restrict__ glp2,
                                                   const uint32_t* __restrict__ gcomb, uint32_t KL, uint32_t hdr0,
                                                   uint32_t hdr1) {
  constexpr uint32_t kTab = crtab_bytes<CR>(), kComb = kTab, kStg = kComb + kCombBytes;
  __shared__ __attribute__((aligned(1024))) uint8_t lds[pipe_lds<LD, CR, NW, NB>()];
  {
    const uint4* src = reinterpret_cast<const uint4*>(CR == CR_OLD ? gold : glp2);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t i = threadIdx.x; i < kTab / 16; i += blockDim.x) dst[i] = src[i];
    const uint4* cs = reinterpret_cast<const uint4*>(gcomb);
    uint4* cd = reinterpret_cast<uint4*>(lds + kComb);
    for (uint32_t i = threadIdx.x; i < kCombBytes / 16; i += blockDim.x) cd[i] = cs[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t j = lane & 3u, grp = lane >> 2;
  const uint32_t lb = (uint32_t)(lane & 31) * 4u;
  const uint32_t* tab = reinterpret_cast<const uint32_t*>(lds);
  const uint32_t* comb = reinterpret_cast<const uint32_t*>(lds + kComb) + (j == 3 ? 0 : (2 - j) * 1024);
  const uint64_t nbatch = (nent + kE - 1) / kE;
  const uint64_t bs = (uint64_t)gridDim.x * NW;
  uint8_t* stg = lds + kStg + (uint32_t)wave * kStage;
  const uint64_t b0 = (uint64_t)blockIdx.x * NW + wave;
  uint4 q[NB][6];
#pragma unroll
  for (int k = 0; k < NB; ++k) pipe_load<LD>(img, b0 + k * bs, nbatch, lane, j, grp, q[k]);
  for (uint64_t it = 0;; it += NB) {
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const uint64_t b = b0 + (it + k) * bs;
      if (b >= nbatch) return;
      const uint64_t e = b * kE + grp;
      const uint64_t x = e * kSz;
      uint32_t d[24];
      uint32_t sh;
      if (LD == LD_GATHER) {
        const uint32_t ws = (uint32_t)(512 + grp * kSz) + 4 - kT + j * kP;
        sh = ws & 3u;
#pragma unroll
        for (int r = 0; r < 6; ++r) { d[4 * r] = q[k][r].x; d[4 * r + 1] = q[k][r].y; d[4 * r + 2] = q[k][r].z; d[4 * r + 3] = q[k][r].w; }
      } else {
#pragma unroll
        for (int r = 0; r < 6; ++r) *reinterpret_cast<uint4*>(stg + 1024 * r + 16 * lane) = q[k][r];
        pipe_load<LD>(img, b + NB * bs, nbatch, lane, j, grp, q[k]);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t x0 = b * kE * kSz;
        const int64_t base = ((int64_t)x0 - 20) & ~15ll;
        const uint32_t ws = (uint32_t)((int64_t)x - base) + 4 - kT + j * kP;
        sh = ws & 3u;
        const uint32_t* w32 = reinterpret_cast<const uint32_t*>(stg + (ws & ~3u));
#pragma unroll
        for (int i = 0; i < 24; ++i) d[i] = w32[i];
      }
      // stored crc and header words: window bytes [20, 32) of lane 0
      const uint32_t crc_st = funnel(d[6], d[5], sh), h0 = funnel(d[7], d[6], sh), h1 = funnel(d[8], d[7], sh);
      uint32_t reg = 0;
#pragma unroll
      for (int kk = 0; kk < 11; ++kk) {
        uint32_t w0 = funnel(d[2 * kk + 1], d[2 * kk], sh), w1 = funnel(d[2 * kk + 2], d[2 * kk + 1], sh);
        if (kk < 3) {
          w0 = j == 0 ? 0u : w0;
          w1 = j == 0 ? 0u : w1;
        }
        if (CR == CR_OLD) reg = step_old(tab, reg, w0, w1);
        else if (CR == CR_LP2) reg = step_lp2(lds, lb, step_lp2(lds, lb, reg, w0), w1);
        else reg ^= w0 ^ w1;
      }
      if (LD == LD_GATHER) {
        pipe_load<LD>(img, b + NB * bs, nbatch, lane, j, grp, q[k]);
        __builtin_amdgcn_sched_barrier(0);
      }
      uint32_t z = reg;
      if (CR != CR_XOR) {
        const uint32_t s = comb[reg & 0xFFu] ^ comb[256 + ((reg >> 8) & 0xFFu)] ^ comb[512 + ((reg >> 16) & 0xFFu)] ^
                           comb[768 + (reg >> 24)];
        z = j == 3 ? reg : s;
      }
      z ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)z, 0xB1, 0xF, 0xF, false);
      z ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)z, 0x4E, 0xF, 0xF, false);
      if (j == 0 && e < nent) {
        const uint32_t ok = ((z ^ KL) == ~crc_st) && h0 == hdr0 && h1 == hdr1;
        out[e] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), ok, z);
      }
    }
  }
}

// calibration: grid-stride streaming XOR, 8 nt 16-B loads in flight per lane (tools/microbench/mb_read.hip nt8),
// plus (ST) one 16-B store per 332 B read, as the tuple writes
template <bool ST>
__global__ __launch_bounds__(256) void k_nt8(const uint8_t* __restrict__ img8, uint64_t nent, uint4* __restrict__ out,
                                             const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint32_t) {
  const uint4* p = reinterpret_cast<const uint4*>(img8);
  const uint64_t n16 = nent * kSz / 16;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t acc = 0;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    uint4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const v4u32 v = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p + i + u * stride));
      x[u] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    if (ST && (i % 83) < 4) out[(i / 83 * 4 + i % 83) % nent] = make_uint4(acc, 0, 0, 0);
  }
  for (; i < n16; i += stride) {
    const uint4 x = p[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9E3779B9u) out[0].w = acc;
}

// memory-path experiments (XOR only, results wrong by design):
//   M 0: gather rows (product pattern), plain loads      M 1: gather rows, nt loads
//   M 2: the batch's 6 KiB as coalesced 1-KiB rows, nt  M 3: M 2 with plain loads
// ST: the 16-B tuple of each entry is stored (lane 4g of the wave, 256 B per batch)
template <int M, bool ST, int NW>
__global__ __launch_bounds__(64 * NW) void k_exp(const uint8_t* __restrict__ img, uint64_t nent, uint4* __restrict__ out,
                                                  const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint32_t) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t j = lane & 3u, grp = lane >> 2;
  const uint64_t nbatch = (nent + kE - 1) / kE;
  const uint64_t bs = (uint64_t)gridDim.x * NW;
  for (uint64_t b = (uint64_t)blockIdx.x * NW + wave; b < nbatch; b += bs) {
    const uint64_t x0 = b * kE * kSz;
    uint4 q[6];
    if (M <= 1) {
      const int64_t base = (int64_t)x0 - 512;
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
      const uint32_t ws = (uint32_t)(512 + grp * kSz) + 4 - kT + j * kP;
#pragma unroll
      for (int r = 0; r < 6; ++r) q[r] = M == 1 ? ld16<2>(rs, (ws & ~3u) + 16 * r) : ld16<0>(rs, (ws & ~3u) + 16 * r);
    } else {
      const int64_t base = ((int64_t)x0 - 20) & ~15ll;
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
#pragma unroll
      for (int r = 0; r < 6; ++r) q[r] = M == 2 ? ld16<2>(rs, 1024 * r + 16 * lane) : ld16<0>(rs, 1024 * r + 16 * lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    uint32_t z = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) z ^= q[r].x ^ q[r].y ^ q[r].z ^ q[r].w;
    const uint64_t e = b * kE + grp;
    if (ST) {
      if (j == 0 && e < nent) out[e] = make_uint4((uint32_t)e, 0, 0, z);
    } else if (z == 0x9E3779B9u) {
      out[e % nent].w = z;
    }
  }
}

// store experiments on the gather pattern (XOR only): how the 16-B tuples are written
//   S 1 plain global store   S 2 __builtin_nontemporal_store   S 3/4/5 buffer store, aux 1 / 2 / 3
//   S 6: each wave takes 4 consecutive batches (its batches grid-stride in groups of 4), stages the 64
//        tuples in LDS and writes them as one 1-KiB coalesced store
template <int S, int NW>
__global__ __launch_bounds__(64 * NW) void k_st(const uint8_t* __restrict__ img, uint64_t nent, uint4* __restrict__ out,
                                                 const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint32_t) {
  __shared__ __attribute__((aligned(16))) uint4 tl[NW][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t j = lane & 3u, grp = lane >> 2;
  const uint64_t nbatch = (nent + kE - 1) / kE;
  constexpr int kC = S == 6 ? 4 : 1;
  const uint64_t bs = (uint64_t)gridDim.x * NW * kC;
  for (uint64_t b4 = ((uint64_t)blockIdx.x * NW + wave) * kC; b4 < nbatch; b4 += bs) {
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const uint64_t b = b4 + c;
      if (b >= nbatch) break;
      const uint64_t x0 = b * kE * kSz;
      uint4 q[6];
      const int64_t base = (int64_t)x0 - 512;
      const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
      const uint32_t ws = (uint32_t)(512 + grp * kSz) + 4 - kT + j * kP;
#pragma unroll
      for (int r = 0; r < 6; ++r) q[r] = ld16<0>(rs, (ws & ~3u) + 16 * r);
      __builtin_amdgcn_sched_barrier(0);
      uint32_t z = 0;
#pragma unroll
      for (int r = 0; r < 6; ++r) z ^= q[r].x ^ q[r].y ^ q[r].z ^ q[r].w;
      const uint64_t e = b * kE + grp;
      const uint4 t = make_uint4((uint32_t)e, 0, 0, z);
      if (S == 6) {
        if (j == 0) tl[wave][c * 16 + grp] = t;
      } else if (j == 0 && e < nent) {
        if (S == 1) out[e] = t;
        else if (S == 2) __builtin_nontemporal_store(v4u32{t.x, t.y, t.z, t.w}, reinterpret_cast<v4u32*>(out + e));
        else {
          const __amdgpu_buffer_rsrc_t ro = rsrc_of(out + b * kE, 256);
          __builtin_amdgcn_raw_buffer_store_b128(v4u32{t.x, t.y, t.z, t.w}, ro, grp * 16, 0, S == 3 ? 1 : (S == 4 ? 2 : 3));
        }
      }
    }
    if (S == 6) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint64_t e = b4 * kE + lane;
      const uint4 t = tl[wave][lane];
      if (e < nent) out[e] = t;
    }
  }
}

// write experiments: W 0 the tuple array alone, written as a dense sweep (64 lanes x 16 B per
// instruction, grid-stride); W 1: the gather XOR pass storing its tuples into a 1 MiB ring (L2-resident);
// W 2: the gather XOR pass storing 4 B per entry (the ok word only) into out
template <int W, int NW>
__global__ __launch_bounds__(64 * NW) void k_wr(const uint8_t* __restrict__ img, uint64_t nent, uint4* __restrict__ out,
                                                 const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, uint32_t, uint32_t) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (W == 0) {
    const uint64_t stride = (uint64_t)gridDim.x * NW * 64;
    for (uint64_t e = ((uint64_t)blockIdx.x * NW + wave) * 64 + lane; e < nent; e += stride)
      out[e] = make_uint4((uint32_t)(e * kSz), (uint32_t)((e * kSz) >> 32), 1, 0);
    return;
  }
  const uint32_t j = lane & 3u, grp = lane >> 2;
  const uint64_t nbatch = (nent + kE - 1) / kE;
  const uint64_t bs = (uint64_t)gridDim.x * NW;
  for (uint64_t b = (uint64_t)blockIdx.x * NW + wave; b < nbatch; b += bs) {
    const uint64_t x0 = b * kE * kSz;
    uint4 q[6];
    const int64_t base = (int64_t)x0 - 512;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(img + base, 8192);
    const uint32_t ws = (uint32_t)(512 + grp * kSz) + 4 - kT + j * kP;
#pragma unroll
    for (int r = 0; r < 6; ++r) q[r] = ld16<0>(rs, (ws & ~3u) + 16 * r);
    __builtin_amdgcn_sched_barrier(0);
    uint32_t z = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) z ^= q[r].x ^ q[r].y ^ q[r].z ^ q[r].w;
    const uint64_t e = b * kE + grp;
    if (j == 0 && e < nent) {
      if (W == 1) out[e & 65535] = make_uint4((uint32_t)e, 0, 0, z);
      else reinterpret_cast<uint32_t*>(out)[e] = z;
    }
  }
}

// reference: one thread per entry, byte-at-a-time
__global__ void k_ref(const uint8_t* __restrict__ img, uint64_t nent, uint4* __restrict__ out, const uint32_t* __restrict__ t8,
                      uint32_t hdr0, uint32_t hdr1, int fill) {
  __shared__ uint32_t T[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) T[i] = t8[i];
  __syncthreads();
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nent) return;
  const uint8_t* p = img + e * kSz;
  uint32_t c = 0xFFFFFFFFu;
  for (uint32_t i = 4; i < kSz; ++i) c = T[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  c = ~c;
  if (fill) {
    uint8_t* q = const_cast<uint8_t*>(p);
    q[0] = (uint8_t)c; q[1] = (uint8_t)(c >> 8); q[2] = (uint8_t)(c >> 16); q[3] = (uint8_t)(c >> 24);
    return;
  }
  const uint32_t st = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
  const uint32_t h0 = p[4] | (p[5] << 8) | (p[6] << 16) | ((uint32_t)p[7] << 24);
  const uint32_t h1 = p[8] | (p[9] << 8) | (p[10] << 16) | ((uint32_t)p[11] << 24);
  out[e] = make_uint4((uint32_t)(e * kSz), (uint32_t)((e * kSz) >> 32), (st == c) && h0 == hdr0 && h1 == hdr1, 0);
}

__global__ void k_gen(uint8_t* img, uint64_t len, uint32_t hdr0, uint32_t hdr1) {
  const uint64_t n4 = len / 4;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
    z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 29;
    reinterpret_cast<uint32_t*>(img)[i] = (uint32_t)z;
  }
}
__global__ void k_hdr(uint8_t* img, uint64_t len, uint32_t hdr0, uint32_t hdr1) {   // bytes [4, 12) of every entry
  const uint64_t nent = len / kSz;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nent; e += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* p = img + e * kSz;
    for (int i = 0; i < 4; ++i) { p[4 + i] = (uint8_t)(hdr0 >> (8 * i)); p[8 + i] = (uint8_t)(hdr1 >> (8 * i)); }
  }
}

__global__ void k_cmp(const uint4* a, const uint4* b, uint64_t n, unsigned long long* diff, unsigned long long* nok) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 x = a[i], y = b[i];
    if (x.x != y.x || x.y != y.y || x.z != y.z) atomicAdd(diff, 1ull);
    if (x.z) atomicAdd(nok, 1ull);
  }
}

int main(int argc, char** argv) {
  const uint64_t len = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (4ull << 30)) / kSz * kSz;
  const uint64_t nent = len / kSz;
  const uint32_t hdr0 = 0x40801000u | 0x02, hdr1 = 0x00020004u;
  uint8_t* raw = nullptr;
  CK(hipMalloc(&raw, len + 2 * kPad));
  CK(hipMemset(raw, 0, len + 2 * kPad));
  uint8_t* img = raw + kPad;
  uint4 *ref = nullptr, *out = nullptr;
  CK(hipMalloc(&ref, nent * 16));
  CK(hipMalloc(&out, nent * 16));
  unsigned long long* cnt = nullptr;
  CK(hipMalloc(&cnt, 16));

  std::vector<uint32_t> t8(256), old(kOldWords), lp2(16384), comb(3 * 1024);
  for (uint32_t i = 0; i < 256; ++i) t8[i] = step_bits(i, 8);
  const int off[3] = {0, 11, 22}, wid[3] = {11, 11, 10}, bse[3] = {0, 2048, 4096};
  for (int q = 0; q < 3; ++q)
    for (uint32_t v = 0; v < (1u << wid[q]); ++v) old[bse[q] + v] = step_bits(v << off[q], 32);
  for (uint32_t i = 0; i < 256; ++i)
    for (int l = 0; l < 32; ++l) {
      lp2[i * 64 + l] = step_bits(i, 16);
      lp2[i * 64 + 32 + l] = step_bits(i, 8);
    }
  for (int d = 1; d <= 3; ++d)
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) comb[(d - 1) * 1024 + q * 256 + b] = step_bits(b << (8 * q), 8ull * d * kP);
  const uint32_t KL = step_bits(0xFFFFFFFFu, 8ull * kL);
  uint32_t *d_t8, *d_old, *d_lp2, *d_comb;
  CK(hipMalloc(&d_t8, 1024));
  CK(hipMalloc(&d_old, kOldWords * 4));
  CK(hipMalloc(&d_lp2, 65536));
  CK(hipMalloc(&d_comb, 3 * 4096));
  CK(hipMemcpy(d_t8, t8.data(), 1024, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_old, old.data(), kOldWords * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_lp2, lp2.data(), 65536, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_comb, comb.data(), 3 * 4096, hipMemcpyHostToDevice));

  hipLaunchKernelGGL(k_gen, dim3(8192), dim3(256), 0, 0, img, len, hdr0, hdr1);
  hipLaunchKernelGGL(k_hdr, dim3(8192), dim3(256), 0, 0, img, len, hdr0, hdr1);
  hipLaunchKernelGGL(k_ref, dim3((nent + 255) / 256), dim3(256), 0, 0, img, nent, ref, d_t8, hdr0, hdr1, 1);
  // corrupt 1000 entries (one byte each, spread), then the reference verdicts
  for (int i = 0; i < 1000; ++i) {
    const uint64_t e = (uint64_t)i * 7919ull * 131ull % nent;
    const uint64_t o = e * kSz + 4 + (i * 37) % kL;
    uint8_t v;
    CK(hipMemcpy(&v, img + o, 1, hipMemcpyDeviceToHost));
    v ^= 0x5A;
    CK(hipMemcpy(img + o, &v, 1, hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(k_ref, dim3((nent + 255) / 256), dim3(256), 0, 0, img, nent, ref, d_t8, hdr0, hdr1, 0);
  CK(hipDeviceSynchronize());
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* only = getenv("MB_ONLY");
  auto run = [&](const char* name, int wg_per_cu, auto kern, int nw) {
    if (only && !strstr(name, only)) return;
    const unsigned grid = ncu * wg_per_cu;
    auto launch = [&] {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * nw), 0, 0, img, nent, out, d_old, d_lp2, d_comb, KL, hdr0, hdr1);
    };
    if (strstr(name, "nost_")) CK(hipMemcpy(out, ref, nent * 16, hipMemcpyDeviceToDevice));
    else CK(hipMemset(out, 0, nent * 16));
    launch();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long h[2] = {0, 0};
    CK(hipMemset(cnt, 0, 16));
    hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, out, ref, nent, cnt, cnt + 1);
    CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
    CK(hipEventRecord(e0));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 20;
    std::printf("%-22s %7.4f ms  %7.1f GB/s  frac %.3f  diff %llu ok %llu/%llu\n", name, ms, len / (ms * 1e-3) / 1e9,
                len / (ms * 1e-3) / 8e12, h[0], h[1], (unsigned long long)nent);
    std::fflush(stdout);
  };
#define V(LD, CR, NW, DB, WG) run(#LD "_" #CR "_w" #NW "_db" #DB "_g" #WG, WG, k_var<LD, CR, NW, DB>, NW)
#define VP(LD, CR, NW, NB, WG) run("pipe_" #LD "_" #CR "_w" #NW "_nb" #NB "_g" #WG, WG, k_pipe<LD, CR, NW, NB>, NW)
#define VE(M, ST, NW, WG) run("exp_M" #M "_st" #ST "_w" #NW "_g" #WG, WG, k_exp<M, ST, NW>, NW)
#define VS(S, NW, WG) run("st_S" #S "_w" #NW "_g" #WG, WG, k_st<S, NW>, NW)
#define VW(W, NW, WG) run("wr_W" #W "_w" #NW "_g" #WG, WG, k_wr<W, NW>, NW)
#define VN(LD, CR, NW, DB, WG) run("nost_" #LD "_" #CR "_w" #NW "_db" #DB "_g" #WG, WG, k_var<LD, CR, NW, DB, true>, NW)
  run("calib_nt8_g16", 16, k_nt8<false>, 4);
  VE(0, 0, 16, 2);
  V(LD_GATHER, CR_OLD, 16, 0, 2);
  VN(LD_GATHER, CR_OLD, 16, 0, 2);
  VN(LD_GATHER, CR_LP2, 16, 0, 2);
  VN(LD_GATHER, CR_LP2, 16, 0, 1);
  VN(LD_DMA, CR_OLD, 10, 2, 1);
  VN(LD_DMA, CR_OLD, 8, 2, 1);
  VN(LD_DMA, CR_LP2, 7, 2, 1);
  VN(LD_TRANS, CR_OLD, 16, 0, 1);
  VN(LD_TRANS, CR_LP2, 12, 0, 1);
  VW(0, 16, 2);
  VE(0, 0, 16, 2);
  run("calib_nt8_g16", 16, k_nt8<false>, 4);
  return 0;
}
