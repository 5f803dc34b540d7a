// ldb_devmem.h — device memory and CRC-table primitives shared by the scan kernels (ldb_scan.hip) and the
// sweep tier (ldb_sweep_kern.h): buffer descriptors and range-checked row loads / stores, tuple stores, the
// lane-private LP2 CRC block, the result word of a finished scan. Included by ldb_scan.hip inside its kernel
// namespace; tests/emu/sweep_emu.cpp includes it under its SIMT emulation of these intrinsics (test harness).
#pragma once

// the counted waits the kernels place by hand (the emulator, tests/emu/simt.h, runs them as no-ops)
#ifndef LDB_WAIT_LGKM0
#define LDB_WAIT_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define LDB_WAIT_VM0() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
// the same where a wave's lanes exchange data through memory (one lane's stores, another lane's loads: the
// sweep's hit list, its slab records). Wave-uniform points; the emulator synchronises the wave's lanes there
#define LDB_WAVE_XCHG_LDS() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")
#define LDB_WAVE_XCHG_VM() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#endif

// what a k_sweep / k_region workgroup's LDS holds (its phases copy their tables once per workgroup, not per item)
constexpr int kLdsNone = 0, kLdsSweep = 1, kLdsFin = 2, kLdsRegion = 3;

constexpr uint64_t kUniDone = 0xD0E5CA11D0E5CA11ull;

__device__ __forceinline__ void store_tuple(ldb_index_tuple* dst, uint64_t pos, uint32_t k, uint32_t v) {
  uint4 t;
  t.x = (uint32_t)pos;
  t.y = (uint32_t)(pos >> 32);
  t.z = k;
  t.w = v;
  *reinterpret_cast<uint4*>(dst) = t;
}
// the same as a streaming store (not kept in L2: the INDEX sweep's tuples are read by the host or the
// next kernel, and a release fence after the sweep would otherwise write them back from L2)
__device__ __forceinline__ void store_tuple_nt(ldb_index_tuple* dst, uint64_t pos, uint32_t k, uint32_t v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 t = {(uint32_t)pos, (uint32_t)(pos >> 32), k, v};
  __builtin_nontemporal_store(t, reinterpret_cast<u32x4*>(dst));
}

// Range-checked buffer stores: one buffer_store_dwordx4 per call whatever the lanes' offsets;
// a lane whose voffset is kDrop (past the descriptor's size) writes nothing. k_scan_main issues a
// fixed number of them per region, so its counted vmcnt wait retires the next region's DMA
// without waiting for the stores issued after it.
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
constexpr int kSc1 = 16;   // buffer cache-policy bit: sc1 (gfx940+: coherent past the CU's L1)
constexpr uint32_t kDrop = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;   // wave-uniform
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  // every field through readfirstlane: a descriptor the compiler thinks divergent becomes a waterfall
  // loop around every buffer load (k_uniform: 1.21 ms against 0.80 when a divergent loop exit made
  // the batch index, and with it the descriptor, look divergent)
  return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
template <int kAux = 0>
__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t x, uint32_t y, uint32_t z,
                                        uint32_t w) {
  const v4u32 d = {x, y, z, w};
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, off, 0, kAux);
}
// The run prefix's CRC (round 3): 2-byte slicing on LANE-PRIVATE byte tables, so a wave's table reads
// never bank-conflict. Row i of the 64 KiB block is 256 B: dwords [0, 32) hold T16[i] = the register
// after byte i and one zero byte, dwords [32, 64) hold T8[i] = after byte i alone, each replicated
// once per bank; lane l reads dword l mod 32 of a half, so the 32 lanes of a ds_read_b32 group always
// hit 32 distinct banks (MI355X_MICROARCH.md LDS: ds_read_b32 serves lanes {0-31}, {32-63}, bank
// (a/4) mod 32). The address (byte << 8 | 4 (l mod 32)) is one v_perm_b32 and the xors v_bitop3.
// Against the 11/11/10-bit shared tables (round 2: 60 % of LDS-active cycles were conflict cycles at
// config 4) one lookup per byte instead of 0.75, all conflict-free (tools/microbench/mb_uni.hip:
// config 4 verify 0.794 -> 0.724 ms on one box, within 1 % of the same loads XOR-reduced).
constexpr uint32_t kLp2Bytes = 65536;
__device__ __forceinline__ uint32_t lp2_read(const uint8_t* lp2, uint32_t a) {
  return *reinterpret_cast<const uint32_t*>(lp2 + a);
}
__device__ __forceinline__ uint32_t lp2_xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// reg' after the 4 message bytes of w (little-endian, first byte lowest), raw register (no init/final)
__device__ __forceinline__ uint32_t lp2_step4(const uint8_t* lp2, uint32_t lb, uint32_t reg, uint32_t w) {
  const uint32_t x = reg ^ w;
  const uint32_t y = lp2_xor3(x >> 16, lp2_read(lp2, __builtin_amdgcn_perm(x, lb, 0x0C0C0400u)),
                              lp2_read(lp2, __builtin_amdgcn_perm(x, lb, 0x0C0C0500u) + 128u));
  return lp2_xor3(y >> 16, lp2_read(lp2, __builtin_amdgcn_perm(y, lb, 0x0C0C0400u)),
                  lp2_read(lp2, __builtin_amdgcn_perm(y, lb, 0x0C0C0500u) + 128u));
}
// the block from the byte table T8 (the table block's kT8Off): T16[i] = T8[T8[i] & 0xFF] ^ (T8[i] >> 8);
// every thread of the workgroup writes 4 x 16 B (1024 threads: one quarter row each)
__device__ __forceinline__ void lp2_build(uint8_t* lp2, const uint32_t* __restrict__ gtab) {
  const uint32_t* t8 = gtab + kT8Off;
  for (uint32_t q = threadIdx.x; q < 1024u; q += blockDim.x) {
    const uint32_t row = q >> 2, part = q & 3u;
    const uint32_t a = t8[row];
    const uint32_t v = part < 2 ? (t8[a & 0xFFu] ^ (a >> 8)) : a;
    uint4* d = reinterpret_cast<uint4*>(lp2 + row * 256u + part * 64u);
    const uint4 vv = make_uint4(v, v, v, v);
    d[0] = vv; d[1] = vv; d[2] = vv; d[3] = vv;
  }
}
constexpr int kUniPolicy = 0;
__device__ __forceinline__ uint4 ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kUniPolicy);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint32_t ld4(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, kUniPolicy);
}


__device__ __forceinline__ void decode_entry_global(const Pipe& p, uint64_t off, ldb_entry* out) {
  struct G {
    const uint8_t* q;
    __device__ uint32_t operator()(int i) const { return q[i]; }
  };
  Header h;
  decode_header(G{p.img + off}, &h);
  ldb_entry e;
  e.offset = off;
  e.expired_at = h.expired_at;
  e.tx_id = h.tx_id;
  e.crc = h.crc;
  e.k_size = h.k_size;
  e.v_size = h.v_size;
  e.tx_stat = (uint16_t)h.tx_stat;
  e.stat = (uint8_t)h.stat;
  e.hdr_size = (uint8_t)h.size;
  e.enc_hdr_size = (uint8_t)h.enc_size;
  e.pad_[0] = e.pad_[1] = e.pad_[2] = 0;
  e.fid = p.fid;
  *out = e;
}

