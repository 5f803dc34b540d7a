// simt.h — a CPU emulation of the gfx950 execution model the sweep tier's kernels are written in
// (TEST HARNESS ONLY: tests/emu/sweep_emu.cpp; never linked into liblazydb_gpu.so, never a fallback).
//
// Every thread of a workgroup is a fiber (ucontext) on its own stack, run in turn by one scheduler on one
// host thread. The cross-lane operations -- ballot, readlane, readfirstlane, DPP moves, ds_bpermute,
// shuffles -- are collectives of the 64 lanes of a wave: each lane leaves its operand and yields until the
// wave's last lane has arrived and computed every lane's result, so the kernel code runs unmodified, lane
// by lane, with the hardware's cross-lane semantics. __syncthreads is the same over the workgroup. Between
// collectives a lane runs ahead of the others, so lanes that exchange data through memory must say where
// (LDB_WAVE_XCHG_*, ldb_devmem.h: a counted wait on the GPU, a wave synchronisation here). Lanes
// that reach different collectives (divergent code around a cross-lane operation, which the kernels must
// not have) or a wave that waits for a lane that has returned abort with a message: a deadlock here is a
// bug in the kernel's convergence, not in the emulation.
//
// Buffer descriptors carry their range: a dword of a buffer load past it reads zero and a dword of a
// buffer store past it is dropped (the raw-buffer range check the kernels rely on, kDrop offsets
// included). DPP reads of a lane outside the pattern return a poison word (0xDEADBEEF): results that
// depend on it differ from the oracle. Atomics and fences are plain operations (one host thread).
#pragma once

#include <ucontext.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <vector>

namespace simt {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Dim3 {
  uint32_t x, y, z;
};
struct Rsrc {
  const uint8_t* base;
  uint32_t bytes;
};

[[noreturn]] inline void die(const char* what) {
  std::fprintf(stderr, "simt: %s\n", what);
  std::abort();
}

enum Op { kBallot = 1, kReadlane, kFirst, kDpp, kBperm, kShfl, kShflUp, kSync };

struct WaveSync {
  int arrived = 0;
  int op = 0;
  uint64_t gen = 0;
  uint64_t a[64], b[64], c[64], out[64];
};
struct Fiber {
  ucontext_t uc;
  char* stack = nullptr;
  bool done = false;
};
// fiber stacks, kept across workgroups (a workgroup is 1,024 fibers; allocating their stacks per workgroup
// dominated the sanitizer build's time)
inline char* stack_at(uint32_t i, size_t bytes) {
  static std::vector<std::unique_ptr<char[]>> pool;
  static size_t pool_bytes = 0;
  if (pool_bytes != bytes) {
    pool.clear();
    pool_bytes = bytes;
  }
  while (pool.size() <= i) pool.emplace_back(new char[bytes]);
  return pool[i].get();
}
struct Block {
  uint32_t n = 0;
  Dim3 bidx{}, bdim{}, gdim{};
  std::vector<Fiber> f;
  std::vector<WaveSync> w;
  int bar_arrived = 0, bar_acc = 0, bar_res = 0;
  uint64_t bar_gen = 0;
  ucontext_t sched;
  int cur = -1;
  uint64_t progress = 0;
  std::function<void()> body;
};
inline Block*& blk() {
  static Block* b = nullptr;
  return b;
}
inline uint32_t tid() { return (uint32_t)blk()->cur; }
inline Dim3 thread_idx() { return Dim3{tid(), 0, 0}; }
inline Dim3 block_idx() { return blk()->bidx; }
inline Dim3 block_dim() { return blk()->bdim; }
inline Dim3 grid_dim() { return blk()->gdim; }
inline int lane() { return (int)(tid() & 63u); }

inline void yield() {
  Block* b = blk();
  swapcontext(&b->f[b->cur].uc, &b->sched);
}

inline void fiber_entry() {
  Block* b = blk();
  b->body();
  b->f[b->cur].done = true;
  ++b->progress;
  swapcontext(&b->f[b->cur].uc, &b->sched);
  die("a finished fiber was resumed");
}

// One workgroup of n threads (a multiple of 64) running body on every thread to completion.
inline void run_block(Dim3 bidx, Dim3 gdim, uint32_t n, std::function<void()> body, size_t stack_bytes = 256 << 10) {
  if (n == 0 || n % 64) die("workgroups are whole waves");
  Block b;
  b.n = n;
  b.bidx = bidx;
  b.bdim = Dim3{n, 1, 1};
  b.gdim = gdim;
  b.body = std::move(body);
  b.f.resize(n);
  b.w.resize(n / 64);
  Block* prev = blk();
  blk() = &b;
  for (uint32_t i = 0; i < n; ++i) {
    Fiber& f = b.f[i];
    f.stack = stack_at(i, stack_bytes);
    getcontext(&f.uc);
    f.uc.uc_stack.ss_sp = f.stack;
    f.uc.uc_stack.ss_size = stack_bytes;
    f.uc.uc_link = nullptr;
    makecontext(&f.uc, fiber_entry, 0);
  }
  uint32_t left = n;
  while (left) {
    const uint64_t before = b.progress;
    for (uint32_t i = 0; i < n; ++i) {
      if (b.f[i].done) continue;
      b.cur = (int)i;
      swapcontext(&b.sched, &b.f[i].uc);
      if (b.f[i].done) --left;
    }
    if (left && b.progress == before) die("deadlock: lanes wait at a collective or barrier others never reach");
  }
  blk() = prev;
}

// a wave collective: every lane leaves (a, b, c); the last to arrive fills out[] for all
template <class F>
inline uint64_t collective(int op, uint64_t a, uint64_t b, uint64_t c, F compute) {
  Block* bk = blk();
  const uint32_t t = tid();
  WaveSync& w = bk->w[t >> 6];
  const int l = (int)(t & 63u);
  if (w.arrived == 0) w.op = op;
  else if (w.op != op) die("lanes of a wave reached different collectives (divergent cross-lane code)");
  w.a[l] = a;
  w.b[l] = b;
  w.c[l] = c;
  ++bk->progress;
  if (++w.arrived == 64) {
    compute(w);
    w.arrived = 0;
    ++w.gen;
  } else {
    const uint64_t g = w.gen;
    while (w.gen == g) yield();
  }
  return w.out[l];
}

inline int barrier_or(int pred) {
  Block* b = blk();
  b->bar_acc |= pred ? 1 : 0;
  ++b->progress;
  if (++b->bar_arrived == (int)b->n) {
    b->bar_res = b->bar_acc;
    b->bar_acc = 0;
    b->bar_arrived = 0;
    ++b->bar_gen;
  } else {
    const uint64_t g = b->bar_gen;
    while (b->bar_gen == g) yield();
  }
  return b->bar_res;
}

inline uint64_t ballot(bool p) {
  return collective(kBallot, p ? 1 : 0, 0, 0, [](WaveSync& w) {
    uint64_t m = 0;
    for (int i = 0; i < 64; ++i) m |= (w.a[i] & 1) << i;
    for (int i = 0; i < 64; ++i) w.out[i] = m;
  });
}
// the kernels' marked exchange points (LDB_WAVE_XCHG_*): every lane's stores before any lane's next loads
inline void wave_sync() {
  collective(kSync, 0, 0, 0, [](WaveSync& w) {
    for (int i = 0; i < 64; ++i) w.out[i] = 0;
  });
}
inline uint32_t readlane(uint32_t v, int src) {
  return (uint32_t)collective(kReadlane, v, (uint64_t)(uint32_t)src, 0, [](WaveSync& w) {
    const uint64_t s = w.b[0];
    for (int i = 0; i < 64; ++i)
      if (w.b[i] != s) die("readlane: a lane index that is not wave-uniform");
    if (s > 63) die("readlane: lane index out of range");
    for (int i = 0; i < 64; ++i) w.out[i] = w.a[s];
  });
}
inline uint32_t readfirstlane(uint32_t v) {
  return (uint32_t)collective(kFirst, v, 0, 0, [](WaveSync& w) {
    for (int i = 0; i < 64; ++i) w.out[i] = w.a[0];
  });
}
// update_dpp(old, src, ctl, row_mask, bank_mask, bound_ctrl): the patterns the kernels use
inline uint32_t update_dpp(uint32_t old, uint32_t src, int ctl, int row_mask, int bank_mask, bool bound_ctrl) {
  const uint64_t key = (uint64_t)(uint32_t)ctl | ((uint64_t)(row_mask & 0xF) << 16) | ((uint64_t)(bank_mask & 0xF) << 20) |
                       ((uint64_t)bound_ctrl << 24);
  return (uint32_t)collective(kDpp, src, old, key, [](WaveSync& w) {
    const uint64_t k = w.c[0];
    for (int i = 0; i < 64; ++i)
      if (w.c[i] != k) die("dpp: control that is not wave-uniform");
    const int ctl = (int)(k & 0xFFFF), rm = (int)((k >> 16) & 0xF), bm = (int)((k >> 20) & 0xF);
    const bool bc = (k >> 24) & 1;
    for (int l = 0; l < 64; ++l) {
      const int row = l >> 4, bank = (l >> 2) & 3, rl = l & 15;
      if (!((rm >> row) & 1) || !((bm >> bank) & 1)) {
        w.out[l] = w.b[l];   // lane not written: keeps old
        continue;
      }
      int s = -1;
      if (ctl >= 0x111 && ctl <= 0x11F) {   // row_shr:n
        const int n = ctl - 0x110;
        s = rl >= n ? l - n : -1;
      } else if (ctl >= 0x101 && ctl <= 0x10F) {   // row_shl:n
        const int n = ctl - 0x100;
        s = rl + n < 16 ? l + n : -1;
      } else if (ctl == 0x130) {   // wave_shl:1
        s = l < 63 ? l + 1 : -1;
      } else if (ctl == 0x138) {   // wave_shr:1
        s = l > 0 ? l - 1 : -1;
      } else if (ctl == 0x142) {   // row_bcast:15
        s = row >= 1 ? 16 * row - 1 : -1;
      } else if (ctl == 0x143) {   // row_bcast:31
        s = row >= 2 ? 31 : -1;
      } else if (ctl < 0x100) {   // quad_perm
        s = (l & ~3) + ((ctl >> (2 * (l & 3))) & 3);
      } else {
        die("dpp: a control this emulation does not model");
      }
      w.out[l] = s >= 0 ? w.a[s] : (bc ? 0u : w.b[l]);
    }
  });
}
inline uint32_t mov_dpp(uint32_t src, int ctl, int row_mask, int bank_mask, bool bound_ctrl) {
  return update_dpp(0xDEADBEEFu, src, ctl, row_mask, bank_mask, bound_ctrl);
}
inline int bpermute(int addr, int v) {
  return (int)collective(kBperm, (uint32_t)v, (uint32_t)addr, 0, [](WaveSync& w) {
    for (int l = 0; l < 64; ++l) w.out[l] = w.a[(w.b[l] >> 2) & 63];
  });
}
template <class T>
inline T shfl(T v, int src) {
  static_assert(sizeof(T) <= 8, "shfl: up to 64 bits");
  uint64_t u = 0;
  std::memcpy(&u, &v, sizeof(T));
  const uint64_t r = collective(kShfl, u, (uint64_t)(uint32_t)src, 0, [](WaveSync& w) {
    for (int l = 0; l < 64; ++l) w.out[l] = w.a[w.b[l] & 63];
  });
  T o;
  std::memcpy(&o, &r, sizeof(T));
  return o;
}
template <class T>
inline T shfl_up(T v, unsigned d) {
  static_assert(sizeof(T) <= 8, "shfl_up: up to 64 bits");
  uint64_t u = 0;
  std::memcpy(&u, &v, sizeof(T));
  const uint64_t r = collective(kShflUp, u, d, 0, [](WaveSync& w) {
    for (int l = 0; l < 64; ++l) w.out[l] = (uint64_t)l >= w.b[l] ? w.a[l - w.b[l]] : w.a[l];
  });
  T o;
  std::memcpy(&o, &r, sizeof(T));
  return o;
}

// lane-local ALU
inline uint32_t mbcnt_lo(uint32_t m, uint32_t acc) {
  const int l = lane();
  const uint32_t mask = l >= 32 ? ~0u : ((1u << l) - 1u);
  return acc + (uint32_t)__builtin_popcount(m & mask);
}
inline uint32_t mbcnt_hi(uint32_t m, uint32_t acc) {
  const int l = lane();
  const uint32_t mask = l < 32 ? 0u : ((1u << (l - 32)) - 1u);
  return acc + (uint32_t)__builtin_popcount(m & mask);
}
inline uint32_t alignbit(uint32_t a, uint32_t b, uint32_t s) {
  return (uint32_t)((((uint64_t)a << 32) | b) >> (s & 31u));
}
inline uint32_t alignbyte(uint32_t a, uint32_t b, uint32_t s) {
  return (uint32_t)((((uint64_t)a << 32) | b) >> (8u * (s & 3u)));
}
// v_perm_b32: byte i of the result by selector byte i over {src0 (bytes 4-7), src1 (bytes 0-3)}
inline uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t c = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t q = (sel >> (8 * i)) & 0xFFu;
    uint32_t v;
    if (q < 8) v = (uint32_t)(c >> (8 * q)) & 0xFFu;
    else if (q == 0x0C) v = 0;
    else if (q >= 0x0D) v = 0xFF;
    else die("perm: a sign-replicating selector this emulation does not model");
    r |= v << (8 * i);
  }
  return r;
}
inline uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c, uint32_t t) {
  uint32_t r = 0;
  for (int i = 0; i < 32; ++i) {
    const uint32_t idx = (((a >> i) & 1u) << 2) | (((b >> i) & 1u) << 1) | ((c >> i) & 1u);
    r |= ((t >> idx) & 1u) << i;
  }
  return r;
}

// buffer descriptors and range-checked loads / stores (per dword)
inline Rsrc make_rsrc(const void* p, int, int bytes, int) { return Rsrc{static_cast<const uint8_t*>(p), (uint32_t)bytes}; }
inline uint32_t bload4(const Rsrc& r, uint32_t off) {
  if ((uint64_t)off + 4 > r.bytes) return 0;
  uint32_t v;
  std::memcpy(&v, r.base + off, 4);
  return v;
}
inline uint32_t buf_load_b32(const Rsrc& r, uint32_t off, uint32_t soff, int) { return bload4(r, off + soff); }
inline u32x2 buf_load_b64(const Rsrc& r, uint32_t off, uint32_t soff, int) {
  const uint32_t o = off + soff;
  u32x2 v = {bload4(r, o), bload4(r, o + 4)};
  return v;
}
inline u32x4 buf_load_b128(const Rsrc& r, uint32_t off, uint32_t soff, int) {
  const uint32_t o = off + soff;
  u32x4 v = {bload4(r, o), bload4(r, o + 4), bload4(r, o + 8), bload4(r, o + 12)};
  return v;
}
inline void buf_store_b128(u32x4 d, const Rsrc& r, uint32_t off, uint32_t soff, int) {
  const uint32_t o = off + soff;
  for (uint32_t i = 0; i < 4; ++i)
    if ((uint64_t)o + 4 * i + 4 <= r.bytes) {
      const uint32_t x = d[i];
      std::memcpy(const_cast<uint8_t*>(r.base) + o + 4 * i, &x, 4);
    }
}

template <class T, class U>
inline T atomic_add(T* p, U v) {
  const T o = *p;
  *p = (T)(o + (T)v);
  return o;
}
template <class T, class U>
inline T atomic_min(T* p, U v) {
  const T o = *p;
  if ((T)v < o) *p = (T)v;
  return o;
}

}  // namespace simt

// ---- the HIP / gfx950 vocabulary of the kernel sources, mapped onto the emulation
struct uint4 {
  uint32_t x, y, z, w;
};
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }

#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __shared__ static
#define __launch_bounds__(...)
#define threadIdx (::simt::thread_idx())
#define blockIdx (::simt::block_idx())
#define blockDim (::simt::block_dim())
#define gridDim (::simt::grid_dim())
#define __amdgpu_buffer_rsrc_t ::simt::Rsrc
#define __HIP_MEMORY_SCOPE_AGENT 3
#define LDB_WAIT_LGKM0() ((void)0)
#define LDB_WAIT_VM0() ((void)0)
#define LDB_WAVE_XCHG_LDS() ::simt::wave_sync()
#define LDB_WAVE_XCHG_VM() ::simt::wave_sync()

#define __ballot(p) ::simt::ballot((p))
#define __shfl(v, s) ::simt::shfl((v), (s))
#define __shfl_up(v, d) ::simt::shfl_up((v), (d))
#define __syncthreads() ((void)::simt::barrier_or(0))
#define __syncthreads_or(p) ::simt::barrier_or((p))
#define atomicAdd(p, v) ::simt::atomic_add((p), (v))
#define atomicMin(p, v) ::simt::atomic_min((p), (v))
#define __hip_atomic_load(p, o, s) (*(p))
#define __hip_atomic_store(p, v, o, s) ((void)(*(p) = (v)))
#define __builtin_amdgcn_fence(o, s) ((void)0)
#define __builtin_amdgcn_sched_barrier(x) ((void)0)
#define __builtin_amdgcn_readfirstlane(v) ::simt::readfirstlane((uint32_t)(v))
#define __builtin_amdgcn_readlane(v, l) ::simt::readlane((uint32_t)(v), (l))
#define __builtin_amdgcn_mov_dpp(v, c, rm, bm, bc) ((int)::simt::mov_dpp((uint32_t)(v), (c), (rm), (bm), (bc)))
#define __builtin_amdgcn_update_dpp(o, v, c, rm, bm, bc) \
  ((int)::simt::update_dpp((uint32_t)(o), (uint32_t)(v), (c), (rm), (bm), (bc)))
#define __builtin_amdgcn_ds_bpermute(a, v) ::simt::bpermute((a), (v))
#define __builtin_amdgcn_mbcnt_lo(m, a) ::simt::mbcnt_lo((m), (a))
#define __builtin_amdgcn_mbcnt_hi(m, a) ::simt::mbcnt_hi((m), (a))
#define __builtin_amdgcn_alignbit(a, b, s) ::simt::alignbit((a), (b), (s))
#define __builtin_amdgcn_alignbyte(a, b, s) ::simt::alignbyte((a), (b), (s))
#define __builtin_amdgcn_perm(a, b, s) ::simt::perm((a), (b), (s))
#define __builtin_amdgcn_bitop3_b32(a, b, c, t) ::simt::bitop3((a), (b), (c), (t))
#define __builtin_amdgcn_make_buffer_rsrc(p, st, n, f) ::simt::make_rsrc((p), (st), (n), (f))
#define __builtin_amdgcn_raw_buffer_load_b32(r, o, so, a) ::simt::buf_load_b32((r), (o), (so), (a))
#define __builtin_amdgcn_raw_buffer_load_b64(r, o, so, a) ::simt::buf_load_b64((r), (o), (so), (a))
#define __builtin_amdgcn_raw_buffer_load_b128(r, o, so, a) ::simt::buf_load_b128((r), (o), (so), (a))
#define __builtin_amdgcn_raw_buffer_store_b128(d, r, o, so, a) ::simt::buf_store_b128((d), (r), (o), (so), (a))
