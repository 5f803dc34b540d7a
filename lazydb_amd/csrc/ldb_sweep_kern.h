// ldb_sweep_kern.h — the sweep tier's kernels (ldb_sweep.h has the design, types and tables).
// Included by ldb_scan.hip inside its kernel namespace, after the run prefix (k_uniform: its LP2 block,
// buffer-load helpers, uni_finish's terminal rule) and k_compact (decode_entry_global).
#pragma once

// 0x80 in byte j iff byte j of w <= 2 (exact, no borrow between bytes)
__device__ __forceinline__ uint32_t sw_le2(uint32_t w) {
  const uint32_t t = w & 0xFCFCFCFCu;
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
// 0x80 in byte j iff byte j of w is zero
__device__ __forceinline__ uint32_t sw_zero(uint32_t w) {
  return ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
}
// Candidate mask of a window's dword i (w = dword i, wp = i - 1, wn = i + 1): bit 8 j + 7 set iff the
// position p = 4 (i - 1) + j may start an entry LazyDB's writer emits (db.go:473-523 -> EncodeEntry): the
// Status byte p+4 <= 2 (log_entry.go:9-16), ExpiredAt's first byte p+5 even (a non-negative zig-zag
// varint) and the stored crc [p, p+4) not zero (decode_lean rejects all three, so nothing it would accept
// is dropped). Speculation only: the decode decides.
__device__ __forceinline__ uint32_t sw_hits(uint32_t wp, uint32_t w, uint32_t wn) {
  const uint32_t S = sw_le2(w);
  const uint32_t nb = (w >> 8) | (wn << 24);
  const uint32_t E = ~(nb << 7) & 0x80808080u;
  const uint32_t z8 = msb4(sw_zero(wp)) | (msb4(sw_zero(w)) << 4);
  const uint32_t zz = z8 & (z8 >> 1) & (z8 >> 2) & (z8 >> 3);
  const uint32_t C = (((~zz & 0xFu) * 0x00204081u) & 0x01010101u) << 7;
  return S & E & C;
}
__device__ __forceinline__ uint32_t sw_shift(const uint32_t* T, uint32_t r) {
  return T[r & 0xFFu] ^ T[256 + ((r >> 8) & 0xFFu)] ^ T[512 + ((r >> 16) & 0xFFu)] ^ T[768 + (r >> 24)];
}
template <int kCtl>
__device__ __forceinline__ uint32_t sw_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kCtl, 0xF, 0xF, false);
}

// ---------------------------------------------------------------- k_sweep
// One wave per run: rows [A, B) of the image (B - A a multiple of the batch but for the last run).
// Geometry, identical in every wave: a0 = x_s rounded down to a batch, the rest dealt in runs of rl, at least
// kSwMinBatches batches: a run that one entry covers whole holds no chain start, and when a false start
// inside that entry's value makes it look active the links need a pass of their own to set it aside
// (sw_link); 64-KiB runs keep that to entries above 64 KiB, at no cost to the stream (small files only).
struct SwGeo {
  uint64_t xs, ks, a0, rl, nrun;
  bool active;
};
__device__ __forceinline__ SwGeo sw_geo(const Pipe& p, uint64_t nwaves) {
  SwGeo g;
  g.xs = chain_x0(p);
  g.ks = run_k(p);
  g.a0 = g.xs & ~(kSwBatch - 1);
  g.active = g.xs < p.len && !read_eof(p.len, p.io, (int64_t)g.xs, kMaxHeader);
  const uint64_t total = g.active ? p.len - g.a0 : 0;
  const uint64_t nb = (total + kSwBatch - 1) / kSwBatch;   // batches
  uint64_t nr = nwaves < kSwMaxRuns ? nwaves : kSwMaxRuns;
  uint64_t per = nr ? (nb + nr - 1) / nr : 0;              // batches per run
  per = per && per < kSwMinBatches ? kSwMinBatches : per;   // (round 6: runs no entry of <= 64 KiB covers whole)
  g.rl = per * kSwBatch;
  g.nrun = per ? (nb + per - 1) / per : 0;
  return g;
}

__device__ __forceinline__ uint64_t sw_readlane64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
__device__ __forceinline__ uint32_t sw_rank(uint64_t bal, int lane) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

__device__ __forceinline__ uint64_t sw_ld_sc1(const uint64_t* a) {
  return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup-wide inclusive scans for sw_link (1024 threads = 16 waves): within the wave by lane shifts
// (ds_bpermute, 6 rounds, no barrier), then each wave adds the totals of the waves before it (one barrier).
template <class Op, class T>
__device__ __forceinline__ T sw_wg_scan(T v, T ident, Op op, T* s_wtot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T y = __shfl_up(v, o);
    if (lane >= o) v = op(v, y);
  }
  if (lane == 63) s_wtot[wave] = v;
  __syncthreads();
  T pre = ident;
  for (int w = 0; w < wave; ++w) pre = op(pre, s_wtot[w]);
  return op(pre, v);
}

// The links between runs (the last k_sweep workgroup, every thread). The tier's entries are the chain
// from x_s through the runs in order. A run whose walk found a chain (E_r set; "active") continues it when
// E_r is the exit of the last active run before it (x_s before run 0's); a run without one (declined, or no
// walk) is passed when that exit lies at or past its end (an entry longer than the run covers it; its CRC
// is then checked from this run's registers, which every run computes to its end). The tier ends at the first
// run that does neither -- declined, a chain that is not the previous exit's, or an entry start the
// walk could not take -- at the true chain position entering it (the previous exit), or at the end of an
// active run whose chain ended inside it. Fully parallel: the last active run before each run is a
// prefix maximum over the runs, each thread checks a contiguous share; the runs' bases a prefix sum.
// Both scans are wave-level lane shifts plus one pass over the 16 wave totals (four barriers in all).
// Round 6 (found by the CPU emulation of the tier, tests/emu): when the first event is a run whose own walk
// is not the chain's -- its walk took a false start inside an entry's value, as binary values offer, or
// found none -- it is fixed and the links resolved again, up to kSwRelink times: a run the chain passes
// over whole (the exit entering it lies at or past its end) is made inactive (no walk, no entries:
// k_region's checks skip it); one the chain enters at T is re-walked from T over its slab (wave 0, tag
// kSwTagRelink), which is the serial replay's own walk through the run's candidates.
// LDS (the caller's, kSwLinkLds bytes): X of each thread's last active run, the wave totals of both scans,
// the first event, the tier's end, the run to fix (and how, from where) and the re-walk's result
constexpr uint32_t kSwLinkLds = 8 * 1024 + 8 * 16 + 4 * 16 + 8 * 8;
constexpr int kSwRelink = 64;

// the chain from T through run r's slab records (ncand of them, in file order) to the run's end B or the first
// position no record holds; its records tagged kSwTagRelink. One wave (wave 0 of the links' workgroup).
__device__ __forceinline__ void sw_rewalk(const Pipe& p, uint64_t r, uint64_t nrun, uint64_t T, uint64_t B, uint32_t ncand,
                                          uint64_t* Xo, uint64_t* no, bool* deado) {
  const int lane = threadIdx.x & 63;
  const uint64_t cap64 = p.scratch_bytes / 16 / nrun;   // (the run's slab, as sweep_item dealt them)
  const __amdgpu_buffer_rsrc_t srs = rsrc_of(p.scratch + r * cap64, ncand * 16u);
  uint4 rec = make_uint4(0, 0, 0, 0);
  uint64_t lp = ~0ull;
  uint32_t lsz = 0, bi = 0;
  bool dirty = false;
  auto load_blk = [&](uint32_t blk) {
    const uint32_t i = blk * 64u + (uint32_t)lane;
    const v4u32 q = __builtin_amdgcn_raw_buffer_load_b128(srs, i < ncand ? i * 16u : kDrop, 0, kSc1);
    rec = make_uint4(q[0], q[1], q[2], q[3]);
    const uint64_t pos = ((uint64_t)rec.y << 32) | rec.x;
    lp = i < ncand ? (pos & 0xFFFFFFFFFFull) : ~0ull;
    lsz = (uint32_t)((pos >> 40) & 0x3Fu) + rec.z + rec.w;
  };
  auto write_blk = [&](uint32_t blk) {
    const uint32_t i = blk * 64u + (uint32_t)lane;
    store16(srs, i < ncand ? i * 16u : kDrop, rec.x, rec.y, rec.z, rec.w);
  };
  load_blk(0);
  uint64_t x = T, n = 0;
  bool dead = false;
  while (x < B) {
    for (;;) {   // the block holding x (or the last)
      const uint32_t nv = ncand - bi * 64u < 64u ? ncand - bi * 64u : 64u;
      const uint64_t lastp = nv ? sw_readlane64(lp, (int)nv - 1) : 0;
      if (nv == 0 || lastp >= x || (bi + 1) * 64u >= ncand) break;
      if (dirty) write_blk(bi);
      dirty = false;
      load_blk(++bi);
    }
    const uint64_t mt = __ballot(lp == x);
    if (!mt) {
      dead = true;
      break;
    }
    const int L = __builtin_ctzll(mt);
    if (lane == L) {
      rec.y = (rec.y & 0x0FFFFFFFu) | (kSwTagRelink << 28);
      dirty = true;
    }
    ++n;
    x += (uint32_t)__builtin_amdgcn_readlane((int)lsz, L);
  }
  if (dirty) write_blk(bi);
  *Xo = x;
  *no = n;
  *deado = dead;
}
__device__ __forceinline__ void sw_link(const Pipe& p, const SwGeo& g, uint8_t* lds) {
  uint64_t* s_x = reinterpret_cast<uint64_t*>(lds);
  uint64_t* s_wsum = s_x + 1024;
  int32_t* s_wmax = reinterpret_cast<int32_t*>(s_wsum + 16);
  unsigned long long& s_ev = *reinterpret_cast<unsigned long long*>(s_wmax + 16);
  uint64_t* s_w = reinterpret_cast<uint64_t*>(s_wmax + 16);
  uint64_t& s_xe = s_w[1];
  uint64_t& s_fix = s_w[2];   // the run to fix (~0: none), then how (1 inactive, 2 re-walk) and from where
  uint64_t& s_mode = s_w[3];
  uint64_t& s_T = s_w[4];
  uint64_t& s_rx = s_w[5];    // the re-walk's exit, entries, whether it ended inside the run
  uint64_t& s_rn = s_w[6];
  uint64_t& s_rd = s_w[7];
  constexpr int kPer = (kSwMaxRuns + 1023) / 1024;   // runs per thread (blockDim.x = 1024)
  static_assert(64 * kSwWaves == 1024, "sw_link: one 1024-thread workgroup");
  SwCtl* c = p.swctl;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint64_t nrun = g.active ? g.nrun : 0;
  const uint64_t r0 = (uint64_t)tid * kPer;
  // this thread's runs, every load in flight together
  uint64_t E[kPer], X[kPer], hi[kPer], n[kPer];
  uint32_t fl[kPer], nc[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const bool v = r0 + k < nrun;
    const SwRun* q = p.swrun + (v ? r0 + k : 0);
    E[k] = v ? q->E : ~0ull;
    X[k] = q->X;
    hi[k] = q->hi;
    n[k] = q->n;
    fl[k] = v ? q->flags : kSwDecl;
    nc[k] = q->ncand;
  }
  auto mx = [](int32_t a, int32_t b) { return a > b ? a : b; };
  uint64_t evm = ~0ull;
  int32_t incl = -1;
  int pass = 0;
  for (;; ++pass) {
    int32_t la = -1;   // the last active run of this thread's share, and its exit
    uint64_t lx = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (!(fl[k] & kSwDecl) && E[k] != ~0ull) {
        la = (int32_t)(r0 + k);
        lx = X[k];
      }
    s_x[tid] = lx;
    if (tid == 0) {
      s_ev = ~0ull;
      s_fix = ~0ull;
    }
    incl = sw_wg_scan<decltype(mx), int32_t>(la, -1, mx, s_wmax);   // (its barrier publishes s_x)
    int32_t prev0 = __shfl_up(incl, 1);   // the last active run before this share
    if ((tid & 63u) == 0) {
      prev0 = -1;
      for (uint32_t w = 0; w < (tid >> 6); ++w) prev0 = mx(prev0, s_wmax[w]);
    }
    uint64_t T = prev0 >= 0 ? s_x[(uint32_t)prev0 / kPer] : g.xs;   // the chain's position entering the share
    uint64_t ev = ~0ull, xe_mine = 0, fix_mine = 0, T_mine = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (ev != ~0ull || r0 + k >= nrun) continue;
      const uint64_t r = r0 + k;
      const bool relink = pass < kSwRelink && (fl[k] >> 8) != kSwTagRelink;
      if (!(fl[k] & kSwDecl) && E[k] != ~0ull) {
        if (E[k] != T) {
          ev = 2 * r;
          xe_mine = T;
          // passed over whole: its walk is no part of the chain; entered at T: re-walked from there
          fix_mine = relink ? (T >= hi[k] ? 1 : (nc[k] ? 2 : 0)) : 0;
          T_mine = T;
          continue;
        }
        if (fl[k] & kSwDead) { ev = 2 * r + 1; xe_mine = X[k]; continue; }
        T = X[k];
      } else if (T < hi[k]) {   // not covered: the chain has an entry in this run that no walk took
        ev = 2 * r;
        xe_mine = T;
        fix_mine = relink && !(fl[k] & kSwDecl) && nc[k] ? 2 : 0;
        T_mine = T;
      }
    }
    if (ev != ~0ull) atomicMin(&s_ev, (unsigned long long)ev);
    __syncthreads();
    evm = s_ev;
    if (evm != ~0ull && ev == evm) {
      s_xe = xe_mine;
      if (fix_mine) {
        s_fix = evm / 2;
        s_mode = fix_mine;
        s_T = T_mine;
      }
    }
    __syncthreads();
    const uint64_t fix = s_fix;
    if (fix == ~0ull) break;
    const uint64_t mode = s_mode, Tf = s_T;
    if (mode == 2 && tid < 64) {
      uint64_t rx, rn;
      bool rd;
      sw_rewalk(p, fix, nrun, Tf, p.swrun[fix].hi, p.swrun[fix].ncand, &rx, &rn, &rd);
      if (tid == 0) {
        s_rx = rx;
        s_rn = rn;
        s_rd = rd ? 1u : 0u;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      if (r0 + k == fix) {
        if (mode == 1) {   // no walk, no entries, no tag (k_region's checks skip a run with tag 0)
          E[k] = ~0ull;
          n[k] = 0;
          fl[k] &= kSwDecl;
        } else {           // the chain from T
          E[k] = Tf;
          X[k] = s_rx;
          n[k] = s_rn;
          fl[k] = (s_rd ? kSwDead : 0u) | (kSwTagRelink << 8);
        }
        p.swrun[fix].E = E[k];
        p.swrun[fix].X = X[k];
        p.swrun[fix].n = n[k];
        p.swrun[fix].flags = fl[k];
      }
    __syncthreads();   // (every thread has read s_fix, s_ev and the re-walk before the next pass resets them)
  }
  if (evm == ~0ull && tid == nt - 1) s_xe = incl >= 0 ? s_x[(uint32_t)incl / kPer] : g.xs;
  // bases: an exclusive prefix of the runs' entry counts (inactive runs count 0)
  const uint64_t ncov = evm == ~0ull ? nrun : ((evm & 1) ? evm / 2 + 1 : evm / 2);
  uint64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) sum += r0 + k < ncov ? n[k] : 0;
  auto add = [](uint64_t a, uint64_t b) { return a + b; };
  const uint64_t tot = sw_wg_scan<decltype(add), uint64_t>(sum, 0ull, add, s_wsum);   // (its barrier publishes s_xe)
  uint64_t b = tot - sum;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    if (r0 + k < ncov) p.swrun[r0 + k].base = b;
    b += r0 + k < ncov ? n[k] : 0;
  }
  if (tid == nt - 1) {
    c->xs = g.xs;
    c->ks = g.ks;
    c->xe = s_xe;
    c->ke = g.ks + tot;
    c->ncov = ncov;
    c->nrun = nrun;
    c->relinks = (uint64_t)pass;
    c->state = 1;
  }
}

// phase stamps (LDB_STAMPS builds, tools/sweep_time.py): s_memtime cycles summed over the waves. 0 setup,
// 1 loads waited for in a quarter, 2 candidates, 3 CRC + tree, 4 decode (drain), 5 streaming loop in all,
// 6 final decode + walk, 7 links (last workgroup), 8 waves
#ifdef LDB_STAMPS
__device__ uint64_t g_swstamps[16];
#define SW_T(v)   \
  uint64_t v;     \
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory")
#define SW_ADD(k, a, b) swacc[k] += (b) - (a)
#else
#define SW_T(v)
#define SW_ADD(k, a, b)
#endif

// k_sweep's phase S, item vb of vg (one per workgroup): waves run vb kSwWaves + wave of the
// geometry of vg workgroups. LDS (k_sweep's): lp2 the LP2 block, sh shift by 64, 128, ..., 2048, then 16, 32,
// 48 bytes (9 x 1024 words), hits each wave's candidate list (kSwWaves x kSwList words); built once per
// workgroup (tabs).
constexpr uint32_t kSwShBytes = 9 * 1024 * 4;
constexpr uint32_t kSwLds = kSwShBytes + kLp2Bytes + kSwWaves * kSwList * 4;
static_assert(kSwShBytes + 256 < 65536 && kSwShBytes % 128 == 0, "k_sweep: the LP2 base in a DS offset, bank-aligned");
__device__ __forceinline__ void sweep_item(const Pipe& p, uint32_t vb, uint32_t vg, uint8_t* lp2, uint32_t* sh,
                                           uint32_t* hits, int& tabs) {
#ifdef LDB_STAMPS
  uint64_t swacc[9] = {};
#endif
  SW_T(ts0);
  const SwGeo g = sw_geo(p, (uint64_t)vg * kSwWaves);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t r = (uint64_t)vb * kSwWaves + wave;
  const bool mine = g.active && r < g.nrun;
  if (__syncthreads_or(mine ? 1 : 0) && tabs != kLdsSweep) {
    lp2_build(lp2, p.gtab);
    for (uint32_t i = threadIdx.x; i < 6 * 1024; i += blockDim.x) {
      const uint32_t a = p.swt[i], b = i < 3 * 1024 ? p.swt[kSwRowOff + i] : 0u;
      sh[i] = a;
      if (i < 3 * 1024) sh[6 * 1024 + i] = b;
    }
    __syncthreads();
    tabs = kLdsSweep;
  }
  SW_T(ts1);
  SW_ADD(0, ts0, ts1);
  if (mine) {
    const uint64_t A = g.a0 + r * g.rl;
    const uint64_t B = A + g.rl < p.len ? A + g.rl : p.len;
    const uint64_t lo = r == 0 ? g.xs : A;
    const uint32_t lb = ((uint32_t)lane & 31u) * 4u;
    uint32_t* hl = hits + wave * kSwList;
    // the run's slab: an equal share of the scratch tuples
    const uint64_t cap64 = p.scratch_bytes / 16 / g.nrun;
    const uint32_t cap = (uint32_t)(cap64 < 0x7FFFFFFFull ? cap64 : 0x7FFFFFFFull);
    ldb_index_tuple* slab = p.scratch + r * cap64;
    const __amdgpu_buffer_rsrc_t srs = rsrc_of(slab, cap * 16u);
    const uint64_t ib = (p.len - A + 3) & ~3ull;   // (a ternary: min() on 64-bit unsigned is HIP's double overload)
    const __amdgpu_buffer_rsrc_t irs = rsrc_of(p.img + A, (uint32_t)(ib < 0xFFFFFFFFull ? ib : 0xFFFFFFFFull));
    uint32_t npend = 0, ncand = 0;
    bool decl = false;
    // The stop word (SwCtl::stop): run 0 sets it when the tier surely ends inside run 0 -- it declined, or the
    // chain from x_s died within run 0's first decode block (a position no candidate holds: a header
    // decode_lean_w rejects, as in a log of empty keys or negative expiries) -- and the other runs, whose
    // registers then serve no entry of the tier, stop streaming. Polled once per pair of quarters, the value
    // used a pair later (its load completes under the next quarters' loads: no wait of its own).
    const __amdgpu_buffer_rsrc_t krs = rsrc_of(&p.swctl->stop, 8);
    auto stop_tier = [&] {
      if (lane == 0) __hip_atomic_store(&p.swctl->stop, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    bool probe = r == 0;
    // decode hl[0, nf) (one candidate per lane) and append the entries decode_lean accepts to the slab
    auto flush = [&](uint32_t nf) {
      const bool v = (uint32_t)lane < nf;
      const uint32_t off = v ? hl[lane] : 0u;
      const uint32_t oa = off & ~3u, s8 = off & 3u;
      const uint4 q0 = ld16(irs, v ? oa : kDrop), q1 = ld16(irs, v ? oa + 16 : kDrop), q2 = ld16(irs, v ? oa + 32 : kDrop);
      const uint32_t d[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
      uint32_t w[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) w[i] = funnel(d[i + 1], d[i], s8);
      const uint64_t at = A + off;
      Lean e;
      const bool ok = decode_lean_w(w, at, 0u, p.len, p.io, &e) && v && at >= lo;
      const uint64_t bal = __ballot(ok);
      const uint32_t idx = ncand + sw_rank(bal, lane);
      const uint64_t pos = (at & 0xFFFFFFFFFFull) | ((uint64_t)e.hs << 40) | ((uint64_t)e.hs << 46) | ((uint64_t)e.stat << 52);
      store16(srs, ok && idx < cap ? idx * 16u : kDrop, (uint32_t)pos, (uint32_t)(pos >> 32), e.k, e.vv);
      ncand += (uint32_t)__builtin_popcountll(bal);
      if (ncand > cap) decl = true;
      if (probe) {   // run 0's first block holds every candidate up to its last position: walk the chain in it
        probe = false;
        const uint64_t last = sw_readlane64(v ? at : 0ull, (int)nf - 1);
        const uint32_t sz = e.hs + e.k + e.vv;
        uint64_t x = g.xs;
        bool dies = false;
        for (uint32_t s = 0; s < 64u && x <= last; ++s) {   // (x rises through distinct candidates)
          const uint64_t mt = __ballot(ok && at == x);
          if (!mt) {
            dies = true;
            break;
          }
          x += (uint32_t)__builtin_amdgcn_readlane((int)sz, __builtin_ctzll(mt));
        }
        if (dies) stop_tier();
      }
    };
    // The run in quarters of 4 KiB: lane l holds the quarter's bytes [64 l, 64 l + 64) as 4 rows (a row
    // instruction reads 4 KiB in 64-B steps; the lane's bytes stay contiguous for its CRC), lane 63 also the
    // next quarter's first 8 bytes. The next quarter's rows are in flight while one is processed.
    struct QB {
      uint32_t d[16];
      uint32_t n0, n1;
    };
    auto load_q = [&](QB& q, uint32_t qo) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 x = ld16(irs, qo + 64u * (uint32_t)lane + 16u * k);
        q.d[4 * k] = x.x; q.d[4 * k + 1] = x.y; q.d[4 * k + 2] = x.z; q.d[4 * k + 3] = x.w;
      }
      // the look-ahead (used by lane 63): one wave-uniform address, one request. Every load here and in the
      // loop below is unconditional (past the run's end the bytes are unused, past the file's the buffer
      // returns zeros), so the compiler's vmcnt waits count exactly: the next quarter's rows stay in flight
      // while this one is processed (a load under a branch made it wait for all of them)
      const v2u32 x = __builtin_amdgcn_raw_buffer_load_b64(irs, qo + 4096u, 0, 0);
      q.n0 = x[0];
      q.n1 = x[1];
    };
    // The group registers (RG, 4 KiB = one quarter), four quarters at once: row t of rga holds quarter t's 16
    // window registers (lane 16 t + m <- window m); a 4-level tree in each row (shifts by 256 .. 2048 B)
    // leaves the group's register in the row's lane 15. One tree per four quarters instead of four levels
    // per quarter with one active lane.
    uint32_t rga = 0;
    const uint32_t bpa = (4u * ((uint32_t)lane & 15u) + 3u) * 4u;   // ds_bpermute: from lane 4 (l mod 16) + 3
    auto rg_tree = [&](uint32_t qo_last) {
      uint32_t r = rga, y;
      y = sw_dpp<0x111>(r);                                   // row_shr:1
      if (lane & 1) r ^= sw_shift(sh + 2048, y);
      y = sw_dpp<0x112>(r);                                   // row_shr:2
      if ((lane & 3) == 3) r ^= sw_shift(sh + 3072, y);
      y = sw_dpp<0x114>(r);                                   // row_shr:4
      if ((lane & 7) == 7) r ^= sw_shift(sh + 4096, y);
      y = sw_dpp<0x118>(r);                                   // row_shr:8
      if ((lane & 15) == 15) {
        r ^= sw_shift(sh + 5120, y);
        if ((uint32_t)(lane >> 4) <= ((qo_last >> 12) & 3u))
          p.swrg[((A + (qo_last & ~0x3FFFu)) >> 12) + (uint32_t)(lane >> 4)] = r;
      }
      rga = 0;
    };
    // one quarter: its candidates appended to the hit list (in file order), each lane's register over its
    // 64 bytes, the window (RW) and quarter (RG) registers. False when the run is too dense for the tier.
    auto proc_q = [&](const QB& q, uint32_t qo) -> bool {
      SW_T(tq0);
      const uint32_t wo = qo + 64u * (uint32_t)lane;   // the lane's window, from A
      // the next window's first two dwords: the next lane's (lane 63: loaded with the quarter)
      uint32_t n0 = sw_dpp<0x130>(q.d[0]), n1 = sw_dpp<0x130>(q.d[1]);   // wave_shl:1
      n0 = lane == 63 ? q.n0 : n0;
      n1 = lane == 63 ? q.n1 : n1;
      auto D = [&](int i) -> uint32_t { return i < 16 ? q.d[i] : (i == 16 ? n0 : n1); };
#ifdef LDB_STAMPS
      asm volatile("" ::"v"(n0), "v"(n1));
#endif
      SW_T(tq1);
      SW_ADD(1, tq0, tq1);
      // the lane's raw register over its 64 bytes (LP2: conflict-free lane-private tables)
      uint32_t reg = 0;
      {   // one chain per 16-B row (four in flight), joined by shifts of 48, 32 and 16 bytes
        uint32_t c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          c[k] = lp2_step4(lp2, lb, lp2_step4(lp2, lb, lp2_step4(lp2, lb, lp2_step4(lp2, lb, 0u, q.d[4 * k]), q.d[4 * k + 1]),
                                              q.d[4 * k + 2]), q.d[4 * k + 3]);
        reg = sw_shift(sh + 8 * 1024, c[0]) ^ sw_shift(sh + 7 * 1024, c[1]) ^ sw_shift(sh + 6 * 1024, c[2]) ^ c[3];
      }
      // a tree over the lanes (DPP): level i joins runs of 2^i lanes with a shift by 64 2^i bytes. Lane 4m+3
      // ends level 2 with window m's register (RW, 256 B); the quarter's 16 go to the group accumulator
      const uint64_t w0 = (A + qo) >> 8;
      uint32_t v = reg, y;
      y = sw_dpp<0x111>(v);                                   // row_shr:1
      if (lane & 1) v ^= sw_shift(sh, y);
      y = sw_dpp<0x112>(v);                                   // row_shr:2
      if ((lane & 3) == 3) {
        v ^= sw_shift(sh + 1024, y);
        p.swrw[w0 + (uint32_t)(lane >> 2)] = v;
      }
      {   // quarter t of its 16-KiB batch (the run starts on a batch): its RWs to row t of the accumulator
        const uint32_t t = (qo >> 12) & 3u;
        const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute((int)bpa, (int)v);
        if ((uint32_t)(lane >> 4) == t) rga = x;
        if (t == 3u) rg_tree(qo);
      }
#ifdef LDB_STAMPS
      asm volatile("" ::"v"(v));
#endif
      SW_T(tq2);
      SW_ADD(3, tq1, tq2);
      // candidates: a 64-bit map of the lane's positions p = 4 i + j whose Status byte p + 4 is <= 2
      // (log_entry.go:9-16; 3 VALU per dword). The decode (flush: decode_lean_w) decides; this only has to
      // keep every true start, and text values have no such byte. A lane window of zeros holds none whose
      // status byte is its own (the crc before it would be zero, which the decode rejects). A pair of
      // dwords' masks packs to 8 bits with one multiply (bit 7 + 8 j of the even dword's mask and 4 + 8 j
      // after the odd one's shift both move by 24 - 7 j: to bit 24 + j and 28 + j, no two partial products
      // on one bit).
      uint32_t mlo = 0, mhi = 0;
      bool has = false;
      {
        uint32_t orw = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) orw |= q.d[i];
        // (the last dword's candidates, p = 60..63, need a nonzero crc byte: here or in the next window's first
        // dword -- a zero tail would otherwise offer 4 per window and flood the list)
        const uint32_t zk = orw ? 0x80808080u : 0u, zk16 = (orw | n0) ? 0x80808080u : 0u;
        uint32_t cm[16], any = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t w = D(i + 1);
          cm[i] = ~(((w & 0x7C7C7C7Cu) + 0x7F7F7F7Fu) | w) & (i < 15 ? zk : zk16);
          any |= cm[i];
        }
        const uint64_t hb = __ballot(any != 0u);
        has = hb != 0;
        // binary values (about 3 of 256 bytes pass the Status test): in a quarter where many lanes hold
        // candidates, those whose next byte is odd go too -- decode_lean_w takes only an even first byte of
        // ExpiredAt (a zig-zag varint of a time >= 0), so they would be decoded for nothing (half of them)
        if (__builtin_popcountll(hb) > 16) {
#pragma unroll
          for (int i = 0; i < 16; ++i) cm[i] &= ~__builtin_amdgcn_alignbit(D(i + 2), D(i + 1), 1u);
        }
        auto pack = [&] {
          uint32_t pk[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) pk[k] = (((cm[2 * k + 1] >> 3) | (cm[2 * k] >> 7)) * 0x01020408u) >> 24;
          mlo = mhi = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            mlo |= pk[k] << (8 * k);
            mhi |= pk[4 + k] << (8 * k);
          }
        };
        if (has) {   // (text values: about half the quarters hold no header byte <= 2)
          pack();
          // a lane with many: zero runs inside values (every zero byte passes the Status test). Positions
          // whose crc bytes are surely zero go (dword i zero and bytes 0-2 of dword i + 1 zero: the crc of
          // every start in dword i + 1's status bytes); the decode would reject them, the list would fill
          if (__ballot(__builtin_popcount(mlo) + __builtin_popcount(mhi) > 8)) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if ((D(i) | (D(i + 1) << 8)) == 0u) cm[i] = 0u;
            pack();
          }
        }
      }
      if (has && !decl) {   // (a declined run keeps its registers, not its candidates)
        const uint32_t cnt = (uint32_t)__builtin_popcount(mlo) + (uint32_t)__builtin_popcount(mhi);
        // exclusive prefix of the counts over the lanes (DPP scan: rows, then row 15 / lane 31 broadcasts)
        uint32_t inc = cnt;
        inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x111, 0xF, 0xF, true);
        inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x112, 0xF, 0xF, true);
        inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x114, 0xF, 0xF, true);
        inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x118, 0xF, 0xF, true);
        inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x142, 0xA, 0xF, false);
        inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x143, 0xC, 0xF, false);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (tot) {
          if (npend + tot > kSwList) return false;   // too dense for the tier: the region pipeline takes it
          // the lanes before a candidate's lane in its 256-B window keep their 64-B registers, so k_sweep_fin
          // gets P(x) of an entry start from <= 3 of them and <= 63 bytes
          const uint64_t cb = __ballot(cnt != 0u);
          const uint32_t quad = (uint32_t)(cb >> ((uint32_t)lane & 60u)) & 0xFu;
          if ((quad >> (((uint32_t)lane & 3u) + 1u))) p.swpl[(A + wo) >> 6] = reg;
          // the positions, in file order (lane-major: the windows are in lane order)
          uint32_t j = npend + inc - cnt;
          while (mlo) {
            hl[j++] = wo + (uint32_t)__builtin_ctz(mlo);
            mlo &= mlo - 1;
          }
          while (mhi) {
            hl[j++] = wo + 32u + (uint32_t)__builtin_ctz(mhi);
            mhi &= mhi - 1;
          }
          npend += tot;
        }
      }

      SW_T(tq3);
      SW_ADD(2, tq2, tq3);
      return true;
    };
    auto drain = [&] {   // decode while 64 or more candidates wait
      SW_T(td0);
      LDB_WAVE_XCHG_LDS();   // the hit list's stores, before other lanes read them
      while (npend >= 64 && !decl) {
        flush(64);
        npend -= 64;
        for (uint32_t i = (uint32_t)lane; i < npend; i += 64) {   // (npend < kSwList - 64: one or few rounds)
          const uint32_t t = hl[64 + i];
          LDB_WAIT_LGKM0();
          hl[i] = t;
        }
        LDB_WAVE_XCHG_LDS();
      }
      SW_T(td1);
      SW_ADD(4, td0, td1);
    };
    const uint32_t nq = (uint32_t)((B - A + 4095) / 4096);
    SW_T(tl0);
    QB P, Q;
    if (nq > 0) load_q(P, 0);
    // Every run streams to its end, declined or not: a declined run (too many candidates) ends the tier
    // unless an entry from an earlier run covers it whole (sw_link), and that entry's CRC is then checked
    // from this run's window and group registers, so they are always complete. (Round 5 broke out of the
    // loop at a decline and polled a stop word; an entry spanning a declined run was then verified from
    // stale registers.) The one exception is the stop word above: set only when the tier ends inside run 0.
    uint32_t sv = 0;   // the stop word, as loaded a pair of quarters ago
    for (uint32_t i = 0; i < nq; i += 2) {
      if (r != 0 && sv) {   // (the run's registers are not needed: run 0 ends the tier)
        decl = true;
        break;
      }
      load_q(Q, (i + 1) * 4096u);
      __builtin_amdgcn_sched_barrier(0);
      if (!proc_q(P, i * 4096u)) decl = true;
      sv = __builtin_amdgcn_raw_buffer_load_b32(krs, 0, 0, kSc1);   // (before the next rows: done by their wait)
      load_q(P, (i + 2) * 4096u);
      __builtin_amdgcn_sched_barrier(0);
      if (i + 1 < nq && !proc_q(Q, (i + 1) * 4096u)) decl = true;
      drain();
      if (r == 0 && decl) {   // run 0 declined: the tier ends at x_s
        stop_tier();
        break;
      }
    }
    if (nq & 3u) rg_tree((nq - 1u) * 4096u);   // a final batch of fewer than four quarters
    SW_T(tl1);
    SW_ADD(5, tl0, tl1);
    if (!decl && npend) flush(npend);
    LDB_WAVE_XCHG_VM();   // the slab's stores, before the walk reads them (other lanes' records)
    // ---- the walk: from the run's first entry, each entry's end is the next candidate
    uint64_t E = ~0ull, X = 0, cnt = 0;
    uint32_t fl = decl ? kSwDecl : 0u, tag = 1, si = 0;
    uint64_t lp = ~0ull;   // this lane's record of the current block: position
    uint32_t lsz = 0;
    uint4 rec = make_uint4(0, 0, 0, 0);
    uint32_t bi = 0;
    bool dirty = false;
    auto load_blk = [&](uint32_t blk) {
      const uint32_t i = blk * 64u + (uint32_t)lane;
      const bool v = i < ncand;
      const v4u32 q = __builtin_amdgcn_raw_buffer_load_b128(srs, v ? i * 16u : kDrop, 0, kSc1);
      rec = make_uint4(q[0], q[1], q[2], q[3]);
      const uint64_t pos = ((uint64_t)rec.y << 32) | rec.x;
      lp = v ? (pos & 0xFFFFFFFFFFull) : ~0ull;
      lsz = (uint32_t)((pos >> 40) & 0x3Fu) + rec.z + rec.w;
    };
    auto write_blk = [&](uint32_t blk) {
      const uint32_t i = blk * 64u + (uint32_t)lane;
      store16(srs, i < ncand ? i * 16u : kDrop, rec.x, rec.y, rec.z, rec.w);
    };
    if (!decl && ncand <= cap) {
      if (ncand) load_blk(0);
      if (r == 0) E = g.xs;
      else if (ncand) E = sw_readlane64(lp, 0);
      uint64_t x = E;
      // the block holding x (or the last): blocks are searched forward from the current one
      auto seek = [&](uint64_t xx) {
        for (;;) {
          const uint32_t nv = ncand - bi * 64u < 64u ? ncand - bi * 64u : 64u;
          const uint64_t lastp = nv ? sw_readlane64(lp, (int)nv - 1) : 0;
          if (nv == 0 || lastp >= xx || (bi + 1) * 64u >= ncand) break;
          if (dirty) write_blk(bi);
          dirty = false;
          load_blk(++bi);
        }
      };
      // A speculated chain of fewer than kSwTrust entries is weak, whether it leaves the run (a false start
      // inside a value can claim a size past the run's end) or ends in it (the file's last run). Later
      // starts are tried, and the first weak chain is taken back (re-walked, so its records carry its tag
      // again) only if none of them holds; the links then check it like any other.
      // Round 6 (found by the CPU emulation of the tier, tests/emu): of several weak chains the one taken back
      // leaves the run if any does, and has the most entries among those (the first of equals). In a run
      // that an entry's binary value fills up to a few short true entries, the value's false starts end
      // inside or claim one huge entry, while the true chain leaves with more; in the file's last run no
      // chain can leave (the decode bounds every entry by the file).
      uint64_t wE = ~0ull;
      uint32_t wtag = 0, wrank = 0;
      while (E != ~0ull) {
        if (x >= B) {
          if (r == 0 || cnt >= kSwTrust || tag == kSwTagWalk) { X = x; break; }
          if (wE == ~0ull || 64u + (uint32_t)cnt > wrank) { wE = E; wtag = tag; wrank = 64u + (uint32_t)cnt; }
        } else {
          seek(x);
          const uint64_t mt = __ballot(lp == x);
          if (mt) {
            const int L = __builtin_ctzll(mt);
            if (lane == L) {
              rec.y = (rec.y & 0x0FFFFFFFu) | (tag << 28);
              dirty = true;
            }
            ++cnt;
            x += (uint32_t)__builtin_amdgcn_readlane((int)lsz, L);
            continue;
          }
          // x is no candidate: the chain ends here (run 0's is the true chain from x_s; a speculated one
          // that held kSwTrust entries is kept and its end checked by the links), or the speculated first
          // entry was false and the next candidate is tried
          if (r == 0 || cnt >= kSwTrust || tag == kSwTagWalk) { fl |= kSwDead; X = x; break; }
          if (wE == ~0ull || (uint32_t)cnt > wrank) { wE = E; wtag = tag; wrank = (uint32_t)cnt; }   // weak too: a short chain that ends (the file's last run)
        }
        ++si;
        ++tag;
        cnt = 0;
        if (si >= ncand) { E = ~0ull; break; }
        if (dirty) write_blk(bi);
        dirty = false;
        bi = si / 64u;
        load_blk(bi);
        E = x = sw_readlane64(lp, (int)(si % 64u));
      }
      if (E == ~0ull && wE != ~0ull) {
        if (dirty) write_blk(bi);
        dirty = false;
        bi = 0;
        load_blk(0);
        E = x = wE;
        tag = wtag;
        cnt = 0;
        while (x < B) {
          seek(x);
          const uint64_t mt = __ballot(lp == x);
          if (!mt) {   // the weak chain ended inside the run
            fl |= kSwDead;
            break;
          }
          const int L = __builtin_ctzll(mt);
          if (lane == L) {
            rec.y = (rec.y & 0x0FFFFFFFu) | (tag << 28);
            dirty = true;
          }
          ++cnt;
          x += (uint32_t)__builtin_amdgcn_readlane((int)lsz, L);
        }
        X = x;
      }
      if (dirty) write_blk(bi);
    }
    if (E == ~0ull || (fl & kSwDecl)) {   // no chain: no record of this run is the tier's (k_sweep_fin: tag 0)
      tag = 0;
      cnt = 0;
    }
    {   // the run record (SwRun, 64 B): lanes 0-3 store 16 B each
      const uint64_t u0 = lane == 0 ? E : (lane == 1 ? cnt : (lane == 2 ? lo : 0ull));
      const uint64_t u1 = lane == 0 ? X : (lane == 1 ? ((uint64_t)ncand << 32 | (fl | (tag << 8))) : (lane == 2 ? B : 0ull));
      const __amdgpu_buffer_rsrc_t rrs = rsrc_of(p.swrun + r, 64);
      store16(rrs, lane < 4 ? (uint32_t)lane * 16u : kDrop, (uint32_t)u0, (uint32_t)(u0 >> 32), (uint32_t)u1,
              (uint32_t)(u1 >> 32));
    }
    SW_T(tl2);
    SW_ADD(6, tl1, tl2);
  }
#ifdef LDB_STAMPS
  swacc[8] = mine ? 1 : 0;
  if (lane == 0)
    for (int k = 0; k < 9; ++k) atomicAdd((unsigned long long*)&g_swstamps[k], (unsigned long long)swacc[k]);
#endif
}

// after the last phase-S item, in the workgroup that completed it (every item released, then acquired by
// k_sweep): the links between runs, with the geometry every item used
__device__ __forceinline__ void sweep_last(const Pipe& p, uint32_t vg, uint8_t* lds) {
  SW_T(tk0);
  sw_link(p, sw_geo(p, (uint64_t)vg * kSwWaves), lds);
  SW_T(tk1);
#ifdef LDB_STAMPS
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&g_swstamps[7], (unsigned long long)(tk1 - tk0));
#endif
}

// ---------------------------------------------------------------- k_sweep_fin
// slicing-by-16 / -by-4 register steps over little-endian words (S: kSwSl16Off tables, S[k][b] = the raw
// register after byte b and k zero bytes)
__device__ __forceinline__ uint32_t sw_sl16(const uint32_t* S, uint32_t reg, const uint4& q) {
  const uint32_t a = reg ^ q.x;
  return S[15 * 256 + (a & 0xFFu)] ^ S[14 * 256 + ((a >> 8) & 0xFFu)] ^ S[13 * 256 + ((a >> 16) & 0xFFu)] ^
         S[12 * 256 + (a >> 24)] ^ S[11 * 256 + (q.y & 0xFFu)] ^ S[10 * 256 + ((q.y >> 8) & 0xFFu)] ^
         S[9 * 256 + ((q.y >> 16) & 0xFFu)] ^ S[8 * 256 + (q.y >> 24)] ^ S[7 * 256 + (q.z & 0xFFu)] ^
         S[6 * 256 + ((q.z >> 8) & 0xFFu)] ^ S[5 * 256 + ((q.z >> 16) & 0xFFu)] ^ S[4 * 256 + (q.z >> 24)] ^
         S[3 * 256 + (q.w & 0xFFu)] ^ S[2 * 256 + ((q.w >> 8) & 0xFFu)] ^ S[1 * 256 + ((q.w >> 16) & 0xFFu)] ^
         S[q.w >> 24];
}
__device__ __forceinline__ uint32_t sw_sl4(const uint32_t* S, uint32_t reg, uint32_t w) {
  const uint32_t a = reg ^ w;
  return S[3 * 256 + (a & 0xFFu)] ^ S[2 * 256 + ((a >> 8) & 0xFFu)] ^ S[1 * 256 + ((a >> 16) & 0xFFu)] ^ S[a >> 24];
}
// the register over the first m (< 16) bytes of row q
__device__ __forceinline__ uint32_t sw_row_head(const uint32_t* S, uint32_t reg, const uint4& q, uint32_t m) {
  const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (4 * k + 4 <= m) reg = sw_sl4(S, reg, qw[k]);
  const uint32_t k4 = m >> 2, w = k4 == 0 ? q.x : (k4 == 1 ? q.y : (k4 == 2 ? q.z : q.w));
#pragma unroll
  for (uint32_t t = 0; t < 3; ++t)
    if (t < (m & 3u)) reg = S[(reg ^ (w >> (8 * t))) & 0xFFu] ^ (reg >> 8);
  return reg;
}

// raw register over image bytes [x & ~255, x) (the window-local prefix P(x)): every row it needs loaded
// at once (one memory round trip), then slicing-by-16
__device__ __forceinline__ uint32_t sw_prefix(const Pipe& p, const uint32_t* S, uint64_t x) {
  const uint64_t ws = x & ~(uint64_t)(kSwW - 1);
  const uint32_t n = (uint32_t)(x - ws);
  const uint4* row = reinterpret_cast<const uint4*>(p.img + ws);
  uint32_t reg = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // two rounds of 8 rows (registers)
    if (128u * h >= n) break;
    uint4 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = 16u * (8 * h + i) < n ? row[8 * h + i] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t lo = 16u * (8 * h + i);
      if (lo + 16u <= n) reg = sw_sl16(S, reg, q[i]);
      else if (lo < n) reg = sw_row_head(S, reg, q[i], n - lo);
    }
  }
  return reg;
}

// P(x) from the lane registers k_sweep kept: swpl[i] is the register of image bytes [64 i, 64 i + 64),
// written for the lanes before a candidate's lane in its 256-B window (so for those of every chain entry's
// start), folded with shifts by 64 B (T64), then the <= 63 bytes [x & ~63, x)
__device__ __forceinline__ uint32_t sw_prefix_pl(const Pipe& p, const uint32_t* S, const uint32_t* T64, uint64_t x) {
  const uint64_t ws = x & ~63ull, l = x >> 6;
  const uint32_t n = (uint32_t)(x - ws), j = (uint32_t)l & 3u;
  const uint4* row = reinterpret_cast<const uint4*>(p.img + ws);
  uint4 q[4];
  uint32_t lr[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = 16u * i < n ? row[i] : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (uint32_t t = 0; t < 3; ++t) lr[t] = t < j ? p.swpl[(l & ~3ull) + t] : 0u;
  uint32_t reg = 0;
#pragma unroll
  for (uint32_t t = 0; t < 3; ++t)
    if (t < j) reg = sw_shift(T64, reg) ^ lr[t];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t lo = 16u * i;
    if (lo + 16u <= n) reg = sw_sl16(S, reg, q[i]);
    else if (lo < n) reg = sw_row_head(S, reg, q[i], n - lo);
  }
  return reg;
}

// little-endian dword at image offset x (x + 4 <= len)
__device__ __forceinline__ uint32_t sw_word(const Pipe& p, uint64_t x) {
  const uint32_t* a = reinterpret_cast<const uint32_t*>(p.img + (x & ~3ull));
  const uint32_t s = (uint32_t)(x & 3u);
  return s ? funnel(a[1], a[0], s) : a[0];
}

// R = shift(R, 256) ^ rw[w] over windows w in [w0, w0 + n), n < 16: the loads in flight together
__device__ __forceinline__ uint32_t sw_fold_win(const Pipe& p, const uint32_t* T256, uint32_t R, uint64_t w0, uint32_t n) {
  uint32_t v[15];
#pragma unroll
  for (uint32_t i = 0; i < 15; ++i) v[i] = i < n ? p.swrw[w0 + i] : 0u;
#pragma unroll
  for (uint32_t i = 0; i < 15; ++i)
    if (i < n) R = sw_shift(T256, R) ^ v[i];
  return R;
}

// getEntryCrc(entry at s, size sz) == its stored crc (log_entry.go:110-121, log_file.go:141-143): the raw
// CRC register of the span [a, e) = [s + 4, s + sz) from ~0, from the window registers:
//   same window:  R = shift(~0 ^ P(a), e - a) ^ P(e)
//   otherwise:    R = shift(~0 ^ P(a), end(a) - a) ^ RW[w(a)], then R = shift(R, 256) ^ RW[w] over the whole
//                 windows between (shift(R, 4096) ^ RG[g] over whole groups), then R = shift(R, e - w(e)) ^ P(e)
// where P(x) is the raw register over [x & ~255, x) and shift by n bytes multiplies by x^(8n) mod P.
// P(a) is P(s) stepped over the stored crc (restarting at a window edge); P(e) is the next chain entry's
// P(s), except after the tier's last entry (e == xe), whose end need not hold a candidate.
// Ps = P(s), this entry's start prefix; Pe = P(e) when the caller has it (the next chain entry's Ps from
// another lane, have_pe), else computed here.
__device__ __forceinline__ bool sw_verify(const Pipe& p, const uint32_t* S, const uint32_t* T256, const uint32_t* T4096,
                                          const uint32_t* T64, uint64_t s, uint64_t sz, uint64_t xe, uint32_t Ps,
                                          bool have_pe, uint32_t Pe_in) {
  const uint64_t a = s + 4, e = s + sz;
  const uint32_t crc = sw_word(p, s);
  uint32_t Pa = Ps;
#pragma unroll
  for (uint32_t t = 0; t < 4; ++t) {
    Pa = S[(Pa ^ (crc >> (8 * t))) & 0xFFu] ^ (Pa >> 8);
    if (((s + t + 1) & (kSwW - 1)) == 0) Pa = 0;   // a window edge after the byte: P restarts there
  }
  const uint32_t Pe = have_pe ? Pe_in : (e == xe ? sw_prefix(p, S, e) : sw_prefix_pl(p, S, T64, e));
  const uint64_t wa = a >> 8, we = e >> 8;
  uint32_t R;
  if (wa == we) {
    R = multmodp(p.xw[e - a], ~Pa) ^ Pe;
  } else {
    R = multmodp(p.xw[((wa + 1) << 8) - a], ~Pa) ^ p.swrw[wa];
    uint64_t w = wa + 1;
    // windows up to the first group boundary, whole groups 16 at a time, the windows after the last group
    const uint64_t g0 = (w + kSwG - 1) & ~(uint64_t)(kSwG - 1);
    const uint64_t w1 = g0 < we ? g0 : we;
    R = sw_fold_win(p, T256, R, w, (uint32_t)(w1 - w));
    w = w1;
    uint64_t ng = (we - w) / kSwG;
    while (ng) {
      const uint32_t m = ng < 16 ? (uint32_t)ng : 16u;
      uint32_t v[16];
#pragma unroll
      for (uint32_t i = 0; i < 16; ++i) v[i] = i < m ? p.swrg[w / kSwG + i] : 0u;
#pragma unroll
      for (uint32_t i = 0; i < 16; ++i)
        if (i < m) R = sw_shift(T4096, R) ^ v[i];
      w += (uint64_t)m * kSwG;
      ng -= m;
    }
    R = sw_fold_win(p, T256, R, w, (uint32_t)(we - w));
    R = multmodp(p.xw[e - (we << 8)], R) ^ Pe;
  }
  return R == ~crc;
}

__device__ __forceinline__ void sw_finish(const Pipe& p) {
  SwCtl* c = p.swctl;
  const int lane = threadIdx.x & 63;
  const uint64_t ks = c->ks, ke = c->ke, nsw = ke - ks;
  const uint64_t fail = __hip_atomic_load(&c->fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ldb_scan_result res;
  res.fid = p.fid;
  res.n_repairs = 0;
  res.n_regions = 0;
  res.n_fast = 0;
  res.n_broken = 0;
  res.n_run = ks;
  bool done = false;
  if (fail < nsw) {
    // the failing entry: the run whose entries hold index `fail` (bases ascend), then its tagged record
    uint64_t lo = 0, hi = c->ncov - 1;
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) / 2;
      if (p.swrun[mid].base <= fail) lo = mid; else hi = mid - 1;
    }
    const SwRun q = p.swrun[lo];
    const uint64_t tag = q.flags >> 8;
    uint64_t rank = q.base, pos = 0;
    for (uint32_t b0 = 0; b0 < q.ncand; b0 += 64) {
      const uint32_t i = b0 + (uint32_t)lane;
      const ldb_index_tuple t = p.scratch[lo * (p.scratch_bytes / 16 / c->nrun) + (i < q.ncand ? i : 0)];
      const bool on = i < q.ncand && (t.pos >> 60) == tag;
      const uint64_t bal = __ballot(on);
      const uint32_t k = sw_rank(bal, lane);
      const uint64_t hit = __ballot(on && rank + k == fail);
      if (hit) {
        pos = sw_readlane64(t.pos & 0xFFFFFFFFFFull, __builtin_ctzll(hit));
        break;
      }
      rank += (uint64_t)__builtin_popcountll(bal);
    }
    res.status = LDB_ERR_CRC;
    res.n_entries = ks + fail;
    res.end_off = pos;
    res.n_sweep = fail;
    done = true;
  } else {
    const uint64_t x0 = c->xe;
    int32_t st;
    if (read_eof(p.len, p.io, (int64_t)x0, kMaxHeader)) {
      st = LDB_EOF_WINDOW;
    } else {
      const uint32_t b = x0 + (uint64_t)lane < p.len ? (uint32_t)p.img[x0 + lane] : 0u;
      auto fetch = [&](int i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)b, i); };
      st = classify_entry(fetch, p.len, p.io, x0).status;
    }
    if (st == LDB_EOF_WINDOW || st == LDB_EOF_SENTINEL || st == LDB_EOF_KV || st == LDB_ERR_MALFORMED) {
      res.status = st;
      res.n_entries = ke;
      res.end_off = x0;
      res.n_sweep = nsw;
      done = true;
    } else if (lane == 0) {   // the region pipeline replays from x0, after the K entries before it
      p.dyn[0] = ke;
      p.dyn[5] = x0;
      p.dyn[7] = nsw;
    }
  }
  if (lane == 0) {
    if (done) {
      if (res.n_entries > p.cap) res.status = LDB_ERR_CAPACITY;
      *p.result = res;
      p.dyn[7] = res.n_sweep;
      p.dyn[3] = kUniDone;
    }
    c->fail = ~0ull;   // (state stays 1 until the next pipeline's init: every k_region workgroup reads it)
  }
}

// k_region phase F, item vb of vg (rounds 1-5 the k_sweep_fin kernel): wave w takes runs vb kSwWaves + w, stepping
// by vg kSwWaves, one lane per chain entry. st: the shift by 256 and 4096 bytes, the slicing-by-16 tables and
// the shift by 64 (kSwFinLds bytes of k_sweep's LDS), copied once per workgroup (tabs)
constexpr uint32_t kSwFinLds = (2 * 1024 + 16 * 256 + 1024) * 4;
__device__ __forceinline__ void fin_item(const Pipe& p, uint32_t vb, uint32_t vg, uint32_t* st, int& tabs) {
  SwCtl* c = p.swctl;
  if (tabs != kLdsFin) {   // every load in flight before the stores
    static_assert(kSwFinLds / 4 % (64 * kSwWaves) == 0, "fin_item: the workgroup copies whole rounds of words");
    constexpr int kR = kSwFinLds / 4 / (64 * kSwWaves);
    uint32_t v[kR];
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      const uint32_t i = threadIdx.x + 64u * kSwWaves * k;
      v[k] = p.swt[i < 1024 ? 2 * 1024 + i : (i < 2048 ? 6 * 1024 + i - 1024 : (i < 6144 ? kSwSl16Off + i - 2048 : i - 6144))];
    }
#pragma unroll
    for (int k = 0; k < kR; ++k) st[threadIdx.x + 64u * kSwWaves * k] = v[k];
    __syncthreads();
    tabs = kLdsFin;
  }
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t ks = c->ks, ncov = c->ncov, nrun = c->nrun, xe = c->xe;
  const uint64_t cap64 = nrun ? p.scratch_bytes / 16 / nrun : 0;
  for (uint64_t r = (uint64_t)vb * kSwWaves + wave; r < ncov; r += (uint64_t)vg * kSwWaves) {
    const SwRun q = p.swrun[r];
    const uint64_t tag = q.flags >> 8;
    if (tag == 0) continue;   // a covered run (sw_link): no entry of the chain starts in it
    uint64_t rank = q.base;
    const ldb_index_tuple* slab = p.scratch + r * cap64;
    ldb_index_tuple tn{};
    if ((uint32_t)lane < q.ncand) tn = slab[lane];
    for (uint32_t b0 = 0; b0 < q.ncand; b0 += 64) {
      const uint32_t i = b0 + (uint32_t)lane;
      const ldb_index_tuple t = tn;
      if (i + 64u < q.ncand) tn = slab[i + 64u];   // the next block's record in flight during this one's checks
      const bool on = i < q.ncand && (t.pos >> 60) == tag;
      const uint64_t bal = __ballot(on);
      const uint64_t my = rank + sw_rank(bal, lane);
      rank += (uint64_t)__builtin_popcountll(bal);
      const uint64_t s = t.pos & 0xFFFFFFFFFFull;
      const uint64_t sz = ((t.pos >> 40) & 0x3Fu) + (uint64_t)t.k_size + t.v_size;
      // each entry's start prefix once: the next chain entry (the next lane with a record of the chain,
      // whose start is this one's end) hands its P to this lane
      const uint32_t Ps = on ? sw_prefix_pl(p, st + 2048, st + 6144, s) : 0u;
      const uint64_t after = lane < 63 ? bal & (~0ull << (lane + 1)) : 0ull;
      const int nl = after ? (int)__builtin_ctzll(after) : lane;
      const uint32_t Pn = (uint32_t)__shfl((int)Ps, nl);
      if (!on) continue;
      if (!sw_verify(p, st + 2048, st, st + 1024, st + 6144, s, sz, xe, Ps, after != 0ull, Pn))
        atomicMin((unsigned long long*)&c->fail, (unsigned long long)my);
      const uint64_t k = ks + my;
      if (k < p.cap) {
        if (p.kind == LDB_TUPLE_ENTRY) decode_entry_global(p, s, reinterpret_cast<ldb_entry*>(p.out) + k);
        else store_tuple(reinterpret_cast<ldb_index_tuple*>(p.out) + k, t.pos & kSwPosMask, t.k_size, t.v_size);
      }
    }
  }
}
