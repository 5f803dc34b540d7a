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
// Geometry, identical in every wave: a0 = x_s rounded down to a batch, the rest dealt in runs of rl.
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
  const uint64_t per = nr ? (nb + nr - 1) / nr : 0;        // batches per run
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

// The links between runs (the last k_sweep workgroup, every thread). The tier's entries are the chain
// from x_s through the runs in order. Run r continues it when its first walked entry E_r is the previous
// run's exit; a run the previous exit jumps over (an entry longer than the run: no start inside it) is
// covered and passes that exit on. The tier ends at the first run that declined or does not continue the
// chain (at its true entry, the exit before it), or at the end of a run whose chain ended inside it.
// Every run linked to its predecessor is the common case and is checked in parallel; from the first
// run that is not, wave 0 follows the chain run by run (64 run records in registers at a time).
__device__ void sw_link(const Pipe& p, const SwGeo& g) {
  __shared__ unsigned long long s_ev;
  __shared__ uint64_t s_sum[1024];
  __shared__ uint64_t s_ncov, s_xe;
  SwCtl* c = p.swctl;
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const int lane = (int)(tid & 63u);
  if (tid == 0) s_ev = ~0ull;
  __syncthreads();
  const uint64_t nrun = g.active ? g.nrun : 0;
  for (uint64_t r = tid; r < nrun; r += nt) {
    const SwRun q = p.swrun[r];
    uint64_t ev = ~0ull;
    if ((q.flags & kSwDecl) || q.E == ~0ull || (r > 0 && p.swrun[r - 1].X != q.E)) ev = 2 * r;
    else if (q.flags & kSwDead) ev = 2 * r + 1;
    if (ev != ~0ull) atomicMin(&s_ev, (unsigned long long)ev);
  }
  __syncthreads();
  if (tid < 64) {
    const uint64_t ev = s_ev;
    uint64_t ncov, xe;
    if (nrun == 0) {
      ncov = 0;
      xe = g.xs;
    } else if (ev == ~0ull) {
      ncov = nrun;
      xe = p.swrun[nrun - 1].X;
    } else if (ev & 1) {
      ncov = ev / 2 + 1;
      xe = p.swrun[ev / 2].X;
    } else {
      const uint64_t r0 = ev / 2;
      uint64_t T = r0 ? p.swrun[r0 - 1].X : g.xs;   // the chain's position entering run r0
      ncov = ~0ull;
      xe = 0;
      for (uint64_t c0 = r0; c0 < nrun && ncov == ~0ull; c0 += 64) {
        const uint64_t i = c0 + (uint64_t)lane;
        SwRun q{};
        if (i < nrun) q = p.swrun[i];
        const uint32_t nl = nrun - c0 < 64 ? (uint32_t)(nrun - c0) : 64u;
        for (uint32_t l = 0; l < nl; ++l) {
          const uint64_t E = sw_readlane64(q.E, (int)l), X = sw_readlane64(q.X, (int)l), hi = sw_readlane64(q.hi, (int)l);
          const uint32_t fl = (uint32_t)__builtin_amdgcn_readlane((int)q.flags, (int)l);
          if (T >= hi) {   // covered: the chain has no entry in this run (its walk followed false candidates)
            if ((uint32_t)lane == l) {
              p.swrun[i].n = 0;
              p.swrun[i].flags = fl & 0xFFu;   // walk tag 0: no record is the tier's
            }
            continue;
          }
          if ((fl & kSwDecl) || E != T) { ncov = c0 + l; xe = T; break; }
          T = X;
          if (fl & kSwDead) { ncov = c0 + l + 1; xe = X; break; }
        }
      }
      if (ncov == ~0ull) { ncov = nrun; xe = T; }
    }
    if (tid == 0) { s_ncov = ncov; s_xe = xe; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint64_t ncov = s_ncov, xe = s_xe;
  // bases: an exclusive prefix of the runs' entry counts, each thread a contiguous share (read past the
  // CU's L1: wave 0 may just have zeroed a covered run's count)
  const uint64_t per = (ncov + nt - 1) / nt;
  const uint64_t r0 = tid * per, r1 = r0 + per < ncov ? r0 + per : ncov;
  uint64_t s = 0;
  for (uint64_t r = r0; r < r1; ++r) s += sw_ld_sc1(&p.swrun[r].n);
  s_sum[tid] = s;
  __syncthreads();
  for (uint32_t o = 1; o < nt; o <<= 1) {   // Hillis-Steele over the threads' sums
    const uint64_t y = tid >= o ? s_sum[tid - o] : 0;
    __syncthreads();
    s_sum[tid] += y;
    __syncthreads();
  }
  uint64_t b = s_sum[tid] - s;
  for (uint64_t r = r0; r < r1; ++r) {
    p.swrun[r].base = b;
    b += sw_ld_sc1(&p.swrun[r].n);
  }
  if (tid == nt - 1) {
    c->xs = g.xs;
    c->ks = g.ks;
    c->xe = xe;
    c->ke = g.ks + s_sum[nt - 1];
    c->ncov = ncov;
    c->nrun = nrun;
    c->stop = ~0ull;
    c->done0 = 0;
    c->state = 1;
  }
}

// kHitGroups: every 64-B row of a window whose dwords may hold a candidate's Status byte
__global__ __launch_bounds__(64 * kSwWaves) void k_sweep(Pipe p) {
  __shared__ __attribute__((aligned(256))) uint8_t lp2[kLp2Bytes];
  __shared__ __attribute__((aligned(16))) uint32_t sh[4 * 1024];   // shift by 256, 512, 1024, 2048 bytes
  __shared__ uint32_t hits[kSwWaves][kSwList];
  __shared__ int s_last;
  if (scan_done(p)) return;   // the run prefix ended the scan
  const SwGeo g = sw_geo(p, (uint64_t)gridDim.x * kSwWaves);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t r = (uint64_t)blockIdx.x * kSwWaves + wave;
  const bool mine = g.active && r < g.nrun;
  if (__syncthreads_or(mine ? 1 : 0)) {
    lp2_build(lp2, p.gtab);
    for (uint32_t i = threadIdx.x; i < 4 * 1024; i += blockDim.x) sh[i] = p.swt[i];
    __syncthreads();
  }
  if (mine) {
    const uint64_t A = g.a0 + r * g.rl;
    const uint64_t B = A + g.rl < p.len ? A + g.rl : p.len;
    const uint64_t lo = r == 0 ? g.xs : A;
    const uint32_t lb = ((uint32_t)lane & 31u) * 4u;
    uint32_t* hl = hits[wave];
    // the run's slab: an equal share of the scratch tuples
    const uint64_t cap64 = p.scratch_bytes / 16 / g.nrun;
    const uint32_t cap = (uint32_t)(cap64 < 0x7FFFFFFFull ? cap64 : 0x7FFFFFFFull);
    ldb_index_tuple* slab = p.scratch + r * cap64;
    const __amdgpu_buffer_rsrc_t srs = rsrc_of(slab, cap * 16u);
    const __amdgpu_buffer_rsrc_t irs = rsrc_of(p.img + A, (uint32_t)min((p.len - A + 3) & ~3ull, (uint64_t)0xFFFFFFFFu));
    const __amdgpu_buffer_rsrc_t krs = rsrc_of(&p.swctl->stop, 8);
    uint32_t npend = 0, ncand = 0;
    bool decl = false;
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
    };
    v2u32 kv = {0xFFFFFFFFu, 0xFFFFFFFFu};
    for (uint64_t b = A; b < B; b += kSwBatch) {
      {   // a run before this one ends the tier: nothing here is used
        const uint64_t stop = ((uint64_t)__builtin_amdgcn_readfirstlane(kv[1]) << 32) | __builtin_amdgcn_readfirstlane(kv[0]);
        if (stop < r) { decl = true; break; }
      }
      const uint32_t wo = (uint32_t)(b - A) + (uint32_t)lane * kSwW;
      uint32_t d[64];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint4 q = ld16(irs, wo + 16u * k);
        d[4 * k] = q.x; d[4 * k + 1] = q.y; d[4 * k + 2] = q.z; d[4 * k + 3] = q.w;
      }
      const uint32_t n0l = ld4(irs, lane == 63 ? wo + kSwW : kDrop), n1l = ld4(irs, lane == 63 ? wo + kSwW + 4 : kDrop);
      kv = __builtin_amdgcn_raw_buffer_load_b64(krs, 0, 0, kSc1);
      __builtin_amdgcn_sched_barrier(0);
      // the next window's first two dwords (lane 63: the next batch's, loaded)
      uint32_t n0 = (uint32_t)__shfl_down((int)d[0], 1), n1 = (uint32_t)__shfl_down((int)d[1], 1);
      n0 = lane == 63 ? n0l : n0;
      n1 = lane == 63 ? n1l : n1;
      auto D = [&](int i) -> uint32_t { return i < 64 ? d[i] : (i == 64 ? n0 : n1); };
      uint32_t orw = 0;
#pragma unroll
      for (int i = 0; i < 64; ++i) orw |= d[i];
      const uint32_t zmask = orw ? 0xFFFFFFFFu : 0u;   // an all-zero window has no candidate but in its last 4 bytes
      // pass 1: rows (groups of 4 dwords) where some lane may have a candidate; the lane's count
      uint32_t gm = 0, cnt = 0;
#pragma unroll
      for (int gi = 0; gi < 16; ++gi) {
        uint32_t any = 0;
#pragma unroll
        for (int k = 1; k <= 4; ++k) any |= small_bytes(D(4 * gi + k));
        if (gi < 15) any &= zmask;
        if (__ballot(any != 0u)) {
          gm |= 1u << gi;
#pragma unroll
          for (int k = 1; k <= 4; ++k) cnt += (uint32_t)__builtin_popcount(sw_hits(D(4 * gi + k - 1), D(4 * gi + k), D(4 * gi + k + 1)));
        }
      }
      if (gm) {
        uint32_t x = cnt;   // inclusive scan over the lanes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)x, o);
          if (lane >= o) x += y;
        }
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
        if (npend + tot > kSwList) { decl = true; break; }   // too dense for the tier: the region pipeline takes it
        // pass 2: the positions, in file order (lane-major: the windows are in lane order)
        uint32_t j = npend + x - cnt;
#pragma unroll
        for (int gi = 0; gi < 16; ++gi) {
          if ((gm >> gi) & 1u) {
#pragma unroll
            for (int k = 1; k <= 4; ++k) {
              uint32_t m = sw_hits(D(4 * gi + k - 1), D(4 * gi + k), D(4 * gi + k + 1));
              if (gi < 15 || k < 4) m &= zmask;
              const uint32_t base = wo + 4u * (4 * gi + k - 1);
#pragma unroll
              for (int t = 0; t < 4; ++t) {
                if (m) {
                  hl[j++] = base + ((uint32_t)__builtin_ctz(m) >> 3);
                  m &= m - 1;
                }
              }
            }
          }
        }
        npend += tot;
      }
      // the window's raw register (LP2: conflict-free lane-private tables)
      uint32_t reg = 0;
#pragma unroll
      for (int k = 0; k < 32; ++k) reg = lp2_step4(lp2, lb, lp2_step4(lp2, lb, reg, d[2 * k]), d[2 * k + 1]);
      const uint64_t wi = (b >> 8) + (uint64_t)lane;
      p.swrw[wi] = reg;
      // group registers: a tree over each 16-lane row (DPP row shifts), lane 15 of the row ends with it
      {
        uint32_t v = reg, y;
        y = sw_dpp<0x111>(v);
        if (lane & 1) v ^= sw_shift(sh, y);
        y = sw_dpp<0x112>(v);
        if ((lane & 3) == 3) v ^= sw_shift(sh + 1024, y);
        y = sw_dpp<0x114>(v);
        if ((lane & 7) == 7) v ^= sw_shift(sh + 2048, y);
        y = sw_dpp<0x118>(v);
        if ((lane & 15) == 15) {
          v ^= sw_shift(sh + 3072, y);
          p.swrg[wi >> 4] = v;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the hit list's stores, before other lanes read them
      while (npend >= 64 && !decl) {
        flush(64);
        npend -= 64;
        for (uint32_t i = (uint32_t)lane; i < npend; i += 64) {   // (npend < kSwList - 64: one or few rounds)
          const uint32_t t = hl[64 + i];
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          hl[i] = t;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      if (decl) break;
    }
    if (!decl && npend) flush(npend);
    if (decl) atomicMin((unsigned long long*)&p.swctl->stop, (unsigned long long)r);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slab's stores, before the walk reads them
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
      while (E != ~0ull) {
        if (x >= B) { X = x; break; }
        for (;;) {   // the block holding x, or the last
          const uint32_t nv = ncand - bi * 64u < 64u ? ncand - bi * 64u : 64u;
          const uint64_t lastp = nv ? sw_readlane64(lp, (int)nv - 1) : 0;
          if (nv == 0 || lastp >= x || (bi + 1) * 64u >= ncand) break;
          if (dirty) write_blk(bi);
          dirty = false;
          load_blk(++bi);
        }
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
        if (r == 0 || cnt >= kSwTrust || tag == 15) { fl |= kSwDead; X = x; break; }
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
      if (dirty) write_blk(bi);
    }
    {   // the run record (SwRun, 64 B): lanes 0-3 store 16 B each
      const uint64_t u0 = lane == 0 ? E : (lane == 1 ? cnt : (lane == 2 ? lo : 0ull));
      const uint64_t u1 = lane == 0 ? X : (lane == 1 ? ((uint64_t)ncand << 32 | (fl | (tag << 8))) : (lane == 2 ? B : 0ull));
      const __amdgpu_buffer_rsrc_t rrs = rsrc_of(p.swrun + r, 64);
      store16(rrs, lane < 4 ? (uint32_t)lane * 16u : kDrop, (uint32_t)u0, (uint32_t)(u0 >> 32), (uint32_t)u1,
              (uint32_t)(u1 >> 32));
    }
  }
  // the last workgroup resolves the links
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = atomicAdd((unsigned long long*)&p.swctl->done0, 1ull) == (unsigned long long)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  sw_link(p, g);
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
__device__ __forceinline__ bool sw_verify(const Pipe& p, const uint32_t* S, const uint32_t* T256, const uint32_t* T4096,
                                          uint64_t s, uint64_t sz) {
  const uint64_t a = s + 4, e = s + sz;
  const uint32_t crc = sw_word(p, s);
  const uint32_t Pa = sw_prefix(p, S, a), Pe = sw_prefix(p, S, e);
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

__device__ __attribute__((noinline)) void sw_finish(const Pipe& p) {
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
    c->fail = ~0ull;
    c->done1 = 0;
    c->state = 0;
  }
}

__global__ __launch_bounds__(64 * kSwFinWaves) void k_sweep_fin(Pipe p) {
  __shared__ __attribute__((aligned(16))) uint32_t st[2 * 1024 + 16 * 256];
  __shared__ int s_last;
  if (scan_done(p)) return;
  SwCtl* c = p.swctl;
  if (c->state != 1) return;
  for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) {
    st[i] = p.swt[i];                         // shift by 256
    st[1024 + i] = p.swt[4 * 1024 + i];       // shift by 4096
  }
  for (uint32_t i = threadIdx.x; i < 16 * 256; i += blockDim.x) st[2048 + i] = p.swt[kSwSl16Off + i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t ks = c->ks, ncov = c->ncov, nrun = c->nrun;
  const uint64_t cap64 = nrun ? p.scratch_bytes / 16 / nrun : 0;
  for (uint64_t r = (uint64_t)blockIdx.x * kSwFinWaves + wave; r < ncov; r += (uint64_t)gridDim.x * kSwFinWaves) {
    const SwRun q = p.swrun[r];
    const uint64_t tag = q.flags >> 8;
    if (tag == 0) continue;   // a covered run (sw_link): no entry of the chain starts in it
    uint64_t rank = q.base;
    const ldb_index_tuple* slab = p.scratch + r * cap64;
    for (uint32_t b0 = 0; b0 < q.ncand; b0 += 64) {
      const uint32_t i = b0 + (uint32_t)lane;
      ldb_index_tuple t{};
      if (i < q.ncand) t = slab[i];
      const bool on = i < q.ncand && (t.pos >> 60) == tag;
      const uint64_t bal = __ballot(on);
      const uint64_t my = rank + sw_rank(bal, lane);
      rank += (uint64_t)__builtin_popcountll(bal);
      if (!on) continue;
      const uint64_t s = t.pos & 0xFFFFFFFFFFull;
      const uint64_t sz = ((t.pos >> 40) & 0x3Fu) + (uint64_t)t.k_size + t.v_size;
      if (!sw_verify(p, st + 2048, st, st + 1024, s, sz)) atomicMin((unsigned long long*)&c->fail, (unsigned long long)my);
      const uint64_t k = ks + my;
      if (k < p.cap) {
        if (p.kind == LDB_TUPLE_ENTRY) decode_entry_global(p, s, reinterpret_cast<ldb_entry*>(p.out) + k);
        else store_tuple(reinterpret_cast<ldb_index_tuple*>(p.out) + k, t.pos & kSwPosMask, t.k_size, t.v_size);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_last = atomicAdd((unsigned long long*)&c->done1, 1ull) == (unsigned long long)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last || threadIdx.x >= 64) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sw_finish(p);
}
