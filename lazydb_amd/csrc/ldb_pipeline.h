// ldb_pipeline.h — cross-region stitching of the per-region summaries (host+device).
//
// After every region ran region_process speculatively, the chain of
// ReadLogEntry positions (index.go:84-95) is verified region to region:
//   link    : a region's exit must be the start of the region it lands in, and every region it
//             jumps over must contain no entry start of its own;
//   repair  : walk the true chain from the first broken link, re-running regions with the
//             entering position forced, until it merges back into a verified region;
//   combine : entries that cross region boundaries are CRC-verified by folding the regions'
//             raw pieces with GF(2) shifts;
//   final   : the scan stops at the first terminal along the chain; tuples before it are kept.
#pragma once

#include "ldb_chain.h"

namespace ldb {

struct SwRun;
struct SwCtl;

struct Pipe {
  const uint8_t* img;
  uint64_t len;
  int io;
  uint32_t fid;
  uint64_t nreg;
  const uint32_t* gtab;     // kTabWords table block (global copy)
  const uint32_t* xw;       // x^(8n) mod P for n = 0..kW
  const uint32_t* gsh;      // kGsTables x 1024 register-shift byte tables (build_gshift)
  RegionSum* rs;             // per-region summaries (48-B records)
  ldb_index_tuple* scratch;   // nreg * kRegionCap
  // control
  int64_t* fail_src;          // regions whose outgoing link failed (-1: region 0 does not start at 0)
  uint32_t* ctr;              // [0] fail count, [1] overflow, [2] repairs, [3] fast regions, [4] unused
  uint64_t* tpos;             // [0] min terminal position, [1] its status (packed with position)
  uint64_t* blk;              // per kBlkRegions-region block: count sum (k_combine)
  uint64_t* dyn;              // [0] K: entries of the equal-sized run k_uniform verified, [1] their size,
                              // [2] kUniReady once a k_uniform launch published its setup to `uni`,
                              // [3] kUniDone once the run prefix ended the scan (uni_finish), [4] its counter,
                              // [5] x0 (uni_finish) or ~0
  uint8_t* uni;               // the run prefix's published setup (memo, slicing, combine tables)
  uint64_t* hash_out;         // merge mode (nullable): ldb::key_hash_w of the key of run entry k at [k]
  void* out;
  uint64_t cap;
  int kind;
  uint32_t epoch;             // this scan's number on its workspace (k_uniform's run-list word carries it)
  ldb_scan_result* result;
  // the sweep tier (ldb_sweep.h; null where it does not run): per-window and per-group raw registers,
  // its run records and control block, its global tables; its candidate slabs are the scratch tuples
  uint32_t* swrw;
  uint32_t* swrg;
  uint32_t* swpl;
  SwRun* swrun;
  SwCtl* swctl;
  const uint32_t* swt;
  uint64_t scratch_bytes;
  // k_sweep and k_region (ldb_scan.hip): their control words (tickets, items done, published phases, phase stamps; 256 B,
  // zeroed where the pipeline starts), the per-phase time accumulators (null unless ldb_kernel_timing is
  // on) and whether the sweep tier runs
  uint32_t* tail;
  uint64_t* tacc;
  uint32_t sweep;
};

constexpr uint32_t kTailCtlBytes = 256;   // Pipe::tail
constexpr int kBlkRegions = 1024;   // regions per block of the count prefix (k_region phases C and K: one thread each)

// ---------------------------------------------------------------- the run prefix (k_uniform)
// k_uniform verifies, in parallel, that the log starts with K entries that all have entry 0's header
// bytes (so its size sz) and a correct CRC: the chain's first K entries are at k * sz. The region
// pipeline then replays only from x0 = K * sz on, as if the file started there: it skips every
// region before x0's region, takes x0 as the chain's entry point (where it used to take offset 0),
// and emits its tuples after the K the run wrote. K = 0 (no run) is the plain pipeline.
LDB_HD uint64_t run_k(const Pipe& p) { return p.dyn[0] == ~0ull ? 0ull : p.dyn[0]; }
// dyn[5]: x0 as the run prefix's last workgroup computed it over its runs (a log of several runs of
// equal-sized entries, k_uniform uni_finish); ~0 where no such finish ran (a batched scan: one run, x0 =
// K sz)
LDB_HD uint64_t chain_x0(const Pipe& p) { return p.dyn[5] != ~0ull ? p.dyn[5] : run_k(p) * p.dyn[1]; }
// first region of the replay; nreg when the header window at x0 is already unreadable (the replay
// stops there with io.EOF, log_file.go:117-122, and no region has work)
LDB_HD uint64_t first_region(const Pipe& p) {
  const uint64_t x0 = chain_x0(p);
  if (x0 && read_eof(p.len, p.io, (int64_t)x0, kMaxHeader)) return p.nreg;
  const uint64_t r = x0 / kW;
  return r < p.nreg ? r : p.nreg;
}

// Register-shift byte tables for k_combine (global memory, L2-resident): table t holds
// T[q * 256 + b] = shift(b << 8q, n_t bytes) = (b << 8q) * x^(8 n_t) mod P, so a shift by n_t is
// 4 independent lookups instead of a 32-step GF(2) multiply.
//   t = kGsW            : n = kW           (a whole covered region)
//   t = kGsE0 + k - 1   : n = kS * k       (k = 1..64: to the end of the landing slice)
//   t = kGsD + d        : n = d            (d = 0..kS)
//   t = kGsU + d        : n = -d           (d = 0..3: inverse shifts, CRC spans starting past a region end)
constexpr int kGsW = 0, kGsE0 = 1, kGsD = kGsE0 + kLanes, kGsU = kGsD + kS + 1, kGsTables = kGsU + 4;
constexpr uint64_t kGsWords = (uint64_t)kGsTables * 1024;

inline void build_gshift(uint32_t* g) {
  auto fill = [&](int t, uint64_t n) {
    const uint32_t xn = x8n_modp(n);
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) g[(uint64_t)t * 1024 + q * 256 + b] = multmodp(xn, b << (8 * q));
  };
  fill(kGsW, kW);
  for (int k = 1; k <= kLanes; ++k) fill(kGsE0 + k - 1, (uint64_t)kS * k);
  for (int d = 0; d <= kS; ++d) fill(kGsD + d, d);
  // inverse shifts: invert the 32x32 GF(2) matrix of "shift by d bytes" (Gauss-Jordan)
  for (int d = 0; d < 4; ++d) {
    const uint32_t xn = x8n_modp((uint64_t)d);
    uint32_t m[32], inv[32];   // m[j] = image of basis vector j; row-reduce [m | I] column-wise
    for (int j = 0; j < 32; ++j) { m[j] = multmodp(xn, 1u << j); inv[j] = 1u << j; }
    for (int bit = 0; bit < 32; ++bit) {   // make m[bit] the only vector with `bit` set
      int piv = bit;
      while (!((m[piv] >> bit) & 1u)) ++piv;
      uint32_t t = m[piv]; m[piv] = m[bit]; m[bit] = t;
      t = inv[piv]; inv[piv] = inv[bit]; inv[bit] = t;
      for (int j = 0; j < 32; ++j)
        if (j != bit && ((m[j] >> bit) & 1u)) { m[j] ^= m[bit]; inv[j] ^= inv[bit]; }
    }
    // now m[j] = e_j and inv[j] = S^-1(e_j)
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) {
        uint32_t x = b << (8 * q), y = 0;
        for (int j = 0; j < 32; ++j)
          if ((x >> j) & 1u) y ^= inv[j];
        g[(uint64_t)(kGsU + d) * 1024 + q * 256 + b] = y;
      }
  }
}

LDB_HD uint32_t gshift(const uint32_t* g, int t, uint32_t r) {
  const uint32_t* T = g + (uint64_t)t * 1024;
  return T[r & 0xFFu] ^ T[256 + ((r >> 8) & 0xFFu)] ^ T[512 + ((r >> 16) & 0xFFu)] ^ T[768 + (r >> 24)];
}

LDB_HD void store_region(const Pipe& p, uint64_t r, const RegionSum& s) { p.rs[r] = s; }

LDB_HD uint32_t region_len(const Pipe& p, uint64_t r) {
  const uint64_t R0 = r * (uint64_t)kW;
  return (uint32_t)((p.len - R0) < (uint64_t)kW ? (p.len - R0) : (uint64_t)kW);
}

// The run's template: entry 0's header, decoded exactly as decodeHeader does (classify_entry,
// log_entry.go:81-107 / log_file.go:116-139). An entry whose header bytes [4, hs) equal these decodes
// to the same fields (every varint of a canonical header ends inside [5, hs)), so it has the same size.
struct UniMemo {
  uint32_t ok;          // entry 0 is a canonical, readable, non-sentinel entry with a CRC span
  uint32_t hs, enc, stat, tx_stat, k, v;
  uint32_t nw;          // header dwords compared (bytes [4, 4 + 4 nw) cover [4, hs))
  int64_t expired_at;
  uint64_t tx_id;
  uint64_t sz;          // entry size hs + k + v
  uint32_t w[9], msk[9];   // header bytes [4, 40) and the mask of those before hs
};

// k_uniform's slicing of a run member's CRC span [x + 4, x + sz), L = sz - 4 bytes: G lanes per entry
// (a power of 2), lane j CRC-32s the P-byte window [x + 4 - t + j P, + P) from register 0 in S = P / 8
// table steps, where t = G P - L. The windows tile [x + 4 - t, x + sz); every byte before the span
// start is masked to zero (lane j masks its first min(P, max(0, t - j P)) bytes), and leading zeros
// leave a zero register unchanged, so each lane holds the raw register of its piece of the span and a
// tree combine over the group shifts by d P bytes at level d. The span's register from ~0 is then the
// combined raw register ^ KL, KL = shift(~0, L). G is the smallest that keeps P <= 8 kUniSteps (a
// lane's bytes stay in registers): fewer, longer windows amortise a batch's fixed cost best.
constexpr int kUniSteps = 12;                            // 8-byte steps per lane at most
constexpr int kUniLevels = 6;                            // combine levels (G <= 64)
constexpr uint64_t kUniMaxSize = 4 + 64ull * 8 * kUniSteps;   // larger entries never form a run
// the smallest entry a run may have: a 10-byte header (crc, stat, five one-byte varints) and no key or
// value (round 3: 16, so logs of 11-B entries -- adversarial "tiny" -- went through the region pipeline)
constexpr uint64_t kUniMinSize = 10;
static_assert(kUniMaxSize - 4 < 2ull * kW && 8ull * kUniSteps << (kUniLevels - 1) <= (uint64_t)kW,
              "uni_geometry reads its shifts from the x^(8n) table");

struct UniGeo {
  uint32_t ok, G, lg, P, S, t, KL, pad;
};

// xw[n] = x^(8n) mod P for n = 0..kW (the pipeline's table); L < 2 kW
LDB_HD UniGeo uni_geometry(const uint32_t* xw, uint32_t L) {
  UniGeo g{};
  for (uint32_t lg = 0; lg < kUniLevels + 1; ++lg) {
    const uint32_t G = 1u << lg;
    const uint32_t P = ((L + G - 1) / G + 7) & ~7u;
    if (P <= 8 * kUniSteps) {
      g.ok = 1; g.G = G; g.lg = lg; g.P = P; g.S = P / 8; g.t = G * P - L;
      const uint32_t xl = L <= (uint32_t)kW ? xw[L] : multmodp(xw[kW], xw[L - kW]);
      g.KL = multmodp(xl, 0xFFFFFFFFu);
      return g;
    }
  }
  return g;
}

// bytes lane j of a group masks at its window's start
LDB_HD uint32_t uni_lead(const UniGeo& g, uint32_t j) {
  const uint32_t o = j * g.P;
  return g.t > o ? (g.t - o < g.P ? g.t - o : g.P) : 0u;
}

// fetch(i) = image byte off + i (i in [0, 38)); off = the entry's image offset (the IOController bounds)
template <class Fetch>
LDB_HD UniMemo uni_memo(Fetch fetch, uint64_t len, int io, uint64_t off = 0) {
  UniMemo m;
  m.ok = 0;
  const EntryInfo e = classify_entry(fetch, len, io, off);
  if (e.status != kCont || !e.h.canonical || e.h.size < 10 || e.h.size > kMaxHeader) return m;
  if (e.size > kUniMaxSize || e.size < kUniMinSize) return m;
  m.hs = (uint32_t)e.h.size;
  m.enc = (uint32_t)e.h.enc_size;
  m.stat = e.h.stat;
  m.tx_stat = e.h.tx_stat;
  m.k = e.h.k_size;
  m.v = e.h.v_size;
  m.expired_at = e.h.expired_at;
  m.tx_id = e.h.tx_id;
  m.sz = e.size;
  m.nw = (m.hs - 4 + 3) / 4;
  for (int i = 0; i < 9; ++i) {
    const int n = (int)m.hs - 4 - 4 * i;
    m.msk[i] = n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * n)));
    uint32_t w = 0;
    for (int b = 0; b < 4; ++b) w |= (4 + 4 * i + b < kMaxHeader ? fetch(4 + 4 * i + b) : 0u) << (8 * b);
    m.w[i] = w & m.msk[i];
  }
  m.ok = 1;
  return m;
}

// ReadLogEntry(x) of a run member up to the CRC: the header window and key/value are readable
// (log_file.go:117-122, 130-139), the header bytes equal the template's and the entry is not the
// zero sentinel (:124-126). word(i) = little-endian dword at x + 4 i (i = 0: the stored crc).
template <class Word>
LDB_HD bool uni_header_ok(const UniMemo& m, Word word, uint64_t x, uint64_t len, int io) {
  if (read_eof(len, io, (int64_t)x, kMaxHeader)) return false;
  if (m.k || m.v) {
    if (read_eof(len, io, (int64_t)(x + m.hs), (uint64_t)m.k + m.v)) return false;
  } else if (word(0) == 0u) {
    return false;   // crc == 0 && kSize == 0 && vSize == 0: ErrLogEndOfFile
  }
  uint32_t d = 0;
  for (uint32_t i = 0; i < m.nw; ++i) d |= (word(1 + i) ^ m.w[i]) & m.msk[i];
  return d == 0u;
}

LDB_HD uint64_t uni_pos(const UniMemo& m, uint64_t x) {
  return (x & 0xFFFFFFFFFFull) | ((uint64_t)(m.hs & 0x3F) << 40) | ((uint64_t)(m.enc & 0x3F) << 46) |
         ((uint64_t)(m.stat & 0xFF) << 52);
}

// Link check of region r. Returns true when r's outgoing link is broken (or the first region does not
// start at the chain's entry point x0, reported by the caller as the virtual source first_region - 1).
LDB_HD bool link_broken(const Pipe& p, uint64_t r) {
  if (p.rs[r].start == kNone64 || p.rs[r].status != kCont) return false;
  const uint64_t x = p.rs[r].exitp;
  if (x >= p.len) return false;  // chain ends exactly at the file end (tail terminal)
  const uint64_t m = x / kW;
  for (uint64_t k = r + 1; k < m; ++k)
    if (p.rs[k].start != kNone64) return true;
  return p.rs[m].start != x;
}

// ---------------------------------------------------------------- CRC helpers (global memory)
// CRC-32 register over image bytes [a, b) from register `reg` (byte at a time; rare paths only).
LDB_HD uint32_t g_crc_bytes(const Pipe& p, uint32_t reg, uint64_t a, uint64_t b) {
  const uint32_t* t8 = p.gtab + kT8Off;
  for (uint64_t i = a; i < b; ++i) reg = crc_byte(t8, reg, p.img[i]);
  return reg;
}

// Verify the straddle-out entry of region r (its CRC span crosses into later regions).
// Returns true when it matches its stored crc.
LDB_HD bool combine_region(const Pipe& p, uint64_t r) {
  const uint32_t fl = p.rs[r].sflag;
  if (fl & kNoCrc) return true;
  {
    // the region the entry ends in verified it in-wave (kOwnerOk, ldb_chain.h)
    const uint64_t x = p.rs[r].exitp, m = x / kW;
    if (m < p.nreg && (p.rs[m].sflag & kOwnerOk) && p.rs[m].start == x) return true;
  }
  const uint64_t o = p.rs[r].soff;
  const uint64_t end = p.rs[r].exitp;
  const uint64_t lo = o + 4;
  uint32_t reg;
  uint64_t k;
  if (fl & kSkip) {
    // the span starts d = lo - R1 in [0, 3] bytes into region r+1 (lane_walk: o + 4 >= region end).
    // Use the virtual register V at R1 for which the usual fold is exact:
    //   shift(V, d) ^ raw(bytes [R1, lo)) = ~0   ->   V = shift^-1(~0 ^ raw_d, d)
    const uint64_t R1 = (r + 1) * (uint64_t)kW;
    const int d = (int)(lo - R1);
    uint32_t raw_d = 0;
    for (int i = 0; i < d; ++i) raw_d = crc_byte(p.gtab + kT8Off, raw_d, p.img[R1 + i]);
    reg = gshift(p.gsh, kGsU + d, 0xFFFFFFFFu ^ raw_d);
  } else {
    reg = p.rs[r].rout;
  }
  k = r + 1;
  const uint64_t m = end / kW;  // region holding the entry's end (may be == nreg when end == len)
  for (; k < m; ++k) reg = gshift(p.gsh, kGsW, reg) ^ p.rs[k].rpre;
  const uint32_t want = ~p.rs[r].scrc;
  if (m < p.nreg) {
    const uint64_t n = end - m * (uint64_t)kW;
    if (n) {
      if (p.rs[m].start == kNone64) {
        reg = multmodp(p.xw[n], reg) ^ p.rs[m].rpre;   // region covered up to the end of the file
      } else {
        // rpre[m] = shift(raw([R0, n)), E0 - n), E0 = end of the slice holding n (region_process):
        // reg(n) == want  <=>  shift(reg, E0) ^ rpre[m] == shift(want, E0 - n)
        const int k0 = (int)(n / kS) + 1;   // E0 = kS * k0
        const int d = kS * k0 - (int)n;     // 1..kS
        return (gshift(p.gsh, kGsE0 + k0 - 1, reg) ^ p.rs[m].rpre) == gshift(p.gsh, kGsD + d, want);
      }
    }
  }
  return reg == want;
}

LDB_HD uint64_t pack_term(uint64_t pos, int32_t status) {
  // smallest position wins; status in the low 4 bits (statuses -2..3 -> 0..5)
  return (pos << 4) | (uint64_t)(status + 2);
}
LDB_HD uint64_t term_pos(uint64_t t) { return t >> 4; }
LDB_HD int32_t term_status(uint64_t t) { return (int32_t)(t & 15) - 2; }

}  // namespace ldb

namespace ldb {

// Link failures and walker claims share the workspace block of p.fail_src (8 (nreg + 1) bytes):
//   fail flags  uint8_t[nreg + 1]: flag i <-> source rf - 1 + i (source rf - 1: region rf does not
//               start at the chain's entry point x0; source r >= rf: region r's outgoing link is broken).
//               k_link writes every flag of the pipeline, so nothing is cleared between scans.
//   claims      uint32_t[nreg] after them: a region one optimistic walker re-runs (k_link zeroes them).
LDB_HD uint8_t* fail_flags(const Pipe& p) { return reinterpret_cast<uint8_t*>(p.fail_src); }
LDB_HD uint32_t* repair_claims(const Pipe& p) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(p.fail_src) + ((p.nreg + 1 + 15) & ~15ull));
}
LDB_HD uint64_t n_fail_flags(const Pipe& p) { return p.nreg - first_region(p) + 1; }
// k_repair's serial pass reads two bitmaps over the claims (which only its walkers use): flag bits
// (bit i <-> fail flag i) and terminal bits (bit r <-> region r stopped on a terminal status with a
// start: a superset once the serial pass re-runs regions, each hit re-checked live). One wave then
// finds the next flagged source or terminal region 4096 at a time instead of 64 (1 GiB writer mix:
// 209 716 regions, 8.6 ms of k_repair in dependent 64-flag loads before).
LDB_HD uint64_t* flag_bits(const Pipe& p) { return reinterpret_cast<uint64_t*>(repair_claims(p)); }
LDB_HD uint64_t* term_bits(const Pipe& p) { return flag_bits(p) + (p.nreg + 1 + 63) / 64; }

// Repair walk. Wave-uniform control flow: every lane of the one repairing
// wavefront evaluates the same loads. `next_fail(done)` returns the smallest flagged source > done
// (INT64_MAX: none), `rd` reads summaries coherently, `first_term(lo, hi)` returns the first region
// in (lo, hi] whose (verified) walk stopped with a terminal status or -1, and `run(r, enter)`
// re-processes region r with its entering position forced and returns its new summary.
// Correct for ANY set of region summaries, each a valid processing of its region from its own start,
// provided the flags name every region whose outgoing link is broken. Returns the regions re-processed.
template <class NextFail, class Rd, class FirstTerm, class Run>
LDB_HD uint32_t repair(const Pipe& p, NextFail next_fail, Rd rd, FirstTerm first_term, Run run) {
  const int64_t rf = (int64_t)first_region(p);   // source rf - 1: the chain's entry point x0
  int64_t done = rf - 2;
  uint32_t repairs = 0;
  for (;;) {
    const int64_t src = next_fail(done);
    if (src == INT64_MAX) break;
    if (first_term(done, src) >= 0) break;  // a verified region before src already ends the scan
    uint64_t x = src < rf ? chain_x0(p) : rd.exitp((uint64_t)src);
    int64_t cur = src;
    bool stop = false;
    for (;;) {
      if (x >= p.len) { stop = true; break; }
      const uint64_t m = x / kW;
      for (int64_t k = cur + 1; k < (int64_t)m; ++k) {
        if (rd.start((uint64_t)k) != kNone64) { run((uint64_t)k, kForceNone); ++repairs; }
      }
      if (rd.start(m) == x) {
        // Merged into a region whose first start is x. If that region verified its owner in-wave
        // (kOwnerOk, ldb_chain.h), it checked the entry ending at x on ITS run's chain, which need
        // not be the entry the true chain ends there with: re-run it so k_combine checks the owner.
        if (rd.sflag(m) & kOwnerOk) { run(m, (uint32_t)(x - m * kW)); ++repairs; }
        done = (int64_t)m - 1;
        break;
      }
      const RegionSum s = run(m, (uint32_t)(x - m * (uint64_t)kW));
      ++repairs;
      if (s.status != kCont) { stop = true; break; }
      cur = (int64_t)m;
      x = s.exitp;
    }
    if (stop) break;
  }
  return repairs;
}

// One optimistic walker (k_repair, first phase): assume source src lies on the true chain and
// re-run the regions its exit leads through, as repair() would, until the walk merges into a region
// that already starts there, ends, meets a region another walker claimed, or has taken kWalkMax
// steps. Every region it writes is claimed first (`claim(r)`: true for the one walker that gets r), so
// walkers never write the same region; what they read may be stale or another walker's, which is
// harmless: each region they write is a valid processing from its new start, and the links are
// checked again over all regions before the serial repair() runs (its precondition above).
constexpr int kWalkMax = 256;
struct NoLink {
  LDB_HD bool operator()(uint64_t) const { return false; }
};
// `hold_covered(k)`: leave region k alone rather than re-run it as covered by the walk's entry
// (see k_repair); `hold_landing(m)`: stop before re-running the landing region m
template <class Rd, class Claim, class Run, class HoldC = NoLink, class HoldL = NoLink>
LDB_HD uint32_t walk_source(const Pipe& p, int64_t src, Rd rd, Claim claim, Run run, HoldC hold_covered = HoldC{},
                            HoldL hold_landing = HoldL{}) {
  const int64_t rf = (int64_t)first_region(p);
  uint64_t x = src < rf ? chain_x0(p) : rd.exitp((uint64_t)src);
  int64_t cur = src;
  uint32_t runs = 0;
  for (int step = 0; step < kWalkMax; ++step) {
    if (x >= p.len) break;
    const uint64_t m = x / kW;
    bool stop = false;
    for (int64_t k = cur + 1; k < (int64_t)m && !stop; ++k) {
      if (rd.start((uint64_t)k) != kNone64) {
        if (hold_covered((uint64_t)k) || !claim((uint64_t)k)) stop = true;
        else { run((uint64_t)k, kForceNone); ++runs; }
      }
    }
    if (stop || rd.start(m) == x || hold_landing(m) || !claim(m)) break;   // merged: the serial pass sees to a kOwnerOk landing
    const RegionSum s = run(m, (uint32_t)(x - m * (uint64_t)kW));
    ++runs;
    if (s.status != kCont) break;
    cur = (int64_t)m;
    x = s.exitp;
  }
  return runs;
}

}  // namespace ldb

#include "ldb_sweep.h"
