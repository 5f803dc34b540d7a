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
  uint32_t* defer;            // regions k_scan_main left to k_fallback (region_process)
  uint32_t* ctr;              // [0] fail count, [1] overflow, [2] repairs, [3] fast regions, [4] deferred
  uint64_t* tpos;             // [0] min terminal position, [1] its status (packed with position)
  uint64_t* blk;              // per kBlkRegions-region block: count sum (k_combine)
  void* out;
  uint64_t cap;
  int kind;
  ldb_scan_result* result;
};

constexpr int kBlkRegions = 256;   // regions per k_combine / k_compact workgroup

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

// Link check of region r. Returns true when r's outgoing link is broken (or r == 0 does not
// start at offset 0, reported by the caller as source -1).
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

// Repair walk. Wave-uniform control flow: every lane of the one repairing
// wavefront evaluates the same loads. `rd` reads summaries coherently, `first_term(lo, hi)`
// returns the first region in (lo, hi] whose (verified) walk stopped with a terminal status
// or -1, and `run(r, enter)` re-processes region r with its entering position forced and
// returns its new summary.  Returns the number of regions re-processed.
template <class Rd, class FirstTerm, class Run>
LDB_HD uint32_t repair(const Pipe& p, uint32_t nfail, Rd rd, FirstTerm first_term, Run run) {
  int64_t done = -2;
  uint32_t repairs = 0;
  for (;;) {
    int64_t src = INT64_MAX;
    for (uint32_t i = 0; i < nfail; ++i) {
      const int64_t s = p.fail_src[i];
      if (s > done && s < src) src = s;
    }
    if (src == INT64_MAX) break;
    if (first_term(done, src) >= 0) break;  // a verified region before src already ends the scan
    uint64_t x = src < 0 ? 0 : rd.exitp((uint64_t)src);
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

}  // namespace ldb
