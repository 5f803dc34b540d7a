// ldb_wave.h — the per-region routine (one wavefront = one region of kW bytes), written
// against a small "wave policy" so the same code runs as 64 SIMT lanes on gfx950
// (GpuWave, ldb_scan.hip) and as a 64-iteration loop in the CPU emulator (tests/emu).
#pragma once

#include "ldb_engine.h"

namespace ldb {

// Region-level result (mirrors the SoA summary arrays of ldb_scan.hip).
struct RegionSum {
  uint64_t start;    // absolute first entry start in the region, or kNone64 (covered region)
  uint64_t exitp;    // status == kCont: absolute offset after the region's last entry; else terminal offset
  uint64_t soff;     // straddle-out entry start (absolute)
  int32_t status;    // kCont / LDB_EOF_* / LDB_ERR_CRC / LDB_ERR_MALFORMED / kOverflow
  uint32_t count;    // accepted entries starting in the region (incl. a pending straddler)
  uint32_t rpre;     // raw CRC register over [R0, start) (whole region piece when start == kNone64)
  uint32_t rout;     // straddler's CRC register at the region end (init-based)
  uint32_t scrc;     // straddler's stored crc
  uint32_t sflag;    // kStraddle | kSkip | kNoCrc
};

constexpr uint32_t kNoOwner = 0xFFFFFFFFu;
constexpr uint32_t kDone = 0xFFFFFFFEu;

// Carry register `reg` (valid at region-relative position k0 * kS) across the covered slices
// k0, k0+1, ... whose whole bytes belong to the same entry, up to position `X` rounded down to a
// slice boundary. Returns the register at that boundary; *kend = X / kS (the first lane not
// absorbed). Constant-distance shifts only (shift_slice).
LDB_HD uint32_t carry_full(const View& v, const WaveSh& sh, uint32_t reg, int k0, int64_t X, int* kend) {
  int k = k0;
  for (; k < kLanes && (int64_t)(k + 1) * kS <= X; ++k) reg = shift_slice(v.tab, reg) ^ sh.ln[k].raw;
  *kend = k;
  return reg;
}

// Register after a covered lane's partial raw piece [k*kS, X) at the end of the file (rare).
LDB_HD uint32_t carry_tail(const View& v, const WaveSh& sh, uint32_t reg, int k, int64_t X) {
  const int64_t n = X - (int64_t)k * kS;
  if (n <= 0 || k >= kLanes) return reg;
  return multmodp(v.xw[n], reg) ^ sh.ln[k].raw;
}

// enter: kForceSpec (speculate), kForceNone (region covered by an earlier entry), or the
// region-relative position where the verified chain enters this region.
// keep(l): lane l's private LaneKeep (a register struct on the GPU).
// emit(slot, pos, k, v): tuple `slot` (0-based within the region) in file order.
template <class WP, class Keep, class Emit>
LDB_HD void region_process(WP& wp, const View& v, WaveSh& sh, uint32_t enter, RegionSum* out, Keep keep,
                           Emit emit) {
  int lt = -1;
  if (enter != kForceSpec && enter != kForceNone) lt = enter < v.rlen ? (int)(enter / kS) : kLanes;
  wp.each([&](int l) {
    uint32_t f;
    if (enter == kForceSpec) f = kForceSpec;
    else if (enter == kForceNone) f = kForceNone;
    else f = l < lt ? kForceNone : (l == lt ? enter : kForceSpec);
    sh.force[l] = f;
  });
  wp.stamp(0);
  // ---- speculative lane walks + link verification / repair
  uint64_t todo = ~0ull;
  int iter = 0;
  bool overflow = false;
  for (;;) {
    wp.each([&](int l) {
      if ((todo >> l) & 1) lane_process(v, l, sh.force[l], &sh.ln[l], &keep(l));
    });
    wp.stamp(iter == 0 ? 1 : 2);
    const uint64_t none = wp.ballot([&](int l) { return sh.ln[l].s == kNone32; });
    int fixl = -1;
    uint32_t fixf = 0;
    if (enter != kForceSpec) {  // lanes before the entry lane covered, entry lane starts at `enter`
      const int e = wp.first([&](int l) {
        if (enter == kForceNone || l < lt) return sh.ln[l].s != kNone32;
        return l == lt && sh.ln[l].s != enter;
      });
      if (e >= 0) {
        fixl = e;
        fixf = (enter == kForceNone || e < lt) ? kForceNone : enter;
      }
    }
    if (fixl < 0) {
      const int tl = wp.first([&](int l) { return sh.ln[l].s != kNone32 && sh.ln[l].term != kCont; });
      const int lim = tl < 0 ? kLanes - 1 : tl;
      const int j = wp.first([&](int l) {
        uint32_t f;
        return l <= lim && lane_link(v, sh, l, none, &f) >= 0;
      });
      if (j >= 0) {
        uint32_t f = 0;
        fixl = lane_link(v, sh, j, none, &f);
        fixf = f;
      }
    }
    if (fixl < 0) break;
    if (++iter > 4 * kLanes) { overflow = true; break; }
    wp.single([&] { sh.force[fixl] = fixf; });
    todo = 1ull << fixl;
  }
  wp.stamp(2);
  // ---- folds. F1: every entry that leaves its slice carries its CRC register across the
  // covered slices (constant 80-byte shifts) to the lane where it ends; the region's own prefix
  // is carried the same way from register 0. F2: that lane CRCs its prefix piece starting from
  // the carried register (no variable-distance shifts) and checks the entry's stored crc.
  int tl = wp.first([&](int l) { return sh.ln[l].s != kNone32 && sh.ln[l].term != kCont; });
  int lim = tl < 0 ? kLanes - 1 : tl;
  const int L0 = wp.first([&](int l) { return sh.ln[l].s != kNone32; });
  wp.each([&](int l) { sh.owner[l] = kNoOwner; });
  uint32_t region_rpre = 0, region_rout = 0, region_sflag_clear = 0;
  wp.each([&](int l) {
    // region entry chain (lane L0, or lane 0 for a covered region)
    if (l == (L0 < 0 ? 0 : L0)) {
      int kend;
      const int64_t X = L0 < 0 ? (int64_t)v.rlen : (int64_t)sh.ln[L0].s;
      uint32_t reg = carry_full(v, sh, 0u, 0, X, &kend);
      if (L0 < 0) {
        region_rpre = carry_tail(v, sh, reg, kend, X);
      } else {
        sh.inreg[L0] = reg;
        sh.owner[L0] = kLanes;
      }
    }
  });
  wp.each([&](int l) {
    LaneState& a = sh.ln[l];
    if (!(l <= lim && a.s != kNone32 && a.term == kCont && (a.sflag & kStraddle))) return;
    const int64_t xr = (int64_t)(a.x - v.R0);
    const int64_t X = xr < (int64_t)kW ? xr : (int64_t)kW;
    if (a.sflag & kNoCrc) {  // no CRC span: the landing lane has nothing to check
      const int m = (int)(X / kS);
      if (X < (int64_t)v.rlen && m < kLanes) sh.owner[m] = kDone;
      return;
    }
    uint32_t reg;
    int k0;
    if (a.sflag & kSkip) {   // span starts < 4 bytes before the slice end: first piece directly
      if (l == kLanes - 1) return;  // region-level skip: k_combine computes it from global memory
      const int64_t e1 = (int64_t)(l + 2) * kS;
      const int64_t hi = X < e1 ? X : e1;
      reg = crc_segment(v, (int64_t)a.so + 4, hi, 0xFFFFFFFFu);
      if (X <= e1) {
        const int m = (int)(X / kS);
        if (X < (int64_t)kW) {
          if (reg != ~a.scrc) { a.term = LDB_ERR_CRC; a.tpos = a.so; a.cnt -= 1; a.sflag = 0; }
          if (X < (int64_t)v.rlen && m < kLanes) sh.owner[m] = kDone;
          return;
        }
        region_rout = reg;   // reaches the region end
        region_sflag_clear = 1;
        return;
      }
      k0 = l + 2;
    } else {
      reg = a.rout;
      k0 = l + 1;
    }
    int kend;
    reg = carry_full(v, sh, reg, k0, X, &kend);
    if (X >= (int64_t)kW) {        // runs past the region: register at the region end
      region_rout = reg;
      region_sflag_clear = (a.sflag & kSkip) ? 1u : 0u;
      return;
    }
    if (X >= (int64_t)v.rlen) {    // ends exactly at the end of the file
      reg = carry_tail(v, sh, reg, kend, X);
      if (reg != ~a.scrc) { a.term = LDB_ERR_CRC; a.tpos = a.so; a.cnt -= 1; a.sflag = 0; }
      return;
    }
    sh.inreg[kend] = reg;          // lane kend starts at X: it finishes the entry (F2)
    sh.owner[kend] = (uint32_t)l;
  });
  wp.each([&](int l) {
    const uint32_t ow = sh.owner[l];
    if (ow == kNoOwner || ow == kDone || l > lim) return;
    const LaneState& a = sh.ln[l];
    const int64_t B = (int64_t)l * kS;
    const uint32_t reg = (int64_t)a.s > B ? crc_segment(v, B, (int64_t)a.s, sh.inreg[l]) : sh.inreg[l];
    if (ow == (uint32_t)kLanes) {
      region_rpre = reg;
    } else {
      LaneState& o = sh.ln[ow];
      if (reg != ~o.scrc) { o.term = LDB_ERR_CRC; o.tpos = o.so; o.cnt -= 1; o.sflag = 0; }
    }
  });
  region_rpre = wp.bcast_or(region_rpre);
  region_rout = wp.bcast_or(region_rout);
  region_sflag_clear = wp.bcast_or(region_sflag_clear);
  wp.stamp(3);
  tl = wp.first([&](int l) { return sh.ln[l].s != kNone32 && sh.ln[l].term != kCont; });
  lim = tl < 0 ? kLanes - 1 : tl;
  const int lz = wp.last([&](int l) { return l <= lim && sh.ln[l].s != kNone32; });
  wp.excl_prefix([&](int l) { return (l <= lim && sh.ln[l].s != kNone32) ? sh.ln[l].cnt : 0u; }, sh.prefix);
  const uint32_t total = wp.sum([&](int l) { return (l <= lim && sh.ln[l].s != kNone32) ? sh.ln[l].cnt : 0u; });
  wp.single([&] {
    RegionSum r;
    r.soff = 0; r.rout = 0; r.scrc = 0; r.sflag = 0; r.count = total; r.exitp = 0;
    r.rpre = region_rpre;
    if (L0 < 0) {
      r.start = kNone64;
      r.status = kCont;
    } else {
      r.start = v.R0 + sh.ln[L0].s;
      if (tl >= 0) {
        r.status = sh.ln[tl].term;
        r.exitp = v.R0 + sh.ln[tl].tpos;
      } else {
        const LaneState& z = sh.ln[lz];
        r.status = kCont;
        r.exitp = z.x;
        if ((z.sflag & kStraddle) && z.x - v.R0 >= (uint64_t)kW) {
          r.sflag = z.sflag;
          r.soff = v.R0 + z.so;
          r.scrc = z.scrc;
          if (z.sflag & kNoCrc) {
            r.rout = 0;
          } else if ((z.sflag & kSkip) && lz == kLanes - 1) {
            r.rout = 0;   // span starts at/after the region end - 3: k_combine computes it
          } else {
            r.rout = region_rout;
            if (region_sflag_clear) r.sflag = z.sflag & ~kSkip;
          }
        }
      }
    }
    if (overflow || total > (uint32_t)kRegionCap) r.status = kOverflow;
    *out = r;
  });
  wp.stamp(4);
  if (!overflow && total <= (uint32_t)kRegionCap) {
    wp.each([&](int l) {
      const LaneState& a = sh.ln[l];
      if (l <= lim && a.s != kNone32 && a.cnt) {
        const uint32_t base = sh.prefix[l];
        lane_emit(v, a, keep(l), [&](uint32_t i, uint64_t pos, uint32_t k, uint32_t vv) { emit(base + i, pos, k, vv); });
      }
    });
  }
  wp.stamp(5);
}

}  // namespace ldb
