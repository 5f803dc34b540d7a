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

// enter: kForceSpec (speculate), kForceNone (region covered by an earlier entry), or the
// region-relative position where the verified chain enters this region.
// emit(slot, pos, k, v): tuple `slot` (0-based within the region) in file order.
template <class WP, class Emit>
LDB_HD void region_process(WP& wp, const View& v, WaveSh& sh, uint32_t enter, RegionSum* out, Emit emit) {
  int lt = -1;
  if (enter != kForceSpec && enter != kForceNone) lt = enter < v.rlen ? (int)(enter / kS) : kLanes;
  wp.each([&](int l) {
    uint32_t f;
    if (enter == kForceSpec) f = kForceSpec;
    else if (enter == kForceNone) f = kForceNone;
    else f = l < lt ? kForceNone : (l == lt ? enter : kForceSpec);
    sh.force[l] = f;
  });
  uint64_t todo = ~0ull;
  int iter = 0;
  bool overflow = false;
  for (;;) {
    wp.each([&](int l) {
      if ((todo >> l) & 1) lane_process(v, l, sh.force[l], &sh.ln[l]);
    });
    const uint64_t none = wp.ballot([&](int l) { return sh.ln[l].s == kNone32; });
    // entering violations: lanes before the entry lane must be covered, the entry lane must start at `enter`
    int fixl = -1;
    uint32_t fixf = 0;
    if (enter != kForceSpec) {
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
  // verify entries that cross slices but end inside the region
  {
    const int tl = wp.first([&](int l) { return sh.ln[l].s != kNone32 && sh.ln[l].term != kCont; });
    const int lim = tl < 0 ? kLanes - 1 : tl;
    wp.each([&](int l) {
      LaneState& a = sh.ln[l];
      if (l <= lim && a.s != kNone32 && a.term == kCont && (a.sflag & kStraddle) && a.x - v.R0 < (uint64_t)kW) {
        if (!fold_verify(v, sh, l)) {
          a.term = LDB_ERR_CRC;
          a.tpos = a.so;
          a.cnt -= 1;
          a.sflag = 0;
        }
      }
    });
  }
  const int tl = wp.first([&](int l) { return sh.ln[l].s != kNone32 && sh.ln[l].term != kCont; });
  const int lim = tl < 0 ? kLanes - 1 : tl;
  const int L0 = wp.first([&](int l) { return sh.ln[l].s != kNone32; });
  const int lz = wp.last([&](int l) { return l <= lim && sh.ln[l].s != kNone32; });
  wp.excl_prefix([&](int l) { return (l <= lim && sh.ln[l].s != kNone32) ? sh.ln[l].cnt : 0u; }, sh.prefix);
  const uint32_t total = wp.sum([&](int l) { return (l <= lim && sh.ln[l].s != kNone32) ? sh.ln[l].cnt : 0u; });
  wp.single([&] {
    RegionSum r;
    r.soff = 0; r.rout = 0; r.scrc = 0; r.sflag = 0; r.count = total; r.exitp = 0;
    if (L0 < 0) {
      r.start = kNone64;
      r.status = kCont;
      r.rpre = fold_prefix(v, sh, (int64_t)v.rlen);
    } else {
      r.start = v.R0 + sh.ln[L0].s;
      r.rpre = fold_prefix(v, sh, (int64_t)sh.ln[L0].s);
      if (tl >= 0) {
        r.status = sh.ln[tl].term;
        r.exitp = v.R0 + sh.ln[tl].tpos;
      } else {
        const LaneState& z = sh.ln[lz];
        r.status = kCont;
        r.exitp = z.x;
        if ((z.sflag & kStraddle) && z.x - v.R0 >= (uint64_t)kW) {
          uint32_t fl = 0;
          r.rout = fold_out(v, sh, lz, &fl);
          r.sflag = fl;
          r.soff = v.R0 + z.so;
          r.scrc = z.scrc;
        }
      }
    }
    if (overflow || total > (uint32_t)kRegionCap) r.status = kOverflow;
    *out = r;
  });
  if (!overflow && total <= (uint32_t)kRegionCap) {
    wp.each([&](int l) {
      const LaneState& a = sh.ln[l];
      if (l <= lim && a.s != kNone32 && a.cnt) {
        const uint32_t base = sh.prefix[l];
        lane_emit(v, a, [&](uint32_t i, uint64_t pos, uint32_t k, uint32_t vv) { emit(base + i, pos, k, vv); });
      }
    });
  }
}

}  // namespace ldb
