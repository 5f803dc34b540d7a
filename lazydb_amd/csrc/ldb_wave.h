// ldb_wave.h — the per-region routine (one wavefront = one region of kW bytes), written
// against a small "wave policy" so the same code runs as 64 SIMT lanes on gfx950
// (GpuWave, ldb_scan.hip) and as a 64-iteration loop in the CPU emulator (tests/emu).
#pragma once

#include "ldb_engine.h"

namespace ldb {

// Region-level result (mirrors the SoA summary arrays of ldb_scan.hip).
struct alignas(16) RegionSum {
  uint64_t start;    // absolute first entry start in the region, or kNone64 (covered region)
  uint64_t exitp;    // status == kCont: absolute offset after the region's last entry; else terminal offset
  uint64_t soff;     // straddle-out entry start (absolute)
  int32_t status;    // kCont / LDB_EOF_* / LDB_ERR_CRC / LDB_ERR_MALFORMED / kOverflow
  uint32_t count;    // accepted entries starting in the region (incl. a pending straddler)
  uint32_t rpre;     // start != kNone64: shift(raw([R0, start)), E0 - start), E0 = end of the start slice;
                     // covered region: raw register of the whole region
  uint32_t rout;     // straddler's CRC register at the region end (init-based)
  uint32_t scrc;     // straddler's stored crc
  uint32_t sflag;    // kStraddle | kSkip | kNoCrc
};
static_assert(sizeof(RegionSum) == 48, "RegionSum is stored as 12 dwords");

// Carry register `reg` (valid at region-relative position k0 * kS) across the covered slices
// k0, k0+1, ... whose whole bytes belong to the same entry, up to position `X` rounded down to a
// slice boundary. Returns the register at that boundary; *kend = X / kS (the first lane not
// absorbed). Constant-distance shifts only (shift_slice).
LDB_HD uint32_t carry_full(const View& v, const WaveSh& sh, uint32_t reg, int k0, int X, int* kend) {
  int k = k0;
  for (; k < kLanes && (k + 1) * kS <= X; ++k) reg = shift_slice(v.tab, reg) ^ sh.raw[k];
  *kend = k;
  return reg;
}

// Register after a covered lane's partial raw piece [k*kS, X) at the end of the file (rare).
LDB_HD uint32_t carry_tail(const View& v, const WaveSh& sh, uint32_t reg, int k, int X) {
  const int n = X - k * kS;
  if (n <= 0 || k >= kLanes) return reg;
  return multmodp(v.xw[n], reg) ^ sh.raw[k];
}

// enter: kForceSpec (speculate), kForceNone (region covered by an earlier entry), or the
// region-relative position where the verified chain enters this region.
// priv(l): lane l's private state (registers on the GPU).
// emit(slot, pos, k, v): tuple `slot` (0-based within the region) in file order.
// buffer_free(): called once every lane is done reading v.buf (before the summary is written).
template <class WP, class Priv, class Emit, class Free>
LDB_HD void region_process(WP& wp, const View& v, WaveSh& sh, uint32_t enter, RegionSum* out, Priv priv,
                           Emit emit, Free buffer_free) {
  int lt = -1;
  if (enter != kForceSpec && enter != kForceNone) lt = enter < v.rlen ? (int)(enter / kS) : kLanes;
  wp.each([&](int l) {
    uint32_t f;
    if (enter == kForceSpec) f = kForceSpec;
    else if (enter == kForceNone) f = kForceNone;
    else f = l < lt ? kForceNone : (l == lt ? enter : kForceSpec);
    priv(l).force = f;
  });
  wp.stamp(0);
  // ---- speculative lane walks + link verification / repair
  uint64_t todo = ~0ull;
  int iter = 0;
  bool overflow = false;
  for (;;) {
    wp.each([&](int l) {
      LanePriv& q = priv(l);
      if ((todo >> l) & 1) {
        lane_walk(v, l, q.force, &q.ln, &q.kp);
        sh.s[l] = q.ln.s;
      }
    });
    wp.stamp(iter == 0 ? 1 : 2);
    const uint64_t none = wp.ballot([&](int l) { return priv(l).ln.s == kNone32; });
    int fixl = -1;
    uint32_t fixf = 0;
    if (enter != kForceSpec) {  // lanes before the entry lane covered, entry lane starts at `enter`
      const int e = wp.first([&](int l) {
        const uint32_t s = priv(l).ln.s;
        if (enter == kForceNone || l < lt) return s != kNone32;
        return l == lt && s != enter;
      });
      if (e >= 0) {
        fixl = e;
        fixf = (enter == kForceNone || e < lt) ? kForceNone : enter;
      }
    }
    if (fixl < 0) {
      const int tl = wp.first([&](int l) { return priv(l).ln.s != kNone32 && priv(l).ln.term != kCont; });
      const int lim = tl < 0 ? kLanes - 1 : tl;
      const int j = wp.first([&](int l) {
        uint32_t f;
        return l <= lim && lane_link(v, sh, priv(l).ln, l, none, &f) >= 0;
      });
      if (j >= 0) {
        const uint64_t fx = wp.from64(j, [&](int l) {
          uint32_t f = 0;
          const int m = lane_link(v, sh, priv(l).ln, l, none, &f);
          return ((uint64_t)(uint32_t)m << 32) | f;
        });
        fixl = (int)(fx >> 32);
        fixf = (uint32_t)fx;
      }
    }
    if (fixl < 0) break;
    if (++iter > 4 * kLanes) { overflow = true; break; }
    wp.each([&](int l) { if (l == fixl) priv(l).force = fixf; });
    todo = 1ull << fixl;
  }
  wp.stamp(2);
  int tl = wp.first([&](int l) { return priv(l).ln.s != kNone32 && priv(l).ln.term != kCont; });
  int lim = tl < 0 ? kLanes - 1 : tl;
  const int L0 = wp.first([&](int l) { return priv(l).ln.s != kNone32; });
  const uint64_t starts = wp.ballot([&](int l) { return l <= lim && priv(l).ln.s != kNone32; });
  wp.each([&](int l) {
    const LaneState& a = priv(l).ln;
    sh.want[l] = ~a.scrc;
    sh.fl[l] = a.sflag;
  });
  // ---- CRC pieces: one uniform two-chain pass per lane. A start lane whose prefix belongs to an
  // entry started earlier in the region (its "owner") injects the owner's expected final register
  // at [s, s+4), so the owner's check at the fold becomes shift_slice(I_B) == raw (no variable shifts).
  wp.each([&](int l) {
    LaneState& a = priv(l).ln;
    uint32_t C = 0, inj = 0;
    const uint64_t below = starts & ((1ull << l) - 1);
    if (l <= lim && a.s != kNone32 && below) {
      const int j = 63 - (int)__builtin_clzll(below);
      const uint32_t ofl = sh.fl[j];
      const bool direct = (ofl & kSkip) && (int)a.s <= (j + 2) * kS;   // owner verified directly below
      if ((ofl & kStraddle) && !(ofl & kNoCrc) && !direct) { C = sh.want[j]; inj = 1; }
    }
    lane_crc(v, l, &a, C, inj);
    sh.raw[l] = a.raw;
  });
  wp.stamp(8);
  // ---- folds (one pass: the region prefix chain and every entry's chain run side by side)
  // The region prefix chain (raw register over [R0, start)) runs in the same carry loop as the
  // entries' chains, on a lane that owns no chain: L0 - 1 (covered), or lane 0 when no lane starts
  // an entry. With L0 == 0 the prefix is lane 0's own chain-A value.
  const int elane = L0 < 0 ? 0 : L0 - 1;
  wp.each([&](int l) {
    LanePriv& q = priv(l);
    LaneState& a = q.ln;
    q.rout_set = 0;
    uint32_t reg = 0;
    int k0 = 0, X = 0;
    const bool entry_role = l == elane;
    if (entry_role) {
      X = L0 < 0 ? (int)v.rlen : (int)sh.s[L0];
    } else {
      // every entry that leaves its slice carries its CRC register across the covered slices
      // (constant 80-byte shifts) to the lane where it ends and checks it there
      if (!(l <= lim && a.s != kNone32 && a.term == kCont && (a.sflag & kStraddle)) || (a.sflag & kNoCrc)) return;
      const uint64_t xr = a.x - v.R0;
      X = xr < (uint64_t)kW ? (int)xr : kW;
      if (a.sflag & kSkip) {   // span starts < 4 bytes before the slice end: first piece directly
        if (l == kLanes - 1) return;  // region-level skip: k_combine handles it
        const int e1 = (l + 2) * kS;
        const int hi = X < e1 ? X : e1;
        reg = crc_segment(v, (int)a.so + 4, hi, 0xFFFFFFFFu);
        if (X <= e1) {
          if (X < kW) {
            if (reg != ~a.scrc) { a.term = LDB_ERR_CRC; a.tpos = a.so; a.cnt -= 1; a.sflag = 0; }
            return;
          }
          q.rout = reg;   // reaches the region end
          q.rout_set = 2;
          return;
        }
        k0 = l + 2;
      } else {
        reg = a.rout;
        k0 = l + 1;
      }
    }
    int kend;
    reg = carry_full(v, sh, reg, k0, X, &kend);
    if (entry_role) {   // A-form prefix (see combine_region), or the raw register of a covered region
      q.rpre = L0 < 0 ? carry_tail(v, sh, reg, kend, X) : (shift_slice(v.tab, reg) ^ sh.raw[L0]);
      return;
    }
    if (X >= kW) {        // runs past the region: register at the region end
      q.rout = reg;
      q.rout_set = (a.sflag & kSkip) ? 2u : 1u;
      return;
    }
    bool ok;
    if (X >= (int)v.rlen) ok = carry_tail(v, sh, reg, kend, X) == ~a.scrc;   // ends exactly at the end of the file
    else ok = shift_slice(v.tab, reg) == sh.raw[kend];                       // lane kend starts at X, injected ~crc
    if (!ok) { a.term = LDB_ERR_CRC; a.tpos = a.so; a.cnt -= 1; a.sflag = 0; }
  });
  const uint32_t region_rpre = L0 == 0 ? sh.raw[0] : wp.from(elane, [&](int l) { return priv(l).rpre; });
  const int rsrc = wp.first([&](int l) { return priv(l).rout_set != 0; });
  const uint32_t region_rout = rsrc >= 0 ? wp.from(rsrc, [&](int l) { return priv(l).rout; }) : 0u;
  const uint32_t region_sflag_clear = rsrc >= 0 ? (wp.from(rsrc, [&](int l) { return priv(l).rout_set; }) == 2u) : 0u;
  wp.stamp(3);
  tl = wp.first([&](int l) { return priv(l).ln.s != kNone32 && priv(l).ln.term != kCont; });
  lim = tl < 0 ? kLanes - 1 : tl;
  const int lz = wp.last([&](int l) { return l <= lim && priv(l).ln.s != kNone32; });
  auto cnt_of = [&](int l) { return (l <= lim && priv(l).ln.s != kNone32) ? priv(l).ln.cnt : 0u; };
  wp.excl_prefix(cnt_of, [&](int l, uint32_t x) { priv(l).prefix = x; });
  const uint32_t total = wp.sum(cnt_of);
  if (!overflow && total <= (uint32_t)kRegionCap) {
    wp.each([&](int l) {
      const LanePriv& q = priv(l);
      if (l <= lim && q.ln.s != kNone32 && q.ln.cnt) {
        const uint32_t base = q.prefix;
        lane_emit(v, q.ln, q.kp, [&](uint32_t i, uint64_t pos, uint32_t k, uint32_t vv) { emit(base + i, pos, k, vv); });
      }
    });
  }
  wp.stamp(5);
  buffer_free();   // last read of the staging buffer is behind us: the caller may refill it
  // ---- region summary (wave-uniform values broadcast from the lanes that own them)
  RegionSum r;
  r.soff = 0; r.rout = 0; r.scrc = 0; r.sflag = 0; r.count = total; r.exitp = 0;
  r.rpre = region_rpre;
  if (L0 < 0) {
    r.start = kNone64;
    r.status = kCont;
  } else {
    r.start = v.R0 + wp.from(L0, [&](int l) { return priv(l).ln.s; });
    if (tl >= 0) {
      r.status = (int32_t)wp.from(tl, [&](int l) { return (uint32_t)priv(l).ln.term; });
      r.exitp = v.R0 + wp.from(tl, [&](int l) { return priv(l).ln.tpos; });
    } else {
      r.status = kCont;
      r.exitp = wp.from64(lz, [&](int l) { return priv(l).ln.x; });
      const uint32_t zf = wp.from(lz, [&](int l) { return priv(l).ln.sflag; });
      if ((zf & kStraddle) && r.exitp - v.R0 >= (uint64_t)kW) {
        r.sflag = zf;
        r.soff = v.R0 + wp.from(lz, [&](int l) { return priv(l).ln.so; });
        r.scrc = wp.from(lz, [&](int l) { return priv(l).ln.scrc; });
        if (zf & kNoCrc) {
          r.rout = 0;
        } else if ((zf & kSkip) && lz == kLanes - 1) {
          r.rout = 0;   // span starts at/after the region end - 3: k_combine computes it
        } else {
          r.rout = region_rout;
          if (region_sflag_clear) r.sflag = zf & ~kSkip;
        }
      }
    }
  }
  if (overflow || total > (uint32_t)kRegionCap) r.status = kOverflow;
  wp.single([&] { *out = r; });
  wp.stamp(4);
}

}  // namespace ldb
