// ldb_chain.h — the chained fast path of the log scan (host+device, like ldb_wave.h).
//
// A wavefront scans a contiguous run of regions in file order. Once one region's result is
// known (region_process, ldb_wave.h), the chain of ReadLogEntry positions (index.go:84-95)
// enters the next region at a known offset `x`, with a known CRC state: the running CRC
// register `I` of the entry that is open at the region start, and the stored crc of the entry
// that ends at `x` (its "owner"). region_chained() uses that state to process a region with no
// cross-region speculation and ONE CRC chain per lane:
//
//   G-chain. Over the region, every lane runs one raw CRC register over its slice with the
//   stored-crc field of each entry start s rewritten in the staging buffer:
//       bytes [s, s+4)   := ~crc(owner of s)     (the owner's expected final register)
//       bytes [s+4, s+8) ^= 0xFFFFFFFF           (CRC-32 init of the entry at s)
//   With that rewrite, the register of the whole byte stream (the "G-chain", slices combined by
//   a 6-step lane scan with constant-distance shift tables) is, just after [s, s+4),
//   shift(delta, 4) where delta = (owner's final register) ^ ~crc(owner): zero iff the owner's
//   CRC matches (getEntryCrc == crc, logfile/log_file.go:141-143). Past s+4 it continues as the
//   register of the entry at s, so the next region's `I` is the scan's last value.
//   Each owner is checked at the 8-byte step boundary P after s+4 (the lane keeps its register
//   before that step and re-runs the step with the bytes >= s+4 masked):
//       check = shift(G(slice start), P - slice start) ^ local(P)  ==  0.
//   GF(2) shifts are injective, so check == 0 <=> delta == 0, exactly, for every entry.
//
//   Speculation is only needed for lanes past the entry lane: each lane decodes its first
//   plausible header candidate, the links (exit of an entry == next start, nothing between) are
//   verified from the known entry, and the first broken link is repaired by decoding at the
//   true position. Anything outside the lean fast path (short entries, terminal statuses, near
//   the end of the file, non-canonical headers, a failed CRC) makes region_chained() restore
//   the buffer and return false: the caller then runs the exact general routine
//   (region_process) with the entry position forced. Results are therefore always those of the
//   serial scan; this path only changes speed.
//
// A region whose first entry's owner was verified here carries kOwnerOk in its summary, and
// k_combine does not verify that owner again (ldb_scan.hip).
#pragma once

#include "ldb_wave.h"

#ifdef LDB_EMU_COUNTERS   // CPU emulator instrumentation only: why region_chained declined a region
namespace ldb { extern uint64_t g_chain_why[16]; }
#define LDB_DECLINE(id) (++ldb::g_chain_why[id], false)
#else
#define LDB_DECLINE(id) false
#endif

namespace ldb {

constexpr uint32_t kOwnerOk = 8u;     // sflag: owner of the region's first start CRC-verified in-wave
constexpr uint32_t kMinFast = kS + 4; // fast path: every entry >= 84 B (one start per slice, one check per lane)

// Chain state carried from one region to the next within a wavefront's run.
struct ChainState {
  uint32_t on;       // 1: x / I / owner are valid
  uint32_t I;        // running CRC register (init-based) of the entry open at the region start
  uint32_t owner;    // stored crc of the entry that ends at x
  uint64_t x;        // absolute offset of the next entry start (>= region start)
};

// register shift by a fixed byte count: 4 lookups in a byte-indexed table set at `off`
LDB_HD uint32_t shift_tab(const uint32_t* tab, int off, uint32_t r) {
  return tab[off + (r & 0xFFu)] ^ tab[off + 256 + ((r >> 8) & 0xFFu)] ^ tab[off + 512 + ((r >> 16) & 0xFFu)] ^
         tab[off + 768 + (r >> 24)];
}

// register shift by 8 * n bytes, n in [0, 15] (binary decomposition over the kVSOff tables)
LDB_HD uint32_t shift_8n(const uint32_t* tab, uint32_t r, uint32_t n) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t t = shift_tab(tab, kVSOff + i * 1024, r);
    r = ((n >> i) & 1u) ? t : r;
  }
  return r;
}

// ---------------------------------------------------------------- lean header decode
// logfile.decodeHeader (log_entry.go:81-107) for the headers LazyDB's writer emits
// (db.go:473-523 -> EncodeEntry): canonical varints, expiredAt/txID <= 5 bytes, txStat one byte
// of value 0..2, key/value sizes <= 4 bytes with kSize >= 1. For such a header Go's decode is
// the plain one below, EncodeEntry re-emits the same header length, and ReadLogEntry returns
// the entry (no sentinel; the caller guarantees the 38-byte window is readable and this checks
// that the key/value bytes end strictly before the file end, i.e. within both bound rules).
// Returns false for everything else (the exact decoder in region_process handles it).
struct Lean {
  uint32_t crc, stat, hs, k, vv;
  uint32_t w1;   // original bytes [p+4, p+8) (restored if the region falls back)
  uint32_t X;    // region-relative exit p + hs + k + vv
};

LDB_HD uint32_t byte_of(const uint32_t* w, uint32_t b) {   // window byte b in [4, 20) (else some byte)
  const uint32_t d = b >> 2;
  const uint32_t x = d == 1 ? w[1] : d == 2 ? w[2] : d == 3 ? w[3] : w[4];
  return (x >> (8 * (b & 3))) & 0xFFu;
}

LDB_HD uint32_t bytes4_at(const uint32_t* w, uint32_t b) {  // window bytes [b, b+4), b in [8, 20) (else some bytes)
  const uint32_t d = b >> 2;
  const uint32_t lo = d == 2 ? w[2] : d == 3 ? w[3] : w[4];
  const uint32_t hi = d == 2 ? w[3] : d == 3 ? w[4] : w[5];
  return funnel(hi, lo, b & 3);
}

LDB_HD uint32_t ctz_or(uint32_t x, uint32_t dflt) { return x ? (uint32_t)__builtin_ctz(x) : dflt; }

// varint payload of a canonical field of n in [1, 4] bytes held little-endian in b;
// *canon = minimal encoding (n == 1 or last byte nonzero)
LDB_HD uint32_t field_value(uint32_t b, uint32_t n, bool* canon) {
  n = n < 1u ? 1u : (n > 4u ? 4u : n);   // other lengths are rejected by the caller
  b = n >= 4 ? b : (b & ((1u << (8 * n)) - 1u));
  *canon = n == 1 || (b >> (8 * (n - 1))) != 0u;
  return pext7(b);
}

LDB_HD bool decode_lean(const View& v, int p, Lean* o) {
  const int a = p + kPre;
  const int q = a & ~3;
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t d[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) d[i] = lds32(v, q + 4 * i);
  uint32_t w[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) w[i] = funnel(d[i + 1], d[i], sh);
  // terminator bits of window bytes 5..19 (bit i <-> byte 4 + i)
  const uint32_t M = msb4(w[1]) | (msb4(w[2]) << 4) | (msb4(w[3]) << 8) | (msb4(w[4]) << 12);
  uint32_t T = (~M) & 0xFFFEu;
  const uint32_t e0 = ctz_or(T, 16); T &= T - 1;
  const uint32_t e1 = ctz_or(T, 16); T &= T - 1;
  const uint32_t e2 = ctz_or(T, 16); T &= T - 1;
  const uint32_t e3 = ctz_or(T, 16); T &= T - 1;
  const uint32_t e4 = ctz_or(T, 16);
  // field lengths: expiredAt e0, txID e1-e0, txStat e2-e1 (== 1), kSize e3-e2, vSize e4-e3
  bool ok = e4 < 16u && e0 <= 5u && e1 - e0 <= 5u && e2 - e1 == 1u && e3 - e2 <= 4u && e4 - e3 <= 4u;
  const uint32_t stat = w[1] & 0xFFu;
  const uint32_t ts = byte_of(w, 4 + e2);          // txStat byte: zz(0..2) = 0, 2, 4
  ok = ok && stat <= 2u && (ts == 0u || ts == 2u || ts == 4u) && ((w[1] >> 8) & 1u) == 0u && w[0] != 0u;
  // minimal expiredAt / txID encodings (EncodeEntry re-emits them as read only then)
  ok = ok && (e0 == 1u || byte_of(w, 4 + e0) != 0u) && (e1 - e0 == 1u || byte_of(w, 4 + e1) != 0u);
  bool ck, cv;
  const uint32_t uk = field_value(bytes4_at(w, 5 + e2), e3 - e2, &ck);
  const uint32_t uv = field_value(bytes4_at(w, 5 + e3), e4 - e3, &cv);
  ok = ok && ck && cv && (uk & 1u) == 0u && uk >= 2u && (uv & 1u) == 0u;
  const uint32_t hs = 5 + e4;
  const uint32_t k = uk >> 1, vv = uv >> 1;
  const uint32_t X = (uint32_t)p + hs + k + vv;
  ok = ok && v.R0 + (uint64_t)X < v.len;   // key/value read within both IOController bound rules
  o->crc = w[0];
  o->stat = stat;
  o->hs = hs;
  o->k = k;
  o->vv = vv;
  o->w1 = w[1];
  o->X = X;
  return ok;
}

// First header candidate of slice [B, B+kS): smallest p with byte p+4 <= 2 (a Status byte,
// log_entry.go:9-16), or kNone32. Speculation only.
LDB_HD uint32_t first_cand(const View& v, int B) {
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  uint32_t best = 0xFFFFFFFFu;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const Row16 q = row[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qd = 4 * k + j - 1;   // dword qd + 1 of the slice holds the stat bytes of positions 4qd..4qd+3
      if (qd < 0 || qd >= kS / 4) continue;
      const uint32_t m = small_bytes(q.w[j]);   // lowest flagged byte is exact
      const uint32_t bit = m ? (uint32_t)__builtin_ctz(m) : 0xFFFFFFFFu;
      const uint32_t c = bit | ((uint32_t)qd << 5);
      best = c < best ? c : best;
    }
  }
  return best == 0xFFFFFFFFu ? kNone32 : (uint32_t)B + (best >> 3);
}

// Raw register over the slice (natural 8-byte grid), plus the check register: the register
// before step kb continued by one step over that step's word masked with mlo.
LDB_HD void crc_slice_cap(const View& v, int B, uint32_t kb, uint64_t mlo, uint32_t* y, uint32_t* yc) {
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  uint32_t reg = 0, cap = 0;
  uint64_t wc = 0;
#pragma unroll
  for (int k2 = 0; k2 < kS / 16; ++k2) {
    const Row16 q = row[k2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t k = 2 * k2 + h;
      const uint64_t w = ((uint64_t)q.w[2 * h + 1] << 32) | q.w[2 * h];
      cap = k == kb ? reg : cap;
      wc = k == kb ? w : wc;
      reg = crc_step8(v.tab, reg, q.w[2 * h], q.w[2 * h + 1]);
    }
  }
  *y = reg;
  wc &= mlo;
  *yc = crc_step8(v.tab, cap, (uint32_t)wc, (uint32_t)(wc >> 32));
}

// Per-lane registers of the chained path.
struct ChainPriv {
  uint32_t s;       // region-relative entry start in this slice, or kNone32
  uint32_t X;       // its exit
  uint32_t crc, k, vv, w1, hs, stat;
  uint32_t wo;      // ~crc of its owner (injected at [s, s+4))
  uint32_t kb;      // check: capture step (or 0), chk: 1 if this lane checks an owner
  uint32_t chk;
  uint64_t mlo;
  uint32_t y, yc, O;
};

// Rewrite (inject = true) or restore the 8 bytes [s, s+8) of a start in the staging buffer.
LDB_HD void rewrite8(uint8_t* wbuf, const ChainPriv& c, bool inject) {
  const uint32_t lo = inject ? c.wo : c.crc;
  const uint32_t hi = inject ? ~c.w1 : c.w1;
  uint8_t* b = wbuf + kPre + c.s;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    b[i] = (uint8_t)(lo >> (8 * i));
    b[4 + i] = (uint8_t)(hi >> (8 * i));
  }
}

// Lane scan of the G-chain: O_l = sum_{i <= l} shift(y_i, (l - i) slices) (Hillis-Steele, 6 steps).
template <class WP, class CPriv>
LDB_HD void lane_scan(WP& wp, const uint32_t* tab, CPriv cpriv) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int d = 1 << i;
    const int off = i == 0 ? kZSOff : kSCOff + (i - 1) * 1024;
    wp.shfl_up(d, [&](int l) { return cpriv(l).O; },
               [&](int l, uint32_t t, bool valid) { if (valid) cpriv(l).O ^= shift_tab(tab, off, t); });
  }
}

// The chained fast path for one region. Returns false (buffer restored, state untouched) when
// the region must go through region_process instead. On success writes *out, emits the
// region's tuples and advances `st`.
template <class WP, class CPriv, class Emit>
LDB_HD bool region_chained(WP& wp, const View& v, uint8_t* wbuf, WaveSh& sh, ChainState& st, RegionSum* out,
                           CPriv cpriv, Emit emit) {
  if (!st.on) return false;
  if (v.rlen != (uint32_t)kW || v.R0 + (uint64_t)(kW + kHalo) > v.len || st.x < v.R0) return LDB_DECLINE(1);
  const uint64_t xr64 = st.x - v.R0;
  if (xr64 >= (uint64_t)kW) {
    // ---- covered region: the open entry runs through it; no header can start here
    wp.each([&](int l) { ChainPriv& c = cpriv(l); c.O = crc_slice_from(v, l * kS, 0); });
    lane_scan(wp, v.tab, cpriv);
    const uint32_t raw = wp.from(kLanes - 1, [&](int l) { return cpriv(l).O; });
    RegionSum r;
    r.start = kNone64; r.exitp = 0; r.soff = 0; r.status = kCont; r.count = 0;
    r.rpre = raw; r.rout = 0; r.scrc = 0; r.sflag = 0;
    wp.single([&] { *out = r; });
    st.I = shift_tab(v.gsh, 0, st.I) ^ raw;   // build_gshift table kGsW: shift by one region
    return true;
  }
  const uint32_t xr = (uint32_t)xr64;
  const int lt = (int)(xr / kS);
  // ---- speculation: the entry lane decodes at x, later lanes at their first candidate
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    c.s = kNone32;
    c.chk = 0;
    const uint32_t p = l < lt ? kNone32 : (l == lt ? xr : first_cand(v, l * kS));
    if (p != kNone32) {
      Lean e;
      if (decode_lean(v, (int)p, &e)) {
        c.s = p; c.X = e.X; c.crc = e.crc; c.k = e.k; c.vv = e.vv; c.w1 = e.w1; c.hs = e.hs; c.stat = e.stat;
      }
    }
    sh.s[l] = c.s;
  });
  if (wp.from(lt, [&](int l) { return cpriv(l).s; }) == kNone32) return LDB_DECLINE(2);
  // ---- links from the entry lane: each start's exit is the next start, no start in between
  uint64_t starts = 0;
  for (int it = 0;; ++it) {
    starts = wp.ballot([&](int l) { return cpriv(l).s != kNone32; });
    const uint64_t sts = starts;
    const int irr = wp.first([&](int l) { const ChainPriv& c = cpriv(l); return c.s != kNone32 && c.X - c.s < kMinFast; });
    if (irr >= 0) return LDB_DECLINE(3);
    const int j = wp.first([&](int l) {
      const ChainPriv& c = cpriv(l);
      if (c.s == kNone32) return false;
      const int m = c.X >= (uint32_t)kW ? kLanes : (int)(c.X / kS);
      const uint64_t between = (m >= kLanes ? ~0ull : ((1ull << m) - 1)) & ~((2ull << l) - 1);
      return (between & sts) != 0 || (m < kLanes && sh.s[m] != c.X);
    });
    if (j < 0) break;
    if (it == 3) return LDB_DECLINE(5);
    const uint32_t Xj = wp.from(j, [&](int l) { return cpriv(l).X; });
    const int m = Xj >= (uint32_t)kW ? kLanes : (int)(Xj / kS);
    wp.each([&](int l) {
      ChainPriv& c = cpriv(l);
      if (l > j && l < m) c.s = kNone32;
      if (l == m) {
        Lean e;
        c.s = kNone32;
        if (decode_lean(v, (int)Xj, &e)) {
          c.s = Xj; c.X = e.X; c.crc = e.crc; c.k = e.k; c.vv = e.vv; c.w1 = e.w1; c.hs = e.hs; c.stat = e.stat;
        }
      }
      sh.s[l] = c.s;
    });
    if (m < kLanes && wp.from(m, [&](int l) { return cpriv(l).s; }) == kNone32) return LDB_DECLINE(6);
  }
  const int z = 63 - (int)__builtin_clzll(starts);
  const uint32_t sz = wp.from(z, [&](int l) { return cpriv(l).s; });
  if (sz + 8 > (uint32_t)kW) return LDB_DECLINE(7);   // the rewrite of the last start would spill past the region
  // ---- owners, check assignment, buffer rewrite
  wp.each([&](int l) { sh.want[l] = ~cpriv(l).crc; });
  const uint32_t want_x = ~st.owner;
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    const uint64_t below = starts & ((1ull << l) - 1);
    c.wo = below ? sh.want[63 - (int)__builtin_clzll(below)] : want_x;
    const uint32_t B = (uint32_t)(l * kS);
    uint32_t cs = kNone32;
    if (c.s != kNone32 && c.s + 4 < B + kS) cs = c.s;
    else if (l > 0 && sh.s[l - 1] != kNone32 && sh.s[l - 1] + 4 >= B) cs = sh.s[l - 1];
    c.chk = cs != kNone32;
    const uint32_t rel = cs != kNone32 ? cs + 4 - B : 0u;   // [0, kS)
    c.kb = rel >> 3;
    const uint32_t nb = rel & 7u;
    c.mlo = nb ? (~0ull >> (64 - 8 * nb)) : 0ull;
    if (c.s != kNone32) rewrite8(wbuf, c, true);
  });
  // ---- one CRC chain per lane, lane scan, owner checks
  wp.each([&](int l) { ChainPriv& c = cpriv(l); crc_slice_cap(v, l * kS, c.kb, c.mlo, &c.y, &c.yc); });
  const uint32_t I0 = shift_tab(v.tab, kZSOff, st.I);
  wp.each([&](int l) { ChainPriv& c = cpriv(l); c.O = c.y ^ (l == 0 ? I0 : 0u); });
  lane_scan(wp, v.tab, cpriv);
  const uint32_t Iin = st.I;
  wp.shfl_up(1, [&](int l) { return cpriv(l).O; }, [&](int l, uint32_t t, bool valid) {
    ChainPriv& c = cpriv(l);
    const uint32_t g = valid ? t : Iin;   // G at the slice start
    c.y = shift_8n(v.tab, g, c.kb + 1) ^ c.yc;   // check value (reuses y)
  });
  const int bad = wp.first([&](int l) { const ChainPriv& c = cpriv(l); return c.chk && c.y != 0u; });
  if (bad >= 0) {
    wp.each([&](int l) { const ChainPriv& c = cpriv(l); if (c.s != kNone32) rewrite8(wbuf, c, false); });
    return LDB_DECLINE(8);
  }
  // ---- tuples and summary
  wp.each([&](int l) {
    const ChainPriv& c = cpriv(l);
    if (c.s == kNone32) return;
    const uint32_t slot = (uint32_t)__builtin_popcountll(starts & ((1ull << l) - 1));
    const uint64_t pos = ((v.R0 + c.s) & 0xFFFFFFFFFFull) | ((uint64_t)(c.hs & 0x3F) << 40) |
                         ((uint64_t)(c.hs & 0x3F) << 46) | ((uint64_t)(c.stat & 0xFF) << 52);
    emit(slot, pos, c.k, c.vv);
  });
  RegionSum r;
  r.start = v.R0 + xr;
  r.status = kCont;
  r.count = (uint32_t)__builtin_popcountll(starts);
  r.exitp = v.R0 + wp.from(z, [&](int l) { return cpriv(l).X; });
  r.soff = v.R0 + sz;
  r.scrc = wp.from(z, [&](int l) { return cpriv(l).crc; });
  r.rout = wp.from(kLanes - 1, [&](int l) { return cpriv(l).O; });
  r.rpre = 0;
  r.sflag = kStraddle | kOwnerOk;
  wp.single([&] { *out = r; });
  st.x = r.exitp;
  st.I = r.rout;
  st.owner = r.scrc;
  return true;
}

// One region of a wavefront's run: the chained fast path when the chain state allows it,
// otherwise region_process (speculative at the start of a run, entry forced after a fallback).
template <class WP, class Priv, class CPriv, class Emit, class Free>
LDB_HD void run_region(WP& wp, const View& v, uint8_t* wbuf, WaveSh& sh, ChainState& st, RegionSum* out, Priv priv,
                       CPriv cpriv, Emit emit, Free buffer_free) {
  if (region_chained(wp, v, wbuf, sh, st, out, cpriv, emit)) {
    buffer_free();
    return;
  }
  uint32_t enter = kForceSpec;
  if (st.on && st.x >= v.R0) enter = st.x - v.R0 < (uint64_t)v.rlen ? (uint32_t)(st.x - v.R0) : kForceNone;
  region_process(wp, v, sh, enter, out, priv, emit, buffer_free);
  const RegionSum r = *out;
  // continue chained only from a clean straddle-out whose register at the region end is known
  st.on = r.status == kCont && r.start != kNone64 && r.sflag == kStraddle && r.exitp >= v.R0 + (uint64_t)kW &&
          v.rlen == (uint32_t)kW;
  st.x = r.exitp;
  st.I = r.rout;
  st.owner = r.scrc;
}

}  // namespace ldb
