// ldb_engine.h — the parallel log-scan algorithm, written once as per-lane phase
// functions (host+device) so the gfx950 kernels (ldb_scan.hip) and the CPU
// wave emulator used by the tests (tests/emu/) execute identical code.
//
// What it computes: the replay loop of index.go:84-95 over one log-file image —
// repeated (*LogFile).ReadLogEntry(offset) (logfile/log_file.go:116-145) — but
// without walking the chain entry by entry.
//
// Decomposition:
//   region = 64 slices of kS bytes, one wavefront; slice = one lane.
//   Each lane speculatively finds the first plausible entry start in its slice
//   (or is told where the chain enters it), walks the entries that START in
//   its slice (Go-exact decode, logfile/log_entry.go:81-107), and CRCs exactly
//   the bytes of its slice: the raw CRC of the prefix that belongs to an entry
//   started in an earlier slice, the complete CRCs of entries inside the slice,
//   and the running CRC register of the entry that continues past the slice.
//   Links between slices are verified (a lane's exit must be the next lane's
//   start); mismatches are repaired by re-running the lane from the true
//   position. Entries spanning slices/regions are verified by combining
//   per-slice CRC pieces with GF(2) shifts (CRC(A||B) = shift(CRC(A),|B|) ^ raw(B)).
// The per-region summaries are stitched across regions by the kernels in
// ldb_scan.hip with the same verify-then-repair rule, so the result equals the
// serial scan for every input, including adversarial ones (values that embed
// valid entries): speculation only ever changes speed, never results.
#pragma once

#include "ldb_common.h"

namespace ldb {

// ---------------------------------------------------------------- geometry
constexpr int kLanes = 64;
constexpr int kS = 80;                    // slice bytes per lane (16 * odd: conflict-free LDS rows)
constexpr int kW = kS * kLanes;           // 5120 bytes per region (one wavefront)
constexpr int kHalo = 64;                 // bytes staged past the region end (headers of late entries)
constexpr int kPre = 16;                  // readable bytes before the region start in a staging buffer
constexpr int kBuf = kPre + kW + kHalo;   // staging buffer bytes per region
constexpr int kRegionCap = kW / 10 + 8;   // tuple slots per region (entries >= 10 B when well formed)
constexpr int kNSeg = 3;                  // CRC segments handled per walk round

// Table block (uint32 offsets) shared by every wave of a workgroup (LDS) / the emulator.
constexpr int kT11Off = 0;                // 2048 + 2048 + 1024 entries: slicing-by-4 on 11/11/10-bit chunks
constexpr int kT8Off = 5120;              // 256: byte-at-a-time table
constexpr int kZSOff = 5376;              // 4 x 256: register shift by kS zero bytes
constexpr int kXOff = 6400;               // kS + 1: x^(8n) mod P, n = 0..kS
constexpr int kTabWords = 6400 + 84;      // padded to 16 bytes
constexpr int kTabBytes = kTabWords * 4;

// Force codes for a lane (re)run.
constexpr uint32_t kForceSpec = 0xFFFFFFFEu;  // search for a plausible start
constexpr uint32_t kForceNone = 0xFFFFFFFFu;  // slice is covered by an entry started earlier

// sflag bits
constexpr uint32_t kStraddle = 1u;   // last entry started here ends beyond the slice
constexpr uint32_t kSkip = 2u;       // its CRC span starts < 4 bytes before (or after) the slice end
constexpr uint32_t kNoCrc = 4u;      // its decoded header size <= 4: getEntryCrc returns 0 (already checked)

constexpr int kOverflow = 100;       // internal: region needs more than kRegionCap tuple slots

// ---------------------------------------------------------------- table building (host)
inline void build_tables(uint32_t* tab) {
  uint32_t t8[256];
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    t8[i] = c;
  }
  auto step_bits = [](uint32_t x, int nbits) {
    for (int k = 0; k < nbits; ++k) x = (x >> 1) ^ (kPoly & (0u - (x & 1u)));
    return x;
  };
  // chunk tables: register after 32 bit-steps of x restricted to the chunk's bits
  const int off[3] = {0, 11, 22}, wid[3] = {11, 11, 10}, base[3] = {0, 2048, 4096};
  for (int q = 0; q < 3; ++q)
    for (uint32_t v = 0; v < (1u << wid[q]); ++v) tab[kT11Off + base[q] + v] = step_bits(v << off[q], 32);
  for (int i = 0; i < 256; ++i) tab[kT8Off + i] = t8[i];
  const uint32_t xs = x8n_modp(kS);
  for (int q = 0; q < 4; ++q)
    for (uint32_t b = 0; b < 256; ++b) tab[kZSOff + q * 256 + b] = multmodp(xs, b << (8 * q));
  for (int n = 0; n <= kS; ++n) tab[kXOff + n] = x8n_modp((uint64_t)n);
  for (int i = kXOff + kS + 1; i < kTabWords; ++i) tab[i] = 0;
}

// ---------------------------------------------------------------- memory views
// `buf` points at the staging buffer (region byte r lives at buf[kPre + r]); `tab` at the
// table block. Both are LDS on the GPU, plain memory in the emulator.
struct View {
  const uint8_t* buf;
  const uint32_t* tab;
  uint64_t R0;      // absolute offset of region byte 0
  uint32_t rlen;    // bytes of the region inside the file (<= kW)
  uint64_t len;     // file length (= IOController bound)
  int io;
};

LDB_HD uint32_t vbyte(const View& v, int64_t rel) { return v.buf[kPre + rel]; }

LDB_HD uint32_t vword_aligned(const View& v, int64_t rel4) {
  return *reinterpret_cast<const uint32_t*>(v.buf + kPre + rel4);
}

// 4 bytes at an arbitrary relative position (two aligned reads + funnel shift).
LDB_HD uint32_t vword(const View& v, int64_t rel) {
  const int64_t a = rel + kPre;
  const int64_t q = a & ~(int64_t)3;
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t d0 = *reinterpret_cast<const uint32_t*>(v.buf + q);
  const uint32_t d1 = *reinterpret_cast<const uint32_t*>(v.buf + q + 4);
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(d1, d0, sh);
#else
  return sh ? (uint32_t)((((uint64_t)d1 << 32) | d0) >> (8 * sh)) : d0;
#endif
}

// Slicing-by-4 on 11/11/10-bit chunks: 3 table reads per 4 bytes.
LDB_HD uint32_t crc_step4(const uint32_t* tab, uint32_t x) {
  return tab[kT11Off + (x & 0x7FFu)] ^ tab[kT11Off + 2048 + ((x >> 11) & 0x7FFu)] ^ tab[kT11Off + 4096 + (x >> 22)];
}

// register shift by kS zero bytes
LDB_HD uint32_t shift_slice(const uint32_t* tab, uint32_t r) {
  return tab[kZSOff + (r & 0xFF)] ^ tab[kZSOff + 256 + ((r >> 8) & 0xFF)] ^ tab[kZSOff + 512 + ((r >> 16) & 0xFF)] ^
         tab[kZSOff + 768 + (r >> 24)];
}

// register shift by n zero bytes, n in [0, kS]
LDB_HD uint32_t shift_n(const uint32_t* tab, uint32_t r, uint32_t n) {
  return n == 0 ? r : multmodp(tab[kXOff + n], r);
}

// CRC over region bytes [lo, hi) (hi - lo >= 1) with words aligned to hi.
//   span = true : register starting from the CRC-32 init value (~0): injected as 0xFF over the
//                 first 4 message bytes, with the short-message correction for |M| < 4.
//   span = false: raw register starting from 0 (leading zero bytes do not change it).
LDB_HD uint32_t crc_segment(const View& v, int64_t lo, int64_t hi, bool span) {
  const int64_t L = hi - lo;
  const int64_t nw = (L + 3) / 4;
  int64_t c = hi - 4 * nw;
  const uint32_t pad = (uint32_t)(lo - c);  // 0..3 leading bytes outside the segment
  uint32_t m0 = 0xFFFFFFFFu << (8 * pad);
  uint32_t i0 = span ? m0 : 0u;
  uint32_t i1 = (span && pad) ? (0xFFFFFFFFu >> (8 * (4 - pad))) : 0u;
  uint32_t reg = 0;
  for (int64_t k = 0; k < nw; ++k, c += 4) {
    uint32_t w = (vword(v, c) & m0) ^ i0;
    reg = crc_step4(v.tab, reg ^ w);
    m0 = 0xFFFFFFFFu;
    i0 = i1;
    i1 = 0;
  }
  if (span && L < 4) reg ^= 0xFFFFFFFFu >> (8 * L);
  return reg;
}

// Byte fetch functor for decode_header at region-relative position p.
struct LdsFetch {
  const View* v;
  int64_t p;
  LDB_HD uint32_t operator()(int i) const { return vbyte(*v, p + i); }
};

LDB_HD EntryInfo classify_at(const View& v, int64_t p) {
  return classify_entry(LdsFetch{&v, p}, v.len, v.io, v.R0 + (uint64_t)p);
}

// 38 zero bytes at p (p + 38 inside the staged bytes)?
LDB_HD bool zero_window(const View& v, int64_t p) {
  for (int i = 0; i < kMaxHeader; ++i)
    if (vbyte(v, p + i)) return false;
  return true;
}

// ---------------------------------------------------------------- per-lane state
struct LaneState {
  uint32_t s;        // first entry start in the slice (region-relative) or kNone32
  uint32_t cnt;      // entries accepted that start in the slice (incl. a pending straddler)
  int32_t term;      // kCont or the ReadLogEntry status that stopped the walk
  uint32_t tpos;     // region-relative position of that status
  uint64_t x;        // absolute offset after the last entry that started here (term == kCont)
  uint32_t rpre;     // raw CRC register over [B, min(s, Eeff))
  uint32_t sflag;    // kStraddle | kSkip | kNoCrc for the last entry (x beyond the slice)
  uint32_t so;       // its region-relative start
  uint32_t scrc;     // its stored crc
  uint32_t rout;     // its CRC register at the slice end (init-based), unless kSkip/kNoCrc
};

// Speculative start search (never decides results; see plausible_start).
LDB_HD uint32_t find_start(const View& v, int64_t B, int64_t Eeff) {
  for (int64_t p = B; p < Eeff; ++p) {
    if (read_eof(v.len, v.io, (int64_t)(v.R0 + p), kMaxHeader)) return (uint32_t)p;  // window EOF from here on
    if (vbyte(v, p + 4) > 2u) continue;                                                 // stat byte prefilter
    const EntryInfo e = classify_at(v, p);
    if (e.status == kCont && plausible_start(e)) {
      const uint64_t nx = (uint64_t)p + e.size;  // one-hop check while the next header is staged
      if (nx + kMaxHeader <= (uint64_t)(kW + kHalo) && v.R0 + nx < v.len) {
        const EntryInfo e2 = classify_at(v, (int64_t)nx);
        const bool ok2 = (e2.status == kCont && plausible_start(e2)) || e2.status == LDB_EOF_WINDOW ||
                         (e2.status == LDB_EOF_SENTINEL && zero_window(v, (int64_t)nx));
        if (!ok2) continue;
      }
      return (uint32_t)p;
    }
    if (e.status == LDB_EOF_SENTINEL && zero_window(v, p)) return (uint32_t)p;
  }
  return kNone32;
}

struct Seg {
  int32_t lo, hi;    // region-relative [lo, hi)
  uint32_t kind;     // 0 raw prefix, 1 verify, 2 span out
  uint32_t crc;      // stored crc (verify)
  uint32_t ord;      // cnt before this entry (verify)
  uint32_t o;        // entry start (verify)
};

// Process one lane's slice: start (by `force`), walk, CRC pieces, in-slice verification.
LDB_HD void lane_process(const View& v, int lane, uint32_t force, LaneState* st) {
  const int64_t B = (int64_t)lane * kS, E = B + kS;
  const int64_t Eeff = E < (int64_t)v.rlen ? E : (int64_t)v.rlen;
  LaneState r;
  r.s = kNone32; r.cnt = 0; r.term = kCont; r.tpos = 0; r.x = 0; r.rpre = 0; r.sflag = 0; r.so = 0; r.scrc = 0;
  r.rout = 0;
  if (B >= Eeff) { *st = r; return; }          // slice entirely past the end of the file
  uint32_t s = force == kForceSpec ? find_start(v, B, Eeff) : (force == kForceNone ? kNone32 : force);
  r.s = s;
  // RAW prefix [B, min(s, Eeff)) belongs to an entry started before this slice
  const int64_t pe = (s == kNone32) ? Eeff : (int64_t)s;
  if (pe > B) r.rpre = crc_segment(v, B, pe, false);
  if (s == kNone32) { *st = r; return; }
  int64_t o = s;
  bool walking = true;
  while (walking) {
    Seg sg[kNSeg];
    int ns = 0;
    while (walking && ns < kNSeg) {
      if (o >= Eeff) {          // next entry starts in a later slice (or exactly at the file end)
        r.x = v.R0 + (uint64_t)o;
        walking = false;
        break;
      }
      const EntryInfo e = classify_at(v, o);
      if (e.status != kCont) { r.term = e.status; r.tpos = (uint32_t)o; walking = false; break; }
      const uint64_t end = (uint64_t)o + e.size;
      if (e.h.size <= 4) {      // getEntryCrc returns 0 (log_entry.go:111): valid iff stored crc == 0
        if (e.h.crc != 0) { r.term = LDB_ERR_CRC; r.tpos = (uint32_t)o; walking = false; break; }
        r.cnt++;
        if (end > (uint64_t)E) {
          r.sflag = kStraddle | kNoCrc; r.so = (uint32_t)o; r.scrc = 0; r.x = v.R0 + end; walking = false; break;
        }
        o = (int64_t)end;
        continue;
      }
      const int64_t lo = o + 4;
      if (end <= (uint64_t)E) {
        sg[ns].lo = (int32_t)lo; sg[ns].hi = (int32_t)end; sg[ns].kind = 1; sg[ns].crc = e.h.crc;
        sg[ns].ord = r.cnt; sg[ns].o = (uint32_t)o; ++ns;
        r.cnt++;
        o = (int64_t)end;
      } else {
        r.cnt++;
        r.sflag = kStraddle; r.so = (uint32_t)o; r.scrc = e.h.crc; r.x = v.R0 + end;
        if (E - lo >= 4) {
          sg[ns].lo = (int32_t)lo; sg[ns].hi = (int32_t)E; sg[ns].kind = 2; sg[ns].crc = 0; sg[ns].ord = 0;
          sg[ns].o = (uint32_t)o; ++ns;
        } else {
          r.sflag |= kSkip;
        }
        walking = false;
      }
    }
    for (int i = 0; i < ns; ++i) {
      const uint32_t reg = crc_segment(v, sg[i].lo, sg[i].hi, true);
      if (sg[i].kind == 2) { r.rout = reg; continue; }
      if (reg != ~sg[i].crc) {   // ErrInvalidCrc (log_file.go:141-143)
        r.term = LDB_ERR_CRC; r.tpos = sg[i].o; r.cnt = sg[i].ord; r.sflag = 0; walking = false;
        break;
      }
    }
  }
  *st = r;
}

// ---------------------------------------------------------------- wave-level state (LDS)
struct WaveSh {
  LaneState ln[kLanes];
  uint32_t force[kLanes];
  uint32_t prefix[kLanes];   // exclusive prefix of emitted tuples per lane
  // region result
  uint64_t start, exitp, soff;
  int32_t status;
  uint32_t count, rpre, rout, scrc, sflag;
  uint32_t chain_end;        // last lane (inclusive) whose entries belong to the region's chain
  uint32_t todo;             // lanes to (re)run: bit mask split in two words
  uint32_t todo_hi;
};

// Link check for lane j (phase after lane_process): returns the lane to repair and its force,
// or -1 when lane j's outgoing link is consistent.  `noneMask`: bit k set iff lane k has no start.
LDB_HD int lane_link(const View& v, const WaveSh& w, int j, uint64_t noneMask, uint32_t* fix_force) {
  const LaneState& a = w.ln[j];
  if (a.s == kNone32 || a.term != kCont) return -1;
  const uint64_t xr = a.x - v.R0;           // region-relative exit (>= E_j)
  if (xr >= (uint64_t)v.rlen) {             // leaves the region (or ends exactly at the file end):
    for (int k = j + 1; k < kLanes; ++k)    // every later lane must be covered
      if (!((noneMask >> k) & 1)) { *fix_force = kForceNone; return k; }
    return -1;
  }
  const int m = (int)(xr / kS);
  for (int k = j + 1; k < m; ++k)
    if (!((noneMask >> k) & 1)) { *fix_force = kForceNone; return k; }
  if (w.ln[m].s != (uint32_t)xr) { *fix_force = (uint32_t)xr; return m; }
  return -1;
}

// Entering check: where the chain enters this region (region-level force).
// enter = kForceSpec: first lane with a start is the entry (nothing to check).
// enter = kForceNone: every lane must be covered. Otherwise enter = region-relative t.
LDB_HD int enter_check(const View& v, const WaveSh& w, uint32_t enter, uint32_t* fix_force) {
  if (enter == kForceSpec) return -1;
  int lt = enter == kForceNone ? kLanes : (int)(enter / kS);
  if (enter != kForceNone && enter >= v.rlen) lt = kLanes;
  for (int k = 0; k < lt && k < kLanes; ++k)
    if (w.ln[k].s != kNone32) { *fix_force = kForceNone; return k; }
  if (lt < kLanes && w.ln[lt].s != enter) { *fix_force = enter; return lt; }
  return -1;
}

// Fold: verify an entry that starts in lane j and ends inside the region (landing lane m).
// Returns true when the CRC matches.
LDB_HD bool fold_verify(const View& v, const WaveSh& w, int j) {
  const LaneState& a = w.ln[j];
  const int64_t xr = (int64_t)(a.x - v.R0);
  const int m = (int)(xr / kS);
  const int64_t Bm = (int64_t)m * kS;
  if (a.sflag & kNoCrc) return true;
  uint32_t reg;
  int k0;
  if (a.sflag & kSkip) {
    // CRC span starts at so+4 >= E_j - 3: compute its first piece directly, up to E_{j+1}
    const int64_t lo = (int64_t)a.so + 4;
    const int64_t e1 = (int64_t)(j + 2) * kS;
    const int64_t hi = xr < e1 ? xr : e1;
    reg = crc_segment(v, lo, hi, true);
    if (xr <= e1) return reg == ~a.scrc;
    k0 = j + 2;
  } else {
    reg = a.rout;
    k0 = j + 1;
  }
  for (int k = k0; k < m; ++k) reg = shift_slice(v.tab, reg) ^ w.ln[k].rpre;
  reg = shift_n(v.tab, reg, (uint32_t)(xr - Bm)) ^ w.ln[m].rpre;
  return reg == ~a.scrc;
}

// Register of the region's straddle-out entry (starting in chain lane j) at the region end.
LDB_HD uint32_t fold_out(const View& v, const WaveSh& w, int j, uint32_t* flags) {
  const LaneState& a = w.ln[j];
  uint32_t reg = 0;
  int k0 = j + 1;
  *flags = a.sflag;
  if (a.sflag & kNoCrc) return 0;
  if (a.sflag & kSkip) {
    if (j == kLanes - 1) return 0;           // span begins at/after the region end - 3: K_combine does it
    const int64_t lo = (int64_t)a.so + 4;
    reg = crc_segment(v, lo, (int64_t)(j + 2) * kS, true);
    *flags = a.sflag & ~kSkip;
    k0 = j + 2;
  } else {
    reg = a.rout;
  }
  for (int k = k0; k < kLanes; ++k) reg = shift_slice(v.tab, reg) ^ w.ln[k].rpre;
  return reg;
}

// Raw CRC over [0, upto) of the region from the lanes' prefix pieces (lanes before `lane_of_upto`
// are fully covered). upto in [0, rlen].
LDB_HD uint32_t fold_prefix(const View& v, const WaveSh& w, int64_t upto) {
  uint32_t reg = 0;
  int k = 0;
  for (; (int64_t)(k + 1) * kS <= upto && k < kLanes; ++k) reg = shift_slice(v.tab, reg) ^ w.ln[k].rpre;
  const int64_t rem = upto - (int64_t)k * kS;
  if (rem > 0) reg = shift_n(v.tab, reg, (uint32_t)rem) ^ w.ln[k].rpre;
  return reg;
}

// Re-walk lane j's accepted entries (headers only) and emit index tuples.
template <class Emit>
LDB_HD void lane_emit(const View& v, const LaneState& a, Emit emit) {
  int64_t o = a.s;
  for (uint32_t i = 0; i < a.cnt; ++i) {
    const EntryInfo e = classify_at(v, o);
    emit(i, pack_pos(v.R0 + (uint64_t)o, e.h), e.h.k_size, e.h.v_size);
    o += (int64_t)e.size;
  }
}

}  // namespace ldb
