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
//
// Latency rules for gfx950 (one wave per slice group, LDS-resident data): every lookup
// chain is an LDS round trip (~100+ cycles), so the hot paths batch independent LDS
// reads (b128 slice loads, one-round-trip header windows) and keep CRC chains short
// (8-byte steps on 11/11/10-bit slicing tables: 6 reads, 3 of them off the chain).
#pragma once

#include "ldb_common.h"

namespace ldb {

// ---------------------------------------------------------------- geometry
constexpr int kLanes = 64;
constexpr int kS = 80;                    // slice bytes per lane (16 * odd: conflict-free b128 rows)
constexpr int kW = kS * kLanes;           // 5120 bytes per region (one wavefront)
constexpr int kHalo = 64;                 // bytes staged past the region end (headers of late entries)
constexpr int kPre = 16;                  // readable bytes before the region start in a staging buffer
constexpr int kBuf = kPre + kW + kHalo;   // staging buffer bytes per region
constexpr int kRegionCap = kW / 10 + 8;   // tuple slots per region (entries >= 10 B when well formed)
constexpr int kKeep = 2;                  // tuples a lane keeps in registers for emission

// Table block (uint32 offsets) shared by every wave of a workgroup (LDS) / the emulator.
// 8-byte CRC step: reg' = A(reg ^ w0) ^ B(w1), A = 64 bit-steps, B = 32 bit-steps, each as three
// lookups on 11/11/10-bit chunks.
constexpr int kTAOff = 0;                 // 2048 + 2048 + 1024
constexpr int kTBOff = 5120;              // 2048 + 2048 + 1024
constexpr int kT8Off = 10240;             // 256: byte-at-a-time table (rare paths)
constexpr int kZSOff = 10496;             // 4 x 256: register shift by kS zero bytes (fold chains)
constexpr int kTabWords = 11520;
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
  auto step_bits = [](uint32_t x, int nbits) {
    for (int k = 0; k < nbits; ++k) x = (x >> 1) ^ (kPoly & (0u - (x & 1u)));
    return x;
  };
  const int off[3] = {0, 11, 22}, wid[3] = {11, 11, 10}, base[3] = {0, 2048, 4096};
  for (int q = 0; q < 3; ++q)
    for (uint32_t v = 0; v < (1u << wid[q]); ++v) {
      tab[kTAOff + base[q] + v] = step_bits(v << off[q], 64);
      tab[kTBOff + base[q] + v] = step_bits(v << off[q], 32);
    }
  for (uint32_t i = 0; i < 256; ++i) tab[kT8Off + i] = step_bits(i, 8);
  for (int q = 0; q < 4; ++q)
    for (uint32_t b = 0; b < 256; ++b) tab[kZSOff + q * 256 + b] = step_bits(b << (8 * q), 8 * kS);
}

// ---------------------------------------------------------------- memory views
// `buf` points at the staging buffer (region byte r lives at buf[kPre + r]); `tab` at the
// table block. Both are LDS on the GPU, plain memory in the emulator. `xw` = x^(8n) mod P,
// n = 0..kW (global memory).
struct View {
  const uint8_t* buf;
  const uint32_t* tab;
  const uint32_t* xw;
  uint64_t R0;      // absolute offset of region byte 0
  uint32_t rlen;    // bytes of the region inside the file (<= kW)
  uint64_t len;     // file length (= IOController bound)
  int io;
};

LDB_HD uint32_t vbyte(const View& v, int64_t rel) { return v.buf[kPre + rel]; }
LDB_HD uint32_t lds32(const View& v, int64_t a) { return *reinterpret_cast<const uint32_t*>(v.buf + a); }

LDB_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {  // bytes [sh, sh+4) of hi:lo
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
  return sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh)) : lo;
#endif
}

// 4 bytes at an arbitrary region-relative position (two aligned reads + funnel shift).
LDB_HD uint32_t vword(const View& v, int64_t rel) {
  const int64_t a = rel + kPre;
  const int64_t q = a & ~(int64_t)3;
  return funnel(lds32(v, q + 4), lds32(v, q), (uint32_t)(a & 3));
}

LDB_HD uint32_t ctz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_ctzll(x);
#else
  return (uint32_t)__builtin_ctzll(x);
#endif
}

// ---------------------------------------------------------------- CRC
LDB_HD uint32_t crc_step8(const uint32_t* tab, uint32_t reg, uint32_t w0, uint32_t w1) {
  const uint32_t x = reg ^ w0;
  const uint32_t b = tab[kTBOff + (w1 & 0x7FFu)] ^ tab[kTBOff + 2048 + ((w1 >> 11) & 0x7FFu)] ^
                     tab[kTBOff + 4096 + (w1 >> 22)];
  return tab[kTAOff + (x & 0x7FFu)] ^ tab[kTAOff + 2048 + ((x >> 11) & 0x7FFu)] ^ tab[kTAOff + 4096 + (x >> 22)] ^ b;
}

LDB_HD uint32_t mask_from(uint32_t nbytes) {  // bytes [nbytes, 4) kept, nbytes in [0, 4]
  return nbytes >= 4 ? 0u : (0xFFFFFFFFu << (8 * nbytes));
}

// CRC register over region bytes [lo, hi) (hi - lo >= 1) in 8-byte steps aligned to hi, starting
// from register `init`: the register is injected (XORed) into the first 4 message bytes, which
// is exact for |M| >= 4; for |M| < 4 the unconsumed part (init >> 8|M|) is added at the end.
// init = ~0: CRC-32 span (getEntryCrc); init = 0: raw register (leading zero bytes are free).
LDB_HD uint32_t crc_segment(const View& v, int64_t lo, int64_t hi, uint32_t init) {
  const int64_t L = hi - lo;
  const int64_t n8 = (L + 7) / 8;
  int64_t c = hi - 8 * n8;
  const uint32_t pad = (uint32_t)(lo - c);  // 0..7 leading bytes outside the segment
  const uint32_t m0 = mask_from(pad), m1 = pad <= 4 ? 0xFFFFFFFFu : mask_from(pad - 4);
  // init bytes land on message bytes [pad, pad+4) of the 12-byte window starting at c
  const uint64_t sh64 = (uint64_t)init << (8 * (pad & 3));
  const uint32_t ilo = (uint32_t)sh64, ihi = (uint32_t)(sh64 >> 32);
  const uint32_t i0 = pad < 4 ? ilo : 0u, i1 = pad < 4 ? ihi : ilo, i2 = pad < 4 ? 0u : ihi;
  const int64_t a0 = c + kPre;
  int64_t q = a0 & ~(int64_t)3;
  const uint32_t sh = (uint32_t)(a0 & 3);
  uint32_t d0 = lds32(v, q);
  uint32_t reg = 0;
  for (int64_t k = 0; k < n8; ++k) {
    const uint32_t d1 = lds32(v, q + 4), d2 = lds32(v, q + 8);
    uint32_t w0 = funnel(d1, d0, sh), w1 = funnel(d2, d1, sh);
    if (k == 0) { w0 = (w0 & m0) ^ i0; w1 = (w1 & m1) ^ i1; }
    else if (k == 1) { w0 ^= i2; }
    reg = crc_step8(v.tab, reg, w0, w1);
    d0 = d2;
    q += 8;
  }
  if (L < 4) reg ^= init >> (8 * L);
  return reg;
}

// register shift by kS zero bytes (constant-distance GF(2) multiply, 4 table reads)
LDB_HD uint32_t shift_slice(const uint32_t* tab, uint32_t r) {
  return tab[kZSOff + (r & 0xFF)] ^ tab[kZSOff + 256 + ((r >> 8) & 0xFF)] ^ tab[kZSOff + 512 + ((r >> 16) & 0xFF)] ^
         tab[kZSOff + 768 + (r >> 24)];
}

// ---------------------------------------------------------------- header decode
// Byte fetch functor for the exact (slow-path) decode at region-relative position p.
struct LdsFetch {
  const View* v;
  int64_t p;
  LDB_HD uint32_t operator()(int i) const { return vbyte(*v, p + i); }
};

LDB_HD EntryInfo classify_slow(const View& v, int64_t p) {
  return classify_entry(LdsFetch{&v, p}, v.len, v.io, v.R0 + (uint64_t)p);
}

// MSBs of the 4 bytes of w -> 4-bit mask (bit j = byte j >= 0x80)
LDB_HD uint32_t msb4(uint32_t w) { return (((w >> 7) & 0x01010101u) * 0x10204080u) >> 28; }

// 7-bit payload of a varint of n <= 4 bytes held little-endian in b
LDB_HD uint32_t pext7(uint32_t b) {
  return (b & 0x7Fu) | ((b >> 1) & 0x3F80u) | ((b >> 2) & 0x1FC000u) | ((b >> 3) & 0xFE00000u);
}

LDB_HD uint32_t vlen32(uint64_t ux) {  // bytes of PutUvarint(ux)
  uint32_t n = 1;
  while (ux >= 0x80u) { ux >>= 7; ++n; }
  return n;
}

// ReadLogEntry(off) up to the CRC comparison (classify_entry semantics), fast path for headers
// whose five varints end within bytes [5, 20) with ts/k/v varints <= 4 bytes and expiredAt/txID
// varints <= 5 bytes — every header LazyDB's writer emits for sizes < 128 MiB. Anything else
// (and every status other than kCont) goes through the exact byte-wise decoder.
LDB_HD EntryInfo classify_at(const View& v, int64_t p) {
  EntryInfo r;
  r.size = 0;
  const uint64_t off = v.R0 + (uint64_t)p;
  if (read_eof(v.len, v.io, (int64_t)off, kMaxHeader)) { r.status = LDB_EOF_WINDOW; return r; }
  // window bytes [p, p+24) -> w[0..5]
  const int64_t a = p + kPre;
  const int64_t q = a & ~(int64_t)3;
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t d[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) d[i] = lds32(v, q + 4 * i);
  uint32_t w[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) w[i] = funnel(d[i + 1], d[i], sh);
  // continuation bits of bytes 4..23, terminators among bytes 5..19
  const uint32_t M = msb4(w[1]) | (msb4(w[2]) << 4) | (msb4(w[3]) << 8) | (msb4(w[4]) << 12) | (msb4(w[5]) << 16);
  uint32_t T = (~M) & 0xFFFEu;   // bit i <-> byte 4 + i; keep bytes 5..19
  uint32_t e[5];
  uint32_t prev = 0;
  bool fast = true;
#pragma unroll
  for (int f = 0; f < 5; ++f) {
    if (T == 0) { fast = false; e[f] = 0; continue; }
    e[f] = __builtin_ctz(T);   // byte index - 4
    T &= T - 1;
    const uint32_t n = e[f] - prev;
    fast = fast && n <= (f < 2 ? 5u : 4u);
    prev = e[f];
  }
  if (fast) {
    // field f occupies window bytes [4 + e[f-1] + 1, 4 + e[f]]
    uint32_t val[3], lastb[5], n[5];
    uint32_t pe = 0;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      const uint32_t s = 5 + pe;                 // first byte of the field (window index)
      n[f] = e[f] - pe;
      // 4 bytes at window index s (s in [5, 19]): dword s>>2 .. +1 of w
      const uint32_t di = s >> 2, bs = s & 3;
      const uint32_t lo = di == 1 ? w[1] : di == 2 ? w[2] : di == 3 ? w[3] : w[4];
      const uint32_t hi = di == 1 ? w[2] : di == 2 ? w[3] : di == 3 ? w[4] : w[5];
      uint32_t b = funnel(hi, lo, bs);
      const uint32_t nn = n[f] > 4 ? 4 : n[f];
      if (n[f] > 4) {  // 5-byte expiredAt / txID: its last byte is window byte 4 + e[f] (9..14)
        const uint32_t li = 4 + e[f];
        lastb[f] = ((li >> 2) == 2 ? w[2] : w[3]) >> (8 * (li & 3)) & 0xFFu;
      } else {
        lastb[f] = (b >> (8 * (nn - 1))) & 0xFFu;
      }
      if (f >= 2) {
        b &= nn == 4 ? 0xFFFFFFFFu : ((1u << (8 * nn)) - 1);
        val[f - 2] = pext7(b);
      }
      if (f == 0) r.h.expired_at = (b & 1u) ? -1 : 0;   // sign only (zigzag LSB); value unused here
      pe = e[f];
    }
    bool canon = true;
#pragma unroll
    for (int f = 0; f < 5; ++f) canon = canon && (n[f] == 1 || lastb[f] != 0);
    if (canon) {
      const uint32_t ts_ux = val[0], k_ux = val[1], v_ux = val[2];
      const int64_t ts = zigzag(ts_ux), ks = zigzag(k_ux), vs = zigzag(v_ux);
      r.h.crc = w[0];
      r.h.stat = w[1] & 0xFFu;
      r.h.tx_id = 0;   // value unused on the fast path (ENTRY tuples re-decode in k_compact)
      r.h.tx_stat = (uint32_t)(uint16_t)ts;
      r.h.k_size = (uint32_t)ks;
      r.h.v_size = (uint32_t)vs;
      r.h.size = (int32_t)(5 + e[4]);
      r.h.raw_tx_stat_ok = (ts >= 0 && ts <= 2) ? 1u : 0u;
      r.h.canonical = ks >= 0 && vs >= 0;
      r.h.enc_size = (int32_t)(5 + n[0] + n[1] + vlen32((uint64_t)r.h.tx_stat << 1) + vlen32((uint64_t)r.h.k_size << 1) +
                               vlen32((uint64_t)r.h.v_size << 1));
      if (r.h.crc == 0 && r.h.k_size == 0 && r.h.v_size == 0) { r.status = LDB_EOF_SENTINEL; return r; }
      const uint64_t kv = (uint64_t)r.h.k_size + (uint64_t)r.h.v_size;
      if (kv && read_eof(v.len, v.io, (int64_t)(off + (uint64_t)r.h.size), kv)) { r.status = LDB_EOF_KV; return r; }
      r.size = (uint64_t)r.h.size + kv;
      r.status = kCont;
      return r;
    }
  }
  return classify_slow(v, p);
}

// 38 zero bytes at p (p + 38 inside the staged bytes)?
LDB_HD bool zero_window(const View& v, int64_t p) {
  uint32_t o = 0;
  for (int i = 0; i < kMaxHeader; ++i) o |= vbyte(v, p + i);
  return o == 0;
}

// ---------------------------------------------------------------- per-lane state
struct LaneState {
  uint32_t s;        // first entry start in the slice (region-relative) or kNone32
  uint32_t cnt;      // entries accepted that start in the slice (incl. a pending straddler)
  int32_t term;      // kCont or the ReadLogEntry status that stopped the walk
  uint32_t tpos;     // region-relative position of that status
  uint64_t x;        // absolute offset after the last entry that started here (term == kCont)
  uint32_t raw;      // s == kNone32: raw CRC register over the whole slice [B, Eeff); else unused
  uint32_t sflag;    // kStraddle | kSkip | kNoCrc for the last entry (x beyond the slice)
  uint32_t so;       // its region-relative start
  uint32_t scrc;     // its stored crc
  uint32_t rout;     // its CRC register at the slice end (init-based), unless kSkip/kNoCrc
};

// Tuples a lane keeps for emission (registers on the GPU).
struct LaneKeep {
  uint64_t pos[kKeep];
  uint32_t k[kKeep];
  uint32_t v[kKeep];
};

// hasless(w, 3): a byte of w is < 3 (may flag extra bytes above a true hit; prefilter only)
LDB_HD uint32_t small_bytes(uint32_t w) { return (w - 0x03030303u) & ~w & 0x80808080u; }

// Speculative start search (never decides results; see plausible_start).
LDB_HD uint32_t find_start(const View& v, int64_t B, int64_t Eeff) {
  // first window-EOF position (every later position is one too)
  int64_t pe = Eeff;
  {
    const int64_t lim = (int64_t)(v.len - v.R0) - kMaxHeader + (v.io == LDB_IO_MMAP ? 0 : 1);
    if (lim < pe) pe = lim < B ? B : lim;
  }
  // stat bytes of positions B..B+79 are bytes B+4..B+83: dwords at B+4+4q (aligned, B % 16 == 0)
  uint32_t cand[3] = {0, 0, 0};  // bit i <-> position B + i
#pragma unroll
  for (int qd = 0; qd < kS / 4; ++qd) {
    const uint32_t t = small_bytes(lds32(v, kPre + B + 4 + 4 * qd));
    const uint32_t bits = msb4(t);
    cand[qd >> 3] |= bits << (4 * (qd & 7));
  }
  const int64_t nvalid = pe - B;  // positions [B, pe) are decodable
  for (int wd = 0; wd < 3; ++wd) {
    const int64_t lo = 32 * wd;
    uint32_t m = cand[wd];
    if (nvalid <= lo) m = 0;
    else if (nvalid < lo + 32) m &= (1u << (nvalid - lo)) - 1;
    while (m) {
      const int64_t p = B + lo + __builtin_ctz(m);
      m &= m - 1;
      const EntryInfo e = classify_at(v, p);
      if (plausible_start(e)) {
        // cheap one-hop check: the implied next entry must pass the same stat-byte prefilter
        // (or lie past the staged bytes / in the header-window EOF zone)
        const uint64_t nx = (uint64_t)p + e.size;
        if (nx + 8 > (uint64_t)(kW + kHalo) || v.R0 + nx + kMaxHeader > v.len || vbyte(v, (int64_t)nx + 4) <= 2u)
          return (uint32_t)p;
        continue;
      }
      if (e.status == LDB_EOF_SENTINEL && zero_window(v, p)) return (uint32_t)p;
    }
  }
  return pe < Eeff ? (uint32_t)pe : kNone32;
}

// Process one lane's slice: start (by `force`), walk, CRC pieces, in-slice verification.
LDB_HD void lane_process(const View& v, int lane, uint32_t force, LaneState* st, LaneKeep* kp) {
  const int64_t B = (int64_t)lane * kS, E = B + kS;
  const int64_t Eeff = E < (int64_t)v.rlen ? E : (int64_t)v.rlen;
  LaneState r;
  r.s = kNone32; r.cnt = 0; r.term = kCont; r.tpos = 0; r.x = 0; r.raw = 0; r.sflag = 0; r.so = 0; r.scrc = 0;
  r.rout = 0;
  if (B >= Eeff) { *st = r; return; }          // slice entirely past the end of the file
  const uint32_t s = force == kForceSpec ? find_start(v, B, Eeff) : (force == kForceNone ? kNone32 : force);
  r.s = s;
  // a covered slice contributes its raw register; a slice with a start CRCs its prefix later
  // (lane_finish), continuing the register carried in from the entry that covers it
  if (s == kNone32) {
    r.raw = crc_segment(v, B, Eeff, 0u);
    *st = r;
    return;
  }
  int64_t o = s;
  for (;;) {
    if (o >= Eeff) { r.x = v.R0 + (uint64_t)o; break; }   // next entry starts in a later slice
    const EntryInfo e = classify_at(v, o);
    if (e.status != kCont) { r.term = e.status; r.tpos = (uint32_t)o; break; }
    const uint64_t end = (uint64_t)o + e.size;
    if (e.h.size <= 4 && e.h.crc != 0) { r.term = LDB_ERR_CRC; r.tpos = (uint32_t)o; break; }  // getEntryCrc == 0
    if (r.cnt < kKeep) {
      kp->pos[r.cnt] = pack_pos(v.R0 + (uint64_t)o, e.h);
      kp->k[r.cnt] = e.h.k_size;
      kp->v[r.cnt] = e.h.v_size;
    }
    if (end <= (uint64_t)E) {
      if (e.h.size > 4 && crc_segment(v, o + 4, (int64_t)end, 0xFFFFFFFFu) != ~e.h.crc) {  // ErrInvalidCrc
        r.term = LDB_ERR_CRC; r.tpos = (uint32_t)o; break;
      }
      r.cnt++;
      o = (int64_t)end;
      continue;
    }
    // straddles out of the slice: CRC the part inside, finish in the fold
    r.cnt++;
    r.sflag = kStraddle; r.so = (uint32_t)o; r.scrc = e.h.crc; r.x = v.R0 + end;
    if (e.h.size <= 4) r.sflag |= kNoCrc;
    else if (E - (o + 4) >= 4) r.rout = crc_segment(v, o + 4, E, 0xFFFFFFFFu);
    else r.sflag |= kSkip;
    break;
  }
  *st = r;
}

// ---------------------------------------------------------------- wave-level state (LDS)
struct WaveSh {
  LaneState ln[kLanes];
  uint32_t force[kLanes];
  uint32_t prefix[kLanes];   // exclusive prefix of emitted tuples per lane
  uint32_t inreg[kLanes];    // register carried into a lane's prefix piece by the fold chains
  uint32_t owner[kLanes];    // lane whose entry covers the prefix piece (kLanes: region entry)
};

// Link check for lane j (phase after lane_process): returns the lane to repair and its force,
// or -1 when lane j's outgoing link is consistent.  `noneMask`: bit k set iff lane k has no start.
LDB_HD int lane_link(const View& v, const WaveSh& w, int j, uint64_t noneMask, uint32_t* fix_force) {
  const LaneState& a = w.ln[j];
  if (a.s == kNone32 || a.term != kCont) return -1;
  const uint64_t xr = a.x - v.R0;           // region-relative exit (>= E_j)
  // lanes strictly between j and the landing lane must be covered
  const int m = xr >= (uint64_t)v.rlen ? kLanes : (int)(xr / kS);
  const uint64_t between = (m >= kLanes ? ~0ull : ((1ull << m) - 1)) & ~((2ull << j) - 1);
  const uint64_t bad = between & ~noneMask;
  if (bad) { *fix_force = kForceNone; return (int)ctz64(bad); }
  if (m < kLanes && w.ln[m].s != (uint32_t)xr) { *fix_force = (uint32_t)xr; return m; }
  return -1;
}

// Re-walk lane j's accepted entries beyond the kept ones (rare) and emit index tuples.
template <class Emit>
LDB_HD void lane_emit(const View& v, const LaneState& a, const LaneKeep& kp, Emit emit) {
  int64_t o = a.s;
  for (uint32_t i = 0; i < a.cnt; ++i) {
    if (i < kKeep) {
      emit(i, kp.pos[i], kp.k[i], kp.v[i]);
      o = (int64_t)(LDB_POS_OFFSET(kp.pos[i]) - v.R0) + LDB_POS_HDR(kp.pos[i]) + kp.k[i] + kp.v[i];
      continue;
    }
    const EntryInfo e = classify_at(v, o);
    emit(i, pack_pos(v.R0 + (uint64_t)o, e.h), e.h.k_size, e.h.v_size);
    o += (int64_t)e.size;
  }
}

}  // namespace ldb
