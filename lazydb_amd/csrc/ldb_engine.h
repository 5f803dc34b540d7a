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

#ifdef LDB_EMU_COUNTERS   // CPU emulator instrumentation only (tests/emu): per-lane event counts
namespace ldb { extern int g_emu_lane; extern uint32_t g_emu_cnt[8][64]; }
#define LDB_COUNT(id) (++ldb::g_emu_cnt[id][ldb::g_emu_lane & 63])
#else
#define LDB_COUNT(id) ((void)0)
#endif

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
//
// 8-byte CRC step on 11/11/10-bit chunk tables: one table set S = shift by 32 bits,
// reg' = S(S(reg ^ w0) ^ w1) (20 KB of LDS). Chained fast path (ldb_chain.h): register shifts by
// byte-indexed tables, 4 of 256 each (4 lookups per shift). Measured and rejected alternatives (DESIGN.md,
// round 4): lane-private 2-byte slicing tables with nibble-indexed shifts (k_scan_main config 3 3.55 vs
// 2.65 ms: the region pipeline is bound by its dependent lookup chains, not by bank conflicts), and a
// shift-by-64 / shift-by-32 table pair.
constexpr int kShW = 1024;                // words per chain shift table
constexpr int kTBOff = 0;                 // 2048 + 2048 + 1024: S
constexpr int kT8Off = kTBOff + 5120;     // 256: byte-at-a-time table (rare paths)
constexpr int kZSOff = kT8Off + 256;      // 4 x 256: register shift by kS zero bytes (fold chains)
constexpr int kKOff = kZSOff + 1024;      // kS + 1 (padded to 96): K[n] = register after n zero bytes from ~0
constexpr int kVSOff = kKOff + 96;        // 4 x kShW: shift by 8, 16, 32, 64 bytes (check-point shifts)
constexpr int kSCOff = kVSOff + 4 * kShW; // 5 x kShW: shift by 2, 4, 8, 16, 32 slices (lane scan)
constexpr int kZCOff = kZSOff;            // shift by 1 slice, chain layout
constexpr int kTabWords = kSCOff + 5 * kShW;
constexpr int kTabBytes = kTabWords * 4;

// Force codes for a lane (re)run.
constexpr uint32_t kForceSpec = 0xFFFFFFFEu;  // search for a plausible start
constexpr uint32_t kForceNone = 0xFFFFFFFFu;  // slice is covered by an entry started earlier

// sflag bits
constexpr uint32_t kStraddle = 1u;   // last entry started here ends beyond the slice
constexpr uint32_t kSkip = 2u;       // its CRC span starts < 4 bytes before (or after) the slice end
constexpr uint32_t kNoCrc = 4u;      // its decoded header size <= 4: getEntryCrc returns 0 (already checked)

constexpr int kOverflow = 100;       // internal: region needs more than kRegionCap tuple slots
#ifndef LDB_KWARM
#define LDB_KWARM 2
#endif
constexpr uint64_t kWarm = LDB_KWARM;   // k_scan_main: regions a wave's run starts early, processed dry (chain warm-up)
#ifndef LDB_SWALLOW_LOG2
#define LDB_SWALLOW_LOG2 18
#endif
constexpr uint64_t kWarmSwallow = 1ull << LDB_SWALLOW_LOG2;   // (256 KiB) a speculated entry whose chain leaves a region inside an
                                                // entry reaching this far ahead is taken for false (k_scan_main)

// ---------------------------------------------------------------- table building (host)
inline void build_tables(uint32_t* tab) {
  auto step_bits = [](uint32_t x, int nbits) {
    for (int k = 0; k < nbits; ++k) x = (x >> 1) ^ (kPoly & (0u - (x & 1u)));
    return x;
  };
  const int off[3] = {0, 11, 22}, wid[3] = {11, 11, 10}, base[3] = {0, 2048, 4096};
  for (int q = 0; q < 3; ++q)
    for (uint32_t v = 0; v < (1u << wid[q]); ++v) tab[kTBOff + base[q] + v] = step_bits(v << off[q], 32);
  for (int q = 0; q < 4; ++q)
    for (uint32_t b = 0; b < 256; ++b) tab[kZSOff + q * 256 + b] = step_bits(b << (8 * q), 8 * kS);
  for (uint32_t i = 0; i < 256; ++i) tab[kT8Off + i] = step_bits(i, 8);
  for (int n = 0; n < kVSOff - kKOff; ++n) tab[kKOff + n] = n <= kS ? step_bits(0xFFFFFFFFu, 8 * n) : 0u;
  auto shift_table = [&](int off, int nbytes) {
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) tab[off + q * 256 + b] = step_bits(b << (8 * q), 8 * nbytes);
  };
  for (int i = 0; i < 4; ++i) shift_table(kVSOff + i * kShW, 8 << i);
  for (int i = 0; i < 5; ++i) shift_table(kSCOff + i * kShW, kS << (i + 1));
}

// ---------------------------------------------------------------- memory views
// `buf` points at the staging buffer (region byte r lives at buf[kPre + r]); `tab` at the
// table block. Both are LDS on the GPU, plain memory in the emulator. `xw` = x^(8n) mod P,
// n = 0..kW (global memory).
struct View {
  const uint8_t* buf;
  const uint32_t* tab;
  const uint32_t* xw;
  const uint32_t* gsh;  // register-shift byte tables in global memory (build_gshift), uniform lookups
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
  const uint32_t y = tab[kTBOff + (x & 0x7FFu)] ^ tab[kTBOff + 2048 + ((x >> 11) & 0x7FFu)] ^
                     tab[kTBOff + 4096 + (x >> 22)] ^ w1;
  return tab[kTBOff + (y & 0x7FFu)] ^ tab[kTBOff + 2048 + ((y >> 11) & 0x7FFu)] ^ tab[kTBOff + 4096 + (y >> 22)];
}

LDB_HD uint32_t mask_from(uint32_t nbytes) {  // bytes [nbytes, 4) kept, nbytes in [0, 4]
  return nbytes >= 4 ? 0u : (0xFFFFFFFFu << (8 * nbytes));
}

// CRC register over region bytes [lo, hi) (hi - lo >= 1) in 8-byte steps aligned to hi, starting
// from register `init`: the register is injected (XORed) into the first 4 message bytes, which
// is exact for |M| >= 4; for |M| < 4 the unconsumed part (init >> 8|M|) is added at the end.
// init = ~0: CRC-32 span (getEntryCrc); init = 0: raw register (leading zero bytes are free).
LDB_HD uint32_t crc_segment(const View& v, int lo, int hi, uint32_t init) {
  const int L = hi - lo;
  const int n8 = (L + 7) >> 3;
  const int c = hi - 8 * n8;
  const uint32_t pad = (uint32_t)(lo - c);  // 0..7 leading bytes outside the segment
  const uint32_t m0 = mask_from(pad), m1 = pad <= 4 ? 0xFFFFFFFFu : mask_from(pad - 4);
  // init bytes land on message bytes [pad, pad+4) of the 12-byte window starting at c
  const uint64_t sh64 = (uint64_t)init << (8 * (pad & 3));
  const uint32_t ilo = (uint32_t)sh64, ihi = (uint32_t)(sh64 >> 32);
  const uint32_t i0 = pad < 4 ? ilo : 0u, i1 = pad < 4 ? ihi : ilo, i2 = pad < 4 ? 0u : ihi;
  const int a0 = c + kPre;
  int q = a0 & ~3;
  const uint32_t sh = (uint32_t)(a0 & 3);
  uint32_t d0 = lds32(v, q);
  uint32_t reg = 0;
  for (int k = 0; k < n8; ++k) {
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

// 16-byte LDS row (slices start 16-byte aligned in the staging buffer)
struct alignas(16) Row16 { uint32_t w[4]; };

// Uniform slice pass: raw CRC register (init 0) over slice bytes [B + r0, B + kS) on the slice's
// natural 8-byte grid, bytes before B + r0 masked to zero (free while the register is 0).
// Every lane runs the same kS/8 steps whatever its r0 (r0 >= kS: empty, returns 0).
// A CRC span with init ~0 over the same bytes is this value ^ K[kS - r0] (linearity).
LDB_HD uint32_t crc_slice_from(const View& v, int B, int r0) {
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  uint32_t reg = 0;
#pragma unroll
  for (int k = 0; k < kS / 16; ++k) {
    const Row16 q = row[k];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = r0 - 16 * k - 8 * h;   // bytes of this word before the piece
      const int c0 = r < 0 ? 0 : (r > 4 ? 4 : r), c1 = r < 4 ? 0 : (r > 8 ? 4 : r - 4);
      const uint32_t m0 = (uint32_t)(0xFFFFFFFFull << (8 * c0)), m1 = (uint32_t)(0xFFFFFFFFull << (8 * c1));
      reg = crc_step8(v.tab, reg, q.w[2 * h] & m0, q.w[2 * h + 1] & m1);
    }
  }
  return reg;
}

// Uniform two-chain slice pass (every lane, same kS/8 steps on the slice's natural 8-byte grid):
//   chain A keeps bytes [B, B + tA), XORs C into bytes [B + tA, B + tA + 4) and zeroes the rest:
//     A = shift(raw([B, B+tA)), kS - tA) ^ shift(C, kS - tA)   (the C >> 8L fix covers tA > kS - 4)
//   chain B keeps bytes [B + uB, B + kS), zeroes the bytes before (free while its register is 0):
//     Bv = raw([B + uB, B + kS))
// tA >= kS: A = raw of the whole slice (C must be 0); uB >= kS: Bv = 0.
LDB_HD void crc_slice2(const View& v, int B, int tA, uint32_t C, int uB, uint32_t* ra, uint32_t* rb) {
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  // per-lane boundary words, computed once: chain A keeps words < kA, the low ta bytes of word kA
  // with C injected at byte ta (its bytes past the word spill into word kA + 1); chain B keeps the
  // bytes >= ub of word kB and every word after it.
  const int kA = tA >> 3, ta = tA & 7, kB = uB >> 3, ub = uB & 7;
  const uint64_t mA = ta ? (~0ull >> (64 - 8 * ta)) : 0ull;
  const uint64_t iA = (uint64_t)C << (8 * ta);
  const uint64_t sA = ta > 4 ? ((uint64_t)C >> (8 * (8 - ta))) : 0ull;
  const uint64_t mB = ~0ull << (8 * ub);
  uint32_t a = 0, b = 0;
#pragma unroll
  for (int k2 = 0; k2 < kS / 16; ++k2) {
    const Row16 q = row[k2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 2 * k2 + h;
      const uint64_t w = ((uint64_t)q.w[2 * h + 1] << 32) | q.w[2 * h];
      const uint64_t wa = k < kA ? w : (k == kA ? ((w & mA) ^ iA) : (k == kA + 1 ? sA : 0ull));
      const uint64_t wb = k > kB ? w : (k == kB ? (w & mB) : 0ull);
      a = crc_step8(v.tab, a, (uint32_t)wa, (uint32_t)(wa >> 32));
      b = crc_step8(v.tab, b, (uint32_t)wb, (uint32_t)(wb >> 32));
    }
  }
  const int L = kS - tA;
  if (L > 0 && L < 4) a ^= C >> (8 * L);
  *ra = a;
  *rb = b;
}

// register shift by kS zero bytes (constant-distance GF(2) multiply: 4 byte-table reads)
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

// bytes of PutUvarint(ux), ux < 2^32
LDB_HD uint32_t vlen32(uint32_t ux) {
  const uint32_t bits = ux ? 32u - (uint32_t)__builtin_clz(ux) : 1u;
  return ((bits + 6u) * 147u) >> 10;   // ceil(bits / 7) for bits in [1, 32]
}

// ReadLogEntry(off) up to the CRC comparison, as the walk needs it.
struct Hot {
  int32_t status;     // kCont (decoded and readable) or the ReadLogEntry status at this position
  uint32_t crc;
  int32_t hsize;      // decodeHeader's offset (<= 4 only for degenerate headers: no CRC span)
  uint32_t esize;     // header length EncodeEntry re-emits
  uint32_t stat;
  uint32_t k, v;
  uint32_t plaus;     // plausible_start (speculation only)
  uint64_t size;      // entrySize = hsize + k + v (status == kCont)
};

LDB_HD Hot hot_from(const EntryInfo& e) {
  Hot r;
  r.status = e.status;
  r.crc = e.h.crc;
  r.hsize = e.h.size;
  r.esize = (uint32_t)e.h.enc_size;
  r.stat = e.h.stat;
  r.k = e.h.k_size;
  r.v = e.h.v_size;
  r.plaus = plausible_start(e) ? 1u : 0u;
  r.size = e.size;
  return r;
}

LDB_HD uint64_t pack_hot(uint64_t off, const Hot& h) {
  return (off & 0xFFFFFFFFFFull) | ((uint64_t)(h.hsize & 0x3F) << 40) | ((uint64_t)(h.esize & 0x3F) << 46) |
         ((uint64_t)(h.stat & 0xFF) << 52);
}

// Header-window bytes [b, b+4), b in [4, 31], from the window dwords w[0..8] (bytes 0..35):
// win_word's select chain, four words further.
LDB_HD uint32_t win_word9(const uint32_t* w, uint32_t b) {
  const uint32_t d = b >> 2;
  uint32_t lo = w[1], hi = w[2];
#pragma unroll
  for (uint32_t i = 2; i <= 7; ++i) {
    lo = d >= i ? w[i] : lo;
    hi = d >= i ? w[i + 1] : hi;
  }
  return funnel(hi, lo, b & 3u);
}

// Fast decode at region-relative p for headers whose five varints end within bytes [5, 36)
// with ts/k/v varints <= 4 bytes and expiredAt/txID <= 10 bytes (every header LazyDB's writer
// emits for sizes < 128 MiB, snowflake TxIDs included). Everything else, and every status other than kCont, goes through
// the exact byte-wise decoder (classify_entry, Go semantics).
// Returns false when the fast path cannot decide (the caller falls back to the exact decoder).
LDB_HD bool classify_fast(const View& v, int p, Hot* out) {
  const uint64_t off = v.R0 + (uint64_t)p;
  if (read_eof(v.len, v.io, (int64_t)off, kMaxHeader)) {
    out->status = LDB_EOF_WINDOW;
    out->plaus = 0;
    out->size = 0;
    return true;
  }
  {
    const int a = p + kPre;
    const int q = a & ~3;
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) d[i] = lds32(v, q + 4 * i);
    uint32_t w[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) w[i] = funnel(d[i + 1], d[i], sh);
    // terminator bits (bit i <-> window byte 4 + i), bytes 5..35
    const uint32_t M = msb4(w[1]) | (msb4(w[2]) << 4) | (msb4(w[3]) << 8) | (msb4(w[4]) << 12) | (msb4(w[5]) << 16) |
                       (msb4(w[6]) << 20) | (msb4(w[7]) << 24) | (msb4(w[8]) << 28);
    uint32_t T = (~M) & 0xFFFFFFFEu;
    uint32_t e[5];
    uint32_t prev = 0;
    bool fast = true;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
      e[f] = T ? (uint32_t)__builtin_ctz(T) : 32u;
      T &= T - 1;
      fast = fast && e[f] < 32u && e[f] - prev <= (f < 2 ? 10u : 4u);
      prev = e[f];
    }
    if (fast) {
      uint32_t val[3];
      uint32_t pe = 0, sign0 = 0;
      bool canon = true;
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        const uint32_t st = 5 + pe;               // first byte of the field (window index, 5..31)
        const uint32_t n = e[f] - pe;
        uint32_t b = win_word9(w, st & 31u);
        const uint32_t nn = n > 4 ? 4 : n;
        // the field's last byte: window byte 4 + e[f] (expiredAt / txID may be up to 10 bytes)
        const uint32_t lastb = n > 4 ? (win_word9(w, (4 + e[f]) & 31u) & 0xFFu) : ((b >> (8 * (nn - 1))) & 0xFFu);
        canon = canon && (n == 1 || lastb != 0) && (n < 10 || lastb <= 1u);   // 10 bytes: no uint64 overflow
        if (f == 0) sign0 = b & 1u;
        if (f >= 2) {
          b &= nn == 4 ? 0xFFFFFFFFu : ((1u << (8 * nn)) - 1);
          val[f - 2] = pext7(b);
        }
        pe = e[f];
      }
      if (canon) {
        Hot r;
        const int32_t ts = (int32_t)(val[0] >> 1) ^ -(int32_t)(val[0] & 1u);
        const int32_t ks = (int32_t)(val[1] >> 1) ^ -(int32_t)(val[1] & 1u);
        const int32_t vs = (int32_t)(val[2] >> 1) ^ -(int32_t)(val[2] & 1u);
        r.crc = w[0];
        r.stat = w[1] & 0xFFu;
        r.k = (uint32_t)ks;   // uint32(int64) of a value in (-2^27, 2^27)
        r.v = (uint32_t)vs;
        r.hsize = (int32_t)(5 + e[4]);
        const uint32_t tx_stat = (uint32_t)(uint16_t)ts;
        // exp + txID occupy window bytes [5, 5 + e[1]); EncodeEntry re-emits them as read
        r.esize = 5 + e[1] + vlen32(tx_stat << 1) + vlen32(r.k << 1) + vlen32(r.v << 1);
        const bool sentinel = r.crc == 0 && r.k == 0 && r.v == 0;
        const uint64_t kv = (uint64_t)r.k + (uint64_t)r.v;
        r.status = sentinel ? LDB_EOF_SENTINEL
                            : ((kv && read_eof(v.len, v.io, (int64_t)(off + (uint64_t)r.hsize), kv)) ? LDB_EOF_KV : kCont);
        r.size = (uint64_t)r.hsize + kv;
        // speculation heuristic only (results never depend on it): what LazyDB's writers emit --
        // every call site passes a user key (str.go, list.go, tx.go), so an empty key is a hint
        // that this "header" is really the tail of a CRC field (k_size read from the stat byte)
        r.plaus = (r.status == kCont && r.stat <= 2u && ts >= 0 && ts <= 2 && ks >= 1 && vs >= 0 && sign0 == 0 &&
                   (uint32_t)r.hsize == r.esize && r.crc != 0) ? 1u : 0u;
        *out = r;
        return true;
      }
    }
  }
  return false;
}

// ReadLogEntry(off) up to the CRC comparison, exact for every input.
LDB_HD Hot classify_at(const View& v, int p) {
  Hot r;
  if (classify_fast(v, p, &r)) return r;
  LDB_COUNT(3);
  return hot_from(classify_slow(v, p));
}

// 38 zero bytes at p (p + 38 inside the staged bytes)?
LDB_HD bool zero_window(const View& v, int p) {
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
  uint32_t raw;      // lane_crc chain A: covered slice: raw register of [B, Eeff); else shift(raw([B,s)) ^ C, E-s)
  uint32_t sflag;    // kStraddle | kSkip | kNoCrc for the last entry (x beyond the slice)
  uint32_t so;       // its region-relative start
  uint32_t scrc;     // its stored crc
  uint32_t rout;     // its CRC register at the slice end (init-based), unless kSkip/kNoCrc
};

// Tuples a lane keeps for emission (registers on the GPU).
struct LaneKeep {
  uint64_t pos0, pos1;
  uint32_t k0, k1, v0, v1;
  LDB_HD void put(uint32_t i, uint64_t pos, uint32_t k, uint32_t v) {
    if (i == 0) { pos0 = pos; k0 = k; v0 = v; }
    else { pos1 = pos; k1 = k; v1 = v; }
  }
};
static_assert(kKeep == 2, "LaneKeep holds two tuples");

// hasless(w, 3): a byte of w is < 3 (may flag extra bytes above a true hit; prefilter only)
LDB_HD uint32_t small_bytes(uint32_t w) { return (w - 0x03030303u) & ~w & 0x80808080u; }

// Speculative start search (never decides results; see plausible_start). Returns the start
// (or kNone32) and its decode in *h (valid when the start is not kNone32).
LDB_HD uint32_t find_start(const View& v, int B, int Eeff, Hot* h) {
  // first window-EOF position (every later position is one too)
  int pe = Eeff;
  {
    const int64_t lim = (int64_t)(v.len - v.R0) - kMaxHeader + (v.io == LDB_IO_MMAP ? 0 : 1);
    if (lim < (int64_t)pe) pe = lim < (int64_t)B ? B : (int)lim;
  }
  // stat bytes of positions B..B+79 are bytes B+4..B+83: dwords 1..20 of the rows at B. A plausible
  // start also has a non-negative ExpiredAt, so the byte after its stat byte is even (zig-zag sign
  // bit): candidates whose next byte is odd are dropped before the decode (about half the stat-byte
  // hits in random value bytes; the plausible set is unchanged, an odd byte fails the check anyway)
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  uint32_t dw[24];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const Row16 q = row[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) dw[4 * k + j] = q.w[j];
  }
  uint32_t cand[3] = {0, 0, 0};  // bit i <-> position B + i
#pragma unroll
  for (int qd = 0; qd < kS / 4; ++qd) {   // dword qd + 1 holds the stat bytes of positions 4qd..4qd+3
    const uint32_t w = dw[qd + 1], nx = (w >> 8) | (dw[qd + 2] << 24);
    cand[qd >> 3] |= msb4(small_bytes(w) & ~((nx << 7) & 0x80808080u)) << (4 * (qd & 7));
  }
  const int nvalid = pe - B;  // positions [B, pe) are decodable
  uint32_t m0 = cand[0], m1 = cand[1], m2 = cand[2];
  if (nvalid < 32) { m0 &= nvalid <= 0 ? 0u : (0xFFFFFFFFu >> (32 - nvalid)); m1 = 0; m2 = 0; }
  else if (nvalid < 64) { m1 &= nvalid == 32 ? 0u : (0xFFFFFFFFu >> (64 - nvalid)); m2 = 0; }
  else if (nvalid < 96) { m2 &= nvalid == 64 ? 0u : (0xFFFFFFFFu >> (96 - nvalid)); }
  while (m0 | m1 | m2) {
    int bit;
    if (m0) { bit = __builtin_ctz(m0); m0 &= m0 - 1; }
    else if (m1) { bit = 32 + __builtin_ctz(m1); m1 &= m1 - 1; }
    else { bit = 64 + __builtin_ctz(m2); m2 &= m2 - 1; }
    const int p = B + bit;
    LDB_COUNT(0);
    Hot e;
    // speculation only: a header the fast decoder cannot take (non-canonical or very long varints)
    // is not a plausible start; the true chain still reaches such entries through the link repair
    if (!classify_fast(v, p, &e)) continue;
    if (e.plaus) {
      // cheap one-hop check: the implied next entry must pass the same stat-byte prefilter
      // (or lie past the staged bytes / in the header-window EOF zone)
      const uint64_t nx = (uint64_t)p + e.size;
      if (nx + 8 > (uint64_t)(kW + kHalo) || v.R0 + nx + kMaxHeader > v.len || vbyte(v, (int)nx + 4) <= 2u) {
        *h = e;
        return (uint32_t)p;
      }
      continue;
    }
    if (e.status == LDB_EOF_SENTINEL && zero_window(v, p)) { *h = e; return (uint32_t)p; }
  }
  if (pe < Eeff) {
    h->status = LDB_EOF_WINDOW;
    return (uint32_t)pe;
  }
  return kNone32;
}

// Walk one lane's slice: start (by `force`), entries that start in the slice, in-slice CRC
// verification of entries that end inside it. The open pieces are CRC'd later by lane_crc.
LDB_HD void lane_walk(const View& v, int lane, uint32_t force, LaneState* st, LaneKeep* kp) {
  const int B = lane * kS, E = B + kS;
  const int Eeff = E < (int)v.rlen ? E : (int)v.rlen;
  LaneState r;
  r.s = kNone32; r.cnt = 0; r.term = kCont; r.tpos = 0; r.x = 0; r.raw = 0; r.sflag = 0; r.so = 0; r.scrc = 0;
  r.rout = 0;
  if (B < Eeff) {
    Hot e;
    e.status = kCont - 1;   // "not decoded yet"
    const uint32_t s = force == kForceSpec ? find_start(v, B, Eeff, &e) : (force == kForceNone ? kNone32 : force);
    r.s = s;
    if (s != kNone32) {
      int o = (int)s;
      for (;;) {
        if (o >= Eeff) { r.x = v.R0 + (uint64_t)o; break; }   // next entry starts in a later slice
        if (e.status == kCont - 1 || o != (int)s) { LDB_COUNT(1); e = classify_at(v, o); }
        if (e.status != kCont) { r.term = e.status; r.tpos = (uint32_t)o; break; }
        if (e.hsize <= 4 && e.crc != 0) { r.term = LDB_ERR_CRC; r.tpos = (uint32_t)o; break; }  // getEntryCrc == 0
        if (r.cnt < kKeep) kp->put(r.cnt, pack_hot(v.R0 + (uint64_t)o, e), e.k, e.v);
        const uint64_t end = (uint64_t)o + e.size;
        if (end <= (uint64_t)E) {
          LDB_COUNT(2);
          if (e.hsize > 4 && crc_segment(v, o + 4, (int)end, 0xFFFFFFFFu) != ~e.crc) {  // ErrInvalidCrc
            r.term = LDB_ERR_CRC; r.tpos = (uint32_t)o; break;
          }
          r.cnt++;
          o = (int)end;
          continue;
        }
        // straddles out of the slice: lane_crc CRCs the part inside, the folds finish it
        r.cnt++;
        r.sflag = kStraddle; r.so = (uint32_t)o; r.scrc = e.crc; r.x = v.R0 + end;
        if (e.hsize <= 4) r.sflag |= kNoCrc;
        else if (o + 4 >= E) r.sflag |= kSkip;
        break;
      }
    }
  }
  *st = r;
}

// The lane's CRC pieces in one uniform pass (crc_slice2):
//   raw  <- chain A: covered slice: raw register of the whole slice; slice with a start s:
//           shift(raw([B, s)) ^ C, E - s), C = the covering entry's expected final register
//           (inject = 1) or nothing (inject = 0: region entry / no CRC check pending);
//   rout <- chain B: the straddling entry's CRC register at the slice end (init ~0).
LDB_HD void lane_crc(const View& v, int lane, LaneState* a, uint32_t C, uint32_t inject) {
  const int B = lane * kS, E = B + kS;
  const int Eeff = E < (int)v.rlen ? E : (int)v.rlen;
  const bool open = (a->sflag & kStraddle) && !(a->sflag & (kNoCrc | kSkip)) && a->term == kCont;
  const int tA = a->s == kNone32 ? kS : (int)a->s - B;
  const int uB = open ? (int)a->so + 4 - B : kS;
  uint32_t ra, rb;
  crc_slice2(v, B, tA, inject ? C : 0u, uB, &ra, &rb);
  if (a->s == kNone32 && Eeff < E) ra = B < Eeff ? crc_segment(v, B, Eeff, 0u) : 0u;   // last slice of the file
  a->raw = ra;
  a->rout = open ? rb ^ v.tab[kKOff + (kS - uB)] : 0u;
}

// ---------------------------------------------------------------- wave-level state
// Per-lane private state (registers on the GPU; one element per lane in the emulator).
struct LanePriv {
  LaneState ln;
  LaneKeep kp;
  uint32_t force;
  uint32_t prefix;   // exclusive prefix of emitted tuples
  // fold results produced by one lane and broadcast with wp.from (no cross-lane reductions)
  uint32_t rpre;     // region prefix (the region-entry lane)
  uint32_t rout;     // register at the region end of the entry that runs past it
  uint32_t rout_set; // 1: this lane produced rout; 2: ... and its span began past its slice (kSkip)
};

// The only per-lane values other lanes read (LDS): 1 KiB per wavefront.
struct WaveSh {
  uint32_t s[kLanes];      // first entry start (link checks)
  uint32_t raw[kLanes];    // lane_crc chain A (fold chains, landing checks)
  uint32_t want[kLanes];   // ~stored crc of the lane's straddling entry (the next start lane injects it)
  uint32_t fl[kLanes];     // its sflag
};

// Link check for lane j (own state a): returns the lane to repair and its force, or -1 when
// lane j's outgoing link is consistent. `noneMask`: bit k set iff lane k has no start.
LDB_HD int lane_link(const View& v, const WaveSh& w, const LaneState& a, int j, uint64_t noneMask,
                     uint32_t* fix_force) {
  if (a.s == kNone32 || a.term != kCont) return -1;
  const uint64_t xr = a.x - v.R0;           // region-relative exit (>= E_j)
  // lanes strictly between j and the landing lane must be covered
  const int m = xr >= (uint64_t)v.rlen ? kLanes : (int)(xr / kS);
  const uint64_t between = (m >= kLanes ? ~0ull : ((1ull << m) - 1)) & ~((2ull << j) - 1);
  const uint64_t bad = between & ~noneMask;
  if (bad) { *fix_force = kForceNone; return (int)ctz64(bad); }
  if (m < kLanes && w.s[m] != (uint32_t)xr) { *fix_force = (uint32_t)xr; return m; }
  return -1;
}

// Re-walk lane j's accepted entries beyond the kept ones (rare) and emit index tuples.
template <class Emit>
LDB_HD void lane_emit(const View& v, const LaneState& a, const LaneKeep& kp, Emit emit) {
  int o = (int)a.s;
  for (uint32_t i = 0; i < a.cnt; ++i) {
    if (i < kKeep) {
      const uint64_t pos = i == 0 ? kp.pos0 : kp.pos1;
      const uint32_t k = i == 0 ? kp.k0 : kp.k1, vv = i == 0 ? kp.v0 : kp.v1;
      emit(i, pos, k, vv);
      o = (int)(LDB_POS_OFFSET(pos) - v.R0) + (int)LDB_POS_HDR(pos) + (int)(k + vv);
      continue;
    }
    const Hot e = classify_at(v, o);
    emit(i, pack_hot(v.R0 + (uint64_t)o, e), e.k, e.v);
    o += (int)e.size;
  }
}

}  // namespace ldb
