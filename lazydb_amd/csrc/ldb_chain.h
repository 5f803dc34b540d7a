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

// Timing ablations (tools/build_variants.py abl<N>; results are NOT valid in these builds):
// bit 0: main-chain CRC without table lookups, bit 1: lane scan and check without lookups,
// bit 2: no tuple stores. Checks always pass so the fast path runs.

namespace ldb {

constexpr uint32_t kOwnerOk = 8u;     // sflag: owner of the region's first start CRC-verified in-wave
constexpr uint32_t kMinFast = kS + 4; // memo (predicted starts) entries: one start per slice

// Chain state carried from one region to the next within a wavefront's run.
//
// The header memo (m_*) is a template for predicted starts: the header of an entry the lean decode
// accepted (its bytes [4, hs): Status and the five varints; decode_lean, log_entry.go:81-107). An
// entry whose header bytes [4, hs) equal the memo's decodes to the same fields, so it has the same
// size, and a log of equal-sized entries continues at x, x + size, x + 2 size, ... A chained region
// first tries exactly that chain (predict_starts); every predicted start is verified by the byte
// compare (plus its own crc field and IOController bounds), so a wrong guess only costs the compare
// and the region takes the speculative route. Any memo is a valid hypothesis: results never depend
// on where it came from.
struct ChainState {
  uint32_t on;       // 1: x / I / owner are valid
  uint32_t I;        // running CRC register (init-based) of the entry open at the region start
  uint32_t owner;    // stored crc of the entry that ends at x
  uint64_t x;        // absolute offset of the next entry start (>= region start)
  uint32_t m_meta;   // memo: bit 0 valid (a lean-decoded header), bits 1-5 header size hs, 8-15 Status
  uint32_t m_k, m_vv;   // its key/value sizes (entry size hs + k + vv)
  uint32_t m_w[3];   // its header bytes [4, 16), bytes at and past hs zeroed (hs <= 16)
  LDB_HD uint32_t m_ok() const { return m_meta & 1u; }
  LDB_HD uint32_t m_hs() const { return (m_meta >> 1) & 31u; }
  LDB_HD uint32_t m_stat() const { return (m_meta >> 8) & 0xFFu; }
  LDB_HD uint32_t m_sz() const { return m_hs() + m_k + m_vv; }
};

LDB_HD void chain_reset(ChainState& st) {
  st.on = 0; st.I = 0; st.owner = 0; st.x = 0;
  st.m_meta = 0; st.m_k = 0; st.m_vv = 0;
  st.m_w[0] = st.m_w[1] = st.m_w[2] = 0;
}

// Mask of the header bytes of dword i (bytes [4 + 4i, 8 + 4i)) that lie before hs.
LDB_HD uint32_t memo_mask(uint32_t hs, int i) {
  const int n = (int)hs - 4 - 4 * i;
  return n >= 4 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * n)));
}

// A wave-uniform value in a scalar register on the GPU (table lookups with it become scalar loads,
// counted on lgkmcnt: a vector load's vmcnt wait would also wait for the region DMA in flight).
LDB_HD uint32_t uniform(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
#else
  return x;
#endif
}

// shift_tab with a wave-uniform register on a global-memory table: on the GPU the table is read
// through the constant address space so the four lookups are scalar loads (s_load, lgkmcnt).
LDB_HD uint32_t shift_tab_uniform(const uint32_t* gtab, uint32_t r) {
  r = uniform(r);
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const uint32_t __attribute__((address_space(4))) * cptr;
  const cptr t = (cptr)gtab;
  return t[r & 0xFFu] ^ t[256 + ((r >> 8) & 0xFFu)] ^ t[512 + ((r >> 16) & 0xFFu)] ^ t[768 + (r >> 24)];
#else
  return gtab[r & 0xFFu] ^ gtab[256 + ((r >> 8) & 0xFFu)] ^ gtab[512 + ((r >> 16) & 0xFFu)] ^ gtab[768 + (r >> 24)];
#endif
}

// register shift by a fixed byte count: 4 lookups in a byte-indexed table set at `off`
LDB_HD uint32_t shift_tab(const uint32_t* tab, int off, uint32_t r) {
  return tab[off + (r & 0xFFu)] ^ tab[off + 256 + ((r >> 8) & 0xFFu)] ^ tab[off + 512 + ((r >> 16) & 0xFFu)] ^
         tab[off + 768 + (r >> 24)];
}

// register shift by 8 * n bytes, n in [0, 15] (binary decomposition over the kVSOff tables)
LDB_HD uint32_t shift_8n(const uint32_t* tab, uint32_t r, uint32_t n) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t t = shift_tab(tab, kVSOff + i * kShW, r);
    r = ((n >> i) & 1u) ? t : r;
  }
  return r;
}

// ---------------------------------------------------------------- lean header decode
// logfile.decodeHeader (log_entry.go:81-107) for the headers LazyDB's writer emits
// (db.go:473-523 -> EncodeEntry): canonical varints, expiredAt/txID <= 5 bytes, txStat one byte
// of value 0..2, key/value sizes <= 4 bytes with kSize >= 1. For such a header Go's decode is
// the plain one below, EncodeEntry re-emits the same header length, and ReadLogEntry returns
// the entry (no sentinel; this checks that the 38-byte header window and the key/value bytes
// are readable under the IOController's bound rule).
// Returns false for everything else (the exact decoder in region_process handles it).
struct Lean {
  uint32_t crc, stat, hs, k, vv;
  uint32_t w1;   // original bytes [p+4, p+8) (restored if the region falls back)
  uint32_t X;    // region-relative exit p + hs + k + vv
};

// Header-window bytes [b, b+4), b in [4, 20], from the window dwords w[0..5] (bytes 0..23).
// Written as a chain of >= selects: an equality switch over the word index is turned into a
// lookup in a private (scratch) array, whose vmcnt wait would also wait for the in-flight DMA.
LDB_HD uint32_t win_word(const uint32_t* w, uint32_t b) {
  const uint32_t d = b >> 2;
  uint32_t lo = w[1], hi = w[2];
  lo = d >= 2u ? w[2] : lo;
  hi = d >= 2u ? w[3] : hi;
  lo = d >= 3u ? w[3] : lo;
  hi = d >= 3u ? w[4] : hi;
  lo = d >= 4u ? w[4] : lo;
  hi = d >= 4u ? w[5] : hi;
  return funnel(hi, lo, b & 3u);
}

// Index of the lowest set bit, 0xFFFFFFFF for 0: v_ffbl_b32 as is (__builtin_ctz(0) is undefined,
// so the compiler adds a compare and select around it).
LDB_HD uint32_t ffbl_raw(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
#else
  return x ? (uint32_t)__builtin_ctz(x) : 0xFFFFFFFFu;
#endif
}

// dflt <= 32 (a bit count): min(ffbl, dflt) is the lowest set bit or dflt
LDB_HD uint32_t ctz_or(uint32_t x, uint32_t dflt) {
  const uint32_t b = ffbl_raw(x);
  return b < dflt ? b : dflt;
}

// varint payload of a canonical field of n in [1, 4] bytes held little-endian in b;
// *canon = minimal encoding (n == 1 or last byte nonzero)
LDB_HD uint32_t field_value(uint32_t b, uint32_t n, bool* canon) {
  n = n < 1u ? 1u : (n > 4u ? 4u : n);   // other lengths are rejected by the caller
  b = n >= 4 ? b : (b & ((1u << (8 * n)) - 1u));
  *canon = n == 1 || (b >> (8 * (n - 1))) != 0u;
  return pext7(b);
}

// The lean decode takes Go's whole varint range for ExpiredAt and TxID (up to 10 bytes each: a
// snowflake TxID, tx.go:47-56, is a 9-10 byte varint), so Tx.Commit's entries stay on the lean path.
// The decode itself over the header-window dwords w[0..8] (bytes [p, p + 36)) of the entry at image
// offset `at` (the IOController bounds); o->X is relative: p + the entry size. The sweep tier
// (ldb_sweep.h) calls it on dwords held in registers.
LDB_HD bool decode_lean_w(const uint32_t* w, uint64_t at, uint32_t p, uint64_t len, int io, Lean* o);

LDB_HD bool decode_lean(const View& v, int p, Lean* o) {
  const int a = p + kPre;
  const int q = a & ~3;
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t d[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) d[i] = lds32(v, q + 4 * i);
  uint32_t w[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) w[i] = funnel(d[i + 1], d[i], sh);
  return decode_lean_w(w, v.R0 + (uint64_t)p, (uint32_t)p, v.len, v.io, o);
}

LDB_HD bool decode_lean_w(const uint32_t* w, uint64_t at, uint32_t p, uint64_t len, int io, Lean* o) {
  // terminator bits of window bytes 5..35 (bit i <-> byte 4 + i)
  const uint32_t M = msb4(w[1]) | (msb4(w[2]) << 4) | (msb4(w[3]) << 8) | (msb4(w[4]) << 12) | (msb4(w[5]) << 16) |
                     (msb4(w[6]) << 20) | (msb4(w[7]) << 24) | (msb4(w[8]) << 28);
  uint32_t T = (~M) & 0xFFFFFFFEu;
  const uint32_t e0 = ctz_or(T, 32); T &= T - 1;
  const uint32_t e1 = ctz_or(T, 32); T &= T - 1;
  const uint32_t e2 = ctz_or(T, 32); T &= T - 1;
  const uint32_t e3 = ctz_or(T, 32); T &= T - 1;
  const uint32_t e4 = ctz_or(T, 32);
  // field lengths: expiredAt e0, txID e1-e0, txStat e2-e1 (== 1), kSize e3-e2, vSize e4-e3
  bool ok = e4 < 32u && e0 <= 10u && e1 - e0 <= 10u && e2 - e1 == 1u && e3 - e2 <= 4u && e4 - e3 <= 4u;
  const uint32_t stat = w[1] & 0xFFu;
  const uint32_t ts = win_word9(w, (4 + e2) & 31u) & 0xFFu;   // txStat byte: zz(0..2) = 0, 2, 4
  ok = ok && stat <= 2u && (ts == 0u || ts == 2u || ts == 4u) && ((w[1] >> 8) & 1u) == 0u && w[0] != 0u;
  // minimal expiredAt / txID encodings (EncodeEntry re-emits them as read only then); a 10-byte
  // varint's last byte must be 0 or 1 (binary.Varint overflows past 64 bits: decodeHeader differs)
  const uint32_t lb0 = win_word9(w, (4 + e0) & 31u) & 0xFFu, lb1 = win_word9(w, (4 + e1) & 31u) & 0xFFu;
  ok = ok && (e0 == 1u || lb0 != 0u) && (e1 - e0 == 1u || lb1 != 0u) && (e0 < 10u || lb0 <= 1u) &&
       (e1 - e0 < 10u || lb1 <= 1u);
  bool ck, cv;
  const uint32_t uk = field_value(win_word9(w, (5 + e2) & 31u), e3 - e2, &ck);
  const uint32_t uv = field_value(win_word9(w, (5 + e3) & 31u), e4 - e3, &cv);
  ok = ok && ck && cv && (uk & 1u) == 0u && uk >= 2u && (uv & 1u) == 0u;
  const uint32_t hs = 5 + e4;
  const uint32_t k = uk >> 1, vv = uv >> 1;
  const uint32_t X = p + hs + k + vv;
  ok = ok && !read_eof(len, io, (int64_t)(at + hs), k + vv);   // key/value read (log_file.go:130-139)
  ok = ok && !read_eof(len, io, (int64_t)at, kMaxHeader);   // header window (log_file.go:117-122)
  o->crc = w[0];
  o->stat = stat;
  o->hs = hs;
  o->k = k;
  o->vv = vv;
  o->w1 = w[1];
  o->X = X;
  return ok;
}

// The ReadLogEntry statuses a chain may end on inside the lean path (log_file.go:117-126): the
// header window past the file end, or the all-zero sentinel (10 zero bytes decode as crc 0,
// stat 0 and five one-byte zero varints). kCont: anything else (region_process decides).
LDB_HD int32_t lean_terminal(const View& v, uint32_t p) {
  if (read_eof(v.len, v.io, (int64_t)(v.R0 + (uint64_t)p), kMaxHeader)) return LDB_EOF_WINDOW;
  const uint32_t a = vword(v, (int)p), b = vword(v, (int)p + 4), c = vword(v, (int)p + 8) & 0xFFFFu;
  return (a | b | c) == 0u ? LDB_EOF_SENTINEL : kCont;
}

// First header candidate of slice [B, B+kS) at or after slice offset `from`: smallest p with
// byte p+4 <= 2 (a Status byte, log_entry.go:9-16), or kNone32. Speculation only.
LDB_HD uint32_t first_cand(const View& v, int B, uint32_t from = 0) {
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  uint32_t best = 0xFFFFFFFFu;
  const uint32_t lo = from << 3;   // bit index of position `from` in the (qd << 5 | byte bit) order
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const Row16 q = row[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qd = 4 * k + j - 1;   // dword qd + 1 of the slice holds the stat bytes of positions 4qd..4qd+3
      if (qd < 0 || qd >= kS / 4) continue;
      uint32_t m = small_bytes(q.w[j]);   // lowest flagged byte is exact
      // drop positions before `from` (only their flags can be borrow artefacts of a lower hit)
      const int rel = (int)lo - (qd << 5);
      m = rel <= 0 ? m : (rel >= 32 ? 0u : (m & (0xFFFFFFFFu << rel)));
      const uint32_t c = ffbl_raw(m) | ((uint32_t)qd << 5);   // no hit: 0xFFFFFFFF
      best = c < best ? c : best;
    }
  }
  return best == 0xFFFFFFFFu ? kNone32 : (uint32_t)B + (best >> 3);
}

// Raw register over the slice (natural 8-byte grid) as two independent chains, bytes [0, 48)
// (steps 0-5) and [48, 80) (steps 6-9), joined by one shift of 32 bytes: half the dependent LDS
// round trips of one 10-step chain. Also keeps, for the owner check, the register of the chain
// holding step kb just before that step (*cap) and the step's word (*wc); *ya = the first chain.
constexpr int kSplit = 6;   // steps in the first chain
static_assert(kS == 80 && kSplit == 6, "slice split: 48 + 32 bytes (kVSOff shift-by-32 joins them)");

struct SliceRows { Row16 q[kS / 16]; };

LDB_HD SliceRows load_rows(const View& v, int B) {
  const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + B);
  SliceRows r;
#pragma unroll
  for (int k2 = 0; k2 < kS / 16; ++k2) r.q[k2] = row[k2];
  return r;
}

// kb == 10 (lane 63, a start in the region's last 4 bytes): the capture is after the whole slice,
// over the 8 bytes past it (w10, from the staging buffer's halo).
LDB_HD void crc_slice_cap(const uint32_t* tab, const SliceRows& rows, uint32_t kb, uint32_t* y, uint32_t* ya,
                          uint32_t* cap, uint64_t* wc, uint64_t w10 = 0) {
  const Row16* q = rows.q;
  uint32_t ra = 0, rb = 0, c = 0;
  uint64_t cw = w10;
#pragma unroll
  for (int k = 0; k < kSplit; ++k) {   // interleaved: step k of chain A, step kSplit + k of chain B
    {
      const uint64_t w = ((uint64_t)q[k >> 1].w[2 * (k & 1) + 1] << 32) | q[k >> 1].w[2 * (k & 1)];
      c = (uint32_t)k == kb ? ra : c;
      cw = (uint32_t)k == kb ? w : cw;
      ra = crc_step8(tab, ra, (uint32_t)w, (uint32_t)(w >> 32));
    }
    const int kbb = kSplit + k;
    if (kbb < kS / 8) {
      const uint64_t w = ((uint64_t)q[kbb >> 1].w[2 * (kbb & 1) + 1] << 32) | q[kbb >> 1].w[2 * (kbb & 1)];
      c = (uint32_t)kbb == kb ? rb : c;
      cw = (uint32_t)kbb == kb ? w : cw;
      rb = crc_step8(tab, rb, (uint32_t)w, (uint32_t)(w >> 32));
    }
  }
  *ya = ra;
  *y = shift_tab(tab, kVSOff + 2 * kShW, ra) ^ rb;
  *cap = kb == (uint32_t)(kS / 8) ? rb : c;   // chain B's register after the slice
  *wc = cw;
}

// Raw register over the whole slice (two chains as above).
LDB_HD uint32_t crc_slice_raw2(const uint32_t* tab, const SliceRows& rows) {
  uint32_t y, ya, cap;
  uint64_t wc;
  crc_slice_cap(tab, rows, 0, &y, &ya, &cap, &wc);
  return y;
}

// Per-lane registers of the chained path.
struct ChainPriv {
  uint32_t s;       // region-relative FIRST entry start in this slice, or kNone32
  uint32_t X;       // the exit of the slice's LAST entry (the lane's link to the next start lane)
  uint32_t crc, k, vv, w1, hs, stat;   // the last entry's header (its owner role, the summary, the memo)
  uint32_t sl;      // the last entry's start (= s when the slice holds one start)
  uint32_t cnt;     // entries starting in the slice (round 4: several, when entries end inside it)
  uint32_t pre;     // exclusive prefix of cnt over the lanes (tuple slots)
  uint32_t wo;      // ~crc of the first start's owner (injected at [s, s+4))
  uint32_t kb;      // check: capture step (or 0), chk: 1 if this lane checks an owner
  uint32_t chk;
  uint32_t chkB;    // 1: this lane also checks the previous lane's single start in that lane's last 4
                    // bytes (at its step 0); 2: a local CRC of an inner entry failed (the region declines)
  uint64_t mlo;     // bytes of the capture step's word that precede the checked entry's CRC span
  uint64_t wc;      // that word
  uint64_t wB;      // chkB: the slice's first 8 bytes, those at or past that start's CRC span masked
  uint32_t y, ya, cap, O, yB;
};

// Round 4: a slice may hold several entry starts. From the lane's first start p (decode_lean in e), an
// entry that ends inside the slice is followed by the next at its exit, and so on; the lane keeps its
// first start, the last entry's fields and the count. Returns false when such an exit does not decode as
// a lean header (a terminal, a non-canonical or long-varint header, or a false speculative start): the
// lane then has no start (region_process decides a region the true chain cannot cross that way).
// Rounds 1-3 declined any region with an entry < kMinFast = 84 B (two starts in one slice); LazyDB's
// writers emit many (a Delete is 21 B): 98 % of a writer-realistic log's regions went to region_process.
template <class CP>
LDB_HD bool lean_walk(const View& v, int l, uint32_t p, const Lean& e, CP& c) {
  const uint32_t E = (uint32_t)(l * kS + kS);
  Lean cur = e;
  uint32_t q = p, n = 1;
  while (cur.X < E) {
    Lean nx;
    if (!decode_lean(v, (int)cur.X, &nx)) return false;
    q = cur.X;
    cur = nx;
    ++n;
  }
  c.s = p; c.sl = q; c.cnt = n;
  c.X = cur.X; c.crc = cur.crc; c.k = cur.k; c.vv = cur.vv; c.w1 = cur.w1; c.hs = cur.hs; c.stat = cur.stat;
  return true;
}

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
template <int I, class WP, class CPriv>
LDB_HD void scan_step(WP& wp, const uint32_t* tab, CPriv cpriv) {
  constexpr int off = I == 0 ? kZCOff : kSCOff + (I - 1) * kShW;
  wp.template shfl_up<(1 << I)>([&](int l) { return cpriv(l).O; },
                                [&](int l, uint32_t t, bool valid) { if (valid) cpriv(l).O ^= shift_tab(tab, off, t); });
}

// Segmented scan: lanes below `seg` and lanes from `seg` on are combined separately (seg = 0:
// one segment).
template <int I, class WP, class CPriv>
LDB_HD void scan_step_seg(WP& wp, const uint32_t* tab, CPriv cpriv, int seg) {
  constexpr int off = I == 0 ? kZCOff : kSCOff + (I - 1) * kShW;
  constexpr int d = 1 << I;
  wp.template shfl_up<d>([&](int l) { return cpriv(l).O; }, [&](int l, uint32_t t, bool valid) {
    if (valid && (l < seg || l - d >= seg)) cpriv(l).O ^= shift_tab(tab, off, t);
  });
}

template <class WP, class CPriv>
LDB_HD void lane_scan(WP& wp, const uint32_t* tab, CPriv cpriv, int seg = 0) {
  scan_step_seg<0>(wp, tab, cpriv, seg);
  scan_step_seg<1>(wp, tab, cpriv, seg);
  scan_step_seg<2>(wp, tab, cpriv, seg);
  scan_step_seg<3>(wp, tab, cpriv, seg);
  scan_step_seg<4>(wp, tab, cpriv, seg);
  scan_step_seg<5>(wp, tab, cpriv, seg);
}

// Tree reduction of the G-chain (the up-sweep of a scan): after step i, every lane l with its low
// i + 1 bits set holds the register of slices [l - 2^(i+1) + 1, l]; lane 63 ends with the whole
// region. A covered region needs only that total: the 63 combines cost 1/5 of the scan's lookups
// (lanes that do not combine stay off the LDS).
template <int I, class WP, class CPriv>
LDB_HD void reduce_step(WP& wp, const uint32_t* tab, CPriv cpriv) {
  constexpr int off = I == 0 ? kZCOff : kSCOff + (I - 1) * kShW;
  constexpr int d = 1 << I;
  wp.template shfl_up<d>([&](int l) { return cpriv(l).O; }, [&](int l, uint32_t t, bool valid) {
    if (valid && (l & (2 * d - 1)) == 2 * d - 1) cpriv(l).O ^= shift_tab(tab, off, t);
  });
}

template <class WP, class CPriv>
LDB_HD void lane_reduce(WP& wp, const uint32_t* tab, CPriv cpriv) {
  reduce_step<0>(wp, tab, cpriv);
  reduce_step<1>(wp, tab, cpriv);
  reduce_step<2>(wp, tab, cpriv);
  reduce_step<3>(wp, tab, cpriv);
  reduce_step<4>(wp, tab, cpriv);
  reduce_step<5>(wp, tab, cpriv);
}

// Zero-region shortcut (k_scan_main and the emulator call it before region_chained): a speculative
// region (!st.on) whose bytes and halo are all zero -- the preallocated tail of a log file,
// iocontroller/fileio.go:66-68 -- has no plausible start (every candidate decodes with kSize == 0),
// so region_chained would end in covered(false) with raw register 0. zero_region() decides that
// with one 16-B LDS read per 16 bytes and a ballot, without the candidate rounds and the CRC pass.
// Only for full regions whose halo lies inside the file (past it the buffer holds other bytes).
template <class WP>
LDB_HD bool zero_region(WP& wp, const View& v) {
  if (v.rlen != (uint32_t)kW || v.R0 + (uint64_t)(kW + kHalo) > v.len) return false;
  return !wp.ballot([&](int l) {
    const Row16* row = reinterpret_cast<const Row16*>(v.buf + kPre + l * kS);
    uint32_t o = 0;
    for (int k2 = 0; k2 < kS / 16; ++k2) o |= row[k2].w[0] | row[k2].w[1] | row[k2].w[2] | row[k2].w[3];
    if (l < kHalo / 16) {
      const Row16 h = reinterpret_cast<const Row16*>(v.buf + kPre + kW)[l];
      o |= h.w[0] | h.w[1] | h.w[2] | h.w[3];
    }
    return o != 0;
  });
}

LDB_HD RegionSum zero_summary() {   // covered(false) of an all-zero region
  RegionSum r;
  r.start = kNone64; r.exitp = 0; r.soff = 0; r.status = kCont; r.count = 0;
  r.rpre = 0; r.rout = 0; r.scrc = 0; r.sflag = 0;
  return r;
}

// Predicted starts of a chained region (see ChainState): lane l's candidate is the first chain
// position x + j * m_sz at or after its slice start. Returns true when every candidate inside the
// region verifies against the memo; then cpriv(l).s / X / crc / k / vv / w1 / hs / stat are set for
// the starting lanes (kNone32 elsewhere) and sh.s mirrors them. Returns false (nothing else
// changed) as soon as one candidate does not verify: the region then takes the speculative route.
template <class WP, class CPriv>
LDB_HD bool predict_starts(WP& wp, const View& v, WaveSh& sh, const ChainState& st, uint32_t xr, CPriv cpriv) {
  const uint32_t hs = st.m_hs(), kv = st.m_k + st.m_vv, sz = hs + kv, stat = st.m_stat();
  // floor(n / sz) for n < kW: (n + 0.5) / sz lies at least 0.5 / sz from the integers around it,
  // far beyond the rounding error of the float reciprocal
  const float rsz = 1.0f / (float)sz;
  const uint32_t k0 = memo_mask(hs, 0), k1 = memo_mask(hs, 1), k2 = memo_mask(hs, 2);
  const uint64_t bad = wp.ballot([&](int l) {
    ChainPriv& c = cpriv(l);
    const uint32_t B = (uint32_t)(l * kS);
    uint32_t p = kNone32;
    if (B <= xr) {
      p = xr < B + (uint32_t)kS ? xr : kNone32;
    } else {
      const uint32_t q = (uint32_t)(((float)(B - xr - 1) + 0.5f) * rsz);   // floor((B - xr - 1) / sz)
      p = xr + (q + 1) * sz;
      p = p < B + (uint32_t)kS ? p : kNone32;
    }
    c.s = kNone32;
    c.cnt = 0;
    if (p == kNone32) return false;
    const int a = (int)p + kPre;
    const int qd = a & ~3;
    const uint32_t sh4 = (uint32_t)(a & 3);
    uint32_t d[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) d[i] = lds32(v, qd + 4 * i);
    const uint32_t w0 = funnel(d[1], d[0], sh4), w1 = funnel(d[2], d[1], sh4), w2 = funnel(d[3], d[2], sh4);
    const uint32_t w3 = funnel(d[4], d[3], sh4);
    const uint64_t off = v.R0 + (uint64_t)p;
    const bool ok = w0 != 0u && ((w1 ^ st.m_w[0]) & k0) == 0u && ((w2 ^ st.m_w[1]) & k1) == 0u &&
                    ((w3 ^ st.m_w[2]) & k2) == 0u &&
                    !read_eof(v.len, v.io, (int64_t)off, kMaxHeader) &&            // log_file.go:117-122
                    !read_eof(v.len, v.io, (int64_t)(off + hs), kv);               // log_file.go:130-139
    if (ok) {
      c.s = p; c.X = p + sz; c.crc = w0; c.k = st.m_k; c.vv = st.m_vv; c.w1 = w1; c.hs = hs; c.stat = stat;
      c.sl = p; c.cnt = 1;   // memo entries are >= kMinFast: one start per slice
    }
    return !ok;
  });
  if (bad) {
    wp.each([&](int l) { cpriv(l).s = kNone32; cpriv(l).cnt = 0; });
    return false;
  }
  wp.each([&](int l) { sh.s[l] = cpriv(l).s; });
  return true;
}

// The lean path for one region, in one of two modes:
//   chained (st.on): the chain enters at st.x with the CRC state st.I / st.owner; the owner of the
//     region's first start is CRC-checked here (kOwnerOk);
//   speculative (!st.on; a run's first region, or after region_process): every lane speculates,
//     the first plausible start L0 is taken as the chain's entry. Its owner is unknown, so its
//     stored-crc field is rewritten to 0 and the region reports the A-form prefix register
//     rpre = shift(raw([R0, s_L0)), end of L0's slice - s_L0) for k_combine (as region_process
//     does); the lane scan is segmented at L0 so the G-chain starts clean there. k_link / k_repair
//     verify the speculative entry like any region_process result.
// Returns false (buffer restored, state untouched) when the region must go through region_process.
// On success stores the summary, emits the region's tuples and advances `st` to chained mode.
// `release()` is called once the staging buffer is no longer read (the caller may start refilling
// it); if the region must then fall back, `restage()` reloads the region into the buffer first.
// Once the region's starts are final, `emit(valid, slot, pos, k, v)` is called exactly once per
// lane (valid: the lane's tuple), before the CRC work and before `release()`: the tuple fields die
// early, and a region that then declines is redone by region_process, which rewrites its slots
// (k_compact reads only as many as the final summary counts). A covered region emits nothing. On
// success `store(r)` writes the region summary (called by every lane with the same r) after
// `release()`: one store instruction per region after the next region's DMA, which the GPU
// caller's counted vmcnt wait relies on (ldb_scan.hip).
template <class WP, class CPriv, class Emit, class Free, class Restage, class Store>
LDB_HD bool region_chained(WP& wp, const View& v, uint8_t* wbuf, WaveSh& sh, ChainState& st, CPriv cpriv, Emit emit,
                           Free release, Restage restage, Store store) {
  // st.on: 0 = speculative (entry and owner unknown), 1 = chained (entry x, owner's CRC state I),
  // 2 = entry x known but its owner verified elsewhere (the replay's first region after the run
  // prefix, or region 0 with x = 0): start discovery as chained, CRC handling as speculative
  const bool known = st.on != 0, spec = st.on != 1;
  if (known && st.x < v.R0) return LDB_DECLINE(1);
  // covered region: raw register of the whole region (rpre); chained mode also advances st.I
  auto covered = [&](bool chained) {
    const uint32_t Ishift = chained ? shift_tab_uniform(v.gsh, st.I) : 0u;   // build_gshift kGsW: one region
    // the slice's rows go to registers and the buffer is released at once: the next region's DMA
    // overlaps this region's CRC chains, scan and summary
    wp.each([&](int l) {
      const SliceRows rows = load_rows(v, l * kS);
      release();
      cpriv(l).O = crc_slice_raw2(v.tab, rows);
    });
    // the region's register is lane 63's; a partial region (the file's last) needs a prefix as well
    if (v.rlen == (uint32_t)kW) lane_reduce(wp, v.tab, cpriv);
    else lane_scan(wp, v.tab, cpriv);
    const uint32_t raw = wp.from(kLanes - 1, [&](int l) { return cpriv(l).O; });
    wp.stamp(16);
    RegionSum r;
    r.start = kNone64; r.exitp = 0; r.soff = 0; r.status = kCont; r.count = 0;
    r.rpre = raw; r.rout = 0; r.scrc = 0; r.sflag = 0;
    // the file ends in the region: raw register of [R0, len) (rare). The buffer is still intact
    // although released: a partial region is the file's last, the last of its run (no refill).
    if (v.rlen < (uint32_t)kW) {
      const int q = (int)(v.rlen / kS), n = (int)(v.rlen % kS);
      uint32_t reg = q > 0 ? wp.from(q - 1, [&](int l) { return cpriv(l).O; }) : 0u;
      if (n) reg = multmodp(v.xw[n], reg);
      uint32_t part = 0;
      for (int i = 0; i < n; ++i) part = crc_byte(v.tab + kT8Off, part, vbyte(v, q * kS + i));
      r.rpre = reg ^ part;
    }
    store(r);
    if (chained) st.I = Ishift ^ raw;
  };
  uint32_t xr = 0;
  int lt = -1;
  if (known) {
    const uint64_t xr64 = st.x - v.R0;
    if (xr64 >= (uint64_t)kW) {   // the open entry runs through the region: no header can start here
      // entry known but CRC state not (st.on == 2): the region's raw register goes to k_combine, which
      // carries the open entry's check across it; the chain state stays as it is
      covered(!spec);
      return true;
    }
    xr = (uint32_t)xr64;
    lt = (int)(xr / kS);
  }
  // ---- predicted starts (memo of equal headers, see ChainState)
  const bool predicted = known && st.m_ok() && predict_starts(wp, v, sh, st, xr, cpriv);
#ifdef LDB_EMU_COUNTERS
  if (known) ++g_chain_why[predicted ? 14 : 15];   // chained regions with / without a verified prediction
  if (known && st.m_ok()) ++g_chain_why[13];          // ... of which a prediction was tried
#endif
  uint32_t tpos = kNone32;
  int32_t tstat = kCont;
  uint64_t starts = 0;
  if (predicted) {
    wp.each([&](int l) { cpriv(l).chk = 0; });
    starts = wp.ballot([&](int l) { return cpriv(l).s != kNone32; });
  } else {
  // ---- speculation: the entry lane decodes at x, later lanes (all lanes when speculative) at
  // their first candidate
  // chained: each lane decodes its first candidate (the pointer round recovers true starts behind
  // a false candidate); speculative: lanes keep trying their next candidate until one decodes as
  // a plausible header, since the region's entry lane L0 has no pointer to recover from
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    c.s = kNone32;
    c.cnt = 0;
    c.chk = 0;
    c.X = l == lt ? xr : (l > lt ? first_cand(v, l * kS) : kNone32);   // candidate (X reused)
  });
  for (int it = 0; it < (known ? 1 : 6); ++it) {
    wp.each([&](int l) {
      ChainPriv& c = cpriv(l);
      const uint32_t p = c.s == kNone32 ? c.X : kNone32;
      if (p == kNone32) return;
      Lean e;
      if (!(decode_lean(v, (int)p, &e) && lean_walk(v, l, p, e, c))) {
        const uint32_t nxt = p + 1 - (uint32_t)(l * kS);
        c.X = (!known && nxt < (uint32_t)kS) ? first_cand(v, l * kS, nxt) : kNone32;
      }
    });
    if (known || !wp.ballot([&](int l) { return cpriv(l).s == kNone32 && cpriv(l).X != kNone32; })) break;
  }
  wp.each([&](int l) { sh.s[l] = cpriv(l).s; });
  wp.stamp(10);
  // A chain may end inside the region on a terminal status (lean_terminal): tpos / tstat. Its last
  // entry's owner check then runs at a check-only "pseudo start" at tpos (rewritten like a start,
  // no tuple, not in `starts`).
  if (known && wp.from(lt, [&](int l) { return cpriv(l).s; }) == kNone32) {
    tstat = lean_terminal(v, xr);
    if (tstat == kCont) return LDB_DECLINE(2);
    tpos = xr;   // the chain enters on its terminal: nothing in the region is on it
    wp.each([&](int l) { cpriv(l).s = kNone32; cpriv(l).cnt = 0; sh.s[l] = kNone32; });
  }
  if (tpos == kNone32) {
  // ---- pointer round: a lane without a plausible first candidate that the nearest start below
  // lands in decodes at that exit (typically a true start whose first candidate was a stored-crc
  // byte <= 2); one batched pass instead of one link repair per lane
  {
    wp.each([&](int l) { sh.raw[l] = cpriv(l).s != kNone32 ? cpriv(l).X : kNone32; });   // exits
    const uint64_t sts = wp.ballot([&](int l) { return cpriv(l).s != kNone32; });
    auto target = [&](int l) -> uint32_t {
      const uint64_t below = sts & ((1ull << l) - 1);
      if (cpriv(l).s != kNone32 || !below) return kNone32;
      const uint32_t X = sh.raw[63 - (int)__builtin_clzll(below)];
      return X < (uint32_t)kW && (int)(X / kS) == l ? X : kNone32;
    };
    if (wp.ballot([&](int l) { return target(l) != kNone32; })) {
      wp.each([&](int l) {
        ChainPriv& c = cpriv(l);
        const uint32_t X = target(l);
        if (X != kNone32) {
          Lean e;
          if (decode_lean(v, (int)X, &e)) lean_walk(v, l, X, e, c);
        }
      });
      wp.each([&](int l) { sh.s[l] = cpriv(l).s; });
    }
  }
  // ---- links from the entry lane: each start's exit is the next start, no start in between
  for (int it = 0;; ++it) {
    starts = wp.ballot([&](int l) { return cpriv(l).s != kNone32; });
    const uint64_t sts = starts;
    const int j = wp.first([&](int l) {
      const ChainPriv& c = cpriv(l);
      if (c.s == kNone32) return false;
      const int m = c.X >= (uint32_t)kW ? kLanes : (int)(c.X / kS);
      const uint64_t between = (m >= kLanes ? ~0ull : ((1ull << m) - 1)) & ~((2ull << l) - 1);
      return (between & sts) != 0 || (m < kLanes && sh.s[m] != c.X);
    });
    if (j < 0) break;
    if (it == 8) return LDB_DECLINE(5);   // one false candidate repaired per pass
    const uint32_t Xj = wp.from(j, [&](int l) { return cpriv(l).X; });
    const int m = Xj >= (uint32_t)kW ? kLanes : (int)(Xj / kS);
    wp.each([&](int l) {
      ChainPriv& c = cpriv(l);
      if (l > j && l < m) c.s = kNone32;
      if (l == m) {
        Lean e;
        c.s = kNone32;
        c.cnt = 0;
        if (decode_lean(v, (int)Xj, &e)) lean_walk(v, l, Xj, e, c);
      }
      sh.s[l] = c.s;
    });
    if (m < kLanes && wp.from(m, [&](int l) { return cpriv(l).s; }) == kNone32) {
      // the verified chain from j ends at Xj unless a valid entry the lean decode rejects starts there
      tstat = lean_terminal(v, Xj);
      if (tstat == kCont) return LDB_DECLINE(6);
      tpos = Xj;
      wp.each([&](int l) {
        if (l > j) { cpriv(l).s = kNone32; cpriv(l).cnt = 0; }
        sh.s[l] = cpriv(l).s;
      });
      starts = wp.ballot([&](int l) { return cpriv(l).s != kNone32; });
      break;
    }
  }
  }   // tpos == kNone32
  }   // !predicted
  wp.stamp(11);
  if (!starts && tpos == kNone32) {   // speculative, no plausible header anywhere: a covered region
    covered(false);
    return true;
  }
  if (tpos != kNone32) {   // the pseudo start (see above)
    const int mt = (int)(tpos / kS);
    wp.each([&](int l) {
      ChainPriv& c = cpriv(l);
      if (l == mt) { c.s = tpos; c.sl = tpos; c.X = tpos; c.crc = 0; c.w1 = 0; c.cnt = 0; }
      sh.s[l] = c.s;
    });
  }
  const int L0 = known ? lt : (int)__builtin_ctzll(starts);
  const uint32_t sL0 = wp.from(L0, [&](int l) { return cpriv(l).s; });
  const int z = starts ? 63 - (int)__builtin_clzll(starts) : L0;
  const uint32_t sz = wp.from(z, [&](int l) { return cpriv(l).sl; });   // the region's last entry start
  // the next regions' memo: the region's last entry (the owner of the next x), read while the
  // staging buffer still holds this region (a predicted region keeps the memo it verified against)
  // Only a region whose first and last entries look alike (same size and leading header bytes) sets
  // a memo to predict with: logs of varying entry sizes then never pay for compares that fail.
  ChainState nm = st;
  if (!predicted && tpos == kNone32 && starts) {
    nm.m_meta = 0;
    if (z != L0) {
      const uint32_t esz = wp.from(z, [&](int l) { return cpriv(l).X; }) - sz;
      const uint32_t hsz = uniform(wp.from(z, [&](int l) { return cpriv(l).hs; }));
      const uint32_t kz = wp.from(z, [&](int l) { return cpriv(l).k; });
      const uint32_t vz = wp.from(z, [&](int l) { return cpriv(l).vv; });
      const uint32_t w1z = wp.from(z, [&](int l) { return cpriv(l).w1; });
      const bool alike = wp.from(L0, [&](int l) {
        const ChainPriv& c = cpriv(l);
        return (uint32_t)(c.cnt == 1 && c.X - c.s == esz && c.hs == hsz && c.k == kz && c.vv == vz && c.w1 == w1z);
      }) != 0u;
      if (alike && esz >= kMinFast && hsz <= 16u) {
        nm.m_meta = uniform(1u | (hsz << 1) | (wp.from(z, [&](int l) { return cpriv(l).stat; }) << 8));
        nm.m_k = uniform(kz);
        nm.m_vv = uniform(vz);
#pragma unroll
        for (int i = 0; i < 3; ++i) nm.m_w[i] = uniform(vword(v, (int)sz + 4 + 4 * i)) & memo_mask(hsz, i);
      }
    }
  }
  // ---- tuples (see emit above). A lane with several starts walks them again (decode_lean on the
  // staging buffer, unmodified until the rewrite below), emits each, and CRC-checks every entry that
  // ends inside its slice right here (crc_segment, init ~0 against ~stored crc): such an entry's owner
  // check needs no G-chain capture. A failure declines the region before any byte is rewritten.
  auto cnt_of = [&](int l) { return ((starts >> l) & 1u) ? cpriv(l).cnt : 0u; };
  const bool multi = wp.ballot([&](int l) { return cnt_of(l) > 1u; }) != 0;
  if (multi) wp.excl_prefix(cnt_of, [&](int l, uint32_t x) { cpriv(l).pre = x; });
  auto pos_of = [&](uint32_t s0, uint32_t hs0, uint32_t st0) {
    return ((v.R0 + s0) & 0xFFFFFFFFFFull) | ((uint64_t)(hs0 & 0x3F) << 40) | ((uint64_t)(hs0 & 0x3F) << 46) |
           ((uint64_t)(st0 & 0xFF) << 52);
  };
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    const bool valid = ((starts >> l) & 1u);   // an entry (not the pseudo start)
    c.chkB = 0;
    if (!multi || c.cnt <= 1) {
      const uint32_t slot = multi ? c.pre : (uint32_t)__builtin_popcountll(starts & ((1ull << l) - 1));
      emit(valid, slot, pos_of(c.s, c.hs, c.stat), c.k, c.vv);
      return;
    }
    uint32_t q = c.s;
    for (uint32_t i = 0; i < c.cnt; ++i) {
      Lean e;
      decode_lean(v, (int)q, &e);   // (decoded before: a start of the lane's walk)
      emit(valid, c.pre + i, pos_of(q, e.hs, e.stat), e.k, e.vv);
      if (i + 1 < c.cnt && crc_segment(v, (int)q + 4, (int)e.X, 0xFFFFFFFFu) != ~e.crc) c.chkB = 2;   // ErrInvalidCrc
      q = e.X;
    }
  });
  if (multi && wp.ballot([&](int l) { return cpriv(l).chkB == 2u; })) return LDB_DECLINE(9);
  // The last start's 8-byte rewrite may run past the region end (into the staged halo):
  //   kW - sz in (4, 8): its CRC-init bytes straddle the end; the true init-based register at the
  //     region end is the G-chain's ^ (~0 >> 8 * (bytes of the init inside the region));
  //   kW - sz <= 4: its CRC span starts at/after the region end (region_process's kSkip case,
  //     k_combine finishes it); its owner is checked in lane 63 over the halo (capture step 10).
  const uint32_t tail = (uint32_t)kW - sz;
  // ---- owners, check assignment, buffer rewrite
  // sh.want: ~crc of each lane's LAST start (the owner of the next start above); sh.fl: a lane's start
  // when it holds exactly one (or the pseudo start), whose owner check may fall in the next lane
  wp.each([&](int l) {
    const ChainPriv& c = cpriv(l);
    sh.want[l] = ~c.crc;
    sh.fl[l] = c.s != kNone32 && c.cnt <= 1 ? c.s : kNone32;
  });
  const uint32_t want_x = spec ? 0u : ~st.owner;   // speculative: the entry's stored crc field becomes 0
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    const uint64_t below = starts & ((1ull << l) - 1);
    c.wo = below ? sh.want[63 - (int)__builtin_clzll(below)] : want_x;
    const uint32_t B = (uint32_t)(l * kS);
    uint32_t cs = kNone32;
    if (c.s != kNone32 && (c.s + 4 < B + kS || l == kLanes - 1)) cs = c.s;   // lane 63: P may be past E (halo)
    // speculative: L0's owner is checked by k_combine (rpre); its capture only yields the prefix
    c.chk = cs != kNone32 && !(spec && cs == sL0);
    const uint32_t rel = cs != kNone32 ? cs + 4 - B : 0u;   // [0, kS + 4): kb == 10 only in lane 63
    c.kb = rel >> 3;
    const uint32_t nb = rel & 7u;
    c.mlo = nb ? (~0ull >> (64 - 8 * nb)) : 0ull;
    // the previous lane's single start in that lane's last 4 bytes: its owner's check point lies in this
    // slice, at step 0 (the register before it is 0); kept apart from this lane's own capture
    const uint32_t sb = l > 0 ? sh.fl[l - 1] : kNone32;
    const uint32_t nbB = sb != kNone32 && sb + 4 >= B ? sb + 4 - B : 8u;   // 0..3, or 8: none
    c.chkB = nbB < 8u && !(spec && sb == sL0) ? 1u : 0u;
    c.wB = c.chkB && nbB ? (~0ull >> (64 - 8 * nbB)) : 0ull;   // the mask until the rows are read
    if (c.s == kNone32) return;
    if (c.cnt <= 1) {
      rewrite8(wbuf, c, true);
      return;
    }
    uint32_t q = c.s, own = c.wo;   // every start of the slice: [s, s+4) := ~crc(owner), [s+4, s+8) ^= ~0
    for (uint32_t i = 0; i < c.cnt; ++i) {
      Lean e;
      decode_lean(v, (int)q, &e);
      uint8_t* b = wbuf + kPre + q;
      const uint32_t hi = ~e.w1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        b[k] = (uint8_t)(own >> (8 * k));
        b[4 + k] = (uint8_t)(hi >> (8 * k));
      }
      own = ~e.crc;
      q = e.X;
    }
  });
  wp.stamp(12);
  // ---- one CRC chain per lane, lane scan, owner checks
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    const SliceRows rows = load_rows(v, l * kS);   // the (rewritten) slice, the buffer's last read
    const uint64_t w10 = (l == kLanes - 1 && c.kb == (uint32_t)(kS / 8))
                             ? (((uint64_t)vword(v, kW + 4) << 32) | vword(v, kW)) : 0ull;   // halo
    c.wB &= ((uint64_t)rows.q[0].w[1] << 32) | rows.q[0].w[0];
    release();
    crc_slice_cap(v.tab, rows, c.kb, &c.y, &c.ya, &c.cap, &c.wc, w10);
  });
  wp.stamp(13);
  uint32_t chainA = 0;   // speculative: shift(raw([B_L0, s_L0)), E_L0 - s_L0), lane L0's prefix contribution
  if (spec) {
    chainA = wp.from(L0, [&](int l) {
      const ChainPriv& c = cpriv(l);
      if (c.s + 4 >= (uint32_t)(l * kS + kS)) return c.y;   // [s, E) is the zeroed crc field: y is the prefix
      const uint64_t w = c.wc & c.mlo;
      const uint32_t loc = crc_step8(v.tab, c.cap, (uint32_t)w, (uint32_t)(w >> 32));   // chain-local, at P
      const bool second = c.kb >= (uint32_t)kSplit;
      const uint32_t at_p = second ? (shift_8n(v.tab, c.ya, c.kb + 1 - kSplit) ^ loc) : loc;   // slice-local
      return shift_8n(v.tab, at_p, (uint32_t)(kS / 8 - 1) - c.kb);   // from P to the slice end
    });
  }
  const uint32_t I0 = spec ? 0u : shift_tab(v.tab, kZCOff, st.I);
  wp.each([&](int l) {
    ChainPriv& c = cpriv(l);
    c.O = c.y ^ (l == 0 ? I0 : 0u) ^ (spec && l == L0 ? chainA : 0u);
  });
  lane_scan(wp, v.tab, cpriv, spec ? L0 : 0);
  uint32_t rpre = 0;
  if (spec) rpre = (L0 > 0 ? shift_tab(v.tab, kZCOff, wp.from(L0 - 1, [&](int l) { return cpriv(l).O; })) : 0u) ^ chainA;
  const uint32_t Iin = st.I;
  wp.template shfl_up<1>([&](int l) { return cpriv(l).O; }, [&](int l, uint32_t t, bool valid) {
    ChainPriv& c = cpriv(l);
    if (!c.chk && !c.chkB) return;   // lanes without a check stay off the LDS (fewer bank conflicts)
    const uint32_t g = valid ? t : Iin;   // G at the slice start
    if (c.chkB) c.yB = shift_tab(v.tab, kVSOff, g) ^ crc_step8(v.tab, 0u, (uint32_t)c.wB, (uint32_t)(c.wB >> 32));
    if (!c.chk) return;
    const uint64_t w = c.wc & c.mlo;
    // G at P = slice start + 8 (kb + 1) = shift(G at the chain start, P - chain start) ^ the chain's
    // register at P; the second chain starts at byte 48, where G = shift48(G) ^ (first chain)
    const bool second = c.kb >= (uint32_t)kSplit;
    const uint32_t base = second ? shift_tab(v.tab, kVSOff + 2 * kShW, shift_tab(v.tab, kVSOff + kShW, g)) ^ c.ya : g;
    const uint32_t n = second ? c.kb + 1 - kSplit : c.kb + 1;
    c.y = shift_8n(v.tab, base, n) ^ crc_step8(v.tab, c.cap, (uint32_t)w, (uint32_t)(w >> 32));
  });
  const int bad = wp.first([&](int l) {
    const ChainPriv& c = cpriv(l);
    return (c.chk && c.y != 0u) || (c.chkB && c.yB != 0u);
  });
  if (bad >= 0) {
    restage();   // the buffer may already hold the next region: reload this one (original bytes)
    return LDB_DECLINE(8);
  }
  wp.stamp(14);
  // ---- summary
  const uint32_t nstarts = multi ? wp.sum(cnt_of) : (uint32_t)__builtin_popcountll(starts);
  RegionSum r;
  r.start = v.R0 + sL0;
  if (tpos != kNone32) {   // the chain ends here (status at tpos, as region_process reports it)
    r.status = tstat;
    r.count = nstarts;
    r.exitp = v.R0 + tpos;
    r.soff = 0; r.scrc = 0; r.rout = 0;
    r.rpre = rpre;
    r.sflag = spec ? 0u : kOwnerOk;
    store(r);
    st = nm;
    st.on = 0;
    wp.stamp(15);
    return true;
  }
  r.status = kCont;
  r.count = nstarts;
  r.exitp = v.R0 + wp.from(z, [&](int l) { return cpriv(l).X; });
  r.soff = v.R0 + sz;
  r.scrc = wp.from(z, [&](int l) { return cpriv(l).crc; });
  r.rout = wp.from(kLanes - 1, [&](int l) { return cpriv(l).O; });
  if (tail > 4 && tail < 8) r.rout ^= 0xFFFFFFFFu >> (8 * (tail - 4));
  r.rpre = rpre;
  r.sflag = spec ? kStraddle : (kStraddle | kOwnerOk);
  if (tail <= 4) { r.sflag |= kSkip; r.rout = 0; }
  store(r);
  st = nm;
  st.on = tail > 4 ? 1u : 2u;   // after a kSkip straddler: the entry is known, its CRC state not (k_combine)
  st.x = r.exitp;
  st.I = r.rout;
  st.owner = r.scrc;
  wp.stamp(15);
  return true;
}

// The chain after region_process entered with `enter`: on (1) from a clean straddle-out whose register
// at the region end is known; entry known but CRC state not (2, the next region's straddler is then
// verified by k_combine, as after the run prefix) from any other straddle-out, or through a region the
// open entry covers; off (speculate) after a terminal status. Round 3: rounds 1-2 speculated after
// every kSkip / kNoCrc straddle-out too, and each wrong speculation was a walker's stretch of re-runs.
LDB_HD void chain_after_general(ChainState& st, const RegionSum& o, const View& v, uint32_t enter) {
  if (o.status == kCont && o.start != kNone64 && o.exitp >= v.R0 + (uint64_t)kW) {
    st.on = (o.sflag == kStraddle && v.rlen == (uint32_t)kW) ? 1u : 2u;
    st.x = o.exitp;
    st.I = o.rout;
    st.owner = o.scrc;
  } else if (o.status == kCont && o.start == kNone64 && enter == kForceNone && st.on) {
    st.on = 2;   // still inside the entry that covers the region: x unchanged
  } else {
    st.on = 0;
  }
}

// One region of a wavefront's run: the chained fast path when the chain state allows it,
// otherwise region_process (speculative at the start of a run, entry forced after a fallback).
// buffer_free(): the staging buffer is no longer read (start refilling it); restage(): wait for any
// refill in flight and reload this region's bytes into the buffer. Returns true when the chained
// fast path did the region.
// The fast path stores its summary with store(r); after region_process it is in *out (the caller
// stores it).
template <class WP, class Priv, class CPriv, class Emit, class Free, class Restage, class Store>
LDB_HD bool run_region(WP& wp, const View& v, uint8_t* wbuf, WaveSh& sh, ChainState& st, RegionSum* out, Priv priv,
                       CPriv cpriv, Emit emit, Free buffer_free, Restage restage, Store store) {
  if (region_chained(wp, v, wbuf, sh, st, cpriv, emit, buffer_free, restage, store)) return true;
  uint32_t enter = kForceSpec;
  if (st.on && st.x >= v.R0) enter = st.x - v.R0 < (uint64_t)v.rlen ? (uint32_t)(st.x - v.R0) : kForceNone;
  region_process(wp, v, sh, enter, out, priv, emit, buffer_free);
  chain_after_general(st, *out, v, enter);
  return false;
}

}  // namespace ldb
