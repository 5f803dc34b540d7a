// ldb_sweep.h — the sweep tier of the log scan (round 5): variable-length entries at the HBM roofline.
//
// The replay (index.go:84-95) is a chain: entry i+1 starts where entry i ends, and each entry's
// CRC-32 covers its bytes [off+4, off+size) (logfile/log_entry.go:110-121, log_file.go:141-143). The run
// prefix (k_uniform) verifies runs of equal-sized entries; the region pipeline (k_scan_main ...) walks
// anything. The sweep sits between them for logs of long variable-length entries (BASELINE config 3:
// Zipf values of 16 B - 64 KiB, 5.2 KB per entry on average), where the region pipeline spends its time
// on per-region machinery around one or two entry starts. It splits the work by what it depends on:
//
//   k_sweep      one streaming pass over the image, 16-B rows straight into registers: lane l of a wave
//                holds bytes [64 l, 64 l + 64) of a 4-KiB quarter (four row instructions per quarter, the
//                next quarter in flight while one is processed). Every lane CRC-32s its 64 bytes from
//                register 0 on the lane-private LP2 tables (four 16-B row chains joined by shifts); a
//                2-level DPP tree gives each 256-B window's raw register (RW), and the windows of four
//                quarters at a time go to one row of an accumulator (ds_bpermute) whose 4-level row tree
//                gives each 4-KiB group's register (RG). Every byte position is a header candidate when
//                its Status byte (p + 4) is <= 2 (three VALU per dword; a zero window offers none): the
//                positions go to a per-wave list in LDS, in file order, and are decoded 64 at a time
//                (decode_lean_w, the region pipeline's Go-exact decode of canonical headers, with the
//                IOController bounds) into the wave's slab of index tuples. The lanes of a 256-B window
//                before a candidate's lane keep their 64-B registers (LR, one word per 64 B), so the
//                prefix of an entry start costs k_sweep_fin at most 3 registers and 63 bytes.
//                Each wave owns a contiguous run of the image and then walks its slab: from the run's
//                first candidate (run 0: the chain's entry point x_s), each entry's end must be the
//                next candidate; a speculated start whose chain leaves the run after fewer than
//                kSwTrust entries is weak (a false start inside a binary value can claim a size past
//                the run), and later starts are tried first. The last workgroup checks the links
//                between runs (a run's exit must be the next run's first entry; wave-level scans) and
//                fixes where the tier ends: at the first broken link, declined run (too many
//                candidates, slab full) or chain end.
//   k_sweep_fin  one lane per chain entry: its CRC from the registers (the start's prefix from LR and at
//                most 63 bytes, the partial windows folded by RW, whole groups by RG, the end's prefix
//                likewise, two GF(2) multiplies), the tuple written at its index. The last workgroup
//                writes the result when the tier ends on a terminal (io.EOF, ErrLogEndOfFile, a failed
//                CRC) or hands the rest to the region pipeline: K entries and position x, as the run
//                prefix does (dyn[0], dyn[5]).
//
// Results are the serial scan's for every input: a candidate is decoded exactly as decodeHeader
// would, a chain entry is accepted only when its header, bounds and CRC check, and wherever the tier
// cannot decide (a non-canonical header, a speculated run start that is off the chain) it stops and the
// region pipeline continues from that position. Speculation (a run's first candidate) only changes how
// much of the file the tier takes.
#pragma once

namespace ldb {

constexpr uint32_t kSwW = 256;                 // window: one lane's bytes per batch
constexpr uint64_t kSwBatch = 64ull * kSwW;    // a wave's batch (16 KiB)
constexpr uint32_t kSwG = 16;                  // windows per group register (4 KiB)
constexpr int kSwWaves = 16;                   // waves per k_sweep workgroup (1 per CU: LDS)
constexpr uint32_t kSwList = 512;              // candidate positions awaiting decode, per wave (LDS)
constexpr uint32_t kSwTrust = 4;               // a speculated chain this long is kept when it ends in its run
constexpr uint32_t kSwTagWalk = 14;            // the walk's last start tag (it takes that chain whatever it is)
constexpr uint32_t kSwTagRelink = 15;          // a chain the links re-walked from the true position (sw_link)
constexpr uint32_t kSwMaxRuns = 4096;
constexpr uint64_t kSwMinBatches = 4;          // a run's least length in batches (64 KiB)
constexpr uint32_t kSwDead = 1u, kSwDecl = 2u;
constexpr uint64_t kSwPosMask = (1ull << 60) - 1;   // slab records: index tuple, walk tag in pos bits 60-63
constexpr int kSwFinWaves = 4;

// global tables (ldb_ctx::d_swt): register shift by 64 << i bytes (i = 0..6: 64 ... 4096), the slicing-by-16
// tables (S[k][b]: the raw register after byte b and k zero bytes), then shifts by 16, 32 and 48 bytes (a
// lane's four row registers joined)
constexpr int kSwShTabs = 7;
constexpr uint32_t kSwSl16Off = kSwShTabs * 1024;
constexpr uint32_t kSwRowOff = kSwSl16Off + 16 * 256;
constexpr uint32_t kSwTabWords = kSwRowOff + 3 * 1024;

struct alignas(16) SwRun {
  uint64_t E;       // the run's first chain entry as walked (run 0: x_s), ~0 none
  uint64_t X;       // its exit (first chain position >= hi), or (kSwDead) where the chain ended
  uint64_t n;       // entries on that chain
  uint32_t flags;   // kSwDead | kSwDecl | walk tag << 8
  uint32_t ncand;   // slab records
  uint64_t lo, hi;  // candidate positions [lo, hi)
  uint64_t base;    // index of its first entry among the tier's (link resolution)
  uint64_t pad;
};
static_assert(sizeof(SwRun) == 64, "run records are 64 B");

struct alignas(16) SwCtl {
  uint64_t xs, ks;    // where the tier starts (chain_x0 after the run prefix) and that entry's index
  uint64_t xe, ke;    // where it ends (link resolution)
  uint64_t ncov;      // runs whose chain entries are the tier's
  uint64_t fail;      // smallest tier index of an entry whose CRC failed (k_sweep_fin), ~0
  uint64_t stop;      // set by run 0 when the tier surely ends inside it (declined, or its chain died within
                      // its first decode block): no other run's registers serve an entry, they stop streaming
  uint64_t done0, done1;   // workgroups finished (k_sweep, k_sweep_fin): the last one resolves
  uint64_t state;     // 1 once k_sweep resolved the links; k_sweep_fin's last workgroup clears it
  uint64_t nrun;      // runs of this scan (each run's slab: scratch_bytes / 16 / nrun records)
  uint64_t relinks;   // runs the links set aside or re-walked (sw_link's extra passes)
  uint64_t pad[4];
};
static_assert(sizeof(SwCtl) == 128, "sweep control block");

inline void build_swtab(uint32_t* t) {
  for (int i = 0; i < kSwShTabs; ++i) {
    const uint32_t xn = x8n_modp(64ull << i);
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) t[i * 1024 + q * 256 + b] = multmodp(xn, b << (8 * q));
  }
  uint32_t* s = t + kSwSl16Off;
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t c = b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
    s[b] = c;
  }
  for (int k = 1; k < 16; ++k)
    for (uint32_t b = 0; b < 256; ++b) s[k * 256 + b] = (s[(k - 1) * 256 + b] >> 8) ^ s[s[(k - 1) * 256 + b] & 0xFFu];
  for (int i = 0; i < 3; ++i) {
    const uint32_t xn = x8n_modp(16ull * (i + 1));
    for (int q = 0; q < 4; ++q)
      for (uint32_t b = 0; b < 256; ++b) t[kSwRowOff + i * 1024 + q * 256 + b] = multmodp(xn, b << (8 * q));
  }
}

}  // namespace ldb
