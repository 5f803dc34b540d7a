// ldb_scan.hip — gfx950 kernels + C ABI of the LazyDB log-scan engine (liblazydb_gpu.so).
//
// Pipeline per file (all on one HIP stream, no host round trip):
//   k_uniform    : the run prefix: equal-sized entries verified in parallel (then k_uniform_fill)
//   k_scan_main  : one wavefront per run of 5 KiB regions, LDS-DMA ring staging, the chained lean path
//                  (region_chained, ldb_chain.h) or the general routine inline (region_process, ldb_wave.h)
//   k_link       : verify region-to-region links of the ReadLogEntry chain
//   k_repair     : one wavefront re-walks the true chain from each broken link (rare)
//   k_combine    : CRC-verify entries crossing region boundaries; terminal reduction
//   k_final      : stop position, status and entry count (index.go:84-95 semantics)
//   k_compact    : copy the per-region tuples into the caller's dense array
//   k_serial     : single-lane reference walker (ldb_scan_file_dev_serial, overflow fallback)
// Reference semantics: logfile/log_file.go:116-145, logfile/log_entry.go:48-121, index.go:55-110.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "ldb_pipeline.h"

using namespace ldb;

#define LDB_HIP(x)                                                 \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) return LDB_ERR_HIP;                      \
  } while (0)

namespace {

#ifndef LDB_WPB
// 16 waves per CU fit beside the round-3 table block (62.8 KB); the LP2 block (70 KB, ldb_engine.h)
// leaves room for 14 staging rings of 6.1 KiB
#define LDB_WPB 16
#endif
#ifndef LDB_NB
#define LDB_NB 1
#endif
constexpr int kWPB = LDB_WPB;  // wavefronts per workgroup of k_sweep and k_region (1024 threads)
constexpr int kNB = LDB_NB;    // LDS ring depth per wavefront
#ifndef LDB_BLOCKS_PER_CU
#define LDB_BLOCKS_PER_CU 0   // 0: as many as fit in a CU's 160 KiB of LDS
#endif
constexpr int kG = kW / 1024 + 1;  // LDS-DMA instructions per region (5 x 1 KiB + the halo)

// ---------------------------------------------------------------- wave policy (SIMT)
[[maybe_unused]] constexpr int kStampSlots = 18;   // phase ids of region_process / region_chained / k_scan_main (tools/stamps.py)
struct GpuWave {
  int lane;
#ifdef LDB_STAMPS
  uint64_t t_last = 0;
  uint64_t acc[kStampSlots] = {};
  __device__ void stamp(int id) {
    // s_memtime returns out of order with LDS reads on lgkmcnt: drain it inside the stamp, or the
    // compiler's counted lgkmcnt waits around it stop meaning what they say (MI355X guide)
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    if (t_last) acc[id] += t - t_last;
    t_last = t;
  }
#else
  __device__ void stamp(int) {}
#endif
  __device__ static void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  template <class F> __device__ void each(F f) { f(lane); sync(); }
  template <class P> __device__ uint64_t ballot(P p) { return __ballot(p(lane) ? 1 : 0); }
  template <class P> __device__ int first(P p) {
    const uint64_t b = __ballot(p(lane) ? 1 : 0);
    return b ? __builtin_ctzll(b) : -1;
  }
  template <class P> __device__ int last(P p) {
    const uint64_t b = __ballot(p(lane) ? 1 : 0);
    return b ? 63 - __builtin_clzll(b) : -1;
  }
  // Sums / exclusive prefixes of small per-lane counts (< 128) by bit-planes: one ballot per
  // bit and v_mbcnt for "set bits below me" -- no cross-lane data movement (ds_bpermute).
  template <class V> __device__ uint32_t sum(V v) {
    const uint32_t x = v(lane);
    uint32_t s = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) s += (uint32_t)__builtin_popcountll(__ballot((x >> b) & 1u)) << b;
    return s;
  }
  template <class V, class O> __device__ void excl_prefix(V v, O out) {
    const uint32_t x = v(lane);
    uint32_t s = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
      const uint64_t m = __ballot((x >> b) & 1u);
      s += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << b;
    }
    out(lane, s);
  }
  // f(l) of the wave-uniform lane `src`, broadcast (v_readlane); uniform control flow only
  template <class F> __device__ uint32_t from(int src, F f) {
    return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)f(lane), src);
  }
  template <class F> __device__ uint64_t from64(int src, F f) {
    const uint64_t x = f(lane);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), src);
    return (uint64_t)lo | ((uint64_t)hi << 32);
  }
  template <class F> __device__ void single(F f) {
    if (lane == 0) f();
    sync();
  }
  // Lanes shifted up by 16: permlane16_swap gives rows (R0, R0, R2, R2) and (R1, R1, R3, R3);
  // permlane32_swap of the latter puts R1 into row 2.
  __device__ static uint32_t up16(uint32_t x, int lane) {
    const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);
    return (lane >> 4) == 2 ? b[0] : a[0];
  }
  // put(lane, value of lane - D, lane >= D), all in VALU (DPP / permlane swaps, no LDS):
  // D = 1 wave_shr; D = 32 permlane32_swap; D = 16 up16; D = 2, 4, 8 row_shr inside a row and, for
  // the first D lanes of a row, row_ror moved up one row.
  template <int D, class G, class P> __device__ void shfl_up(G get, P put) {
    const uint32_t x = get(lane);
    uint32_t y;
    if constexpr (D == 1) {
      y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, false);
    } else if constexpr (D == 32) {
      y = __builtin_amdgcn_permlane32_swap(x, x, false, false)[0];
    } else if constexpr (D == 16) {
      y = up16(x, lane);
    } else {
      static_assert(D == 2 || D == 4 || D == 8, "lane shift");
      const uint32_t in_row = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + D, 0xf, 0xf, false);
      const uint32_t wrap = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x120 + D, 0xf, 0xf, false);
      const uint32_t prev_row = up16(wrap, lane);
      y = (lane & 15) >= D ? in_row : prev_row;
    }
    put(lane, y, lane >= D);
  }
};

// LDS image of one wavefront's working state
struct alignas(16) WaveLds {
  WaveSh sh;
  RegionSum rs;
};

#ifndef LDB_DMA_NT
#define LDB_DMA_NT 1   // 1: the staging DMA reads with the non-temporal hint (streamed once, MI355X guide: LDS-DMA fill 6.4 -> 6.5-6.8 TB/s)
#endif
#if LDB_DMA_NT
#define LDB_GLDS_POLICY " nt"
#else
#define LDB_GLDS_POLICY ""
#endif
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" LDB_GLDS_POLICY "\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Stage region r ([R0, R0 + kW + kHalo) clipped to len) into a buffer by LDS-DMA: kG wave instructions.
__device__ __forceinline__ void stage_dma(const uint8_t* img, uint64_t len, uint64_t r, uint32_t buf_lds, int lane) {
  const uint64_t R0 = r * (uint64_t)kW;
#pragma unroll
  for (int k = 0; k < kG - 1; ++k) {
    const uint64_t off = R0 + (uint64_t)k * 1024 + (uint64_t)lane * 16;
    // Keep the instruction count wave-uniform for vmcnt accounting: lanes past the end of the
    // file reload the region's first chunk (harmless bytes that are never used).
    glds16(img + (off < len ? off : R0), buf_lds + kPre + k * 1024);
  }
  // halo: 64 bytes past the region end, lanes 0..3 only (always active -> always issued)
  if (lane < kHalo / 16) {
    const uint64_t off = R0 + (uint64_t)(kG - 1) * 1024 + (uint64_t)lane * 16;
    glds16(img + (off < len ? off : R0), buf_lds + kPre + (kG - 1) * 1024);
  }
}

// Region summary record (48 B) from its LDS copy: lanes 0-11 move one dword each -- one LDS read
// and one coalesced global_store_dword (global, in-order on vmcnt: k_scan_main counts it).
__device__ __forceinline__ void write_region_wave(const Pipe& p, uint64_t r, const RegionSum* lds_rs, int lane) {
  if (lane < 12) {
    const uint32_t x = reinterpret_cast<const uint32_t*>(lds_rs)[lane];
    reinterpret_cast<uint32_t*>(p.rs + r)[lane] = x;
  }
}

#include "ldb_devmem.h"

constexpr int kFillThreads = 1024;   // k_uniform_fill workgroup
// A 48-B region summary from wave-uniform values: lanes 0-2 store 16 B each (one instruction).
// drop: the instruction still issues (k_scan_main's counted vmcnt waits) but writes nothing
__device__ __forceinline__ void store_summary(const Pipe& p, uint64_t r, const RegionSum& s, int lane, bool drop = false) {
  uint32_t w[12];
  __builtin_memcpy(w, &s, sizeof(w));
  uint32_t d[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) d[j] = lane == 0 ? w[j] : (lane == 1 ? w[4 + j] : w[8 + j]);
  store16(rsrc_of(p.rs + r, (uint32_t)sizeof(RegionSum)), lane < 3 && !drop ? (uint32_t)lane * 16u : kDrop, d[0], d[1],
          d[2], d[3]);
}
constexpr int kStoresPerRegion = 1;   // lean path: the summary (tuples are stored before the release)

// Global -> LDS copy of the table block: 16-B loads, kBatch of them in flight per thread before
// the stores (one global round trip per batch, not per word).
static_assert(kTabWords % 4 == 0, "table block is a whole number of 16-B words");
__device__ __forceinline__ void copy_tables(uint32_t* tab, const uint32_t* gtab) {
  constexpr int kQ = kTabWords / 4, kBatch = 8;
  const uint4* __restrict__ g = reinterpret_cast<const uint4*>(gtab);   // no aliasing: all loads before the stores
  uint4* __restrict__ t = reinterpret_cast<uint4*>(tab);
  for (int i0 = 0; i0 < kQ; i0 += kBatch * (int)blockDim.x) {
    uint4 x[kBatch];
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int i = i0 + b * (int)blockDim.x + (int)threadIdx.x;
      x[b] = g[i < kQ ? i : kQ - 1];   // unconditional (clamped): the batch stays in registers
    }
    asm volatile("" ::: "memory");   // keep the whole batch of loads in flight before the stores
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int i = i0 + b * (int)blockDim.x + (int)threadIdx.x;
      if (i < kQ) t[i] = x[b];
    }
  }
}

#ifdef LDB_STAMPS
__device__ uint64_t g_stamps[kStampSlots];
// k_uniform's phases (tools/uni_stamps.py), thread 0 of every workgroup: 0 run 0's window, 1 its decode +
// combine tables + publication, 2 header probes, 3 later runs' windows, 4 their decodes, 5 combine
// rebuilds between runs, 6 the verify loops, 7 the INDEX fill, 8 uni_finish
constexpr int kUniStampSlots = 24;
__device__ uint64_t g_ustamps[kUniStampSlots];
__device__ __forceinline__ uint64_t uni_now() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}
#define UNI_T(v) const uint64_t v = uni_now()
#define UNI_ADD(slot, a, b) \
  do { if (threadIdx.x == 0) atomicAdd((unsigned long long*)&g_ustamps[slot], (unsigned long long)((b) - (a))); } while (0)
#else
#define UNI_T(v)
#define UNI_ADD(slot, a, b)
#endif

// ---------------------------------------------------------------- k_uniform
// The run prefix (ldb_pipeline.h). Entry e of a run of equal-sized entries starts at e * sz; it is a
// run member when its header bytes equal entry 0's (uni_header_ok) and its CRC is right. k_uniform
// verifies all candidates in parallel and K = the first that fails (atomicMin) bounds the prefix; the
// region pipeline replays from K * sz. No region summary, link, scan or owner check is involved.
//
// Entry-aligned slices (uni_geometry): a wave holds E = 64 / G whole entries, G lanes each. Lane j of
// an entry loads its P-byte window [x + 4 - t + j P, + P) as <= kUniRows 16-B rows, all in flight at
// once (a wave's rows cover its E entries' bytes contiguously, so every fetched line is consumed while
// it is in L1), and runs S = P / 8 S-table steps from register 0 (lane 0 masks its first t bytes).
// The group's registers are combined by a tree: at level d, lanes j = 2d - 1 (mod 2d) take the value
// of lane j - d by DPP / permlane and shift it by d P bytes (a 4-lookup byte table built by
// each workgroup, uni_prepare). The group's last lane ends with the raw register of the whole span, checks
// raw ^ KL == ~crc and the header, and writes the tuple at out[e].
//
// Bytes are read with buffer loads from a wave-uniform base 512 B before the wave's first entry (so
// no masked lead reaches below it), ranged to len rounded up to a dword: dwords past the
// image read as zero, and the dword holding the image's last byte is real (the same 16-B granule the
// staging DMA reads, ldb_scan.hip stage_dma). The first waves of the file (base 0) load dword by
// dword, as their lead may start before byte 0 (those dwords read as zero, and are masked anyway).
#ifndef LDB_UNI_WAVES
#define LDB_UNI_WAVES 16
#endif
constexpr int kUniWaves = LDB_UNI_WAVES;
struct UniSetup {
  UniMemo m;
  UniGeo g;
};
// Round 4: a log may be several runs of equal-sized entries one after another (the reference bench's
// log: keys bench_test_key_<i> grow a digit at entries 10, 100, ..., 100000, so its entry size steps up
// five times, bench/db_bench_test.go:17-36; any fixed-schema writer whose key or value width steps).
// uni_prepare finds where each run's headers stop matching its memo and speculates the next run there;
// k_uniform verifies every run's candidates in one launch, and K counts entries along the chain across
// the runs (run r's entry e is chain entry gbase + e). A boundary that is not the chain's (an entry of
// run r failing its CRC before it) only costs the later runs' work: K stops at that first failure.
constexpr int kUniMaxRuns = 8;
struct UniRun {
  UniMemo m;
  UniGeo g;
  uint64_t y;       // image offset of the run's entry 0
  uint64_t gbase;   // its chain index (entries of the earlier runs)
  uint64_t nc;      // candidates: entries e in [0, nc) at y + e sz
};
struct UniRuns {
  UniRun r[kUniMaxRuns];
  int n;
};
// Combine tables in LDS (4 byte-indexed 256-word tables each = 1024 words): G <= kUniDirectG uses the
// direct form, G - 1 tables "shift by d P bytes" (d = 1 .. G - 1); larger G the tree, lg tables
// "shift by 2^i P bytes".
constexpr uint32_t kUniDirectG = 8;
constexpr uint32_t kUniHalfTab = (kUniDirectG - 1 > kUniLevels ? kUniDirectG - 1 : kUniLevels);   // its table index
constexpr uint64_t kUniTabWords = kUniHalfTab * 1024;
LDB_HD uint32_t uni_ntab(const UniGeo& g) { return g.G <= kUniDirectG ? g.G - 1 : g.lg; }

constexpr uint64_t kUniReady = 0x5E7A11ED5E7A11EDull;   // dyn[2]: the setup in p.uni is complete
constexpr uint64_t kUniSetupBytes = 1024;                // UniSetup, then the combine tables
constexpr uint32_t kUniWin = 8192;                       // image bytes uni_prepare stages (entries 0 and 1)
static_assert(kUniMaxSize + 48 + 3 <= kUniWin, "entry 1's header lies in the staged window");
static_assert(sizeof(UniSetup) <= kUniSetupBytes, "run-prefix setup block");
// The first k_uniform launch of a pipeline derives the run's parameters in every workgroup (no
// separate setup launch) and its workgroup 0 publishes them to p.uni, so the later launches of a
// chunked scan (ChunkPlan) only copy them:
// entry 0's memo, the slicing, KL and the combine tables (shift by 2^i P bytes, built straight into
// LDS). Entry 0's and entry 1's header windows are staged into LDS by one coalesced load each (the
// decode is a chain of dependent byte reads; all workgroups read the same L2-resident 128 bytes).
// When entry 1 is not a run member the prefix is skipped outright (K = 0: the region pipeline from
// offset 0 -- the same scan, without a run of one). Shifts come from the x^(8n) table (n <= kW).
// Workgroup 0 publishes K = 0 or the entry size for the pipeline. Returns false when there is no run.
// Every pipeline kernel serves one scan (its Pipe by value, p0) or, with kB, one file of a batched
// scan: grid.y = file. k_sweep and k_region take a batch's pipes by value too (PipeArg: up to kUniBatch
// of them in the kernel arguments), each read through the kernarg segment: pointers loaded from there are
// known to be global, where pointers loaded from a device array of pipes left every access of the batched
// kernels a FLAT one (round 6: k_region<true> 1088 flat instructions, k_sweep<true> 59; its workgroups ran
// ~15 % slower than k_sweep<false>'s, tools/sw_trace.py)
typedef __attribute__((address_space(4))) const Pipe* CPipe;
#define LDB_PIPE_SELECT                                                                              \
  const Pipe& p = *(const Pipe*)((CPipe)__builtin_amdgcn_kernarg_segment_ptr() + (kB ? blockIdx.y : 0u)); \
  (void)a0

// Header probes of a one-run launch (chunked, batched or hashed scans; every workgroup probes, 64 probes
// in round 0: the device path's several runs use uni_search below, one workgroup). The first header
// mismatch of a run past its entry 1: the
// smallest e in (1, nc - 1) whose header bytes or IOController bounds differ from the memo
// (uni_header_ok), where candidate nc - 1 lies past the file's last whole entry and always fails. Rounds
// of one probe per thread: the smallest failing probe bounds it from above, the largest passing probe
// below that from below, so the interval shrinks ~1000-fold per round; the first round probes powers of
// two, then evenly, so a break near the run's start (the reference bench's log: entry 10) or anywhere
// else is bracketed at once. A run is a contiguous block of equal headers, so the search is exact; where
// it is not (a header equal to the memo again after a different one) it returns a later mismatch, which
// costs speed only: the verification's K stops at the first real failure. Returns nc - 1 when no probe of
// the first round fails (the run reaches the end of the file as far as sampled, and no refinement round
// is paid: a file one run covers, configs 2, 4, 5). Probes whose bytes lie at or past probe_hi (a chunked
// scan's bytes still in flight) are not taken. All threads of the workgroup call it.
// One probe: run r's candidate at x matches the memo (uni_header_ok) -- the header words by aligned
// dword loads (<= 12 of them, one round trip) instead of byte loads.
__device__ __forceinline__ bool uni_probe_ok(const Pipe& p, const UniMemo& m, uint64_t x) {
  const uint64_t xa = x & ~3ull;
  const uint32_t sh = (uint32_t)(x & 3u);
  uint32_t d[11];
#pragma unroll
  for (int i = 0; i < 11; ++i) {
    const uint64_t a = xa + 4ull * i;
    uint32_t v = 0;
    if (i <= (int)m.nw + 1) {
      if (a + 4 <= p.len) {
        v = *reinterpret_cast<const uint32_t*>(p.img + a);
      } else {
        for (uint32_t k = 0; k < 4; ++k) v |= (a + k < p.len ? (uint32_t)p.img[a + k] : 0u) << (8 * k);
      }
    }
    d[i] = v;
  }
  auto word = [&](int i) -> uint32_t { return funnel(d[i + 1], d[i], sh); };
  return uni_header_ok(m, word, x, p.len, p.io);
}

__device__ uint64_t uni_boundary(const Pipe& p, const UniMemo& m, uint64_t y, uint64_t nc, uint64_t probe_hi,
                             uint32_t nt0) {
  __shared__ unsigned long long s_fail, s_pass;
  const uint64_t sz = m.sz, need = sz > 48 ? sz : 48;
  uint64_t lo = 1, hi = nc - 1;
  for (int round = 0; hi > lo + 1; ++round) {
    // round 0: threads 0..nt0-1 (entries lo + 2^(t+1) for t < 24, then evenly); later rounds: every
    // thread evenly over (lo, hi), so the interval shrinks ~blockDim-fold per round
    const uint32_t nt = round == 0 ? nt0 : blockDim.x, t = threadIdx.x;
    if (t == 0) {
      s_fail = hi;
      s_pass = lo;
    }
    __syncthreads();
    const uint64_t w = hi - lo - 1;
    uint64_t e = 0;
    if (t < nt) e = round == 0 ? (t < 24 ? lo + (2ull << t) : lo + 1 + (w * (t - 23)) / (nt - 23)) : lo + 1 + (w * t) / nt;
    const uint64_t x = y + e * sz;
    bool pass = false;
    if (t < nt && e > lo && e < hi && x + need <= probe_hi) {
      pass = uni_probe_ok(p, m, x);
      if (!pass) atomicMin(&s_fail, (unsigned long long)e);
    }
    __syncthreads();
    const uint64_t f = s_fail;
    if (round == 0 && f == hi) return hi;
    if (pass && e < f) atomicMax(&s_pass, (unsigned long long)e);
    __syncthreads();
    lo = s_pass;
    hi = f;
    __syncthreads();
  }
  return hi;
}

// The combine tables for geometry g: T[t][q][b] = shift(b << 8q, n_t bytes) are linear in b: 32 basis
// registers per table (one multmodp each, one thread each), then every entry an xor of its bits' basis
// values. (Round 2: one 32-step multmodp per entry, 3 x 1024 of them per workgroup: most of the setup.)
// gT: also written there (workgroup 0's publication), or null. All threads call it.
__device__ __forceinline__ void uni_build_comb(const Pipe& p, const UniGeo& g, uint32_t* T, uint32_t* gT) {
  __shared__ uint32_t basis[kUniTabWords / 1024][32];
  const uint32_t nt = uni_ntab(g);
  const uint32_t t = threadIdx.x >> 5, bit = threadIdx.x & 31u;
  if (t < nt) {
    const uint32_t xt = g.G <= kUniDirectG ? p.xw[(t + 1) * g.P] : p.xw[g.P << t];   // d P <= 7 * 96 < kW
    basis[t][bit] = multmodp(xt, 1u << bit);
  }
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < (uint32_t)kUniTabWords; e += blockDim.x) {
    if (e >= nt * 1024u && e < kUniHalfTab * 1024u) continue;
    const uint32_t tt = e >> 10, q = (e >> 8) & 3u, b = e & 255u;
    uint32_t v = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) v ^= ((b >> i) & 1u) ? basis[tt][8 * q + i] : 0u;
    T[e] = v;
    if (gT) gT[e] = v;
  }
  __syncthreads();
}

// kMulti (the device path's whole-image launch): a log of several runs one after another. Workgroup 0
// finds them (uni_discover) while the others stage their tables; the list is published once complete
// (dyn[6] = the number of runs | kUniFinal, UniRun records at p.uni + kUniRunsOff), and every workgroup
// then verifies the runs in order. Each run r has its own first-failure word F_r (run 0: dyn[0], then
// p.uni + kUniFOff), the smallest candidate index within the run known to fail: workgroup 0 starts it
// at the run's end M_r (its header boundary; the next run's entry 0 lies there), and the verification
// lowers it at a failing entry. K is then the first run's gbase + F_r with F_r < M_r (a failure inside
// the run), or the last run's gbase + F_r (uni_finish).
// Otherwise (a chunked, batched or hashed scan) there is one run, and a boundary inside it is a failure:
// *bound = its chain index, and workgroup 0 lowers K (dyn[0]) to it.
// Round 4 history (config 1, the reference bench's log of six runs, k_uniform): every workgroup finding
// the runs itself, 0.287 ms (256 workgroups probing the same lines: ~5 us a probe round); workgroup 0
// publishing each run as soon as a probe round bracketed it, so the others verified while it searched,
// 0.196 ms; the list published once complete, 0.184 ms -- the search is a chain of dependent loads,
// and the verification's traffic only lengthens it. The chain: per run 1-3 probe rounds (a load round
// trip, ~1 us, plus three barriers), the next run's header from a probe's own loads (no extra load),
// decoded through readlane by one wave; the slicing (uni_geometry: a table load and two multmodp) is
// left to the verifying workgroups, one wave per run.
#ifndef LDB_FOLD_INIT
#define LDB_FOLD_INIT 1   // k_uniform<false, false> sets the control words itself (no k_init launch): config 1
                          // pipeline 0.150 -> 0.145 ms, config 4 neutral (profiles/r04_fold_init_ab.txt); 0 restores k_init
#endif
#ifndef LDB_UNI_SPIN
#define LDB_UNI_SPIN 4   // s_sleep between polls of dyn[6] (x 64 cycles)
#endif
constexpr uint64_t kUniRunsOff = kUniSetupBytes + 4 * kUniTabWords;
constexpr uint64_t kUniFOff = kUniRunsOff + 256 * kUniMaxRuns;
constexpr uint64_t kUniFinal = 1ull << 32;
constexpr int kUniEpochShift = 33;   // dyn[6] = epoch << 33 | kUniFinal | count: a word left by an earlier
                                     // scan on the workspace never reads as this scan's
__device__ __forceinline__ uint64_t uni_word(const Pipe& p, uint64_t v) {
  return ((uint64_t)(p.epoch & 0x7FFFFFFFu) << kUniEpochShift) | v;
}
constexpr uint64_t kUniBlockBytes = kUniFOff + 8 * kUniMaxRuns;   // the workspace's p.uni block
static_assert(sizeof(UniRun) <= 256, "run records are 256 B apart");
__device__ __forceinline__ UniRun* uni_recs(const Pipe& p) { return reinterpret_cast<UniRun*>(p.uni + kUniRunsOff); }
__device__ __forceinline__ uint64_t* uni_fword(const Pipe& p, int r) {
  return r == 0 ? p.dyn : reinterpret_cast<uint64_t*>(p.uni + kUniFOff) + r;
}
__device__ __forceinline__ uint64_t uni_fload(const uint64_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bytes [a, a + kUniWin) of the image into win (zero past len), one coalesced load per thread and dword
__device__ __forceinline__ void uni_stage_win(const Pipe& p, uint32_t* win, uint64_t a) {
  for (uint32_t i = threadIdx.x; i < kUniWin / 4; i += blockDim.x) {
    const uint64_t a0 = a + 4ull * i;
    uint32_t w = 0;
    if (a0 + 4 <= p.len) {
      w = *reinterpret_cast<const uint32_t*>(p.img + a0);
    } else {
      for (uint32_t k = 0; k < 4; ++k) w |= (a0 + k < p.len ? (uint32_t)p.img[a0 + k] : 0u) << (8 * k);
    }
    win[i] = w;
  }
}

// the slicing exists for entries of L = sz - 4 CRC'd bytes (uni_geometry's shapes, without its KL)
__device__ __forceinline__ bool uni_sliceable(uint32_t L) {
  for (uint32_t lg = 0; lg < kUniLevels + 1; ++lg) {
    const uint32_t G = 1u << lg;
    if ((((L + G - 1) / G + 7) & ~7u) <= 8 * kUniSteps) return true;
  }
  return false;
}

// uni_memo of the entry at image offset y, computed across the wave: lane i holds byte y + i (zero past
// len). The five header varints (log_entry.go:86-106, Go's binary.Uvarint) end at the first five bytes
// below 0x80 from byte 5 on (one ballot); each is read by one lane from its bytes (shuffles), and a memo
// exists only when all five are canonical, at most 10 bytes (no overflow) and inside the 38-byte window
// -- exactly the headers uni_memo accepts (it needs `canonical`), with the same fields. The generic
// decode run by one lane through readlane is ~2,000 scalar instructions (4.5 K cycles a run at config
// 1, on the run search's chain); this is a few hundred.
__device__ __forceinline__ UniMemo uni_memo_wave(const Pipe& p, uint64_t y, uint32_t b) {
  UniMemo m;
  m.ok = 0;
  const int lane = (int)(threadIdx.x & 63u);
  // the five varints' last bytes: the first five set bits of T (bytes 5 .. 37 of the window)
  const uint64_t T = __ballot(lane >= 5 && lane < kMaxHeader && b < 0x80u);
  // lane j < 5: varint j's first byte s and last byte e; every lane gathers the 10 bytes from its s
  uint64_t t = T;
  int e = -1, s0 = 5;
  for (int j = 0; j < 5; ++j) {
    const int ej = t ? __builtin_ctzll(t) : 64;
    if (j == lane) { e = ej; }
    if (j < lane) s0 = ej + 1;
    t &= t - 1;
  }
  const int sj = lane < 5 ? s0 : 0;
  uint64_t u = 0;
  uint32_t last = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const uint32_t bk = (uint32_t)__shfl((int)b, (sj + k) & 63);
    if (lane < 5 && sj + k <= e) {
      u |= (uint64_t)(bk & 0x7Fu) << (7 * k);
      last = bk;
    }
  }
  const int n = e - sj + 1;   // the varint's length (lane < 5)
  // per varint: terminated inside the window, <= 10 bytes, no overflow in byte 10, canonical
  const bool vok = lane >= 5 || (e < kMaxHeader && n <= 10 && !(n == 10 && last > 1u) && (n == 1 || last != 0u));
  if (__ballot(!vok)) return m;
  const int64_t zz = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);   // binary.Varint's zig-zag
  auto field = [&](int j) -> int64_t {
    const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)zz >> 32), j) << 32) |
                       (uint32_t)__shfl((int)(uint32_t)(uint64_t)zz, j);
    return (int64_t)v;
  };
  const int64_t ea = field(0), tx = field(1), ts = field(2), ks = field(3), vs = field(4);
  const int hs = __shfl(e, 4) + 1;   // decodeHeader's offset after the five varints
  if (ks < 0 || vs < 0 || ks > 0xFFFFFFFFll || vs > 0xFFFFFFFFll) return m;   // (canonical)
  const uint32_t crc = (uint32_t)__shfl((int)b, 0) | ((uint32_t)__shfl((int)b, 1) << 8) |
                       ((uint32_t)__shfl((int)b, 2) << 16) | ((uint32_t)__shfl((int)b, 3) << 24);
  // classify_entry: the header window readable, not the zero sentinel, key/value readable
  if (read_eof(p.len, p.io, (int64_t)y, kMaxHeader)) return m;
  const uint32_t k = (uint32_t)ks, v = (uint32_t)vs;
  if (crc == 0u && k == 0u && v == 0u) return m;
  const uint64_t kv = (uint64_t)k + v;
  if (kv && read_eof(p.len, p.io, (int64_t)(y + (uint64_t)hs), kv)) return m;
  const uint64_t size = (uint64_t)hs + kv;
  if (hs < 10 || hs > kMaxHeader || size > kUniMaxSize || size < kUniMinSize) return m;
  m.hs = (uint32_t)hs;
  m.enc = (uint32_t)(5 + varint_len(ea) + varint_len(tx) + varint_len((int64_t)(uint16_t)ts) + varint_len((int64_t)k) +
                     varint_len((int64_t)v));
  m.stat = (uint32_t)__shfl((int)b, 4);
  m.tx_stat = (uint32_t)(uint16_t)ts;
  m.k = k;
  m.v = v;
  m.expired_at = ea;
  m.tx_id = (uint64_t)tx;
  m.sz = size;
  m.nw = (m.hs - 4 + 3) / 4;
  // header dwords [4 + 4 i, + 4) (bytes past the 38-byte window read as 0, as uni_memo's fetch)
  const int lb = 4 + 4 * (lane < 9 ? lane : 0);
  uint32_t dw = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t bq = (uint32_t)__shfl((int)b, lb + q);
    dw |= (lb + q < kMaxHeader ? bq : 0u) << (8 * q);
  }
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int nb = (int)m.hs - 4 - 4 * i;
    m.msk[i] = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * nb)));
    m.w[i] = (uint32_t)__shfl((int)dw, i) & m.msk[i];
  }
  m.ok = 1;
  return m;
}

// Wave 0 of the workgroup, all 64 lanes (wave-uniform control): run q's memo from the entry at image
// offset y, lane i holding byte y + i (zero past len), decoded through readlane, not by one lane's
// dependent byte reads (each an LDS or memory round trip: ~5 us per run). kGeo: its slicing too (a
// table load and two multmodp); otherwise only whether it has one. Lane 0 writes q.m (q.g), q.y.
template <bool kGeo>
__device__ __forceinline__ bool uni_decode_wave(const Pipe& p, uint64_t y, uint32_t b, UniRun& q) {
  UNI_T(d0);
  const UniMemo m = uni_memo_wave(p, y, b);
  UNI_T(d1);
  if (blockIdx.x == 0) UNI_ADD(4, d0, d1);
  UniGeo g{};
  bool ok = m.ok;
  if (kGeo) {
    if (ok) g = uni_geometry(p.xw, (uint32_t)(m.sz - 4));
    ok = g.ok;
  } else {
    ok = ok && uni_sliceable((uint32_t)(m.sz - 4));
  }
  if ((threadIdx.x & 63u) == 0) {
    q.m = m;
    if (kGeo) q.g = g;
    q.y = y;
  }
  return ok;
}

// One discovery probe: candidate x of a run matches its memo (uni_header_ok). The header's dwords from
// x rounded down, as three 16-B loads (x + 48 <= len, so they stay inside the image); kept in d for the
// stash (uni_search).
__device__ __forceinline__ bool uni_probe16(const Pipe& p, const UniMemo& m, uint64_t x, uint32_t* d) {
  const uint64_t xa = x & ~3ull;
  const uint32_t sh = (uint32_t)(x & 3u);
  const uint4* q = reinterpret_cast<const uint4*>(p.img + xa);
  const uint4 r0 = q[0], r1 = q[1], r2 = q[2];
  d[0] = r0.x; d[1] = r0.y; d[2] = r0.z; d[3] = r0.w;
  d[4] = r1.x; d[5] = r1.y; d[6] = r1.z; d[7] = r1.w;
  d[8] = r2.x; d[9] = r2.y; d[10] = r2.z; d[11] = r2.w;
  auto word = [&](int i) -> uint32_t { return funnel(d[i + 1], d[i], sh); };
  return uni_header_ok(m, word, x, p.len, p.io);
}

// Run q's end M: the smallest candidate in (lo, nc - 1) whose header mismatches (as uni_boundary), by
// rounds of probes over the whole workgroup. Round 0: 128 probes at lo + 1 .. lo + 128, then kUniR0 - 128
// spaced geometrically to nc - 1, so a short run ends exactly in one round and a long one is bracketed to
// ~7 % (128 of them) or ~1 % (896); later rounds probe every candidate of the bracket (<= blockDim of them) or spread evenly over it. The
// probes of a wave are in increasing order, so its smallest failing and largest passing probe are one
// ballot each (one LDS atomic per wave, not per lane). The probe that sets the final M leaves its 48
// header bytes in stash[0..12) (stash[12] = x & 3): the next run's entry 0 without another load.
// (Measured and rejected: one barrier a round, every thread reducing the waves' pairs from LDS -- config
// 1 k_uniform 0.142 -> 0.158 ms.)
// Runs the search from bracket (lo, hi) (lo: a passing candidate or the start, hi: a failing one or nc - 1)
// and returns true with hi = M, or, when `stop_wide` and round 0 left a bracket of more than blockDim
// candidates (two rounds more), false after round 0 with the bracket in (lo, hi). `first`: round 0 is the
// dense + geometric one (a continuation probes the bracket only).
#ifndef LDB_UNI_R0
#define LDB_UNI_R0 256   // threads probing in round 0: 128 dense, the rest geometric. Measured (config 1
                         // k_uniform, 3 alternating reps, profiles/r04_uni_r0_ab.txt): 256 0.119 ms, 512
                         // 0.122, 1024 0.139 -- fewer rounds, but each round waits on more scattered loads
#endif
constexpr uint32_t kUniR0 = LDB_UNI_R0;
__device__ bool uni_search(const Pipe& p, const UniRun& q, uint64_t& lo, uint64_t& hi, uint32_t* stash, bool first,
                           bool stop_wide) {
  // a round's smallest failing and largest passing probe: two slots, alternating by round, so the next
  // round's pair is set up before this round's last barrier (two barriers a round)
  __shared__ unsigned long long s_fail[2], s_pass[2];
  const UniMemo& m = q.m;
  const uint64_t sz = m.sz, need = sz > 48 ? sz : 48;
  const uint32_t t = threadIdx.x, nt = blockDim.x, lane = t & 63u;
  if (t == 0) {
    s_fail[0] = hi;
    s_pass[0] = 0;
  }
  __syncthreads();
  for (int round = 0; hi > lo + 1; ++round) {
    UNI_T(r0);
    const int cur = round & 1;
    const bool rz = first && round == 0;
    const uint64_t w = hi - lo - 1;   // candidates strictly between
    uint64_t e = 0;
    if (rz) {
      const uint32_t ng = (kUniR0 < nt ? kUniR0 : nt) - 128;   // geometric probes
      if (t < 128) {
        e = lo + 1 + t;
      } else if (t < 128 + ng) {
        const float a = fmaxf(0.0f, __logf((float)w / 128.0f) / (float)ng);
        e = lo + (uint64_t)(128.0f * __expf(a * (float)(t - 127)));
      }
    } else {
      e = w <= nt ? lo + 1 + t : lo + 1 + (w * t) / nt;
    }
    const uint64_t x = q.y + e * sz;
    const bool act = e > lo && e < hi && x + need <= p.len;
    bool pass = false;
    uint32_t d[12];
    UNI_T(ra);
    if (act) pass = uni_probe16(p, m, x, d);
    const uint64_t fm = __ballot(act && !pass);
    if (fm && lane == (uint32_t)__builtin_ctzll(fm)) atomicMin(&s_fail[cur], (unsigned long long)e);
    UNI_T(rb);
    UNI_ADD(14, ra, rb);
    __syncthreads();
    UNI_T(rc);
    UNI_ADD(15, rb, rc);
    const uint64_t f = s_fail[cur];
    if (act && !pass && e == f) {   // the header at the (so far) end: the next run's entry 0
#pragma unroll
      for (int i = 0; i < 12; ++i) stash[i] = d[i];
      stash[12] = (uint32_t)(x & 3u);
    }
    if (rz && f == hi) return true;   // no mismatch: the run reaches the file's end
    const uint64_t pm = __ballot(act && pass && e < f);
    if (pm && lane == 63u - (uint32_t)__builtin_clzll(pm)) atomicMax(&s_pass[cur], (unsigned long long)e);
    if (t == 0) {   // the next round's pair (last read before this round's first barrier)
      s_fail[cur ^ 1] = f;
      s_pass[cur ^ 1] = 0;
    }
    __syncthreads();
    const uint64_t sp = s_pass[cur];   // 0, or a passing probe > lo
    lo = sp > lo ? sp : lo;
    hi = f;
    UNI_T(r1);
    UNI_ADD(10, 0, 1);
    UNI_ADD(11, r0, r1);
    if (rz && stop_wide && hi - lo - 1 > nt) return false;
  }
  return true;
}

// Publishes runs [from, to) of ru (records, F words: a run's M, or its probe bound hi for the run still
// being searched, or "none"), then dyn[6] = to (| kUniFinal). Every thread of workgroup 0.
__device__ void uni_publish_runs(const Pipe& p, const UniRuns& ru, int from, int to, const unsigned long long* s_f,
                                 bool fin) {
  UNI_T(p0);
  for (int r = from; r < to; ++r) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&ru.r[r]);
    uint32_t* dst = reinterpret_cast<uint32_t*>(uni_recs(p) + r);
    for (uint32_t i = threadIdx.x; i < sizeof(UniRun) / 4; i += blockDim.x) dst[i] = src[i];
  }
  if ((int)threadIdx.x >= from && (int)threadIdx.x < to) *uni_fword(p, threadIdx.x) = s_f[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(&p.dyn[6], uni_word(p, (uint64_t)to | (fin ? kUniFinal : 0ull)), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
  UNI_T(p1);
  UNI_ADD(12, p0, p1);
}

// Workgroup 0 of a kMulti launch, run 0's memo in ru: for each run, its end M (uni_search), then the
// entry at M as the next run's entry 0 when it decodes as a run start (a memo and a slicing; its entry 1
// is the next search's first probe), up to kUniMaxRuns runs. A run whose first probe round leaves a wide
// bracket (a long run: two rounds more) is published right then, with the runs before it, its F = the
// bracket's failing end (INDEX-kind scans: no candidate's verification stores anything); the others
// verify them while this workgroup narrows the bracket, and its M then lowers F. The rest of the list
// is published at the end, with kUniFinal.
__device__ void uni_discover(const Pipe& p, UniRuns& ru) {
  __shared__ int s_next;
  __shared__ uint32_t stash[13];
  __shared__ unsigned long long s_f[kUniMaxRuns];
  const bool early = p.kind == LDB_TUPLE_INDEX;
  int published = 0;
  for (;;) {
    const int r = ru.n - 1;
    UniRun& q = ru.r[r];
    UNI_T(b0);
    uint64_t lo = r == 0 ? 1 : 0, hi = q.nc - 1;
    bool wide = false;
    if (!uni_search(p, q, lo, hi, stash, true, early)) {   // published now, narrowed below
      wide = true;
      if (threadIdx.x == 0) {
        s_f[r] = hi;
        ru.r[r].nc = hi + 1;
      }
      __syncthreads();
      uni_publish_runs(p, ru, published, r + 1, s_f, false);
      published = r + 1;
      uni_search(p, q, lo, hi, stash, false, false);
    }
    const uint64_t M = hi;
    UNI_T(b1);
    UNI_ADD(2, b0, b1);
    const bool brk = M < (p.len - q.y) / q.m.sz;   // (uniform) M below the first candidate past the file
    if (r > 0 && M < 2) {   // a later "run" of one entry (entry 1 differs): no run; the chain goes on from
      if (threadIdx.x == 0) ru.n = r;   // its entry 0 in the region pipeline (K = its gbase)
      __syncthreads();
      break;
    }
    if (threadIdx.x == 0) {
      s_f[r] = brk ? M : ~0ull;
      if (brk) q.nc = M;
      // (Measured and rejected: these two stores deferred to the final publication, sparing the next
      // barrier their drain -- config 1 k_uniform 0.119 -> 0.124 ms, profiles/r04_defer_f_ab.txt: M must
      // reach the verifiers at once, or they verify past it.)
      if (wide) {   // already published: its F may be lower by now (a verified failure)
        atomicMin((unsigned long long*)uni_fword(p, r), (unsigned long long)M);
        uni_recs(p)[r].nc = q.nc;
      }
      s_next = brk && r + 1 < kUniMaxRuns;
    }
    __syncthreads();
    if (s_next && threadIdx.x < 64) {   // the entry at M from the stash, one byte per lane of wave 0
      const uint32_t lane = threadIdx.x, i = lane + stash[12];
      const uint32_t b = i < 48 ? (stash[i >> 2] >> (8 * (i & 3u))) & 0xFFu : 0u;
      const uint64_t yn = q.y + M * q.m.sz;
      UniRun& n = ru.r[r + 1];
      const bool ok = uni_decode_wave<false>(p, yn, b, n);
      if (lane == 0) {
        s_next = ok;
        if (ok) {
          n.gbase = q.gbase + M;
          n.nc = (p.len - yn) / n.m.sz + 1;
          ru.n = r + 2;
        }
      }
    }
    __syncthreads();
    UNI_T(b2);
    UNI_ADD(3, b1, b2);
    if (!s_next) break;
  }
  uni_publish_runs(p, ru, published, ru.n, s_f, true);
}

// Every workgroup of a kMulti launch: the runs published beyond the first `have` (spinning on dyn[6];
// workgroup 0 is dispatched first), copied in, each new run's slicing computed (uni_geometry, one wave
// per run; run 0's only unless `have0`). Returns the published word (count | kUniFinal).
__device__ __forceinline__ uint64_t uni_take_runs(const Pipe& p, UniRuns& ru, int have, bool have0) {
  __shared__ unsigned long long s_w;
  UNI_T(w0);
  if (threadIdx.x == 0) {
    uint64_t w;
    for (;;) {
      w = __hip_atomic_load(&p.dyn[6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((w >> kUniEpochShift) == (p.epoch & 0x7FFFFFFFu) && ((int)(uint32_t)w > have || (w & kUniFinal))) break;
      __builtin_amdgcn_s_sleep(LDB_UNI_SPIN);   // (every workgroup's thread 0 polls one word)
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_w = w;
  }
  __syncthreads();
  const uint64_t w = s_w;
  const int n = (int)(uint32_t)w;
  if (blockIdx.x != 0) {   // (workgroup 0: its own list; the others have run 0 but for its nc)
    for (int r = have > 1 ? have : 1; r < n; ++r) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(uni_recs(p) + r);
      uint32_t* dst = reinterpret_cast<uint32_t*>(&ru.r[r]);
      for (uint32_t i = threadIdx.x; i < sizeof(UniRun) / 4; i += blockDim.x) dst[i] = src[i];
    }
    if (threadIdx.x == 0 && have == 0 && n > 0) ru.r[0].nc = uni_recs(p)[0].nc;
  }
  __syncthreads();
  const int wv = have + (int)(threadIdx.x >> 6);
  if (wv < n && (wv > 0 || !have0)) {
    UniRun& q = ru.r[wv];
    const UniGeo g = uni_geometry(p.xw, (uint32_t)(q.m.sz - 4));
    if ((threadIdx.x & 63u) == 0) q.g = g;
  }
  if (threadIdx.x == 0) ru.n = n;
  __syncthreads();
  UNI_T(w1);
  UNI_ADD(9, w0, w1);
  return w;
}

// Once the list is final: every run's nc as last published (a long run published early got its M
// after), for the INDEX sweep's slices -- the same in every workgroup
__device__ __forceinline__ void uni_refresh_nc(const Pipe& p, UniRuns& ru) {
  if (blockIdx.x != 0 && (int)threadIdx.x < ru.n) ru.r[threadIdx.x].nc = uni_recs(p)[threadIdx.x].nc;
  __syncthreads();
}

template <bool kMulti>
__device__ __forceinline__ bool uni_prepare(const Pipe& p, UniSetup& su, UniRuns& ru, uint32_t* T,
                                            uint64_t probe_hi, uint64_t& bound) {
  bound = ~0ull;
  __shared__ int published;
  UniSetup* gsu = reinterpret_cast<UniSetup*>(p.uni);
  uint32_t* gT = reinterpret_cast<uint32_t*>(p.uni + kUniSetupBytes);
  if (threadIdx.x == 0) {   // (kMulti: one launch, nothing published before it)
    published = !kMulti && __hip_atomic_load(&p.dyn[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == kUniReady;
    if (published) su = *gsu;
  }
  __syncthreads();
  auto run0 = [&] {   // thread 0
    ru.r[0].m = su.m;
    ru.r[0].g = su.g;
    ru.r[0].y = 0;
    ru.r[0].gbase = 0;
    ru.r[0].nc = p.len / su.m.sz + 1;
    ru.n = 1;
  };
  if (published) {
    if (!su.g.ok) return false;
    if (threadIdx.x == 0) run0();
    for (uint32_t e = threadIdx.x; e < (uint32_t)kUniTabWords; e += blockDim.x) T[e] = gT[e];
    __syncthreads();
    return true;
  }
  // bytes [0, kUniWin) of the image, zero past len, staged once: entry 0's header and entry 1's (sz <=
  // kUniMaxSize) come from the same round trip (round 2 staged them in two dependent rounds)
  __shared__ uint32_t win[kUniWin / 4];
  UNI_T(s0);
  uni_stage_win(p, win, 0);
  __syncthreads();
  UNI_T(s1);
  UNI_ADD(0, s0, s1);
  const uint8_t* wb = reinterpret_cast<const uint8_t*>(win);
  if (threadIdx.x < 64) {   // entry 0 decoded by wave 0 (readlane), entry 1's header from the window
    UniRun& q = ru.r[0];
    // (workgroup 0 of a kMulti launch leaves the slicing for later: it finds the runs first)
    UNI_T(q0);
    bool ok = kMulti && blockIdx.x == 0 ? uni_decode_wave<false>(p, 0, wb[threadIdx.x], q)
                                        : uni_decode_wave<true>(p, 0, wb[threadIdx.x], q);
    UNI_T(q1);
    if (blockIdx.x != 0) UNI_ADD(16, q0, q1);
    if (threadIdx.x == 0) {
      if (ok) {
        const uint8_t* h = wb + q.m.sz;   // sz + 40 < kUniWin
        auto word = [&](int i) -> uint32_t {
          return (uint32_t)h[4 * i] | ((uint32_t)h[4 * i + 1] << 8) | ((uint32_t)h[4 * i + 2] << 16) |
                 ((uint32_t)h[4 * i + 3] << 24);
        };
        ok = uni_header_ok(q.m, word, q.m.sz, p.len, p.io);
      }
      su.m = q.m;
      su.g = q.g;
      su.g.ok = ok;
      if (ok) {
        if (blockIdx.x == 0) p.dyn[1] = su.m.sz;
        run0();
      } else if (blockIdx.x == 0) {
        p.dyn[0] = 0;   // no run: the pipeline starts at offset 0
      }
    }
  }
  __syncthreads();
  UNI_T(q2);
  if (blockIdx.x != 0) UNI_ADD(17, s1, q2);
  if (kMulti) {
    if (!su.g.ok) return false;
    if (blockIdx.x != 0) {
      uni_build_comb(p, su.g, T, nullptr);   // while workgroup 0 finds the runs
      UNI_T(q3);
      UNI_ADD(18, q2, q3);
    } else {
      uni_discover(p, ru);
    }
    UNI_T(s2);
    UNI_ADD(1, s1, s2);
    return true;
  }
  if (su.g.ok) uni_build_comb(p, su.g, T, blockIdx.x == 0 ? gT : nullptr);
  if (blockIdx.x == 0) {   // publish run 0 (a chunked scan's later launches): the tables, the setup, the flag
    if (threadIdx.x == 0) *gsu = su;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&p.dyn[2], kUniReady, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  UNI_T(s2);
  UNI_ADD(1, s1, s2);
  if (!su.g.ok) return false;
  const UniRun& r = ru.r[0];
  const uint64_t M = uni_boundary(p, r.m, r.y, r.nc, probe_hi, 64u);   // every workgroup probes: few probes
  if (M < r.nc - 1) {   // a failure of the run: K <= bound
    bound = M;
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicMin((unsigned long long*)&p.dyn[0], (unsigned long long)M);
  }
  __syncthreads();
  return true;
}

// Combine level D of the group's tree: lanes j = 2D - 1 (mod 2D) take lane j - D's register shifted
// by D P bytes. c = ~j & (j + 1) is 2^(trailing ones of j): lane j combines at level D iff c > D.
// Branch-free per lane (the shifted value is masked in).
template <int D>
__device__ __forceinline__ void uni_level(GpuWave& wp, const uint32_t* T, uint32_t G, uint32_t c, uint32_t& reg) {
  if ((uint32_t)D >= G) return;   // wave-uniform
  wp.shfl_up<D>([&](int) { return reg; }, [&](int, uint32_t y, bool) {
    const int32_t q = (int32_t)(c / (2 * D));   // > 0 iff c > D (c is a power of 2)
    const uint32_t z = T[y & 0xFFu] ^ T[256 + ((y >> 8) & 0xFFu)] ^ T[512 + ((y >> 16) & 0xFFu)] ^ T[768 + (y >> 24)];
    reg ^= z & (uint32_t)((q | -q) >> 31);
  });
}

// One wave's share of the run prefix, S steps per lane (a compile-time count: the rows stay in
// registers with static indices and the step loop has no per-step branch).
// kFill: the tuples of INDEX-kind scans are written afterwards by k_uniform_fill as one dense sweep, so
// the verify loop carries no store at all (a per-batch tuple store in the loop cost 0.10-0.21 ms per
// 4 GiB even into an L2-resident ring: the wave's next row loads then wait on the store's completion;
// tools/microbench/mb_uni.hip wr_W1, st_S1..S6). ENTRY-kind tuples (per-entry crc) and the merge's key
// hashes are still stored in the loop.
// kAl: every window and header starts on a dword (sz and t multiples of 4, as for LazyDB's 332-B
// config 2/4/5 entries): no funnel shifts (22 v_alignbyte per batch at S = 11).
// One run (ru): its entry e at ru.y + e sz is chain entry ru.gbase + e; candidates e < ru.nc.
// NW: the workgroup's verifying waves (waves 0 .. NW-1; kUniWaves, or one fewer beside a fill wave).
template <int S, bool kChunk, bool kHash, bool kFill, bool kAl, int NW>
__device__ __forceinline__ void uni_waves(const Pipe& p, const UniRun& su, uint64_t* F, const uint8_t* lp2,
                                          const uint32_t* T, int lane, int wave, uint32_t wg, uint32_t nwg,
                                          uint64_t a_lo, uint64_t a_hi, uint64_t bound) {
  if (!kChunk) {   // the whole image in one launch (the device-resident API): no range arithmetic
    a_lo = 0;
    a_hi = p.len;
  }
  constexpr int R = (2 * S + 1 + 3) / 4;   // 16-B rows per lane
  const uint32_t sz = (uint32_t)su.m.sz, G = su.g.G, lg = su.g.lg, P = su.g.P, t = su.g.t, KL = su.g.KL;
  const uint32_t E = 64u >> lg;
  // This launch's candidates, by bytes rather than entry indices (no 64-bit division): entry e at
  // x = e sz is a candidate when x <= len (the one at len or past it fails, so the run stops there),
  // and, for a launch over an image still being copied in (ChunkPlan), when its bytes and the 48
  // header bytes its last lane loads lie in [0, a_hi) but not in [0, a_lo) (the earlier launch's).
  const uint64_t need = sz > 48 ? sz : 48, Esz = (uint64_t)E * sz;
  const bool all_hi = a_hi >= p.len;
  // first batch: an underestimate (float quotient, minus 2) is harmless, its entries are not ours
  const uint64_t b_first = a_lo > need ? (uint64_t)max(0.0f, (float)(a_lo - need) / (float)Esz - 2.0f) : 0;
  const uint32_t j = (uint32_t)lane & (G - 1);
  const bool last = j == G - 1;
  const uint32_t lead0 = uni_lead(su.g, j);   // bytes lane j masks at its window's start
  const uint32_t lb = ((uint32_t)lane & 31u) * 4u;   // this lane's bank in the LP2 rows
  const uint32_t nw = su.m.nw, hrows = (nw + 2 + 3) / 4;
  const uint32_t dsh = G - 1 - j;   // direct combine: this lane's shift, in windows
  const bool fill = kFill && p.kind == LDB_TUPLE_INDEX;
  // the lead masks of every step, once per lane (loop-invariant, 2 S VGPRs): keep the window's bytes >= lead.
  // Round 2 recomputed them per batch behind a per-step uniform branch and an opaque copy (to stay
  // under 64 VGPRs); with the LP2 block's 4 waves per SIMD the registers are there, and the branchy
  // form cost 0.34 ms of 1.19 at config 4 (tools/sweep_uni.sh, LDB_UNI_NOMASK)
  uint32_t lm0[S], lm1[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const uint32_t n = lead0 > 8u * k ? lead0 - 8u * k : 0u;
    lm0[k] = n >= 4 ? 0u : 0xFFFFFFFFu << (8 * n);
    lm1[k] = n >= 8 ? 0u : (n > 4 ? 0xFFFFFFFFu << (8 * (n - 4)) : 0xFFFFFFFFu);
  }
  GpuWave wp{lane};
  const uint64_t nbatch = kChunk ? ~0ull : (su.nc + E - 1) / E;   // !kChunk: ceil(nc / E)
  const uint64_t y0 = su.y, gb = su.gbase;   // (kChunk: one run, y0 = gb = 0)
  // K as last seen: the load issued in one batch is tested at the top of the next, so its latency hides
  // behind the batch (a batch past K only costs its own time: the run's tuples stop at K anyway)
  // (F: the run's first-failure word, candidate indices within the run; K itself for a one-run scan)
  v2u32 kv = {(uint32_t)bound, (uint32_t)(bound >> 32)};   // F as loaded during the previous batch (vector value:
                                                           // read at the next top); first the probes' bound
  const __amdgpu_buffer_rsrc_t krs = rsrc_of(F, 8);
  // (wg, nwg: this workgroup's place among the verifying ones; a kMulti launch leaves workgroup 0 out)
  for (uint64_t b = b_first + (uint64_t)wg * NW + wave; b < nbatch; b += (uint64_t)nwg * NW) {
    if (kChunk && b * Esz > (all_hi ? p.len : a_hi)) break;   // wave-uniform: no candidate of this launch from here on
    // uniform by construction (one address), but a load's result is divergent to the compiler: the
    // loop exit on it would make b, and every descriptor built from b, divergent (waterfall loops)
    const uint64_t kseen = ((uint64_t)__builtin_amdgcn_readfirstlane(kv[1]) << 32) | __builtin_amdgcn_readfirstlane(kv[0]);
    if (b * E >= kseen) break;

    // Opaque per-batch copies: the uniform step / level conditions and the lane masks derived from
    // them are evaluated inside the batch, not hoisted out of the loop as a bank of held SGPR masks.
    uint32_t GG = __builtin_amdgcn_readfirstlane(G), c = ~j & (j + 1);
    asm volatile("" : "+s"(GG), "+v"(c));
    const uint64_t e = b * E + ((uint32_t)lane >> lg);
    const uint64_t x = y0 + e * sz;
    if (kChunk && (b + 1) * Esz + need <= a_lo) continue;   // wave-uniform: below the launch's range (b_first's slack)
    const uint64_t b0 = y0 + b * E * sz;
    const uint64_t base = b0 >= 512 ? (b0 - 512) & ~15ull : 0;   // wave-uniform; the lead t < 8 G <= 512
    const uint64_t nrec = (p.len - base + 3) & ~3ull;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(p.img + base, (uint32_t)(nrec < 0xFFFFFFFFull ? nrec : 0xFFFFFFFFull));
    // the group's last lane: the header (stored crc and bytes [4, 40)), in flight with the rows
    const uint32_t hx = (uint32_t)(x - base), ha = hx & ~3u, hsh = kAl ? 0u : hx & 3u;
    // the header rows the check reads: dwords [0, nw + 2) from ha (the stored crc, nw template words and
    // the funnel's next dword), so 1 row for LazyDB's 10-13-byte Set headers, 3 at most (wave-uniform)
    uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0, h2 = h0;
    if (last) {
      h0 = ld16(rs, ha);
      if (hrows > 1) h1 = ld16(rs, ha + 16);
      if (hrows > 2) h2 = ld16(rs, ha + 32);
    }
    const int32_t ws = (int32_t)hx + 4 - (int32_t)t + (int32_t)(j * P);   // < 0 only when base = 0
    const uint32_t a = (uint32_t)ws & ~3u, sh = kAl ? 0u : (uint32_t)ws & 3u;
    uint32_t d[4 * R];
    if (base) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint4 q = ld16(rs, a + 16 * r);
        d[4 * r] = q.x; d[4 * r + 1] = q.y; d[4 * r + 2] = q.z; d[4 * r + 3] = q.w;
      }
    } else {   // dwords before byte 0 get an out-of-range offset (no folded immediate can wrap them back)
#pragma unroll
      for (int i = 0; i < 4 * R; ++i) {
        const int32_t o = (int32_t)a + 4 * i;
        d[i] = ld4(rs, o < 0 ? kDrop : (uint32_t)o);
      }
    }
    // K for the next batch's exit test: a buffer load with sc1 (past this CU's L1, so it sees other CUs'
    // atomicMin), vector memory only, consumed at the next batch's top so its latency hides behind this
    // batch. (A relaxed atomic load compiled to a flat load, which also counts on lgkmcnt, and the
    // compiler waited for it before issuing the rows.)
    kv = __builtin_amdgcn_raw_buffer_load_b64(krs, 0, 0, kSc1);
    // every row (and header) load in flight before the first use: left alone, the scheduler trades them
    // for registers and issues them one step ahead of the CRC (3 in flight: 1.26 vs 0.82 ms, mb_uni.hip)
    __builtin_amdgcn_sched_barrier(0);
    // lane j's window: S steps from register 0, lane 0's first t bytes masked
    uint32_t reg = 0;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const uint32_t w0 = funnel(d[2 * k + 1], d[2 * k], sh) & lm0[k], w1 = funnel(d[2 * k + 2], d[2 * k + 1], sh) & lm1[k];
      reg = lp2_step4(lp2, lb, lp2_step4(lp2, lb, reg, w0), w1);
    }
    if (GG <= kUniDirectG) {
      // direct: lane j shifts its register by (G - 1 - j) P bytes (4 lookups in its own table), then the
      // group's registers are xor-reduced by DPP (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror), so
      // every lane of the group ends with the span's register: 4 lookups per lane against the tree's 8
      const uint32_t* Td = T + (dsh ? dsh - 1 : 0) * 1024u;
      const uint32_t sv = Td[reg & 0xFFu] ^ Td[256 + ((reg >> 8) & 0xFFu)] ^ Td[512 + ((reg >> 16) & 0xFFu)] ^
                          Td[768 + (reg >> 24)];
      reg = dsh ? sv : reg;
      if (GG >= 2) reg ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)reg, 0xB1, 0xF, 0xF, false);
      if (GG >= 4) reg ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)reg, 0x4E, 0xF, 0xF, false);
      if (GG >= 8) reg ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)reg, 0x141, 0xF, 0xF, false);
    } else {
    uni_level<1>(wp, T, GG, c, reg);
    uni_level<2>(wp, T + 1024, GG, c, reg);
    uni_level<4>(wp, T + 2048, GG, c, reg);
    uni_level<8>(wp, T + 3072, GG, c, reg);
    uni_level<16>(wp, T + 4096, GG, c, reg);
    uni_level<32>(wp, T + 5120, GG, c, reg);
    }
    // the header: bytes [4, hs) against the memo's (uni_header_ok). The memo is read from LDS through
    // an opaque offset, so its words stay per-batch VGPR loads instead of SGPRs held across the loop.
    bool ok = false;
    uint32_t crc = 0;
    bool mine = e < su.nc && x <= p.len;
    if (kChunk) {
      uint64_t lo_ = a_lo, hi_ = all_hi ? ~0ull : a_hi;   // opaque per batch: not held across the loop
      lo_ = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo_ >> 32)) << 32) |
            __builtin_amdgcn_readfirstlane((uint32_t)lo_);
      hi_ = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(hi_ >> 32)) << 32) |
            __builtin_amdgcn_readfirstlane((uint32_t)hi_);
      asm volatile("" : "+s"(lo_), "+s"(hi_));
      mine = mine && (lo_ == 0 || x + need > lo_) && x + need <= hi_;
    }
    if (last && mine) {
      const uint32_t hd[12] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w, h2.x, h2.y, h2.z, h2.w};
      uint32_t z = 0;
      asm volatile("" : "+v"(z));
      const UniMemo* mv = &su.m + z;
      crc = funnel(hd[1], hd[0], hsh);
      ok = !read_eof(p.len, p.io, (int64_t)x, kMaxHeader);
      if (mv->k || mv->v) ok = ok && !read_eof(p.len, p.io, (int64_t)(x + mv->hs), (uint64_t)mv->k + mv->v);
      else ok = ok && crc != 0u;   // crc == 0 && kSize == 0 && vSize == 0: ErrLogEndOfFile
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 9; ++i)
        if ((uint32_t)i < nw) diff |= (funnel(hd[i + 2], hd[i + 1], hsh) ^ mv->w[i]) & mv->msk[i];   // wave-uniform
      ok = ok && diff == 0u && (reg ^ KL) == ~crc;   // getEntryCrc == stored crc (log_file.go:141-143)
    }
    const uint64_t bad = __ballot((last && mine && !ok) ? 1 : 0);
    if (bad && lane == 0)
      atomicMin((unsigned long long*)F, (unsigned long long)(b * E + ((uint32_t)__builtin_ctzll(bad) >> lg)));
    if (ok && gb + e < p.cap && (!fill || kHash)) {
      uint32_t z = 0;
      asm volatile("" : "+v"(z));
      const UniMemo& m = *(&su.m + z);
      if (p.kind == LDB_TUPLE_ENTRY) {
        ldb_entry en;
        en.offset = x;
        en.expired_at = m.expired_at;
        en.tx_id = m.tx_id;
        en.crc = crc;
        en.k_size = m.k;
        en.v_size = m.v;
        en.tx_stat = (uint16_t)m.tx_stat;
        en.stat = (uint8_t)m.stat;
        en.hdr_size = (uint8_t)m.hs;
        en.enc_hdr_size = (uint8_t)m.enc;
        en.pad_[0] = en.pad_[1] = en.pad_[2] = 0;
        en.fid = p.fid;
        reinterpret_cast<ldb_entry*>(p.out)[gb + e] = en;
      } else {
        store_tuple(reinterpret_cast<ldb_index_tuple*>(p.out) + gb + e, uni_pos(m, x), m.k, m.v);
      }
      if (kHash) {   // merge mode: the key's hash, from the lines this wave just loaded
        const uint32_t kx = hx + m.hs;
        p.hash_out[gb + e] = key_hash_w(
            [&](uint32_t i, uint64_t* w) {
              const uint32_t a0 = kx + i, al = a0 & ~3u, s0 = a0 & 3u;
              const uint4 q = ld16(rs, al);
              const uint32_t q4 = ld4(rs, al + 16);
              w[0] = (uint64_t)funnel(q.y, q.x, s0) | ((uint64_t)funnel(q.z, q.y, s0) << 32);
              w[1] = (uint64_t)funnel(q.w, q.z, s0) | ((uint64_t)funnel(q4, q.w, s0) << 32);
            },
            m.k);
      }
    }
  }
}

// The runs' INDEX tuples, written by each workgroup once its waves' verify loops are done, as a dense
// sweep of its own slice of the chain's tuples (so the stores of early workgroups overlap the loads of
// the others, and no fill launch follows). A tuple's bytes depend only on its index (uni_pos of its x and
// the run's memo), not on who verified the entry, so the slice covers every entry of run r below F_r
// as visible now (and below cap): every one below the final K is written, and one at or past the final
// K (F may still drop) lies beyond n_entries, where the region pipeline writes its own tuples from K on.
// F_r <= M_r (uni_discover), so no run writes into the next run's tuples. The slices come from the runs'
// nc (the same in every workgroup; F as seen here is not).
// (Round 4: writing each run's tuples before verifying it, once its end is known, so the stores would
// drain under the verification's loads, measured and rejected: config 4 k_uniform 0.764 -> 0.792 ms.
// Per-wave stores of each wave's own batches, 4 scattered 256-B pieces per instruction, cost
// 61 us at config 4 against 33 for the separate dense sweep; a fill per run, after each run's verify
// loop, 20 us at config 1 against 8 for this one sweep -- a barrier per run. Streaming stores (nt):
// config 4 k_uniform 0.808 -> 0.768 ms on one box -- with plain stores the tuples sat dirty in L2, and
// uni_finish's agent-scope release wrote them back before the last workgroup could go on. A fill wave writing the
// slice while the other 15 verify -- K re-read every 4096 tuples -- was measured and rejected: config 4
// k_uniform 0.897 ms against 0.84, 15 verifying waves per CU lose more than the overlap gains.)
__device__ __forceinline__ void uni_post_fill(const Pipe& p, const UniRuns& ru) {
  __syncthreads();
  const UniRun& rl = ru.r[ru.n - 1];
  const uint64_t ntot = rl.gbase + rl.nc;   // chain entries over every run's candidates
  const uint64_t per = ((ntot + gridDim.x - 1) / gridDim.x + 63) & ~63ull;   // whole KiB of tuples each
  const uint64_t lo = (uint64_t)blockIdx.x * per;
  uint64_t hi = lo + per < ntot ? lo + per : ntot;
  hi = hi < p.cap ? hi : p.cap;
  ldb_index_tuple* out = reinterpret_cast<ldb_index_tuple*>(p.out);
  for (int r = 0; r < ru.n; ++r) {
    const UniRun& q = ru.r[r];
    if (q.gbase >= hi || q.gbase + q.nc <= lo) continue;
    const uint64_t f = uni_fload(uni_fword(p, r));
    const uint64_t a = lo > q.gbase ? lo : q.gbase;
    uint64_t z = q.gbase + (q.nc < f ? q.nc : f);
    z = z < hi ? z : hi;
    const uint64_t sz = q.m.sz, ya = q.y - q.gbase * sz;   // x of chain entry g: ya + g sz (mod 2^64)
    for (uint64_t g = a + threadIdx.x; g < z; g += blockDim.x) {
      store_tuple_nt(out + g, uni_pos(q.m, ya + g * sz), q.m.k, q.m.v);
    }
  }
}

// The device path's run prefix, finished (the last k_uniform workgroup to be done, after every
// workgroup's F updates). kMulti: K = gbase + F of the first run whose F lies below its end M (a failure
// inside it; M = the next run's gbase - this one's), or of the last run; x0 = the position of chain entry
// K (dyn[0] = K, dyn[5] = x0, chain_x0). When the chain stops right there -- the header window there is
// unreadable (io.EOF), or it decodes as the zero sentinel (ErrLogEndOfFile), a key/value read past the
// bound (io.EOF) or a malformed header (log_file.go:116-139) -- the scan is complete: this writes the
// ldb_scan_result and sets dyn[3] = kUniDone, and the region pipeline's kernels leave at once. A file the
// runs cover to its terminal (BASELINE configs 1, 2, 4, 5) then pays no region kernel work. Wave 0 of the
// last workgroup: the entry at x0 is decoded through readlane, one byte per lane.
template <bool kMulti>
__device__ __forceinline__ void uni_finish(const Pipe& p, const UniRuns& ru) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    s_last = atomicAdd((unsigned long long*)&p.dyn[4], 1ull) == (unsigned long long)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last || threadIdx.x >= 64) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const uint32_t lane = threadIdx.x;
  uint64_t K = ~0ull, x0 = 0;
  if (kMulti) {
    for (int r = 0; r < ru.n; ++r) {
      const uint64_t f = uni_fload(uni_fword(p, r));
      const bool last = r == ru.n - 1;
      if (last || f < ru.r[r + 1].gbase - ru.r[r].gbase) {
        if (f == ~0ull) break;
        K = ru.r[r].gbase + f;
        x0 = ru.r[r].y + f * ru.r[r].m.sz;
        break;
      }
    }
  } else {
    K = uni_fload(p.dyn);
    if (K != ~0ull) x0 = K * ru.r[0].m.sz;
  }
  if (lane == 0) {
    p.dyn[4] = 0;
    if (K != ~0ull) {
      p.dyn[0] = K;
      p.dyn[5] = x0;
    }
  }
  if (K == ~0ull) return;   // (unreachable: the candidate at or past len always fails)
  int32_t st;
  if (read_eof(p.len, p.io, (int64_t)x0, kMaxHeader)) {
    st = LDB_EOF_WINDOW;
  } else {
    const uint32_t b = x0 + lane < p.len ? (uint32_t)p.img[x0 + lane] : 0u;
    auto fetch = [&](int i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)b, i); };
    st = classify_entry(fetch, p.len, p.io, x0).status;
  }
  if (st != LDB_EOF_WINDOW && st != LDB_EOF_SENTINEL && st != LDB_EOF_KV && st != LDB_ERR_MALFORMED) return;
  if (lane != 0) return;
  ldb_scan_result res;
  res.status = K > p.cap ? LDB_ERR_CAPACITY : st;
  res.fid = p.fid;
  res.n_entries = K;
  res.end_off = x0;
  res.n_repairs = 0;
  res.n_regions = 0;
  res.n_fast = 0;
  res.n_broken = 0;
  res.n_run = K;
  res.n_sweep = 0;
  *p.result = res;
  p.dyn[3] = kUniDone;
}
// the region pipeline's kernels: nothing to do once the run prefix finished the scan
__device__ __forceinline__ bool scan_done(const Pipe& p) { return p.dyn[3] == kUniDone; }

// One run's verification: uni_waves instantiated for its slicing S and alignment (a switch over S on
// a wave-uniform value).
template <bool kChunk, bool kHash, bool kFill, int NW>
__device__ __forceinline__ void uni_run(const Pipe& p, const UniRun& q, uint64_t* F, const uint8_t* lp2,
                                        const uint32_t* comb, int lane, int wave, uint64_t a_lo, uint64_t a_hi,
                                        uint64_t bound, uint32_t wg = blockIdx.x, uint32_t nwg = gridDim.x) {
  const bool al = (q.m.sz & 3u) == 0 && (q.g.t & 3u) == 0 && (q.y & 3u) == 0;   // every window and header dword-aligned
  switch (q.g.S) {   // uni_geometry: 1 <= S <= kUniSteps
#define LDB_UNI_CASE(n)                                                                                 \
  case n:                                                                                               \
    if (al) uni_waves<n, kChunk, kHash, kFill, true, NW>(p, q, F, lp2, comb, lane, wave, wg, nwg, a_lo, a_hi, bound); \
    else uni_waves<n, kChunk, kHash, kFill, false, NW>(p, q, F, lp2, comb, lane, wave, wg, nwg, a_lo, a_hi, bound);  \
    break;
    LDB_UNI_CASE(1) LDB_UNI_CASE(2) LDB_UNI_CASE(3) LDB_UNI_CASE(4) LDB_UNI_CASE(5) LDB_UNI_CASE(6)
    LDB_UNI_CASE(7) LDB_UNI_CASE(8) LDB_UNI_CASE(9) LDB_UNI_CASE(10) LDB_UNI_CASE(11) LDB_UNI_CASE(12)
#undef LDB_UNI_CASE
    default: break;
  }
}

// The run prefix's LDS: the combine tables first, then the LP2 block at a byte offset below 64 KiB, so every
// table read carries its base in the DS instruction's 16-bit offset (round 6: with the LP2 block first, the
// combine tables sat above 64 KiB and the kernel kept ~20 table bases in VGPRs, at the 128-VGPR cap of a
// 1024-thread workgroup: 7 VGPRs spilled to scratch). The LP2 base stays a multiple of 128 B (its lanes'
// dwords map to 32 distinct banks).
constexpr uint32_t kUniLp2Off = (4 * (uint32_t)kUniTabWords + 255u) & ~255u;
static_assert(kUniLp2Off + 256 < 65536, "the LP2 block's base must fit a DS offset");
#define LDB_UNI_LDS                                                                 \
  __shared__ __attribute__((aligned(256))) uint8_t uni_lds[kUniLp2Off + kLp2Bytes]; \
  uint32_t* const comb = reinterpret_cast<uint32_t*>(uni_lds);                     \
  uint8_t* const lp2 = uni_lds + kUniLp2Off

// kChunk: a_lo, a_hi: image bytes [0, a_hi) are in place; candidates not already taken by a launch
// with a_hi = a_lo are this launch's (a_hi >= len: every remaining candidate). !kChunk: the whole image.
// LDS: the 64 KiB LP2 block, the combine tables and the setup (~90 KiB): one workgroup of 16 waves per
// CU, 4 waves per SIMD, up to 128 VGPRs. The device path (!kChunk, !kHash) verifies every run of the
// log (UniRuns) and writes the INDEX tuples itself; a chunked scan (the image still arriving over
// PCIe) and the merge's hashed scans take the first run only.
template <bool kChunk, bool kHash>
__global__ __launch_bounds__(64 * kUniWaves) void k_uniform(Pipe p, uint64_t a_lo, uint64_t a_hi) {
  LDB_UNI_LDS;   // comb: the combine tables (shift by 2^i P bytes), lp2: the LP2 block
  __shared__ UniSetup su;
  __shared__ UniRuns ru;
  constexpr bool kMulti = !kChunk && !kHash;
#ifdef LDB_STAMPS   // setup cost: slot 9 the LP2 block, slot 17 uni_prepare (thread 0 of every workgroup)
  uint64_t t0_, t1_, t2_;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0_) :: "memory");
#endif
  // kMulti: workgroup 0 sets the control words k_init sets on the other paths (enqueue_scan): the region
  // pipeline's counters, the done flag and its counter (no other workgroup touches them before it has
  // taken the run list, which workgroup 0 publishes after this), x0 unset
  if (kMulti && LDB_FOLD_INIT && blockIdx.x == 0 && threadIdx.x < 8) {
    p.ctr[threadIdx.x] = 0u;
    if (threadIdx.x == 3 || threadIdx.x == 4 || threadIdx.x == 7) p.dyn[threadIdx.x] = 0;
    if (threadIdx.x == 5) p.dyn[5] = ~0ull;
    if (p.swctl && threadIdx.x == 0) {   // the sweep tier's control words (k_sweep follows)
      p.swctl->fail = ~0ull;
      p.swctl->state = 0;
      p.swctl->stop = 0;
    }
  }
  if (kMulti && LDB_FOLD_INIT && blockIdx.x == 0 && threadIdx.x < kTailCtlBytes / 4)
    p.tail[threadIdx.x] = threadIdx.x >= kTailCtlBytes / 4 - 2 ? ~0u : 0u;   // (k_sweep's tail_init)
  // (workgroup 0 of a kMulti launch finds the runs first: its LP2 block afterwards, off that chain)
  if (!kMulti || blockIdx.x != 0) lp2_build(lp2, p.gtab);
#ifdef LDB_STAMPS
  __syncthreads();
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_) :: "memory");
#endif
  uint64_t bound;
  if (!uni_prepare<kMulti>(p, su, ru, comb, kChunk ? a_hi : p.len, bound)) return;   // (its __syncthreads also publish the LP2 block)
  if (kMulti && blockIdx.x == 0 && gridDim.x == 1) lp2_build(lp2, p.gtab);   // (published by uni_take_runs' barriers)
  __syncthreads();
#ifdef LDB_STAMPS
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t2_) :: "memory");
  if (threadIdx.x == 0) {
    atomicAdd((unsigned long long*)&g_stamps[9], (unsigned long long)(t1_ - t0_));
    atomicAdd((unsigned long long*)&g_stamps[17], (unsigned long long)(t2_ - t1_));
  }
#endif
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (!kMulti) {
    UNI_T(v0);
    uni_run<kChunk, kHash, !kHash, kUniWaves>(p, ru.r[0], p.dyn, lp2, comb, lane, wave, a_lo, a_hi, bound);
    UNI_T(v1);
    UNI_ADD(6, v0, v1);
    if (!kChunk || a_hi >= p.len) uni_finish<false>(p, ru);
  } else {
    // the runs as workgroup 0 publishes them (uni_discover), each verified up to its F; once the list is
    // final, the INDEX tuples written
    const bool verifies = gridDim.x == 1 || blockIdx.x != 0;   // workgroup 0 found the runs, and starts last
    bool built0 = blockIdx.x != 0;   // (workgroup 0 builds its combine tables only to verify)
    for (int have = 0;;) {
      const uint64_t w = uni_take_runs(p, ru, have, blockIdx.x != 0);
      const int n = (int)(uint32_t)w;
      if (verifies) {
        if (!built0 && n > 0) {
          uni_build_comb(p, ru.r[0].g, comb, nullptr);
          built0 = true;
        }
        for (int r = have; r < n; ++r) {
          const UniRun& q = ru.r[r];
          uint64_t* F = uni_fword(p, r);
          if (r > 0 && (q.g.G != ru.r[r - 1].g.G || q.g.P != ru.r[r - 1].g.P)) {
            UNI_T(c0);
            __syncthreads();   // every wave is done with the old tables
            uni_build_comb(p, q.g, comb, nullptr);
            UNI_T(c1);
            UNI_ADD(5, c0, c1);
          }
          UNI_T(v0);
          if (gridDim.x == 1) uni_run<kChunk, kHash, !kHash, kUniWaves>(p, q, F, lp2, comb, lane, wave, a_lo, a_hi, ~0ull);
          else
            uni_run<kChunk, kHash, !kHash, kUniWaves>(p, q, F, lp2, comb, lane, wave, a_lo, a_hi, ~0ull, blockIdx.x - 1,
                                                      gridDim.x - 1);
          UNI_T(v1);
          UNI_ADD(6, v0, v1);
        }
      }
      have = n;
      if (w & kUniFinal) break;
      __syncthreads();   // (every wave past the runs before the next copy-in)
    }
    uni_refresh_nc(p, ru);
    UNI_T(f0);
    if (p.kind == LDB_TUPLE_INDEX) uni_post_fill(p, ru);
    UNI_T(f1);
    UNI_ADD(7, f0, f1);
    uni_finish<true>(p, ru);
    UNI_T(f2);
    UNI_ADD(8, f1, f2);
  }
}
static_assert(kUniSteps == 12, "k_uniform's switch covers S = 1..12");

// The run's INDEX tuples as one dense sweep after k_uniform (kFill): entry e < K (and < cap) at x = e sz
// gets {uni_pos(memo, x), k, v}. A chunked scan fills per chunk, the entries that launch's k_uniform
// took (the same byte predicate); every one of them below the K seen now was verified by that launch
// (a later chunk only lowers K past its own entries).
template <bool kChunk>
__device__ __forceinline__ void uni_fill(const Pipe& p, uint64_t a_lo, uint64_t a_hi) {
  if (p.kind != LDB_TUPLE_INDEX || p.dyn[2] != kUniReady) return;
  const UniSetup* gsu = reinterpret_cast<const UniSetup*>(p.uni);
  if (!gsu->g.ok) return;
  const UniMemo m = gsu->m;
  const uint64_t sz = m.sz, K = p.dyn[0];   // raw: ~0 while a chunked scan has seen no failure yet
  uint64_t e_lo = 0, e_hi = K < p.cap ? K : p.cap;
  if (kChunk) {   // entries whose bytes and 48 header bytes lie in [0, a_hi) but not in [0, a_lo)
    const uint64_t need = sz > 48 ? sz : 48;
    if (a_lo) e_lo = a_lo >= need ? (a_lo - need) / sz + 1 : 0;   // x + need > a_lo
    if (a_hi < p.len) {
      const uint64_t hi = a_hi >= need ? (a_hi - need) / sz + 1 : 0;   // x + need <= a_hi
      e_hi = e_hi < hi ? e_hi : hi;
    }
  }
  ldb_index_tuple* out = reinterpret_cast<ldb_index_tuple*>(p.out);
  for (uint64_t e = e_lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e_hi; e += (uint64_t)gridDim.x * blockDim.x)
    store_tuple(out + e, uni_pos(m, e * sz), m.k, m.v);
}
template <bool kChunk>
__global__ __launch_bounds__(kFillThreads) void k_uniform_fill(Pipe p, uint64_t a_lo, uint64_t a_hi) {
  uni_fill<kChunk>(p, a_lo, a_hi);
}

// a batched scan's run prefixes: grid.y = file. The Pipes travel as kernel arguments (not through
// a device pointer like the other batched stages): kernarg loads stay re-loadable constants.
constexpr int kUniBatch = 16;
struct UniBatch {
  Pipe p[kUniBatch];
};
template <bool kB>
using PipeArg = typename std::conditional<kB, UniBatch, Pipe>::type;
// the batched scan's fill: grid.y = file. With hashes (merge mode) the same pass also emits each run
// entry's key hash (ldb::key_hash_w): one thread per entry reads its key as dword-aligned 16-B pieces.
// In the verify loop the hash was serial work on one lane in G plus key loads issued after the CRC and
// waited for at once (config 5 replay: 1.64 ms with it there, 0.97 without).
template <bool kHash>
__global__ __launch_bounds__(kFillThreads) void k_uniform_fill_batch(UniBatch b) {
  const Pipe p = b.p[blockIdx.y];
  uni_fill<false>(p, 0, p.len);
  if (!kHash || p.dyn[2] != kUniReady) return;
  const UniSetup* gsu = reinterpret_cast<const UniSetup*>(p.uni);
  if (!gsu->g.ok) return;
  const uint64_t sz = gsu->m.sz, K = p.dyn[0];
  const uint32_t hs = gsu->m.hs, kl = gsu->m.k;
  const uint64_t n = K < p.cap ? K : p.cap;
  // a wave's 64 entries share one descriptor based at its first entry's key (descriptors must be
  // wave-uniform: rsrc_of reads lane 0's base), each lane at its own offset from there
  for (uint64_t e0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); e0 < n; e0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = e0 + (threadIdx.x & 63u);
    const uint64_t wb = (e0 * sz + hs) & ~3ull;
    const uint64_t wbn = (p.len - wb + 3) & ~3ull;
    const __amdgpu_buffer_rsrc_t rs = rsrc_of(p.img + wb, (uint32_t)(wbn < 0xFFFFFFFFull ? wbn : 0xFFFFFFFFull));
    if (e >= n) continue;
    const uint32_t kx = (uint32_t)(e * sz + hs - wb), ka = kx & ~3u, s0 = kx & 3u;
    p.hash_out[e] = key_hash_w(
        [&](uint32_t i, uint64_t* w) {
          const uint4 q = ld16(rs, ka + i);
          const uint32_t q4 = ld4(rs, ka + i + 16);
          w[0] = (uint64_t)funnel(q.y, q.x, s0) | ((uint64_t)funnel(q.z, q.y, s0) << 32);
          w[1] = (uint64_t)funnel(q.w, q.z, s0) | ((uint64_t)funnel(q4, q.w, s0) << 32);
        },
        kl);
  }
}
template <bool kHash>
__global__ __launch_bounds__(64 * kUniWaves) void k_uniform_batch(UniBatch b) {
  const Pipe p = b.p[blockIdx.y];
  LDB_UNI_LDS;
  __shared__ UniSetup su;
  __shared__ UniRuns ru;
  lp2_build(lp2, p.gtab);
  uint64_t bound;
  if (!uni_prepare<false>(p, su, ru, comb, p.len, bound)) return;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uni_run<false, false, true, kUniWaves>(p, ru.r[0], p.dyn, lp2, comb, lane, wave, 0, p.len, bound);
}
// ---------------------------------------------------------------- the region pipeline's main phase
// (k_region phase M; rounds 1-5 the k_scan_main kernel). Item vb of vg: its kWPB waves each scan a contiguous
// run of regions, the runs dealt as if vg workgroups were launched. tab: the CRC table block in LDS (a
// static array of k_region: its address is a link-time constant, so every table read folds the table base
// into the ds_read offset field), copied once per workgroup (tabs); smem: the waves' rings after it.
__device__ __forceinline__ void main_item(const Pipe& p, uint32_t vb, uint32_t vg, uint32_t* tab, uint8_t* smem,
                                          int& tabs) {
  // ctr[] was zeroed by k_init, which opens every pipeline (enqueue_scan), or on a run-prefix scan by
  // k_uniform's workgroup 0 (LDB_FOLD_INIT); the terminal words start at "none" (read only by the later
  // phases, after this one completes)
  if (vb == 0 && threadIdx.x < 2) p.tpos[threadIdx.x] = ~0ull;
  {   // an item whose waves have no region (the run prefix took them) is done before the table copy
    const uint64_t rf0 = first_region(p), nr0 = p.nreg - rf0, nw0 = (uint64_t)vg * kWPB;
    if (rf0 + (uint64_t)vb * kWPB * ((nr0 + nw0 - 1) / nw0) >= p.nreg) return;
  }
  if (tabs != kLdsRegion) {
    copy_tables(tab, p.gtab);
    __syncthreads();
    tabs = kLdsRegion;
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* wbase = smem + wave * (sizeof(WaveLds) + kNB * kBuf);
  WaveLds* wl = reinterpret_cast<WaveLds*>(wbase);
  uint8_t* ring = wbase + sizeof(WaveLds);
  const uint32_t ring_lds = (uint32_t)(uintptr_t)smem + (uint32_t)(ring - smem);
  // each wavefront scans a contiguous run of regions in file order, so the chain state of one
  // region (ldb_chain.h) carries into the next
  // the replay covers regions [rf, nreg): the run prefix (k_uniform) took everything before x0
  const uint64_t rf = first_region(p), nr = p.nreg - rf;
  const uint64_t gw = (uint64_t)vb * kWPB + wave, nw = (uint64_t)vg * kWPB;
  const uint64_t per = (nr + nw - 1) / nw;
  const uint64_t rb = rf + gw * per;
  const uint64_t count = rb < p.nreg ? (p.nreg - rb < per ? p.nreg - rb : per) : 0;
  GpuWave wp{lane};
  ChainState st;
  chain_reset(st);
  if (rb == rf && count) {   // the replay's entry point: known, its owner verified by the run prefix
    st.on = 2;
    st.x = chain_x0(p);
  }
  // Warm-up: a run after the first starts kWarm regions early and processes those dry (no tuple, no
  // summary), so the speculative entry has settled onto the chain by the run's first region (a chain
  // from a false start falls back onto the true one within a few entries): far fewer broken links
  // between runs for k_repair to walk.
  const uint64_t warm = (count && rb > rf) ? ((uint64_t)kWarm < rb - rf ? (uint64_t)kWarm : rb - rf) : 0;
  const uint64_t r00 = rb - warm, total = count + warm;
  uint32_t n_fast = 0;
  uint32_t declines = 0;        // consecutive lean declines (give-up mode, below)
  uint32_t backoff = 0;         // give-up windows in a row that ended in another decline
  // LDS-DMA ring of kNB buffers: region i+kNB is staged into region i's buffer as soon as region i
  // has read it for the last time (buffer_free), so the DMA overlaps the summary, its stores and
  // the next region's wait.
  for (int b = 0; b < kNB; ++b)
    if ((uint64_t)b < total) stage_dma(p.img, p.len, r00 + (uint64_t)b, ring_lds + b * kBuf, lane);
  for (uint64_t i = 0; i < total; ++i) {
    // Wait for region i's DMA: vmcnt(N) retires all but the N youngest VM ops (issue order, global
    // ops only in this kernel). Younger than DMA(i) are, in steady state, the kStoresPerRegion
    // buffer stores of iteration i-kNB (every region, lean or general, dry or not, issues exactly
    // those after its next region's DMA) and, for kNB > 1, the DMAs of regions
    // i+1 .. i+kNB-1 (kG instructions each; their stores are not counted: conservative).
    // Near the end of the run fewer DMAs were issued after DMA(i) (none past the run's last region).
    {
      const uint64_t left = total - 1 - i;
      const uint64_t ahead = left < (uint64_t)(kNB - 1) ? left : (uint64_t)(kNB - 1);   // DMAs issued after DMA(i)
      if (ahead == (uint64_t)(kNB - 1) && i >= (uint64_t)kNB) wait_vm<(kNB - 1) * kG + kStoresPerRegion>();
      else if (kNB >= 3 && ahead >= 2) wait_vm<2 * kG>();
      else if (kNB >= 2 && ahead >= 1) wait_vm<kG>();
      else wait_vm<0>();
    }
    GpuWave::sync();
    wp.stamp(6);
    const uint64_t r = r00 + i;
    const bool dry = i < warm;   // warm-up: every store of the region dropped (still issued: the counted waits)
    const uint32_t slot = (uint32_t)(i % kNB);
    View v;
    v.buf = ring + slot * kBuf;
    v.tab = tab;
    v.xw = p.xw;
    v.gsh = p.gsh;
    v.R0 = r * (uint64_t)kW;
    v.rlen = region_len(p, r);
    v.len = p.len;
    v.io = p.io;
    ldb_index_tuple* sc = p.scratch + r * (uint64_t)kRegionCap;
    const __amdgpu_buffer_rsrc_t sc_rs = rsrc_of(sc, (uint32_t)(kRegionCap * sizeof(ldb_index_tuple)));
    ChainPriv cq;
    if (!st.on && zero_region(wp, v)) {
      // all-zero speculative region (a preallocated file tail, fileio.go:66-68): covered, raw register 0
      // (ldb_chain.h zero_region)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      GpuWave::sync();
      if (i + kNB < total) stage_dma(p.img, p.len, r00 + i + kNB, ring_lds + slot * kBuf, lane);
      store_summary(p, r, zero_summary(), lane, dry);
      n_fast += dry ? 0u : 1u;
      declines = 0;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      GpuWave::sync();
      continue;
    }
    // The warm-up ended inside an entry covering the run's whole first region: most often a false
    // header the warm-up speculated onto (its size a random varint), which would leave the run on a
    // false chain until its CRC fails and a walker re-runs the run region by region. The run's first
    // region speculates afresh instead (1 GiB writer mix, emulated: 6 broken links and 190 serial
    // re-runs -> none); a true entry that long costs one speculation, which finds it covered.
    if (i == warm && warm && st.on && st.x >= v.R0 + (uint64_t)kW) chain_reset(st);
    bool released = false;
    const bool spec_entry = !st.on;   // this region's entry is speculated (run start, warm-up, after a terminal)
    // after 2 declines in a row the next 8 regions go straight to region_process, then one lean
    // attempt; each attempt that declines again doubles the window (up to 256 regions): a log whose
    // regions cannot go lean (11-B entries, adversarial "tiny": 1.45 ms of k_scan_main with a fixed
    // window of 8 against 0.96 before the lean path took several starts per slice) stops paying for
    // attempts, and one success returns to attempting every region
    const uint32_t win = 8u << (backoff < 5 ? backoff : 5);
    const bool skip = declines >= 2 && declines < 2 + win;
    // (round 4: a single-start form of region_chained until a wave's first decline was measured and
    // rejected -- config 3 2.73 -> 2.84 ms, and the writer mix's speculation then took false starts
    // where a lane's true first start has a second one behind it: 1 ms of k_repair)
    const bool fast = !skip && region_chained(
        wp, v, ring + slot * kBuf, wl->sh, st, [&](int) -> ChainPriv& { return cq; },
        [&](bool valid, uint32_t slot_, uint64_t pos, uint32_t k, uint32_t vv) {
          store16(sc_rs, valid && !dry ? slot_ * 16u : kDrop, (uint32_t)pos, (uint32_t)(pos >> 32), k, vv);
        },
        [&] {   // the buffer's last read is behind us: stage the run's region i + kNB into it
          const uint64_t nx = i + kNB;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          GpuWave::sync();
          if (nx < total) stage_dma(p.img, p.len, r00 + nx, ring_lds + slot * kBuf, lane);
          released = true;
        },
        [] {},   // a declined region is reloaded below
        [&](const RegionSum& s) { store_summary(p, r, s, lane, dry); });
    if (fast) {
      n_fast += dry ? 0u : 1u;
      declines = 0;
      backoff = 0;
    } else {
      // The exact general routine, inline (run_region, ldb_chain.h): entered at the chain's position
      // when the chain is on, else speculating; its exit carries the chain into the next region. A
      // log whose regions mostly decline (entries < kMinFast) is thus replayed chained within each
      // wave's run instead of speculated region by region in a later kernel, whose wrong starts the
      // repair then re-ran (1 GiB writer mix: 6039 region re-runs, 8.6 ms of k_repair).
      if (released) {   // the ring slot may already hold region i + kNB: reload this one
        wait_vm<0>();
        GpuWave::sync();
        for (int k = lane; k < (kW + kHalo) / 16; k += 64) {
          const uint64_t off = v.R0 + (uint64_t)k * 16;
          uint4 x = make_uint4(0, 0, 0, 0);
          if (off < p.len) x = *reinterpret_cast<const uint4*>(p.img + off);
          *reinterpret_cast<uint4*>(ring + slot * kBuf + kPre + k * 16) = x;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        GpuWave::sync();
      }
      uint32_t enter = kForceSpec;
      if (st.on && st.x >= v.R0) enter = st.x - v.R0 < (uint64_t)v.rlen ? (uint32_t)(st.x - v.R0) : kForceNone;
      LanePriv q;
      region_process(
          wp, v, wl->sh, enter, &wl->rs, [&](int) -> LanePriv& { return q; },
          [&](uint32_t slot_, uint64_t pos, uint32_t k, uint32_t vv) {
            store16(sc_rs, dry ? kDrop : slot_ * 16u, (uint32_t)pos, (uint32_t)(pos >> 32), k, vv);
          },
          [] {});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      GpuWave::sync();
      const RegionSum o = wl->rs;
      // the next region's DMA, then this region's one summary store (the counted waits above)
      if (i + kNB < total) stage_dma(p.img, p.len, r00 + i + kNB, ring_lds + slot * kBuf, lane);
      store_summary(p, r, o, lane, dry);
      chain_after_general(st, o, v, enter);
      if (++declines >= 3 + win) {   // the attempt after a window declined too
        declines = 2;
        backoff += 1;
      }
    }
    // A speculated entry that leaves the chain inside an entry reaching more than kWarmSwallow past
    // this region: most likely a false header (random value bytes decode to random varint sizes),
    // whose covered regions a walker would later re-run one after another. The next region speculates
    // afresh instead; a true entry that long only costs that region a speculation.
    if (spec_entry && st.on && st.x > v.R0 + kWarmSwallow) chain_reset(st);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    GpuWave::sync();
    wp.stamp(7);
  }
  if (lane == 0 && n_fast) atomicAdd(&p.ctr[3], n_fast);
#ifdef LDB_STAMPS
  if (lane == 0)
    for (int k = 0; k < kStampSlots; ++k) atomicAdd((unsigned long long*)&g_stamps[k], (unsigned long long)wp.acc[k]);
#endif
}

// ---------------------------------------------------------------- k_link
// One thread per region: its outgoing link's flag (ldb_pipeline.h fail_flags; every flag of the
// pipeline is written, the first region's also for the virtual source rf - 1) and its walker claim
// cleared. ctr[0] counts the broken links.
// (k_region phase L; item vb of vg strides over the regions [rf, nreg) in pieces of blockDim)
__device__ __forceinline__ void link_item(const Pipe& p, uint32_t vb, uint32_t vg) {
  const uint64_t rf = first_region(p);
  uint8_t* fl = fail_flags(p);
  uint32_t nb = 0;
  for (uint64_t r = rf + (uint64_t)vb * blockDim.x + threadIdx.x; r < p.nreg; r += (uint64_t)vg * blockDim.x) {
    const bool bad = link_broken(p, r);
    fl[r - rf + 1] = bad ? 1 : 0;
    repair_claims(p)[r] = 0;
    nb += bad ? 1u : 0u;
    if (r == rf) {
      const bool b0 = p.rs[rf].start != chain_x0(p);
      fl[0] = b0 ? 1 : 0;
      nb += b0 ? 1u : 0u;
    }
  }
  if (nb) atomicAdd(&p.ctr[0], nb);
}

// ---------------------------------------------------------------- k_repair
struct CohRd {
  const Pipe* p;
  __device__ uint64_t start(uint64_t r) const {
    return __hip_atomic_load(&p->rs[r].start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ uint64_t exitp(uint64_t r) const {
    return __hip_atomic_load(&p->rs[r].exitp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ uint32_t sflag(uint64_t r) const {
    return __hip_atomic_load(&p->rs[r].sflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// Nothing to do unless k_link flagged a broken link (ctr[0]). Then, DESIGN.md §3.3:
// 1. every wave of the grid takes flagged sources (64 flags per ballot) and walks each one
//    optimistically (ldb_pipeline.h walk_source), claiming every region it re-runs;
// 2. the last workgroup to finish (ctr[6]) re-checks every link over the summaries as they now are
//    (the same flags, rewritten), and its first wave runs the serial repair() from those flags.
// ctr[2] = regions re-run (both phases).
constexpr int kRepWaves = 16;   // k_repair: as many waves as fit beside the table block
// (k_region phase R, run only when phase L flagged a broken link: ctr[0]. Item vb of vg: the walkers of
// phase 1; the workgroup that completes the last item then runs phase 2, repair_item(..., true).)
static_assert(kRepWaves == kWPB && sizeof(WaveLds) + kBuf <= sizeof(WaveLds) + kNB * kBuf,
              "k_region: the repair waves use the main phase's per-wave LDS");
__device__ __forceinline__ void repair_item(const Pipe& p, uint32_t vb, uint32_t vg, uint32_t* tab, uint8_t* smem,
                                            int& tabs, bool phase2) {
  if (tabs != kLdsRegion) {
    copy_tables(tab, p.gtab);
    __syncthreads();
    tabs = kLdsRegion;
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveLds* wl = reinterpret_cast<WaveLds*>(smem + wave * (sizeof(WaveLds) + kNB * kBuf));
  uint8_t* buf = smem + wave * (sizeof(WaveLds) + kNB * kBuf) + sizeof(WaveLds);
  GpuWave wp{lane};
  CohRd rd{&p};
  const int64_t rf = (int64_t)first_region(p);
  uint8_t* fl = fail_flags(p);
  uint32_t* claims = repair_claims(p);
  const uint64_t nflag = n_fail_flags(p);
  bool serial_phase = false;
  auto run = [&](uint64_t r, uint32_t enter) -> RegionSum {
    const uint64_t R0 = r * (uint64_t)kW;
    // synchronous staging through registers
    for (int k = lane; k < (kW + kHalo) / 16; k += 64) {
      const uint64_t off = R0 + (uint64_t)k * 16;
      uint4 d = make_uint4(0, 0, 0, 0);
      if (off < p.len) d = *reinterpret_cast<const uint4*>(p.img + off);
      *reinterpret_cast<uint4*>(buf + kPre + k * 16) = d;
    }
    GpuWave::sync();
    View v;
    v.buf = buf;
    v.tab = tab;
    v.xw = p.xw;
    v.gsh = p.gsh;
    v.R0 = R0;
    v.rlen = region_len(p, r);
    v.len = p.len;
    v.io = p.io;
    ldb_index_tuple* sc = p.scratch + r * (uint64_t)kRegionCap;
    LanePriv q;
    region_process(
        wp, v, wl->sh, enter, &wl->rs, [&](int) -> LanePriv& { return q; },
        [&](uint32_t slot, uint64_t pos, uint32_t k, uint32_t vv) { store_tuple(sc + slot, pos, k, vv); }, [] {});
    const RegionSum s = wl->rs;
    if (lane == 0) {
      store_region(p, r, s);
      if (serial_phase && s.status != kCont && s.start != kNone64)   // keep the terminal bits a superset
        atomicOr((unsigned long long*)&term_bits(p)[r / 64], 1ull << (r % 64));
      // the serial repair reads its own summaries back coherently; a walker's reads are hints only,
      // and an agent-scope fence per region (an L2 writeback and invalidate on gfx950) cost ~1 ms a
      // region with many walkers writing: phase 1 fences once, before the done count
      if (serial_phase) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (serial_phase) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    GpuWave::sync();
    return s;
  };
  // ---- 1. optimistic walkers
  // One window of 64 consecutive flags per wave, its sources walked in order (a walker then starts
  // from the exit an earlier walker of the same window may just have rewritten; handing the sources of
  // one window to several waves measured 4-40x slower: walkers from stale exits walk garbage). Windows
  // are dealt across the CUs first (wave-major), so a file with few windows still gets one CU each.
  uint32_t runs = 0;
  const uint64_t nwave = (uint64_t)vg * kRepWaves;
  if (!phase2)
  for (uint64_t w = (uint64_t)wave * vg + vb; w * 64 < nflag; w += nwave) {
    const uint64_t b = w * 64;
    uint64_t m = __ballot(b + lane < nflag && fl[b + lane] != 0);
    while (m) {
      const int i = __builtin_ctzll(m);
      m &= m - 1;
      // a source region another walker has claimed is being rewritten: its exit is stale, and that
      // walker's walk continues through it anyway
      const int64_t src = rf - 1 + (int64_t)(b + i);
      if (src >= rf && __hip_atomic_load(&claims[src], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) continue;
      // the window's first source whose own region's incoming link is broken too: the previous
      // window's wave walks through it from the true side; walking from its stale exit meanwhile
      // writes off-chain regions the serial pass must then re-run one by one (binary values)
      if (i == 0 && b > 0 && fl[b - 1] != 0) continue;
      runs += walk_source(p, src, rd,
                          [&](uint64_t r) {   // wave-uniform: lane 0 claims, the wave follows
                            uint32_t won = 0;
                            if (lane == 0) won = atomicCAS(&claims[r], 0u, 1u) == 0u ? 1u : 0u;
                            return __shfl((int)won, 0) != 0;
                          },
                          run,
                          // a region the walk would re-run as covered but whose incoming link k_link
                          // found intact is left alone: it sits on a chain with its predecessor, and a
                          // walk from a false source (a speculated header whose size reaches far ahead)
                          // re-running such regions started cascades of re-runs the serial pass redid
                          // one by one (emulated, walkers in reverse order: 1898 + 1723 runs against 180)
                          [&](uint64_t k) { return k > (uint64_t)rf && fl[k - (uint64_t)rf] == 0; });
    }
  }
  if (lane == 0 && runs) atomicAdd(&p.ctr[2], runs);
  if (!phase2) return;
  // ---- 2. the workgroup that completed the last item (every item's summaries and tuples released, then
  // acquired by k_region): links again, then the serial repair
  uint32_t nb = 0;
  // the flags again, 64 to a thread, with their bitmap word; then the terminal bits (flag_bits)
  uint64_t* fb = flag_bits(p);
  uint64_t* tb = term_bits(p);
  const uint64_t nfw = (nflag + 63) / 64, ntw = (p.nreg + 63) / 64;
  for (uint64_t w = threadIdx.x; w < nfw; w += blockDim.x) {
    uint64_t bits = 0;
    for (uint32_t b = 0; b < 64; ++b) {
      const uint64_t i = 64 * w + b;
      if (i >= nflag) break;
      const bool bad = i == 0 ? rd.start((uint64_t)rf) != chain_x0(p) : link_broken(p, (uint64_t)rf - 1 + i);
      fl[i] = bad ? 1 : 0;
      bits |= (uint64_t)(bad ? 1u : 0u) << b;
    }
    fb[w] = bits;
    nb += (uint32_t)__builtin_popcountll(bits);
  }
  for (uint64_t w = (uint64_t)rf / 64 + threadIdx.x; w < ntw; w += blockDim.x) {
    uint64_t bits = 0;
    for (uint32_t b = 0; b < 64; ++b) {
      const uint64_t r = 64 * w + b;
      if (r >= p.nreg) break;
      if (r >= (uint64_t)rf && p.rs[r].status != kCont && p.rs[r].start != kNone64) bits |= 1ull << b;
    }
    tb[w] = bits;
  }
  if (nb) atomicAdd(&p.ctr[7], nb);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (wave != 0 || __hip_atomic_load(&p.ctr[7], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
  serial_phase = true;
  // the lowest set bit at index >= a in bitmap words [0, nw): a lane per word, 64 words per round
  auto next_bit = [&](const uint64_t* bm, uint64_t nw, uint64_t a, bool coherent) -> uint64_t {
    for (uint64_t w0 = a / 64; w0 < nw; w0 += 64) {
      const uint64_t w = w0 + lane;
      uint64_t bits = 0;
      if (w < nw) bits = coherent ? __hip_atomic_load(&bm[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : bm[w];
      if (w == a / 64) bits &= ~0ull << (a % 64);
      const uint64_t m = __ballot(bits != 0);
      if (m) {
        const int L = __builtin_ctzll(m);
        const uint64_t bw = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), L) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bits, L);
        return 64 * (w0 + (uint64_t)L) + (uint64_t)__builtin_ctzll(bw);
      }
    }
    return ~0ull;
  };
  auto next_fail = [&](int64_t done) -> int64_t {   // smallest flagged source > done
    const uint64_t i = next_bit(fb, nfw, (uint64_t)(done - (rf - 1) + 1), false);
    return i < nflag ? rf - 1 + (int64_t)i : INT64_MAX;
  };
  auto first_term = [&](int64_t lo, int64_t hi) -> int64_t {   // candidates from the bits, checked live
    for (uint64_t a = (uint64_t)(lo + 1 > rf ? lo + 1 : rf);;) {
      const uint64_t r = next_bit(tb, ntw, a, true);
      if (r >= p.nreg || (int64_t)r > hi) return -1;
      const int32_t st = __hip_atomic_load(&p.rs[r].status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (st != kCont && rd.start(r) != kNone64) return (int64_t)r;
      a = r + 1;
    }
  };
  const uint32_t n = repair(p, next_fail, rd, first_term, run);
  if (lane == 0 && n) atomicAdd(&p.ctr[2], n);
}

// ---------------------------------------------------------------- k_combine
// (k_region phase C; item vb of vg strides over the kBlkRegions-region blocks, one thread per region)
static_assert(kBlkRegions == 64 * kWPB, "k_region: one thread per region of a block");
__device__ __forceinline__ void combine_item(const Pipe& p, uint32_t vb, uint32_t vg, uint64_t* s_sum) {
  const uint64_t nblk = (p.nreg + kBlkRegions - 1) / kBlkRegions;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint64_t b = vb; b < nblk; b += vg) {
  const uint64_t r = b * kBlkRegions + threadIdx.x;
  uint64_t cnt = 0;
  if (r < p.nreg && r >= first_region(p)) {
    const int32_t st = p.rs[r].status;
    const uint64_t start = p.rs[r].start;
    cnt = p.rs[r].count;
    if (st == kOverflow) {
      atomicOr(&p.ctr[1], 1u);
    } else if (start != kNone64) {
      if (st != kCont) {
        atomicMin((unsigned long long*)&p.tpos[0], (unsigned long long)pack_term(p.rs[r].exitp, st));
      } else {
        const uint64_t x = p.rs[r].exitp;
        if (x >= p.len) atomicMin((unsigned long long*)&p.tpos[0], (unsigned long long)pack_term(p.len, LDB_EOF_WINDOW));
        if ((p.rs[r].sflag & kStraddle) && !combine_region(p, r))
          atomicMin((unsigned long long*)&p.tpos[0], (unsigned long long)pack_term(p.rs[r].soff, LDB_ERR_CRC));
      }
    }
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) cnt += __shfl_xor(cnt, o);
  if (lane == 0) s_sum[wave] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int w = 0; w < kBlkRegions / 64; ++w) t += s_sum[w];
    p.blk[b] = t;
  }
  __syncthreads();   // (s_sum is reused by the next block)
  }
}

// ---------------------------------------------------------------- k_serial
// One lane walks the chain exactly like index.go:84-95 (global memory, byte-wise CRC).
__device__ void serial_walk(const Pipe& p) {
  struct G {
    const uint8_t* q;
    __device__ uint32_t operator()(int i) const { return q[i]; }
  };
  uint64_t off = chain_x0(p), n = run_k(p);   // after the run prefix (0, 0 on the serial test path)
  int st;
  for (;;) {
    EntryInfo e;
    if (read_eof(p.len, p.io, (int64_t)off, kMaxHeader)) {
      e.status = LDB_EOF_WINDOW;
    } else {
      e = classify_entry(G{p.img + off}, p.len, p.io, off);
    }
    if (e.status != kCont) { st = e.status; break; }
    uint32_t crc = 0;
    if (e.h.size > 4) crc = ~g_crc_bytes(p, 0xFFFFFFFFu, off + 4, off + e.size);
    if (crc != e.h.crc) { st = LDB_ERR_CRC; break; }
    if (n < p.cap) {
      if (p.kind == LDB_TUPLE_ENTRY) {
        decode_entry_global(p, off, reinterpret_cast<ldb_entry*>(p.out) + n);
      } else {
        ldb_index_tuple t;
        t.pos = pack_pos(off, e.h);
        t.k_size = e.h.k_size;
        t.v_size = e.h.v_size;
        reinterpret_cast<ldb_index_tuple*>(p.out)[n] = t;
      }
    }
    ++n;
    off += e.size;
  }
  ldb_scan_result res;
  res.status = n > p.cap ? LDB_ERR_CAPACITY : st;
  res.fid = p.fid;
  res.n_entries = n;
  res.end_off = off;
  res.n_repairs = 0;
  res.n_regions = (uint32_t)p.nreg;
  res.n_fast = 0;
  res.n_broken = 0;
  res.n_run = run_k(p) - p.dyn[7];
  res.n_sweep = p.dyn[7];
  *p.result = res;
}
template <bool kB>
__global__ __launch_bounds__(64) void k_serial(Pipe p0, int only_on_overflow, const Pipe* __restrict__ pb) {
  const Pipe p = kB ? pb[blockIdx.y] : p0;  // (a copy: a reference into the kernel arguments costs 28 VGPRs here)
  if (threadIdx.x != 0) return;
  if (only_on_overflow && !p.ctr[1]) return;
  serial_walk(p);
}

// ---------------------------------------------------------------- k_compact
// One workgroup per 1024-region block; each wavefront copies whole regions.

// One workgroup per kBlkRegions regions: its output base is the sum of the earlier blocks'
// counts (k_combine), its regions are scanned in LDS, and tuples are copied flat (thread j of
// the block's output range finds its region by binary search). The block holding the terminal
// region writes the ldb_scan_result.
// (k_region phase K; item vb of vg strides over the blocks. LDS: s_off kBlkRegions + 1 words, s_wsum and s_part
// one word per wave)
__device__ __forceinline__ void compact_item(const Pipe& p, uint32_t vb, uint32_t vg, uint32_t* s_off, uint32_t* s_wsum,
                                             uint64_t* s_part) {
  if (p.ctr[1]) {   // a region overflowed its tuple slots (phase C): the serial walker redoes the scan
    if (vb == 0 && threadIdx.x == 0) serial_walk(p);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t T = p.tpos[0];
  uint64_t tp = term_pos(T);
  int32_t ts = term_status(T);
  if (T == ~0ull) { tp = p.len; ts = LDB_ERR_MALFORMED; }  // unreachable: the chain always stops
  const uint64_t rf = first_region(p), K = run_k(p);      // the run prefix's tuples are out[0, K)
  if (rf >= p.nreg) {   // the replay stops right after the run: io.EOF at x0 (log_file.go:117-122)
    if (vb == 0 && tid == 0) {
      ldb_scan_result res;
      res.status = LDB_EOF_WINDOW;
      res.fid = p.fid;
      res.n_entries = K;
      res.end_off = chain_x0(p);
      res.n_repairs = 0;
      res.n_regions = 0;
      res.n_fast = 0;
      res.n_broken = 0;
      res.n_run = K - p.dyn[7];
      res.n_sweep = p.dyn[7];
      if (K > p.cap) res.status = LDB_ERR_CAPACITY;
      *p.result = res;
    }
    return;
  }
  const uint64_t regT = tp / kW;                          // may be nreg when tp == len == nreg * kW
  const uint64_t lastR = regT < p.nreg ? regT : p.nreg - 1;
  // a capped grid strides over the blocks (a file the run prefix took whole launches few workgroups)
  const uint64_t nblk = (p.nreg + kBlkRegions - 1) / kBlkRegions;
  for (uint64_t b = vb; b < nblk; b += vg) {
  const uint64_t r0 = b * kBlkRegions;
  if (r0 > lastR) break;
  // base = sum of the counts of every earlier block (all their regions precede the terminal)
  uint64_t part = 0;
  for (uint64_t i = tid; i < b; i += kBlkRegions) part += p.blk[i];
#pragma unroll
  for (int o = 32; o; o >>= 1) part += __shfl_xor(part, o);
  if (lane == 0) s_part[wave] = part;
  // this block's effective counts, exclusive scan
  const uint64_t r = r0 + tid;
  uint32_t c = 0;
  if (r < p.nreg && r <= regT && r >= rf) {
    c = p.rs[r].count;
    // the terminal is this region's straddle-out entry failing its CRC
    if (r == regT && p.rs[r].status == kCont && (p.rs[r].sflag & kStraddle) && p.rs[r].soff == tp && c > 0) c -= 1;
  }
  uint32_t x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  uint32_t wbase = 0;
  uint64_t base = 0;
#pragma unroll
  for (int w = 0; w < kBlkRegions / 64; ++w) {
    wbase += w < wave ? s_wsum[w] : 0u;
    base += s_part[w];
  }
  s_off[tid] = wbase + x - c;
  if (tid == kBlkRegions - 1) s_off[kBlkRegions] = wbase + x;
  __syncthreads();
  const uint32_t total = s_off[kBlkRegions];
  base += K;
  if (b == lastR / kBlkRegions && tid == 0) {
    const uint64_t n = base + total;
    ldb_scan_result res;
    res.status = ts;
    res.fid = p.fid;
    res.n_entries = n;
    res.end_off = tp;
    res.n_repairs = p.ctr[2];
    res.n_regions = (uint32_t)(p.nreg - rf);
    res.n_fast = p.ctr[3];
    res.n_broken = p.ctr[7];
    res.n_run = K - p.dyn[7];
    res.n_sweep = p.dyn[7];
    if (n > p.cap) res.status = LDB_ERR_CAPACITY;
    if (p.ctr[5]) res.status = LDB_ERR_INTERNAL;   // a device-side index guard fired (never expected)
    if (p.ctr[1]) res.status = kOverflow;  // k_serial redoes the scan
    *p.result = res;
  }
  if (p.ctr[1]) return;
  for (uint32_t j = tid; j < total; j += kBlkRegions) {
    // region i: the last with s_off[i] <= j (empty regions share their successor's offset)
    int lo = 0, hi = kBlkRegions - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_off[mid] <= j) lo = mid; else hi = mid - 1;
    }
    const uint64_t dst = base + j;
    if (dst >= p.cap) break;
    const ldb_index_tuple t = p.scratch[(r0 + lo) * (uint64_t)kRegionCap + (j - s_off[lo])];
    if (p.kind == LDB_TUPLE_ENTRY) decode_entry_global(p, t.pos & 0xFFFFFFFFFFull, reinterpret_cast<ldb_entry*>(p.out) + dst);
    else reinterpret_cast<ldb_index_tuple*>(p.out)[dst] = t;
  }
  __syncthreads();   // s_off / s_wsum / s_part are reused by the next block
  }
}

// Read-only reduction over the image (ldb_read_ceiling): four 16-B loads in flight per thread.
// The practical read ceiling: grid-stride XOR of every 16-B word, 8 non-temporal loads in flight per
// lane, 16 workgroups of 256 per CU (the best of the streaming forms in tools/microbench/mb_read.hip:
// 6.47 TB/s against 5.68 for plain loads and 6.19 for per-wave contiguous chunks).
__global__ __launch_bounds__(256) void k_read_reduce(const uint4* __restrict__ p, uint64_t n16, uint32_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint32_t acc = 0;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n16; i += 8 * stride) {
    v4u32 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p + i + u * stride));
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= x[u][0] ^ x[u][1] ^ x[u][2] ^ x[u][3];
  }
  for (; i < n16; i += stride) {
    const uint4 x = p[i];
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  acc = __reduce_xor_sync(~0ull, acc);
  if ((threadIdx.x & 63) == 0) atomicXor(&sink[blockIdx.x], acc);
}

#include "ldb_sweep_kern.h"

// ---------------------------------------------------------------- k_sweep, k_region
// Everything after the run prefix, in two launches (rounds 1-5: seven, k_sweep, k_sweep_fin, k_scan_main,
// k_link, k_repair, k_combine, k_compact; on a file the run prefix covers each returned at its first
// instruction, ~10-14 us of every config-2/4 step, profiles/r06_tail_ab.txt):
//   k_sweep   the sweep tier's stream (phase S, sweep_item: one item per workgroup), then the links between
//             its runs (sweep_last, the last workgroup to finish)
//   k_region  F the sweep tier's per-entry CRC checks and tuples (fin_item), then where it ends (sw_finish);
//             then the region pipeline from where the run prefix and the sweep tier stopped: M the regions
//             (main_item), L their links (link_item), R the repair when a link broke (repair_item), C the
//             cross-region CRCs and block counts (combine_item), K the compaction (compact_item)
// The scan may end after any phase (the run prefix's uni_finish or sw_finish writes the result and the done
// word): every workgroup then returns. In k_region each phase is a number of items, the workgroups of the
// launch that kernel used to have, claimed one at a time from a ticket counter by the workgroups that are
// running; the workgroup that completes a phase's last item runs its follow-up (finish, serial repair) and
// publishes the phase, and every workgroup waits for that before its next phase. A workgroup only ever waits
// after the phase's tickets are all taken, i.e. for items that running workgroups hold, so the launch cannot
// deadlock however few of its workgroups are resident (another stream's kernels, a smaller chip). Completion
// releases at agent scope and the wait acquires, as the kernel boundaries did (L2 write-back across the XCDs).
// Measured and rejected (profiles/r06_tail_fused_ab.txt): all seven phases in one launch (the region code's
// register pressure spilled every phase's values to scratch, 224-272 B per lane, and a wave's first scratch
// access costs tens of us at launch scale, tools/microbench/mb_scratch.hip: the sweep 5-7 % slower); S and F
// in one launch (S's stream loop then held the protocol's values in SGPRs and spilled them into the loop: 3 %).
constexpr int kPhS = 0, kPhF = 1, kPhM = 2, kPhL = 3, kPhR = 4, kPhC = 5, kPhK = 6;
constexpr uint32_t kMainLds = kWPB * (sizeof(WaveLds) + kNB * kBuf);
constexpr uint32_t kCompactWsum = (4 * (kBlkRegions + 1) + 15) & ~15u, kCompactPart = kCompactWsum + 4 * kWPB;
constexpr uint32_t kCompactLds = kCompactPart + 8 * kWPB;
constexpr uint32_t cmax(uint32_t a, uint32_t b) { return a > b ? a : b; }
constexpr uint32_t kRegionLds = cmax(cmax(kTabBytes + kMainLds, kCompactLds), kSwFinLds);
static_assert(kTabBytes % 16 == 0 && kLp2Bytes % 256 == 0, "LDS carve alignment");
static_assert(cmax(kSwLds, kSwLinkLds) + 64 <= 160 * 1024 && kRegionLds + 64 <= 160 * 1024, "LDS per workgroup");
static_assert(kRepWaves == kWPB && kSwWaves == kWPB, "every phase runs kWPB waves");

// item counts: the grids the kernels had (every phase has at least one item: its last one runs the
// follow-up and publishes it)
__device__ __forceinline__ uint32_t tail_items(uint64_t want, uint32_t ncu) {
  return (uint32_t)(want < 1 ? 1 : (want < ncu ? want : ncu));
}

// the pipe, fetched again in every phase through a pointer the compiler cannot see through (the kernel
// argument itself, p0 at the kernarg segment's offset 0; a batched launch's device array), so no phase holds
// another's Pipe fields in registers. Made in the kernel's own body (the kernarg segment pointer exists only
// there), every use inlined.
template <bool kB>
struct PipeSrc {
  CPipe ka;
  __device__ __forceinline__ const Pipe& get() const {
    CPipe q = kB ? ka + blockIdx.y : ka;
    asm volatile("" : "+s"(q));
    return *(const Pipe*)q;
  }
};
#define LDB_PIPE_SRC(kB) const PipeSrc<kB> src{(CPipe)__builtin_amdgcn_kernarg_segment_ptr()}

// The phase protocol over Pipe::tail: [0, 8) tickets, [8, 16) items done, [16, 24) published, then the phases'
// start stamps (u64 [16, 24)). s_tail_tk / s_tail_fl: the workgroup's broadcast words.
__shared__ uint32_t s_tail_tk;
__shared__ int s_tail_fl;
struct TailSync {
  __device__ __forceinline__ uint32_t claim(const Pipe& p, int ph) const {
    __syncthreads();   // (every thread has read the previous ticket)
    if (threadIdx.x == 0) {
      s_tail_tk = atomicAdd(&p.tail[ph], 1u);
      if (s_tail_tk == 0) reinterpret_cast<uint64_t*>(p.tail + 32)[ph] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    return s_tail_tk;
  }
  __device__ __forceinline__ bool complete(const Pipe& p, int ph, uint32_t n) const {   // true in the workgroup that completed the last item
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      s_tail_fl = atomicAdd(&p.tail[8 + ph], 1u) == n - 1;
      if (s_tail_fl) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();   // (the workgroup's other threads are ordered after thread 0's acquire by the barrier)
    return s_tail_fl != 0;
  }
  __device__ __forceinline__ void publish(const Pipe& p, int ph) const {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if (p.tacc) {
        const uint64_t t0 = __hip_atomic_load(reinterpret_cast<uint64_t*>(p.tail + 32) + ph, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd((unsigned long long*)&p.tacc[ph], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t0));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store(&p.tail[16 + ph], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __device__ __forceinline__ void wait(const Pipe& p, int ph) const {
    // Thread 0 polls and acquires; the barrier orders the workgroup's other threads after it. (Every thread's
    // own agent-scope acquire, 16 waves per workgroup each invalidating, cost ~30 us per phase boundary.)
    if (threadIdx.x == 0) {
      while (__hip_atomic_load(&p.tail[16 + ph], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) __builtin_amdgcn_s_sleep(4);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
  // a phase whose items are cheap or rare: the plain claim loop
  template <class Body, class Last>
  __device__ __forceinline__ void loop(const Pipe& p, int ph, uint32_t n, Body body, Last last) const {
    for (uint32_t t; (t = claim(p, ph)) < n;) {
      body(t);
      if (complete(p, ph, n)) {
        last(t);
        publish(p, ph);
      }
    }
    wait(p, ph);
  }
  // the first item peeled off the claim loop (a workgroup's usual share is one item): what the compiler
  // hoists out of a loop and holds across it then stays in the loop's copy, and the usual path holds nothing
  // over the item (k_sweep: no scratch access outside the loop copy)
  template <class Body, class Last>
  __device__ __forceinline__ void peeled(const Pipe& p, int ph, uint32_t n, Body body, Last last) const {
    uint32_t t = claim(p, ph);
    if (t < n) {
      body(t);
      if (complete(p, ph, n)) {
        last(t);
        publish(p, ph);
      }
      loop(p, ph, n, body, last);
    } else {
      wait(p, ph);
    }
  }
};
__device__ __forceinline__ bool tail_done(const Pipe& p) {   // after a wait: the scan ended in the phase just published
  return __builtin_amdgcn_readfirstlane((uint32_t)(__hip_atomic_load(&p.dyn[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                                   kUniDone)) != 0u;
}

// The sweep tier's stream (phase S): one item per workgroup, the workgroups of the launch (the round-5 kernel,
// whose code it keeps: no phase protocol inside, so nothing is held across its stream loop -- the same body
// behind k_region's tickets spilled SGPRs into that loop, 3 % slower), then the links by the last workgroup to
// finish (a done counter, no waiting).
#ifdef LDB_SW_TRACE
// (trace builds: per workgroup of k_sweep, [file fid - 1][blockIdx.x] -> start, stream end, end, CU id; real-time
// clock, 100 MHz; tools/sw_trace.py)
constexpr int kSwTraceWgs = 8 * 1024;
__device__ uint64_t g_swtrace[kSwTraceWgs * 4];
#define LDB_SW_STAMP(k, v)                                                                            \
  do {                                                                                                \
    const uint64_t slot_ = (uint64_t)(p.fid - 1) * gridDim.x + blockIdx.x;                            \
    if (threadIdx.x == 0 && slot_ < (uint64_t)kSwTraceWgs) g_swtrace[slot_ * 4 + (k)] = (v);            \
  } while (0)
#else
#define LDB_SW_STAMP(k, v) do {} while (0)
#endif

template <bool kB>
__global__ __launch_bounds__(64 * kSwWaves) void k_sweep(PipeArg<kB> a0) {
  __shared__ __attribute__((aligned(256))) uint8_t lds[cmax(kSwLds, kSwLinkLds)];
  __shared__ int s_last;
  LDB_PIPE_SELECT;
  if (!p.sweep || scan_done(p)) return;   // (uni_finish ended the scan)
  LDB_SW_STAMP(0, __builtin_amdgcn_s_memrealtime());
  LDB_SW_STAMP(3, (uint64_t)__smid());
  int tabs = kLdsNone;
  // the shift tables first, then the LP2 block below 64 KiB, then the hit lists (kSwLds: every table base
  // in the DS instructions' 16-bit offsets, as k_uniform's LDB_UNI_LDS)
  sweep_item(p, blockIdx.x, gridDim.x, lds + kSwShBytes, reinterpret_cast<uint32_t*>(lds),
             reinterpret_cast<uint32_t*>(lds + kSwShBytes + kLp2Bytes), tabs);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  LDB_SW_STAMP(1, __builtin_amdgcn_s_memrealtime());
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    s_last = atomicAdd(&p.tail[8 + kPhS], 1u) == gridDim.x - 1;
    if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!s_last) return;
  sweep_last(p, gridDim.x, lds);
  LDB_SW_STAMP(2, __builtin_amdgcn_s_memrealtime());
}

template <bool kB>
__global__ __launch_bounds__(64 * kWPB) void k_region(PipeArg<kB> a0, uint32_t ncu) {
  __shared__ __attribute__((aligned(256))) uint8_t lds[kRegionLds];
  (void)a0;   // (read through src)
  LDB_PIPE_SRC(kB);
  if (scan_done(src.get())) return;   // the run prefix or the sweep tier ended the scan
  const TailSync ts;
  int tabs = kLdsNone;
  uint32_t* const tab = reinterpret_cast<uint32_t*>(lds);
  uint8_t* const smem = lds + kTabBytes;
  auto none = [](uint32_t) __attribute__((always_inline)) {};
  // ---- the sweep tier's checks (phase F), when k_sweep resolved its links (SwCtl::state, reset where the
  // pipeline starts): one lane per chain entry, then where the tier ends (sw_finish)
  if (src.get().sweep && src.get().swctl->state == 1) {
    const Pipe& p = src.get();
    const uint64_t ncov = p.swctl->ncov;
    const uint32_t nF = tail_items((ncov + kSwWaves - 1) / kSwWaves, ncu);
    ts.peeled(
        p, kPhF, nF,
        [&](uint32_t t) __attribute__((always_inline)) { fin_item(src.get(), t, nF, reinterpret_cast<uint32_t*>(lds), tabs); },
        [&](uint32_t) __attribute__((always_inline)) {
          if (threadIdx.x < 64) sw_finish(src.get());
        });
    if (tail_done(p)) return;
    tabs = kLdsNone;
  }
  {
    const Pipe& p = src.get();
    const uint32_t nM = tail_items((p.nreg + kWPB - 1) / kWPB, ncu);
    ts.loop(p, kPhM, nM, [&](uint32_t t) __attribute__((always_inline)) { main_item(src.get(), t, nM, tab, smem, tabs); }, none);
  }
  {
    const Pipe& p = src.get();
    const uint32_t nL = tail_items((p.nreg - first_region(p) + blockDim.x - 1) / blockDim.x, ncu);
    ts.loop(p, kPhL, nL, [&](uint32_t t) __attribute__((always_inline)) { link_item(src.get(), t, nL); }, none);
  }
  {
    const Pipe& p = src.get();
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&p.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0u) {
      const uint32_t nR = tail_items((p.nreg + 1 + 63) / 64, ncu);
      ts.loop(
          p, kPhR, nR, [&](uint32_t t) __attribute__((always_inline)) { repair_item(src.get(), t, nR, tab, smem, tabs, false); },
          [&](uint32_t t) __attribute__((always_inline)) { repair_item(src.get(), t, nR, tab, smem, tabs, true); });
    }
  }
  tabs = kLdsNone;   // (phases C and K use the LDS as scratch)
  {
    const Pipe& p = src.get();
    const uint32_t nC = tail_items((p.nreg + kBlkRegions - 1) / kBlkRegions, ncu);
    ts.loop(p, kPhC, nC, [&](uint32_t t) __attribute__((always_inline)) { combine_item(src.get(), t, nC, reinterpret_cast<uint64_t*>(lds)); }, none);
  }
  {
    const Pipe& p = src.get();
    const uint32_t nK = tail_items((p.nreg + kBlkRegions - 1) / kBlkRegions, ncu);
    for (uint32_t t; (t = ts.claim(p, kPhK)) < nK;) {   // (the last phase: nothing waits for it)
      compact_item(src.get(), t, nK, reinterpret_cast<uint32_t*>(lds), reinterpret_cast<uint32_t*>(lds + kCompactWsum),
                   reinterpret_cast<uint64_t*>(lds + kCompactPart));
      if (ts.complete(p, kPhK, nK)) ts.publish(p, kPhK);
    }
  }
}

}  // namespace

// ==================================================================== host runtime
struct ldb_ctx {
  int device = 0;
  int n_cu = 256;
  uint32_t* d_tab = nullptr;   // kTabWords
  uint32_t* d_xw = nullptr;    // kW + 1
  uint32_t* d_gsh = nullptr;   // kGsWords register-shift tables (k_combine)
  uint32_t* d_swt = nullptr;   // kSwTabWords: the sweep tier's shift and slicing-by-16 tables (ldb_sweep.h)
  uint64_t* d_tacc = nullptr;  // the tail kernels' per-phase time accumulators (s_memrealtime ticks), read by ldb_kernel_timing_tail
  uint8_t* ws = nullptr;       // workspace
  uint64_t ws_bytes = 0;
  // Workspace fence: the event recorded after the last pipeline enqueued on this context, and the
  // stream it went to. A pipeline enqueued on a different stream first waits on it, so two streams
  // never share the workspace at once (ldb_scan_file_dev only enqueues: the previous scan may still
  // be running when the next call arrives).
  hipEvent_t ws_ev = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_ev_live = false;
  uint32_t scan_epoch = 0;   // device scans enqueued on this context (Pipe::epoch)
  // kernel timing: one event triple per timed launch, recorded without host synchronisation and
  // resolved when the timing is queried (or when the pool is full)
  // start, after the run prefix (k_uniform, and a chunked scan's fills), after k_sweep, after k_region (the end)
  struct EvTriple { hipEvent_t e0, eu, es, e2; };
  std::vector<EvTriple> evs;
  size_t ev_used = 0;
  bool timing = false;
  // host-pointer API staging (ldb_scan_file), grow-only
  uint8_t* h_img = nullptr;
  uint64_t h_img_cap = 0;
  void* h_out = nullptr;
  uint64_t h_out_cap = 0;
  ldb_scan_result* h_res = nullptr;
  hipStream_t h_stream = nullptr;
  // host-image copies (ldb_scan_file): 64 MiB chunks dealt round-robin over n_cp streams
  // (LDB_H2D_STREAMS, default 2: the e2e timings of gpurun_out/e2e_streams.log), one
  // event per chunk for the chunked run prefix (ChunkPlan)
  static constexpr int kMaxCp = 4;
  int n_cp = 0;
  hipStream_t cp[kMaxCp] = {};
  std::vector<hipEvent_t> chunk_ev;
  double t_run = 0, t_sweep = 0, t_main = 0, t_total = 0;
  double t_ph[16] = {};   // k_sweep's and k_region's phases (device clock, d_tacc), summed over the timed scans
  double rt_khz = 100000.0;   // the device's constant clock (s_memrealtime)
  uint64_t t_n = 0;
  // batched scans (enqueue_scan_batch): page-locked staging of the per-file Pipes, reused once the
  // copy of the previous batch has completed (pipes_ev)
  Pipe* h_pipes = nullptr;
  int h_pipes_cap = 0;
  hipEvent_t pipes_ev = nullptr;
  bool pipes_ev_live = false;
  void* merge = nullptr;       // merge/GC workspace (ldb_merge.hip), created on first use
  // host ranges page-locked through ldb_host_register: ldb_scan_file reads or writes a host buffer
  // in place only when one of them covers it whole (the device mapping alone says nothing of its size)
  std::vector<std::pair<uintptr_t, uint64_t>> regs;
  // ldb_scan_file_count's tuples, left in h_out for ldb_scan_copy_out (any other scan call clears it)
  bool ret_valid = false;
  uint64_t ret_n = 0, ret_tsz = 0;
  bool registered(const void* p, uint64_t n) const {
    const uintptr_t a = (uintptr_t)p;
    for (const auto& r : regs)
      if (a >= r.first && n <= r.second && a - r.first <= r.second - n) return true;
    return false;
  }
};

// internal hooks for ldb_merge.hip (not part of the C ABI)
__attribute__((visibility("hidden"))) void ldb_merge_release_(void* m);
__attribute__((visibility("hidden"))) int ldb_ctx_device_(ldb_ctx* c) { return c->device; }
__attribute__((visibility("hidden"))) void** ldb_ctx_merge_slot_(ldb_ctx* c) { return &c->merge; }

static int resolve_timing(ldb_ctx* c) {
  if (!c->ev_used) return LDB_OK;
  for (size_t i = 0; i < c->ev_used; ++i) {
    const ldb_ctx::EvTriple& t = c->evs[i];
    if (hipEventSynchronize(t.e2) != hipSuccess) return LDB_ERR_HIP;
    float u = 0, w = 0, a = 0, b = 0;
    if (hipEventElapsedTime(&u, t.e0, t.eu) != hipSuccess || hipEventElapsedTime(&w, t.eu, t.es) != hipSuccess ||
        hipEventElapsedTime(&a, t.es, t.e2) != hipSuccess || hipEventElapsedTime(&b, t.e0, t.e2) != hipSuccess)
      return LDB_ERR_HIP;
    c->t_run += u;
    c->t_sweep += w;
    c->t_main += a;
    c->t_total += b;
    c->t_n += 1;
  }
  c->ev_used = 0;
  // the tail kernels' phase accumulators (every timed scan has completed: its e2 fired)
  uint64_t acc[16];
  if (hipMemcpy(acc, c->d_tacc, sizeof(acc), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemset(c->d_tacc, 0, sizeof(acc)) != hipSuccess)
    return LDB_ERR_HIP;
  for (int k = 0; k < 16; ++k) c->t_ph[k] += (double)acc[k] / c->rt_khz;
  return LDB_OK;
}

namespace {

struct WsLayout {
  uint64_t nreg, nblk;
  uint64_t o_rs, o_scratch, o_fail, o_ctr, o_tpos, o_dyn, o_uni, o_blk, o_swrw, o_swrg, o_swpl, o_swrun, o_swctl, o_tail, total;
};

WsLayout layout(uint64_t len) {
  WsLayout L;
  L.nreg = (len + kW - 1) / kW;
  if (L.nreg == 0) L.nreg = 1;
  L.nblk = (L.nreg + kBlkRegions - 1) / kBlkRegions;
  uint64_t o = 0;
  auto take = [&](uint64_t bytes) {
    const uint64_t at = o;
    o += (bytes + 255) & ~255ull;
    return at;
  };
  // control words: ctr (8 x u32, zeroed by a hipMemsetAsync at the start of every pipeline), then
  // tpos (2 x u64, set by k_scan_main's first workgroup); take() rounds each field to 256 B
  L.o_ctr = take(32);
  L.o_tpos = take(16);
  L.o_dyn = take(64);   // run prefix: K, entry size, setup-published flag, done flag, done counter (k_uniform)
  L.o_uni = take(kUniBlockBytes);   // run prefix: the published setup, the run list, the runs' F words
  L.o_blk = take(8 * L.nblk);
  L.o_rs = take(sizeof(RegionSum) * L.nreg);
  L.o_fail = take(8 * (L.nreg + 1) + 64);   // fail flags + walker claims (ldb_pipeline.h fail_flags)
  L.o_scratch = take(sizeof(ldb_index_tuple) * (uint64_t)kRegionCap * L.nreg);
  // the sweep tier (ldb_sweep.h): a register per 256-B window and per 16 windows (the image's batches,
  // rounded up, plus one), its run records and control block; its slabs are the scratch tuples above
  L.o_swrw = take(4 * ((len + kSwBatch) / kSwW + 1));
  L.o_swrg = take(4 * ((len + kSwBatch) / (kSwW * kSwG) + 1));
  L.o_swpl = take(4 * ((len + kSwBatch) / 64 + 1));
  L.o_swrun = take(sizeof(SwRun) * (uint64_t)kSwMaxRuns);
  L.o_swctl = take(sizeof(SwCtl));
  L.o_tail = take(kTailCtlBytes);   // the tail kernels' control words
  L.total = o;
  return L;
}

int ensure_ws(ldb_ctx* c, uint64_t bytes) {
  if (c->ws_bytes >= bytes) return LDB_OK;
  // The old workspace may still be read by launches in flight on any stream that used this
  // context (the merge engine alternates two contexts on two streams): drain the device before
  // the free, so a growth can never pull memory from under a running kernel. Growth is rare.
  if (c->ws) {
    (void)hipDeviceSynchronize();
    (void)hipFree(c->ws);
  }
  c->ws = nullptr;
  c->ws_bytes = 0;
  c->ws_ev_live = false;   // nothing in flight uses the new workspace
  if (hipMalloc(&c->ws, bytes) != hipSuccess) return LDB_ERR_NOMEM;
  c->ws_bytes = bytes;
  return LDB_OK;
}

// LDB_SWEEP=0 turns the sweep tier off (A/B: the region pipeline from the run prefix's end, rounds 1-4)
bool sweep_enabled() {
  static const bool on = ldb_knob_int("LDB_SWEEP", 1) != 0;
  return on;
}

Pipe make_pipe(ldb_ctx* c, const WsLayout& L, const uint8_t* img, uint64_t len, uint32_t fid, int io, int kind,
               void* out, uint64_t cap, ldb_scan_result* res, uint8_t* w = nullptr) {
  Pipe p;
  if (!w) w = c->ws;
  p.img = img;
  p.len = len;
  p.io = io;
  p.fid = fid;
  p.nreg = L.nreg;
  p.gtab = c->d_tab;
  p.xw = c->d_xw;
  p.gsh = c->d_gsh;
  p.rs = reinterpret_cast<RegionSum*>(w + L.o_rs);
  p.scratch = reinterpret_cast<ldb_index_tuple*>(w + L.o_scratch);
  p.fail_src = reinterpret_cast<int64_t*>(w + L.o_fail);
  p.ctr = reinterpret_cast<uint32_t*>(w + L.o_ctr);
  p.tpos = reinterpret_cast<uint64_t*>(w + L.o_tpos);
  p.blk = reinterpret_cast<uint64_t*>(w + L.o_blk);
  p.dyn = reinterpret_cast<uint64_t*>(w + L.o_dyn);
  p.uni = w + L.o_uni;
  p.hash_out = nullptr;
  p.out = out;
  p.cap = cap;
  p.kind = kind;
  p.result = res;
  p.swrw = reinterpret_cast<uint32_t*>(w + L.o_swrw);
  p.swrg = reinterpret_cast<uint32_t*>(w + L.o_swrg);
  p.swpl = reinterpret_cast<uint32_t*>(w + L.o_swpl);
  p.swrun = reinterpret_cast<SwRun*>(w + L.o_swrun);
  p.swctl = reinterpret_cast<SwCtl*>(w + L.o_swctl);
  p.swt = c->d_swt;
  p.scratch_bytes = sizeof(ldb_index_tuple) * (uint64_t)kRegionCap * L.nreg;
  p.tail = reinterpret_cast<uint32_t*>(w + L.o_tail);
  p.tacc = c->timing ? c->d_tacc : nullptr;
  p.sweep = sweep_enabled() ? 1u : 0u;
  return p;
}

// Note the stream of the pipeline just enqueued (see ldb_ctx::ws_ev). No marker is recorded per
// pipeline (one was ~10 us between the config-4 pipelines): a scan stream used alone pays nothing.
int fence_ws(ldb_ctx* c, hipStream_t s) {
  c->ws_stream = s;
  c->ws_ev_live = true;
  return LDB_OK;
}
// The workspace is free for stream s once the last pipeline enqueued on another stream has finished.
// An event is recorded on the old stream only when the context owns it (h_stream lives as long as the
// context) or is the null stream; a caller's stream may have been destroyed since its last call (the C ABI
// allows that), and recording on a dead handle is undefined, so a switch away from one drains the device
// instead. A context used from one stream never switches; the merge's scan contexts keep to their own
// streams.
int ws_wait(ldb_ctx* c, hipStream_t s) {
  if (!c->ws_ev_live || c->ws_stream == s) return LDB_OK;
  // (the null stream and the context's own stream always exist: an event on them is safe)
  if (c->ws_stream != nullptr && (c->ws_stream != c->h_stream || !c->h_stream)) {
    LDB_HIP(hipDeviceSynchronize());
    c->ws_ev_live = false;
    return LDB_OK;
  }
  if (!c->ws_ev && hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming) != hipSuccess) return LDB_ERR_HIP;
  LDB_HIP(hipEventRecord(c->ws_ev, c->ws_stream));
  LDB_HIP(hipStreamWaitEvent(s, c->ws_ev, 0));
  return LDB_OK;
}

// kernel timing (ldb_kernel_timing): the event triple of the pipeline about to be enqueued, its start
// recorded; null when timing is off
int timing_begin(ldb_ctx* c, hipStream_t s, const ldb_ctx::EvTriple** out) {
  *out = nullptr;
  if (!c->timing) return LDB_OK;
  if (c->ev_used == c->evs.size()) {
    if (c->evs.size() < 4096) {
      ldb_ctx::EvTriple t{};
      LDB_HIP(hipEventCreate(&t.e0));
      LDB_HIP(hipEventCreate(&t.eu));
      LDB_HIP(hipEventCreate(&t.es));
      LDB_HIP(hipEventCreate(&t.e2));
      c->evs.push_back(t);
    } else {
      const int rc = resolve_timing(c);
      if (rc != LDB_OK) return rc;
    }
  }
  const ldb_ctx::EvTriple* ev = &c->evs[c->ev_used++];
  LDB_HIP(hipEventRecord(ev->e0, s));
  *out = ev;
  return LDB_OK;
}

// the control words every region pipeline starts from (enqueue_scan)
// dyn: [0] K (dyn_val: ~0 = no failure seen, 0 = no run), [1] entry size, [2] setup flag, [3] done
// flag (uni_finish), [4] k_uniform's done counter, [5] x0 (uni_finish), [6] runs published (uni_discover)
// the tail kernels' control words and the sweep tier's (every path but the device path's run prefix, which sets
// them in k_uniform's workgroup 0)
__device__ __forceinline__ void tail_init(const Pipe& p, uint32_t t) {
  if (t < kTailCtlBytes / 4) p.tail[t] = t >= kTailCtlBytes / 4 - 2 ? ~0u : 0u;   // (the last u64: a min stamp)
  if (t == 0) {
    p.swctl->fail = ~0ull;
    p.swctl->state = 0;
    p.swctl->stop = 0;
  }
}
__global__ __launch_bounds__(64) void k_init(Pipe p, uint64_t dyn_val) {
  if (threadIdx.x < 8) p.ctr[threadIdx.x] = 0u;
  if (threadIdx.x < 3) p.dyn[threadIdx.x] = dyn_val;
  if (threadIdx.x == 3 || threadIdx.x == 4 || threadIdx.x == 6 || threadIdx.x == 7) p.dyn[threadIdx.x] = 0;
  if (threadIdx.x == 5) p.dyn[5] = ~0ull;   // x0 not finished: K sz (no run: 0)
  tail_init(p, threadIdx.x);
}

// k_sweep, k_region: one workgroup per CU (their LDS), fewer for a file whose phases have fewer items
// (tail_items: the sweep's stream, the region pipeline's main phase)
int sweep_grid(const ldb_ctx* c, uint64_t len) {
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((len / kSwBatch + 2 + kSwWaves - 1) / kSwWaves, (uint64_t)c->n_cu));
}
int region_grid(const ldb_ctx* c, uint64_t nreg) {
  return (int)std::max<uint64_t>(1, std::min<uint64_t>((nreg + kWPB - 1) / kWPB, (uint64_t)c->n_cu));
}

int uniform_grid(const ldb_ctx* c, uint64_t bytes) {
  const uint64_t batches = bytes / kUniMinSize / 64 + 1;   // entries are >= kUniMinSize B in a run, <= 64 per wave
  return std::max(1, (int)std::min<uint64_t>((batches + kUniWaves - 1) / kUniWaves, (uint64_t)c->n_cu));
}
// k_uniform_fill: a dense sweep, 2 workgroups of 1024 threads per CU (tools/microbench/mb_uni.hip wr_W0:
// 207 MB of tuples in 34 us)
int fill_grid(const ldb_ctx* c, uint64_t bytes) {
  return std::max(1, (int)std::min<uint64_t>(bytes / 16 / kFillThreads + 1, (uint64_t)c->n_cu * 2));
}


// An image that is still being copied in: bytes [0, avail[i]) are in place once ev[i] has fired
// (avail ascending, the last = len). The run prefix then verifies its candidates chunk by chunk,
// each launch waiting only for its chunk, so it overlaps the copy; the region pipeline waits for all.
struct ChunkPlan {
  int n;
  const uint64_t* avail;
  const hipEvent_t* ev;
};

// no_run: skip the run prefix (k_uniform), e.g. for an image read in place from host memory, where
// its per-lane gathered rows would cross PCIe several times; the region pipeline's LDS-DMA staging
// reads every byte once in 1 KiB pieces.
int enqueue_scan(ldb_ctx* c, const uint8_t* d_img, uint64_t len, uint32_t fid, int io, int kind, void* d_out,
                 uint64_t cap, ldb_scan_result* d_res, hipStream_t s, bool serial, bool no_run = false,
                 const ChunkPlan* plan = nullptr, uint64_t* hash_out = nullptr) {
  if (!c || !d_res || (io != LDB_IO_FILEIO && io != LDB_IO_MMAP) ||
      (kind != LDB_TUPLE_INDEX && kind != LDB_TUPLE_ENTRY) || (cap && !d_out))
    return LDB_ERR_ARG;
  if (len && !d_img) return LDB_ERR_ARG;
  if (((uintptr_t)d_img & 15) != 0) return LDB_ERR_ARG;
  if (len >= (1ull << 40)) return LDB_ERR_ARG;  // tuple offsets are 40-bit
  const WsLayout L = layout(len);
  int rc = ensure_ws(c, L.total);
  if (rc != LDB_OK) return rc;
  Pipe p = make_pipe(c, L, d_img, len, fid, io, kind, d_out, cap, d_res);
  p.hash_out = hash_out;
  // the workspace is free once the last pipeline enqueued on another stream has finished
  rc = ws_wait(c, s);
  if (rc != LDB_OK) return rc;
  // every pipeline starts from zeroed control words, in stream order: nothing depends on how the
  // previous pipeline on this workspace ended, or on what a fresh allocation held
  // (the region pipeline's control words are set by k_init below; the serial path's here)
  const bool chunked = plan && plan->n > 0 && !serial && len >= (uint64_t)kMaxHeader && !no_run;
  if (plan && !chunked)   // nothing overlaps the copy: the whole image first
    for (int i = 0; i < plan->n; ++i) LDB_HIP(hipStreamWaitEvent(s, plan->ev[i], 0));
  if (serial || len < (uint64_t)kMaxHeader) {
    LDB_HIP(hipMemsetAsync(c->ws + L.o_ctr, 0, 32, s));
    LDB_HIP(hipMemsetAsync(c->ws + L.o_tpos, 0xFF, 16, s));
    LDB_HIP(hipMemsetAsync(c->ws + L.o_dyn, 0, 64, s));   // no run prefix: the walk starts at 0 (dyn[5] = x0 = 0)
    hipLaunchKernelGGL(k_serial<false>, dim3(1), dim3(64), 0, s, p, 0, nullptr);
    LDB_HIP(hipGetLastError());
    return fence_ws(c, s);
  }
  const ldb_ctx::EvTriple* ev = nullptr;
  rc = timing_begin(c, s, &ev);
  if (rc != LDB_OK) return rc;
  // the run prefix: K = ~0 until k_uniform lowers it to the first entry outside the run
  // ctr zero; K = ~0 and the setup not published (no_run: K = 0): one tiny launch instead of two
  // memsets (a blit launch each, ~10 us of the config-4 step between them)
  // the device path's whole-image run prefix (k_uniform<false, false>) sets the control words itself
  // (its workgroup 0, before it publishes the run list; the list word carries this scan's epoch): one
  // launch fewer, ~4.5 us of every such scan
  p.epoch = ++c->scan_epoch;
  const bool fold_init = !no_run && !chunked && !p.hash_out && LDB_FOLD_INIT;
  if (!fold_init) hipLaunchKernelGGL(k_init, dim3(1), dim3(64), 0, s, p, no_run ? 0ull : ~0ull);
  if (!no_run) {
    auto launch = [&](uint64_t lo, uint64_t hi) {
      const int ug = uniform_grid(c, hi - lo);
      if (chunked)
        hipLaunchKernelGGL((k_uniform<true, false>), dim3(ug), dim3(64 * kUniWaves), 0, s, p, lo, hi);
      else if (p.hash_out)
        hipLaunchKernelGGL((k_uniform<false, true>), dim3(ug), dim3(64 * kUniWaves), 0, s, p, lo, hi);
      else
        hipLaunchKernelGGL((k_uniform<false, false>), dim3(ug), dim3(64 * kUniWaves), 0, s, p, lo, hi);
    };
    if (chunked) {   // each chunk's run entries are filled as soon as that chunk is verified
      uint64_t lo = 0;
      for (int i = 0; i < plan->n; ++i) {
        LDB_HIP(hipStreamWaitEvent(s, plan->ev[i], 0));
        const uint64_t hi = i + 1 == plan->n ? len : std::min(plan->avail[i], len);
        launch(lo, hi);
        if (kind == LDB_TUPLE_INDEX)
          hipLaunchKernelGGL(k_uniform_fill<true>, dim3(fill_grid(c, hi - lo)), dim3(kFillThreads), 0, s, p, lo, hi);
        lo = hi;
      }
    } else {
      launch(0, len);   // its workgroups also write the runs' INDEX tuples (uni_post_fill)
    }
  }
  if (ev) LDB_HIP(hipEventRecord(ev->eu, s));
#ifdef LDB_TAIL_ABL   // attribution builds only (results wrong unless the run prefix covers the file): no tail
  if (ev) LDB_HIP(hipEventRecord(ev->es, s));
  if (ev) LDB_HIP(hipEventRecord(ev->e2, s));
  return fence_ws(c, s);
#endif
  // everything after the run prefix: the sweep tier (k_sweep), then the region pipeline (k_region)
  hipLaunchKernelGGL(k_sweep<false>, dim3(sweep_grid(c, len)), dim3(64 * kSwWaves), 0, s, p);
  if (ev) LDB_HIP(hipEventRecord(ev->es, s));
  hipLaunchKernelGGL(k_region<false>, dim3(region_grid(c, L.nreg)), dim3(64 * kWPB), 0, s, p, (uint32_t)c->n_cu);
  if (ev) LDB_HIP(hipEventRecord(ev->e2, s));
  LDB_HIP(hipGetLastError());
  return fence_ws(c, s);
}

// ---------------------------------------------------------------- batched scans
// Several device-resident images scanned as ONE pipeline: every stage is one launch whose grid.y
// is the file (each file's Pipe in a device array at the head of the workspace, each file its own
// workspace slice), so the per-file run prefixes share one dispatch with a single tail and the small
// stitching kernels run once for all files instead of once per file. Every file must be a plain
// device scan (len >= kMaxHeader, 16-B aligned); the caller falls back to enqueue_scan otherwise.
struct BatchFile {
  const uint8_t* img;
  uint64_t len;
  uint32_t fid;
  void* out;
  uint64_t cap;
  ldb_scan_result* res;
  uint64_t* hash_out;   // all files or none
};

bool batch_eligible(const uint8_t* img, uint64_t len) {
  return img && len >= (uint64_t)kMaxHeader && ((uintptr_t)img & 15) == 0 && len < (1ull << 40);
}

// the control words every pipeline starts from (enqueue_scan's memsets): ctr zero, K = ~0, setup
// not published
__global__ __launch_bounds__(64) void k_batch_init(const Pipe* __restrict__ pb) {
  const Pipe& p = pb[blockIdx.x];
  if (threadIdx.x < 8) p.ctr[threadIdx.x] = 0u;
  if (threadIdx.x < 4 || threadIdx.x == 5) p.dyn[threadIdx.x] = ~0ull;   // [3]: not done; [5]: x0 = K sz
  if (threadIdx.x == 4 || threadIdx.x == 6 || threadIdx.x == 7) p.dyn[threadIdx.x] = 0;
  tail_init(p, threadIdx.x);
}

int enqueue_scan_batch(ldb_ctx* c, int nf, const BatchFile* f, int io, int kind, hipStream_t s) {
  if (!c || nf < 0 || (io != LDB_IO_FILEIO && io != LDB_IO_MMAP) ||
      (kind != LDB_TUPLE_INDEX && kind != LDB_TUPLE_ENTRY))
    return LDB_ERR_ARG;
  if (nf == 0) return LDB_OK;
  const bool hashed = f[0].hash_out != nullptr;
  std::vector<WsLayout> Ls(nf);
  std::vector<uint64_t> off(nf);
  uint64_t o = (sizeof(Pipe) * (uint64_t)nf + 255) & ~255ull;
  int ug = 1;
  uint64_t max_len = 0, max_nreg = 1;
  for (int i = 0; i < nf; ++i) {
    if (!batch_eligible(f[i].img, f[i].len) || !f[i].res || (f[i].cap && !f[i].out) ||
        (f[i].hash_out != nullptr) != hashed)
      return LDB_ERR_ARG;
    Ls[i] = layout(f[i].len);
    off[i] = o;
    o += Ls[i].total;
    ug = std::max(ug, uniform_grid(c, f[i].len));
    max_len = std::max(max_len, f[i].len);
    max_nreg = std::max(max_nreg, Ls[i].nreg);
  }
  int rc = ensure_ws(c, o);
  if (rc != LDB_OK) return rc;
  if (!c->pipes_ev) LDB_HIP(hipEventCreateWithFlags(&c->pipes_ev, hipEventDisableTiming));
  if (c->pipes_ev_live) LDB_HIP(hipEventSynchronize(c->pipes_ev));   // the previous batch's copy is done
  c->pipes_ev_live = false;
  if (c->h_pipes_cap < nf) {
    if (c->h_pipes) (void)hipHostFree(c->h_pipes);
    c->h_pipes = nullptr;
    c->h_pipes_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_pipes), sizeof(Pipe) * (size_t)nf) != hipSuccess)
      return LDB_ERR_NOMEM;
    c->h_pipes_cap = nf;
  }
  for (int i = 0; i < nf; ++i) {
    c->h_pipes[i] = make_pipe(c, Ls[i], f[i].img, f[i].len, f[i].fid, io, kind, f[i].out, f[i].cap, f[i].res,
                              c->ws + off[i]);
    c->h_pipes[i].hash_out = f[i].hash_out;
  }
  const Pipe* d_pipes = reinterpret_cast<const Pipe*>(c->ws);
  UniBatch ub{};   // a launch's pipes, by value (k_sweep<true>, k_region<true>)
  // k_sweep, k_region: the chip's workgroups dealt over the files, not one file's grid per file (round 3: 16 files of
  // 256 MiB launched 16 x 256 k_scan_main workgroups that queued behind each other even when every run
  // prefix covered its file; profiles/r03_s35_merge_spread_ab.json, r04_batch_spread_writer_mix_ab.txt)
  const int tg = std::max(1, (c->n_cu + nf - 1) / nf);
  rc = ws_wait(c, s);
  if (rc != LDB_OK) return rc;
  LDB_HIP(hipMemcpyAsync(const_cast<Pipe*>(d_pipes), c->h_pipes, sizeof(Pipe) * (size_t)nf, hipMemcpyHostToDevice, s));
  LDB_HIP(hipEventRecord(c->pipes_ev, s));
  c->pipes_ev_live = true;
  const ldb_ctx::EvTriple* ev = nullptr;
  rc = timing_begin(c, s, &ev);
  if (rc != LDB_OK) return rc;
  const unsigned n = (unsigned)nf;
  hipLaunchKernelGGL(k_batch_init, dim3(n), dim3(64), 0, s, d_pipes);
  // the run prefixes: the whole batch gets the workgroups one file's launch would (uniform_grid, 2
  // per CU at most), dealt evenly over its files (LDB_UNI_BATCH_BPC: workgroups per CU, A/B)
  static const int bpc = std::max(1, ldb_knob_int("LDB_UNI_BATCH_BPC", 1));
  for (int i0 = 0; i0 < nf; i0 += kUniBatch) {
    UniBatch ub{};
    const int m = std::min(kUniBatch, nf - i0);
    const int ugb = std::min(ug, std::max(1, (c->n_cu * bpc + m - 1) / m));
    for (int i = 0; i < m; ++i) ub.p[i] = c->h_pipes[i0 + i];
    hipLaunchKernelGGL(k_uniform_batch<false>, dim3(ugb, (unsigned)m), dim3(64 * kUniWaves), 0, s, ub);
    if (kind == LDB_TUPLE_INDEX || hashed) {
      uint64_t maxlen = 0;
      for (int i = 0; i < m; ++i) maxlen = std::max(maxlen, ub.p[i].len);
      const int fg = std::max(1, std::min(fill_grid(c, maxlen), (c->n_cu * 2 + m - 1) / m));
      if (hashed)
        hipLaunchKernelGGL(k_uniform_fill_batch<true>, dim3(fg, (unsigned)m), dim3(kFillThreads), 0, s, ub);
      else
        hipLaunchKernelGGL(k_uniform_fill_batch<false>, dim3(fg, (unsigned)m), dim3(kFillThreads), 0, s, ub);
    }
  }
  if (ev) LDB_HIP(hipEventRecord(ev->eu, s));
  // LDB_SWEEP_SPLIT=1 (A/B): one k_sweep launch per file instead of one over (vg, n). While the batch's pipes came
  // from a device array (flat accesses) that won for the writer mix (2.39 -> 2.19 ms); with the pipes in the
  // kernel arguments the one launch is level there and faster for Zipf values and the merge
  // (profiles/r06_sweep_split_ab.txt, r06_batch_kernarg_ab.txt)
  static const bool split = ldb_knob_int("LDB_SWEEP_SPLIT", 0) == 1;
  if (split)
    for (unsigned i = 0; i < n; ++i)
      hipLaunchKernelGGL(k_sweep<false>, dim3(sweep_grid(c, c->h_pipes[i].len)), dim3(64 * kSwWaves), 0, s,
                         c->h_pipes[i]);
  else
    for (int i0 = 0; i0 < nf; i0 += kUniBatch) {   // (the pipes by value: kUniBatch files per launch)
      const int m = std::min(kUniBatch, nf - i0);
      for (int i = 0; i < m; ++i) ub.p[i] = c->h_pipes[i0 + i];
      hipLaunchKernelGGL(k_sweep<true>, dim3(sweep_grid(c, max_len), (unsigned)m), dim3(64 * kSwWaves), 0, s, ub);
    }
  if (ev) LDB_HIP(hipEventRecord(ev->es, s));
  for (int i0 = 0; i0 < nf; i0 += kUniBatch) {
    const int m = std::min(kUniBatch, nf - i0);
    for (int i = 0; i < m; ++i) ub.p[i] = c->h_pipes[i0 + i];
    hipLaunchKernelGGL(k_region<true>, dim3(std::min(tg, region_grid(c, max_nreg)), (unsigned)m), dim3(64 * kWPB), 0, s,
                       ub, (uint32_t)c->n_cu);
  }
  if (ev) LDB_HIP(hipEventRecord(ev->e2, s));
  LDB_HIP(hipGetLastError());
  return fence_ws(c, s);
}

// LDB_SCAN_BATCH=0 turns the batched multi-file path off (A/B)
bool batch_enabled() {
  static const bool on = ldb_knob_int("LDB_SCAN_BATCH", 1) != 0;
  return on;
}

}  // namespace

extern "C" {

int ldb_abi_version(void) { return LDB_ABI_VERSION; }

// internal (merge engine): ldb_scan_file_dev that also writes the key hash of every run-prefix entry
// k < min(n_run, cap) to d_hash[k] (ldb::key_hash_w, the merge table's hash)
__attribute__((visibility("hidden"))) int ldb_scan_file_dev_hashed(ldb_ctx* c, const uint8_t* d_image, uint64_t len,
                                                                   uint32_t fid, int io_type, void* d_out,
                                                                   uint64_t cap, ldb_scan_result* d_result,
                                                                   void* stream, uint64_t* d_hash) {
  if (!c) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  return enqueue_scan(c, d_image, len, fid, io_type, LDB_TUPLE_INDEX, d_out, cap, d_result, (hipStream_t)stream,
                      false, false, nullptr, d_hash);
}

// internal (merge engine): the replay scans of several device images in one batched pipeline
// (enqueue_scan_batch), index tuples; d_hash null or one array per file (ldb_scan_file_dev_hashed).
// Returns LDB_ERR_ARG without enqueuing anything when the batch is off or a file is not eligible.
__attribute__((visibility("hidden"))) int ldb_scan_files_dev_batched(ldb_ctx* c, int n_files,
                                                                     const uint8_t* const* d_images,
                                                                     const uint64_t* lens, const uint32_t* fids,
                                                                     int io_type, void* const* d_outs,
                                                                     const uint64_t* caps,
                                                                     ldb_scan_result* d_results, void* stream,
                                                                     uint64_t* const* d_hash) {
  if (!c || n_files <= 0 || !batch_enabled()) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  std::vector<BatchFile> bf(n_files);
  for (int i = 0; i < n_files; ++i) {
    if (!batch_eligible(d_images[i], lens[i])) return LDB_ERR_ARG;
    bf[i] = BatchFile{d_images[i], lens[i], fids[i], d_outs[i], caps[i], d_results + i, d_hash ? d_hash[i] : nullptr};
  }
  return enqueue_scan_batch(c, n_files, bf.data(), io_type, LDB_TUPLE_INDEX, (hipStream_t)stream);
}

const char* ldb_status_str(int s) {
  switch (s) {
    case LDB_OK: return "ok";
    case LDB_EOF_WINDOW: return "eof (header window)";
    case LDB_EOF_SENTINEL: return "end of log entries (zero header)";
    case LDB_EOF_KV: return "eof (key/value)";
    case LDB_ERR_CRC: return "invalid crc";
    case LDB_ERR_MALFORMED: return "malformed entry header";
    case LDB_ERR_CAPACITY: return "output capacity exceeded";
    case LDB_ERR_ARG: return "invalid argument";
    case LDB_ERR_HIP: return "hip runtime error";
    case LDB_ERR_NOMEM: return "out of device memory";
    case LDB_ERR_INTERNAL: return "internal error (device-side index guard)";
    default: return "unknown status";
  }
}

uint64_t ldb_workspace_bytes(uint64_t len) { return layout(len).total; }

int ldb_ctx_create(int device, ldb_ctx** out) {
  if (!out) return LDB_ERR_ARG;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return LDB_ERR_HIP;
  ldb_ctx* c = new (std::nothrow) ldb_ctx();
  if (!c) return LDB_ERR_NOMEM;
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0) c->rt_khz = khz;
  std::vector<uint32_t> tab(kTabWords), xw(kW + 1), gsh(kGsWords), swt(kSwTabWords);
  build_tables(tab.data());
  for (int n = 0; n <= kW; ++n) xw[n] = x8n_modp((uint64_t)n);
  build_gshift(gsh.data());
  build_swtab(swt.data());
  if (hipMalloc(&c->d_tab, tab.size() * 4) != hipSuccess || hipMalloc(&c->d_xw, xw.size() * 4) != hipSuccess ||
      hipMalloc(&c->d_gsh, gsh.size() * 4) != hipSuccess || hipMalloc(&c->d_swt, swt.size() * 4) != hipSuccess) {
    ldb_ctx_destroy(c);
    return LDB_ERR_NOMEM;
  }
  if (hipMemcpy(c->d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_xw, xw.data(), xw.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_gsh, gsh.data(), gsh.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_swt, swt.data(), swt.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    ldb_ctx_destroy(c);
    return LDB_ERR_HIP;
  }
  if (hipMalloc(&c->d_tacc, 8 * 16) != hipSuccess || hipMemset(c->d_tacc, 0, 8 * 16) != hipSuccess) {
    ldb_ctx_destroy(c);
    return LDB_ERR_NOMEM;
  }
  *out = c;
  return LDB_OK;
}

int ldb_ctx_destroy(ldb_ctx* c) {
  if (!c) return LDB_ERR_ARG;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();   // no launch of this context may outlive its buffers
  if (c->d_tab) (void)hipFree(c->d_tab);
  if (c->d_xw) (void)hipFree(c->d_xw);
  if (c->d_gsh) (void)hipFree(c->d_gsh);
  if (c->d_swt) (void)hipFree(c->d_swt);
  if (c->d_tacc) (void)hipFree(c->d_tacc);
  if (c->ws) (void)hipFree(c->ws);
  if (c->h_img) (void)hipFree(c->h_img);
  if (c->h_out) (void)hipFree(c->h_out);
  if (c->h_res) (void)hipFree(c->h_res);
  if (c->h_stream) (void)hipStreamDestroy(c->h_stream);
  if (c->h_pipes) (void)hipHostFree(c->h_pipes);
  if (c->pipes_ev) (void)hipEventDestroy(c->pipes_ev);
  for (int i = 0; i < c->n_cp; ++i)
    if (c->cp[i]) (void)hipStreamDestroy(c->cp[i]);
  for (hipEvent_t e : c->chunk_ev) (void)hipEventDestroy(e);
  if (c->merge) ldb_merge_release_(c->merge);
  if (c->ws_ev) (void)hipEventDestroy(c->ws_ev);
  for (const ldb_ctx::EvTriple& t : c->evs) {
    (void)hipEventDestroy(t.e0);
    (void)hipEventDestroy(t.eu);
    (void)hipEventDestroy(t.es);
    (void)hipEventDestroy(t.e2);
  }
  delete c;
  return LDB_OK;
}

int ldb_ctx_reserve(ldb_ctx* c, uint64_t max_len) {
  if (!c) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  return ensure_ws(c, layout(max_len).total);
}

int ldb_scan_file_dev(ldb_ctx* c, const uint8_t* d_image, uint64_t len, uint32_t fid, int io_type, int tuple_kind,
                      void* d_out, uint64_t cap, ldb_scan_result* d_result, void* stream) {
  if (!c) return LDB_ERR_ARG;
  c->ret_valid = false;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  return enqueue_scan(c, d_image, len, fid, io_type, tuple_kind, d_out, cap, d_result, (hipStream_t)stream, false);
}

int ldb_scan_file_dev_serial(ldb_ctx* c, const uint8_t* d_image, uint64_t len, uint32_t fid, int io_type,
                             int tuple_kind, void* d_out, uint64_t cap, ldb_scan_result* d_result, void* stream) {
  if (!c) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  return enqueue_scan(c, d_image, len, fid, io_type, tuple_kind, d_out, cap, d_result, (hipStream_t)stream, true);
}

int ldb_scan_files_dev(ldb_ctx* c, int n_files, const uint8_t* const* d_images, const uint64_t* lens,
                       const uint32_t* fids, int io_type, int tuple_kind, void* const* d_outs, const uint64_t* caps,
                       ldb_scan_result* d_results, void* stream) {
  if (!c || n_files < 0 || (n_files && (!d_images || !lens || !fids || !d_outs || !caps || !d_results)))
    return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  bool batch = batch_enabled() && n_files > 1;
  for (int i = 0; batch && i < n_files; ++i) batch = batch_eligible(d_images[i], lens[i]);
  if (batch) {
    std::vector<BatchFile> bf(n_files);
    for (int i = 0; i < n_files; ++i)
      bf[i] = BatchFile{d_images[i], lens[i], fids[i], d_outs[i], caps[i], d_results + i, nullptr};
    return enqueue_scan_batch(c, n_files, bf.data(), io_type, tuple_kind, (hipStream_t)stream);
  }
  uint64_t mx = 0;
  for (int i = 0; i < n_files; ++i) mx = std::max(mx, lens[i]);
  int rc = ensure_ws(c, layout(mx).total);
  if (rc != LDB_OK) return rc;
  for (int i = 0; i < n_files; ++i) {
    rc = enqueue_scan(c, d_images[i], lens[i], fids[i], io_type, tuple_kind, d_outs[i], caps[i], d_results + i,
                      (hipStream_t)stream, false);
    if (rc != LDB_OK) return rc;
  }
  return LDB_OK;
}

int ldb_host_register(ldb_ctx* c, const void* h_ptr, uint64_t len) {
  if (!c || !h_ptr || !len) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  if (hipHostRegister(const_cast<void*>(h_ptr), len, hipHostRegisterDefault) != hipSuccess) return LDB_ERR_HIP;
  c->regs.emplace_back((uintptr_t)h_ptr, len);
  return LDB_OK;
}

int ldb_host_unregister(ldb_ctx* c, const void* h_ptr) {
  if (!c || !h_ptr) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  if (hipHostUnregister(const_cast<void*>(h_ptr)) != hipSuccess) return LDB_ERR_HIP;
  for (size_t i = 0; i < c->regs.size(); ++i)
    if (c->regs[i].first == (uintptr_t)h_ptr) {
      c->regs.erase(c->regs.begin() + (long)i);
      break;
    }
  return LDB_OK;
}

// ldb_scan_file's body; retain: the count half of ldb_scan_file_count / ldb_scan_copy_out (no h_out: the
// tuples stay in the context's device staging for the copy-out, cap tuples of it)
static int scan_file_impl(ldb_ctx* c, const uint8_t* h_image, uint64_t len, uint32_t fid, int io_type, int tuple_kind,
                          void* h_out, uint64_t cap, ldb_scan_result* h_result, bool retain) {
  if (!c || !h_result || (len && !h_image) || (cap && !h_out && !retain)) return LDB_ERR_ARG;
  c->ret_valid = false;
  if (tuple_kind != LDB_TUPLE_INDEX && tuple_kind != LDB_TUPLE_ENTRY) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  const size_t tsz = tuple_kind == LDB_TUPLE_ENTRY ? sizeof(ldb_entry) : sizeof(ldb_index_tuple);
  // context-owned staging (grow-only): image, tuples, result; one stream per context
  if (!c->h_stream && hipStreamCreateWithFlags(&c->h_stream, hipStreamNonBlocking) != hipSuccess) return LDB_ERR_HIP;
  // An image this context page-locked (ldb_host_register) for all len bytes is scanned in place, below
  // (opt-in, LDB_DIRECT_IMAGE=1: measured slower than the staged copy, 23.7 vs 21.0 ms at config 2 --
  // the CUs' PCIe reads reach 52 GB/s against the DMA engines' 57.6). Memory pinned any other way
  // (hipHostMalloc, torch pin_memory, another context's registration) is staged like pageable memory.
  if (cap > UINT64_MAX / tsz) return LDB_ERR_ARG;
  void* mapped = nullptr;
  if (len && ldb_knob("LDB_DIRECT_IMAGE") != nullptr && c->registered(h_image, len) &&
      (hipHostGetDevicePointer(&mapped, const_cast<uint8_t*>(h_image), 0) != hipSuccess || ((uintptr_t)mapped & 15))) {
    mapped = nullptr;   // pageable (the error is expected) or not 16-B aligned: the staged copy
    (void)hipGetLastError();
  }
  // a page-locked output array is written in place too (the tuple writes cross PCIe while the scan
  // runs, in the other direction), else the tuples are staged on the device and copied back. Only a
  // range this context registered for all cap tuples qualifies: a shorter registration would let the
  // kernels write past the mapping
  void* out_mapped = nullptr;
  if (cap && ldb_knob("LDB_NO_DIRECT_OUT") == nullptr && c->registered(h_out, cap * tsz) &&
      hipHostGetDevicePointer(&out_mapped, h_out, 0) != hipSuccess) {
    out_mapped = nullptr;
    (void)hipGetLastError();
  }
  const uint64_t img_need = mapped ? 0 : (len + 15) & ~15ull, out_need = out_mapped ? 0 : cap * tsz;
  if ((img_need > c->h_img_cap || out_need > c->h_out_cap) && (c->h_img || c->h_out))
    (void)hipDeviceSynchronize();   // staging buffers are freed below: nothing may still use them
  if (img_need > c->h_img_cap || (!c->h_img && !mapped)) {
    if (c->h_img) (void)hipFree(c->h_img);
    c->h_img = nullptr;
    c->h_img_cap = 0;
    if (hipMalloc(&c->h_img, img_need ? img_need : 16) != hipSuccess) return LDB_ERR_NOMEM;
    c->h_img_cap = img_need;
  }
  if (out_need > c->h_out_cap || (!c->h_out && !out_mapped)) {
    if (c->h_out) (void)hipFree(c->h_out);
    c->h_out = nullptr;
    c->h_out_cap = 0;
    if (hipMalloc(&c->h_out, out_need ? out_need : 16) != hipSuccess) return LDB_ERR_NOMEM;
    c->h_out_cap = out_need;
  }
  if (!c->h_res && hipMalloc(&c->h_res, sizeof(ldb_scan_result)) != hipSuccess) return LDB_ERR_NOMEM;
  hipStream_t s = c->h_stream;
  if (!c->n_cp) {
    const char* e = ldb_knob("LDB_H2D_STREAMS");
    const int want = std::min(std::max(e ? atoi(e) : 2, 1), (int)ldb_ctx::kMaxCp);
    for (int i = 0; i < want; ++i) {
      if (hipStreamCreateWithFlags(&c->cp[i], hipStreamNonBlocking) != hipSuccess)
        return LDB_ERR_HIP;
      c->n_cp = i + 1;
    }
  }
  // The image goes up in 64 MiB chunks dealt over the copy streams (SDMA; at PCIe rate from a
  // page-locked mapping), and the run prefix verifies each chunk's entries as soon as it lands, so
  // the decode overlaps the transfer; the region pipeline runs after the last
  // chunk. Opt-in alternative: the image scanned in place through its device mapping (run prefix
  // skipped, enqueue_scan no_run). Every stream is drained before the call returns, so no copy or
  // read outlives the caller's buffer (a Go slice or an mmap'd file).
  int rc = LDB_OK;
  if (mapped) {
    rc = enqueue_scan(c, static_cast<const uint8_t*>(mapped), len, fid, io_type, tuple_kind,
                      out_mapped ? out_mapped : c->h_out, cap, c->h_res, s, false, true);
    if (rc != LDB_OK) {
      (void)hipStreamSynchronize(s);
      return rc;
    }
  }
  constexpr uint64_t kChunk = 64ull << 20;
  const int nch = mapped ? 0 : (int)((len + kChunk - 1) / kChunk);
  while ((int)c->chunk_ev.size() < nch && rc == LDB_OK) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = LDB_ERR_HIP;
    else c->chunk_ev.push_back(e);
  }
  std::vector<uint64_t> avail(nch);
  for (int i = 0; i < nch && rc == LDB_OK; ++i) {
    const uint64_t off = (uint64_t)i * kChunk, nb = std::min(kChunk, len - off);
    hipStream_t cs = c->cp[i % c->n_cp];
    // chunk i lands after chunk i - n_cp on the same copy stream: the prefix [0, off + nb) is in
    // place once every stream's latest chunk up to i has landed, which the scan stream's waits on
    // ev[0..i] in order give
    if (hipMemcpyAsync(c->h_img + off, h_image + off, nb, hipMemcpyHostToDevice, cs) != hipSuccess ||
        hipEventRecord(c->chunk_ev[i], cs) != hipSuccess)
      rc = LDB_ERR_HIP;
    avail[i] = off + nb;
  }
  if (rc == LDB_OK && !mapped) {
    const ChunkPlan plan{nch, avail.data(), c->chunk_ev.data()};
    rc = enqueue_scan(c, c->h_img, len, fid, io_type, tuple_kind, out_mapped ? out_mapped : c->h_out, cap, c->h_res, s,
                      false, false, &plan);
  }
  for (int j = 0; j < c->n_cp; ++j) (void)hipStreamSynchronize(c->cp[j]);
  if (rc != LDB_OK) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  ldb_scan_result res;
  if (hipMemcpyAsync(&res, c->h_res, sizeof(res), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LDB_ERR_HIP;
  const uint64_t n = out_mapped ? 0 : std::min<uint64_t>(res.n_entries, cap);
  if (retain) {   // the tuples stay on the device for ldb_scan_copy_out
    c->ret_valid = true;
    c->ret_n = n;
    c->ret_tsz = tsz;
    *h_result = res;
    return LDB_OK;
  }
  if (n && (hipMemcpyAsync(h_out, c->h_out, n * tsz, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess))
    return LDB_ERR_HIP;
  *h_result = res;
  return LDB_OK;
}

int ldb_scan_file(ldb_ctx* c, const uint8_t* h_image, uint64_t len, uint32_t fid, int io_type, int tuple_kind,
                  void* h_out, uint64_t cap, ldb_scan_result* h_result) {
  return scan_file_impl(c, h_image, len, fid, io_type, tuple_kind, h_out, cap, h_result, false);
}

// Count, then copy: the image goes up once and is scanned with no room for tuples (the kernels count the
// entries whatever the capacity); when there are any, the staged device image is scanned again into a
// device array of exactly n_entries tuples (a few ms of kernels against the copy's ~20 ms per GiB), which
// ldb_scan_copy_out then moves into the caller's array sized n. Device staging: the image plus n tuples
// (round 5 staged len / 10 + 1 tuples first: 4.8x the image for the 48-B ldb_entry kind).
int ldb_scan_file_count(ldb_ctx* c, const uint8_t* h_image, uint64_t len, uint32_t fid, int io_type, int tuple_kind,
                        ldb_scan_result* h_result) {
  int rc = scan_file_impl(c, h_image, len, fid, io_type, tuple_kind, nullptr, 0, h_result, true);
  if (rc != LDB_OK || h_result->status != LDB_ERR_CAPACITY) return rc;
  if (c->h_img_cap < len)   // (the opt-in in-place image, LDB_DIRECT_IMAGE: nothing staged, scan it again)
    return scan_file_impl(c, h_image, len, fid, io_type, tuple_kind, nullptr, h_result->n_entries, h_result, true);
  // the second pass over the image already in HBM (c->h_img), exactly n tuples
  const uint64_t n = h_result->n_entries, tsz = c->ret_tsz;
  c->ret_valid = false;
  if (n > UINT64_MAX / tsz) return LDB_ERR_ARG;
  if (n * tsz > c->h_out_cap) {
    (void)hipStreamSynchronize(c->h_stream);
    if (c->h_out) (void)hipFree(c->h_out);
    c->h_out = nullptr;
    c->h_out_cap = 0;
    if (hipMalloc(&c->h_out, n * tsz) != hipSuccess) return LDB_ERR_NOMEM;
    c->h_out_cap = n * tsz;
  }
  hipStream_t s = c->h_stream;
  rc = enqueue_scan(c, c->h_img, len, fid, io_type, tuple_kind, c->h_out, n, c->h_res, s, false);
  if (rc != LDB_OK) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  ldb_scan_result res;
  if (hipMemcpyAsync(&res, c->h_res, sizeof(res), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return LDB_ERR_HIP;
  c->ret_valid = true;
  c->ret_n = std::min<uint64_t>(res.n_entries, n);
  *h_result = res;
  return LDB_OK;
}

int ldb_scan_copy_out(ldb_ctx* c, void* h_out, uint64_t cap, uint64_t* n_copied) {
  if (!c || !c->ret_valid || (cap && !h_out) || !n_copied) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  const uint64_t n = std::min<uint64_t>(c->ret_n, cap);
  if (n && (hipMemcpyAsync(h_out, c->h_out, n * c->ret_tsz, hipMemcpyDeviceToHost, c->h_stream) != hipSuccess ||
            hipStreamSynchronize(c->h_stream) != hipSuccess))
    return LDB_ERR_HIP;
  *n_copied = n;
  return LDB_OK;
}

#ifdef LDB_SW_TRACE
int ldb_debug_swtrace(uint64_t* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_swtrace), sizeof(g_swtrace)) != hipSuccess) return LDB_ERR_HIP;
  if (reset) {
    static uint64_t z[kSwTraceWgs * 4];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_swtrace), z, sizeof(z)) != hipSuccess) return LDB_ERR_HIP;
  }
  return LDB_OK;
}
#endif
#ifdef LDB_STAMPS
int ldb_debug_stamps(uint64_t* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), 8 * kStampSlots) != hipSuccess) return LDB_ERR_HIP;
  if (reset) {
    uint64_t z[kStampSlots] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, 8 * kStampSlots) != hipSuccess) return LDB_ERR_HIP;
  }
  return LDB_OK;
}
int ldb_debug_swstamps(uint64_t* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_swstamps), 8 * 16) != hipSuccess) return LDB_ERR_HIP;
  if (reset) {
    uint64_t z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_swstamps), z, 8 * 16) != hipSuccess) return LDB_ERR_HIP;
  }
  return LDB_OK;
}
int ldb_debug_ustamps(uint64_t* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ustamps), 8 * kUniStampSlots) != hipSuccess) return LDB_ERR_HIP;
  if (reset) {
    uint64_t z[kUniStampSlots] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_ustamps), z, 8 * kUniStampSlots) != hipSuccess) return LDB_ERR_HIP;
  }
  return LDB_OK;
}
#endif

// Diagnostics (not in the C ABI header): the sweep tier's run records and control block of the last scan of
// length len on this context, after it completed (tools/sweep_debug.py).
extern "C" int ldb_debug_sweep_state(ldb_ctx* c, uint64_t len, void* h_runs, uint64_t max_runs, void* h_ctl) {
  if (!c || !h_runs || !h_ctl) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  const WsLayout L = layout(len);
  if (L.total > c->ws_bytes) return LDB_ERR_ARG;
  const uint64_t n = max_runs < (uint64_t)kSwMaxRuns ? max_runs : (uint64_t)kSwMaxRuns;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h_runs, c->ws + L.o_swrun, n * sizeof(SwRun), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(h_ctl, c->ws + L.o_swctl, sizeof(SwCtl), hipMemcpyDeviceToHost) != hipSuccess)
    return LDB_ERR_HIP;
  return LDB_OK;
}

int ldb_read_ceiling(ldb_ctx* c, const uint8_t* d_image, uint64_t len, int iters, double* gbps) {
  if (!c || !gbps || (len && !d_image) || iters < 1 || (uintptr_t)d_image % 16) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  *gbps = 0.0;
  const uint64_t n16 = len / 16;
  if (!n16) return LDB_OK;
  hipStream_t s;
  hipEvent_t a, b;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return LDB_ERR_HIP;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  uint32_t* d_sink = nullptr;
  const unsigned grid = (unsigned)c->n_cu * 16;
  int rc = hipMalloc(&d_sink, grid * sizeof(uint32_t)) == hipSuccess ? LDB_OK : LDB_ERR_HIP;
  if (rc == LDB_OK) {
    hipLaunchKernelGGL(k_read_reduce, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(d_image), n16, d_sink);
    (void)hipEventRecord(a, s);
    for (int i = 0; i < iters; ++i)
      hipLaunchKernelGGL(k_read_reduce, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(d_image), n16, d_sink);
    (void)hipEventRecord(b, s);
    float ms = 0.f;
    if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess || ms <= 0.f) rc = LDB_ERR_HIP;
    else *gbps = (double)(n16 * 16) / ((double)ms / iters * 1e-3) / 1e9;
  }
  if (d_sink) (void)hipFree(d_sink);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipStreamDestroy(s);
  return rc;
}

int ldb_kernel_timing(ldb_ctx* c, int enable, double* avg_main_ms, double* avg_total_ms, uint64_t* n) {
  if (!c) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  const int rc = resolve_timing(c);
  if (rc != LDB_OK) return rc;
  if (avg_main_ms) *avg_main_ms = c->t_n ? c->t_main / c->t_n : 0.0;
  if (avg_total_ms) *avg_total_ms = c->t_n ? c->t_total / c->t_n : 0.0;
  if (n) *n = c->t_n;
  if (enable >= 0) {
    c->timing = enable != 0;
    c->t_run = c->t_sweep = c->t_main = c->t_total = 0;
    for (double& x : c->t_ph) x = 0;
    c->t_n = 0;
  }
  return LDB_OK;
}

int ldb_kernel_timing_split(ldb_ctx* c, int enable, double* avg_run_ms, double* avg_main_ms, double* avg_total_ms,
                            uint64_t* n) {
  if (!c) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  const int rc = resolve_timing(c);
  if (rc != LDB_OK) return rc;
  if (avg_run_ms) *avg_run_ms = c->t_n ? c->t_run / c->t_n : 0.0;
  return ldb_kernel_timing(c, enable, avg_main_ms, avg_total_ms, n);
}

int ldb_kernel_timing_tail(ldb_ctx* c, double* avg_phase_ms, int n_phases) {
  if (!c || !avg_phase_ms || n_phases < 0) return LDB_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return LDB_ERR_HIP;
  const int rc = resolve_timing(c);
  if (rc != LDB_OK) return rc;
  for (int k = 0; k < n_phases; ++k) avg_phase_ms[k] = k < 16 && c->t_n ? c->t_ph[k] / c->t_n : 0.0;
  return LDB_OK;
}

int ldb_kernel_timing_sweep(ldb_ctx* c, double* avg_sweep_ms, double* avg_fin_ms) {
  if (!c || !avg_sweep_ms || !avg_fin_ms) return LDB_ERR_ARG;
  double ph[2];
  const int rc = ldb_kernel_timing_tail(c, ph, 2);
  *avg_sweep_ms = c->t_n ? c->t_sweep / c->t_n : 0.0;
  *avg_fin_ms = ph[1];
  return rc;
}

}  // extern "C"
