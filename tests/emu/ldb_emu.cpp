// ldb_emu.cpp — CPU emulation of the gfx950 scan pipeline (TEST HARNESS ONLY).
//
// Runs the engine's own phase functions (lazydb_amd/csrc/ldb_engine.h, ldb_wave.h,
// ldb_pipeline.h) with a sequential 64-lane "wave policy", region after region, then the
// link / repair / combine / final / compact stages exactly as the kernels in ldb_scan.hip
// order them. It exists so the algorithm can be checked against the oracle in this
// GPU-less container; it is not linked into liblazydb_gpu.so and is not a fallback.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>
#include <cstdio>
#include <cstdlib>

#include "../../lazydb_amd/csrc/ldb_pipeline.h"

using namespace ldb;

#ifdef LDB_EMU_COUNTERS
namespace ldb { int g_emu_lane; uint32_t g_emu_cnt[8][64]; uint64_t g_chain_why[16]; }
extern "C" void emu_chain_why(uint64_t* out) { for (int i = 0; i < 16; ++i) { out[i] = ldb::g_chain_why[i]; ldb::g_chain_why[i] = 0; } }
static uint64_t g_sum[8], g_max[8], g_regions;
extern "C" void emu_counters(uint64_t* out) {   // [0..7] sums over lanes, [8..15] sums of per-region lane maxima, [16] regions
  for (int i = 0; i < 8; ++i) { out[i] = g_sum[i]; out[8 + i] = g_max[i]; g_sum[i] = g_max[i] = 0; }
  out[16] = g_regions; g_regions = 0;
}
static void fold_counters() {
  for (int i = 0; i < 8; ++i) {
    uint32_t mx = 0;
    for (int l = 0; l < 64; ++l) {
      const uint32_t c = ldb::g_emu_cnt[i][l];
      g_sum[i] += c; mx = c > mx ? c : mx; ldb::g_emu_cnt[i][l] = 0;
    }
    g_max[i] += mx;
  }
  ++g_regions;
}
#define EMU_SET_LANE(l) (ldb::g_emu_lane = (l))
#define EMU_FOLD() fold_counters()
#else
#define EMU_SET_LANE(l) ((void)0)
#define EMU_FOLD() ((void)0)
#endif

namespace {

struct CpuWave {
  template <class F> void each(F f) { for (int l = 0; l < kLanes; ++l) { EMU_SET_LANE(l); f(l); } }
  template <class P> uint64_t ballot(P p) {
    uint64_t b = 0;
    for (int l = 0; l < kLanes; ++l)
      if (p(l)) b |= 1ull << l;
    return b;
  }
  template <class P> int first(P p) {
    for (int l = 0; l < kLanes; ++l)
      if (p(l)) return l;
    return -1;
  }
  template <class P> int last(P p) {
    for (int l = kLanes - 1; l >= 0; --l)
      if (p(l)) return l;
    return -1;
  }
  template <class V> uint32_t sum(V v) {
    uint32_t s = 0;
    for (int l = 0; l < kLanes; ++l) s += v(l);
    return s;
  }
  template <class V, class O> void excl_prefix(V v, O out) {
    uint32_t s = 0;
    for (int l = 0; l < kLanes; ++l) { const uint32_t x = v(l); out(l, s); s += x; }
  }
  template <class F> uint32_t from(int src, F f) { return (uint32_t)f(src); }
  template <class F> uint64_t from64(int src, F f) { return (uint64_t)f(src); }
  template <class F> void single(F f) { f(); }
  // put(l, value of lane l - d, l >= d) for every lane, all reads before any write
  template <int d, class G, class P> void shfl_up(G get, P put) {
    uint32_t t[kLanes];
    for (int l = 0; l < kLanes; ++l) t[l] = get(l);
    for (int l = 0; l < kLanes; ++l) { EMU_SET_LANE(l); put(l, l >= d ? t[l - d] : 0u, l >= d); }
  }
  void stamp(int) {}
};

struct Emu {
  std::vector<uint32_t> tab, xw, gsh;
  std::vector<uint8_t> buf;
  WaveSh sh;
  uint64_t garbage = 0x1234567;
  Emu() : tab(kTabWords), xw(kW + 1), gsh(kGsWords), buf(kBuf) {
    build_tables(tab.data());
    build_gshift(gsh.data());
    for (int n = 0; n <= kW; ++n) xw[n] = x8n_modp((uint64_t)n);
  }
  void stage(const Pipe& p, uint64_t r) {
    const uint64_t R0 = r * (uint64_t)kW;
    for (int i = 0; i < kBuf; ++i) {
      const int64_t a = (int64_t)R0 + i - kPre;
      garbage = garbage * 6364136223846793005ull + 1442695040888963407ull;
      buf[i] = (a >= 0 && (uint64_t)a < p.len) ? p.img[a] : (uint8_t)(garbage >> 56);
    }
  }
  View view(const Pipe& p, uint64_t r) {
    View v;
    v.buf = buf.data();
    v.tab = tab.data();
    v.xw = xw.data();
    v.gsh = gsh.data();
    v.R0 = r * (uint64_t)kW;
    v.rlen = region_len(p, r);
    v.len = p.len;
    v.io = p.io;
    return v;
  }
  // one region of a wavefront's run (k_scan_main): the lean path (false: the caller runs region_process)
  bool run_chained(const Pipe& p, uint64_t r, ChainState& st) {
    stage(p, r);
    const View v = view(p, r);
    CpuWave wp;
    ldb_index_tuple* sc = p.scratch + r * (uint64_t)kRegionCap;
    ChainPriv cpriv[kLanes];
    if (!st.on && zero_region(wp, v)) {   // as k_scan_main
      store_region(p, r, zero_summary());
      EMU_FOLD();
      return true;
    }
    bool released = false;
    const bool fast = region_chained(
        wp, v, buf.data(), sh, st, [&](int l) -> ChainPriv& { return cpriv[l]; },
        [&](bool valid, uint32_t slot, uint64_t pos, uint32_t k, uint32_t vv) {
          if (!valid) return;
          sc[slot].pos = pos;
          sc[slot].k_size = k;
          sc[slot].v_size = vv;
        },
        [&] { released = true; }, [] {}, [&](const RegionSum& rs) { store_region(p, r, rs); });
    (void)released;   // a decline leaves st untouched: the caller runs region_process from it (k_scan_main)
    EMU_FOLD();
    return fast;
  }
  RegionSum run(const Pipe& p, uint64_t r, uint32_t enter) {
    stage(p, r);
    View v;
    v.buf = buf.data();
    v.tab = tab.data();
    v.xw = xw.data();
    v.gsh = gsh.data();
    v.R0 = r * (uint64_t)kW;
    v.rlen = region_len(p, r);
    v.len = p.len;
    v.io = p.io;
    RegionSum s;
    CpuWave wp;
    ldb_index_tuple* sc = p.scratch + r * (uint64_t)kRegionCap;
    LanePriv priv[kLanes];
    region_process(wp, v, sh, enter, &s, [&](int l) -> LanePriv& { return priv[l]; }, [&](uint32_t slot, uint64_t pos, uint32_t k, uint32_t vv) {
      sc[slot].pos = pos;
      sc[slot].k_size = k;
      sc[slot].v_size = vv;
    }, [] {});
    store_region(p, r, s);
    EMU_FOLD();
    return s;
  }
};

struct Rd {
  const Pipe* p;
  uint64_t start(uint64_t r) const { return p->rs[r].start; }
  uint64_t exitp(uint64_t r) const { return p->rs[r].exitp; }
  uint32_t sflag(uint64_t r) const { return p->rs[r].sflag; }
};

}  // namespace

// k_uniform on the CPU: the same template and header checks (ldb_pipeline.h), byte-wise CRC-32.
// Writes the run's tuples and dyn = {K, size}.
// k_uniform: the same verdicts, CRC-32 by the kernel's entry-aligned slices (uni_geometry): lane j's
// window from register 0 with its masked lead, then the group's tree combine with byte-table shifts,
// then raw ^ KL against ~crc. Bytes of the image's last partial dword are real (the kernel's buffer
// range is len rounded up to a dword); bytes past len read as zero and are never used by a member.
static void emu_uniform(const Emu& emu, const uint8_t* img, uint64_t len, int io, ldb_index_tuple* out, uint64_t cap,
                        uint64_t* dyn) {
  struct F {
    const uint8_t* q;
    uint64_t len;
    uint32_t operator()(int i) const { return (uint64_t)i < len ? q[i] : 0u; }
  };
  const UniMemo m = uni_memo(F{img, len}, len, io);
  dyn[0] = 0;
  dyn[1] = 0;
  if (!m.ok) return;
  const UniGeo g = uni_geometry(emu.xw.data(), (uint32_t)(m.sz - 4));
  if (!g.ok) return;
  dyn[1] = m.sz;
  std::vector<uint32_t> ct((size_t)g.lg * 1024);   // k_uniform_setup's combine tables
  for (uint32_t i = 0; i < g.lg; ++i) {
    const uint32_t xn = x8n_modp((uint64_t)g.P << i);
    for (uint32_t e = 0; e < 1024; ++e) ct[i * 1024 + e] = multmodp(xn, (e & 255u) << (8 * (e >> 8)));
  }
  auto byte = [&](int64_t a) -> uint32_t { return a >= 0 && (uint64_t)a < len ? img[a] : 0u; };
  {   // k_uniform_setup: no run unless entry 1 has the memo's header too
    auto word1 = [&](int i) -> uint32_t {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b) w |= byte((int64_t)(m.sz + 4 * (uint64_t)i + b)) << (8 * b);
      return w;
    };
    if (!uni_header_ok(m, word1, m.sz, len, io)) return;
  }
  const uint64_t ncand = len / m.sz + 1;
  uint64_t k = 0;
  std::vector<uint32_t> v(g.G);
  for (; k < ncand; ++k) {
    const uint64_t x = k * m.sz;
    auto word = [&](int i) -> uint32_t {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b) w |= byte((int64_t)(x + 4 * (uint64_t)i + b)) << (8 * b);
      return w;
    };
    if (!uni_header_ok(m, word, x, len, io)) break;
    for (uint32_t j = 0; j < g.G; ++j) {
      const int64_t ws = (int64_t)x + 4 - (int64_t)g.t + (int64_t)j * g.P;
      const uint32_t lead = uni_lead(g, j);
      uint32_t reg = 0;
      for (uint32_t s = 0; s < g.S; ++s) {
        uint32_t w[2] = {0, 0};
        for (int b = 0; b < 8; ++b)
          if (8 * s + b >= lead) w[b >> 2] |= byte(ws + 8 * s + b) << (8 * (b & 3));
        reg = crc_step8(emu.tab.data(), reg, w[0], w[1]);
      }
      v[j] = reg;
    }
    for (uint32_t i = 0, d = 1; d < g.G; ++i, d <<= 1)
      for (uint32_t j = 0; j < g.G; ++j)
        if ((j & (2 * d - 1)) == 2 * d - 1) {
          const uint32_t y = v[j - d], *T = ct.data() + i * 1024;
          v[j] ^= T[y & 0xFFu] ^ T[256 + ((y >> 8) & 0xFFu)] ^ T[512 + ((y >> 16) & 0xFFu)] ^ T[768 + (y >> 24)];
        }
    if ((v[g.G - 1] ^ g.KL) != ~word(0)) break;
    if (k < cap) { out[k].pos = uni_pos(m, x); out[k].k_size = m.k; out[k].v_size = m.v; }
  }
  dyn[0] = k;
}

#ifdef LDB_EMU_SWEEP
int emu_sweep_phase(Pipe& p, uint32_t vg, uint32_t vgf);   // tests/emu/sweep_emu.cpp
#endif

// run_len: regions per wavefront run (k_scan_main gives each wave a contiguous run); 0 = every
// region speculative (the pre-chain pipeline). use_run: the run prefix (k_uniform) first. sweep_vg > 0
// (libldb_emu_sweep.so): the sweep tier after the run prefix (k_sweep of sweep_vg workgroups, phase F of
// at most sweep_vgf items), as the GPU pipeline orders it; the region pipeline continues where it ends.
static int scan_impl(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                     ldb_scan_result* res, uint32_t* stats, uint64_t run_len, int use_run, uint32_t sweep_vg,
                     uint32_t sweep_vgf) {
  Emu emu;
  const uint64_t nreg = std::max<uint64_t>(1, (len + kW - 1) / kW);
  const uint64_t nblk = (nreg + kBlkRegions - 1) / kBlkRegions;
  std::vector<uint64_t> blk(nblk, 0), tpos(2, ~0ull), dyn(8, 0);
  dyn[5] = ~0ull;   // x0 = K sz (one run; the GPU's uni_finish writes x0 over several runs)
  std::vector<RegionSum> rs(nreg);
  std::vector<uint32_t> ctr(8, 0);
  std::vector<ldb_index_tuple> scratch(nreg * (uint64_t)kRegionCap);
  std::vector<int64_t> fail(nreg + 9);   // fail flags + walker claims (8 (nreg + 1) + 64 B, as the GPU)
  Pipe p;
  p.img = img; p.len = len; p.io = io; p.fid = fid; p.nreg = nreg;
  p.gtab = emu.tab.data(); p.xw = emu.xw.data(); p.gsh = emu.gsh.data();
  p.rs = rs.data();
  p.scratch = scratch.data(); p.fail_src = fail.data(); p.ctr = ctr.data(); p.tpos = tpos.data();
  p.blk = blk.data(); p.out = out; p.cap = cap; p.kind = LDB_TUPLE_INDEX; p.result = res; p.dyn = dyn.data();
  res->n_run = 0;
  res->n_sweep = 0;
  if (len < (uint64_t)kMaxHeader) {
    // the kernels route tiny images to k_serial; mirror it
    res->status = LDB_EOF_WINDOW; res->fid = fid; res->n_entries = 0; res->end_off = 0; res->n_repairs = 0;
    res->n_regions = (uint32_t)nreg;
    return 0;
  }
  if (use_run) emu_uniform(emu, img, len, io, out, cap, dyn.data());
  // the sweep tier's buffers, sized as the GPU workspace (WsLayout), and the image with a garbage tail (the
  // GPU's staging buffer holds whatever lies past len; no result may depend on it)
  (void)sweep_vg;
  (void)sweep_vgf;
#ifdef LDB_EMU_SWEEP
  std::vector<uint8_t> padded;
  std::vector<uint32_t> swrw, swrg, swpl, swt;
  std::vector<SwRun> swrun;
  SwCtl swctl{};
  if (sweep_vg && first_region(p) < nreg) {
    padded.resize(len + 65536);
    std::copy(img, img + len, padded.begin());
    uint64_t g = 0x9E3779B97F4A7C15ull ^ len;
    for (size_t i = len; i < padded.size(); ++i) {
      g = g * 6364136223846793005ull + 1442695040888963407ull;
      padded[i] = (uint8_t)(g >> 56);
    }
    p.img = padded.data();
    swrw.assign((len + kSwBatch) / kSwW + 1, 0u);
    swrg.assign((len + kSwBatch) / (kSwW * kSwG) + 1, 0u);
    swpl.assign((len + kSwBatch) / 64 + 1, 0u);
    swrun.assign(kSwMaxRuns, SwRun{});
    swt.assign(kSwTabWords, 0u);
    build_swtab(swt.data());
    p.swrw = swrw.data();
    p.swrg = swrg.data();
    p.swpl = swpl.data();
    p.swrun = swrun.data();
    p.swctl = &swctl;
    p.swt = swt.data();
    p.scratch_bytes = sizeof(ldb_index_tuple) * scratch.size();
    p.tail = nullptr;
    p.tacc = nullptr;
    p.sweep = 1;
    const int rc = emu_sweep_phase(p, sweep_vg, sweep_vgf);
    if (rc < 0) return rc - 200;
    if (stats) stats[3] = (uint32_t)swctl.relinks;   // the links' extra passes (sw_link)
    if (rc == 1) {   // sw_finish wrote *p.result
      if (stats) { stats[0] = 0; stats[1] = 0; stats[2] = 0; }
      return 0;
    }
  }
#endif
  const uint64_t rf = first_region(p), K = run_k(p), x0 = chain_x0(p);
  res->n_run = K;
  res->n_sweep = 0;
  if (rf >= nreg) {   // k_compact: io.EOF right after the run
    res->status = K > cap ? LDB_ERR_CAPACITY : LDB_EOF_WINDOW; res->fid = fid; res->n_entries = K; res->end_off = x0;
    res->n_repairs = 0; res->n_regions = 0;
    if (stats) { stats[0] = 0; stats[1] = 0; stats[2] = 0; }
    return 0;
  }
  // k_scan_main
  uint32_t n_fast = 0;
  if (run_len == 0) {
    for (uint64_t r = rf; r < nreg; ++r) emu.run(p, r, kForceSpec);
  } else {
    for (uint64_t r0 = rf; r0 < nreg; r0 += run_len) {   // k_scan_main: one wave's run
      ChainState st;
      chain_reset(st);
      if (r0 == rf) { st.on = 2; st.x = x0; }   // as k_scan_main: the replay's entry point
      const uint64_t warm = r0 > rf ? std::min<uint64_t>(kWarm, r0 - rf) : 0;   // dry warm-up regions
      uint32_t declines = 0, backoff = 0;
      std::vector<RegionSum> keep;
      for (uint64_t r = r0 - warm; r < nreg && r < r0 + run_len; ++r) {
        const bool dry = r < r0;
        const bool spec_entry = !st.on;
        // as k_scan_main: the warm-up ended inside an entry that covers the run's whole first region
        if (r == r0 && warm && st.on && st.x >= r0 * (uint64_t)kW + kW) chain_reset(st);
        const RegionSum saved = rs[r];   // a dry region's summary and tuples belong to the previous run
        std::vector<ldb_index_tuple> saved_sc;
        if (dry) saved_sc.assign(scratch.begin() + r * (uint64_t)kRegionCap, scratch.begin() + (r + 1) * (uint64_t)kRegionCap);
        const uint32_t win = 8u << (backoff < 5 ? backoff : 5);   // give-up mode (as k_scan_main)
        const bool skip = declines >= 2 && declines < 2 + win;
        static const long dbg_r = getenv("LDB_EMU_DBG_R") ? atol(getenv("LDB_EMU_DBG_R")) : -1;
        if ((long)r == dbg_r || (long)r + 1 == dbg_r)
          fprintf(stderr, "region %llu dry=%d st.on=%u st.x=%llu declines=%u skip=%d\n", (unsigned long long)r, (int)dry,
                  st.on, (unsigned long long)st.x, declines, (int)skip);
        if (!skip && emu.run_chained(p, r, st)) {
          n_fast += dry ? 0u : 1u;
          declines = 0;
          backoff = 0;
        } else {
          // the general routine inline (run_region, ldb_chain.h)
          uint32_t enter = kForceSpec;
          if (st.on && st.x >= r * (uint64_t)kW)
            enter = st.x - r * (uint64_t)kW < (uint64_t)region_len(p, r) ? (uint32_t)(st.x - r * (uint64_t)kW) : kForceNone;
          const RegionSum o = emu.run(p, r, enter);
          chain_after_general(st, o, emu.view(p, r), enter);
          if (++declines >= 3 + win) {
            declines = 2;
            backoff += 1;
          }
        }
        if (spec_entry && st.on && st.x > r * (uint64_t)kW + kWarmSwallow) chain_reset(st);   // as k_scan_main
        if ((long)r == dbg_r)
          fprintf(stderr, "  -> start=%llu exit=%llu status=%d sflag=%u | st.on=%u st.x=%llu\n", (unsigned long long)rs[r].start,
                  (unsigned long long)rs[r].exitp, rs[r].status, rs[r].sflag, st.on, (unsigned long long)st.x);
        if (dry) {
          rs[r] = saved;
          std::copy(saved_sc.begin(), saved_sc.end(), scratch.begin() + r * (uint64_t)kRegionCap);
        }
      }
    }
  }
  // k_link: every flag of the pipeline (ldb_pipeline.h fail_flags), claims cleared
  uint8_t* fl = fail_flags(p);
  uint32_t* claims = repair_claims(p);
  const uint64_t nflag = n_fail_flags(p);
  auto relink = [&]() -> uint32_t {
    uint32_t nb = 0;
    for (uint64_t r = rf; r < nreg; ++r) {
      const bool bad = link_broken(p, r);
      if (bad && getenv("LDB_EMU_DEBUG")) {
        const uint64_t m = rs[r].exitp / kW;
        fprintf(stderr, "fail r=%llu start=%llu exit=%llu st=%d -> m=%llu rs[m].start=%llu (rel %lld) st[m]=%d\n",
                (unsigned long long)r, (unsigned long long)rs[r].start, (unsigned long long)rs[r].exitp, rs[r].status,
                (unsigned long long)m, (unsigned long long)rs[m].start, (long long)(rs[m].start - m * kW), rs[m].status);
      }
      fl[r - rf + 1] = bad ? 1 : 0;
      nb += bad ? 1u : 0u;
      if (r == rf) {
        fl[0] = rs[rf].start != x0 ? 1 : 0;
        nb += fl[0];
      }
    }
    return nb;
  };
  for (uint64_t r = rf; r < nreg; ++r) claims[r] = 0;
  const uint32_t nfail = relink();
  ctr[0] = nfail;
  // k_repair: the optimistic walkers (in flag order here; any order is correct), the links again,
  // then the serial repair from the fresh flags
  uint32_t walker_runs = 0, n2 = 0;
  auto run = [&](uint64_t r, uint32_t enter) { return emu.run(p, r, enter); };
  if (nfail) {
    // LDB_EMU_WALKERS: "0" none (the serial repair alone), "rev" in reverse flag order (each walker
    // reads its source before an earlier walker rewrites it: stale starting points, lost claims)
    const char* wm = getenv("LDB_EMU_WALKERS");
    // "win": windows of 64 flags in reverse order, each in flag order (GPU waves running windows
    // concurrently, the later one first)
    const bool walk = !(wm && wm[0] == '0'), rev = wm && wm[0] == 'r', win = wm && wm[0] == 'w';
    const uint64_t nwin = (nflag + 63) / 64;
    const std::vector<uint8_t> fl0(fl, fl + nflag);   // k_link's flags, as the walkers read them
    // as k_repair: hold covered re-runs of linked regions (bit 0); LDB_EMU_HOLD A/Bs the rules
    const int hold = getenv("LDB_EMU_HOLD") ? atoi(getenv("LDB_EMU_HOLD")) : 1;
    for (uint64_t j = 0; walk && j < nflag; ++j) {
      const uint64_t i = rev ? nflag - 1 - j : win ? (nwin - 1 - j / 64) * 64 + j % 64 : j;
      if (i >= nflag) continue;
      if (i % 64 == 0 && i > 0 && fl[i - 1]) continue;   // as k_repair: left to the previous window's walker
      if (fl[i])
        walker_runs += walk_source(p, (int64_t)rf - 1 + (int64_t)i, Rd{&p},
                                   [&](uint64_t r) { return claims[r]++ == 0; }, run,
                                   [&](uint64_t r) { return (hold & 1) && r > rf && fl0[r - rf] == 0; },
                                   [&](uint64_t r) { return (hold & 2) && r > rf && fl0[r - rf] == 0; });
    }
    n2 = relink();
  }
  if (n2) {
    auto next_fail = [&](int64_t done) -> int64_t {
      for (uint64_t i = (uint64_t)(done - ((int64_t)rf - 1) + 1); i < nflag; ++i)
        if (fl[i]) return (int64_t)rf - 1 + (int64_t)i;
      return INT64_MAX;
    };
    auto first_term = [&](int64_t lo, int64_t hi) -> int64_t {
      for (int64_t r = std::max<int64_t>(lo + 1, (int64_t)rf); r <= hi && (uint64_t)r < nreg; ++r)
        if (rs[r].status != kCont && rs[r].start != kNone64) return r;
      return -1;
    };
    ctr[2] = repair(p, next_fail, Rd{&p}, first_term, run);
  }
  ctr[2] += walker_runs;
  if (getenv("LDB_EMU_REPAIR_STATS"))
    fprintf(stderr, "repair: %u flagged, %u walker runs, %u flagged after, %u serial runs\n", nfail, walker_runs, n2,
            ctr[2] - walker_runs);
  // k_combine
  for (uint64_t r = rf; r < nreg; ++r) {
    const int32_t st = rs[r].status;
    if (st == kOverflow) { ctr[1] = 1; continue; }
    blk[r / kBlkRegions] += rs[r].count;
    if (rs[r].start == kNone64) continue;
    if (st != kCont) {
      tpos[0] = std::min(tpos[0], pack_term(rs[r].exitp, st));
    } else {
      if (rs[r].exitp >= len) tpos[0] = std::min(tpos[0], pack_term(len, LDB_EOF_WINDOW));
      if ((rs[r].sflag & kStraddle) && !combine_region(p, r)) tpos[0] = std::min(tpos[0], pack_term(rs[r].soff, LDB_ERR_CRC));
    }
  }
  if (ctr[1]) return -100;  // overflow: the GPU pipeline re-runs k_serial
  // k_final + k_compact
  const uint64_t T = tpos[0];
  if (T == ~0ull) return -101;
  const uint64_t tp = term_pos(T);
  const uint64_t regT = tp / kW;
  uint64_t n = K;
  for (uint64_t r = rf; r < nreg && r <= regT; ++r) {
    uint64_t c = rs[r].count;
    if (r == regT && rs[r].status == kCont && (rs[r].sflag & kStraddle) && rs[r].soff == tp && c > 0) c -= 1;
    for (uint64_t j = 0; j < c; ++j)
      if (n + j < cap) out[n + j] = scratch[r * (uint64_t)kRegionCap + j];
    n += c;
  }
  res->status = n > cap ? LDB_ERR_CAPACITY : term_status(T);
  res->fid = fid;
  res->n_entries = n;
  res->end_off = tp;
  res->n_repairs = ctr[2];
  res->n_regions = (uint32_t)(nreg - rf);
  res->n_sweep = sweep_vg ? dyn[7] : 0;
  if (stats) { stats[0] = nfail; stats[1] = ctr[2]; stats[2] = n_fast; }
  return 0;
}

extern "C" int emu_scan_ex(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                           ldb_scan_result* res, uint32_t* stats, uint64_t run_len, int use_run) {
  return scan_impl(img, len, io, fid, out, cap, res, stats, run_len, use_run, 0, 0);
}

#ifdef LDB_EMU_SWEEP
extern "C" int emu_scan_sweep(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                              ldb_scan_result* res, uint32_t* stats, uint64_t run_len, uint32_t sweep_vg,
                              uint32_t sweep_vgf) {
  return scan_impl(img, len, io, fid, out, cap, res, stats, run_len, 1, sweep_vg, sweep_vgf);
}
#endif

extern "C" int emu_scan_runs(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                             ldb_scan_result* res, uint32_t* stats, uint64_t run_len) {
  return emu_scan_ex(img, len, io, fid, out, cap, res, stats, run_len, 0);
}

extern "C" int emu_scan(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                        ldb_scan_result* res, uint32_t* stats) {
  return emu_scan_runs(img, len, io, fid, out, cap, res, stats, 0);
}
