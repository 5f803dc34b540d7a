// sweep_emu.cpp — the sweep tier's kernel code (lazydb_amd/csrc/ldb_sweep_kern.h) run on the CPU under the
// SIMT emulation of tests/emu/simt.h (TEST HARNESS ONLY: linked with ldb_emu.cpp into
// tests/emu/_build/libldb_emu_sweep.so; never part of liblazydb_gpu.so, never a fallback).
//
// emu_sweep_phase plays what the GPU enqueues after the run prefix, in the order the kernels order it:
//   k_sweep   phase S: sweep_item for every workgroup of the launch (one item each), then sweep_last (the
//             links) in one workgroup, as the last workgroup to finish runs it;
//   k_region  phase F (when the links resolved: SwCtl::state == 1): fin_item for every item, then sw_finish
//             on wave 0, as the workgroup that completes the phase runs it.
// The workgroups of a phase run one after another, each to completion: the hardware runs them concurrently,
// and the kernels' only cross-workgroup dependences are the phase boundaries modelled here and the stop word
// (SwCtl::stop), which a later workgroup then sees set from the start -- the sharpest case of its race.
#include "simt.h"

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "../../lazydb_amd/csrc/ldb_pipeline.h"

using namespace ldb;

namespace {
#include "../../lazydb_amd/csrc/ldb_devmem.h"
#include "../../lazydb_amd/csrc/ldb_sweep_kern.h"
}  // namespace

// After the run prefix (dyn[0], dyn[1], dyn[5] as k_uniform leaves them): the tier's phases. vg: k_sweep's
// workgroups (sweep_grid on the GPU); vgf: the most phase-F items (the CU count on the GPU). Returns 1 when
// the tier ended the scan (*p.result written, dyn[3] = kUniDone), 0 when the region pipeline continues from
// dyn[0] / dyn[5].
int emu_sweep_phase(Pipe& p, uint32_t vg, uint32_t vgf) {
  SwCtl* c = p.swctl;
  c->fail = ~0ull;
  c->state = 0;
  c->stop = 0;
  if (vg == 0 || vgf == 0) return -1;
  std::vector<uint8_t> lds_v(std::max<size_t>(kSwLds, kSwLinkLds) + 256);
  uint8_t* lds = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(lds_v.data()) + 255) & ~uintptr_t(255));
  for (uint32_t b = 0; b < vg; ++b)
    simt::run_block(simt::Dim3{b, 0, 0}, simt::Dim3{vg, 1, 1}, 64 * kSwWaves, [&] {
      int tabs = kLdsNone;
      sweep_item(p, b, vg, lds + kSwShBytes, reinterpret_cast<uint32_t*>(lds),
                 reinterpret_cast<uint32_t*>(lds + kSwShBytes + kLp2Bytes), tabs);   // (k_sweep's layout)
    });
  simt::run_block(simt::Dim3{vg - 1, 0, 0}, simt::Dim3{vg, 1, 1}, 64 * kSwWaves, [&] { sweep_last(p, vg, lds); });
  if (c->state != 1) return -2;
  if (getenv("LDB_EMU_SWEEP_DEBUG")) {   // the run records and where the links ended the tier
    std::fprintf(stderr, "sweep: xs %llu xe %llu ks %llu ke %llu ncov %llu nrun %llu\n", (unsigned long long)c->xs,
                 (unsigned long long)c->xe, (unsigned long long)c->ks, (unsigned long long)c->ke,
                 (unsigned long long)c->ncov, (unsigned long long)c->nrun);
    for (uint64_t r = 0; r < c->nrun; ++r) {
      const SwRun& q = p.swrun[r];
      std::fprintf(stderr, "  run %llu [%llu, %llu) E %lld X %llu n %llu flags %x ncand %u\n", (unsigned long long)r,
                   (unsigned long long)q.lo, (unsigned long long)q.hi, (long long)q.E, (unsigned long long)q.X,
                   (unsigned long long)q.n, q.flags, q.ncand);
      if (r < 2) {
        const uint64_t cap64 = p.scratch_bytes / 16 / c->nrun;
        for (uint32_t i = 0; i < q.ncand && i < 64; ++i)
          std::fprintf(stderr, "    cand %llu tag %u\n", (unsigned long long)(p.scratch[r * cap64 + i].pos & 0xFFFFFFFFFFull),
                       (unsigned)(p.scratch[r * cap64 + i].pos >> 60));
      }
    }
  }
  const uint64_t want = (c->ncov + kSwWaves - 1) / kSwWaves;
  const uint32_t nf = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, vgf));
  std::vector<uint32_t> st_v(kSwFinLds / 4 + 64);
  for (uint32_t t = 0; t < nf; ++t)
    simt::run_block(simt::Dim3{t, 0, 0}, simt::Dim3{nf, 1, 1}, 64 * kSwWaves, [&] {
      int tabs = kLdsNone;
      fin_item(p, t, nf, st_v.data(), tabs);
    });
  simt::run_block(simt::Dim3{0, 0, 0}, simt::Dim3{nf, 1, 1}, 64, [&] { sw_finish(p); });
  return p.dyn[3] == kUniDone ? 1 : 0;
}
