// Sanitizer driver (TEST INFRASTRUCTURE ONLY): the CPU wave emulator of the engine (tests/emu, the very
// phase code the kernels run: ldb_engine.h, ldb_chain.h, ldb_wave.h, ldb_pipeline.h) and the C oracle,
// built with -fsanitize=address,undefined and run over the golden fixtures and generated logs (every
// generator of oracle/ldb_oracle.c, tiled adversarial shapes, both IO rules, run prefix on and off). Any
// out-of-bounds access, use of uninitialised heap, signed overflow, misaligned access or shift past the
// width aborts the process; any mismatch against the oracle exits non-zero.
// Built and run by tests/test_sanitizers.py (make -C tests/san).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
#include "../../oracle/ldb_oracle.h"
int emu_scan_runs(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                  ldb_scan_result* res, uint32_t* st, uint64_t run_len);
int emu_scan_ex(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                ldb_scan_result* res, uint32_t* st, uint64_t run_len, int run_prefix);
#ifdef LDB_EMU_SWEEP
int emu_scan_sweep(const uint8_t* img, uint64_t len, int io, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                   ldb_scan_result* res, uint32_t* st, uint64_t run_len, uint32_t vg, uint32_t vgf);
#endif
}

// modes: 0-2 the region pipeline alone (every region speculative; runs of 3 and 64 regions), 3 the run prefix
// first, 4 (the sweep build, san_sweep) the run prefix, then the sweep tier's kernel code under tests/emu/simt.h
#ifdef LDB_EMU_SWEEP
static const int kMode0 = 4, kModes = 5;   // (san_sweep: the sweep mode only; san_main runs the others)
#else
static const int kMode0 = 0, kModes = 4;
#endif

static int g_fail = 0, g_cases = 0;

static void check(const char* name, const std::vector<uint8_t>& img) {
  const uint64_t len = img.size();
  const uint8_t* p = len ? img.data() : nullptr;
  for (int io = 0; io < 2; ++io) {
    ldb_scan_result ref{};
    ldbo_scan(p, len, io, 0, 0, nullptr, 0, &ref);
    std::vector<ldb_index_tuple> rt(ref.n_entries + 1);
    ldbo_scan(p, len, io, 0, 0, rt.data(), ref.n_entries, &ref);
    const uint64_t cap = len / 5 + 8;
    for (int mode = kMode0; mode < kModes; ++mode) {
      std::vector<ldb_index_tuple> out(cap);
      ldb_scan_result res{};
      uint32_t st[4] = {0, 0, 0, 0};
      int rc;
      if (mode < 3) rc = emu_scan_runs(p, len, io, 0, out.data(), cap, &res, st, mode == 0 ? 0 : (mode == 1 ? 3 : 64));
      else if (mode == 3) rc = emu_scan_ex(p, len, io, 0, out.data(), cap, &res, st, 64, 1);
#ifdef LDB_EMU_SWEEP
      else rc = emu_scan_sweep(p, len, io, 0, out.data(), cap, &res, st, 64, 3, 4);
#endif
      ++g_cases;
      bool ok = rc == 0 && res.status == ref.status && res.end_off == ref.end_off && res.n_entries == ref.n_entries;
      for (uint64_t i = 0; ok && i < ref.n_entries && i < cap; ++i)
        ok = out[i].pos == rt[i].pos && out[i].k_size == rt[i].k_size && out[i].v_size == rt[i].v_size;
      if (!ok) {
        std::printf("MISMATCH %s io=%d mode=%d rc=%d got (%d,%llu,%llu) want (%d,%llu,%llu)\n", name, io, mode, rc,
                    res.status, (unsigned long long)res.end_off, (unsigned long long)res.n_entries, ref.status,
                    (unsigned long long)ref.end_off, (unsigned long long)ref.n_entries);
        ++g_fail;
      }
    }
  }
}

static std::vector<uint8_t> read_file(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = std::fopen(path, "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  v.resize((size_t)n);
  if (n && std::fread(v.data(), 1, (size_t)n, f) != (size_t)n) v.clear();
  std::fclose(f);
  return v;
}

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    if (kMode0 && (i & 1) == 0) continue;   // (san_sweep: every other fixture, to keep the CPU suite short)
    std::vector<uint8_t> img = read_file(argv[i]);
    check(argv[i], img);
    // the fixture cut at every length mod 16 near its end (ragged tails, both IO rules; san_sweep: one cut)
    for (uint64_t d = 1; d < (kMode0 ? 2u : 16u) && d < img.size(); d += 5) {
      std::vector<uint8_t> cut(img.begin(), img.end() - (long)d);
      check((std::string(argv[i]) + "-cut").c_str(), cut);
    }
  }
  // generated logs: fixed shapes (run prefix), Zipf values, the reference bench's keys, the writer mix
  {
    std::vector<uint8_t> img(1 << 20);
    uint64_t end = 0;
    ldbo_gen_log(img.data(), img.size(), 5, 64, 256, 0, 1.1, 4096, ~0ull, &end);
    check("gen_fixed", img);
    std::fill(img.begin(), img.end(), 0);
    ldbo_gen_log(img.data(), img.size(), 6, 64, 0, 1, 1.1, 512, ~0ull, &end);
    check("gen_zipf", img);
    std::fill(img.begin(), img.end(), 0);
    ldbo_gen_bench_log(img.data(), img.size(), 7, 1500, 512, &end);
    check("gen_bench", img);
    std::fill(img.begin(), img.end(), 0);
    ldbo_gen_writer_log(img.data(), img.size(), 8, ~0ull, 1760000000, 1000, 2048, 100, 100, 100, &end);
    check("gen_writer", img);
    img[end / 2] ^= 0x10;   // a corrupt byte mid-log
    check("gen_writer_corrupt", img);
  }
  std::printf("sanitized emulator + oracle: %d cases, %d mismatches\n", g_cases, g_fail);
  return g_fail ? 1 : 0;
}
