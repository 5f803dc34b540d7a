/*
 * ldb_oracle.h — CPU restatement of LazyDB's log codec and replay scan.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker that the MI355X engine
 * (lazydb_amd/, liblazydb_gpu.so) is compared against; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path never calls it.
 *
 * Parity pinning: the reference (Go, module `lazydb`) cannot be built here
 * (no Go toolchain; and mmap/mmap.go:24 calls `msync`, which the Linux file
 * mmap/mmap_linux.go:75 names `mSync`). This restatement is pinned by the
 * reference's literal known-answer vectors in logfile/log_entry_test.go:18-32,
 * 57-69, 93-104 and db_test.go:203-229 (tests/test_oracle_golden.py), and by
 * a second, independent Python restatement (oracle/pyoracle.py, zlib CRC).
 *
 * Go stdlib semantics restated (Go 1.18, go.mod:3):
 *   encoding/binary.Uvarint / Varint / PutVarint, hash/crc32 IEEE.
 */
#ifndef LDB_ORACLE_H
#define LDB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/lazydb_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LDBO_MAX_HEADER 38 /* logfile/log_entry.go:32 */

/* Decoded header + sizes, the fields of logfile.LogEntry (log_entry.go:35-45). */
typedef struct ldbo_header {
  uint32_t crc;
  uint8_t stat;
  int64_t expired_at;
  uint64_t tx_id;
  uint16_t tx_stat;
  uint32_t k_size;
  uint32_t v_size;
  int32_t size;          /* decodeHeader's returned offset (may be negative for malformed varints) */
  int32_t enc_size;      /* header bytes EncodeEntry would emit for these fields */
} ldbo_header;

/* hash/crc32: Update(crc, IEEETable, p) — crc is the finalized value (0 to start). */
uint32_t ldbo_crc32_update(uint32_t crc, const uint8_t* p, size_t n);
/* Raw reflected register update (no pre/post inversion): the GPU engine's unit. */
uint32_t ldbo_crc32_reg(uint32_t reg, const uint8_t* p, size_t n);
/* the same register update by slicing-by-8 tables only (no carry-less folding): a second formulation */
uint32_t ldbo_crc32_reg_tables(uint32_t reg, const uint8_t* p, size_t n);

/* encoding/binary */
int ldbo_uvarint(const uint8_t* buf, size_t len, uint64_t* x);
int ldbo_varint(const uint8_t* buf, size_t len, int64_t* x);
int ldbo_put_varint(uint8_t* buf, int64_t x);
int ldbo_varint_len(int64_t x);

/* logfile.EncodeEntry (log_entry.go:48-78). Writes the entry to `out` (must hold
 * 38 + klen + vlen bytes) and returns its size. */
size_t ldbo_encode_entry(uint8_t stat, int64_t expired_at, uint64_t tx_id, uint16_t tx_stat,
                         const uint8_t* key, uint32_t klen, const uint8_t* val, uint32_t vlen, uint8_t* out);

/* logfile.decodeHeader (log_entry.go:81-107) on a 38-byte window.
 * Returns 0, or LDB_ERR_MALFORMED where Go would panic (negative slice index). */
int ldbo_decode_header(const uint8_t* win, ldbo_header* h);

/* (*LogFile).ReadLogEntry(off) (log_file.go:116-145) over an image of `len` bytes
 * under the given IOController bound rule. Returns LDB_OK (entry accepted,
 * *entry_size set), an LDB_EOF_* status, LDB_ERR_CRC or LDB_ERR_MALFORMED. */
int ldbo_read_log_entry(const uint8_t* img, uint64_t len, int io_type, uint64_t off, ldbo_header* h,
                        uint64_t* entry_size);

/* The replay loop of index.go:84-95 over one file: tuples in file order.
 * Writes min(n, cap) tuples; res->status is how ReadLogEntry stopped the loop. */
int ldbo_scan(const uint8_t* img, uint64_t len, int io_type, uint32_t fid, int tuple_kind, void* out,
              uint64_t cap, ldb_scan_result* res);

/* "Faithful" replay port used as the CPU baseline: per entry it pread()s the
 * 38-byte header and the k+v bytes from `fd` into fresh heap buffers
 * (log_file.go:117,132), verifies the CRC, and re-encodes the entry to get its
 * size (index.go:20 -> EncodeEntry, a second CRC pass), like the reference. */
int ldbo_scan_faithful(int fd, uint64_t len, int io_type, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                       ldb_scan_result* res);

/* ---- synthetic log generator (format producer: db.go:473-523 writeLogEntry) ----
 * value_mode 0: fixed vsize; 1: vsize = 16*r, r ~ Zipf(zipf_s) on [1, zipf_max].
 * Keys are "key-%0*llu" padded to ksize (ksize >= 5). Values come from a
 * splitmix64-driven 36-character alphabet (bench/db_bench_test.go:21-27).
 * Entries are appended while offset+size <= cap_bytes (the rollover rule of
 * db.go:485); the rest of the image stays zero (fileio.go:66-68 preallocation).
 * Returns the number of entries; *end_off receives the append offset. */
uint64_t ldbo_gen_log(uint8_t* img, uint64_t cap_bytes, uint64_t seed, uint32_t ksize, uint32_t vsize,
                      int value_mode, double zipf_s, uint32_t zipf_max, uint64_t max_entries, uint64_t* end_off);

/* Merge/GC restatement (db.go:243-265, 383-427, 473-523 over the index of index.go:15-26, 68-95).
 * files[i].d_image is a HOST pointer here. Same outputs and capacity rules as ldb_merge_files_dev. */
int ldbo_merge(int n_files, const ldb_merge_file* files, int io_type, uint32_t active_fid, uint64_t active_off,
               uint64_t max_size, int64_t now, uint8_t* stream, uint64_t stream_cap, ldb_merge_pos* pos,
               uint64_t pos_cap, ldb_merge_segment* segs, uint32_t seg_cap, uint8_t* live, uint64_t live_cap,
               ldb_merge_file_stat* stats, ldb_merge_result* res);

/* Merge test set (config 5 shape): every key written twice (half the records stale), optional SDelete /
 * ExpiredAt mix, consecutive files of cap_bytes at imgs + f*cap_bytes. */
uint64_t ldbo_gen_bench_log(uint8_t* img, uint64_t cap_bytes, uint64_t seed, uint64_t n_entries, uint32_t vsize,
                            uint64_t* end_off);
uint64_t ldbo_gen_writer_log(uint8_t* img, uint64_t cap_bytes, uint64_t seed, uint64_t max_entries, int64_t now,
                             uint32_t key_space, uint32_t vmax, uint32_t p_setex, uint32_t p_del, uint32_t p_tx,
                             uint64_t* end_off);
uint64_t ldbo_gen_merge(uint8_t* imgs, uint32_t n_files, uint64_t cap_bytes, uint64_t n_records, uint64_t seed,
                        uint32_t ksize, uint32_t vsize, uint32_t p_delete_ppm, uint32_t p_expire_ppm, int64_t now,
                        uint64_t* end_offs);

/* splitmix64 (shared by generator and tests) */
uint64_t ldbo_splitmix64(uint64_t* state);

#ifdef __cplusplus
}
#endif
#endif
