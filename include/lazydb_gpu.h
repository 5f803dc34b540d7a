/*
 * lazydb_gpu.h — C ABI of the MI355X log-scan engine (liblazydb_gpu.so).
 *
 * The engine replaces the per-entry body of LazyDB's log-file replay:
 *   reference  logfile/log_file.go:116-145   (*LogFile).ReadLogEntry(offset)
 *              logfile/log_entry.go:81-121    decodeHeader / getEntryCrc
 *              logfile/log_entry.go:48-78     EncodeEntry (only its size is used at replay)
 *              index.go:84-95                 the replay loop that calls ReadLogEntry until EOF
 * One call scans a whole log-file image and returns, in file order, exactly the
 * (fid, offset, entrySize, key/value extents, status) tuples the replay loop
 * would have produced, plus how and where the loop stopped.
 *
 * No torch / HIP types appear in these signatures: device pointers are plain
 * pointers, the HIP stream is passed as `void*` (a hipStream_t, NULL = default).
 * Every function returns an ldb_status (0 = LDB_OK) and never aborts the process.
 */
#ifndef LAZYDB_GPU_H
#define LAZYDB_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDB_ABI_VERSION 4

/* ---- status codes ------------------------------------------------------
 * Normal terminations of the replay loop (index.go:86-88 `break`) are > 0;
 * conditions the reference treats as fatal (index.go:90 log.Fatalf, or a Go
 * runtime panic) are < 0.  LDB_OK (0) is returned by API calls that succeed. */
typedef enum ldb_status {
  LDB_OK = 0,
  LDB_EOF_WINDOW = 1,    /* 38-byte header read hit EOF  -> io.EOF (log_file.go:117-122;
                            iocontroller/fileio.go:35-37 short ReadAt, iocontroller/mmap.go:46-52) */
  LDB_EOF_SENTINEL = 2,  /* crc==0 && kSize==0 && vSize==0 -> ErrLogEndOfFile (log_file.go:124-126) */
  LDB_EOF_KV = 3,        /* key+value read hit EOF -> io.EOF (log_file.go:130-139) */
  LDB_ERR_CRC = -1,      /* stored crc != recomputed -> ErrInvalidCrc (log_file.go:141-143) */
  LDB_ERR_MALFORMED = -2,/* the reference would panic (slice bounds in decodeHeader / getEntryCrc
                            with a negative header size) or get a non-EOF read error */
  LDB_ERR_CAPACITY = -3, /* output array too small (n_entries still reports the full count) */
  LDB_ERR_ARG = -4,      /* bad argument */
  LDB_ERR_HIP = -5,      /* HIP runtime error */
  LDB_ERR_NOMEM = -6,    /* device workspace allocation failed */
  LDB_ERR_INTERNAL = -7  /* a device-side bounds guard fired; results must not be used (never expected) */
} ldb_status;

/* IOController kind of the LogFile being scanned (logfile/log_file.go:35-41).
 * It selects the end-of-file bound rule of the reference:
 *   FileIO: bound = file size, a read of [o, o+n) fails iff o+n >  bound  (os.File.ReadAt)
 *   Mmap  : bound = mapping length (= MaxLogFileSize), fails iff o+n >= bound (mmap.go:48) */
typedef enum ldb_io_type { LDB_IO_FILEIO = 0, LDB_IO_MMAP = 1 } ldb_io_type;

/* ---- output tuples -------------------------------------------------------
 * LDB_TUPLE_INDEX (16 B): what index.go:15-26 needs to build Value{fid, offset, entrySize}
 * and to slice the key out of the file image:
 *   key       = image[offset + hdr_size, + k_size)
 *   value     = image[offset + hdr_size + k_size, + v_size)
 *   next      = offset + hdr_size + k_size + v_size       (index.go:94 offset += entSize)
 *   entrySize = enc_hdr_size + k_size + v_size            (index.go:20 len(EncodeEntry(entry)))
 * `pos` packs: bits [0,40) offset, [40,46) hdr_size, [46,52) enc_hdr_size, [52,60) stat.
 * (fid is the same for every tuple of a call and is returned in ldb_scan_result.) */
typedef struct ldb_index_tuple {
  uint64_t pos;
  uint32_t k_size;
  uint32_t v_size;
} ldb_index_tuple;

#define LDB_POS_OFFSET(p)  ((p) & 0xFFFFFFFFFFull)
#define LDB_POS_HDR(p)     ((uint32_t)(((p) >> 40) & 0x3F))
#define LDB_POS_ENCHDR(p)  ((uint32_t)(((p) >> 46) & 0x3F))
#define LDB_POS_STAT(p)    ((uint32_t)(((p) >> 52) & 0xFF))

/* LDB_TUPLE_ENTRY (48 B): every field of logfile.LogEntry (log_entry.go:35-45) except the
 * key/value bytes, so a host-side ReadLogEntry(offset) can be answered without re-decoding. */
typedef struct ldb_entry {
  uint64_t offset;
  int64_t expired_at;
  uint64_t tx_id;
  uint32_t crc;
  uint32_t k_size;
  uint32_t v_size;
  uint16_t tx_stat;
  uint8_t stat;
  uint8_t hdr_size;
  uint8_t enc_hdr_size;
  uint8_t pad_[3];
  uint32_t fid;
} ldb_entry;

typedef enum ldb_tuple_kind { LDB_TUPLE_INDEX = 0, LDB_TUPLE_ENTRY = 1 } ldb_tuple_kind;

/* Result of one file scan. Tuples [0, n_entries) were produced in file order. */
typedef struct ldb_scan_result {
  int32_t status;        /* how the replay loop stopped: LDB_EOF_* (normal) or LDB_ERR_CRC / _MALFORMED;
                            LDB_ERR_CAPACITY if cap < n_entries (then only cap tuples were written) */
  uint32_t fid;
  uint64_t n_entries;    /* entries accepted before the stop */
  uint64_t end_off;      /* offset at which ReadLogEntry returned `status`; for EOF statuses this is the
                            append position index.go:97-99 stores into LogFile.Offset */
  uint32_t n_repairs;    /* diagnostics: speculative-walk repairs performed (0 on well-formed logs) */
  uint32_t n_regions;    /* diagnostics: regions the region pipeline replayed (after the run prefix) */
  uint32_t n_fast;       /* diagnostics: of those, regions verified by the chained fast path (ldb_chain.h) */
  uint32_t n_broken;     /* diagnostics: links still broken after the repair's parallel walkers (the serial
                            repair's sources; 0 on well-formed logs) */
  uint64_t n_run;        /* diagnostics: leading entries verified as one run of equal-sized entries
                            (k_uniform); they are tuples [0, n_run) */
  uint64_t n_sweep;      /* diagnostics (ABI 3): the entries after them verified by the sweep tier
                            (k_sweep: variable-length entries, ldb_sweep.h); tuples [n_run, n_run + n_sweep) */
} ldb_scan_result;

/* ---- context ---------------------------------------------------------------
 * One context per device and concurrent caller. Holds the device's CRC tables and a
 * growable scan workspace. A context serves one call at a time but is bound to no
 * thread (every entry point selects its device first): callers may pool contexts and
 * hand them to any thread, never to two at once (index.go:103-108 replays the 5 value
 * types from 5 goroutines: 5 contexts). */
typedef struct ldb_ctx ldb_ctx;

int ldb_abi_version(void);
const char* ldb_status_str(int status);

int ldb_ctx_create(int device, ldb_ctx** out);
int ldb_ctx_destroy(ldb_ctx* ctx);
/* Pre-size the workspace for images up to max_len bytes, so later scans do no allocation. */
int ldb_ctx_reserve(ldb_ctx* ctx, uint64_t max_len);
/* Device bytes of workspace a scan of `len` bytes needs. */
uint64_t ldb_workspace_bytes(uint64_t len);

/* Device-resident scan (the hot path).  d_image: `len` bytes in device memory, len = bound
 * (FileIO: the file size; Mmap: the mapping length), 16-byte aligned (LDB_ERR_ARG otherwise).
 * The kernels load whole 16-byte granules, so they may read up to 15 bytes past `len`, inside the
 * granule that holds byte len-1: never past a page boundary, so no allocation that holds the `len`
 * bytes can fault. The values of those bytes never affect any result (tests/test_gpu_abi_contract.py
 * poisons them).  d_out: device array of `cap` tuples of `tuple_kind`.  d_result: device
 * ldb_scan_result written at the end of the stream work.
 * Asynchronous with respect to the host: enqueues work on `stream` and returns. A context may be
 * driven from several streams: a call on a stream other than the previous call's first waits for
 * the context's earlier work (a device-wide drain when the earlier stream is the caller's, which may
 * have been destroyed since), so streams may be created and destroyed freely between calls. */
int ldb_scan_file_dev(ldb_ctx* ctx, const uint8_t* d_image, uint64_t len, uint32_t fid, int io_type,
                      int tuple_kind, void* d_out, uint64_t cap, ldb_scan_result* d_result, void* stream);

/* Host-memory scan: copies the image to HBM, scans, copies tuples and result back.
 * Synchronous. This is what a cgo caller holding an mmap'd file uses. */
int ldb_scan_file(ldb_ctx* ctx, const uint8_t* h_image, uint64_t len, uint32_t fid, int io_type,
                  int tuple_kind, void* h_out, uint64_t cap, ldb_scan_result* h_result);

/* Host-memory scan in two calls, for callers that size their output exactly (ABI 3). The replay's
 * ReadLogEntry loop (logfile/log_file.go:116, index.go:84-95) returns one tuple per entry; a caller
 * that cannot bound the count beforehand would otherwise allocate len/10 + 1 tuples (4.8x the image for
 * ldb_entry). ldb_scan_file_count scans like ldb_scan_file and keeps the tuples in the context's device
 * staging; *h_result says how many there are (n_entries). ldb_scan_copy_out then copies
 * min(n_entries, cap) of them into h_out and sets *n_copied. Synchronous. The tuples stay valid until
 * the next scan call on the same context (copy_out returns LDB_ERR_ARG after one). Device memory held by
 * the context (grow-only, until ldb_ctx_destroy): the image (len bytes, 16-B rounded) plus exactly
 * n_entries tuples of the largest count so far (the count runs with no tuple room, then the staged image
 * is scanned again into an array of n_entries), plus the workspace ldb_workspace_bytes(len). */
int ldb_scan_file_count(ldb_ctx* ctx, const uint8_t* h_image, uint64_t len, uint32_t fid, int io_type,
                        int tuple_kind, ldb_scan_result* h_result);
int ldb_scan_copy_out(ldb_ctx* ctx, void* h_out, uint64_t cap, uint64_t* n_copied);

/* Page-lock a host range (e.g. an mmap'd log file, mmap/mmap_linux.go:14-20) for the lifetime of the
 * mapping, so ldb_scan_file's host-to-device copy runs as direct DMA at PCIe rate instead of through
 * the runtime's pageable staging. Optional: ldb_scan_file works on any host memory. A tuple array
 * registered here for at least cap tuples is written in place by the kernels; any other output
 * array (unregistered, pinned elsewhere, or registered shorter than cap tuples) is staged on the
 * device and copied back. Likewise only an image registered through THIS context for all `len`
 * bytes may be read in place by the kernels (the opt-in direct-image mode); any other image is
 * copied to HBM first (at DMA rate when the runtime knows it as pinned, however it was pinned). */
int ldb_host_register(ldb_ctx* ctx, const void* h_ptr, uint64_t len);
int ldb_host_unregister(ldb_ctx* ctx, const void* h_ptr);

/* Batch of device-resident files scanned back to back on one stream (one device).
 * Multi-GPU callers give each device its own context and file subset. */
int ldb_scan_files_dev(ldb_ctx* ctx, int n_files, const uint8_t* const* d_images, const uint64_t* lens,
                       const uint32_t* fids, int io_type, int tuple_kind, void* const* d_outs,
                       const uint64_t* caps, ldb_scan_result* d_results, void* stream);

/* Serial single-lane GPU walker: same results as ldb_scan_file_dev, one entry at a time.
 * Exists as an independent second implementation for tests; not a fast path. */
int ldb_scan_file_dev_serial(ldb_ctx* ctx, const uint8_t* d_image, uint64_t len, uint32_t fid, int io_type,
                             int tuple_kind, void* d_out, uint64_t cap, ldb_scan_result* d_result,
                             void* stream);

/* Timing hook for bench.py: average device time (ms) of the region pipeline (avg_main_ms: the k_region
 * launch, ABI 4) and of the whole pipeline over the scans since the last reset, measured with HIP events
 * recorded on the scan stream around the launches (no host synchronisation while enabled; the query waits
 * for the recorded events). enable: 1 on + reset, 0 off + reset, -1 query only. */
int ldb_kernel_timing(ldb_ctx* ctx, int enable, double* avg_main_ms, double* avg_total_ms, uint64_t* n);
/* The same with the run prefix (k_uniform, the equal-sized entries at the file start, and on a chunked host
 * scan its per-chunk fills) timed on its own: avg_run_ms; avg_main_ms is k_region. */
int ldb_kernel_timing_split(ldb_ctx* ctx, int enable, double* avg_run_ms, double* avg_main_ms, double* avg_total_ms,
                            uint64_t* n);
/* The phases after the run prefix over the same scans, from the device's constant clock (first item claimed
 * to the phase published, 0 where a phase did not run): [0] 0 (the sweep tier's stream is the k_sweep launch:
 * ldb_kernel_timing_sweep), k_region's [1] the sweep tier's CRC checks and tuples, [2] the regions, [3] their
 * links, [4] the repair, [5] the cross-region CRCs, [6] the compaction. n_phases entries are written (7 are
 * defined, the rest 0). Query only; the reset is ldb_kernel_timing's / ldb_kernel_timing_split's. (ABI 4:
 * replaces ldb_kernel_timing_fill.) */
int ldb_kernel_timing_tail(ldb_ctx* ctx, double* avg_phase_ms, int n_phases);
/* The sweep tier: avg_sweep_ms the k_sweep launch (events), avg_fin_ms its check phase (ldb_kernel_timing_tail's [1]). */
int ldb_kernel_timing_sweep(ldb_ctx* ctx, double* avg_sweep_ms, double* avg_fin_ms);

/* Practical HBM-read ceiling for the roofline report: a read-only XOR
 * reduction over the device image d_image[0, len), 16-B loads, `iters` timed launches after one
 * warm-up, on the context's device and its own stream. *gbps = len / average launch time / 1e9. */
int ldb_read_ceiling(ldb_ctx* ctx, const uint8_t* d_image, uint64_t len, int iters, double* gbps);

/* ---- merge / GC: last-writer-wins liveness and the compacted entry stream ------------------
 * Replaces, for the string value type, the scan + liveness + rewrite body of
 *   db.go:370-427  (*LazyDB).Merge       per target file: ReadLogEntry loop, drop SDelete (:403),
 *                                        drop ExpiredAt != 0 && <= now (:406-409), mergeStr (:413)
 *   db.go:243-265  mergeStr              live iff index[key] == (fid, offset) (:255)
 *   db.go:473-523  writeLogEntry         EncodeEntry + rollover to fid+1 when Offset+size > MaxLogFileSize
 *   index.go:15-26 buildStrIndex         the index those checks read: Put per record, Delete on SDelete,
 *                                        applied in (fid, offset) order (index.go:68-95)
 * and the per-record liveness that lets a replay do one Put per live key. */

/* One log file of the value type, in ascending fid order (index.go:68 sorts fids). */
typedef struct ldb_merge_file {
  const uint8_t* d_image;  /* device image of the file, `len` bytes (the IOController bound) */
  uint64_t len;
  uint32_t fid;
  uint32_t is_target;      /* 1: in the compaction candidate list (discard.go:192-230 getCCL) */
} ldb_merge_file;

/* The ValuePos a rewritten record gets (db.go:516-520), plus where it came from, so the caller can
 * update its index (db.go:260 updateIndexTree) without re-reading the key. */
typedef struct ldb_merge_pos {
  uint64_t offset;      /* offset in the output log file */
  uint32_t fid;         /* output log file (active fid, or a rollover successor) */
  uint32_t entry_size;  /* len(EncodeEntry(entry)) */
  uint64_t src_offset;  /* offset of the record in its input file */
  uint32_t src_file;    /* index of the input file in the ldb_merge_file array */
  uint32_t reserved_;
} ldb_merge_pos;

/* A run of the compacted stream that goes to one log file: stream[stream_off, +n_bytes) is written at
 * file_off of log file `fid`. Segments are in stream order; a rollover starts a new segment. */
typedef struct ldb_merge_segment {
  uint32_t fid;
  uint32_t reserved_;
  uint64_t file_off;
  uint64_t stream_off;
  uint64_t n_bytes;
} ldb_merge_segment;

/* Per input file: its replay scan result and its live records (the index's final values). */
typedef struct ldb_merge_file_stat {
  int32_t status;       /* scan status of the file (ldb_scan_result.status) */
  uint32_t fid;
  uint64_t n_entries;
  uint64_t end_off;
  uint64_t live_count;  /* records that are the final index value of their key */
  uint64_t live_bytes;  /* their EncodeEntry sizes; total - live = the stale bytes discard.go tracks */
} ldb_merge_file_stat;

typedef struct ldb_merge_result {
  int32_t status;       /* LDB_OK; a file's fatal scan status (then bad_file is set); LDB_ERR_CAPACITY */
  int32_t bad_file;     /* -1, or the first input file whose replay scan failed (index.go:90 Fatalf) */
  uint64_t n_records;   /* records replayed over all files */
  uint64_t n_live;      /* records that are the final index value of their key */
  uint64_t n_emit;      /* records rewritten by the merge (live, in a target file, not expired) */
  uint64_t emit_bytes;  /* bytes of the compacted stream */
  uint32_t end_fid;     /* the active file after the merge (rollovers advance it) */
  uint32_t n_segments;
  uint64_t end_off;     /* its append offset (LogFile.Offset) */
} ldb_merge_result;

/* Merge the target files of one value type.  Synchronous; all work runs on `stream` of the context's
 * device.  files: host array of n_files descriptors, ascending fid; the active file (active_fid, append
 * offset active_off) may be among them but must not be a target.  The compacted stream goes to
 * d_stream (device, stream_cap bytes), the new positions to d_pos (device, pos_cap entries), the
 * segments to h_segs (host, seg_cap), per-record liveness (1 byte per replayed record, file order,
 * files concatenated) to d_live (device, live_cap; may be NULL), per-file stats to h_stats (host,
 * n_files; may be NULL).  With no target file this is the replay pre-resolution alone (f1).
 * LDB_ERR_CAPACITY: some output was too small; h_result holds the sizes needed. */
int ldb_merge_files_dev(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type, uint32_t active_fid,
                        uint64_t active_off, uint64_t max_file_size, int64_t now, uint8_t* d_stream,
                        uint64_t stream_cap, ldb_merge_pos* d_pos, uint64_t pos_cap, ldb_merge_segment* h_segs,
                        uint32_t seg_cap, uint8_t* d_live, uint64_t live_cap, ldb_merge_file_stat* h_stats,
                        ldb_merge_result* h_result, void* stream);

/* ---- batch writeLogEntry: EncodeEntry + CRC-32 + rollover for bulk writes ------------------------
 * Replaces the per-entry loop of a transaction commit (tx.go:156-206: for each pending entry,
 * db.writeLogEntry, db.go:473-523) for entries whose bytes are already on the device: every entry is
 * encoded as logfile.EncodeEntry does (log_entry.go:48-78, CRC-32/IEEE over header[4:] ++ key ++ value)
 * and placed with writeLogEntry's rollover rule starting at the active file's append offset. */
typedef struct ldb_encode_item {
  uint64_t key_off;    /* key bytes at d_blob + key_off */
  uint64_t value_off;  /* value bytes at d_blob + value_off */
  uint32_t k_size;
  uint32_t v_size;
  int64_t expired_at;
  uint64_t tx_id;
  uint16_t tx_stat;
  uint8_t stat;
  uint8_t pad_[5];
} ldb_encode_item;

/* Encode n items (device array d_items, bytes in d_blob) into d_stream in item order. Outputs as
 * ldb_merge_files_dev: d_pos[i] = the ValuePos of item i (src_offset = i, src_file = 0), h_segs = the
 * runs per log file, h_result: n_emit = n, emit_bytes, end_fid / end_off / n_segments.
 * Synchronous; LDB_ERR_CAPACITY (sizes in h_result) when an output is too small. */
int ldb_encode_entries_dev(ldb_ctx* ctx, uint64_t n, const ldb_encode_item* d_items, const uint8_t* d_blob,
                           uint32_t active_fid, uint64_t active_off, uint64_t max_file_size, uint8_t* d_stream,
                           uint64_t stream_cap, ldb_merge_pos* d_pos, uint64_t pos_cap, ldb_merge_segment* h_segs,
                           uint32_t seg_cap, ldb_merge_result* h_result, void* stream);

/* Cross-GPU merge (SURVEY.md 8(e), config 5 over N GPUs): each rank merges a contiguous fid block,
 * and the ranks' compacted streams form one writeLogEntry rollover chain (db.go:485-510) in rank
 * order. This re-places n records (entry sizes d_sizes, stream order; NULL: d_pos[i].entry_size) from
 * the start state (active_fid, active_off): h_result gets emit_bytes, end_fid, end_off, n_segments;
 * h_segs (host, seg_cap; may be NULL) the segments; d_pos (device; may be NULL) has offset and fid of
 * every record rewritten, other fields kept. Synchronous. LDB_ERR_CAPACITY: more than seg_cap
 * segments (d_pos is still complete). */
int ldb_merge_repack_dev(ldb_ctx* ctx, uint64_t n, const uint32_t* d_sizes, ldb_merge_pos* d_pos,
                         uint32_t active_fid, uint64_t active_off, uint64_t max_file_size,
                         ldb_merge_segment* h_segs, uint32_t seg_cap, ldb_merge_result* h_result, void* stream);

/* ---- hash-partitioned cross-GPU merge -----------------------------------------
 * Config 5 over N ranks, each holding a contiguous fid block (blocks ascending in rank order):
 *   1. ldb_merge_route_dev on every rank: replay scans of its files, then every record is routed to
 *      the owner of its key (owner = ((hash >> 32) * N) >> 32): route records and key bytes grouped
 *      by owner, ready for one all-to-all (RCCL).
 *   2. ldb_merge_resolve_dev on every owner, over what it received from all ranks: per record, is it
 *      the last record of its key in the global order (source rank, seq)?  One flag byte per record,
 *      returned to the sender by a second all-to-all.
 *   3. ldb_merge_apply_dev on every rank: ldb_merge_files_dev with that liveness instead of its own
 *      table (db.go:255 index[key] == (fid, offset) == last record of the key and not an SDelete).
 *   4. ldb_merge_repack_dev: the rollover chain across ranks, as before. */
typedef struct ldb_route_rec {
  uint64_t hash;      /* 64-bit hash of the key bytes */
  uint32_t seq;       /* the record's index in the sender's replay order (its files concatenated) */
  uint32_t k_size;    /* key length */
  uint64_t key_off;   /* offset of the key bytes in the sender's blob for this owner (16-B aligned) */
} ldb_route_rec;

/* Route the records of this rank's files (ascending fids) to n_owners owners (1..64). d_recs: device,
 * rec_cap records; d_keys: device, key_cap bytes. On return h_counts[o] = records for owner o and
 * h_counts[n_owners + o] = key bytes for owner o (16-B padded per key); owner o's records are
 * d_recs[sum_{p<o} h_counts[p] ...] and its keys d_keys[sum_{p<o} h_counts[n_owners+p] ...], in no
 * particular order inside an owner. h_result: n_records, or a file's fatal scan status (bad_file).
 * LDB_ERR_CAPACITY: rec_cap or key_cap too small (h_counts holds the sizes). Synchronous. */
int ldb_merge_route_dev(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type, uint32_t n_owners,
                        ldb_route_rec* d_recs, uint64_t rec_cap, uint8_t* d_keys, uint64_t key_cap,
                        uint64_t* h_counts, ldb_merge_result* h_result, void* stream);

/* Owner side: n received route records (device), their key bytes (device; each record's key_off
 * already rebased into this concatenated blob) and their global order d_ord[i] = source rank << 32 |
 * seq (device). d_last[i] = 1 iff record i is the last record of its key. Synchronous. */
int ldb_merge_resolve_dev(ldb_ctx* ctx, uint64_t n, const ldb_route_rec* d_recs, const uint8_t* d_keys,
                          const uint64_t* d_ord, uint8_t* d_last, void* stream);

/* ldb_merge_files_dev with the liveness resolved elsewhere: d_last (device, one byte per replayed record
 * of `files`, replay order) = "last record of its key" from the owners. Reuses the replay scan of the
 * preceding ldb_merge_route_dev on this context when the file list is the same (images unchanged). */
int ldb_merge_apply_dev(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type, const uint8_t* d_last,
                        uint32_t active_fid, uint64_t active_off, uint64_t max_file_size, int64_t now,
                        uint8_t* d_stream, uint64_t stream_cap, ldb_merge_pos* d_pos, uint64_t pos_cap,
                        ldb_merge_segment* h_segs, uint32_t seg_cap, uint8_t* d_live, uint64_t live_cap,
                        ldb_merge_file_stat* h_stats, ldb_merge_result* h_result, void* stream);

/* Timing hook for bench.py: device time (ms) of the last ldb_merge_files_dev call, split into the
 * replay scans, the liveness resolution (hash + last-writer-wins) and the compaction (prefix sums,
 * rollover packing, stream copy), measured with HIP events on the merge stream. */
int ldb_merge_timing(ldb_ctx* ctx, double* scan_ms, double* live_ms, double* compact_ms);

#ifdef __cplusplus
}
#endif
#endif /* LAZYDB_GPU_H */
