// ldb_merge.hip — merge/GC engine: last-writer-wins liveness over the replayed records of one value
// type, and the compacted entry stream of the target files.
//
// Reference semantics restated (kakosute/lazydb):
//   index.go:15-26, 68-95   replay: per record in (fid, offset) order, SDelete -> Delete(key), else
//                           Put(key, {fid, offset, EncodeEntry size}); the index holds each key's LAST
//                           record unless that record is an SDelete.
//   db.go:383-427           Merge: for each target file in ascending fid (getCCL sorts, discard.go:224),
//                           for each record: skip SDelete (:403), skip ExpiredAt != 0 && <= now (:406),
//                           mergeStr (:413).
//   db.go:243-265           mergeStr: rewrite iff index[key] == (fid, offset) (:255).
//   db.go:473-523           writeLogEntry: EncodeEntry, then if Offset + size > MaxLogFileSize the active
//                           file rolls over to fid+1 at offset 0 (one check per record, :485), append.
// Because a key's index value is its last record, "index[key] == (fid, offset)" is "this record is the
// last record of its key and not an SDelete"; rewriting one target file never changes that predicate for
// a record of a later target file (its key's last record is elsewhere), so merging the targets in one
// batch equals calling Merge once per target fid, ascending.
//
// Device pipeline (one context stream, synchronous API):
//   replay scans    ldb_scan_file_dev per file (ldb_scan.hip), 16-B index tuples, one slot per file
//   k_insert        per record: 64-bit key hash, open-addressing table of 8-B slots keyed by the full
//                   key bytes, (tag | max record) by CAS + atomicMax     (key bytes + random slot lines)
//   k_live          per record: live = (slot max == seq) && !SDelete; emit flag, sizes; per-block partials
//   k_file_stats    per file: live counts and bytes
//   k_scan_*        exclusive prefix sums of emitted bytes and counts (3-kernel reduce-then-scan)
//   k_pack          one wave: greedy rollover packing by 64-ary search over the byte prefix
//   k_emit_copy     one wave per 64 records: new ValuePos, unaligned 16-B copies of the emitted bytes,
//                   re-encoded header + CRC-32 for the (rare) non-canonical records
// and the batch writeLogEntry of a transaction commit (ldb_encode_entries_dev: k_enc_size, the same
// prefix sums and k_pack, k_enc_copy, k_enc_hdr).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/lazydb_gpu.h"
#include "ldb_common.h"

__attribute__((visibility("hidden"))) int ldb_ctx_device_(ldb_ctx* c);
extern "C" __attribute__((visibility("hidden"))) int ldb_scan_files_dev_batched(
    ldb_ctx* c, int n_files, const uint8_t* const* d_images, const uint64_t* lens, const uint32_t* fids, int io_type,
    void* const* d_outs, const uint64_t* caps, ldb_scan_result* d_results, void* stream, uint64_t* const* d_hash);
extern "C" __attribute__((visibility("hidden"))) int ldb_scan_file_dev_hashed(ldb_ctx* c, const uint8_t* d_image, uint64_t len,
                                                                   uint32_t fid, int io_type, void* d_out,
                                                                   uint64_t cap, ldb_scan_result* d_result,
                                                                   void* stream, uint64_t* d_hash);
__attribute__((visibility("hidden"))) void** ldb_ctx_merge_slot_(ldb_ctx* c);

namespace {

constexpr uint8_t kSDelete = 1;  // logfile/log_entry.go:13-14
constexpr int kScanItems = 8;    // items per thread in the prefix-sum kernels
constexpr int kScanBlock = 256;
constexpr uint64_t kScanTile = (uint64_t)kScanItems * kScanBlock;
constexpr uint32_t kMaxOwners = 64;   // ranks of a hash-partitioned merge (ldb_merge_route_dev)
constexpr uint64_t kGBits = 40;       // record positions in the liveness table: 1 TiB of input per merge
constexpr uint64_t kGMask = (1ull << kGBits) - 1;

struct FileDesc {       // one input file, in device memory
  const uint8_t* img;
  const ldb_index_tuple* recs;   // the file's replayed records (record seq is recs[seq - seq_base])
  uint64_t seq_base;    // first record index of the file; desc[n_files].seq_base = total records
  uint32_t is_target;
  uint32_t fid;
  const uint64_t* hashes;   // key hashes of the file's first n_hashed records (the scan's run prefix)
  uint64_t n_hashed;
  uint64_t gbase;       // the file's first byte in the concatenation of all images (the table's
                        // record positions g; desc[n_files].gbase = total bytes)
};

struct Tail {           // k_pack output
  uint32_t end_fid;
  uint32_t n_segments;
  uint64_t end_off;
  uint64_t tot_b;        // emitted bytes P[n] and records C[n] (C may be null: tot_c = 0)
  uint32_t tot_c;
  uint32_t pad_;
};

struct MergeWs {
  int device = 0;
  ldb_index_tuple* recs = nullptr;   // replayed records: one slot per file (or dense, after a capacity miss)
  uint64_t* hashes = nullptr;        // key hashes, same slots as recs (the scans' run prefixes fill them)
  uint64_t rec_cap = 0;
  uint8_t* seqbuf = nullptr;     // per-record arrays + hash table + scan sums
  uint64_t seqbuf_bytes = 0;
  uint8_t* small = nullptr;      // scan results, file descriptors, stats, tail, segments
  uint64_t small_bytes = 0;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  float t_scan = 0, t_live = 0, t_compact = 0;
  // more scan contexts, each on its own stream: files are dealt round-robin over the caller's
  // context and these (LDB_MERGE_SCAN_LANES, default 4), so one file's small pipeline kernels
  // (k_link .. k_compact, launch-bound) overlap the other files' scans
  static constexpr int kMaxAux = 7;
  int n_aux = 0;
  ldb_ctx* aux[kMaxAux] = {};
  hipStream_t aux_s[kMaxAux] = {};
  hipEvent_t fork = nullptr, join[kMaxAux] = {};
  // the last replay scan (ldb_merge_route_dev), reused by ldb_merge_apply_dev on the same files
  bool cache_ok = false;
  int cache_io = 0;
  std::vector<ldb_merge_file> cache_files;
  std::vector<FileDesc> cache_fdh;
  std::vector<ldb_scan_result> cache_rh;
  uint64_t cache_n = 0;
};

#define MHIP(x)                                    \
  do {                                             \
    if ((x) != hipSuccess) return LDB_ERR_HIP;     \
  } while (0)

// ------------------------------------------------------------------------------ device helpers
__device__ __forceinline__ uint64_t load8u(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

// ldb::key_hash_w over key bytes in memory: whole 16-B (unaligned) loads, the tail byte by byte (it
// never reads past the key)
__device__ uint64_t key_hash(const uint8_t* p, uint32_t n) {
  return ldb::key_hash_w(
      [&](uint32_t i, uint64_t* w) {
        if (i + 16 <= n) {
          __builtin_memcpy(w, p + i, 16);
        } else {
          uint8_t t[16] = {};
          for (uint32_t j = 0; i + j < n; ++j) t[j] = p[i + j];
          __builtin_memcpy(w, t, 16);
        }
      },
      n);
}

__device__ bool key_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  uint32_t i = 0;
  for (; i + 16 <= n; i += 16) {
    uint4 x, y;
    __builtin_memcpy(&x, a + i, 16);
    __builtin_memcpy(&y, b + i, 16);
    if (((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) != 0) return false;
  }
  for (; i + 8 <= n; i += 8)
    if (load8u(a + i) != load8u(b + i)) return false;
  for (; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// the file holding position g of the images' concatenation (last file with gbase <= g)
__device__ __forceinline__ uint32_t file_of_g(const FileDesc* d, uint32_t n_files, uint64_t g) {
  uint32_t lo = 0, hi = n_files - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (d[mid].gbase <= g) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ uint32_t file_of(const FileDesc* d, uint32_t n_files, uint64_t seq) {
  uint32_t lo = 0, hi = n_files - 1;   // last file with seq_base <= seq
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (d[mid].seq_base <= seq) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// File descriptors staged in LDS (small file counts, the common case): the per-record binary search
// then costs LDS reads instead of dependent global loads. Every thread of the block must call it.
constexpr uint32_t kFdLds = 256;
__device__ __forceinline__ const FileDesc* stage_fd(const FileDesc* fd, uint32_t n_files, FileDesc* s) {
  if (n_files + 1 > kFdLds) return fd;
  for (uint32_t i = threadIdx.x; i <= n_files; i += blockDim.x) s[i] = fd[i];
  __syncthreads();
  return s;
}

// Go binary.PutVarint (zig-zag) — encoding/binary/varint.go; EncodeEntry's field encoder
__device__ int put_varint(uint8_t* b, int64_t x) {
  uint64_t ux = (uint64_t)x << 1;
  if (x < 0) ux = ~ux;
  int i = 0;
  while (ux >= 0x80) {
    b[i++] = (uint8_t)(ux | 0x80);
    ux >>= 7;
  }
  b[i++] = (uint8_t)ux;
  return i;
}

__device__ __forceinline__ uint32_t crc_byte(uint32_t c, uint8_t b) {   // reflected CRC-32/IEEE register
  c ^= b;
#pragma unroll
  for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  return c;
}

// ------------------------------------------------------------------------------ liveness
// Insert every record into an open-addressing table keyed by the FULL key bytes: a slot word is
// (hash tag << 32 | representative seq + 1), claimed by CAS; a probe that meets its tag compares its key
// with the representative's, so distinct keys never share a slot whatever their hashes. The slot's
// max word (atomicMax of seq + 1) ends as the key's last record (index.go: later Put/Delete wins).
struct Rec {   // an index tuple unpacked (lazydb_gpu.h LDB_POS_*)
  uint64_t offset;
  uint32_t hdr_size, enc_hdr_size, stat, k_size, v_size;
};

__device__ __forceinline__ Rec rec_of(const FileDesc* fd, uint32_t f, uint64_t seq) {
  const ldb_index_tuple t = fd[f].recs[seq - fd[f].seq_base];
  Rec r;
  r.offset = LDB_POS_OFFSET(t.pos);
  r.hdr_size = LDB_POS_HDR(t.pos);
  r.enc_hdr_size = LDB_POS_ENCHDR(t.pos);
  r.stat = LDB_POS_STAT(t.pos);
  r.k_size = t.k_size;
  r.v_size = t.v_size;
  return r;
}

// The record's header decoded exactly as logfile.decodeHeader does (ldb_common.h), from its 38-byte
// window in the image (readable: the replay accepted the record, log_file.go:117-122).
__device__ __forceinline__ ldb::Header header_of(const uint8_t* img, uint64_t offset) {
  ldb::Header h;
  const uint8_t* w = img + offset;
  ldb::decode_header([&](int i) -> uint32_t { return w[i]; }, &h);
  return h;
}

// ExpiredAt of a record: the first varint after crc and stat (log_entry.go:90-91); a single 0 byte
// (every record without a TTL) is decided without the full decode.
__device__ __forceinline__ int64_t expired_at_of(const uint8_t* img, uint64_t offset) {
  if (img[offset + 5] == 0) return 0;
  return header_of(img, offset).expired_at;
}

__device__ __forceinline__ const uint8_t* key_of(const FileDesc* fd, uint32_t n_files, uint64_t seq, uint32_t* kl) {
  const uint32_t f = file_of(fd, n_files, seq);
  const Rec e = rec_of(fd, f, seq);
  *kl = e.k_size;
  return fd[f].img + e.offset + e.hdr_size;
}

// the record's key hash: from the scan (its file's run prefix) or computed here from the key bytes
__device__ __forceinline__ uint64_t record_hash(const FileDesc* fd, uint32_t n_files, uint64_t seq, const uint8_t* kp,
                                                uint32_t kl) {
  const uint32_t f = file_of(fd, n_files, seq);
  const uint64_t i = seq - fd[f].seq_base;
  return i < fd[f].n_hashed ? fd[f].hashes[i] : key_hash(kp, kl);
}

// The key length of the record whose key starts at byte ko of img, from the bytes before the key: the
// header ends with the k_size and v_size varints (log_entry.go:66-67), and in a binary.Varint every
// byte but the last carries the continuation bit, so walking back from the key, v_size's bytes end
// at ko - 1 and k_size's bytes are those after the previous varint's last byte. The up to 32 bytes
// before the key hold both (<= 10 bytes each) and the last byte of the varint before them; they are
// the lines the key itself is read from.
__device__ __forceinline__ uint32_t key_len_before(const uint8_t* img, uint64_t ko) {
  const uint32_t K = ko < 32 ? (uint32_t)ko : 32u;
  const uint8_t* w = img + ko - K;
  uint32_t m = 0;   // bit i: window byte i carries the continuation bit
  uint64_t W[4] = {0, 0, 0, 0};
  if (K == 32) {
    __builtin_memcpy(W, w, 32);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t c = (uint32_t)(W[j >> 1] >> (32 * (j & 1))) & 0x80808080u;
      m |= (((c >> 7) | (c >> 14) | (c >> 21) | (c >> 28)) & 0xFu) << (4 * j);
    }
  } else {   // a file's first record: no bytes before the image
    for (uint32_t i = 0; i < K; ++i) m |= (uint32_t)(w[i] >> 7) << i;
  }
  const uint32_t z = ~m & (K == 32 ? 0xFFFFFFFFu : ((1u << K) - 1u));   // last bytes of varints
  const uint32_t bv = z & ((1u << (K - 1)) - 1u);   // below v_size's last byte (K - 1)
  const int p = 31 - __builtin_clz(bv | 1u);        // k_size's last byte
  const uint32_t bk = z & ((1u << p) - 1u);
  const int q = bk ? 31 - __builtin_clz(bk) : -1;   // the previous varint's last byte
  const int L = p - q;                              // k_size's bytes [q + 1, p]
  uint64_t u = 0;
  if (K == 32 && L <= 8) {   // from the registers: the 8 bytes from q + 1, 7-bit groups packed
    const int b0 = q + 1, wi = b0 >> 3, sh = 8 * (b0 & 7);
    const uint64_t lo = wi == 0 ? W[0] : wi == 1 ? W[1] : wi == 2 ? W[2] : W[3];
    const uint64_t hi = wi == 0 ? W[1] : wi == 1 ? W[2] : wi == 2 ? W[3] : 0ull;
    uint64_t x = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    x &= L == 8 ? ~0ull : ((1ull << (8 * L)) - 1ull);
#pragma unroll
    for (int j = 0; j < 8; ++j) u |= (x >> j) & (0x7Full << (7 * j));
  } else {
    for (int i = q + 1, sh = 0; i <= p && sh < 64; ++i, sh += 7) u |= (uint64_t)(w[i] & 0x7Fu) << sh;
  }
  return (uint32_t)(int64_t)((u >> 1) ^ (0ull - (u & 1ull)));   // zig-zag (binary.Varint)
}

// A slot is one 64-bit word (hash tag << 40 | g + 1), g = the position of the record's KEY in the
// concatenation of the images (FileDesc::gbase + offset + hdr_size): g grows with the replay order,
// so it names the record AND orders it. The slot is claimed by CAS and then raised by a 64-bit
// atomicMax: every record that reaches a slot has the slot's key (it claimed it, or compared its key
// bytes equal with the slot's current record), so the tag never changes and the low 40 bits end as
// the key's last record. A probe that meets its tag reads the slot's key straight from g (its length
// from the bytes before it, key_len_before), with no detour through the record's index tuple. 8-B
// slots keep the table within the Infinity Cache at config-5 sizes.
// kCasFirst: claim by CAS straight away (the CAS returns the slot's word when it is taken) instead
// of a load first. The slot id goes to slot[seq] with bit 31 = "expired" (db.go:255, ExpiredAt <=
// now): the header sits next to the key this kernel reads, so k_live needs no image access for it.
template <bool kCasFirst>
__global__ __launch_bounds__(256) void k_insert(uint64_t n, const FileDesc* __restrict__ gfd, uint32_t n_files,
                                                unsigned long long* tab, uint64_t mask, uint32_t* __restrict__ slot,
                                                int64_t now, uint64_t tagmask) {
  __shared__ FileDesc s_fd[kFdLds];
  const FileDesc* fd = stage_fd(gfd, n_files, s_fd);
  uint64_t seq = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (seq >= n) return;
  const uint32_t f = file_of(fd, n_files, seq);
  const Rec e = rec_of(fd, f, seq);
  const uint32_t kl = e.k_size;
  const uint8_t* kp = fd[f].img + e.offset + e.hdr_size;
  // a record of its file's run prefix (the records the scan hashed) has entry 0's header bytes, so
  // entry 0's ExpiredAt (one line every such record shares) instead of a line of its own
  const bool in_run = seq - fd[f].seq_base < fd[f].n_hashed;
  const int64_t ea = expired_at_of(fd[f].img, in_run ? 0 : e.offset);
  const bool expired = ea != 0 && ea <= now;
  const uint64_t h = in_run ? fd[f].hashes[seq - fd[f].seq_base] : key_hash(kp, kl);
  const unsigned long long mine = (h & ~kGMask) | (fd[f].gbase + e.offset + e.hdr_size + 1);
  uint64_t i = h & mask;
  for (;;) {
    unsigned long long v;
    if (kCasFirst) {
      v = atomicCAS(&tab[i], 0ull, mine);
      if (v == 0) break;
    } else {
      v = __hip_atomic_load(&tab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == 0) {
        const unsigned long long prev = atomicCAS(&tab[i], 0ull, mine);
        if (prev == 0) break;
        v = prev;
      }
    }
    if (((v ^ mine) & tagmask) == 0) {   // tagmask: ~kGMask (0 = every probe compares keys: a test mode)
      const uint64_t g = (v & kGMask) - 1;
      const uint32_t fr = file_of_g(fd, n_files, g);
      const uint64_t ko = g - fd[fr].gbase;
      const uint32_t rl = key_len_before(fd[fr].img, ko);
      const uint8_t* rp = fd[fr].img + ko;
      if (rl == kl && key_equal(kp, rp, kl)) {
        atomicMax(&tab[i], mine);
        break;
      }
    }
    i = (i + 1) & mask;
  }
  slot[seq] = (uint32_t)i | (expired ? 0x80000000u : 0u);
}

// live = last record of its key and not an SDelete (index.go:16-25); emit = live && target file &&
// not expired (db.go:403-409, 255). Per-file live counts/bytes: a block whose records all lie in one
// file writes one partial (k_file_stats sums them); a block that straddles files adds per record.
// last_in (cross-GPU merge, ldb_merge_apply_dev): "last record of its key" per record, resolved at the
// key's owner rank, instead of the local table.
__global__ __launch_bounds__(256) void k_live(uint64_t n, const FileDesc* __restrict__ gfd, uint32_t n_files,
                                              const unsigned long long* __restrict__ tab,
                                              const uint32_t* __restrict__ slot, const uint8_t* __restrict__ last_in,
                                              int64_t now, uint8_t* __restrict__ live_out,
                                              uint32_t* __restrict__ esz, unsigned long long* __restrict__ part,
                                              unsigned long long* __restrict__ fstat) {
  __shared__ unsigned long long sc[4], sb[4];
  __shared__ FileDesc s_fd[kFdLds];
  const FileDesc* fd = stage_fd(gfd, n_files, s_fd);
  const uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x;
  const uint64_t seq = b0 + threadIdx.x;
  const bool valid = seq < n;
  uint32_t f = 0, size = 0;
  bool live = false;
  if (valid) {
    f = file_of(fd, n_files, seq);
    const Rec e = rec_of(fd, f, seq);
    const uint32_t sl = last_in ? 0u : slot[seq];   // k_insert's slot, bit 31 = expired
    const bool lastw = last_in ? last_in[seq] != 0 : (tab[sl & 0x7FFFFFFFu] & kGMask) == fd[f].gbase + e.offset + e.hdr_size + 1;
    live = lastw && e.stat != kSDelete;
    size = e.enc_hdr_size + e.k_size + e.v_size;
    bool emit = live && fd[f].is_target;
    if (emit) {
      if (last_in) {   // no k_insert ran (ldb_merge_apply_dev): the header from the image
        const int64_t ea = expired_at_of(fd[f].img, e.offset);
        emit = !(ea != 0 && ea <= now);
      } else {
        emit = !(sl >> 31);
      }
    }
    esz[seq] = emit ? size : 0u;
    if (live_out) live_out[seq] = live ? 1 : 0;
  }
  const uint64_t last = (n < b0 + blockDim.x ? n : b0 + blockDim.x) - 1;
  const bool uniform = file_of(fd, n_files, b0) == file_of(fd, n_files, last);
  if (!uniform) {
    if (valid && live) {
      atomicAdd(&fstat[2 * f], 1ull);
      atomicAdd(&fstat[2 * f + 1], (unsigned long long)size);
    }
    if (threadIdx.x == 0) part[2 * blockIdx.x] = part[2 * blockIdx.x + 1] = 0;
    return;
  }
  unsigned long long c = live ? 1ull : 0ull, b = live ? (unsigned long long)size : 0ull;
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    sc[threadIdx.x >> 6] = c;
    sb[threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
    part[2 * blockIdx.x + 1] = sb[0] + sb[1] + sb[2] + sb[3];
  }
}

// ------------------------------------------------------------------------------ hash-partitioned liveness
// Cross-GPU merge: every rank routes its replayed records to the rank that owns
// their key (a function of the key hash), the owner resolves last-writer-wins over the keys it owns,
// and returns one "last record of its key" flag per record. A key's records all meet at its owner,
// so the owner's maximum of the global record order (source rank, record index) per key is exactly
// the key's last record over all files (index.go:68-95 replays fids in ascending order, the fid
// blocks are ascending in rank order).
__device__ __forceinline__ uint32_t owner_of(uint64_t h, uint32_t n_own) {
  return (uint32_t)(((h >> 32) * (uint64_t)n_own) >> 32);   // the high half: the tables use the low bits
}
__device__ __forceinline__ uint64_t pad16(uint32_t k) { return ((uint64_t)k + 15) & ~15ull; }

// pass 1: the key hash of every record, and per owner the record count and the key bytes (16-B
// padded), aggregated per workgroup in LDS
__global__ __launch_bounds__(256) void k_route_count(uint64_t n, const FileDesc* __restrict__ gfd, uint32_t n_files,
                                                     uint32_t n_own, uint64_t* __restrict__ hsh,
                                                     unsigned long long* __restrict__ tot) {
  __shared__ FileDesc s_fd[kFdLds];
  __shared__ unsigned long long sc[2 * kMaxOwners];
  const FileDesc* fd = stage_fd(gfd, n_files, s_fd);
  for (uint32_t i = threadIdx.x; i < 2 * n_own; i += blockDim.x) sc[i] = 0;
  __syncthreads();
  const uint64_t seq = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (seq < n) {
    uint32_t kl;
    const uint8_t* kp = key_of(fd, n_files, seq, &kl);
    const uint64_t h = record_hash(fd, n_files, seq, kp, kl);
    hsh[seq] = h;
    const uint32_t o = owner_of(h, n_own);
    atomicAdd(&sc[o], 1ull);
    atomicAdd(&sc[n_own + o], (unsigned long long)pad16(kl));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 2 * n_own; i += blockDim.x)
    if (sc[i]) atomicAdd(&tot[i], sc[i]);
}

// pass 2: each record's route record and key bytes into its owner's bucket. A workgroup reserves one
// range per owner (one global atomic per owner), then its records take slots inside it (LDS atomics):
// the order inside a bucket is arbitrary, the owner orders by (source rank, seq).
__global__ __launch_bounds__(256) void k_route_fill(uint64_t n, const FileDesc* __restrict__ gfd, uint32_t n_files,
                                                    uint32_t n_own, const uint64_t* __restrict__ hsh,
                                                    const unsigned long long* __restrict__ base,
                                                    unsigned long long* __restrict__ cur,
                                                    ldb_route_rec* __restrict__ recs, uint8_t* __restrict__ keys) {
  __shared__ FileDesc s_fd[kFdLds];
  __shared__ unsigned long long sc[2 * kMaxOwners], sb[2 * kMaxOwners];
  const FileDesc* fd = stage_fd(gfd, n_files, s_fd);
  for (uint32_t i = threadIdx.x; i < 2 * n_own; i += blockDim.x) sc[i] = 0;
  __syncthreads();
  const uint64_t seq = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = seq < n;
  uint32_t kl = 0, o = 0;
  const uint8_t* kp = nullptr;
  uint64_t h = 0, my_r = 0, my_k = 0;
  if (valid) {
    kp = key_of(fd, n_files, seq, &kl);
    h = hsh[seq];
    o = owner_of(h, n_own);
    my_r = atomicAdd(&sc[o], 1ull);
    my_k = atomicAdd(&sc[n_own + o], (unsigned long long)pad16(kl));
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 2 * n_own; i += blockDim.x) sb[i] = sc[i] ? atomicAdd(&cur[i], sc[i]) : 0;
  __syncthreads();
  if (!valid) return;
  const uint64_t r = base[o] + sb[o] + my_r, koff = sb[n_own + o] + my_k;   // key offset inside the owner's blob
  ldb_route_rec rec;
  rec.hash = h;
  rec.seq = (uint32_t)seq;
  rec.k_size = kl;
  rec.key_off = koff;
  recs[r] = rec;
  uint8_t* dst = keys + base[n_own + o] + koff;   // 16-B aligned
  uint32_t i = 0;
  for (; i + 16 <= kl; i += 16) {
    uint4 x;
    __builtin_memcpy(&x, kp + i, 16);
    *reinterpret_cast<uint4*>(dst + i) = x;
  }
  if (i < kl) {
    uint8_t t[16] = {};
    for (uint32_t j = 0; i + j < kl; ++j) t[j] = kp[i + j];
    uint4 x;
    __builtin_memcpy(&x, t, 16);
    *reinterpret_cast<uint4*>(dst + i) = x;
  }
}

// owner: the full-key table over the received records (keys at key_off in the received blob), as
// k_insert, plus the maximum of the global order per key (ord = source rank << 32 | seq)
__global__ __launch_bounds__(256) void k_own_insert(uint64_t n, const ldb_route_rec* __restrict__ recs,
                                                    const uint8_t* __restrict__ keys, const uint64_t* __restrict__ ord,
                                                    unsigned long long* tab, unsigned long long* otab, uint64_t mask,
                                                    uint32_t* __restrict__ slot) {
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= n) return;
  const ldb_route_rec me = recs[i0];
  const uint8_t* kp = keys + me.key_off;
  const unsigned long long mine = (me.hash & 0xFFFFFFFF00000000ull) | (i0 + 1);
  uint64_t i = me.hash & mask;
  for (;;) {
    unsigned long long v = __hip_atomic_load(&tab[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 0) {
      const unsigned long long prev = atomicCAS(&tab[i], 0ull, mine);
      if (prev == 0) break;
      v = prev;
    }
    if ((v >> 32) == (me.hash >> 32)) {
      const ldb_route_rec rep = recs[(v & 0xFFFFFFFFull) - 1];
      if (rep.k_size == me.k_size && key_equal(kp, keys + rep.key_off, me.k_size)) break;
    }
    i = (i + 1) & mask;
  }
  atomicMax(&otab[i], (unsigned long long)(ord[i0] + 1));
  slot[i0] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_own_last(uint64_t n, const uint64_t* __restrict__ ord,
                                                  const unsigned long long* __restrict__ otab,
                                                  const uint32_t* __restrict__ slot, uint8_t* __restrict__ last) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) last[i] = otab[slot[i]] == ord[i] + 1 ? 1 : 0;
}

// one workgroup per file: sum the partials of the k_live blocks that lie wholly inside it
__global__ __launch_bounds__(256) void k_file_stats(const FileDesc* __restrict__ fd, uint32_t n_files, uint64_t n,
                                                    const unsigned long long* __restrict__ part,
                                                    unsigned long long* __restrict__ fstat) {
  __shared__ unsigned long long sc[4], sb[4];
  const uint32_t f = blockIdx.x;
  const uint64_t lo = fd[f].seq_base, hi = fd[f + 1].seq_base;
  unsigned long long c = 0, b = 0;
  if (hi > lo) {
    const uint64_t blo = lo / 256, bhi = (hi - 1) / 256;   // k_live blocks touching the file
    for (uint64_t k = blo + threadIdx.x; k <= bhi; k += blockDim.x) {
      const uint64_t s0 = k * 256, s1 = (n < s0 + 256 ? n : s0 + 256) - 1;
      if (s0 >= lo && s1 < hi) {   // wholly inside: a uniform block (straddlers added per record)
        c += part[2 * k];
        b += part[2 * k + 1];
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    b += __shfl_xor(b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    sc[threadIdx.x >> 6] = c;
    sb[threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&fstat[2 * f], sc[0] + sc[1] + sc[2] + sc[3]);
    atomicAdd(&fstat[2 * f + 1], sb[0] + sb[1] + sb[2] + sb[3]);
  }
}

// ------------------------------------------------------------------------------ prefix sums
// (bytes, count) pairs over esz; exclusive results P (u64 bytes) and C (u32 count), n+1 entries each.
__device__ __forceinline__ void block_exscan(uint64_t& b, uint32_t& c, uint64_t* sb, uint32_t* sc,
                                             uint64_t& tb, uint32_t& tc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t ib = b;
  uint32_t ic = c;
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t xb = __shfl_up(ib, o);
    uint32_t xc = __shfl_up(ic, o);
    if (lane >= o) {
      ib += xb;
      ic += xc;
    }
  }
  if (lane == 63) {
    sb[w] = ib;
    sc[w] = ic;
  }
  __syncthreads();
  uint64_t ob = 0;
  uint32_t oc = 0;
  tb = 0;
  tc = 0;
  for (int k = 0; k < kScanBlock / 64; ++k) {
    if (k < w) {
      ob += sb[k];
      oc += sc[k];
    }
    tb += sb[k];
    tc += sc[k];
  }
  b = ob + ib - b;
  c = oc + ic - c;
  __syncthreads();
}

__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(const uint32_t* __restrict__ esz, uint64_t n,
                                                            uint64_t* __restrict__ bsum, uint32_t* __restrict__ bcnt) {
  __shared__ uint64_t sb[kScanBlock / 64];
  __shared__ uint32_t sc[kScanBlock / 64];
  // the tile's totals only: coalesced loads, order does not matter
  const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile + threadIdx.x;
  uint64_t b = 0;
  uint32_t c = 0;
  for (int k = 0; k < kScanItems; ++k)
    if (t0 + (uint64_t)k * kScanBlock < n) {
      const uint32_t s = esz[t0 + (uint64_t)k * kScanBlock];
      b += s;
      c += s ? 1u : 0u;
    }
  uint64_t tb;
  uint32_t tc;
  block_exscan(b, c, sb, sc, tb, tc);
  if (threadIdx.x == 0) {
    bsum[blockIdx.x] = tb;
    bcnt[blockIdx.x] = tc;
  }
}

// one workgroup: exclusive scan of the per-tile sums in place; totals go to P[n], C[n]
__global__ __launch_bounds__(kScanBlock) void k_scan_tiles(uint64_t* bsum, uint32_t* bcnt, uint64_t nb,
                                                           uint64_t* P, uint32_t* C, uint64_t n) {
  __shared__ uint64_t sb[kScanBlock / 64];
  __shared__ uint32_t sc[kScanBlock / 64];
  uint64_t carry_b = 0;
  uint32_t carry_c = 0;
  for (uint64_t o = 0; o < nb; o += kScanBlock) {
    uint64_t i = o + threadIdx.x;
    uint64_t b = i < nb ? bsum[i] : 0;
    uint32_t c = i < nb ? bcnt[i] : 0;
    uint64_t tb;
    uint32_t tc;
    block_exscan(b, c, sb, sc, tb, tc);
    if (i < nb) {
      bsum[i] = carry_b + b;
      bcnt[i] = carry_c + c;
    }
    carry_b += tb;
    carry_c += tc;
  }
  if (threadIdx.x == 0) {
    P[n] = carry_b;
    C[n] = carry_c;
  }
}

__global__ __launch_bounds__(kScanBlock) void k_scan_write(const uint32_t* __restrict__ esz, uint64_t n,
                                                           const uint64_t* __restrict__ bsum,
                                                           const uint32_t* __restrict__ bcnt,
                                                           uint64_t* __restrict__ P, uint32_t* __restrict__ C) {
  __shared__ uint64_t sb[kScanBlock / 64];
  __shared__ uint32_t sc[kScanBlock / 64];
  // the tile staged through LDS so that global loads and stores are coalesced; thread t scans the
  // tile's items [t kScanItems, (t + 1) kScanItems)
  __shared__ uint32_t s_e[kScanTile];   // sizes in, then the counts C out
  __shared__ uint64_t s_p[kScanTile];   // byte offsets P out
  const uint64_t t0 = (uint64_t)blockIdx.x * kScanTile;
  for (int k = 0; k < kScanItems; ++k) {
    const uint32_t j = k * kScanBlock + threadIdx.x;
    s_e[j] = t0 + j < n ? esz[t0 + j] : 0u;
  }
  __syncthreads();
  uint32_t s[kScanItems];
  uint64_t b = 0;
  uint32_t c = 0;
  for (int k = 0; k < kScanItems; ++k) {
    s[k] = s_e[threadIdx.x * kScanItems + k];
    b += s[k];
    c += s[k] ? 1u : 0u;
  }
  uint64_t tb;
  uint32_t tc;
  block_exscan(b, c, sb, sc, tb, tc);
  b += bsum[blockIdx.x];
  c += bcnt[blockIdx.x];
  for (int k = 0; k < kScanItems; ++k) {   // each thread rewrites only the items it read
    s_p[threadIdx.x * kScanItems + k] = b;
    s_e[threadIdx.x * kScanItems + k] = c;
    b += s[k];
    c += s[k] ? 1u : 0u;
  }
  __syncthreads();
  for (int k = 0; k < kScanItems; ++k) {
    const uint32_t j = k * kScanBlock + threadIdx.x;
    if (t0 + j < n) {
      P[t0 + j] = s_p[j];
      C[t0 + j] = s_e[j];
    }
  }
}

// ------------------------------------------------------------------------------ rollover packing
// largest i in [0, n] with P[i] <= x (P non-decreasing, P[0] = 0): a 64-ary search, one probe per lane
// per round (about 4 dependent rounds over 10^7 records instead of 24), wave-uniform result
__device__ uint64_t last_le(const uint64_t* P, uint64_t n, uint64_t x, int lane) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t step = (hi - lo + 62) / 63;   // lanes 0..63 probe lo .. lo + 63 step >= hi
    const uint64_t idx = lo + (uint64_t)lane * step;
    const uint64_t m = __ballot(idx <= hi && P[idx] <= x);   // a prefix of the lanes; lane 0 always
    const uint64_t nlo = lo + (uint64_t)(63 - __builtin_clzll(m)) * step;
    hi = hi < nlo + step - 1 ? hi : nlo + step - 1;
    lo = nlo;
  }
  return lo;
}

// writeLogEntry's greedy rollover (db.go:485-510) over the emitted records in stream order: a record
// goes to the current file if Offset + size <= MaxLogFileSize, otherwise the file rolls over to fid+1
// and the record is written there at 0 whatever its size. Runs of records that fit are found by binary
// search over the byte prefix, so the loop runs once per output segment. One wave (the searches are
// wave-wide; every lane holds the same state, lane 0 writes).
__global__ __launch_bounds__(64) void k_pack(const uint64_t* __restrict__ P, const uint32_t* __restrict__ C, uint64_t n,
                                             uint32_t active_fid, uint64_t active_off, uint64_t max_size,
                                             ldb_merge_segment* segs, uint32_t seg_cap, Tail* tail) {
  const int lane = threadIdx.x;
  const uint64_t total = P[n];
  uint32_t fid = active_fid, nseg = 0;
  uint64_t off = active_off, x = 0;
  while (x < total) {
    const uint64_t r = last_le(P, n, x, lane);  // the emitted record that starts at stream position x
    const uint64_t size = P[r + 1] - P[r];
    ldb_merge_segment sg;
    sg.reserved_ = 0;
    sg.stream_off = x;
    if (off + size > max_size) {                // rollover, then the record is written unconditionally
      fid += 1;
      off = 0;
      sg.fid = fid;
      sg.file_off = 0;
      off = size;
      x += size;
    } else {
      sg.fid = fid;
      sg.file_off = off;
    }
    if (off < max_size) {                       // extend with every following record that fits
      const uint64_t lim = x + (max_size - off);
      const uint64_t e = last_le(P, n, lim < total ? lim : total, lane);
      const uint64_t x2 = P[e] > x ? P[e] : x;
      off += x2 - x;
      x = x2;
    }
    sg.n_bytes = x - sg.stream_off;
    if (nseg < seg_cap && lane == 0) segs[nseg] = sg;
    ++nseg;
  }
  if (lane == 0) {
    Tail t;
    t.end_fid = fid;
    t.end_off = off;
    t.n_segments = nseg;
    t.tot_b = total;
    t.tot_c = C ? C[n] : 0u;
    t.pad_ = 0;
    *tail = t;
  }
}

// ------------------------------------------------------------------------------ emit + copy
__device__ __forceinline__ uint32_t seg_of(const ldb_merge_segment* s, uint32_t ns, uint64_t sp) {
  uint32_t lo = 0, hi = ns - 1;   // last segment with stream_off <= sp
  while (lo < hi) {
    uint32_t mid = (lo + hi + 1) >> 1;
    if (s[mid].stream_off <= sp) lo = mid; else hi = mid - 1;
  }
  return lo;
}

constexpr int kCopyWaves = 4;

// One wave per 64 consecutive records. Each emitted record is cut into 16-B pieces (unaligned global
// loads/stores; a partial last piece is stored bytewise, so neighbouring records never race); the
// wave's pieces are dealt out over its lanes. Canonical records (hdr_size == enc_hdr_size) are copied
// verbatim: EncodeEntry re-produces their bytes. A non-canonical record gets its key/value copied and
// its header re-encoded by its lane, CRC-32 over the new header and the key/value (log_entry.go:48-78).
// The capacities are checked here, against k_pack's tail, exactly as the host reports them
// (merge_impl): over any of them nothing is written, and no host round trip separates the packing
// from the copy. flags: bit 0 the live-flag output fits, bit 1 the caller takes segments.
__host__ __device__ __forceinline__ bool emit_fits(const Tail& t, uint64_t pos_cap, uint64_t stream_cap, uint32_t seg_cap,
                                          uint32_t flags, bool have_out) {
  return (flags & 1u) && t.tot_c <= pos_cap && t.tot_b <= stream_cap && t.n_segments <= seg_cap &&
         !(t.tot_c && !have_out) && !(t.n_segments && !(flags & 2u));
}

// 16 bytes at any address from whole aligned 16-B granules: the granule holding p, and the next one
// only when p is unaligned (it then holds byte p + 15 of the piece, so it lies inside the image's
// granules, lazydb_gpu.h); the bytes are funnel-shifted into place. An unaligned 16-B load straddles
// two granules per lane instead.
__device__ __forceinline__ uint4 load16_aligned_pair(const uint8_t* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) const v4u* g4_t;
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)15;
  const uint32_t sh = (uint32_t)((uintptr_t)p & 15);
  const v4u lo = *(g4_t)a;
  if (sh == 0) return make_uint4(lo.x, lo.y, lo.z, lo.w);
  const v4u hi = *(g4_t)(a + 16);
  const uint32_t d[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const uint32_t q = sh >> 2, r = sh & 3u;
  uint32_t o[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)   // dwords q .. q + 4 of d
    o[k] = q == 0 ? d[k] : q == 1 ? d[k + 1] : q == 2 ? d[k + 2] : (k + 3 < 8 ? d[k + 3] : 0u);
  return make_uint4(__builtin_amdgcn_alignbyte(o[1], o[0], r), __builtin_amdgcn_alignbyte(o[2], o[1], r),
                    __builtin_amdgcn_alignbyte(o[3], o[2], r), __builtin_amdgcn_alignbyte(o[4], o[3], r));
}

template <int kCopyUnroll>   // pieces in flight per lane
__global__ __launch_bounds__(64 * kCopyWaves) void k_emit_copy(
    uint64_t n, const FileDesc* __restrict__ gfd, uint32_t n_files,
    const uint64_t* __restrict__ P, const uint32_t* __restrict__ C, const ldb_merge_segment* __restrict__ segs,
    const Tail* __restrict__ tail, uint64_t pos_cap, uint64_t stream_cap, uint32_t seg_cap, uint32_t flags,
    uint8_t* __restrict__ stream, ldb_merge_pos* __restrict__ pos) {
  const Tail tl = *tail;
  if (!emit_fits(tl, pos_cap, stream_cap, seg_cap, flags, pos && stream) || tl.tot_c == 0) return;
  const uint32_t n_segs = tl.n_segments;
  __shared__ const uint8_t* s_src[kCopyWaves][64];
  __shared__ uint8_t* s_dst[kCopyWaves][64];
  __shared__ uint32_t s_nb[kCopyWaves][64];
  __shared__ uint32_t s_ex[kCopyWaves][64];
  __shared__ FileDesc s_fd[kFdLds];
  const FileDesc* fd = stage_fd(gfd, n_files, s_fd);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t seq = ((uint64_t)blockIdx.x * kCopyWaves + w) * 64 + lane;
  uint32_t pieces = 0;
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  uint32_t nb = 0;
  Rec e;
  bool canon = true;
  uint64_t sp = 0;
  const uint8_t* fimg = nullptr;
  if (seq < n) {
    sp = P[seq];
    const uint64_t sz = P[seq + 1] - sp;
    if (sz) {
      const uint32_t f = file_of(fd, n_files, seq);
      e = rec_of(fd, f, seq);
      fimg = fd[f].img;
      const ldb_merge_segment& sg = segs[seg_of(segs, n_segs, sp)];
      ldb_merge_pos q;
      q.offset = sg.file_off + (sp - sg.stream_off);
      q.fid = sg.fid;
      q.entry_size = (uint32_t)sz;
      q.src_offset = e.offset;
      q.src_file = f;
      q.reserved_ = 0;
      pos[C[seq]] = q;
      canon = e.hdr_size == e.enc_hdr_size;
      src = fimg + e.offset + (canon ? 0 : e.hdr_size);
      dst = stream + sp + (canon ? 0 : e.enc_hdr_size);
      nb = canon ? (uint32_t)sz : e.k_size + e.v_size;
      // destination-aligned pieces: a head up to the next 16-B boundary, then aligned 16-B stores
      const uint32_t head = min(nb, (16u - (uint32_t)((uintptr_t)dst & 15u)) & 15u);
      pieces = (head ? 1u : 0u) + ((nb - head + 15) >> 4);
    }
  }
  uint32_t inc = pieces;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t x = __shfl_up(inc, o);
    if (lane >= o) inc += x;
  }
  const uint32_t total = __shfl(inc, 63);
  s_src[w][lane] = src;
  s_dst[w][lane] = dst;
  s_nb[w][lane] = nb;
  s_ex[w][lane] = inc - pieces;
  __syncthreads();
  // kCopyUnroll pieces per lane per round: every full piece's load is issued before the round's first
  // store, so a lane keeps that many 16-B reads in flight (one at a time left the copy latency-bound)
  typedef unsigned int v4g __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(1))) v4g* gdst_t;
  for (uint32_t t0 = 0; t0 < total; t0 += 64 * kCopyUnroll) {
    const uint8_t* ss[kCopyUnroll];
    uint8_t* dd[kCopyUnroll];
    uint32_t ll[kCopyUnroll];
    uint4 vv[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint32_t t = t0 + 64u * u + lane;
      ll[u] = 0;
      ss[u] = nullptr;
      dd[u] = nullptr;
      if (t < total) {
        int lo = 0, hi = 63;   // last record with ex <= t and pieces > 0 (ties: the later record owns t)
        while (lo < hi) {
          int mid = (lo + hi + 1) >> 1;
          if (s_ex[w][mid] <= t) lo = mid; else hi = mid - 1;
        }
        const uint32_t j = t - s_ex[w][lo];
        uint8_t* const d0 = s_dst[w][lo];
        const uint32_t nbr = s_nb[w][lo];
        const uint32_t head = min(nbr, (16u - (uint32_t)((uintptr_t)d0 & 15u)) & 15u);
        const uint32_t at = head ? (j ? head + 16 * (j - 1) : 0u) : 16 * j;   // piece start within the record
        ll[u] = (head && j == 0) ? head : min(16u, nbr - at);
        ss[u] = s_src[w][lo] + at;
        dd[u] = d0 + at;
        if (ll[u] == 16) vv[u] = load16_aligned_pair(ss[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint32_t len = ll[u];
      const uint8_t* s = ss[u];
      uint8_t* d = dd[u];
      if (len == 16) {   // d is 16-B aligned here; both sides are touched once: global, non-temporal
        const v4g x = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
        __builtin_nontemporal_store(x, (gdst_t)d);
      } else if (len) {
        uint32_t b = 0;
        if (len & 8) {
          uint64_t v;
          __builtin_memcpy(&v, s, 8);
          __builtin_memcpy(d, &v, 8);
          b = 8;
        }
        if (len & 4) {
          uint32_t v;
          __builtin_memcpy(&v, s + b, 4);
          __builtin_memcpy(d + b, &v, 4);
          b += 4;
        }
        if (len & 2) {
          uint16_t v;
          __builtin_memcpy(&v, s + b, 2);
          __builtin_memcpy(d + b, &v, 2);
          b += 2;
        }
        if (len & 1) d[b] = s[b];
      }
    }
  }
  if (pieces && !canon) {   // re-encode the header (EncodeEntry :52-66) and its CRC (:75-76)
    const ldb::Header dh = header_of(fimg, e.offset);
    uint8_t h[40];
    int o = 5;
    h[4] = (uint8_t)e.stat;
    o += put_varint(h + o, dh.expired_at);
    o += put_varint(h + o, (int64_t)dh.tx_id);
    o += put_varint(h + o, (int64_t)(uint16_t)dh.tx_stat);
    o += put_varint(h + o, (int64_t)e.k_size);
    o += put_varint(h + o, (int64_t)e.v_size);
    uint32_t c = 0xFFFFFFFFu;
    for (int i = 4; i < o; ++i) c = crc_byte(c, h[i]);
    const uint8_t* kv = fimg + e.offset + e.hdr_size;
    for (uint32_t i = 0; i < nb; ++i) c = crc_byte(c, kv[i]);
    c = ~c;
    h[0] = (uint8_t)c;
    h[1] = (uint8_t)(c >> 8);
    h[2] = (uint8_t)(c >> 16);
    h[3] = (uint8_t)(c >> 24);
    uint8_t* d = stream + sp;
    for (int i = 0; i < o; ++i) d[i] = h[i];
  }
}

// ------------------------------------------------------------------------------ batch writeLogEntry
// (tx.go:156-206 commit loop: writeLogEntry per pending entry). Sizes, prefix sums and k_pack are
// shared with the merge; k_enc_copy places the key/value bytes, k_enc_hdr encodes each header and
// its CRC-32 (log_entry.go:48-78).
__device__ __forceinline__ uint32_t enc_hdr_len(const ldb_encode_item& it) {
  return 5u + (uint32_t)ldb::varint_len(it.expired_at) + (uint32_t)ldb::varint_len((int64_t)it.tx_id) +
         (uint32_t)ldb::varint_len((int64_t)it.tx_stat) + (uint32_t)ldb::varint_len((int64_t)it.k_size) +
         (uint32_t)ldb::varint_len((int64_t)it.v_size);
}

__global__ __launch_bounds__(256) void k_enc_size(const ldb_encode_item* __restrict__ items, uint64_t n,
                                                  uint32_t* __restrict__ esz, uint32_t* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ldb_encode_item it = items[i];
  const uint64_t sz = (uint64_t)enc_hdr_len(it) + it.k_size + it.v_size;
  if (sz > 0xFFFFFFFFull) atomicOr(bad, 1u);   // one entry beyond 4 GiB: not representable here
  esz[i] = (uint32_t)sz;
}

// one wave per 64 items: ValuePos and the key and value bytes (two pieces lists per item)
__global__ __launch_bounds__(64 * kCopyWaves) void k_enc_copy(
    const ldb_encode_item* __restrict__ items, uint64_t n, const uint8_t* __restrict__ blob,
    const uint64_t* __restrict__ P, const ldb_merge_segment* __restrict__ segs, uint32_t n_segs,
    uint8_t* __restrict__ stream, ldb_merge_pos* __restrict__ pos) {
  __shared__ const uint8_t* s_src[kCopyWaves][128];
  __shared__ uint8_t* s_dst[kCopyWaves][128];
  __shared__ uint32_t s_nb[kCopyWaves][128];
  __shared__ uint32_t s_ex[kCopyWaves][128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t i = ((uint64_t)blockIdx.x * kCopyWaves + w) * 64 + lane;
  uint32_t pk = 0, pv = 0;
  const uint8_t *ks = nullptr, *vs = nullptr;
  uint8_t *kd = nullptr, *vd = nullptr;
  uint32_t kn = 0, vn = 0;
  if (i < n) {
    const ldb_encode_item it = items[i];
    const uint64_t sp = P[i];
    const ldb_merge_segment& sg = segs[seg_of(segs, n_segs, sp)];
    ldb_merge_pos q;
    q.offset = sg.file_off + (sp - sg.stream_off);
    q.fid = sg.fid;
    q.entry_size = (uint32_t)(P[i + 1] - sp);
    q.src_offset = i;
    q.src_file = 0;
    q.reserved_ = 0;
    pos[i] = q;
    const uint32_t h = enc_hdr_len(it);
    ks = blob + it.key_off;
    vs = blob + it.value_off;
    kd = stream + sp + h;
    vd = kd + it.k_size;
    kn = it.k_size;
    vn = it.v_size;
    pk = (kn + 15) >> 4;
    pv = (vn + 15) >> 4;
  }
  // pieces list: entry 2l = key of lane l, 2l+1 = value of lane l
  const uint32_t mine = pk + pv;
  uint32_t inc = mine;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t x = __shfl_up(inc, o);
    if (lane >= o) inc += x;
  }
  const uint32_t total = __shfl(inc, 63);
  const uint32_t ex = inc - mine;
  s_src[w][2 * lane] = ks;
  s_dst[w][2 * lane] = kd;
  s_nb[w][2 * lane] = kn;
  s_ex[w][2 * lane] = ex;
  s_src[w][2 * lane + 1] = vs;
  s_dst[w][2 * lane + 1] = vd;
  s_nb[w][2 * lane + 1] = vn;
  s_ex[w][2 * lane + 1] = ex + pk;
  __syncthreads();
  for (uint32_t t = lane; t < total; t += 64) {
    int lo = 0, hi = 127;   // last list entry with ex <= t (empty entries share the next one's ex)
    while (lo < hi) {
      int mid = (lo + hi + 1) >> 1;
      if (s_ex[w][mid] <= t) lo = mid; else hi = mid - 1;
    }
    const uint32_t j = t - s_ex[w][lo];
    const uint32_t len = min(16u, s_nb[w][lo] - 16 * j);
    const uint8_t* sp = s_src[w][lo] + 16 * j;
    uint8_t* d = s_dst[w][lo] + 16 * j;
    if (len == 16) {
      uint4 v;
      __builtin_memcpy(&v, sp, 16);
      __builtin_memcpy(d, &v, 16);
    } else {
      for (uint32_t b = 0; b < len; ++b) d[b] = sp[b];
    }
  }
}

// one thread per item: header bytes and CRC-32/IEEE over header[4:] ++ key ++ value, byte-table CRC
__global__ __launch_bounds__(256) void k_enc_hdr(const ldb_encode_item* __restrict__ items, uint64_t n,
                                                 const uint8_t* __restrict__ blob, const uint64_t* __restrict__ P,
                                                 uint8_t* __restrict__ stream) {
  __shared__ uint32_t t8[256];
  for (int b = threadIdx.x; b < 256; b += blockDim.x) {
    uint32_t c = (uint32_t)b;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    t8[b] = c;
  }
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ldb_encode_item it = items[i];
  uint8_t h[40];
  int o = 5;
  h[4] = it.stat;                                 // log_entry.go:54
  o += put_varint(h + o, it.expired_at);          // :57
  o += put_varint(h + o, (int64_t)it.tx_id);      // :59
  o += put_varint(h + o, (int64_t)it.tx_stat);    // :61
  o += put_varint(h + o, (int64_t)it.k_size);     // :63
  o += put_varint(h + o, (int64_t)it.v_size);     // :65
  uint32_t c = 0xFFFFFFFFu;
  for (int k = 4; k < o; ++k) c = t8[(c ^ h[k]) & 0xFF] ^ (c >> 8);
  const uint8_t* kp = blob + it.key_off;
  for (uint32_t k = 0; k < it.k_size; ++k) c = t8[(c ^ kp[k]) & 0xFF] ^ (c >> 8);
  const uint8_t* vp = blob + it.value_off;
  for (uint32_t k = 0; k < it.v_size; ++k) c = t8[(c ^ vp[k]) & 0xFF] ^ (c >> 8);
  c = ~c;                                         // :75 ChecksumIEEE(buf[4:])
  h[0] = (uint8_t)c;                              // :76 LittleEndian.PutUint32
  h[1] = (uint8_t)(c >> 8);
  h[2] = (uint8_t)(c >> 16);
  h[3] = (uint8_t)(c >> 24);
  uint8_t* d = stream + P[i];
  for (int k = 0; k < o; ++k) d[k] = h[k];
}

// ------------------------------------------------------------------------------ host side
int grow(uint8_t** p, uint64_t* have, uint64_t need) {
  if (*have >= need) return LDB_OK;
  if (*p) {   // launches on either merge stream may still read the old buffer
    (void)hipDeviceSynchronize();
    (void)hipFree(*p);
  }
  *p = nullptr;
  *have = 0;
  if (hipMalloc(p, need) != hipSuccess) return LDB_ERR_NOMEM;
  *have = need;
  return LDB_OK;
}

// grow the record array, keeping the first `keep` records
int grow_recs(MergeWs* m, uint64_t need, uint64_t keep, hipStream_t s) {
  if (m->rec_cap >= need) return LDB_OK;
  uint64_t cap = std::max(need, m->rec_cap + m->rec_cap / 2);
  ldb_index_tuple* nr = nullptr;
  uint64_t* nh = nullptr;
  if (hipMalloc(&nr, cap * sizeof(ldb_index_tuple)) != hipSuccess) return LDB_ERR_NOMEM;
  if (hipMalloc(&nh, cap * sizeof(uint64_t)) != hipSuccess) {
    (void)hipFree(nr);
    return LDB_ERR_NOMEM;
  }
  if (keep) MHIP(hipMemcpyAsync(nr, m->recs, keep * sizeof(ldb_index_tuple), hipMemcpyDeviceToDevice, s));
  MHIP(hipStreamSynchronize(s));
  if (m->recs) {   // and the aux stream's scans, which write into the record slots
    (void)hipDeviceSynchronize();
    (void)hipFree(m->recs);
    (void)hipFree(m->hashes);
  }
  m->recs = nr;
  m->hashes = nh;
  m->rec_cap = cap;
  return LDB_OK;
}

MergeWs* get_ws(ldb_ctx* c) {
  void** slot = ldb_ctx_merge_slot_(c);
  if (*slot) return static_cast<MergeWs*>(*slot);
  MergeWs* m = new (std::nothrow) MergeWs();
  if (!m) return nullptr;
  m->device = ldb_ctx_device_(c);
  for (auto& e : m->ev)
    if (hipEventCreate(&e) != hipSuccess) {
      delete m;
      return nullptr;
    }
  *slot = m;
  return m;
}

uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

}  // namespace

__attribute__((visibility("hidden"))) void ldb_merge_release_(void* p) {
  MergeWs* m = static_cast<MergeWs*>(p);
  if (!m) return;
  if (m->recs) (void)hipFree(m->recs);
  if (m->hashes) (void)hipFree(m->hashes);
  if (m->seqbuf) (void)hipFree(m->seqbuf);
  if (m->small) (void)hipFree(m->small);
  for (auto& e : m->ev)
    if (e) (void)hipEventDestroy(e);
  for (int i = 0; i < m->n_aux; ++i) {
    if (m->aux[i]) (void)ldb_ctx_destroy(m->aux[i]);
    if (m->aux_s[i]) (void)hipStreamDestroy(m->aux_s[i]);
    if (m->join[i]) (void)hipEventDestroy(m->join[i]);
  }
  if (m->fork) (void)hipEventDestroy(m->fork);
  delete m;
}

namespace {

// Step 1 of every merge entry point: the replay scans (index.go:84-95 per file), 16-B index tuples.
// All files are enqueued back to back, each into its own slot of len/64 + 1024 records, and read back
// with one synchronisation; only if a file has more records than its slot are the files rescanned
// one by one into dense storage. Fills fdh (nf + 1 descriptors; is_target from `files`) and n. A fatal
// scan status of a file is returned with h_result's status / bad_file / n_records set. With
// use_cache, the previous scan of the same files (ldb_merge_route_dev's) is reused.
int merge_scan_lanes(ldb_ctx* ctx, MergeWs* m, uint32_t nf, const ldb_merge_file* files, int io_type,
                     ldb_scan_result* d_res, const std::vector<uint64_t>& sbase, hipStream_t s, bool scan_hash);
int merge_scan_finish(ldb_ctx* ctx, MergeWs* m, uint32_t nf, const ldb_merge_file* files, int io_type,
                      ldb_scan_result* d_res, std::vector<FileDesc>& fdh, uint64_t& n, ldb_merge_file_stat* h_stats,
                      ldb_merge_result* h_result, hipStream_t s, const std::vector<uint64_t>& sbase,
                      std::vector<ldb_scan_result>& rh, bool scan_hash);

int merge_scan(ldb_ctx* ctx, MergeWs* m, uint32_t nf, const ldb_merge_file* files, int io_type,
               ldb_scan_result* d_res, std::vector<FileDesc>& fdh, uint64_t& n, ldb_merge_file_stat* h_stats,
               ldb_merge_result* h_result, hipStream_t s, bool use_cache, bool produce_cache) {
  fdh.assign(nf + 1, FileDesc{});
  std::vector<ldb_scan_result> rh(nf);
  bool hit = use_cache && m->cache_ok && m->cache_io == io_type && m->cache_files.size() == nf;
  for (uint32_t i = 0; hit && i < nf; ++i)
    hit = m->cache_files[i].d_image == files[i].d_image && m->cache_files[i].len == files[i].len &&
          m->cache_files[i].fid == files[i].fid;
  if (hit) {
    fdh = m->cache_fdh;
    rh = m->cache_rh;
    n = m->cache_n;
    for (uint32_t i = 0; i < nf; ++i) {
      fdh[i].is_target = files[i].is_target;
      if (h_stats) h_stats[i] = ldb_merge_file_stat{rh[i].status, files[i].fid, rh[i].n_entries, rh[i].end_off, 0, 0};
    }
    h_result->n_records = n;
    return LDB_OK;
  }
  m->cache_ok = false;   // m->recs is rewritten below
  int rc = LDB_OK;
  std::vector<uint64_t> sbase(nf + 1, 0);
  for (uint32_t i = 0; i < nf; ++i) sbase[i + 1] = sbase[i] + files[i].len / 64 + 1024;
  rc = grow_recs(m, std::max<uint64_t>(sbase[nf], 4096), 0, s);
  if (rc != LDB_OK) return rc;
  // The scans' run prefixes also emit the key hashes, which k_insert / k_route_count then take instead
  // of reading the key; k_insert reads a run record's ExpiredAt from the file's entry 0 (same header
  // bytes), so such a record's own lines are read only when its hash tag meets a taken slot. Config 5:
  // 4.482 ms against 4.602 without (replay 1.58 vs 1.23 ms, liveness 1.56 vs 2.03; gpurun_out/m3_h*).
  // LDB_MERGE_SCAN_HASH=0 turns it off. Measured and rejected: the entry's G lanes hashing key chunks in
  // parallel (shuffle-combined): replay 1.88-1.97 ms.
  // Round 3: off by default. With the run prefix's verify loop free of stores (k_uniform_fill), the
  // scan-side hash became the most expensive part of the replay: in the loop 1.64 vs 0.97 ms, as a
  // separate pass over the keys 1.84 vs 0.97 ms, against +0.46 ms of liveness when k_insert hashes the
  // key it reads anyway (config 5: 4.58 ms off, 4.74 / 4.94 ms on; gpurun_out/mg1, mg2).
  static const bool scan_hash = ldb::ldb_knob_int("LDB_MERGE_SCAN_HASH", 0) != 0;
  // every file's replay scan in ONE batched pipeline (ldb_scan.hip enqueue_scan_batch) on the
  // caller's context and stream; a set the batch does not take (a tiny image) goes file by file
  {
    std::vector<const uint8_t*> im(nf);
    std::vector<uint64_t> ln(nf), cp(nf);
    std::vector<uint32_t> fi(nf);
    std::vector<void*> ou(nf);
    std::vector<uint64_t*> hs(nf);
    for (uint32_t i = 0; i < nf; ++i) {
      im[i] = files[i].d_image;
      ln[i] = files[i].len;
      fi[i] = files[i].fid;
      ou[i] = m->recs + sbase[i];
      cp[i] = sbase[i + 1] - sbase[i];
      hs[i] = m->hashes + sbase[i];
    }
    rc = nf ? ldb_scan_files_dev_batched(ctx, (int)nf, im.data(), ln.data(), fi.data(), io_type, ou.data(), cp.data(),
                                         d_res, s, scan_hash ? hs.data() : nullptr)
            : LDB_ERR_ARG;
    if (rc != LDB_OK && rc != LDB_ERR_ARG) return rc;
  }
  if (rc != LDB_OK) rc = merge_scan_lanes(ctx, m, nf, files, io_type, d_res, sbase, s, scan_hash);
  if (rc != LDB_OK) return rc;
  if (nf) MHIP(hipMemcpyAsync(rh.data(), d_res, sizeof(ldb_scan_result) * nf, hipMemcpyDeviceToHost, s));
  MHIP(hipStreamSynchronize(s));
  rc = merge_scan_finish(ctx, m, nf, files, io_type, d_res, fdh, n, h_stats, h_result, s, sbase, rh, scan_hash);
  if (!produce_cache) m->cache_ok = false;   // only ldb_merge_route_dev's scan is offered to the next apply
  return rc;
}

// the replay scans file by file, dealt round-robin over the caller's context and the aux contexts
int merge_scan_lanes(ldb_ctx* ctx, MergeWs* m, uint32_t nf, const ldb_merge_file* files, int io_type,
                     ldb_scan_result* d_res, const std::vector<uint64_t>& sbase, hipStream_t s, bool scan_hash) {
  int rc = LDB_OK;
  if (!m->fork) {
    const char* e = ldb::ldb_knob("LDB_MERGE_SCAN_LANES");
    const int want = std::min(std::max(e ? atoi(e) : 4, 1), MergeWs::kMaxAux + 1) - 1;
    MHIP(hipEventCreateWithFlags(&m->fork, hipEventDisableTiming));
    for (int i = 0; i < want; ++i) {
      if (ldb_ctx_create(m->device, &m->aux[i]) != LDB_OK) return LDB_ERR_HIP;
      MHIP(hipStreamCreateWithFlags(&m->aux_s[i], hipStreamNonBlocking));
      MHIP(hipEventCreateWithFlags(&m->join[i], hipEventDisableTiming));
      m->n_aux = i + 1;
    }
  }
  const int lanes = std::min<int>(1 + m->n_aux, (int)nf);   // the caller's context is lane 0
  if (lanes > 1) {
    MHIP(hipEventRecord(m->fork, s));
    for (int a = 0; a + 1 < lanes; ++a) MHIP(hipStreamWaitEvent(m->aux_s[a], m->fork, 0));
  }
  for (uint32_t i = 0; i < nf; ++i) {
    const int lane = (int)(i % (uint32_t)lanes);
    rc = ldb_scan_file_dev_hashed(lane ? m->aux[lane - 1] : ctx, files[i].d_image, files[i].len, files[i].fid,
                                  io_type, m->recs + sbase[i], sbase[i + 1] - sbase[i], d_res + i,
                                  lane ? m->aux_s[lane - 1] : s, scan_hash ? m->hashes + sbase[i] : nullptr);
    if (rc != LDB_OK) {
      // scans already queued on any stream read the caller's images and write m->recs: drain
      // them before the caller can free or reuse anything
      for (int a = 0; a + 1 < lanes; ++a) (void)hipStreamSynchronize(m->aux_s[a]);
      (void)hipStreamSynchronize(s);
      return rc;
    }
  }
  for (int a = 0; a + 1 < lanes; ++a) {
    MHIP(hipEventRecord(m->join[a], m->aux_s[a]));
    MHIP(hipStreamWaitEvent(s, m->join[a], 0));
  }
  return LDB_OK;
}

// after the replay scans: a dense rescan on a capacity miss, then the file descriptors
int merge_scan_finish(ldb_ctx* ctx, MergeWs* m, uint32_t nf, const ldb_merge_file* files, int io_type,
                      ldb_scan_result* d_res, std::vector<FileDesc>& fdh, uint64_t& n, ldb_merge_file_stat* h_stats,
                      ldb_merge_result* h_result, hipStream_t s, const std::vector<uint64_t>& sbase,
                      std::vector<ldb_scan_result>& rh, bool scan_hash) {
  int rc = LDB_OK;
  bool slotted = true;
  for (uint32_t i = 0; i < nf && slotted; ++i) {
    if (rh[i].status == LDB_ERR_CAPACITY) slotted = false;
    if (rh[i].status < 0) break;   // a fatal scan status: later files do not matter
  }
  uint64_t base = 0, gbase = 0;
  for (uint32_t i = 0; i < nf; ++i) {
    if (!slotted) {   // dense rescan, growing the record array as needed
      for (;;) {
        rc = ldb_scan_file_dev(ctx, files[i].d_image, files[i].len, files[i].fid, io_type, LDB_TUPLE_INDEX,
                               m->recs + base, m->rec_cap - base, d_res + i, s);
        if (rc != LDB_OK) return rc;
        MHIP(hipMemcpyAsync(&rh[i], d_res + i, sizeof(ldb_scan_result), hipMemcpyDeviceToHost, s));
        MHIP(hipStreamSynchronize(s));
        if (rh[i].status != LDB_ERR_CAPACITY) break;
        rc = grow_recs(m, base + rh[i].n_entries + 1024, base, s);
        if (rc != LDB_OK) return rc;
      }
    }
    // the run prefix's key hashes (slotted scans only; a dense rescan hashes in the merge kernels)
    const uint64_t nh = slotted && scan_hash ? std::min<uint64_t>(rh[i].n_run, std::min<uint64_t>(rh[i].n_entries,
                                                                                      sbase[i + 1] - sbase[i]))
                                : 0;
    fdh[i] = FileDesc{files[i].d_image, slotted ? m->recs + sbase[i] : m->recs + base, base, files[i].is_target,
                      files[i].fid, slotted ? m->hashes + sbase[i] : nullptr, nh, gbase};
    gbase += files[i].len;
    if (h_stats) {
      h_stats[i] = ldb_merge_file_stat{rh[i].status, files[i].fid, rh[i].n_entries, rh[i].end_off, 0, 0};
    }
    if (rh[i].status < 0) {   // the replay would stop here (index.go:90 log.Fatalf / db.go:399 return err)
      h_result->status = rh[i].status;
      h_result->bad_file = (int32_t)i;
      h_result->n_records = base + rh[i].n_entries;
      return h_result->status;
    }
    base += rh[i].n_entries;
  }
  n = base;
  fdh[nf] = FileDesc{nullptr, nullptr, n, 0, 0, nullptr, 0, gbase};
  h_result->n_records = n;
  if (n >= 0xFFFFFFFFull) return h_result->status = LDB_ERR_ARG;   // record ids are 32-bit
  m->cache_ok = true;
  m->cache_io = io_type;
  m->cache_files.assign(files, files + nf);
  m->cache_fdh = fdh;
  m->cache_rh = rh;
  m->cache_n = n;
  return LDB_OK;
}

}  // namespace


namespace {

int merge_impl(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type, bool ext_live,
               const uint8_t* last_in, uint32_t active_fid, uint64_t active_off, uint64_t max_file_size, int64_t now, uint8_t* d_stream,
               uint64_t stream_cap, ldb_merge_pos* d_pos, uint64_t pos_cap, ldb_merge_segment* h_segs,
               uint32_t seg_cap, uint8_t* d_live, uint64_t live_cap, ldb_merge_file_stat* h_stats,
               ldb_merge_result* h_result, void* stream) {
  if (!ctx || !h_result || n_files < 0 || (n_files && !files) || max_file_size == 0 ||
      (io_type != LDB_IO_FILEIO && io_type != LDB_IO_MMAP))
    return LDB_ERR_ARG;
  std::memset(h_result, 0, sizeof(*h_result));
  h_result->bad_file = -1;
  h_result->end_fid = active_fid;
  h_result->end_off = active_off;
  for (int i = 0; i < n_files; ++i) {
    if (i && files[i].fid <= files[i - 1].fid) return h_result->status = LDB_ERR_ARG;   // ascending fids
    if (files[i].is_target && files[i].fid == active_fid) return h_result->status = LDB_ERR_ARG;
    if (files[i].len && !files[i].d_image) return h_result->status = LDB_ERR_ARG;
  }
  if (hipSetDevice(ldb_ctx_device_(ctx)) != hipSuccess) return LDB_ERR_HIP;
  MergeWs* m = get_ws(ctx);
  if (!m) return LDB_ERR_NOMEM;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t nf = (uint32_t)n_files;

  // small device buffer: scan results | file descriptors (nf+1) | per-file stats (2 u64) | tail | segments
  const uint64_t o_res = 0, o_fd = align256(o_res + sizeof(ldb_scan_result) * (nf + 1));
  const uint64_t o_fst = align256(o_fd + sizeof(FileDesc) * (nf + 1));
  const uint64_t o_tail = align256(o_fst + 16ull * (nf + 1));
  const uint64_t o_seg = align256(o_tail + sizeof(Tail));
  const uint64_t small_need = o_seg + sizeof(ldb_merge_segment) * ((uint64_t)seg_cap + 1);
  int rc = grow(&m->small, &m->small_bytes, small_need);
  if (rc != LDB_OK) return rc;
  ldb_scan_result* d_res = reinterpret_cast<ldb_scan_result*>(m->small + o_res);
  FileDesc* d_fd = reinterpret_cast<FileDesc*>(m->small + o_fd);
  unsigned long long* d_fst = reinterpret_cast<unsigned long long*>(m->small + o_fst);
  Tail* d_tail = reinterpret_cast<Tail*>(m->small + o_tail);
  ldb_merge_segment* d_segs = reinterpret_cast<ldb_merge_segment*>(m->small + o_seg);

  MHIP(hipEventRecord(m->ev[0], s));
  std::vector<FileDesc> fdh;
  uint64_t n = 0;
  rc = merge_scan(ctx, m, nf, files, io_type, d_res, fdh, n, h_stats, h_result, s, ext_live, false);
  if (rc != LDB_OK) return rc;
  if (ext_live && n && !last_in) return h_result->status = LDB_ERR_ARG;   // liveness flags for n records
  MHIP(hipEventRecord(m->ev[1], s));

  // ---- 2. liveness
  // >= (1 + 1/tdiv) slots per record: load <= 0.8 at the default when every key is distinct
  static const uint64_t tdiv = (uint64_t)std::max(1, ldb::ldb_knob_int("LDB_MERGE_TDIV", 4));
  uint64_t tcap = 1024;
  while (tcap < n + n / tdiv) tcap <<= 1;
  if (!ext_live && tcap > (1ull << 31)) return h_result->status = LDB_ERR_ARG;   // slot ids are 31-bit (k_insert)
  if (!ext_live && fdh[nf].gbase >= kGMask) return h_result->status = LDB_ERR_ARG;   // table positions are 40-bit
  const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
  const uint64_t nlb = (n + 255) / 256;
  const uint64_t o_part = 0, o_slot = align256(o_part + 16 * (nlb + 1));
  const uint64_t o_esz = align256(o_slot + 4 * n), o_P = align256(o_esz + 4 * n);
  const uint64_t o_C = align256(o_P + 8 * (n + 1)), o_tk = align256(o_C + 4 * (n + 1));
  const uint64_t o_bs = align256(o_tk + 8 * tcap);
  const uint64_t o_bc = align256(o_bs + 8 * (ntiles + 1)), seq_need = align256(o_bc + 4 * (ntiles + 1));
  rc = grow(&m->seqbuf, &m->seqbuf_bytes, seq_need);
  if (rc != LDB_OK) return rc;
  uint8_t* q = m->seqbuf;
  unsigned long long* d_part = reinterpret_cast<unsigned long long*>(q + o_part);
  uint32_t* d_slot = reinterpret_cast<uint32_t*>(q + o_slot);
  uint32_t* d_esz = reinterpret_cast<uint32_t*>(q + o_esz);
  uint64_t* d_P = reinterpret_cast<uint64_t*>(q + o_P);
  uint32_t* d_C = reinterpret_cast<uint32_t*>(q + o_C);
  unsigned long long* d_tk = reinterpret_cast<unsigned long long*>(q + o_tk);
  uint64_t* d_bs = reinterpret_cast<uint64_t*>(q + o_bs);
  uint32_t* d_bc = reinterpret_cast<uint32_t*>(q + o_bc);

  const bool live_ok = !d_live || live_cap >= n;
  MHIP(hipMemcpyAsync(d_fd, fdh.data(), sizeof(FileDesc) * (nf + 1), hipMemcpyHostToDevice, s));
  MHIP(hipMemsetAsync(d_fst, 0, 16ull * (nf + 1), s));
  if (!ext_live) MHIP(hipMemsetAsync(d_tk, 0, 8 * tcap, s));   // hash table slots
  const uint32_t nbk = (uint32_t)((n + 255) / 256);
  if (n) {
    // LDB_INSERT_CAS=1: claim by CAS without the load first. Off: slower (config 5 k_insert 1.96 ms
    // against 1.72 ms, gpurun_out/ktm_b3) -- a failed CAS costs more than the load it replaces.
    // LDB_MERGE_TAGLESS=1 (tests): no hash tag, every probe that meets a taken slot compares the keys
    const char* tl = ldb::ldb_knob("LDB_MERGE_TAGLESS");
    const uint64_t tagmask = tl && atoi(tl) != 0 ? 0ull : ~kGMask;
    static const bool cas_first = ldb::ldb_knob_int("LDB_INSERT_CAS", 0) != 0;
    if (!ext_live) {
      if (cas_first) k_insert<true><<<nbk, 256, 0, s>>>(n, d_fd, nf, d_tk, tcap - 1, d_slot, now, tagmask);
      else k_insert<false><<<nbk, 256, 0, s>>>(n, d_fd, nf, d_tk, tcap - 1, d_slot, now, tagmask);
    }
    k_live<<<nbk, 256, 0, s>>>(n, d_fd, nf, d_tk, d_slot, last_in, now, live_ok ? d_live : nullptr, d_esz, d_part,
                               d_fst);
    k_file_stats<<<nf, 256, 0, s>>>(d_fd, nf, n, d_part, d_fst);
    MHIP(hipGetLastError());
  }
  MHIP(hipEventRecord(m->ev[2], s));

  // ---- 3. compaction: prefix sums, rollover packing, new positions and the stream
  if (n) {
    k_scan_reduce<<<(uint32_t)ntiles, kScanBlock, 0, s>>>(d_esz, n, d_bs, d_bc);
    k_scan_tiles<<<1, kScanBlock, 0, s>>>(d_bs, d_bc, ntiles, d_P, d_C, n);
    k_scan_write<<<(uint32_t)ntiles, kScanBlock, 0, s>>>(d_esz, n, d_bs, d_bc, d_P, d_C);
  } else {
    MHIP(hipMemsetAsync(d_P, 0, 8, s));
    MHIP(hipMemsetAsync(d_C, 0, 4, s));
  }
  k_pack<<<1, 64, 0, s>>>(d_P, d_C, n, active_fid, active_off, max_file_size, d_segs, seg_cap + 1, d_tail);
  const uint32_t gate = (live_ok ? 1u : 0u) | (h_segs ? 2u : 0u);
  if (n) {   // gated on the device by the capacities (emit_fits): no host round trip in between
    const uint32_t ngrp = (uint32_t)((n + 64 * kCopyWaves - 1) / (64 * kCopyWaves));
    static const int unroll = ldb::ldb_knob_int("LDB_COPY_UNROLL", 1);
    if (unroll >= 4)
      k_emit_copy<4><<<ngrp, 64 * kCopyWaves, 0, s>>>(n, d_fd, nf, d_P, d_C, d_segs, d_tail, pos_cap, stream_cap,
                                                      seg_cap, gate, d_stream, d_pos);
    else if (unroll == 2)
      k_emit_copy<2><<<ngrp, 64 * kCopyWaves, 0, s>>>(n, d_fd, nf, d_P, d_C, d_segs, d_tail, pos_cap, stream_cap,
                                                      seg_cap, gate, d_stream, d_pos);
    else
      k_emit_copy<1><<<ngrp, 64 * kCopyWaves, 0, s>>>(n, d_fd, nf, d_P, d_C, d_segs, d_tail, pos_cap, stream_cap,
                                                      seg_cap, gate, d_stream, d_pos);
  }
  MHIP(hipGetLastError());
  MHIP(hipEventRecord(m->ev[3], s));
  // one copy back: the per-file stats and the tail (adjacent in `small`)
  std::vector<uint8_t> sm(o_tail + sizeof(Tail) - o_fst);
  MHIP(hipMemcpyAsync(sm.data(), m->small + o_fst, sm.size(), hipMemcpyDeviceToHost, s));
  MHIP(hipStreamSynchronize(s));
  Tail tail;
  std::memcpy(&tail, sm.data() + (o_tail - o_fst), sizeof(Tail));
  std::vector<unsigned long long> fst(2 * (nf + 1));
  std::memcpy(fst.data(), sm.data(), 16ull * (nf + 1));
  MHIP(hipEventElapsedTime(&m->t_scan, m->ev[0], m->ev[1]));
  MHIP(hipEventElapsedTime(&m->t_live, m->ev[1], m->ev[2]));
  MHIP(hipEventElapsedTime(&m->t_compact, m->ev[2], m->ev[3]));
  const uint64_t tot_b = tail.tot_b;
  const uint32_t tot_c = tail.tot_c;
  h_result->n_emit = tot_c;
  h_result->emit_bytes = tot_b;
  h_result->end_fid = tail.end_fid;
  h_result->end_off = tail.end_off;
  h_result->n_segments = tail.n_segments;
  for (uint32_t i = 0; i < nf; ++i) {
    h_result->n_live += fst[2 * i];
    if (h_stats) {
      h_stats[i].live_count = fst[2 * i];
      h_stats[i].live_bytes = fst[2 * i + 1];
    }
  }
  if (!emit_fits(tail, pos_cap, stream_cap, seg_cap, gate, d_pos && d_stream))
    return h_result->status = LDB_ERR_CAPACITY;   // k_emit_copy wrote nothing
  if (tail.n_segments) {
    MHIP(hipMemcpyAsync(h_segs, d_segs, sizeof(ldb_merge_segment) * tail.n_segments, hipMemcpyDeviceToHost, s));
    MHIP(hipStreamSynchronize(s));
  }
  h_result->status = LDB_OK;
  return LDB_OK;
}

}  // namespace

extern "C" int ldb_merge_files_dev(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type,
                                   uint32_t active_fid, uint64_t active_off, uint64_t max_file_size, int64_t now,
                                   uint8_t* d_stream, uint64_t stream_cap, ldb_merge_pos* d_pos, uint64_t pos_cap,
                                   ldb_merge_segment* h_segs, uint32_t seg_cap, uint8_t* d_live, uint64_t live_cap,
                                   ldb_merge_file_stat* h_stats, ldb_merge_result* h_result, void* stream) {
  return merge_impl(ctx, n_files, files, io_type, false, nullptr, active_fid, active_off, max_file_size, now,
                    d_stream, stream_cap, d_pos, pos_cap, h_segs, seg_cap, d_live, live_cap, h_stats, h_result, stream);
}

extern "C" int ldb_merge_apply_dev(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type,
                                   const uint8_t* d_last, uint32_t active_fid, uint64_t active_off,
                                   uint64_t max_file_size, int64_t now, uint8_t* d_stream, uint64_t stream_cap,
                                   ldb_merge_pos* d_pos, uint64_t pos_cap, ldb_merge_segment* h_segs, uint32_t seg_cap,
                                   uint8_t* d_live, uint64_t live_cap, ldb_merge_file_stat* h_stats,
                                   ldb_merge_result* h_result, void* stream) {
  // d_last may be NULL only when the files hold no record (checked after the scan)
  const int rc = merge_impl(ctx, n_files, files, io_type, true, d_last, active_fid, active_off, max_file_size, now,
                            d_stream, stream_cap, d_pos, pos_cap, h_segs, seg_cap, d_live, live_cap, h_stats, h_result,
                            stream);
  if (rc != LDB_ERR_CAPACITY) {   // the route's scan is used once (a capacity retry may reuse it)
    MergeWs* m = static_cast<MergeWs*>(*ldb_ctx_merge_slot_(ctx));
    if (m) m->cache_ok = false;
  }
  return rc;
}

extern "C" int ldb_merge_route_dev(ldb_ctx* ctx, int n_files, const ldb_merge_file* files, int io_type,
                                   uint32_t n_owners, ldb_route_rec* d_recs, uint64_t rec_cap, uint8_t* d_keys,
                                   uint64_t key_cap, uint64_t* h_counts, ldb_merge_result* h_result, void* stream) {
  if (!ctx || !h_result || !h_counts || n_files < 0 || (n_files && !files) || n_owners == 0 ||
      n_owners > kMaxOwners || (io_type != LDB_IO_FILEIO && io_type != LDB_IO_MMAP))
    return LDB_ERR_ARG;
  std::memset(h_result, 0, sizeof(*h_result));
  h_result->bad_file = -1;
  std::memset(h_counts, 0, sizeof(uint64_t) * 2 * n_owners);
  for (int i = 0; i < n_files; ++i) {
    if (i && files[i].fid <= files[i - 1].fid) return h_result->status = LDB_ERR_ARG;
    if (files[i].len && !files[i].d_image) return h_result->status = LDB_ERR_ARG;
  }
  if (hipSetDevice(ldb_ctx_device_(ctx)) != hipSuccess) return LDB_ERR_HIP;
  MergeWs* m = get_ws(ctx);
  if (!m) return LDB_ERR_NOMEM;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t nf = (uint32_t)n_files;
  const uint64_t o_res = 0, o_fd = align256(sizeof(ldb_scan_result) * (nf + 1));
  const uint64_t o_cnt = align256(o_fd + sizeof(FileDesc) * (nf + 1));
  int rc = grow(&m->small, &m->small_bytes, o_cnt + 3 * 16ull * kMaxOwners);
  if (rc != LDB_OK) return rc;
  ldb_scan_result* d_res = reinterpret_cast<ldb_scan_result*>(m->small + o_res);
  FileDesc* d_fd = reinterpret_cast<FileDesc*>(m->small + o_fd);
  unsigned long long* d_tot = reinterpret_cast<unsigned long long*>(m->small + o_cnt);   // 2 n_own
  unsigned long long* d_base = d_tot + 2 * kMaxOwners;
  unsigned long long* d_cur = d_base + 2 * kMaxOwners;
  std::vector<FileDesc> fdh;
  uint64_t n = 0;
  rc = merge_scan(ctx, m, nf, files, io_type, d_res, fdh, n, nullptr, h_result, s, false, true);
  if (rc != LDB_OK) return rc;
  rc = grow(&m->seqbuf, &m->seqbuf_bytes, align256(8 * (n + 1)));
  if (rc != LDB_OK) return rc;
  uint64_t* d_h = reinterpret_cast<uint64_t*>(m->seqbuf);
  MHIP(hipMemcpyAsync(d_fd, fdh.data(), sizeof(FileDesc) * (nf + 1), hipMemcpyHostToDevice, s));
  MHIP(hipMemsetAsync(d_tot, 0, 3 * 16ull * kMaxOwners, s));
  const uint32_t nbk = (uint32_t)((n + 255) / 256);
  if (n) k_route_count<<<nbk, 256, 0, s>>>(n, d_fd, nf, n_owners, d_h, d_tot);
  MHIP(hipGetLastError());
  std::vector<unsigned long long> tot(2 * n_owners);
  MHIP(hipMemcpyAsync(tot.data(), d_tot, sizeof(unsigned long long) * 2 * n_owners, hipMemcpyDeviceToHost, s));
  MHIP(hipStreamSynchronize(s));
  std::vector<unsigned long long> base(2 * n_owners);
  uint64_t nr = 0, nk = 0;
  for (uint32_t o = 0; o < n_owners; ++o) {
    h_counts[o] = tot[o];
    h_counts[n_owners + o] = tot[n_owners + o];
    base[o] = nr;
    base[n_owners + o] = nk;
    nr += tot[o];
    nk += tot[n_owners + o];
  }
  h_result->n_records = n;
  if (nr > rec_cap || nk > key_cap || (nr && (!d_recs || !d_keys))) return h_result->status = LDB_ERR_CAPACITY;
  MHIP(hipMemcpyAsync(d_base, base.data(), sizeof(unsigned long long) * 2 * n_owners, hipMemcpyHostToDevice, s));
  if (n) k_route_fill<<<nbk, 256, 0, s>>>(n, d_fd, nf, n_owners, d_h, d_base, d_cur, d_recs, d_keys);
  MHIP(hipGetLastError());
  MHIP(hipStreamSynchronize(s));
  h_result->status = LDB_OK;
  return LDB_OK;
}

extern "C" int ldb_merge_resolve_dev(ldb_ctx* ctx, uint64_t n, const ldb_route_rec* d_recs, const uint8_t* d_keys,
                                     const uint64_t* d_ord, uint8_t* d_last, void* stream) {
  if (!ctx || (n && (!d_recs || !d_keys || !d_ord || !d_last)) || n >= 0xFFFFFFFFull) return LDB_ERR_ARG;
  if (hipSetDevice(ldb_ctx_device_(ctx)) != hipSuccess) return LDB_ERR_HIP;
  MergeWs* m = get_ws(ctx);
  if (!m) return LDB_ERR_NOMEM;
  hipStream_t s = (hipStream_t)stream;
  if (!n) return LDB_OK;
  uint64_t tcap = 1024;
  while (tcap < n + n / 4) tcap <<= 1;
  const uint64_t o_tab = 0, o_otab = align256(8 * tcap), o_slot = align256(o_otab + 8 * tcap);
  // (m->seqbuf only: the route's scan in m->recs stays valid for the rank's ldb_merge_apply_dev)
  int rc = grow(&m->seqbuf, &m->seqbuf_bytes, align256(o_slot + 4 * n));
  if (rc != LDB_OK) return rc;
  unsigned long long* d_tab = reinterpret_cast<unsigned long long*>(m->seqbuf + o_tab);
  unsigned long long* d_otab = reinterpret_cast<unsigned long long*>(m->seqbuf + o_otab);
  uint32_t* d_slot = reinterpret_cast<uint32_t*>(m->seqbuf + o_slot);
  MHIP(hipMemsetAsync(m->seqbuf, 0, o_slot, s));   // both tables
  const uint32_t nbk = (uint32_t)((n + 255) / 256);
  k_own_insert<<<nbk, 256, 0, s>>>(n, d_recs, d_keys, d_ord, d_tab, d_otab, tcap - 1, d_slot);
  k_own_last<<<nbk, 256, 0, s>>>(n, d_ord, d_otab, d_slot, d_last);
  MHIP(hipGetLastError());
  MHIP(hipStreamSynchronize(s));
  return LDB_OK;
}

extern "C" int ldb_encode_entries_dev(ldb_ctx* ctx, uint64_t n, const ldb_encode_item* d_items,
                                      const uint8_t* d_blob, uint32_t active_fid, uint64_t active_off,
                                      uint64_t max_file_size, uint8_t* d_stream, uint64_t stream_cap,
                                      ldb_merge_pos* d_pos, uint64_t pos_cap, ldb_merge_segment* h_segs,
                                      uint32_t seg_cap, ldb_merge_result* h_result, void* stream) {
  if (!ctx || !h_result || (n && (!d_items || !d_blob)) || max_file_size == 0 || n >= 0xFFFFFFFFull)
    return LDB_ERR_ARG;
  std::memset(h_result, 0, sizeof(*h_result));
  h_result->bad_file = -1;
  h_result->end_fid = active_fid;
  h_result->end_off = active_off;
  h_result->n_records = n;
  if (hipSetDevice(ldb_ctx_device_(ctx)) != hipSuccess) return LDB_ERR_HIP;
  MergeWs* m = get_ws(ctx);
  if (!m) return LDB_ERR_NOMEM;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t o_tail = 0, o_bad = align256(sizeof(Tail)), o_seg = align256(o_bad + 4);
  int rc = grow(&m->small, &m->small_bytes, o_seg + sizeof(ldb_merge_segment) * ((uint64_t)seg_cap + 1));
  if (rc != LDB_OK) return rc;
  Tail* d_tail = reinterpret_cast<Tail*>(m->small + o_tail);
  uint32_t* d_bad = reinterpret_cast<uint32_t*>(m->small + o_bad);
  ldb_merge_segment* d_segs = reinterpret_cast<ldb_merge_segment*>(m->small + o_seg);
  const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
  const uint64_t o_esz = 0, o_P = align256(4 * n), o_C = align256(o_P + 8 * (n + 1));
  const uint64_t o_bs = align256(o_C + 4 * (n + 1)), o_bc = align256(o_bs + 8 * (ntiles + 1));
  rc = grow(&m->seqbuf, &m->seqbuf_bytes, align256(o_bc + 4 * (ntiles + 1)));
  if (rc != LDB_OK) return rc;
  uint32_t* d_esz = reinterpret_cast<uint32_t*>(m->seqbuf + o_esz);
  uint64_t* d_P = reinterpret_cast<uint64_t*>(m->seqbuf + o_P);
  uint32_t* d_C = reinterpret_cast<uint32_t*>(m->seqbuf + o_C);
  uint64_t* d_bs = reinterpret_cast<uint64_t*>(m->seqbuf + o_bs);
  uint32_t* d_bc = reinterpret_cast<uint32_t*>(m->seqbuf + o_bc);
  MHIP(hipMemsetAsync(d_bad, 0, 4, s));
  if (n) {
    k_enc_size<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(d_items, n, d_esz, d_bad);
    k_scan_reduce<<<(uint32_t)ntiles, kScanBlock, 0, s>>>(d_esz, n, d_bs, d_bc);
    k_scan_tiles<<<1, kScanBlock, 0, s>>>(d_bs, d_bc, ntiles, d_P, d_C, n);
    k_scan_write<<<(uint32_t)ntiles, kScanBlock, 0, s>>>(d_esz, n, d_bs, d_bc, d_P, d_C);
  } else {
    MHIP(hipMemsetAsync(d_P, 0, 8, s));
  }
  k_pack<<<1, 64, 0, s>>>(d_P, nullptr, n, active_fid, active_off, max_file_size, d_segs, seg_cap + 1, d_tail);
  MHIP(hipGetLastError());
  uint64_t tot = 0;
  uint32_t bad = 0;
  Tail tail;
  MHIP(hipMemcpyAsync(&tot, d_P + n, 8, hipMemcpyDeviceToHost, s));
  MHIP(hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, s));
  MHIP(hipMemcpyAsync(&tail, d_tail, sizeof(Tail), hipMemcpyDeviceToHost, s));
  MHIP(hipStreamSynchronize(s));
  if (bad) return h_result->status = LDB_ERR_ARG;
  h_result->n_emit = n;
  h_result->emit_bytes = tot;
  h_result->end_fid = tail.end_fid;
  h_result->end_off = tail.end_off;
  h_result->n_segments = tail.n_segments;
  if (tot > stream_cap || n > pos_cap || tail.n_segments > seg_cap || (n && (!d_stream || !d_pos)) ||
      (tail.n_segments && !h_segs))
    return h_result->status = LDB_ERR_CAPACITY;
  if (n) {
    const uint32_t ngrp = (uint32_t)((n + 64 * kCopyWaves - 1) / (64 * kCopyWaves));
    k_enc_copy<<<ngrp, 64 * kCopyWaves, 0, s>>>(d_items, n, d_blob, d_P, d_segs, tail.n_segments, d_stream, d_pos);
    k_enc_hdr<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(d_items, n, d_blob, d_P, d_stream);
    MHIP(hipGetLastError());
  }
  if (tail.n_segments)
    MHIP(hipMemcpyAsync(h_segs, d_segs, sizeof(ldb_merge_segment) * tail.n_segments, hipMemcpyDeviceToHost, s));
  MHIP(hipStreamSynchronize(s));
  h_result->status = LDB_OK;
  return LDB_OK;
}

// ------------------------------------------------------------------------------ repack (cross-GPU merge)
// A compacted stream cut into per-rank pieces is placed by one global writeLogEntry rollover chain
// (db.go:485-510): rank r's records start where rank r-1's ended. ldb_merge_repack_dev re-runs k_pack
// over a record-size list from a given (fid, offset) and rewrites the records' ValuePos.
__global__ __launch_bounds__(256) void k_pos_size(uint64_t n, const ldb_merge_pos* __restrict__ pos,
                                                  uint32_t* __restrict__ esz) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i < n) esz[i] = pos[i].entry_size;
}

__global__ __launch_bounds__(256) void k_repos(uint64_t n, const uint64_t* __restrict__ P,
                                               const ldb_merge_segment* __restrict__ segs, uint32_t n_segs,
                                               ldb_merge_pos* __restrict__ pos) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  const uint64_t sp = P[i];
  const ldb_merge_segment& sg = segs[seg_of(segs, n_segs, sp)];
  pos[i].offset = sg.file_off + (sp - sg.stream_off);
  pos[i].fid = sg.fid;
}

extern "C" int ldb_merge_repack_dev(ldb_ctx* ctx, uint64_t n, const uint32_t* d_sizes, ldb_merge_pos* d_pos,
                                    uint32_t active_fid, uint64_t active_off, uint64_t max_file_size,
                                    ldb_merge_segment* h_segs, uint32_t seg_cap, ldb_merge_result* h_result,
                                    void* stream) {
  if (!ctx || !h_result || (n && !d_sizes && !d_pos) || max_file_size == 0 || n >= 0xFFFFFFFFull)
    return LDB_ERR_ARG;
  std::memset(h_result, 0, sizeof(*h_result));
  h_result->bad_file = -1;
  h_result->end_fid = active_fid;
  h_result->end_off = active_off;
  h_result->n_emit = n;
  if (hipSetDevice(ldb_ctx_device_(ctx)) != hipSuccess) return LDB_ERR_HIP;
  MergeWs* m = get_ws(ctx);
  if (!m) return LDB_ERR_NOMEM;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
  const uint64_t o_esz = 0, o_P = align256(4 * n), o_C = align256(o_P + 8 * (n + 1));
  const uint64_t o_bs = align256(o_C + 4 * (n + 1)), o_bc = align256(o_bs + 8 * (ntiles + 1));
  int rc = grow(&m->seqbuf, &m->seqbuf_bytes, align256(o_bc + 4 * (ntiles + 1)));
  if (rc != LDB_OK) return rc;
  uint32_t* d_esz = reinterpret_cast<uint32_t*>(m->seqbuf + o_esz);
  uint64_t* d_P = reinterpret_cast<uint64_t*>(m->seqbuf + o_P);
  uint32_t* d_C = reinterpret_cast<uint32_t*>(m->seqbuf + o_C);
  uint64_t* d_bs = reinterpret_cast<uint64_t*>(m->seqbuf + o_bs);
  uint32_t* d_bc = reinterpret_cast<uint32_t*>(m->seqbuf + o_bc);
  if (n) {
    const uint32_t* esz = d_sizes;
    if (!esz) {
      k_pos_size<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(n, d_pos, d_esz);
      esz = d_esz;
    }
    k_scan_reduce<<<(uint32_t)ntiles, kScanBlock, 0, s>>>(esz, n, d_bs, d_bc);
    k_scan_tiles<<<1, kScanBlock, 0, s>>>(d_bs, d_bc, ntiles, d_P, d_C, n);
    k_scan_write<<<(uint32_t)ntiles, kScanBlock, 0, s>>>(esz, n, d_bs, d_bc, d_P, d_C);
  } else {
    MHIP(hipMemsetAsync(d_P, 0, 8, s));
  }
  // every segment stays on the device for k_repos: a second k_pack with room for all of them if needed
  uint32_t dev_cap = std::max<uint32_t>(seg_cap, 64);
  Tail tail;
  uint64_t tot = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const uint64_t o_tail = 0, o_seg = align256(sizeof(Tail));
    rc = grow(&m->small, &m->small_bytes, o_seg + sizeof(ldb_merge_segment) * ((uint64_t)dev_cap + 1));
    if (rc != LDB_OK) return rc;
    Tail* d_tail = reinterpret_cast<Tail*>(m->small + o_tail);
    ldb_merge_segment* d_segs = reinterpret_cast<ldb_merge_segment*>(m->small + o_seg);
    k_pack<<<1, 64, 0, s>>>(d_P, nullptr, n, active_fid, active_off, max_file_size, d_segs, dev_cap + 1, d_tail);
    MHIP(hipGetLastError());
    MHIP(hipMemcpyAsync(&tot, d_P + n, 8, hipMemcpyDeviceToHost, s));
    MHIP(hipMemcpyAsync(&tail, d_tail, sizeof(Tail), hipMemcpyDeviceToHost, s));
    MHIP(hipStreamSynchronize(s));
    if (tail.n_segments <= dev_cap + 1) {
      if (n && d_pos) {
        k_repos<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(n, d_P, d_segs, tail.n_segments, d_pos);
        MHIP(hipGetLastError());
      }
      if (h_segs && tail.n_segments)
        MHIP(hipMemcpyAsync(h_segs, d_segs, sizeof(ldb_merge_segment) * std::min(tail.n_segments, seg_cap),
                            hipMemcpyDeviceToHost, s));
      MHIP(hipStreamSynchronize(s));
      break;
    }
    dev_cap = tail.n_segments;
  }
  h_result->emit_bytes = tot;
  h_result->end_fid = tail.end_fid;
  h_result->end_off = tail.end_off;
  h_result->n_segments = tail.n_segments;
  if (h_segs && tail.n_segments > seg_cap) return h_result->status = LDB_ERR_CAPACITY;
  h_result->status = LDB_OK;
  return LDB_OK;
}

extern "C" int ldb_merge_timing(ldb_ctx* ctx, double* scan_ms, double* live_ms, double* compact_ms) {
  if (!ctx) return LDB_ERR_ARG;
  MergeWs* m = static_cast<MergeWs*>(*ldb_ctx_merge_slot_(ctx));
  if (!m) return LDB_ERR_ARG;
  if (scan_ms) *scan_ms = m->t_scan;
  if (live_ms) *live_ms = m->t_live;
  if (compact_ms) *compact_ms = m->t_compact;
  return LDB_OK;
}
