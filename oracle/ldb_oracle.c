/*
 * ldb_oracle.c — CPU restatement of LazyDB's log codec + replay scan.
 * TEST INFRASTRUCTURE ONLY (see ldb_oracle.h). Every function cites the
 * reference file:line it restates (paths relative to kakosute/lazydb @ v1).
 */
#define _GNU_SOURCE
#include "ldb_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------ CRC-32/IEEE
 * hash/crc32 IEEE: reflected polynomial 0xEDB88320, crc32.Update(crc, tab, p)
 * = ~reg(~crc, p). Slicing-by-8 (the same algorithm class as Go's amd64
 * fallback path for short inputs). */
static uint32_t crc_tab[8][256];
static int crc_ready = 0;

static void crc_init_tables(void) {
  if (crc_ready) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    crc_tab[0][i] = c;
  }
  for (int j = 1; j < 8; ++j)
    for (int i = 0; i < 256; ++i) crc_tab[j][i] = (crc_tab[j - 1][i] >> 8) ^ crc_tab[0][crc_tab[j - 1][i] & 0xff];
  crc_ready = 1;
}

/* Carry-less-multiply folding (PCLMULQDQ), the algorithm class of Go's amd64 hash/crc32 IEEE path
 * for inputs of 64 bytes and more (ieeeCLMUL): four 128-bit lanes folded by x^512, then by x^128,
 * reduced to 64 bits and Barrett-reduced to the 32-bit register (Gopal et al., "Fast CRC computation
 * for generic polynomials using PCLMULQDQ", bit-reflected constants of the IEEE polynomial).
 * Operates on the raw register like ldbo_crc32_reg; n >= 64, processes n & ~15 bytes. */
#if defined(__x86_64__)
#include <immintrin.h>
#include <stdio.h>
__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_clmul(uint32_t crc, const uint8_t* buf, size_t len) {
  const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596ll, 0x0154442bd4ll);
  const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009ell, 0x01751997d0ll);
  const __m128i k5k0 = _mm_set_epi64x(0, 0x0163cd6124ll);
  const __m128i poly = _mm_set_epi64x(0x01f7011641ll, 0x01db710641ll);
  __m128i x0, x1, x2, x3, x4, x5, x6, x7, x8;
  x1 = _mm_loadu_si128((const __m128i*)(buf + 0x00));
  x2 = _mm_loadu_si128((const __m128i*)(buf + 0x10));
  x3 = _mm_loadu_si128((const __m128i*)(buf + 0x20));
  x4 = _mm_loadu_si128((const __m128i*)(buf + 0x30));
  x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
  x0 = k1k2;
  buf += 64;
  len -= 64;
  while (len >= 64) {   /* fold 4 x 128 bits by x^512 */
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x6 = _mm_clmulepi64_si128(x2, x0, 0x00);
    x7 = _mm_clmulepi64_si128(x3, x0, 0x00);
    x8 = _mm_clmulepi64_si128(x4, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x11);
    x3 = _mm_clmulepi64_si128(x3, x0, 0x11);
    x4 = _mm_clmulepi64_si128(x4, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128((const __m128i*)(buf + 0x00)));
    x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128((const __m128i*)(buf + 0x10)));
    x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128((const __m128i*)(buf + 0x20)));
    x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128((const __m128i*)(buf + 0x30)));
    buf += 64;
    len -= 64;
  }
  x0 = k3k4;   /* fold the four lanes into one by x^128 */
  x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
  x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x2), x5);
  x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
  x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x3), x5);
  x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
  x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x4), x5);
  while (len >= 16) {
    x2 = _mm_loadu_si128((const __m128i*)buf);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x11), x2), x5);
    buf += 16;
    len -= 16;
  }
  /* 128 -> 64 bits */
  x2 = _mm_clmulepi64_si128(x1, x0, 0x10);
  x3 = _mm_setr_epi32(~0, 0, ~0, 0);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2);
  x0 = k5k0;
  x2 = _mm_srli_si128(x1, 4);
  x1 = _mm_and_si128(x1, x3);
  x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, x0, 0x00), x2);
  /* Barrett reduction to 32 bits */
  x0 = poly;
  x2 = _mm_and_si128(x1, x3);
  x2 = _mm_clmulepi64_si128(x2, x0, 0x10);
  x2 = _mm_and_si128(x2, x3);
  x2 = _mm_clmulepi64_si128(x2, x0, 0x00);
  x1 = _mm_xor_si128(x1, x2);
  return (uint32_t)_mm_extract_epi32(x1, 1);
}
static int clmul_ok = -1;
#endif

/* Slicing-by-8 only (the fold path off): the independent second formulation the tests compare. */
uint32_t ldbo_crc32_reg_tables(uint32_t c, const uint8_t* p, size_t n);

uint32_t ldbo_crc32_reg(uint32_t c, const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (clmul_ok < 0) clmul_ok = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  if (clmul_ok && n >= 64) {
    const size_t m = n & ~(size_t)15;
    c = crc_clmul(c, p, m);
    p += m;
    n -= m;
  }
#endif
  return ldbo_crc32_reg_tables(c, p, n);
}

uint32_t ldbo_crc32_reg_tables(uint32_t c, const uint8_t* p, size_t n) {
  crc_init_tables();
  while (n && ((uintptr_t)p & 7)) {
    c = crc_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    --n;
  }
  while (n >= 8) {
    uint32_t a, b;
    memcpy(&a, p, 4);
    memcpy(&b, p + 4, 4);
    a ^= c;
    c = crc_tab[7][a & 0xff] ^ crc_tab[6][(a >> 8) & 0xff] ^ crc_tab[5][(a >> 16) & 0xff] ^ crc_tab[4][a >> 24] ^
        crc_tab[3][b & 0xff] ^ crc_tab[2][(b >> 8) & 0xff] ^ crc_tab[1][(b >> 16) & 0xff] ^ crc_tab[0][b >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = crc_tab[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c;
}

uint32_t ldbo_crc32_update(uint32_t crc, const uint8_t* p, size_t n) { return ~ldbo_crc32_reg(~crc, p, n); }

/* ------------------------------------------------------------------ varints
 * encoding/binary (Go 1.18) varint.go: Uvarint returns (0, 0) if the buffer is
 * too short, (0, -(i+1)) on 64-bit overflow (the 11th byte, or a 10th byte > 1). */
int ldbo_uvarint(const uint8_t* buf, size_t len, uint64_t* out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (size_t i = 0; i < len; ++i) {
    if (i == 10) { *out = 0; return -(int)(i + 1); }
    uint8_t b = buf[i];
    if (b < 0x80) {
      if (i == 9 && b > 1) { *out = 0; return -(int)(i + 1); }
      *out = x | ((uint64_t)b << s);
      return (int)(i + 1);
    }
    x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  *out = 0;
  return 0;
}

int ldbo_varint(const uint8_t* buf, size_t len, int64_t* out) {
  uint64_t ux;
  int n = ldbo_uvarint(buf, len, &ux);
  int64_t x = (int64_t)(ux >> 1);
  if (ux & 1) x = ~x;
  *out = x;
  return n;
}

int ldbo_put_varint(uint8_t* buf, int64_t x) {
  uint64_t ux = (uint64_t)x << 1;
  if (x < 0) ux = ~ux;
  int i = 0;
  while (ux >= 0x80) {
    buf[i++] = (uint8_t)ux | 0x80;
    ux >>= 7;
  }
  buf[i++] = (uint8_t)ux;
  return i;
}

int ldbo_varint_len(int64_t x) {
  uint8_t tmp[10];
  return ldbo_put_varint(tmp, x);
}

/* ------------------------------------------------------------------ codec */
/* logfile/log_entry.go:48-78 EncodeEntry */
size_t ldbo_encode_entry(uint8_t stat, int64_t expired_at, uint64_t tx_id, uint16_t tx_stat, const uint8_t* key,
                         uint32_t klen, const uint8_t* val, uint32_t vlen, uint8_t* out) {
  size_t off = 5;
  out[4] = stat;                                             /* :54 */
  off += ldbo_put_varint(out + off, expired_at);             /* :57 */
  off += ldbo_put_varint(out + off, (int64_t)tx_id);         /* :59 */
  off += ldbo_put_varint(out + off, (int64_t)tx_stat);       /* :61 */
  off += ldbo_put_varint(out + off, (int64_t)klen);          /* :63 */
  off += ldbo_put_varint(out + off, (int64_t)vlen);          /* :65 */
  if (klen) memcpy(out + off, key, klen);                    /* :72 */
  if (vlen) memcpy(out + off + klen, val, vlen);             /* :73 */
  size_t size = off + klen + vlen;                           /* :68 */
  uint32_t crc = ldbo_crc32_update(0, out + 4, size - 4);    /* :75 ChecksumIEEE(newBuf[4:]) */
  out[0] = (uint8_t)crc;                                     /* :76 LittleEndian.PutUint32 */
  out[1] = (uint8_t)(crc >> 8);
  out[2] = (uint8_t)(crc >> 16);
  out[3] = (uint8_t)(crc >> 24);
  return size;
}

/* logfile/log_entry.go:81-107 decodeHeader on the 38-byte window of log_file.go:117.
 * Go evaluates buf[offset:] before each Varint: a negative offset panics. */
int ldbo_decode_header(const uint8_t* win, ldbo_header* h) {
  memset(h, 0, sizeof(*h));
  h->crc = (uint32_t)win[0] | ((uint32_t)win[1] << 8) | ((uint32_t)win[2] << 16) | ((uint32_t)win[3] << 24); /* :86 */
  h->stat = win[4];                                                                                          /* :87 */
  int off = 5;
  int64_t v[5];
  for (int f = 0; f < 5; ++f) {
    if (off < 0) return LDB_ERR_MALFORMED; /* buf[offset:] with offset < 0 */
    int n = ldbo_varint(win + off, (size_t)(LDBO_MAX_HEADER - off), &v[f]);
    off += n;
  }
  h->expired_at = v[0];           /* :91 */
  h->tx_id = (uint64_t)v[1];      /* :94 */
  h->tx_stat = (uint16_t)v[2];    /* :97 */
  h->k_size = (uint32_t)v[3];     /* :100 */
  h->v_size = (uint32_t)v[4];     /* :103 */
  h->size = off;                  /* :106 */
  /* the header EncodeEntry would re-emit (index.go:20 uses its length) */
  h->enc_size = 5 + ldbo_varint_len(h->expired_at) + ldbo_varint_len((int64_t)h->tx_id) +
                ldbo_varint_len((int64_t)h->tx_stat) + ldbo_varint_len((int64_t)h->k_size) +
                ldbo_varint_len((int64_t)h->v_size);
  return LDB_OK;
}

/* IOController read-bound rules (iocontroller/fileio.go:35-37 via os.File.ReadAt;
 * iocontroller/mmap.go:46-52). Returns 1 if Read(b, off) with len(b)=n fails with EOF. */
static int read_eof(uint64_t len, int io_type, int64_t off, uint64_t n) {
  if (io_type == LDB_IO_MMAP) {
    if (off < 0 || (uint64_t)off >= len || (uint64_t)off + n >= len) return 1; /* mmap.go:48 */
    return 0;
  }
  return (uint64_t)off + n > len; /* ReadAt short read -> io.EOF */
}

/* logfile/log_file.go:116-145 ReadLogEntry */
int ldbo_read_log_entry(const uint8_t* img, uint64_t len, int io_type, uint64_t off, ldbo_header* h,
                        uint64_t* entry_size) {
  /* :117-122 headerBuf := make([]byte, MaxHeaderSize); Read(headerBuf, offset) */
  if (read_eof(len, io_type, (int64_t)off, LDBO_MAX_HEADER)) return LDB_EOF_WINDOW;
  /* :123 decodeHeader */
  if (ldbo_decode_header(img + off, h) != LDB_OK) return LDB_ERR_MALFORMED;
  /* :124-126 zero sentinel */
  if (h->crc == 0 && h->k_size == 0 && h->v_size == 0) return LDB_EOF_SENTINEL;
  int64_t size = h->size;
  uint64_t kv = (uint64_t)h->k_size + (uint64_t)h->v_size;
  /* :130-139 read k+v at offset+size */
  if (h->k_size > 0 || h->v_size > 0) {
    int64_t at = (int64_t)off + size;
    if (io_type == LDB_IO_FILEIO && at < 0) return LDB_ERR_MALFORMED; /* ReadAt: "negative offset" (not io.EOF) */
    if (read_eof(len, io_type, at, kv)) return LDB_EOF_KV;
  }
  /* :141-143 getEntryCrc(headerBuf[:size], le) (log_entry.go:110-121) */
  if (size < 0) return LDB_ERR_MALFORMED; /* headerBuf[:size] panics */
  uint32_t crc = 0;
  if (size > 4) crc = ldbo_crc32_update(0, img + off + 4, (size_t)(size - 4) + kv); /* buf[4:] ++ Key ++ Value */
  if (crc != h->crc) return LDB_ERR_CRC;
  *entry_size = (uint64_t)(size + (int64_t)kv); /* :128 entrySize = size + kSize + vSize */
  return LDB_OK;
}

static void emit(void* out, int tuple_kind, uint64_t idx, uint64_t off, const ldbo_header* h, uint32_t fid) {
  if (tuple_kind == LDB_TUPLE_ENTRY) {
    ldb_entry* e = (ldb_entry*)out + idx;
    memset(e, 0, sizeof(*e));
    e->offset = off;
    e->expired_at = h->expired_at;
    e->tx_id = h->tx_id;
    e->crc = h->crc;
    e->k_size = h->k_size;
    e->v_size = h->v_size;
    e->tx_stat = h->tx_stat;
    e->stat = h->stat;
    e->hdr_size = (uint8_t)h->size;
    e->enc_hdr_size = (uint8_t)h->enc_size;
    e->fid = fid;
  } else {
    ldb_index_tuple* t = (ldb_index_tuple*)out + idx;
    t->pos = (off & 0xFFFFFFFFFFull) | ((uint64_t)(h->size & 0x3F) << 40) | ((uint64_t)(h->enc_size & 0x3F) << 46) |
             ((uint64_t)h->stat << 52);
    t->k_size = h->k_size;
    t->v_size = h->v_size;
  }
}

/* index.go:84-95: offset := 0; for { ReadLogEntry(offset); EOF -> break; err -> fatal; offset += entSize } */
int ldbo_scan(const uint8_t* img, uint64_t len, int io_type, uint32_t fid, int tuple_kind, void* out, uint64_t cap,
              ldb_scan_result* res) {
  uint64_t off = 0, n = 0;
  int st;
  for (;;) {
    ldbo_header h;
    uint64_t es = 0;
    st = ldbo_read_log_entry(img, len, io_type, off, &h, &es);
    if (st != LDB_OK) break;
    if (out && n < cap) emit(out, tuple_kind, n, off, &h, fid);
    ++n;
    off += es;
  }
  memset(res, 0, sizeof(*res));
  res->status = (out && n > cap) ? LDB_ERR_CAPACITY : st;
  res->fid = fid;
  res->n_entries = n;
  res->end_off = off;
  return LDB_OK;
}

/* The per-entry work of the reference replay, restated with the same system calls
 * and allocations: log_file.go:117 make+Read(38), :132 make+Read(k+v),
 * :141 getEntryCrc, index.go:20 EncodeEntry (a second allocation + CRC pass). */
static int faithful_read(int fd, uint64_t len, int io_type, int64_t off, uint8_t* buf, uint64_t n) {
  if (read_eof(len, io_type, off, n)) return LDB_EOF_WINDOW;
  uint64_t got = 0;
  while (got < n) {
    ssize_t r = pread(fd, buf + got, n - got, off + (int64_t)got);
    if (r <= 0) return LDB_EOF_WINDOW;
    got += (uint64_t)r;
  }
  return LDB_OK;
}

int ldbo_scan_faithful(int fd, uint64_t len, int io_type, uint32_t fid, ldb_index_tuple* out, uint64_t cap,
                       ldb_scan_result* res) {
  uint64_t off = 0, n = 0;
  int st = LDB_OK;
  for (;;) {
    uint8_t* hdr = (uint8_t*)malloc(LDBO_MAX_HEADER);
    if (faithful_read(fd, len, io_type, (int64_t)off, hdr, LDBO_MAX_HEADER) != LDB_OK) {
      free(hdr);
      st = LDB_EOF_WINDOW;
      break;
    }
    ldbo_header h;
    if (ldbo_decode_header(hdr, &h) != LDB_OK) { free(hdr); st = LDB_ERR_MALFORMED; break; }
    if (h.crc == 0 && h.k_size == 0 && h.v_size == 0) { free(hdr); st = LDB_EOF_SENTINEL; break; }
    uint64_t kv = (uint64_t)h.k_size + h.v_size;
    uint8_t* kvb = NULL;
    if (kv) {
      int64_t at = (int64_t)off + h.size;
      if (io_type == LDB_IO_FILEIO && at < 0) { free(hdr); st = LDB_ERR_MALFORMED; break; }
      if (read_eof(len, io_type, at, kv)) { free(hdr); st = LDB_EOF_KV; break; }
      kvb = (uint8_t*)malloc(kv);
      if (faithful_read(fd, len, io_type, at, kvb, kv) != LDB_OK) { free(hdr); free(kvb); st = LDB_EOF_KV; break; }
    }
    if (h.size < 0) { free(hdr); free(kvb); st = LDB_ERR_MALFORMED; break; }
    uint32_t crc = 0;
    if (h.size > 4) {
      crc = ldbo_crc32_update(0, hdr + 4, (size_t)h.size - 4);
      crc = ldbo_crc32_update(crc, kvb, h.k_size);
      crc = ldbo_crc32_update(crc, kvb ? kvb + h.k_size : NULL, h.v_size);
    }
    if (crc != h.crc) { free(hdr); free(kvb); st = LDB_ERR_CRC; break; }
    /* index.go:15-26 buildStrIndex: SDelete -> Delete(key); else size from EncodeEntry */
    if (h.stat != 1) {
      uint8_t* enc = (uint8_t*)malloc(LDBO_MAX_HEADER + kv);
      size_t es = ldbo_encode_entry(h.stat, h.expired_at, h.tx_id, h.tx_stat, kvb, h.k_size,
                                    kvb ? kvb + h.k_size : NULL, h.v_size, enc);
      if ((int)es - (int)kv != h.enc_size) { free(enc); free(hdr); free(kvb); st = LDB_ERR_MALFORMED; break; }
      free(enc);
    }
    if (out && n < cap) emit(out, LDB_TUPLE_INDEX, n, off, &h, fid);
    ++n;
    off += (uint64_t)(h.size + (int64_t)kv);
    free(hdr);
    free(kvb);
  }
  memset(res, 0, sizeof(*res));
  res->status = st;
  res->fid = fid;
  res->n_entries = n;
  res->end_off = off;
  return LDB_OK;
}

/* ------------------------------------------------------------------ generator */
uint64_t ldbo_splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static const char kAlphabet[] = "0123456789abcdefghijklmnopqrstuvwxyz"; /* bench/db_bench_test.go:21-27 */

uint64_t ldbo_gen_log(uint8_t* img, uint64_t cap_bytes, uint64_t seed, uint32_t ksize, uint32_t vsize,
                      int value_mode, double zipf_s, uint32_t zipf_max, uint64_t max_entries, uint64_t* end_off) {
  uint64_t st = seed;
  double* cdf = NULL;
  if (value_mode == 1) {
    cdf = (double*)malloc(sizeof(double) * zipf_max);
    double acc = 0;
    for (uint32_t r = 1; r <= zipf_max; ++r) {
      acc += pow((double)r, -zipf_s);
      cdf[r - 1] = acc;
    }
    for (uint32_t r = 0; r < zipf_max; ++r) cdf[r] /= acc;
  }
  uint32_t vmax = value_mode == 1 ? 16u * zipf_max : vsize;
  uint8_t* key = (uint8_t*)malloc(ksize + 32);
  uint8_t* val = (uint8_t*)malloc(vmax + 8);
  uint64_t off = 0, n = 0;
  for (; n < max_entries; ++n) {
    uint32_t vl = vsize;
    if (value_mode == 1) {
      double u = (double)(ldbo_splitmix64(&st) >> 11) * (1.0 / 9007199254740992.0);
      uint32_t lo = 0, hi = zipf_max - 1;
      while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        if (cdf[mid] < u) lo = mid + 1; else hi = mid;
      }
      vl = 16u * (lo + 1);
    }
    /* key "key-" + zero-padded decimal n, exactly ksize bytes */
    char num[32];
    int nd = 0;
    uint64_t t = n;
    do { num[nd++] = (char)('0' + t % 10); t /= 10; } while (t);
    memset(key, '0', ksize);
    if (ksize >= 4) memcpy(key, "key-", 4);
    for (int i = 0; ksize >= 4 && i < nd && (uint32_t)i < ksize - 4; ++i) key[ksize - 1 - i] = (uint8_t)num[i];
    for (uint32_t i = 0; i < vl; i += 8) {
      uint64_t r = ldbo_splitmix64(&st);
      for (int b = 0; b < 8 && i + b < vl; ++b) { val[i + b] = (uint8_t)kAlphabet[(r & 0xff) % 36]; r >>= 8; }
    }
    uint64_t need = 5 + ldbo_varint_len(0) * 3 + ldbo_varint_len(ksize) + ldbo_varint_len(vl) + ksize + vl;
    if (off + need > cap_bytes) break; /* db.go:485 rollover: the entry goes to the next file */
    off += ldbo_encode_entry(0, 0, 0, 0, key, ksize, val, vl, img + off);
  }
  free(key);
  free(val);
  free(cdf);
  if (end_off) *end_off = off;
  return n;
}

/* The reference benchmark's own log (bench/db_bench_test.go:17-36, configs[0]): n Sets of
 * GetKey(i) = "bench_test_key_" + decimal i (16..21 bytes as i grows: the entry size changes at
 * i = 10, 100, 1000, ...) and GetValue() = vsize bytes drawn from the 36-char alphabet (:15, :21-27;
 * math/rand is time-seeded there, so the draws are splitmix64 here), each written by Set (str.go:22-33 ->
 * writeLogEntry -> EncodeEntry, db.go:473-523) into one preallocated file of cap_bytes (the Mmap
 * IOController truncates the file to MaxLogFileSize, iocontroller/mmap.go:17-30, so the bytes past the
 * last entry are zero). Stops early when the file would roll over (db.go:485). */
uint64_t ldbo_gen_bench_log(uint8_t* img, uint64_t cap_bytes, uint64_t seed, uint64_t n_entries, uint32_t vsize,
                            uint64_t* end_off) {
  static const char alpha[] = "abcdefghijklmnopqrstuvwxyz0123456789"; /* bench/db_bench_test.go:15 */
  uint64_t st = seed, off = 0, n = 0;
  uint8_t* val = (uint8_t*)malloc(vsize + 8);
  char key[48];
  for (; n < n_entries; ++n) {
    int kl = snprintf(key, sizeof key, "bench_test_key_%llu", (unsigned long long)n); /* :17-19 */
    for (uint32_t i = 0; i < vsize; i += 8) {
      uint64_t r = ldbo_splitmix64(&st);
      for (int b = 0; b < 8 && i + b < vsize; ++b) { val[i + b] = (uint8_t)alpha[(r & 0xff) % 36]; r >>= 8; }
    }
    uint64_t need = 5 + 3 + ldbo_varint_len(kl) + ldbo_varint_len(vsize) + (uint64_t)kl + vsize;
    if (off + need > cap_bytes) break;
    off += ldbo_encode_entry(0, 0, 0, 0, (const uint8_t*)key, (uint32_t)kl, val, vsize, img + off);
  }
  free(val);
  if (end_off) *end_off = off;
  return n;
}

/* A writer-realistic string-type log: what LazyDB's own write paths append, interleaved.
 *   Set / MSet / Append        str.go:26, :200, :266        stat 0, ExpiredAt 0, TxID 0, TxStat 0
 *   SetEX                      str.go:161-162               ExpiredAt = now + duration (Unix seconds)
 *   Delete / GetDel            str.go:111, :136             Stat = SDelete, no value
 *   Tx.Commit of a Tx.Set      tx_str.go:8-9, tx.go:157-160 TxStat = TxCommited (TxID stays 0: no write
 *                                                           path sets it)
 * Keys "user:" + decimal id (ids < key_space, so keys repeat as a live database's do); values of
 * 8..vmax bytes, log-uniform; mix in parts per 1000: set, setex, del, tx (the rest: set). */
uint64_t ldbo_gen_writer_log(uint8_t* img, uint64_t cap_bytes, uint64_t seed, uint64_t max_entries, int64_t now,
                             uint32_t key_space, uint32_t vmax, uint32_t p_setex, uint32_t p_del, uint32_t p_tx,
                             uint64_t* end_off) {
  uint64_t st = seed, off = 0, n = 0;
  uint8_t* val = (uint8_t*)malloc(vmax + 8);
  char key[48];
  double lmax = log((double)vmax / 8.0);
  for (; n < max_entries; ++n) {
    uint64_t r0 = ldbo_splitmix64(&st);
    uint32_t kind = (uint32_t)(r0 % 1000);
    uint32_t id = (uint32_t)((r0 >> 16) % key_space);
    int kl = snprintf(key, sizeof key, "user:%u", id);
    uint8_t stat = 0;
    int64_t expa = 0;
    uint16_t ts = 0;
    uint32_t vl;
    if (kind < p_del) {
      stat = 1; vl = 0; /* SDelete */
    } else {
      double u = (double)(ldbo_splitmix64(&st) >> 11) * (1.0 / 9007199254740992.0);
      vl = (uint32_t)(8.0 * exp(u * lmax));
      if (vl < 8) vl = 8;
      if (vl > vmax) vl = vmax;
      if (kind < p_del + p_setex) expa = now + 1 + (int64_t)((r0 >> 40) % 86400); /* time.Now().Add(d).Unix() */
      else if (kind < p_del + p_setex + p_tx) ts = 1;                             /* logfile.TxCommited */
      for (uint32_t i = 0; i < vl; i += 8) {
        uint64_t r = ldbo_splitmix64(&st);
        memcpy(val + i, &r, 8);
      }
    }
    uint64_t need = 5 + ldbo_varint_len(expa) + 1 + ldbo_varint_len(ts) + ldbo_varint_len(kl) + ldbo_varint_len(vl) +
                    (uint64_t)kl + vl;
    if (off + need > cap_bytes) break;
    off += ldbo_encode_entry(stat, expa, 0, ts, (const uint8_t*)key, (uint32_t)kl, val, vl, img + off);
  }
  free(val);
  if (end_off) *end_off = off;
  return n;
}

/* ================================================================== merge / GC
 * Restates, for the string value type:
 *   index.go:68-95 + :15-26  replay in (fid, offset) order: SDelete -> idxTree.Delete(key), else Put
 *   db.go:383-427            Merge over the target files in ascending fid (discard.go:224 sorts the ccl):
 *                            ReadLogEntry loop; skip SDelete (:403); skip ExpiredAt != 0 && <= now (:406)
 *   db.go:243-265            mergeStr: rewrite iff index[key] == (fid, offset); then updateIndexTree
 *   db.go:473-523            writeLogEntry: EncodeEntry; rollover when Offset + size > MaxLogFileSize
 * The index is an open-addressing map keyed by the full key bytes (FNV-1a): value = record id of the
 * key's current index entry, -1 after Delete, -2 once rewritten to a new position. */
typedef struct { const uint8_t* key; uint32_t klen; int64_t val; } mapent;
typedef struct { mapent* t; uint64_t mask; } kmap;

static uint64_t fnv1a(const uint8_t* p, uint32_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
  return h;
}

static mapent* kmap_find(kmap* m, const uint8_t* key, uint32_t klen, int create) {
  uint64_t i = fnv1a(key, klen) & m->mask;
  for (;;) {
    mapent* e = &m->t[i];
    if (!e->key) {
      if (!create) return NULL;
      e->key = key ? key : (const uint8_t*)"";
      e->klen = klen;
      e->val = -1;
      return e;
    }
    if (e->klen == klen && (klen == 0 || memcmp(e->key, key, klen) == 0)) return e;
    i = (i + 1) & m->mask;
  }
}

int ldbo_merge(int n_files, const ldb_merge_file* files, int io_type, uint32_t active_fid, uint64_t active_off,
               uint64_t max_size, int64_t now, uint8_t* stream, uint64_t stream_cap, ldb_merge_pos* pos,
               uint64_t pos_cap, ldb_merge_segment* segs, uint32_t seg_cap, uint8_t* live, uint64_t live_cap,
               ldb_merge_file_stat* stats, ldb_merge_result* res) {
  memset(res, 0, sizeof(*res));
  res->bad_file = -1;
  res->end_fid = active_fid;
  res->end_off = active_off;
  /* 1. replay every file (index.go:84-95) into one record table */
  uint64_t cap = 0;
  for (int i = 0; i < n_files; ++i) cap += files[i].len / 10 + 2;
  ldb_entry* recs = (ldb_entry*)malloc(sizeof(ldb_entry) * (cap ? cap : 1));
  uint32_t* rfile = (uint32_t*)malloc(sizeof(uint32_t) * (cap ? cap : 1));
  uint64_t n = 0;
  for (int i = 0; i < n_files; ++i) {
    ldb_scan_result r;
    ldbo_scan(files[i].d_image, files[i].len, io_type, files[i].fid, LDB_TUPLE_ENTRY, recs + n, cap - n, &r);
    if (stats) {
      memset(&stats[i], 0, sizeof(stats[i]));
      stats[i].status = r.status;
      stats[i].fid = files[i].fid;
      stats[i].n_entries = r.n_entries;
      stats[i].end_off = r.end_off;
    }
    if (r.status < 0) {
      res->status = r.status;
      res->bad_file = i;
      res->n_records = n + r.n_entries;
      free(recs);
      free(rfile);
      return r.status;
    }
    for (uint64_t j = 0; j < r.n_entries; ++j) rfile[n + j] = (uint32_t)i;
    n += r.n_entries;
  }
  res->n_records = n;
  kmap m;
  uint64_t tc = 1024;
  while (tc < 2 * n) tc <<= 1;
  m.t = (mapent*)calloc(tc, sizeof(mapent));
  m.mask = tc - 1;
#define KEY(s) (files[rfile[s]].d_image + recs[s].offset + recs[s].hdr_size)
  /* buildStrIndex (index.go:15-26) */
  for (uint64_t s = 0; s < n; ++s) {
    mapent* e = kmap_find(&m, KEY(s), recs[s].k_size, 1);
    e->val = recs[s].stat == 1 ? -1 : (int64_t)s; /* SDelete: Delete(key); else Put */
  }
  for (uint64_t s = 0; s < n; ++s) {
    int lv = kmap_find(&m, KEY(s), recs[s].k_size, 0)->val == (int64_t)s;
    if (live && s < live_cap) live[s] = (uint8_t)lv;
    if (lv) {
      res->n_live++;
      if (stats) {
        stats[rfile[s]].live_count++;
        stats[rfile[s]].live_bytes += (uint64_t)recs[s].enc_hdr_size + recs[s].k_size + recs[s].v_size;
      }
    }
  }
  /* 2. Merge (db.go:383-427) with writeLogEntry (db.go:473-523) */
  uint32_t fid = active_fid;
  uint64_t off = active_off, sp = 0, ne = 0;
  uint32_t ns = 0;
  uint8_t* buf = NULL;
  size_t bufcap = 0;
  int over = (live && live_cap < n);
  for (uint64_t s = 0; s < n; ++s) {
    const ldb_entry* e = &recs[s];
    if (!files[rfile[s]].is_target) continue;
    if (e->stat == 1) continue;                                  /* :403 */
    if (e->expired_at != 0 && e->expired_at <= now) continue;    /* :406-409 */
    mapent* me = kmap_find(&m, KEY(s), e->k_size, 0);
    if (me->val != (int64_t)s) continue;                         /* mergeStr :255 */
    size_t need = LDBO_MAX_HEADER + (size_t)e->k_size + e->v_size;
    if (need > bufcap) {
      bufcap = need * 2;
      buf = (uint8_t*)realloc(buf, bufcap);
    }
    const uint8_t* k = KEY(s);
    size_t size = ldbo_encode_entry(e->stat, e->expired_at, e->tx_id, e->tx_stat, k, e->k_size, k + e->k_size,
                                    e->v_size, buf);                 /* :482 EncodeEntry */
    if (off + size > max_size) {                                 /* :485 rollover */
      fid += 1;
      off = 0;
    }
    if (ns == 0 || segs == NULL || ns > seg_cap || segs[ns - 1].fid != fid ||
        segs[ns - 1].file_off + segs[ns - 1].n_bytes != off) {
      if (segs && ns < seg_cap) {
        segs[ns].fid = fid;
        segs[ns].reserved_ = 0;
        segs[ns].file_off = off;
        segs[ns].stream_off = sp;
        segs[ns].n_bytes = 0;
      }
      ++ns;
    }
    if (segs && ns <= seg_cap) segs[ns - 1].n_bytes += size;
    if (stream && sp + size <= stream_cap) memcpy(stream + sp, buf, size);
    else over = 1;
    if (pos && ne < pos_cap) {
      pos[ne].offset = off;
      pos[ne].fid = fid;
      pos[ne].entry_size = (uint32_t)size;
      pos[ne].src_offset = e->offset;
      pos[ne].src_file = rfile[s];
      pos[ne].reserved_ = 0;
    } else {
      over = 1;
    }
    me->val = -2;                                                /* updateIndexTree: new position */
    ++ne;
    sp += size;
    off += size;
  }
#undef KEY
  free(buf);
  free(m.t);
  free(recs);
  free(rfile);
  res->n_emit = ne;
  res->emit_bytes = sp;
  res->end_fid = fid;
  res->end_off = off;
  res->n_segments = ns;
  if (over || ns > seg_cap) res->status = LDB_ERR_CAPACITY;
  return res->status;
}

/* Merge test set (BASELINE config 5 shape): n_records records of ksize-byte keys / vsize-byte values,
 * appended to consecutive files of cap_bytes with writeLogEntry's rollover rule (db.go:485); file f
 * is imgs + f*cap_bytes. Records are paired by a splitmix64(seed) Fisher-Yates permutation: pair i =
 * (perm[2i], perm[2i+1]) shares key i, so each key is written twice and exactly half the records are
 * stale. With probability p_delete_ppm/1e6 a pair's later record is an SDelete (empty value); with
 * p_expire_ppm/1e6 a record carries ExpiredAt = now -/+ 1000 (half expired). Returns the records
 * written; end_offs[f] receives each file's append offset. */
uint64_t ldbo_gen_merge(uint8_t* imgs, uint32_t n_files, uint64_t cap_bytes, uint64_t n_records, uint64_t seed,
                        uint32_t ksize, uint32_t vsize, uint32_t p_delete_ppm, uint32_t p_expire_ppm, int64_t now,
                        uint64_t* end_offs) {
  uint64_t st = seed;
  n_records &= ~1ull;
  uint32_t* perm = (uint32_t*)malloc(sizeof(uint32_t) * (n_records ? n_records : 1));
  uint32_t* keyid = (uint32_t*)malloc(sizeof(uint32_t) * (n_records ? n_records : 1));
  uint8_t* later = (uint8_t*)calloc(n_records ? n_records : 1, 1);
  for (uint64_t i = 0; i < n_records; ++i) perm[i] = (uint32_t)i;
  for (uint64_t i = n_records; i > 1; --i) {
    uint64_t j = ldbo_splitmix64(&st) % i;
    uint32_t t = perm[i - 1];
    perm[i - 1] = perm[j];
    perm[j] = t;
  }
  for (uint64_t i = 0; i < n_records / 2; ++i) {
    uint32_t a = perm[2 * i], b = perm[2 * i + 1];
    keyid[a] = keyid[b] = (uint32_t)i;
    later[a > b ? a : b] = 1;
  }
  uint8_t* key = (uint8_t*)malloc(ksize + 32);
  uint8_t* val = (uint8_t*)malloc(vsize + 8);
  uint64_t off = 0, w = 0;
  uint32_t f = 0;
  for (uint32_t i = 0; i < n_files; ++i) end_offs[i] = 0;
  for (; w < n_records; ++w) {
    char num[32];
    int nd = 0;
    uint64_t t = keyid[w];
    do { num[nd++] = (char)('0' + t % 10); t /= 10; } while (t);
    memset(key, '0', ksize);
    if (ksize >= 4) memcpy(key, "key-", 4);
    for (int i = 0; ksize >= 4 && i < nd && (uint32_t)i < ksize - 4; ++i) key[ksize - 1 - i] = (uint8_t)num[i];
    uint8_t stat = 0;
    uint32_t vl = vsize;
    int64_t exp = 0;
    uint64_t r = ldbo_splitmix64(&st);
    if (later[w] && (r % 1000000) < p_delete_ppm) {
      stat = 1;
      vl = 0;
    }
    r = ldbo_splitmix64(&st);
    if ((r % 1000000) < p_expire_ppm) exp = (r >> 40) & 1 ? now - 1000 : now + 1000;
    for (uint32_t i = 0; i < vl; i += 8) {
      uint64_t x = ldbo_splitmix64(&st);
      for (int b = 0; b < 8 && i + b < vl; ++b) { val[i + b] = (uint8_t)kAlphabet[(x & 0xff) % 36]; x >>= 8; }
    }
    uint64_t need = 5 + ldbo_varint_len(exp) + 2 + ldbo_varint_len(ksize) + ldbo_varint_len(vl) + ksize + vl;
    if (off + need > cap_bytes) { /* db.go:485 rollover */
      end_offs[f] = off;
      if (++f >= n_files) break;
      off = 0;
    }
    off += ldbo_encode_entry(stat, exp, 0, 0, key, ksize, val, vl, imgs + (uint64_t)f * cap_bytes + off);
  }
  if (f < n_files) end_offs[f] = off;
  free(perm);
  free(keyid);
  free(later);
  free(key);
  free(val);
  return w;
}
