/* chunk_oracle.c -- CPU restatement of Shock's "chunkrecord" indexer.
 *
 * TEST INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline leg); never linked by the product.
 *
 * Restates (paths relative to /root/reference/shock-server/):
 *   node/file/index/chunkrecord.go:41-99   driver: curr = 0; n, er = SeekChunk(curr, true);
 *                                          row (curr, er == EOF ? size - curr : n); curr += n
 *   node/file/format/fastq/fastq.go:216-243 SeekChunk: 32 KiB window at curr + CHUNK - 32 KiB,
 *                                          end of the LAST `Record` match (FindAllIndex), else
 *                                          the FIRST match of the following windows
 *   node/file/format/fastq/fastq.go:23      Record = `@\S(.*)?[\n\r]+[A-Za-z\-]+[\n\r]+\+(.*)?[\n\r]+(\S+)[\n\r]+`
 *   node/file/format/fasta/fasta.go:143-173 SeekChunk on "\n>" (then "\r>") per window
 *   node/file/format/sam/sam.go:100-102     SeekChunk returns (0, nil): the Go driver never ends
 *   conf/conf.go:138                        CHUNK_SIZE = 1048576
 *
 * The Record regex is matched with Go regexp's leftmost-first semantics (the match a
 * backtracking engine finds first).  Its only choice points are where each `.*` stops (the
 * line's '\n' first, then every '\r' inside the line, right to left); every other quantifier
 * is forced to its maximal run because the class after it is disjoint from it.  `.` is any
 * byte but '\n'; \S is any byte outside RE2's \s = [\t\n\f\r ] (ASCII only, no \v), which is
 * byte-exact for UTF-8 input because no multi-byte rune contains an ASCII byte.
 * Pinned by tests/test_oracle_chunk.py against an independent restatement with Python's
 * backtracking `re` (same leftmost-first results) and hand-derived vectors.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "shockidx_oracle.h"

#define WIN 32768

static int is_nl(uint8_t c) { return c == '\n' || c == '\r'; }
static int is_sp(uint8_t c) { return c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == ' '; }
static int is_l(uint8_t c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '-'; }

/* From the end `a` of a `.*`: [\n\r]+ ... ; returns match end or -1. stage 0: after the header
 * `.*`: NL+ L+ NL+ '+' .* NL+ S+ NL+; stage 1: after the plus-line `.*`: NL+ S+ NL+. */
static long tail_match(const uint8_t *b, long n, long a, int stage) {
  long p = a;
  if (p >= n || !is_nl(b[p])) return -1;
  while (p < n && is_nl(b[p])) p++;
  if (stage == 0) {
    long q = p;
    while (q < n && is_l(b[q])) q++;
    if (q == p || q >= n || !is_nl(b[q])) return -1;
    while (q < n && is_nl(b[q])) q++;
    if (q >= n || b[q] != '+') return -1;
    /* plus-line `.*` from q+1: longest first ('\n' or end), then each '\r' right to left */
    long e = q + 1;
    while (e < n && b[e] != '\n') e++;
    for (long c = e; c >= q + 1; c--) {
      if (c < n && is_nl(b[c])) {
        long r = tail_match(b, n, c, 1);
        if (r >= 0) return r;
      }
    }
    return -1;
  }
  long q = p;
  while (q < n && !is_sp(b[q])) q++;
  if (q == p || q >= n || !is_nl(b[q])) return -1;
  while (q < n && is_nl(b[q])) q++;
  return q;
}

/* Leftmost-first match of Record anchored at s (b[s] must be '@'); returns the end or -1. */
long oracle_fq_record_at(const uint8_t *b, long n, long s) {
  if (s + 1 >= n || b[s] != '@' || is_sp(b[s + 1])) return -1;
  long e = s + 2;
  while (e < n && b[e] != '\n') e++;
  for (long c = e; c >= s + 2; c--) {
    if (c < n && is_nl(b[c])) {
      long r = tail_match(b, n, c, 0);
      if (r >= 0) return r;
    }
  }
  return -1;
}

/* FindIndex (first = 1) or the last match of FindAllIndex (first = 0) on b[0..n): end or -1 */
static long fq_find(const uint8_t *b, long n, int first) {
  long pos = 0, last = -1;
  while (pos < n) {
    const uint8_t *at = memchr(b + pos, '@', (size_t)(n - pos));
    if (!at) break;
    long s = at - b;
    long e = oracle_fq_record_at(b, n, s);
    if (e < 0) {
      pos = s + 1;
      continue;
    }
    if (first) return e;
    last = e;
    pos = e; /* non-overlapping; matches are never empty */
  }
  return last;
}

static long fa_find(const uint8_t *b, long n, int first) {
  long pos = -1;
  for (int k = 0; k < 2 && pos < 0; k++) { /* "\n>" then "\r>" (fasta.go:157-165) */
    uint8_t c = k == 0 ? '\n' : '\r';
    if (first) {
      for (long i = 0; i + 1 < n; i++)
        if (b[i] == c && b[i + 1] == '>') { pos = i; break; }
    } else {
      for (long i = n - 2; i >= 0; i--)
        if (b[i] == c && b[i + 1] == '>') { pos = i; break; }
    }
  }
  return pos;
}

/* SeekChunk(offSet, lastIndex) on the whole file image; *eof = 1 for io.EOF. */
static int64_t seek_chunk(const uint8_t *d, uint64_t size, int fmt, int64_t chunk, int64_t off, int last,
                          int *eof) {
  int64_t acc = 0;
  for (;;) {
    int64_t w = off + chunk - WIN; /* io.NewSectionReader(f, w, WIN).Read(buf) */
    if ((uint64_t)w + WIN > size) { /* short read (or a window past the end): EOF */
      *eof = 1;
      return acc + ((uint64_t)w < size ? (int64_t)(size - (uint64_t)w) : 0);
    }
    const uint8_t *b = d + w;
    if (fmt == ORC_FMT_FASTQ) {
      long e = fq_find(b, WIN, !last);
      if (e >= 0) {
        long pos = e < WIN - 1 ? e : WIN - 1; /* math.Min(loc[1], len(buf)-1) (fastq.go:241) */
        return acc + chunk - WIN + pos;
      }
    } else {
      long p = fa_find(b, WIN, !last);
      if (p >= 0) return acc + chunk - WIN + p + 1;
    }
    acc += WIN; /* recursion: winSize + SeekChunk(offSet + winSize, false) */
    off += WIN;
    last = 0;
  }
}

int oracle_chunkrecord(const uint8_t *data, size_t n, int fmt, int64_t chunk, uint64_t **rows, uint64_t *count,
                       char *err, size_t errlen) {
  *rows = NULL;
  *count = 0;
  if (fmt < 0) fmt = oracle_detect(data, n, NULL);
  if (fmt == ORC_FMT_NONE) { /* multi.SeekChunk -> DetermineFormat error, no row (chunkrecord.go:62-66) */
    if (err && errlen) {
      strncpy(err, "Invalid file type for filter", errlen - 1);
      err[errlen - 1] = 0;
    }
    return 1;
  }
  if (fmt == ORC_FMT_SAM) { /* sam.SeekChunk = (0, nil): rows (0,0) forever in Go */
    if (err && errlen) {
      strncpy(err, "chunkrecord: sam.SeekChunk never advances (reference loops forever)", errlen - 1);
      err[errlen - 1] = 0;
    }
    return 2;
  }
  if (chunk < WIN) return -1;
  uint64_t cap = n / (uint64_t)(chunk - WIN + 1) + 4, cnt = 0;
  uint64_t *r = malloc(cap * 16);
  if (!r) return -1;
  int64_t curr = 0;
  for (;;) {
    int eof = 0;
    int64_t m = seek_chunk(data, n, fmt, chunk, curr, 1, &eof);
    if (cnt == cap) {
      cap *= 2;
      uint64_t *t = realloc(r, cap * 16);
      if (!t) { free(r); return -1; }
      r = t;
    }
    r[2 * cnt] = (uint64_t)curr;
    r[2 * cnt + 1] = eof ? (uint64_t)((int64_t)n - curr) : (uint64_t)m;
    cnt++;
    curr += m;
    if (eof) break;
  }
  *rows = r;
  *count = cnt;
  return 0;
}

/* index/chunkrecord.go:100-228, a subset node whose format is not "matrix": the subset node's
 * record index (rows = (offset, length) pairs, `nrows` whole rows: ReadAt of a partial row
 * returns io.EOF and ends the loop, :144-150) grouped into chunks of record rows.  Literal
 * transcription of the loop; out rows = (parentOffset, parentLength) = (16 * first record,
 * 16 * records).  Returns 0, or -1 on allocation failure. */
int oracle_chunkrecord_subset(const uint64_t *ri, uint64_t nrows, uint64_t **rows, uint64_t *count) {
  const int64_t LIMIT = 1048576;  /* :170 */
  uint64_t cap = 64, k = 0;
  uint64_t *out = malloc(cap * 16);
  if (!out) return -1;
#define EMIT(o, l)                                                  \
  do {                                                              \
    if (k == cap) {                                                 \
      uint64_t *o2 = realloc(out, (cap *= 2) * 16);                 \
      if (!o2) { free(out); return -1; }                            \
      out = o2;                                                     \
    }                                                               \
    out[2 * k] = (uint64_t)(o);                                     \
    out[2 * k + 1] = (uint64_t)(l);                                 \
    k++;                                                            \
  } while (0)
  int64_t riCount = 0, parentOffset = 0, parentLength = 0, chunkRecordLength = 0;
  for (;;) {
    if ((uint64_t)riCount >= nrows) break;                   /* :146-153 io.EOF */
    const int64_t riLength = (int64_t)ri[2 * riCount + 1];   /* :156 */
    riCount += 1;
    if (chunkRecordLength == 0) {                           /* :159-164 */
      parentOffset = (riCount - 1) * 16;
      parentLength = 16;
    } else {
      parentLength += 16;
    }
    if (chunkRecordLength + riLength >= LIMIT) {            /* :167 */
      if (chunkRecordLength == 0) {                         /* :170-184 */
        EMIT(parentOffset, parentLength);
        chunkRecordLength = 0;
        parentLength = 0;
      } else {                                              /* :185-200 */
        EMIT(parentOffset, parentLength - 16);
        chunkRecordLength = riLength;
        parentOffset = (riCount - 1) * 16;
        parentLength = 16;
      }
    } else {
      chunkRecordLength += riLength;                        /* :204 */
    }
  }
  if (chunkRecordLength != 0) EMIT(parentOffset, parentLength); /* :209-216 */
#undef EMIT
  *rows = out;
  *count = k;
  return 0;
}
