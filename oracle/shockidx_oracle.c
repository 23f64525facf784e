/* shockidx_oracle.c -- CPU restatement of Shock's record/line indexers.
 * TEST INFRASTRUCTURE ONLY (see shockidx_oracle.h).  Single-threaded, streaming over an
 * in-memory buffer with the same control flow as the Go readers; bufio.ReadBytes is
 * restated as a memchr over the buffer (no copy -- lengths are all the driver needs).
 * Citations are relative to /root/reference/shock-server/.
 */
#include "shockidx_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* Go stdlib: utf8.DecodeRune / DecodeLastRune, unicode.IsSpace, bytes.TrimSpace        */
/* ------------------------------------------------------------------------------------ */
#define RUNE_ERROR 0xFFFDu

static int ascii_space(uint8_t c) {
  return c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r' || c == ' ';
}

/* unicode/utf8.DecodeRune on p[0..n) ; returns rune, sets *w */
static uint32_t decode_rune(const uint8_t *p, size_t n, size_t *w) {
  if (n < 1) { *w = 0; return RUNE_ERROR; }
  uint8_t p0 = p[0];
  if (p0 < 0x80) { *w = 1; return p0; }
  size_t sz; uint8_t lo, hi;
  if (p0 >= 0xC2 && p0 <= 0xDF) { sz = 2; lo = 0x80; hi = 0xBF; }
  else if (p0 == 0xE0) { sz = 3; lo = 0xA0; hi = 0xBF; }
  else if ((p0 >= 0xE1 && p0 <= 0xEC) || p0 == 0xEE || p0 == 0xEF) { sz = 3; lo = 0x80; hi = 0xBF; }
  else if (p0 == 0xED) { sz = 3; lo = 0x80; hi = 0x9F; }
  else if (p0 == 0xF0) { sz = 4; lo = 0x90; hi = 0xBF; }
  else if (p0 >= 0xF1 && p0 <= 0xF3) { sz = 4; lo = 0x80; hi = 0xBF; }
  else if (p0 == 0xF4) { sz = 4; lo = 0x80; hi = 0x8F; }
  else { *w = 1; return RUNE_ERROR; }
  if (n < sz) { *w = 1; return RUNE_ERROR; }
  uint8_t b1 = p[1];
  if (b1 < lo || b1 > hi) { *w = 1; return RUNE_ERROR; }
  if (sz == 2) { *w = 2; return ((uint32_t)(p0 & 0x1F) << 6) | (b1 & 0x3F); }
  uint8_t b2 = p[2];
  if (b2 < 0x80 || b2 > 0xBF) { *w = 1; return RUNE_ERROR; }
  if (sz == 3) { *w = 3; return ((uint32_t)(p0 & 0x0F) << 12) | ((uint32_t)(b1 & 0x3F) << 6) | (b2 & 0x3F); }
  uint8_t b3 = p[3];
  if (b3 < 0x80 || b3 > 0xBF) { *w = 1; return RUNE_ERROR; }
  *w = 4;
  return ((uint32_t)(p0 & 0x07) << 18) | ((uint32_t)(b1 & 0x3F) << 12) |
         ((uint32_t)(b2 & 0x3F) << 6) | (b3 & 0x3F);
}

/* unicode/utf8.DecodeLastRune on p[0..end) */
static uint32_t decode_last_rune(const uint8_t *p, size_t end, size_t *w) {
  if (end == 0) { *w = 0; return RUNE_ERROR; }
  ptrdiff_t start = (ptrdiff_t)end - 1;
  if (p[start] < 0x80) { *w = 1; return p[start]; }
  ptrdiff_t lim = (ptrdiff_t)end - 4;
  if (lim < 0) lim = 0;
  for (start--; start >= lim; start--)
    if ((p[start] & 0xC0) != 0x80) break;
  if (start < 0) start = 0;
  size_t size;
  uint32_t r = decode_rune(p + start, end - (size_t)start, &size);
  if ((size_t)start + size != end) { *w = 1; return RUNE_ERROR; }
  *w = size;
  return r;
}

static int unicode_is_space(uint32_t r) {
  if (r <= 0xFF)
    return r == 0x09 || r == 0x0A || r == 0x0B || r == 0x0C || r == 0x0D || r == 0x20 ||
           r == 0x85 || r == 0xA0;
  return r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 ||
         r == 0x202F || r == 0x205F || r == 0x3000;
}

/* bytes.TrimFunc(s, unicode.IsSpace) on s[a..b): bounds into *lo,*hi */
static void trim_func_space(const uint8_t *s, size_t a, size_t b, size_t *lo, size_t *hi) {
  size_t i = a, w;
  while (i < b) {
    uint32_t r = decode_rune(s + i, b - i, &w);
    if (!unicode_is_space(r)) break;
    i += w;
  }
  /* TrimRightFunc on s[i..b): lastIndexFunc then forward width of the rune found */
  size_t j = b;
  ptrdiff_t found = -1;
  while (j > i) {
    uint32_t r = s[j - 1];
    size_t size = 1;
    if (r >= 0x80) r = decode_last_rune(s + i, j - i, &size);
    j -= size;
    if (!unicode_is_space(r)) { found = (ptrdiff_t)j; break; }
  }
  size_t end;
  if (found < 0) {
    end = i; /* everything trimmed */
  } else if (s[found] >= 0x80) {
    decode_rune(s + found, b - (size_t)found, &w);
    end = (size_t)found + w;
  } else {
    end = (size_t)found + 1;
  }
  *lo = i;
  *hi = end;
}

/* bytes.TrimSpace (Go >= 1.13): ASCII fast path, Unicode fallback at a byte >= 0x80 */
static void trim_space(const uint8_t *s, size_t a, size_t b, size_t *lo, size_t *hi) {
  size_t start = a;
  for (; start < b; start++) {
    uint8_t c = s[start];
    if (c >= 0x80) { trim_func_space(s, start, b, lo, hi); return; }
    if (!ascii_space(c)) break;
  }
  size_t stop = b;
  for (; stop > start; stop--) {
    uint8_t c = s[stop - 1];
    if (c >= 0x80) { trim_func_space(s, start, stop, lo, hi); return; }
    if (!ascii_space(c)) break;
  }
  *lo = start;
  *hi = stop;
}

void oracle_trim_space(const uint8_t *s, size_t n, size_t *lo, size_t *hi) {
  trim_space(s, 0, n, lo, hi);
}

/* ------------------------------------------------------------------------------------ */
/* bufio.Reader.ReadBytes restated over a memory buffer                                  */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const uint8_t *d;
  size_t n, p;
} breader;

/* returns [*s, *e) of the ReadBytes result; 1 if EOF (no delimiter found) */
static int read_bytes(breader *r, uint8_t delim, size_t *s, size_t *e) {
  *s = r->p;
  const uint8_t *q = r->p < r->n ? memchr(r->d + r->p, delim, r->n - r->p) : NULL;
  if (!q) { r->p = r->n; *e = r->n; return 1; }
  r->p = (size_t)(q - r->d) + 1;
  *e = r->p;
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Readers.  get_read_offset: returns 0 ok / 1 eof / 2 error (msg set)                    */
/* ------------------------------------------------------------------------------------ */
enum { RD_OK = 0, RD_EOF = 1, RD_ERR = 2 };

typedef struct {
  char *err;
  size_t errlen;
  size_t n; /* message length (messages may hold NUL bytes: FASTA snippets) */
} errbuf;

static int set_err(errbuf *eb, const char *msg) {
  if (eb->err && eb->errlen) {
    snprintf(eb->err, eb->errlen, "%s", msg);
    eb->n = strlen(eb->err);
  }
  return RD_ERR;
}

/* fastq.go:134-213 */
static int fastq_get(breader *r, uint64_t *n, errbuf *eb) {
  size_t is, ie, ss, se, ps, pe, qs, qe;
  int eof, empty = 0;
  *n = 0;
  for (;;) { /* :143-152 */
    eof = read_bytes(r, '\n', &is, &ie);
    if (eof) break;
    if (ie - is > 1) break;
    empty = 1;
  }
  if (eof) { /* :154-158 */
    if (ie - is > 0) return set_err(eb, "Invalid format: truncated fastq record");
    return RD_EOF;
  }
  if (empty) return set_err(eb, "Invalid format: empty line(s) between records");
  if (r->d[is] != '@') return set_err(eb, "Invalid format: id line does not start with @");
  if (ie - is == 2) return set_err(eb, "Invalid format: missing sequence ID");
  uint64_t curr = ie - is;
  eof = read_bytes(r, '\n', &ss, &se); /* :173-182 */
  if (eof) return set_err(eb, "Invalid format: truncated fastq record");
  if (se - ss == 1) return set_err(eb, "Invalid format: empty sequence");
  curr += se - ss;
  eof = read_bytes(r, '\n', &ps, &pe); /* :185-199 */
  if (eof) return set_err(eb, "Invalid format: truncated fastq record");
  if (r->d[ps] != '+') return set_err(eb, "Invalid format: plus line does not start with +");
  size_t plo, phi;
  trim_space(r->d, ps, pe, &plo, &phi);
  if (phi - plo > 1) {
    size_t ilo, ihi;
    trim_space(r->d, is + 1, ie, &ilo, &ihi);
    if (ihi - ilo != phi - plo - 1 || memcmp(r->d + ilo, r->d + plo + 1, ihi - ilo) != 0)
      return set_err(eb, "Invalid format: quality ID does not match sequence ID");
  }
  curr += pe - ps;
  eof = read_bytes(r, '\n', &qs, &qe); /* :202-209 */
  size_t a, b, c, d;
  trim_space(r->d, ss, se, &a, &b);
  trim_space(r->d, qs, qe, &c, &d);
  if (b - a != d - c) return set_err(eb, "Invalid format: length of sequence and quality lines do not match");
  *n = curr + (qe - qs);
  return eof ? RD_EOF : RD_OK;
}

/* fasta.go:93-140 */
static int fasta_get(breader *r, uint64_t *n, errbuf *eb) {
  size_t s, e;
  *n = 0;
  for (;;) {
    int eof = read_bytes(r, '>', &s, &e);
    size_t len = e - s;
    if (len > 1 && memchr(r->d + s, '\n', len)) { /* :111 */
      size_t te = e;
      while (te > s && r->d[te - 1] == '>') te--; /* TrimRight(read, ">") */
      size_t lo, hi;
      trim_space(r->d, s, te, &lo, &hi);
      /* Split(core,'\n')[1:] joined is empty <=> core holds no '\n' (core ends non-space) */
      if (hi <= lo || !memchr(r->d + lo, '\n', hi - lo)) { /* :113-121 */
        if (eb->err && eb->errlen) {
          size_t show = len > 50 ? 50 : len;
          size_t pre = strlen("Invalid fasta entry: ");
          size_t cap = eb->errlen - 1;
          memcpy(eb->err, "Invalid fasta entry: ", pre < cap ? pre : cap);
          if (pre < cap) {
            size_t k = show < cap - pre ? show : cap - pre;
            memcpy(eb->err + pre, r->d + s, k);
            eb->err[pre + k] = 0;
            eb->n = pre + k;
          } else {
            eb->err[cap] = 0;
            eb->n = cap;
          }
        }
        return RD_ERR;
      }
      if (eof) { *n += len; return RD_EOF; } /* :123-125 */
      *n += len - 1;
      r->p--; /* UnreadByte :127-128 */
      return RD_OK;
    }
    *n += len; /* :131-132 */
    if (eof) return RD_EOF;
  }
}

/* sam.go:83-98 */
static int sam_get(breader *r, uint64_t *n, errbuf *eb) {
  (void)eb;
  size_t s, e;
  *n = 0;
  for (;;) {
    int eof = read_bytes(r, '\n', &s, &e);
    *n += e - s;
    if (e - s > 1) {
      if (r->d[s] == '@') continue;
      return RD_OK; /* err stays nil even at EOF */
    } else if (eof) {
      return RD_EOF;
    }
  }
}

/* ------------------------------------------------------------------------------------ */
/* Format detection: hand-written matchers of the three anchored regexes                 */
/* (fasta.go:22, fastq.go:22, sam.go:17); Go \s = [\t\n\f\r ] (no \v).                    */
/* ------------------------------------------------------------------------------------ */
static int is_S(uint8_t c) { return !(c == '\t' || c == '\n' || c == '\f' || c == '\r' || c == ' '); }
static int is_SST(uint8_t c) { return !(c == '\n' || c == '\f' || c == '\r'); }
static int is_NR(uint8_t c) { return c == '\n' || c == '\r'; }
static int is_alpha(uint8_t c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

/* ^[\n\r]*>\S+[\S\t ]*[\n\r]+[A-Za-z\- ]+ */
static int match_fasta(const uint8_t *b, size_t n) {
  size_t i = 0;
  while (i < n && is_NR(b[i])) i++;
  if (i >= n || b[i] != '>') return 0;
  i++;
  if (i >= n || !is_S(b[i])) return 0;
  i++;
  while (i < n && is_SST(b[i])) i++;
  if (i >= n || !is_NR(b[i])) return 0;
  while (i < n && is_NR(b[i])) i++;
  return i < n && (is_alpha(b[i]) || b[i] == '-' || b[i] == ' ');
}

/* ^[\n\r]*@\S+[\S\t ]*[\n\r]+[A-Za-z\-]+[\n\r]+\+[\S\t ]*[\n\r]+\S*[\n\r]+ */
static int match_fastq(const uint8_t *b, size_t n) {
  size_t i = 0;
  while (i < n && is_NR(b[i])) i++;
  if (i >= n || b[i] != '@') return 0;
  i++;
  if (i >= n || !is_S(b[i])) return 0;
  i++;
  while (i < n && is_SST(b[i])) i++;
  if (i >= n || !is_NR(b[i])) return 0;
  while (i < n && is_NR(b[i])) i++;
  if (i >= n || !(is_alpha(b[i]) || b[i] == '-')) return 0;
  while (i < n && (is_alpha(b[i]) || b[i] == '-')) i++;
  if (i >= n || !is_NR(b[i])) return 0;
  while (i < n && is_NR(b[i])) i++;
  if (i >= n || b[i] != '+') return 0;
  i++;
  while (i < n && is_SST(b[i])) i++;
  size_t k = 0;
  while (i + k < n && is_NR(b[i + k])) k++;
  if (k == 0) return 0;
  if (k >= 2) return 1;
  i += 1;
  while (i < n && is_S(b[i])) i++;
  return i < n && is_NR(b[i]);
}

/* ^[\n\r]*[@[A-Z][A-Z][ \t]+[\S \t]+[\n\r]]*   (RE2: class {@,[,A-Z}; trailing \]* ) */
static int match_sam(const uint8_t *b, size_t n) {
  size_t i = 0;
  while (i < n && is_NR(b[i])) i++;
  if (i >= n || !(b[i] == '@' || b[i] == '[' || (b[i] >= 'A' && b[i] <= 'Z'))) return 0;
  i++;
  if (i >= n || !(b[i] >= 'A' && b[i] <= 'Z')) return 0;
  i++;
  if (i >= n || !(b[i] == ' ' || b[i] == '\t')) return 0;
  i++;
  size_t run = 0;
  while (i < n && is_SST(b[i])) { i++; run++; }
  return run >= 1 && i < n && is_NR(b[i]);
}

/* Regex.MatchString(s) semantics (the reference's fasta_test.go / fastq_test.go TestRegex):
 * the three anchored matchers over s itself, no 32 KiB zero padding.  Bit 0 fasta, 1 fastq,
 * 2 sam. */
int oracle_regex_match(const uint8_t *data, size_t n) {
  return (match_fasta(data, n) ? 1 : 0) | (match_fastq(data, n) ? 2 : 0) | (match_sam(data, n) ? 4 : 0);
}

int oracle_detect(const uint8_t *data, size_t n, int *mask) {
  uint8_t buf[32768];
  size_t m = n < sizeof buf ? n : sizeof buf;
  memcpy(buf, data, m);
  memset(buf + m, 0, sizeof buf - m);
  int bits = (match_fasta(buf, sizeof buf) ? 1 : 0) | (match_fastq(buf, sizeof buf) ? 2 : 0) |
             (match_sam(buf, sizeof buf) ? 4 : 0);
  if (mask) *mask = bits;
  if (bits & 1) return ORC_FMT_FASTA;
  if (bits & 2) return ORC_FMT_FASTQ;
  if (bits & 4) return ORC_FMT_SAM;
  return ORC_FMT_NONE;
}

/* ------------------------------------------------------------------------------------ */
/* Drivers                                                                               */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  uint64_t *v;
  uint64_t count, cap;
} rowbuf;

static int push_row(rowbuf *rb, uint64_t off, uint64_t len) {
  if (rb->count == rb->cap) {
    uint64_t nc = rb->cap ? rb->cap * 2 : 1024;
    uint64_t *nv = realloc(rb->v, nc * 2 * sizeof(uint64_t));
    if (!nv) return -1;
    rb->v = nv;
    rb->cap = nc;
  }
  rb->v[2 * rb->count] = off;
  rb->v[2 * rb->count + 1] = len;
  rb->count++;
  return 0;
}

int oracle_record_index(const uint8_t *data, size_t n, int fmt, uint64_t **rows,
                        uint64_t *count, char *err, size_t errlen, size_t *errn) {
  errbuf eb = {err, errlen, 0};
  rowbuf rb = {NULL, 0, 0};
  if (err && errlen) err[0] = 0;
  *rows = NULL;
  *count = 0;
  if (fmt < 0) fmt = oracle_detect(data, n, NULL);
  if (fmt == ORC_FMT_NONE) {
    set_err(&eb, "Invalid file type for filter"); /* errors.go:20, multi.go:61 */
    if (errn) *errn = eb.n;
    return 1;
  }
  breader r = {data, n, 0};
  uint64_t curr = 0;
  int rc = 0;
  for (;;) { /* record.go:51-83 */
    uint64_t len;
    int st = fmt == ORC_FMT_FASTQ ? fastq_get(&r, &len, &eb)
             : fmt == ORC_FMT_FASTA ? fasta_get(&r, &len, &eb)
                                    : sam_get(&r, &len, &eb);
    if (st == RD_ERR) { rc = 1; break; }
    if (st == RD_EOF && len == 0) break;
    if (push_row(&rb, curr, len)) { free(rb.v); return -1; }
    curr += len;
    if (st == RD_EOF) break;
  }
  *rows = rb.v;
  *count = rb.count;
  if (errn) *errn = eb.n;
  return rc;
}

int oracle_line_index(const uint8_t *data, size_t n, uint64_t **rows, uint64_t *count) {
  rowbuf rb = {NULL, 0, 0};
  breader r = {data, n, 0};
  uint64_t curr = 0;
  for (;;) { /* line.go:50-80, no eof&&n==0 guard */
    size_t s, e;
    int eof = read_bytes(&r, '\n', &s, &e);
    if (push_row(&rb, curr, e - s)) { free(rb.v); return -1; }
    curr += e - s;
    if (eof) break;
  }
  *rows = rb.v;
  *count = rb.count;
  return 0;
}

void oracle_free(void *p) { free(p); }
