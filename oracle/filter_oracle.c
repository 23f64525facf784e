/* filter_oracle.c -- CPU restatement of Shock's download filters over a FASTQ section.
 * TEST INFRASTRUCTURE ONLY (see shockidx_oracle.h): the checker of shockidx_filter_device.
 *
 * Restates (paths relative to /root/reference/shock-server/):
 *   node/filter/fq2fa/fq2fa.go:58-84          Reader.Read: records via fastq.Reader.Read,
 *                                             each written with fasta.Format
 *   node/filter/anonymize/anonymize.go:28-56  Reader.Read: seq.ID = fmt.Sprint(counter),
 *                                             counter from 1, the detected format's Format
 *   node/file/format/fastq/fastq.go:50-132    fastq.Reader.Read
 *   node/file/format/fastq/fastq.go:283-285   fastq.Format   fasta/fasta.go:216-218 fasta.Format
 *   fasta/fasta.go:40-88 fasta.Reader.Read   sam/sam.go:44-81 sam.Reader.Read,
 *   sam.go:146-148 sam.Format (anonymize of FASTA / SAM sections)
 * Both filters stop at the first Read error; a record Read returns together with io.EOF (its
 * quality line ends the file without '\n') is dropped (the filter loop breaks on er != nil
 * before formatting it).  The output is the byte stream the filter delivers to io.Copy
 * (the 32 KiB chunking of Read(p) does not change it, except that on a non-EOF error the
 * reference hands io.Copy a stale buffer for its last chunk -- not restated: the stream here
 * ends with the last complete record).
 */
#include "shockidx_oracle.h"

#include <stdlib.h>
#include <string.h>

typedef struct { const uint8_t *d; size_t n, p; } rd_t;

/* bufio.Reader.ReadBytes('\n'): [*s, *e); 1 on EOF (no delimiter) */
static int read_line(rd_t *r, size_t *s, size_t *e) {
  *s = r->p;
  const uint8_t *q = r->p < r->n ? memchr(r->d + r->p, '\n', r->n - r->p) : NULL;
  if (!q) { r->p = r->n; *e = r->n; return 1; }
  r->p = (size_t)(q - r->d) + 1;
  *e = r->p;
  return 0;
}

/* bytes.TrimSpace (shockidx_oracle.c: ASCII fast path, Unicode fallback) on d[a, b) */
static void trim(const uint8_t *d, size_t a, size_t b, size_t *lo, size_t *hi) {
  size_t l = 0, h = 0;
  oracle_trim_space(d + a, b - a, &l, &h);
  *lo = a + l;
  *hi = a + h;
}

enum { R_OK = 0, R_EOF_REC = 1, R_EOF = 2, R_ERR = 3 };

/* fastq.Reader.Read; spans of the trimmed ID / sequence / quality */
static int fq_read(rd_t *r, size_t sp[6], const char **msg) {
  size_t is = 0, ie = 0, ss, se, ps, pe, qs, qe;
  int eof, empty = 0;
  for (;;) { /* :56-66 */
    eof = read_line(r, &is, &ie);
    if (eof) break;
    if (ie - is > 1) break;
    empty = 1;
  }
  if (eof) { /* :68-72 */
    if (ie - is > 0) { *msg = "Invalid format: truncated fastq record"; return R_ERR; }
    return R_EOF;
  }
  if (empty) { *msg = "Invalid format: empty line(s) between records"; return R_ERR; }
  if (r->d[is] != '@') { *msg = "Invalid format: id line does not start with @"; return R_ERR; }
  trim(r->d, is + 1, ie, &sp[0], &sp[1]); /* :83 */
  if (sp[1] == sp[0]) { *msg = "Invalid format: missing sequence ID"; return R_ERR; }
  if (read_line(r, &ss, &se)) { *msg = "Invalid format: truncated fastq record"; return R_ERR; }
  trim(r->d, ss, se, &sp[2], &sp[3]);
  if (sp[3] == sp[2]) { *msg = "Invalid format: empty sequence"; return R_ERR; }
  if (read_line(r, &ps, &pe)) { *msg = "Invalid format: truncated fastq record"; return R_ERR; }
  if (r->d[ps] != '+') { *msg = "Invalid format: plus line does not start with +"; return R_ERR; }
  size_t plo, phi;
  trim(r->d, ps, pe, &plo, &phi);
  if (phi - plo > 1 &&
      (phi - plo - 1 != sp[1] - sp[0] || memcmp(r->d + sp[0], r->d + plo + 1, sp[1] - sp[0]) != 0)) {
    *msg = "Invalid format: quality ID does not match sequence ID";
    return R_ERR;
  }
  eof = read_line(r, &qs, &qe); /* :117-121: EOF is not an error here */
  trim(r->d, qs, qe, &sp[4], &sp[5]);
  if (sp[3] - sp[2] != sp[5] - sp[4]) {
    *msg = "Invalid format: length of sequence and quality lines do not match";
    return R_ERR;
  }
  return eof ? R_EOF_REC : R_OK;
}

typedef struct { uint8_t *v; size_t n, cap; } buf_t;
static int put(buf_t *b, const void *s, size_t k);

/* fmt.Sprint(counter) */
static int put_counter(buf_t *b, uint64_t v) {
  char tmp[24], id[24];
  int dn = 0;
  do { tmp[dn++] = (char)('0' + v % 10); v /= 10; } while (v);
  for (int i = 0; i < dn; ++i) id[i] = tmp[dn - 1 - i];
  return put(b, id, (size_t)dn);
}

/* bufio.Reader.ReadBytes('>'): [*s, *e); 1 on EOF (no delimiter) */
static int read_gt(rd_t *r, size_t *s, size_t *e) {
  *s = r->p;
  const uint8_t *q = r->p < r->n ? memchr(r->d + r->p, '>', r->n - r->p) : NULL;
  if (!q) { r->p = r->n; *e = r->n; return 1; }
  r->p = (size_t)(q - r->d) + 1;
  *e = r->p;
  return 0;
}

/* fasta.go:40-88 Reader.Read: R_OK with the trimmed read in [*lo, *hi) (label = up to its first
 * '\n', Seq = the rest with every '\n' removed: bytes.Join(lines[1:], nil)), R_EOF, or R_ERR
 * ("Invalid fasta entry").  A read at EOF is returned with io.EOF whatever it holds.  Where Go
 * loops forever (an EOF read without '\n', e.g. a file ending in '>' or in a header line: the
 * loop keeps appending ReadBytes' empty results) this returns R_EOF. */
enum { FR_OK = 0, FR_EOF = 1, FR_ERR = 2 };
static int fa_read(rd_t *r, size_t *lo, size_t *hi) {
  size_t ps = (size_t)-1;  /* prev: the bytes read since this call began (contiguous) */
  for (;;) {
    size_t s, e;
    const int eof = read_gt(r, &s, &e);
    const size_t rs = ps != (size_t)-1 ? ps : s;
    const size_t len = e - rs;
    if (len == 1) {                                      /* :58-64 only '>' */
      if (eof) return FR_EOF;
      continue;
    }
    if (!memchr(r->d + rs, '\n', len)) {                /* :66-69 embedded '>' */
      if (eof) return FR_EOF;                            /* Go: endless loop */
      ps = rs;
      continue;
    }
    size_t ee = e;                                       /* :71 TrimRight(read, ">") */
    while (ee > rs && r->d[ee - 1] == '>') ee--;
    trim(r->d, rs, ee, lo, hi);                          /* TrimSpace */
    if (eof) return FR_EOF;                              /* :84-86 */
    return memchr(r->d + *lo, '\n', *hi - *lo) ? FR_OK : FR_ERR;  /* :72-83 */
  }
}

/* sam.go:44-81 Reader.Read: R_OK with the trimmed alignment line in [*lo, *hi), R_EOF (a last
 * line without '\n' ends it, read or not), R_ERR ("sam alignment fields less than 11") */
static int sam_read(rd_t *r, size_t *lo, size_t *hi) {
  for (;;) {
    size_t s, e;
    if (read_line(r, &s, &e)) return FR_EOF;              /* :71-73 */
    /* :50-52 a trailing '\r' is stripped only from a line ending in it: never, the line ends
       in '\n' */
    trim(r->d, s, e, lo, hi);
    if (*hi == *lo) continue;                              /* :53-56 */
    if (r->d[*lo] == '@') continue;                        /* :58-61 */
    size_t tabs = 0;
    for (size_t i = *lo; i < *hi; ++i) tabs += r->d[i] == '\t';
    if (tabs + 1 < 11) return FR_ERR;                      /* :63-67 */
    return FR_OK;
  }
}

static void set_err(char *err, size_t errlen, const char *m) {
  if (!errlen) return;
  size_t k = strlen(m);
  if (k > errlen - 1) k = errlen - 1;
  memcpy(err, m, k);
  err[k] = 0;
}

/* anonymize over a FASTA or SAM section: fasta.Format ">" counter "\n" Seq "\n" (fasta.go:
 * 216-218) / sam.Format Seq "\n" (sam.go:146-148: the ID it was given is not written) */
static int anonymize_other(const uint8_t *data, size_t n, int fasta, buf_t *b, uint64_t *count, char *err,
                           size_t errlen) {
  rd_t r = {data, n, 0};
  uint64_t k = 0;
  for (;;) {
    size_t lo, hi;
    const int st = fasta ? fa_read(&r, &lo, &hi) : sam_read(&r, &lo, &hi);
    if (st == FR_ERR) {
      set_err(err, errlen, fasta ? "Invalid fasta entry" : "sam alignment fields less than 11");
      *count = k;
      return 1;
    }
    if (st != FR_OK) break;
    k += 1;
    int bad = 0;
    if (fasta) {
      const uint8_t *f = memchr(data + lo, '\n', hi - lo);
      bad |= put(b, ">", 1) | put_counter(b, k) | put(b, "\n", 1);
      for (size_t i = (size_t)(f - data) + 1; i < hi;) {  /* Join(lines[1:]): the '\n's dropped */
        const uint8_t *q = memchr(data + i, '\n', hi - i);
        const size_t j = q ? (size_t)(q - data) : hi;
        bad |= put(b, data + i, j - i);
        i = j + 1;
      }
      bad |= put(b, "\n", 1);
    } else {
      bad |= put(b, data + lo, hi - lo) | put(b, "\n", 1);
    }
    if (bad) return -1;
  }
  *count = k;
  return 0;
}

static int put(buf_t *b, const void *s, size_t k) {
  if (b->n + k > b->cap) {
    size_t nc = b->cap ? b->cap : 4096;
    while (nc < b->n + k) nc *= 2;
    uint8_t *nv = realloc(b->v, nc);
    if (!nv) return -1;
    b->v = nv;
    b->cap = nc;
  }
  memcpy(b->v + b->n, s, k);
  b->n += k;
  return 0;
}

int oracle_filter_fastq(const uint8_t *data, size_t n, int kind, uint8_t **out, size_t *outlen, uint64_t *count,
                        char *err, size_t errlen) {
  rd_t r = {data, n, 0};
  buf_t b = {NULL, 0, 0};
  uint64_t k = 0;
  int rc = 0;
  if (errlen) err[0] = 0;
  *out = NULL;
  *outlen = 0;
  *count = 0;
  if (kind == 2) { /* anonymize reads through multi.Reader: DetermineFormat (multi.go:43-62) */
    const int f = oracle_detect(data, n, NULL);
    if (f == ORC_FMT_NONE) {
      static const char m[] = "Invalid file type for filter"; /* errors.go:20 */
      const size_t k2 = sizeof m - 1 < errlen - 1 ? sizeof m - 1 : errlen - 1;
      if (errlen) { memcpy(err, m, k2); err[k2] = 0; }
      return 1;
    }
    if (f != ORC_FMT_FASTQ) {
      rc = anonymize_other(data, n, f == ORC_FMT_FASTA, &b, &k, err, errlen);
      if (rc < 0) { free(b.v); return -1; }
      *out = b.v;
      *outlen = b.n;
      *count = k;
      return rc;
    }
  }
  for (;;) {
    size_t sp[6];
    const char *msg = NULL;
    const int st = fq_read(&r, sp, &msg);
    if (st == R_ERR) {
      size_t m = strlen(msg);
      if (m > errlen - 1) m = errlen - 1;
      if (errlen) { memcpy(err, msg, m); err[m] = 0; }
      rc = 1;
      break;
    }
    if (st != R_OK) break; /* io.EOF, with or without a record: the loop ends unformatted */
    k += 1;
    int bad = 0;
    if (kind == 1) { /* fasta.Format */
      bad |= put(&b, ">", 1) | put(&b, data + sp[0], sp[1] - sp[0]) | put(&b, "\n", 1) |
             put(&b, data + sp[2], sp[3] - sp[2]) | put(&b, "\n", 1);
    } else { /* fastq.Format with ID = fmt.Sprint(counter) */
      char id[24];
      int dn = 0;
      uint64_t v = k;
      char tmp[24];
      do { tmp[dn++] = (char)('0' + v % 10); v /= 10; } while (v);
      for (int i = 0; i < dn; ++i) id[i] = tmp[dn - 1 - i];
      bad |= put(&b, "@", 1) | put(&b, id, (size_t)dn) | put(&b, "\n", 1) | put(&b, data + sp[2], sp[3] - sp[2]) |
             put(&b, "\n+\n", 3) | put(&b, data + sp[4], sp[5] - sp[4]) | put(&b, "\n", 1);
    }
    if (bad) { free(b.v); return -1; }
  }
  *out = b.v;
  *outlen = b.n;
  *count = k;
  return rc;
}
