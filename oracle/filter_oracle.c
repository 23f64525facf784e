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
    if (f != ORC_FMT_FASTQ) return 2; /* FASTA / SAM sections: not restated here */
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
