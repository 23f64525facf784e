/* part_oracle.c -- CPU restatement of Shock's index read path (Idx.Part / Idx.Range) and of
 * CreateSubsetIndex.  TEST INFRASTRUCTURE ONLY (see shockidx_oracle.h): the checker of the
 * device paths shockidx_idx_part / shockidx_idx_range / shockidx_create_subset_index.
 *
 * Restates (paths relative to /root/reference/shock-server/):
 *   node/file/index/index.go:67-117    Idx.Part(part, idxFilePath, idxLength) -> (pos, length, err)
 *   node/file/index/index.go:119-193   Idx.Range(part, idxFilePath, idxLength) -> ([][2]int64, err)
 *   node/file/index/subset.go:36-128   CreateSubsetIndex -> (count, size, err); (-1, -1, err) on error
 *   errors/errors.go:21-23             InvalidIndexRange, IndexOutBounds, IndexNoFile
 * and the Go stdlib pieces they rest on: strings.Split(part, "-")[0:2], strconv.ParseInt(s, 10,
 * 64) (sign, decimal digits, int64 range; any error counts the same here), and
 * binary.Read(io.NewSectionReader(f, off, 16), LittleEndian, &int64): a read past the end of the
 * .idx file fails and leaves the destination as it was (Part: zero; Range: the `rec` slice is
 * reused, so it keeps the last row read).  The .idx file is given as its whole rows
 * (nrows = file size / 16); rows == NULL stands for a missing file (IndexNoFile).
 */
#include "shockidx_oracle.h"

#include <stdlib.h>
#include <string.h>

static const char E_RANGE[] = "Invalid index record range";
static const char E_BOUNDS[] = "Index record out of bounds";
static const char E_NOFILE[] = "Index file is missing";

static int set(char *err, size_t errlen, const char *m) {
  if (errlen) {
    size_t k = strlen(m);
    if (k > errlen - 1) k = errlen - 1;
    memcpy(err, m, k);
    err[k] = 0;
  }
  return 1;
}

/* strconv.ParseInt(s[0:n], 10, 64): 0 ok, 1 any error (syntax or range) */
static int parse_int64(const char *s, size_t n, int64_t *v) {
  size_t i = 0;
  int neg = 0;
  if (n == 0) return 1;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i == n) return 1;
  uint64_t u = 0;
  for (; i < n; ++i) {
    const unsigned d = (unsigned char)s[i] - '0';
    if (d > 9) return 1;
    if (u > (UINT64_MAX - d) / 10) return 1; /* ParseUint range error */
    u = u * 10 + d;
  }
  if (!neg && u > (uint64_t)INT64_MAX) return 1;
  if (neg && u > (uint64_t)INT64_MAX + 1) return 1;
  *v = neg ? (int64_t)(0 - u) : (int64_t)u;
  return 0;
}

/* The part string: 0 single record p, 1 range start-end, -1 parse/bounds error (code in *e) */
static int parse_part(const char *part, int64_t idx_length, int64_t *a, int64_t *b, const char **e) {
  const char *dash = strchr(part, '-');
  if (dash) { /* strings.Split(part, "-"): [0] before the first '-', [1] up to the next one */
    const char *s1 = dash + 1;
    const char *d2 = strchr(s1, '-');
    const size_t n1 = d2 ? (size_t)(d2 - s1) : strlen(s1);
    int64_t start = 0, end = 0;
    const int se = parse_int64(part, (size_t)(dash - part), &start);
    const int ee = parse_int64(s1, n1, &end);
    if (se || ee || start <= 0 || start > idx_length || end <= 0 || end > idx_length) {
      *e = E_RANGE;
      return -1;
    }
    *a = start;
    *b = end;
    return 1;
  }
  int64_t p = 0;
  if (parse_int64(part, strlen(part), &p) || p <= 0 || p > idx_length) {
    *e = E_BOUNDS;
    return -1;
  }
  *a = *b = p;
  return 0;
}

int oracle_idx_part(const uint64_t *rows, uint64_t nrows, const char *part, int64_t idx_length, int64_t *pos,
                    int64_t *length, char *err, size_t errlen) {
  *pos = 0;
  *length = 0;
  if (errlen) err[0] = 0;
  if (!rows) return set(err, errlen, E_NOFILE); /* index.go:70-74 */
  int64_t a = 0, b = 0;
  const char *e = NULL;
  const int kind = parse_part(part, idx_length, &a, &b, &e);
  if (kind < 0) return set(err, errlen, e);
  /* fresh zeroed records: a failed read leaves zeros */
  int64_t s0 = 0, s1 = 0, e0 = 0, e1 = 0;
  if ((uint64_t)(a - 1) < nrows) { s0 = (int64_t)rows[2 * (a - 1)]; s1 = (int64_t)rows[2 * (a - 1) + 1]; }
  if (kind == 0) { /* index.go:100-115 */
    *pos = s0;
    *length = s1;
    return 0;
  }
  if ((uint64_t)(b - 1) < nrows) { e0 = (int64_t)rows[2 * (b - 1)]; e1 = (int64_t)rows[2 * (b - 1) + 1]; }
  *pos = s0; /* index.go:98-99, int64 arithmetic wraps */
  *length = (int64_t)((uint64_t)e0 - (uint64_t)s0 + (uint64_t)e1);
  return 0;
}

typedef struct { int64_t *v; uint64_t n, cap; } recs_t;
static int push(recs_t *r, int64_t p, int64_t l) {
  if (r->n == r->cap) {
    const uint64_t nc = r->cap ? 2 * r->cap : 64;
    int64_t *nv = realloc(r->v, nc * 2 * sizeof(int64_t));
    if (!nv) return -1;
    r->v = nv;
    r->cap = nc;
  }
  r->v[2 * r->n] = p;
  r->v[2 * r->n + 1] = l;
  r->n++;
  return 0;
}

int oracle_idx_range(const uint64_t *rows, uint64_t nrows, const char *part, int64_t idx_length, int64_t **recs,
                     uint64_t *nrecs, char *err, size_t errlen) {
  recs_t o = {NULL, 0, 0};
  *recs = NULL;
  *nrecs = 0;
  if (errlen) err[0] = 0;
  if (!rows) return set(err, errlen, E_NOFILE); /* index.go:122-126 */
  int64_t a = 0, b = 0;
  const char *e = NULL;
  const int kind = parse_part(part, idx_length, &a, &b, &e);
  if (kind < 0) return set(err, errlen, e);
  int64_t rec0 = 0, rec1 = 0; /* rec := make([]int64, 2), reused by every read */
#define READ(i)                                        \
  do {                                                 \
    if ((uint64_t)(i) < nrows) {                       \
      rec0 = (int64_t)rows[2 * (uint64_t)(i)];         \
      rec1 = (int64_t)rows[2 * (uint64_t)(i) + 1];     \
    }                                                  \
  } while (0)
  READ(a - 1);
  if (kind == 0) { /* index.go:178-192 */
    if (push(&o, rec0, rec1)) goto oom;
    goto done;
  }
  {
    int64_t cur_pos = rec0, cur_len = rec1;
    if (a == b) { /* index.go:146-150 */
      if (push(&o, cur_pos, cur_len)) goto oom;
      goto done;
    }
    for (int64_t x = a; x <= b - 1; ++x) { /* index.go:152-177; no pass at all when b < a */
      READ(x);
      const int64_t next_pos = rec0, next_len = rec1;
      const int contig = (uint64_t)cur_len == (uint64_t)next_pos - (uint64_t)cur_pos;
      if (x == b - 1) {
        if (contig) {
          if (push(&o, cur_pos, (int64_t)((uint64_t)cur_len + (uint64_t)next_len))) goto oom;
        } else {
          if (push(&o, cur_pos, cur_len) || push(&o, next_pos, next_len)) goto oom;
        }
        break;
      }
      if (contig) {
        cur_len = (int64_t)((uint64_t)cur_len + (uint64_t)next_len);
        continue;
      }
      if (push(&o, cur_pos, cur_len)) goto oom;
      cur_pos = next_pos;
      cur_len = next_len;
    }
  }
#undef READ
done:
  *recs = o.v;
  *nrecs = o.n;
  return 0;
oom:
  free(o.v);
  return -1;
}

int oracle_create_subset_index(const uint8_t *ids, size_t n, const uint64_t *parent, uint64_t parent_count,
                               int64_t ilength, uint64_t **rows, int64_t *count, int64_t *size, char *err,
                               size_t errlen, size_t *errn) {
  /* subset.go:36-128 checks the ids exactly like CreateSubsetNodeIndexes (:133-303) and
   * writes the same subset rows, without the compressed index; every error returns -1, -1 */
  uint64_t *runs = NULL, cnt = 0, nruns = 0, sz = 0;
  *rows = NULL;
  const int rc = oracle_subset(ids, n, parent, parent_count, ilength, rows, &cnt, &runs, &nruns, &sz, err, errlen, errn);
  free(runs);
  if (rc < 0) return rc;
  if (rc == 1) {
    *count = -1;
    *size = -1;
    return 1;
  }
  *count = (int64_t)cnt;
  *size = (int64_t)sz;
  return 0;
}
