/* subset_oracle.c -- CPU restatement of Shock's subset-index builder.
 * TEST INFRASTRUCTURE ONLY (see shockidx_oracle.h): the checker of the device subset path.
 *
 * Restates (paths relative to /root/reference/shock-server/):
 *   node/file/index/subset.go:133-303   CreateSubsetNodeIndexes ("array" parent index)
 *   node/file/format/line/line.go:28-34 ReadLine = bufio.ReadBytes('\n')
 * and the Go stdlib pieces its error texts depend on: strconv.Atoi (fast path + ParseInt /
 * ParseUint slow path, NumError.Error) and strconv.Quote.
 */
#include "shockidx_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- strconv.Quote ------------------------------------------------------------------ */
static const char HEX[] = "0123456789abcdef";

/* utf8.DecodeRune on s[0:n]: rune and width (RuneError, 1 for invalid) */
static uint32_t dec_rune(const uint8_t *s, size_t n, size_t *w) {
  const uint32_t c0 = s[0];
  if (c0 < 0x80) { *w = 1; return c0; }
  uint32_t sz, lo = 0x80, hi = 0xBF;
  if (c0 >= 0xC2 && c0 <= 0xDF) sz = 2;
  else if (c0 == 0xE0) { sz = 3; lo = 0xA0; }
  else if ((c0 >= 0xE1 && c0 <= 0xEC) || c0 == 0xEE || c0 == 0xEF) sz = 3;
  else if (c0 == 0xED) { sz = 3; hi = 0x9F; }
  else if (c0 == 0xF0) { sz = 4; lo = 0x90; }
  else if (c0 >= 0xF1 && c0 <= 0xF3) sz = 4;
  else if (c0 == 0xF4) { sz = 4; hi = 0x8F; }
  else { *w = 1; return 0xFFFD; }
  if (n < sz || s[1] < lo || s[1] > hi) { *w = 1; return 0xFFFD; }
  for (uint32_t i = 2; i < sz; ++i)
    if (s[i] < 0x80 || s[i] > 0xBF) { *w = 1; return 0xFFFD; }
  *w = sz;
  if (sz == 2) return ((c0 & 0x1F) << 6) | (s[1] & 0x3F);
  if (sz == 3) return ((c0 & 0x0F) << 12) | ((uint32_t)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
  return ((c0 & 0x07) << 18) | ((uint32_t)(s[1] & 0x3F) << 12) | ((uint32_t)(s[2] & 0x3F) << 6) | (s[3] & 0x3F);
}

/* unicode.IsPrint, exact for ASCII and Latin-1; above U+00FF the separators and format
 * characters Go rejects are listed, everything else counts as printable (the full Unicode
 * tables are not restated: non-ASCII id lines are "parity unpinned" in tests/). */
static int go_isprint(uint32_t r) {
  if (r < 0x80) return r >= 0x20 && r < 0x7F;
  if (r <= 0xA0) return 0;      /* C1 controls, NBSP */
  if (r == 0xAD) return 0;      /* soft hyphen (Cf) */
  if (r < 0x100) return 1;
  if (r == 0x1680 || (r >= 0x2000 && r <= 0x200F) || (r >= 0x2028 && r <= 0x202F) ||
      (r >= 0x205F && r <= 0x206F) || r == 0x3000 || r == 0xFEFF || (r >= 0xFFF9 && r <= 0xFFFB) ||
      (r >= 0xD800 && r <= 0xDFFF) || r > 0x10FFFF)
    return 0;
  return 1;
}

static size_t put(char *out, size_t cap, size_t o, char c) {
  if (o < cap) out[o] = c;
  return o + 1;
}

/* strconv.Quote(s) (appendQuotedWith / appendEscapedRune); returns the length written */
size_t oracle_go_quote(const uint8_t *s, size_t n, char *out, size_t cap) {
  size_t o = put(out, cap, 0, '"');
  for (size_t i = 0; i < n;) {
    size_t w;
    uint32_t r = dec_rune(s + i, n - i, &w);
    if (w == 1 && r == 0xFFFD) { /* invalid byte: \xNN */
      o = put(out, cap, o, '\\'); o = put(out, cap, o, 'x');
      o = put(out, cap, o, HEX[s[i] >> 4]); o = put(out, cap, o, HEX[s[i] & 15]);
      i += 1;
      continue;
    }
    if (r == '"' || r == '\\') {
      o = put(out, cap, o, '\\');
      o = put(out, cap, o, (char)r);
    } else if (go_isprint(r)) {
      for (size_t k = 0; k < w; ++k) o = put(out, cap, o, (char)s[i + k]);
    } else {
      const char *esc = NULL;
      switch (r) {
        case '\a': esc = "\\a"; break;
        case '\b': esc = "\\b"; break;
        case '\f': esc = "\\f"; break;
        case '\n': esc = "\\n"; break;
        case '\r': esc = "\\r"; break;
        case '\t': esc = "\\t"; break;
        case '\v': esc = "\\v"; break;
        default: break;
      }
      if (esc) {
        o = put(out, cap, o, esc[0]); o = put(out, cap, o, esc[1]);
      } else if (r < ' ' || r == 0x7F) {
        o = put(out, cap, o, '\\'); o = put(out, cap, o, 'x');
        o = put(out, cap, o, HEX[r >> 4]); o = put(out, cap, o, HEX[r & 15]);
      } else if (r < 0x10000) {
        o = put(out, cap, o, '\\'); o = put(out, cap, o, 'u');
        for (int sh = 12; sh >= 0; sh -= 4) o = put(out, cap, o, HEX[(r >> sh) & 15]);
      } else {
        o = put(out, cap, o, '\\'); o = put(out, cap, o, 'U');
        for (int sh = 28; sh >= 0; sh -= 4) o = put(out, cap, o, HEX[(r >> sh) & 15]);
      }
    }
    i += w;
  }
  return put(out, cap, o, '"');
}

/* ---- strconv.Atoi ------------------------------------------------------------------- */
enum { ATOI_OK = 0, ATOI_SYNTAX = 1, ATOI_RANGE = 2 };

static int go_atoi(const uint8_t *s, size_t n, int64_t *v) {
  if (n > 0 && n < 19) { /* fast path */
    size_t i = 0;
    int neg = 0;
    if (s[0] == '-' || s[0] == '+') {
      neg = s[0] == '-';
      i = 1;
      if (n < 2) return ATOI_SYNTAX;
    }
    int64_t x = 0;
    for (; i < n; ++i) {
      const uint8_t d = (uint8_t)(s[i] - '0');
      if (d > 9) return ATOI_SYNTAX;
      x = x * 10 + d;
    }
    *v = neg ? -x : x;
    return ATOI_OK;
  }
  /* ParseInt(s, 10, 0) */
  if (n == 0) return ATOI_SYNTAX;
  size_t i = 0;
  int neg = 0;
  if (s[0] == '+') i = 1;
  else if (s[0] == '-') { neg = 1; i = 1; }
  if (i == n) return ATOI_SYNTAX; /* ParseUint("") */
  const uint64_t cutoff10 = UINT64_MAX / 10 + 1;
  uint64_t u = 0;
  int range = 0;
  for (; i < n; ++i) { /* ParseUint: the first syntax or overflow event wins */
    const uint8_t c = s[i];
    if (c < '0' || c > '9') return ATOI_SYNTAX;
    if (u >= cutoff10) { range = 1; break; }
    u *= 10;
    const uint64_t u1 = u + (uint64_t)(c - '0');
    if (u1 < u) { range = 1; break; }
    u = u1;
  }
  if (range) return ATOI_RANGE;
  const uint64_t cut = 1ull << 63;
  if (!neg && u >= cut) return ATOI_RANGE;
  if (neg && u > cut) return ATOI_RANGE;
  *v = neg ? (int64_t)(0 - u) : (int64_t)u;
  return ATOI_OK;
}

/* ---- CreateSubsetNodeIndexes -------------------------------------------------------- */
typedef struct { uint64_t *v; uint64_t count, cap; } rows_t;

static int push2(rows_t *b, uint64_t a, uint64_t c) {
  if (b->count == b->cap) {
    uint64_t nc = b->cap ? 2 * b->cap : 1024;
    uint64_t *nv = realloc(b->v, nc * 2 * sizeof(uint64_t));
    if (!nv) return -1;
    b->v = nv;
    b->cap = nc;
  }
  b->v[2 * b->count] = a;
  b->v[2 * b->count + 1] = c;
  b->count++;
  return 0;
}

static size_t emsg(char *err, size_t errlen, const char *fmt, long long a, long long b, int two) {
  char tmp[256];
  int k = two ? snprintf(tmp, sizeof tmp, fmt, a, b) : snprintf(tmp, sizeof tmp, fmt, a);
  size_t m = (size_t)k < errlen ? (size_t)k : (errlen ? errlen - 1 : 0);
  if (errlen) { memcpy(err, tmp, m); err[m] = 0; }
  return m;
}

int oracle_subset(const uint8_t *ids, size_t n, const uint64_t *parent, uint64_t parent_count, int64_t ilength,
                  uint64_t **rows, uint64_t *count, uint64_t **runs, uint64_t *nruns, uint64_t *size, char *err,
                  size_t errlen, size_t *errn) {
  rows_t o = {NULL, 0, 0}, co = {NULL, 0, 0};
  int64_t prev = 0;
  uint64_t osize = 0, co_off = 0, co_len = 0, prev_off = 0, prev_len = 0;
  int rc = 0;
  size_t en = 0;
  if (errlen) err[0] = 0;
  size_t p = 0;
  for (;;) { /* subset.go:186-272 */
    const uint8_t *nl = p < n ? memchr(ids + p, '\n', n - p) : NULL;
    if (!nl) break;                      /* ReadLine error (EOF): the last line is dropped */
    const size_t ln = (size_t)(nl - (ids + p)) + 1;
    const uint8_t *buf = ids + p;
    p += ln;
    if (ln <= 1) continue;               /* :197-199 skip empty line */
    int64_t cur = 0;
    const int a = go_atoi(buf, ln - 1, &cur);  /* :201-206 */
    if (a != ATOI_OK) {
      char q[200];
      size_t qn = oracle_go_quote(buf, ln - 1, q, sizeof q);
      if (qn > sizeof q) qn = sizeof q;
      char tmp[300];
      int k = snprintf(tmp, sizeof tmp, "strconv.Atoi: parsing %.*s: %s", (int)qn, q,
                       a == ATOI_SYNTAX ? "invalid syntax" : "value out of range");
      en = (size_t)k < errlen ? (size_t)k : (errlen ? errlen - 1 : 0);
      if (errlen) { memcpy(err, tmp, en); err[en] = 0; }
      rc = 1;
      break;
    }
    if (cur <= prev) {                   /* :208-211 */
      en = emsg(err, errlen, "Subset indices must be numerically sorted and non-redundant, found value %lld after value %lld",
                (long long)cur, (long long)prev, 1);
      rc = 1;
      break;
    }
    if (cur > ilength) {                 /* :213-216 */
      en = emsg(err, errlen, "Subset index: %lld does not exist in parent index file.", (long long)cur, 0, 0);
      rc = 1;
      break;
    }
    if ((uint64_t)cur > parent_count) {  /* :218-223 ReadAt past the parent index file */
      en = emsg(err, errlen, "Subset index could not read parent index file for part: %lld", (long long)cur, 0, 0);
      rc = 1;
      break;
    }
    const uint64_t off = parent[2 * (cur - 1)], len = parent[2 * (cur - 1) + 1];
    if (push2(&o, off, len)) goto oom;   /* :228-242 */
    osize += len;
    if (prev != 0 && off != prev_off + prev_len) { /* :244-267 compressed index */
      if (push2(&co, co_off, co_len)) goto oom;
      co_off = off;
      co_len = len;
    } else if (prev == 0) {
      co_off = off;
      co_len += len;
    } else {
      co_len += len;
    }
    prev = cur;
    prev_off = off;
    prev_len = len;
  }
  if (rc == 0 && osize != 0)             /* :285-291 final run only when oSize != 0 */
    if (push2(&co, co_off, co_len)) goto oom;
  *rows = o.v; *count = o.count;
  *runs = co.v; *nruns = co.count;
  *size = osize;
  if (errn) *errn = en;
  return rc;
oom:
  free(o.v);
  free(co.v);
  return -1;
}
