/* shockidx_oracle.h -- CPU restatement of Shock's record/line indexers.
 *
 * TEST INFRASTRUCTURE ONLY.  Linked by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker / reported CPU baseline; never by the product library
 * (shock_amd/csrc -> libshockidx.so).
 *
 * A faithful single-threaded restatement of the reference Go path (paths relative to
 * /root/reference/shock-server/):
 *   node/file/index/record.go:34-90      record driver
 *   node/file/index/line.go:33-85        line driver
 *   node/file/format/multi/multi.go:43-62  format detection
 *   node/file/format/fastq/fastq.go:134-213, fasta/fasta.go:93-140, sam/sam.go:83-98,
 *   line/line.go:37-45                   per-record scanners
 * Parity is pinned by SURVEY.md Appendix B KATs and the fixture tables in tests/golden/
 * (the Go reference itself cannot be built here: no Go toolchain).
 */
#ifndef SHOCKIDX_ORACLE_H
#define SHOCKIDX_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_FMT_NONE = 0, ORC_FMT_FASTA = 1, ORC_FMT_FASTQ = 2, ORC_FMT_SAM = 3 };

/* multi.go:43-62 -- first match in fixed order fasta, fastq, sam over the zero-padded
 * first 32768 bytes.  Returns ORC_FMT_*.  `mask` (optional) receives a bitmask of every
 * validator that matches (bit fmt-1), to expose the reference's map-order ambiguity. */
int oracle_detect(const uint8_t *data, size_t n, int *mask);
/* Regex.MatchString on data itself (no zero padding): bit 0 fasta, 1 fastq, 2 sam */
int oracle_regex_match(const uint8_t *data, size_t n);

/* record.go:34-90.  fmt = ORC_FMT_* or -1 for auto-detection.
 * Returns 0 on success, 1 on a reader/format error (message in err), -1 on allocation
 * failure.  *errn = message length (FASTA snippets may hold NUL bytes). *rows (malloc'ed, free with oracle_free) holds *count pairs
 * {u64 offset, u64 length}: on error, the records emitted before the error. */
int oracle_record_index(const uint8_t *data, size_t n, int fmt, uint64_t **rows,
                        uint64_t *count, char *err, size_t errlen, size_t *errn);

/* line.go:33-85 (final entry always emitted). */
int oracle_line_index(const uint8_t *data, size_t n, uint64_t **rows, uint64_t *count);

/* Go bytes.TrimSpace on [s, s+n): writes trimmed bounds. Exposed for unit tests. */
void oracle_trim_space(const uint8_t *s, size_t n, size_t *lo, size_t *hi);

/* index/subset.go:133-303 CreateSubsetNodeIndexes for an "array" parent index (subset_oracle.c).
 * ids: the uploaded subset_indices file; parent: the parent .idx rows; ilength: the parent
 * index's TotalUnits.  Returns 0, 1 (Go error text in err) or -1 (allocation).  *rows /
 * *runs (malloc'ed, oracle_free) receive the subset index and the compressed .subset.idx
 * rows; *size = oSize.  Messages longer than errlen-1 bytes are truncated. */
int oracle_subset(const uint8_t *ids, size_t n, const uint64_t *parent, uint64_t parent_count, int64_t ilength,
                  uint64_t **rows, uint64_t *count, uint64_t **runs, uint64_t *nruns, uint64_t *size, char *err,
                  size_t errlen, size_t *errn);

/* index/index.go:67-117 Idx.Part and :119-193 Idx.Range over an .idx file given as its
 * nrows whole rows (rows == NULL: the file is missing).  Return 0, or 1 with Go's error text
 * in err (IndexNoFile / InvalidIndexRange / IndexOutBounds); -1 on allocation failure.
 * Range: *recs (malloc'ed, oracle_free) receives *nrecs {pos, length} pairs (part_oracle.c). */
int oracle_idx_part(const uint64_t *rows, uint64_t nrows, const char *part, int64_t idx_length, int64_t *pos,
                    int64_t *length, char *err, size_t errlen);
int oracle_idx_range(const uint64_t *rows, uint64_t nrows, const char *part, int64_t idx_length, int64_t **recs,
                     uint64_t *nrecs, char *err, size_t errlen);
/* index/subset.go:36-128 CreateSubsetIndex: the subset rows (*rows, oracle_free) and
 * (count, size), or (-1, -1) and Go's error text (returns 1). */
int oracle_create_subset_index(const uint8_t *ids, size_t n, const uint64_t *parent, uint64_t parent_count,
                               int64_t ilength, uint64_t **rows, int64_t *count, int64_t *size, char *err,
                               size_t errlen, size_t *errn);

/* node/filter/fq2fa (kind 1) and anonymize over FASTQ (kind 2) (filter_oracle.c): the byte
 * stream the filter delivers (*out malloc'ed, oracle_free), *count records; returns 0 (EOF),
 * 1 (a Read error: Go's text in err), 2 (anonymize of a FASTA / SAM section: not restated)
 * or -1 (allocation). */
int oracle_filter_fastq(const uint8_t *data, size_t n, int kind, uint8_t **out, size_t *outlen, uint64_t *count,
                        char *err, size_t errlen);

/* strconv.Quote restated (exposed for tests); returns the quoted length (may exceed cap). */
size_t oracle_go_quote(const uint8_t *s, size_t n, char *out, size_t cap);

/* index/chunkrecord.go:41-99 for a non-subset node (chunk_oracle.c).  fmt = ORC_FMT_* or -1
 * (detect); chunk = conf.CHUNK_SIZE (1048576).  Returns 0, 1 (detection failed: "Invalid file
 * type for filter", no row), 2 (SAM: the reference loops forever), -1 (allocation). */
int oracle_chunkrecord(const uint8_t *data, size_t n, int fmt, int64_t chunk, uint64_t **rows, uint64_t *count,
                       char *err, size_t errlen);
/* index/chunkrecord.go:100-228, subset node (format != "matrix"): the subset node's record
 * index rows grouped into chunks of rows; out rows (16 * first row, 16 * rows). */
int oracle_chunkrecord_subset(const uint64_t *ri, uint64_t nrows, uint64_t **rows, uint64_t *count);
/* End of the leftmost-first match of fastq.Record anchored at s in b[0..n), or -1. */
long oracle_fq_record_at(const uint8_t *b, long n, long s);

void oracle_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
