/* shockidx.h -- C ABI of libshockidx, the MI355X (gfx950) record indexer for Shock.
 *
 * Drop-in boundary: this library replaces the body of the two Shock indexers that scan a
 * node's file, behind Shock's own plug-in registry
 *     index.Indexers = map[string]indexerFunc{ "record": ..., "line": ... }
 *     (shock-server/node/file/index/index.go:21-28)
 *     type Indexer interface { Create(string) (int64, string, error); Close() error }
 *     (shock-server/node/file/index/index.go:30-33)
 * A cgo shim registers NewGPURecordIndexer / NewGPULineIndexer under the
 * same keys; controller/node/index/index.go:176 and node/index.go:108-120 pick them up
 * unchanged.  Plain pointers and sizes only; no HIP or torch types in the signatures.
 *
 * Entry points and the reference code each one replaces (paths relative to
 * /root/reference/shock-server/):
 *   shockidx_create        record.Create / lineRecord.Create: index/record.go:34-90,
 *                          index/line.go:33-85 (scan + 16 MiB block writes + temp/rename)
 *   shockidx_build_fd      the scan of Create over the caller's *os.File (node/index.go:109-120)
 *   shockidx_build_host    the same over a POSTed body already in host memory
 *   shockidx_build_device  the device-resident core (input in HBM, table left in HBM)
 *   shockidx_detect        multi.Reader.DetermineFormat: format/multi/multi.go:43-62
 *   shockidx_write_idx     the .idx output protocol: index/record.go:35-41,65-87
 *   shockidx_chunkrecord_device  chunkRecord.Create (non-subset node): index/chunkrecord.go:41-99
 *   shockidx_chunkrecord_fd      the same over the node's *os.File (chunkrecord.go:43-56 reads it)
 *   shockidx_chunkrecord_subset_device  chunkRecord.Create for subset nodes (chunkrecord.go:100-228)
 *                          with fastq.go:216-243 / fasta.go:143-173 SeekChunk
 *
 * Semantics: results are bit-identical to the Go path on the same bytes, including the
 * exact error strings (fastq.go:156-207, fasta.go:120, errors.go:20) and the record count
 * reached before an error (the `count` Create returns alongside err).
 */
#ifndef SHOCKIDX_H
#define SHOCKIDX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 5: shockidx_slab.seq, the summary's build tag and shockidx_slab_combine's expect_seq (a stale
 *    summary is refused); row-capacity errors of build_device / chunkrecord / subset are
 *    SHOCKIDX_ESPACE (4 returned SHOCKIDX_EINVAL); whole-file builds check their own table's
 *    end invariants (SHOCKIDX_EINTERNAL instead of a short table) */
#define SHOCKIDX_ABI_VERSION 5

/* index kinds = the registry keys served (index/index.go:21-28) */
enum shockidx_kind { SHOCKIDX_RECORD = 0, SHOCKIDX_LINE = 1 };

/* formats (format/multi/multi.go:17-27) */
enum shockidx_format {
  SHOCKIDX_FMT_AUTO = -1, /* detect like multi.DetermineFormat (order fasta, fastq, sam) */
  SHOCKIDX_FMT_NONE = 0,
  SHOCKIDX_FMT_FASTA = 1,
  SHOCKIDX_FMT_FASTQ = 2,
  SHOCKIDX_FMT_SAM = 3,
  SHOCKIDX_FMT_LINE = 4 /* the line indexer (no detection, format/line/line.go) */
};

/* return codes */
enum shockidx_status {
  SHOCKIDX_OK = 0,
  SHOCKIDX_EFORMAT = 1,    /* reader/format error: Go's error string in result.err */
  SHOCKIDX_EINVAL = -1,
  SHOCKIDX_EHIP = -2,      /* HIP runtime error (result.err holds hipGetErrorString) */
  SHOCKIDX_ENOMEM = -3,
  SHOCKIDX_EIO = -4,       /* read/write/rename failure (errno text in result.err) */
  SHOCKIDX_EINTERNAL = -5, /* invariant violated on device (never expected) */
  SHOCKIDX_ESPACE = -6     /* output / record capacity too small: result.size (bytes) or
                              result.count (records) holds what the call needs */
};

typedef struct shockidx_ctx shockidx_ctx; /* one per concurrent caller (goroutine) */

typedef struct shockidx_result {
  uint64_t count;      /* records produced: Create's `count` (records before an error) */
  int32_t format;      /* SHOCKIDX_FMT_* that was indexed */
  int32_t status;      /* SHOCKIDX_OK or SHOCKIDX_EFORMAT (negative codes: system errors) */
  uint64_t err_len;    /* bytes in err (the FASTA message embeds raw file bytes) */
  char err[256];       /* Go error text, NUL-terminated */
  double kernel_ms;    /* device time of the index kernels (HIP events) */
  double h2d_ms;       /* host -> device staging time (host/fd entry points) */
  double d2h_ms;       /* table device -> host time */
  double total_ms;     /* wall time of the call */
  uint32_t path;       /* the build that ran last: 1 tile pass (one read of the input), 2 two-pass,
                          3 slab-pipelined build (build_host of a pinned FASTQ body, build_fd / create),
                          4 the same through two slab slots within the context's device cap
                          (shockidx_ctx_set_dev_cap) */
  uint32_t reruns;     /* builds re-run: a row-capacity overflow, a failed format speculation */
  double index_ms;     /* device time of the main index kernel alone (last pass) */
  uint64_t state_out;  /* format monoid state after the input (slab composition) */
  uint32_t term_code;  /* device status of the terminating record (diagnostic) */
  uint32_t flags;      /* device flags (diagnostic) */
  uint32_t fixups;     /* records / tiles re-validated from global memory (diagnostic) */
  uint32_t fix_tiles;  /* of which whole tiles re-indexed (diagnostic) */
} shockidx_result;

/* Context: owns a HIP stream on `device` plus cached device / pinned workspaces.
 * Thread-compatible: use one context per thread (or serialise calls on a context). */
int shockidx_ctx_create(int device, shockidx_ctx **out);
void shockidx_ctx_destroy(shockidx_ctx *ctx);
/* A context keeps its device workspaces (input staging, row table, tile status, scan and
 * subset space) grown to the largest call so far.  shockidx_ctx_trim frees them down to at
 * most keep_bytes (0: all; they regrow on demand); shockidx_ctx_workspace_bytes reports the
 * bytes held.  With SHOCKIDX_WORKSPACE_CAP=<bytes> in the environment at ctx_create, the
 * host-facing calls (build_host, build_fd, create, chunkrecord_fd) trim to the cap as they
 * return.  Not thread-safe against a concurrent call on the same context. */
int shockidx_ctx_trim(shockidx_ctx *ctx, uint64_t keep_bytes);
/* Device bytes one fd build (shockidx_build_fd / shockidx_create: the drop-in's Create) may hold;
 * 0 (default, or SHOCKIDX_DEV_CAP="2G" at context creation): what the device has free.  A node
 * whose one-pass build would not fit is indexed through two slab slots sized to the cap, so the
 * footprint does not grow with the node (record.go streams through a 4 KiB bufio.Reader,
 * record.go:51-83).  Replaces nothing in the reference (Go has no device memory); the shim
 * sets it from its pool configuration. */
int shockidx_ctx_set_dev_cap(shockidx_ctx *ctx, uint64_t bytes);
uint64_t shockidx_ctx_workspace_bytes(shockidx_ctx *ctx);

/* Device-resident build.  d_data: n bytes in HBM (16-byte aligned); d_rows: row_cap rows of
 * 16 bytes ({u64 offset, u64 length} LE).  stream: hipStream_t or NULL for the context's.
 * On return result->count rows are valid; if count > row_cap returns SHOCKIDX_ESPACE with
 * result->count = rows required (nothing beyond row_cap was written). */
int shockidx_build_device(shockidx_ctx *ctx, const void *d_data, uint64_t n, int kind, int fmt,
                          void *d_rows, uint64_t row_cap, void *stream,
                          shockidx_result *result);

/* Host-memory build (POSTed body).  *rows receives a malloc'ed table of result->count rows
 * (free with shockidx_free); on SHOCKIDX_EFORMAT it holds the rows before the error. */
int shockidx_build_host(shockidx_ctx *ctx, const void *data, uint64_t n, int kind, int fmt,
                        uint64_t **rows, shockidx_result *result);

/* Pin (hipHostRegister) / unpin a caller buffer, e.g. a node body kept in host memory for
 * several builds.  build_host detects pinned input (registered or hipHostMalloc'ed) and DMAs it
 * to HBM directly instead of copying it through the context's pinned staging. */
int shockidx_host_register(shockidx_ctx *ctx, void *p, uint64_t n);
int shockidx_host_unregister(shockidx_ctx *ctx, void *p);

/* File build over an open descriptor (not closed; read with pread from offset 0). */
int shockidx_build_fd(shockidx_ctx *ctx, int fd, uint64_t n, int kind, int fmt, uint64_t **rows,
                      shockidx_result *result);

/* Indexer.Create(outPath): build from fd then write <tmpdir>/<rand><rand>.idx and rename it
 * to outpath (record.go:35,87).  On a format error nothing is renamed into outpath. */
int shockidx_create(shockidx_ctx *ctx, int fd, uint64_t n, int kind, const char *tmpdir,
                    const char *outpath, shockidx_result *result);

/* Write `count` rows as an .idx file through a temp file + rename. */
int shockidx_write_idx(const uint64_t *rows, uint64_t count, const char *tmpdir,
                       const char *outpath, char *err, size_t errlen);

/* multi.DetermineFormat on the first min(n, 32768) bytes, run on the device.
 * *fmt = SHOCKIDX_FMT_FASTA/FASTQ/SAM or NONE; *mask = bit (f-1) set for every matching
 * validator (the reference ranges over a Go map, so overlapping matches are ambiguous). */
int shockidx_detect(shockidx_ctx *ctx, const void *data, uint64_t n, int *fmt, int *mask);

/* Device memory helpers on the context's device (for callers without their own HIP
 * allocator, e.g. a Go server holding a node resident in HBM).  Copies are synchronous. */
int shockidx_dev_alloc(shockidx_ctx *ctx, uint64_t bytes, void **d_ptr);
/* Device memory for a node body kept resident in HBM (what shockidx_build_device streams):
 * physically contiguous when the driver can provide it (the tile passes read it ~10 % faster
 * than memory hipMalloc places badly), else the same as shockidx_dev_alloc.  Free with
 * shockidx_dev_free. */
int shockidx_dev_alloc_node(shockidx_ctx *ctx, uint64_t bytes, void **d_ptr);
int shockidx_dev_free(shockidx_ctx *ctx, void *d_ptr);
int shockidx_memcpy_h2d(shockidx_ctx *ctx, void *d_dst, const void *src, uint64_t bytes);
int shockidx_memcpy_d2h(shockidx_ctx *ctx, void *dst, const void *d_src, uint64_t bytes);
int shockidx_memset(shockidx_ctx *ctx, void *d_dst, int value, uint64_t bytes);
int shockidx_sync(shockidx_ctx *ctx); /* hipDeviceSynchronize on the context's device */
void *shockidx_stream(shockidx_ctx *ctx); /* the context's hipStream_t */

/* ---- Multi-GPU slabs ------------------------------------------------
 * A file too large for one GPU (or split for speed) is cut into byte slabs, one per GPU.
 * Each GPU indexes its slab against a *guessed* incoming reader state (the FASTQ line
 * phase, the FASTA '\n'-since-'>' bit, the SAM open-line class), the GPUs all-gather one
 * 64-byte summary each over RCCL, and a tiny device kernel folds the summaries in slab
 * order: it yields every slab's true incoming state (a wrong guess is re-run; it never is
 * on real data), the global number of the slab's first record and the global result. */
typedef struct shockidx_slab {
  const void *d_data; /* device pointer to the slab's first byte (16-byte aligned unless n == 0) */
  uint64_t n;         /* bytes owned by the slab (records starting here belong to it) */
  uint64_t end;       /* readable bytes from d_data: n + halo (records crossing the slab end) */
  uint64_t front;     /* readable bytes before d_data (>= 16; guesses look back up to 64 KiB) */
  uint64_t base;      /* file offset of d_data[0] */
  int32_t is_first;   /* slab starts at file offset 0 */
  int32_t is_last;    /* end is the end of the file */
  uint32_t seq;       /* the caller's build tag, stamped into the slab's summary */
  uint32_t reserved;
} shockidx_slab;

typedef struct shockidx_slab_summary { /* exchanged between GPUs; 64 bytes */
  uint64_t agg;      /* monoid aggregate of the slab bytes */
  uint64_t state_in; /* state the slab was indexed with */
  uint64_t key;      /* first-bad key (local record number << 28 | tile << 4 | status) or ~0 */
  uint64_t natural;  /* local record count if nothing terminated inside the slab */
  uint64_t row_base; /* local record number of the slab's first row */
  uint64_t err_pos;  /* FASTA error piece (file offset, length) */
  uint64_t err_len;
  uint16_t fmt;
  uint16_t flags;
  uint32_t seq;      /* shockidx_slab.seq of the build that wrote it */
} shockidx_slab_summary;

typedef struct shockidx_slab_plan { /* folded by every rank from all summaries */
  uint64_t state_in;     /* this slab's true incoming state */
  uint64_t first_record; /* global record number of this slab's rows[0] */
  uint64_t count;        /* global record count (Create's `count`) */
  uint64_t err_pos, err_len;
  uint32_t code;         /* device status of the terminating record */
  int32_t err_rank;      /* slab holding the error bytes (-1: none) */
  uint32_t inconsistent; /* bitmask of slabs whose guess was wrong (re-run them) */
  uint32_t flags;        /* 2: a device invariant failed, 4: a record ran past a halo,
                            32: a summary's seq was not the expected one (stale) */
} shockidx_slab_plan;

/* Guess the incoming state of a slab from its first bytes and the bytes before it. */
int shockidx_slab_guess(shockidx_ctx *ctx, const shockidx_slab *slab, int fmt, uint64_t *state_guess);
/* Index one slab with `state_in`; rows of the slab's records go to d_rows[0..), the 64-byte
 * summary to d_summary (device memory).  Asynchronous on the context stream. */
int shockidx_slab_index(shockidx_ctx *ctx, const shockidx_slab *slab, int fmt, uint64_t state_in,
                        void *d_rows, uint64_t row_cap, void *d_summary, shockidx_result *result);
/* Fold `world` gathered summaries (device memory, slab order) into this rank's plan.
 * expect_seq (host memory, `world` tags, or NULL: unchecked): the seq each slab's summary must
 * carry -- the tag its latest shockidx_slab_index was given; any other sets plan->flags 32. */
int shockidx_slab_combine(shockidx_ctx *ctx, const void *d_all, int world, int rank, int fmt,
                          const uint32_t *expect_seq, shockidx_slab_plan *plan);

/* RCCL communicator (one per process / GPU).  The 128-byte unique id is created by rank 0
 * and broadcast by the caller (e.g. over a CPU process group). */
typedef struct shockidx_comm shockidx_comm;
int shockidx_comm_unique_id(void *id128);
int shockidx_comm_init(shockidx_ctx *ctx, int world, int rank, const void *id128, shockidx_comm **out);
int shockidx_comm_allgather(shockidx_comm *comm, const void *d_send, void *d_recv, uint64_t bytes);
int shockidx_comm_destroy(shockidx_comm *comm);
/* ranks the communicator spans (ncclCommCount): what a run reports as the ranks its
 * all-gather actually crossed over RCCL (bench.py --gpus N: "rccl_ranks") */
int shockidx_comm_count(const shockidx_comm *comm, int *nranks);

/* ---- One file across several GPUs from one process -------------------
 * The Shock server is one process: node.AsyncIndexer builds an index in a goroutine
 * (node/index.go:107-121) and never sees ranks.  A multi-device group cuts the node file into
 * byte slabs, one per device, stages each slab (plus 64 KiB before and a 4 MiB halo after it)
 * into its GPU, indexes them concurrently with the tile passes against guessed incoming
 * states, all-gathers the 64-byte slab summaries over RCCL (one communicator per device,
 * ncclCommInitAll; 64 B x n is all that crosses xGMI), folds them on every device, re-runs a
 * slab whose guess was wrong and concatenates the owned rows: the table, count and Go error
 * text equal shockidx_build_host's.  devices[k] takes slab k; a device may be listed more than
 * once (its slabs then run one after another and the summaries go through host memory).  A
 * record longer than the halo crossing a slab end is built on devices[0] alone. */
typedef struct shockidx_multi shockidx_multi;
/* visible GPUs (hipGetDeviceCount); 0 when there is no usable GPU */
int shockidx_device_count(void);
int shockidx_multi_create(const int *devices, int n_devices, shockidx_multi **out);
void shockidx_multi_destroy(shockidx_multi *m);
/* 1: the summaries are all-gathered over RCCL; 0: through host memory */
int shockidx_multi_rccl(const shockidx_multi *m);
/* shockidx_build_host / shockidx_build_fd / shockidx_create across the group's devices */
int shockidx_multi_build_host(shockidx_multi *m, const void *data, uint64_t n, int kind, int fmt, uint64_t **rows,
                              shockidx_result *result);
int shockidx_multi_build_fd(shockidx_multi *m, int fd, uint64_t n, int kind, int fmt, uint64_t **rows,
                            shockidx_result *result);
int shockidx_multi_create_index(shockidx_multi *m, int fd, uint64_t n, int kind, const char *tmpdir,
                                const char *outpath, shockidx_result *result);
/* Device-resident form (benchmarks; a server keeping node bodies in HBM).  Slab k of a file of
 * `size` bytes owns [lo[k], hi[k]) and is held as window [wlo[k], whi[k]) at d_win[k] on
 * devices[k] (shockidx_multi_plan).  Rows stay on the devices: d_rows[k] (row_cap[k] rows)
 * receives the slab's rows, the first rows_owned[k] of which are global records
 * first_record[k]..  Returns like shockidx_build_device (result->count = global count); a row_cap[k]
 * too small for its slab returns SHOCKIDX_ESPACE with result->count = the most rows any short
 * slab needs. */
int shockidx_multi_plan(const shockidx_multi *m, uint64_t size, uint64_t *lo, uint64_t *hi, uint64_t *wlo,
                        uint64_t *whi);
int shockidx_multi_build_resident(shockidx_multi *m, uint64_t size, int kind, int fmt, const void *const *d_win,
                                  void *const *d_rows, const uint64_t *row_cap, uint64_t *first_record,
                                  uint64_t *rows_owned, shockidx_result *result);

/* ---- Subset nodes (BASELINE config C4) -------------------------
 * A subset node is built from an uploaded list of 1-based record ids (one per line) over the
 * parent's record index: index/subset.go:133-303 CreateSubsetNodeIndexes writes one parent
 * row per id (<node>/idx/<parent index>.idx) and the maximal runs of contiguous rows
 * (<node>/<id>.subset.idx); reading the subset node streams those runs of the parent file
 * (controller/node/single.go:500-517, request/streamer.go:58-117). */
typedef struct shockidx_subset_result {
  uint64_t count;    /* oCount: subset index rows (rows written before an error) */
  uint64_t runs;     /* coCount: compressed index rows */
  uint64_t size;     /* oSize: bytes of the subset node (sum of the row lengths) */
  int32_t status;    /* SHOCKIDX_OK, SHOCKIDX_EFORMAT (Go's error text in err) or < 0 */
  uint32_t pad;
  uint64_t err_len;
  char err[256];
  double kernel_ms;  /* device time: the subset kernels (index) / k_gather (gather) */
  double total_ms;
  double gather_ms;  /* shockidx_subset_node: device time of k_gather */
} shockidx_subset_result;

/* CreateSubsetNodeIndexes on device memory.  d_ids: the id text (ids_len bytes, 16-byte
 * aligned); d_parent: parent_count parent rows {u64 off, u64 len}; ilength: the parent
 * index's TotalUnits.  Writes result->count rows to d_rows and result->runs rows to d_runs
 * (capacities in rows; a short capacity returns SHOCKIDX_ESPACE with the needed counts). */
int shockidx_subset_index(shockidx_ctx *ctx, const void *d_ids, uint64_t ids_len, const void *d_parent,
                          uint64_t parent_count, int64_t ilength, void *d_rows, uint64_t rows_cap, void *d_runs,
                          uint64_t runs_cap, shockidx_subset_result *result);

/* The subset node's bytes: the runs of the parent file d_data (data_len bytes) concatenated
 * into d_out (out_cap bytes; result->size = bytes written, or needed with SHOCKIDX_ESPACE). */
int shockidx_subset_gather(shockidx_ctx *ctx, const void *d_data, uint64_t data_len, const void *d_runs,
                           uint64_t nruns, void *d_out, uint64_t out_cap, shockidx_subset_result *result);

/* shockidx_subset_index and shockidx_subset_gather in one call: the counts between them stay
 * on the device, so the host waits only for the id line count and the result.  d_runs is
 * required; d_out receives the node's bytes when the index succeeds (result->size bytes). */
int shockidx_subset_node(shockidx_ctx *ctx, const void *d_ids, uint64_t ids_len, const void *d_parent,
                         uint64_t parent_count, int64_t ilength, void *d_rows, uint64_t rows_cap, void *d_runs,
                         uint64_t runs_cap, const void *d_data, uint64_t data_len, void *d_out, uint64_t out_cap,
                         shockidx_subset_result *result);

/* CreateSubsetIndex (index/subset.go:36-128; caller node/index.go:103): the subset index of
 * a node from an id list over a parent index -- the per-id checks and rows of
 * shockidx_subset_index without the compressed index.  On a Go error (SHOCKIDX_EFORMAT)
 * result->count = result->size = UINT64_MAX, i.e. Go's (-1, -1, err) read as int64. */
int shockidx_create_subset_index(shockidx_ctx *ctx, const void *d_ids, uint64_t ids_len, const void *d_parent,
                                 uint64_t parent_count, int64_t ilength, void *d_rows, uint64_t rows_cap,
                                 shockidx_subset_result *result);

/* ---- Index read path: Idx.Part / Idx.Range ----------------------
 * index/index.go:67-117 and :119-193 (callers: controller/node/single.go:391-508,
 * controller/preauth/preauth.go:84) over an index resident in HBM: d_rows holds the .idx
 * file's nrows rows {u64 offset, u64 length}; d_rows == NULL stands for a missing file
 * (IndexNoFile).  part: the request's part value ("N" or "N-M", strconv.ParseInt semantics,
 * strings.Split on '-'); idx_length: the index's TotalUnits.  Go's error text
 * (IndexNoFile / InvalidIndexRange / IndexOutBounds) comes back with SHOCKIDX_EFORMAT.
 * A row past the table reads like Go's failed binary.Read: Part sees zeros; Range keeps the
 * last row it read.  Part: *pos, *length = Go's (pos, length), int64 arithmetic. */
int shockidx_idx_part(shockidx_ctx *ctx, const void *d_rows, uint64_t nrows, const char *part, int64_t idx_length,
                      int64_t *pos, int64_t *length, shockidx_subset_result *result);
/* Range: result->count {int64 pos, int64 length} records (maximal runs of contiguous rows) in
 * d_recs (recs_cap records; a short capacity returns SHOCKIDX_ESPACE with the needed count).
 * end < start gives an empty list, like Go's loop. */
int shockidx_idx_range(shockidx_ctx *ctx, const void *d_rows, uint64_t nrows, const char *part, int64_t idx_length,
                       void *d_recs, uint64_t recs_cap, shockidx_subset_result *result);

/* ---- Download filters --------------------------------------------
 * node/filter/filter.go:13-16 "fq2fa" (fq2fa/fq2fa.go:58-84) and "anonymize"
 * (anonymize/anonymize.go:28-56) over one FASTQ section (d_data, n bytes in HBM) into d_out:
 * the stream the filter's Read delivers -- every record fastq.Reader.Read (fastq.go:50-132)
 * returns without error, formatted (fq2fa: ">" ID "\n" Seq "\n"; anonymize: "@" counter
 * "\n" Seq "\n+\n" Qual "\n", counter from 1); a record returned together with io.EOF
 * (quality line without '\n' at the end) is dropped like the reference drops it.  Reader
 * errors end the stream: SHOCKIDX_EFORMAT with Go's text, result->count / size = records /
 * bytes delivered before it.  anonymize detects the format (multi.go:43-62): over a FASTA
 * section every sequence fasta.Reader.Read returns (fasta.go:40-88) as ">" counter "\n" Seq "\n"
 * (the sequence read with io.EOF dropped; "Invalid fasta entry" ends the stream), over a SAM
 * section every alignment line sam.Reader.Read returns (sam.go:44-81) as the trimmed line +
 * "\n" ("sam alignment fields less than 11").  A short out_cap returns SHOCKIDX_ESPACE with
 * result->size = the bytes needed. */
int shockidx_filter_device(shockidx_ctx *ctx, const char *filter, const void *d_data, uint64_t n, void *d_out,
                           uint64_t out_cap, shockidx_subset_result *result);

/* ---- chunkrecord index -----------------------------------------
 * Indexers["chunkrecord"] (index/index.go:21-28, index/chunkrecord.go:41-99): rows of ~chunk
 * bytes (conf.CHUNK_SIZE = 1048576 when chunk == 0) ending where fastq.Record's last match in
 * the chunk's final 32 KiB ends (FASTQ) or at the last "\n>" / "\r>" (FASTA); the last row
 * runs to the end of the file.  d_data: n bytes in HBM; d_rows: row_cap rows; at most
 * n / (chunk - 32767) + 2 rows are produced.  fmt AUTO detects like DetermineFormat; a SAM
 * file returns SHOCKIDX_EFORMAT (the reference loops forever there, sam.go:100-102). */
int shockidx_chunkrecord_device(shockidx_ctx *ctx, const void *d_data, uint64_t n, int fmt, uint64_t chunk,
                                void *d_rows, uint64_t row_cap, shockidx_result *result);
/* The same over an open descriptor (not closed; pread from offset 0, short reads retried):
 * *rows receives a malloc'ed table of result->count rows (free with shockidx_free). */
int shockidx_chunkrecord_fd(shockidx_ctx *ctx, int fd, uint64_t n, int fmt, uint64_t chunk, uint64_t **rows,
                            shockidx_result *result);

/* chunkRecord.Create for a subset node whose index format is not "matrix"
 * (index/chunkrecord.go:100-228): the subset node's record index (d_ri: nrows device rows,
 * whole rows only, as its ReadAt loop reads them) grouped into chunks of rows below 1 MiB;
 * d_rows receives result->count rows (16 * first row, 16 * rows): the "matrix" index. */
int shockidx_chunkrecord_subset_device(shockidx_ctx *ctx, const void *d_ri, uint64_t nrows, void *d_rows,
                                       uint64_t row_cap, shockidx_result *result);

void shockidx_free(void *p);
const char *shockidx_strerror(int code);
int shockidx_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SHOCKIDX_H */
