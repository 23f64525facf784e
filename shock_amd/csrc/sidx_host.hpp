// sidx_host.hpp -- host-side helpers of libshockidx shared between translation units
// (defined in sidx_capi.cpp): staging of host bytes into a context's HBM input buffer and the
// table copy-out through its pinned staging buffers, Go's status texts.  Internal: not part
// of the C ABI (include/shockidx.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shockidx.h"

namespace sidx_host {

double now_ms();
int set_msg(shockidx_result *r, int code, const char *msg);
int set_hip(shockidx_result *r, hipError_t e, const char *what);
// Go's text for a FASTQ status code (ST_*), nullptr for codes without one
const char *status_message(uint32_t code);

int ctx_device(shockidx_ctx *c);
hipStream_t ctx_stream(shockidx_ctx *c);
// Bytes [off, off + len) of a host buffer (src) or of a file (src null: fd) into the context's
// input buffer (grown as needed, 16-byte aligned); *d_out = its device address.
int ctx_stage(shockidx_ctx *c, const void *src, int fd, uint64_t off, uint64_t len, const uint8_t **d_out,
              shockidx_result *res);
// bytes of device memory (on the context's device) into host memory through pinned staging
int ctx_to_host(shockidx_ctx *c, const void *d_src, uint64_t bytes, void *dst, shockidx_result *res);
// a row table the caller frees with free() / shockidx_free (2 MiB aligned when large)
uint64_t *alloc_rows(uint64_t bytes);
// Device memory; node = a node body the tile passes stream (the context's input staging,
// shockidx_dev_alloc_node): physically contiguous when the driver can (hipDeviceMallocContiguous),
// else plain hipMalloc.  10 GiB FASTQ, interleaved allocations in one process on MI355X:
// k_fq_tiles 1.93-1.95 ms (median) from contiguous memory in 5 of 5 allocations, 1.92-2.15 ms from
// hipMalloc'd memory depending on where it landed (tools/placement_probe2.py,
// profiles/r04/placement2b.txt).  Written buffers (row tables, tile words) stay plain: the row
// placement ran 0.13 -> 0.18 ms into contiguous memory.  Freed with hipFree.
hipError_t dev_malloc(void **p, size_t bytes, bool node);

}  // namespace sidx_host
