// gpurecord.go -- drop-in for Shock's record / line / chunkrecord indexers (package index),
// backed by libshockidx (hand-written gfx950 kernels behind the C ABI in include/shockidx.h).
//
// Copy this file into shock-server/node/file/index/ next to index.go.  It registers under the
// same keys as index.go:21-28 ("record", "line", "chunkrecord"), so
// controller/node/index/index.go:176 and node/index.go:108 pick it up unchanged.  Build the server with CGO_ENABLED=1 (the reference
// builds with 0, compile-server.sh:5) and point cgo at the library:
//
//	CGO_CFLAGS="-I<shockidx>/include" \
//	CGO_LDFLAGS="-L<shockidx>/shock_amd -lshockidx -Wl,-rpath,<shockidx>/shock_amd" \
//	go build ./shock-server
//
// Package-level names here avoid every import name and top-level identifier of the other files
// of package index (record.go and chunkrecord.go import format/multi as "multi", so the multi-GPU
// group is gpuMulti); tests/test_go_shim.py checks that mechanically against the reference files.
// No Go toolchain exists in this build environment, so this file is checked by that test only.
package index

/*
#cgo LDFLAGS: -lshockidx
#include <stdlib.h>
#include "shockidx.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"os"
	"runtime"
	"sync"
	"unsafe"

	"github.com/MG-RAST/Shock/shock-server/conf"
	"github.com/MG-RAST/Shock/shock-server/logger"
)

const (
	// concurrent GPU index builds per node (each one alone saturates HBM)
	gpuPoolSize = 2
	// device bytes a pooled context may keep cached between builds (shockidx_ctx_trim)
	gpuWorkspaceKeep = 1 << 30
	// device bytes one pooled build may hold (shockidx_ctx_set_dev_cap): a node whose one-pass
	// build needs more (above ~4.4 GiB) is indexed through two 1 GiB slab slots within it -- as
	// fast end to end as the whole node in HBM (47.3 against 47.0 GiB/s from the page cache, and
	// 47.7 against 46.7 with the pool's trim between builds: profiles/r06/calls/l), in 2.9 GB
	// instead of 12.8 GB for a 10 GiB node, so concurrent builds of any size fit one GPU together
	gpuDevCap = 8 << 30
	// below this one MI355X indexes the file in a few ms and PCIe staging dominates, so a
	// single pooled context is as fast and leaves the other GPUs free for concurrent builds
	gpuMultiThreshold = 8 << 30
	// a subset node's record index is read whole and held twice on the device for chunkrecord;
	// past this the Go indexer, which streams it 16 bytes at a time, builds it instead
	gpuChunkSubsetMax = 4 << 30
)

// gpuCtxPool is an explicit, bounded pool of libshockidx contexts on device 0.  A context is
// used by one goroutine at a time (builds of different nodes run in parallel goroutines,
// controller/node/index/index.go:320); get blocks while all are busy.  Unlike a sync.Pool,
// whose items the GC drops without shockidx_ctx_destroy (leaking a HIP stream and pinned
// staging each time), every context lives until gpuCtxPool.close destroys it.
type gpuCtxPool struct {
	free chan *C.shockidx_ctx
	all  []*C.shockidx_ctx
}

var (
	gpuPool *gpuCtxPool
	gpuOnce sync.Once
)

// gpuMulti is the multi-device group over every visible GPU (nil with fewer than two, or
// when the summaries could not go over RCCL).  A multi-device build uses every GPU, so the
// builds are serialised by the mutex.
var gpuMulti struct {
	sync.Mutex
	g *C.shockidx_multi
}

func newGPUCtxPool(device, n int) (*gpuCtxPool, error) {
	p := &gpuCtxPool{free: make(chan *C.shockidx_ctx, n)}
	for i := 0; i < n; i++ {
		var c *C.shockidx_ctx
		if rc := C.shockidx_ctx_create(C.int(device), &c); rc != C.SHOCKIDX_OK {
			p.close()
			return nil, fmt.Errorf("shockidx_ctx_create: %s", C.GoString(C.shockidx_strerror(rc)))
		}
		C.shockidx_ctx_set_dev_cap(c, C.uint64_t(gpuDevCap))
		p.all = append(p.all, c)
		p.free <- c
	}
	return p, nil
}

func (p *gpuCtxPool) get() *C.shockidx_ctx { return <-p.free }

func (p *gpuCtxPool) put(c *C.shockidx_ctx) {
	C.shockidx_ctx_trim(c, C.uint64_t(gpuWorkspaceKeep))
	p.free <- c
}

// close destroys every context (server shutdown); no build may be running.
func (p *gpuCtxPool) close() {
	for _, c := range p.all {
		C.shockidx_ctx_destroy(c)
	}
	p.all = nil
}

// initGPUMulti opens the multi-device group.  A group whose slab summaries would cross between
// GPUs through host memory (RCCL unavailable: shockidx_multi_rccl == 0) is refused and logged,
// so a mis-configured multi-GPU server runs single-GPU builds instead of a silent fallback.
func initGPUMulti() {
	n := int(C.shockidx_device_count())
	if n < 2 {
		return
	}
	devs := make([]C.int, n)
	for i := range devs {
		devs[i] = C.int(i)
	}
	var g *C.shockidx_multi
	if rc := C.shockidx_multi_create(&devs[0], C.int(n), &g); rc != C.SHOCKIDX_OK {
		logger.Errorf("shockidx: multi-GPU group over %d devices: %s", n, C.GoString(C.shockidx_strerror(rc)))
		return
	}
	if C.shockidx_multi_rccl(g) == 0 {
		logger.Errorf("shockidx: RCCL unavailable across %d GPUs; multi-GPU builds disabled", n)
		C.shockidx_multi_destroy(g)
		return
	}
	gpuMulti.g = g
}

// gpuInit runs on the first build, after main has called logger.Initialize (logger.Log is nil
// while package inits run, so nothing here may log from init).  It is also the first call into
// HIP: a server that never builds an index never initialises the GPU runtime.
func gpuInit() {
	if C.shockidx_device_count() < 1 {
		logger.Infof("shockidx: no usable GPU; indexing with the Go readers")
		return
	}
	p, err := newGPUCtxPool(0, gpuPoolSize)
	if err != nil {
		logger.Errorf("shockidx: %s; indexing with the Go readers", err.Error())
		return
	}
	gpuPool = p
	initGPUMulti()
}

// gpuIndexer replaces record (index/record.go:14-95) and lineRecord (index/line.go:13-91).
type gpuIndexer struct {
	f                       *os.File
	kind                    C.int // C.SHOCKIDX_RECORD or C.SHOCKIDX_LINE
	nType, snFormat, snPath string
}

// NewGPURecordIndexer has indexerFunc's signature (index.go:19); like NewRecordIndexer
// (record.go:23-32) it only keeps nType / snFormat / snIndexPath.
func NewGPURecordIndexer(f *os.File, nType string, snFormat string, snIndexPath string) Indexer {
	return &gpuIndexer{f: f, kind: C.SHOCKIDX_RECORD, nType: nType, snFormat: snFormat, snPath: snIndexPath}
}

// NewGPULineIndexer replaces NewLineIndexer (line.go:22-31).
func NewGPULineIndexer(f *os.File, nType string, snFormat string, snIndexPath string) Indexer {
	return &gpuIndexer{f: f, kind: C.SHOCKIDX_LINE, nType: nType, snFormat: snFormat, snPath: snIndexPath}
}

// goIndexer is the reference indexer for the same key, used when no GPU context could be made.
func (g *gpuIndexer) goIndexer() Indexer {
	if g.kind == C.SHOCKIDX_LINE {
		return NewLineIndexer(g.f, g.nType, g.snFormat, g.snPath)
	}
	return NewRecordIndexer(g.f, g.nType, g.snFormat, g.snPath)
}

// Create mirrors record.Create / lineRecord.Create: (count, "array", err).  The library reads
// the caller's file with pread (the offset is not moved, the file is not closed), writes
// PATH_DATA/temp/<rand>.idx and renames it to outPath only on success (record.go:35,87).
func (g *gpuIndexer) Create(outPath string) (count int64, format string, err error) {
	format = "array"
	st, err := g.f.Stat()
	if err != nil {
		return
	}
	gpuOnce.Do(gpuInit)
	if gpuPool == nil {
		// nothing above has read the file (Stat, no offset moved): the Go reader starts at 0
		return g.goIndexer().Create(outPath)
	}
	tmp := C.CString(conf.PATH_DATA + "/temp")
	out := C.CString(outPath)
	defer C.free(unsafe.Pointer(tmp))
	defer C.free(unsafe.Pointer(out))

	var res C.shockidx_result
	var rc C.int
	if gpuMulti.g != nil && st.Size() >= gpuMultiThreshold {
		// a large node on a multi-GPU host: one byte slab per GPU, one RCCL all-gather
		gpuMulti.Lock()
		rc = C.shockidx_multi_create_index(gpuMulti.g, C.int(g.f.Fd()), C.uint64_t(st.Size()), g.kind, tmp, out, &res)
		gpuMulti.Unlock()
	} else {
		ctx := gpuPool.get()
		defer gpuPool.put(ctx)
		// the context's HIP stream is used from one OS thread for the whole call
		runtime.LockOSThread()
		defer runtime.UnlockOSThread()
		rc = C.shockidx_create(ctx, C.int(g.f.Fd()), C.uint64_t(st.Size()), g.kind, tmp, out, &res)
	}
	return int64(res.count), format, gpuError(rc, &res)
}

// gpuError is the Go error of a libshockidx call: nil, the Go reader's error text byte for byte
// (fastq.go:156-207, fasta.go:120), or the library's own failure.
func gpuError(rc C.int, res *C.shockidx_result) error {
	switch rc {
	case C.SHOCKIDX_OK:
		return nil
	case C.SHOCKIDX_EFORMAT:
		return errors.New(C.GoStringN(&res.err[0], C.int(res.err_len)))
	default:
		return fmt.Errorf("shockidx: %s: %s", C.GoString(C.shockidx_strerror(rc)),
			C.GoStringN(&res.err[0], C.int(res.err_len)))
	}
}

// Close mirrors record.Close (record.go:92-95): the file's Close error is discarded.
// node.AsyncIndexer never calls it; it closes the file itself (node/index.go:113).
func (g *gpuIndexer) Close() (err error) {
	g.f.Close()
	return
}

// gpuChunkIndexer replaces chunkRecord (index/chunkrecord.go:15-228).
type gpuChunkIndexer struct {
	f                       *os.File
	nType, snFormat, snPath string
}

// NewGPUChunkRecordIndexer replaces NewChunkRecordIndexer (chunkrecord.go:28-39).
func NewGPUChunkRecordIndexer(f *os.File, nType string, snFormat string, snIndexPath string) Indexer {
	return &gpuChunkIndexer{f: f, nType: nType, snFormat: snFormat, snPath: snIndexPath}
}

// Create mirrors chunkRecord.Create.  A node's file: rows of about conf.CHUNK_SIZE bytes that
// end where SeekChunk says (chunkrecord.go:41-99), format "array".  A subset node: its record
// index's rows grouped into chunks below 1 MiB (chunkrecord.go:100-228), format "matrix"; a
// subset node of a "matrix" index is refused with the reference's error text.
func (g *gpuChunkIndexer) Create(outPath string) (count int64, format string, err error) {
	if g.nType == "subset" && g.snFormat == "matrix" {
		err = errors.New("Shock does not currently support the creation of chunkrecord indices for subset nodes derived from a matrix formatted index.")
		return
	}
	gpuOnce.Do(gpuInit)
	if gpuPool == nil {
		return NewChunkRecordIndexer(g.f, g.nType, g.snFormat, g.snPath).Create(outPath)
	}
	format = "array"
	var ri []byte
	if g.nType == "subset" {
		format = "matrix"
		var fi os.FileInfo
		if fi, err = os.Stat(g.snPath); err != nil {
			return
		}
		if fi.Size() > gpuChunkSubsetMax {
			return NewChunkRecordIndexer(g.f, g.nType, g.snFormat, g.snPath).Create(outPath)
		}
		// the subset node's record index, whole 16-byte rows (its ReadAt loop stops at a partial one)
		if ri, err = os.ReadFile(g.snPath); err != nil {
			return
		}
	}
	st, err := g.f.Stat()
	if err != nil {
		return
	}
	ctx := gpuPool.get()
	defer gpuPool.put(ctx)
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()

	var res C.shockidx_result
	var rows *C.uint64_t
	var rc C.int
	if g.nType != "subset" {
		rc = C.shockidx_chunkrecord_fd(ctx, C.int(g.f.Fd()), C.uint64_t(st.Size()), C.SHOCKIDX_FMT_AUTO,
			C.uint64_t(conf.CHUNK_SIZE), &rows, &res)
	} else {
		rc, rows = gpuChunkSubset(ctx, ri, &res)
	}
	defer C.free(unsafe.Pointer(rows))
	count = int64(res.count)
	if err = gpuError(rc, &res); err != nil {
		return
	}
	tmp := C.CString(conf.PATH_DATA + "/temp")
	out := C.CString(outPath)
	defer C.free(unsafe.Pointer(tmp))
	defer C.free(unsafe.Pointer(out))
	var ebuf [256]C.char
	if wr := C.shockidx_write_idx(rows, res.count, tmp, out, &ebuf[0], C.size_t(len(ebuf))); wr != C.SHOCKIDX_OK {
		err = fmt.Errorf("shockidx: %s: %s", C.GoString(C.shockidx_strerror(wr)), C.GoString(&ebuf[0]))
	}
	return
}

// Close mirrors chunkRecord.Close (chunkrecord.go:230-233).
func (g *gpuChunkIndexer) Close() (err error) {
	g.f.Close()
	return
}

// gpuChunkSubset groups a subset node's record index (ri: its .idx bytes) on the device and
// returns the rows in C memory (free with C.free).
func gpuChunkSubset(ctx *C.shockidx_ctx, ri []byte, res *C.shockidx_result) (C.int, *C.uint64_t) {
	nrows := uint64(len(ri) / 16)
	var dri, drows unsafe.Pointer
	if rc := C.shockidx_dev_alloc(ctx, C.uint64_t(16*nrows+16), &dri); rc != C.SHOCKIDX_OK {
		return rc, nil
	}
	defer C.shockidx_dev_free(ctx, dri)
	if rc := C.shockidx_dev_alloc(ctx, C.uint64_t(16*nrows+16), &drows); rc != C.SHOCKIDX_OK {
		return rc, nil
	}
	defer C.shockidx_dev_free(ctx, drows)
	if nrows > 0 {
		if rc := C.shockidx_memcpy_h2d(ctx, dri, unsafe.Pointer(&ri[0]), C.uint64_t(16*nrows)); rc != C.SHOCKIDX_OK {
			return rc, nil
		}
	}
	// at most one chunk per row
	if rc := C.shockidx_chunkrecord_subset_device(ctx, dri, C.uint64_t(nrows), drows, C.uint64_t(nrows+1), res); rc != C.SHOCKIDX_OK {
		return rc, nil
	}
	rows := (*C.uint64_t)(C.malloc(C.size_t(16*res.count + 16)))
	if rows == nil {
		return C.SHOCKIDX_ENOMEM, nil
	}
	if rc := C.shockidx_memcpy_d2h(ctx, unsafe.Pointer(rows), drows, C.uint64_t(16*res.count)); rc != C.SHOCKIDX_OK {
		C.free(unsafe.Pointer(rows))
		return rc, nil
	}
	return C.SHOCKIDX_OK, rows
}

// init registers the GPU constructors under the reference's keys.  It makes no HIP call: the
// runtime starts, and the device count is read, on the first build (gpuInit); with no usable GPU
// every Create runs the Go indexer it replaces.
func init() {
	Indexers["record"] = NewGPURecordIndexer
	Indexers["line"] = NewGPULineIndexer
	Indexers["chunkrecord"] = NewGPUChunkRecordIndexer
}
