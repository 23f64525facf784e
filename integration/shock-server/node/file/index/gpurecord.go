// gpurecord.go -- drop-in for Shock's record / line indexers (package index), backed by
// libshockidx (hand-written gfx950 kernels behind the C ABI in include/shockidx.h).
//
// Copy this file into shock-server/node/file/index/ next to index.go.  It registers under the
// same keys as index.go:21-28 ("record", "line"), so controller/node/index/index.go:176 and
// node/index.go:108 pick it up unchanged.  Build the server with CGO_ENABLED=1 (the reference
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
	// below this one MI355X indexes the file in a few ms and PCIe staging dominates, so a
	// single pooled context is as fast and leaves the other GPUs free for concurrent builds
	gpuMultiThreshold = 8 << 30
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
// while package inits run, so nothing here may log from init).
func gpuInit() {
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
	count = int64(res.count)
	switch rc {
	case C.SHOCKIDX_OK:
		return count, format, nil
	case C.SHOCKIDX_EFORMAT: // the Go reader's error text, byte for byte (fastq.go:156-207, fasta.go:120)
		return count, format, errors.New(C.GoStringN(&res.err[0], C.int(res.err_len)))
	default:
		return count, format, fmt.Errorf("shockidx: %s: %s", C.GoString(C.shockidx_strerror(rc)),
			C.GoStringN(&res.err[0], C.int(res.err_len)))
	}
}

// Close mirrors record.Close (record.go:92-95): the file's Close error is discarded.
// node.AsyncIndexer never calls it; it closes the file itself (node/index.go:113).
func (g *gpuIndexer) Close() (err error) {
	g.f.Close()
	return
}

// init registers the GPU constructors under the reference's keys when a GPU is visible; the
// contexts themselves are made on the first build (gpuInit).
func init() {
	if C.shockidx_device_count() < 1 {
		return // no usable GPU: the Go indexers stay registered
	}
	Indexers["record"] = NewGPURecordIndexer
	Indexers["line"] = NewGPULineIndexer
}
