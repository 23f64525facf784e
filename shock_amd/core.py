"""Python host API over libshockidx (product path; no CPU fallback)."""
from __future__ import annotations

import ctypes
import os
import weakref
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L


@dataclass
class IndexResult:
    count: int
    fmt: str | None
    status: int
    err: bytes | None
    rows: np.ndarray | None = None  # uint64 [count, 2] {offset, length}
    timings: dict = field(default_factory=dict)
    path: int = 0  # 1: tile pass, 2: two-pass build, 3: slab-pipelined host build (diagnostic)
    reruns: int = 0
    state_out: int = 0
    term_code: int = 0
    flags: int = 0
    fixups: int = 0
    fix_tiles: int = 0

    @property
    def ok(self) -> bool:
        return self.status == L.OK


def _kind(kind) -> int:
    if kind in ("record", L.RECORD):
        return L.RECORD
    if kind in ("line", L.LINE):
        return L.LINE
    raise ValueError(f"unknown index kind {kind!r}")


def _fmt(fmt) -> int:
    if isinstance(fmt, int):
        return fmt
    return L.FMT_CODES[fmt]


def _result(res: L.Result, rc: int, rows=None) -> IndexResult:
    if rc < 0 and rc not in (L.EINVAL, L.ESPACE):
        raise L.ShockIdxError(rc, bytes(res.err)[:res.err_len].decode("utf-8", "replace"))
    msg = ctypes.string_at(ctypes.addressof(res) + L.Result.err.offset, res.err_len)
    return IndexResult(count=int(res.count), fmt=L.FMT_NAMES.get(res.format), status=rc,
                       err=msg if rc != L.OK else None, rows=rows,
                       timings={"kernel_ms": res.kernel_ms, "h2d_ms": res.h2d_ms, "d2h_ms": res.d2h_ms,
                                "total_ms": res.total_ms, "index_ms": res.index_ms},
                       path=int(res.path), reruns=int(res.reruns),
                       state_out=int(res.state_out), term_code=int(res.term_code), flags=int(res.flags),
                       fixups=int(res.fixups), fix_tiles=int(res.fix_tiles))


def _take_rows(ptr, count: int) -> np.ndarray:
    """The library's malloc'ed table as an array without a copy (freed with the array)."""
    lib = L.lib()
    if count == 0:
        lib.shockidx_free(ctypes.cast(ptr, ctypes.c_void_p))
        return np.zeros((0, 2), dtype=np.uint64)
    flat = np.ctypeslib.as_array(ptr, shape=(count * 2,))
    weakref.finalize(flat, lib.shockidx_free, ctypes.cast(ptr, ctypes.c_void_p).value)
    return flat.reshape(count, 2)


class Context:
    """One libshockidx context (HIP stream + workspaces) bound to a device."""

    def __init__(self, device: int = 0):
        self._lib = L.lib()
        h = ctypes.c_void_p()
        rc = self._lib.shockidx_ctx_create(device, ctypes.byref(h))
        if rc != L.OK:
            raise L.ShockIdxError(rc, f"shockidx_ctx_create(device={device}) failed "
                                      f"({self._lib.shockidx_strerror(rc).decode()})")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.shockidx_ctx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-memory build (POSTed body buffer) ------------------------------------------
    def build_host(self, data, kind="record", fmt=None) -> IndexResult:
        if isinstance(data, np.ndarray):
            buf = np.ascontiguousarray(data, dtype=np.uint8)
        else:
            buf = np.frombuffer(bytes(data), dtype=np.uint8)
        ptr = buf.ctypes.data if buf.size else None
        res = L.Result()
        rows_p = ctypes.POINTER(ctypes.c_uint64)()
        rc = self._lib.shockidx_build_host(self._h, ptr, buf.size, _kind(kind), _fmt(fmt),
                                           ctypes.byref(rows_p), ctypes.byref(res))
        rows = _take_rows(rows_p, int(res.count)) if rows_p else None
        return _result(res, rc, rows)

    def host_register(self, buf: np.ndarray) -> None:
        """Pin a host array for direct DMA (shockidx_host_register); build_host on it then
        skips the staging copy.  Undo with host_unregister before the array is freed."""
        rc = self._lib.shockidx_host_register(self._h, buf.ctypes.data, buf.nbytes)
        if rc != 0:
            raise RuntimeError(f"shockidx_host_register failed ({rc})")

    def host_unregister(self, buf: np.ndarray) -> None:
        rc = self._lib.shockidx_host_unregister(self._h, buf.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"shockidx_host_unregister failed ({rc})")

    # -- file build ------------------------------------------------------------------------
    def build_fd(self, fd: int, size: int, kind="record", fmt=None) -> IndexResult:
        res = L.Result()
        rows_p = ctypes.POINTER(ctypes.c_uint64)()
        rc = self._lib.shockidx_build_fd(self._h, fd, size, _kind(kind), _fmt(fmt),
                                         ctypes.byref(rows_p), ctypes.byref(res))
        rows = _take_rows(rows_p, int(res.count)) if rows_p else None
        return _result(res, rc, rows)

    def create(self, fd: int, size: int, kind, tmpdir: str, outpath: str) -> IndexResult:
        res = L.Result()
        rc = self._lib.shockidx_create(self._h, fd, size, _kind(kind), os.fsencode(tmpdir),
                                       os.fsencode(outpath), ctypes.byref(res))
        return _result(res, rc)

    # -- device-resident build ---------------------------------------------------------------
    def build_device(self, d_data: int, n: int, d_rows: int, row_cap: int, kind="record", fmt=None,
                     stream: int | None = None) -> IndexResult:
        """d_data / d_rows are device pointers (e.g. torch tensor .data_ptr())."""
        res = L.Result()
        rc = self._lib.shockidx_build_device(self._h, d_data, n, _kind(kind), _fmt(fmt), d_rows, row_cap,
                                             stream, ctypes.byref(res))
        return _result(res, rc)

    def build_buffer(self, data: "DeviceBuffer", n: int, rows: "DeviceBuffer", kind="record", fmt=None,
                     stream: int | None = None) -> IndexResult:
        """Device-resident build over DeviceBuffers (rows capacity = rows.nbytes // 16)."""
        return self.build_device(data.ptr, n, rows.ptr, rows.nbytes // 16, kind, fmt, stream)

    def chunkrecord_device(self, d_data: int, n: int, d_rows: int, row_cap: int, fmt=None, chunk: int = 0) -> IndexResult:
        """chunkRecord.Create (index/chunkrecord.go:41-99) over device memory; chunk 0 = 1 MiB."""
        res = L.Result()
        rc = self._lib.shockidx_chunkrecord_device(self._h, d_data, n, _fmt(fmt), chunk, d_rows, row_cap,
                                                   ctypes.byref(res))
        return _result(res, rc)

    def chunkrecord_fd(self, fd: int, size: int, fmt=None, chunk: int = 0) -> IndexResult:
        """chunkRecord.Create over an open file (shockidx_chunkrecord_fd); rows on the host."""
        res = L.Result()
        rows_p = ctypes.POINTER(ctypes.c_uint64)()
        rc = self._lib.shockidx_chunkrecord_fd(self._h, fd, size, _fmt(fmt), chunk, ctypes.byref(rows_p),
                                               ctypes.byref(res))
        rows = _take_rows(rows_p, int(res.count)) if rows_p else None
        return _result(res, rc, rows)

    def chunkrecord_subset_device(self, d_ri: int, nrows: int, d_rows: int, row_cap: int) -> IndexResult:
        """chunkRecord.Create for a subset node (index/chunkrecord.go:100-228) over its device-
        resident record index (nrows rows); rows (16 * first row, 16 * rows)."""
        res = L.Result()
        rc = self._lib.shockidx_chunkrecord_subset_device(self._h, d_ri, nrows, d_rows, row_cap, ctypes.byref(res))
        return _result(res, rc, None)

    def chunkrecord_subset(self, ri: np.ndarray) -> IndexResult:
        """The same from a host record index (uint64[k, 2]); the rows come back on the host."""
        ri = np.ascontiguousarray(ri, dtype=np.uint64).reshape(-1, 2)
        k = len(ri)
        src = self.alloc(16 * k + 16)
        out = self.alloc(16 * k + 16)
        try:
            if k:
                src.upload(ri.view(np.uint8).reshape(-1))
            r = self.chunkrecord_subset_device(src.ptr, k, out.ptr, max(k, 1))
            if r.status == L.OK:
                r.rows = out.rows(r.count) if r.count else np.zeros((0, 2), np.uint64)
            return r
        finally:
            src.free()
            out.free()

    def chunkrecord_buffer(self, data: "DeviceBuffer", n: int, rows: "DeviceBuffer", fmt=None,
                           chunk: int = 0) -> IndexResult:
        return self.chunkrecord_device(data.ptr, n, rows.ptr, rows.nbytes // 16, fmt, chunk)

    @staticmethod
    def chunkrecord_capacity(n: int, chunk: int = 0) -> int:
        """Rows a chunkrecord build can produce (include/shockidx.h)."""
        return n // ((chunk or 1048576) - 32767) + 2

    def set_dev_cap(self, nbytes: int) -> None:
        """Device bytes one fd build may hold (shockidx_ctx_set_dev_cap; 0: what is free).  A node
        whose one-pass build would not fit is indexed through two slab slots sized to the cap."""
        rc = self._lib.shockidx_ctx_set_dev_cap(self._h, int(nbytes))
        if rc != 0:
            raise L.ShockIdxError(rc, "shockidx_ctx_set_dev_cap failed")

    def trim(self, keep_bytes: int = 0) -> None:
        """Free the context's cached device workspaces down to keep_bytes (shockidx_ctx_trim)."""
        rc = self._lib.shockidx_ctx_trim(self._h, int(keep_bytes))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_ctx_trim failed")

    def workspace_bytes(self) -> int:
        return int(self._lib.shockidx_ctx_workspace_bytes(self._h))

    def alloc(self, nbytes: int, node: bool = False) -> "DeviceBuffer":
        """node=True: a node body the index streams (shockidx_dev_alloc_node: contiguous HBM)."""
        return DeviceBuffer(self, nbytes, node)

    def sync(self):
        rc = self._lib.shockidx_sync(self._h)
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_sync failed")

    @property
    def stream(self) -> int:
        return self._lib.shockidx_stream(self._h)

    # -- subset nodes (index/subset.go:133-303) -------------------------------------------------
    def subset_index(self, d_ids: int, ids_len: int, d_parent: int, parent_count: int, ilength: int, d_rows: int,
                     rows_cap: int, d_runs: int, runs_cap: int) -> SubsetResult:
        r = L.SubsetResult()
        rc = self._lib.shockidx_subset_index(self._h, d_ids, ids_len, d_parent, parent_count, ilength, d_rows, rows_cap,
                                             d_runs, runs_cap, ctypes.byref(r))
        return _sub_result(r, rc)

    def subset_gather(self, d_data: int, data_len: int, d_runs: int, nruns: int, d_out: int,
                      out_cap: int) -> SubsetResult:
        r = L.SubsetResult()
        rc = self._lib.shockidx_subset_gather(self._h, d_data, data_len, d_runs, nruns, d_out, out_cap,
                                              ctypes.byref(r))
        return _sub_result(r, rc)

    def subset_node(self, d_ids: int, ids_len: int, d_parent: int, parent_count: int, ilength: int, d_rows: int,
                    rows_cap: int, d_runs: int, runs_cap: int, d_data: int, data_len: int, d_out: int,
                    out_cap: int) -> SubsetResult:
        """subset_index + subset_gather in one call (the counts between them stay on the device)."""
        r = L.SubsetResult()
        rc = self._lib.shockidx_subset_node(self._h, d_ids, ids_len, d_parent, parent_count, ilength, d_rows, rows_cap,
                                            d_runs, runs_cap, d_data, data_len, d_out, out_cap, ctypes.byref(r))
        return _sub_result(r, rc)

    def subset_host(self, ids, parent_rows, ilength=None, data=None) -> SubsetResult:
        """Host-memory convenience: upload the id text and the parent rows, build the subset
        index on the device, download rows + runs (and the gathered bytes when `data` is given)."""
        ids = bytes(ids)
        par = np.ascontiguousarray(parent_rows, dtype=np.uint64).reshape(-1, 2)
        n = par.shape[0]
        il = n if ilength is None else int(ilength)
        d_ids = self.alloc(len(ids) + 64)
        d_ids.upload(ids)
        d_par = self.alloc(16 * n + 64)
        if n:
            d_par.upload(par.tobytes())
        cap = max(1, len(ids) // 2 + 2)
        d_rows = self.alloc(16 * cap)
        d_runs = self.alloc(16 * cap)
        r = self.subset_index(d_ids.ptr, len(ids), d_par.ptr, n, il, d_rows.ptr, cap, d_runs.ptr, cap)
        if r.status in (L.OK, L.EFORMAT):
            r.rows = d_rows.rows(r.count) if r.count else np.zeros((0, 2), np.uint64)
            nr = r.runs if r.ok else 0
            r.run_rows = d_runs.rows(nr) if nr else np.zeros((0, 2), np.uint64)
        if data is not None and r.ok:
            d_data = self.alloc(len(data) + 64)
            d_data.upload(bytes(data))
            d_out = self.alloc(max(r.size, 1) + 64)
            g = self.subset_gather(d_data.ptr, len(data), d_runs.ptr, r.runs, d_out.ptr, max(r.size, 1))
            r.gathered = d_out.download(g.size).tobytes() if g.ok else None
            d_data.free()
            d_out.free()
        for b in (d_ids, d_par, d_rows, d_runs):
            b.free()
        return r

    def create_subset_index(self, d_ids: int, ids_len: int, d_parent: int, parent_count: int, ilength: int,
                            d_rows: int, rows_cap: int) -> SubsetResult:
        """subset.go:36-128 CreateSubsetIndex on device memory (count = size = 2**64-1 on error)."""
        r = L.SubsetResult()
        rc = self._lib.shockidx_create_subset_index(self._h, d_ids, ids_len, d_parent, parent_count, ilength, d_rows,
                                                    rows_cap, ctypes.byref(r))
        return _sub_result(r, rc)

    # -- index read path (index/index.go:67-193) ---------------------------------------------------
    def idx_part(self, d_rows, nrows: int, part: str, idx_length: int):
        """Idx.Part over a device-resident index (d_rows None: the file is missing).
        Returns (pos, length, err bytes|None)."""
        r = L.SubsetResult()
        pos, length = ctypes.c_int64(0), ctypes.c_int64(0)
        rc = self._lib.shockidx_idx_part(self._h, d_rows, nrows, part.encode(), int(idx_length), ctypes.byref(pos),
                                         ctypes.byref(length), ctypes.byref(r))
        if rc == L.EFORMAT:
            return 0, 0, r.message
        if rc != L.OK:
            raise RuntimeError(f"shockidx_idx_part: {rc} {r.message!r}")
        return pos.value, length.value, None

    def idx_range(self, d_rows, nrows: int, part: str, idx_length: int, d_recs=None, recs_cap: int = 0):
        """Idx.Range over a device-resident index.  With d_recs the records stay on the device
        (returns (count, None)); without, they are returned as int64[k, 2].  Returns (recs|count, err|None)."""
        r = L.SubsetResult()
        own = None
        if d_recs is None:  # size the output with a first call
            rc = self._lib.shockidx_idx_range(self._h, d_rows, nrows, part.encode(), int(idx_length), None, 0,
                                              ctypes.byref(r))
            if rc == L.EFORMAT:
                return np.zeros((0, 2), np.int64), r.message
            if rc not in (L.OK, L.ESPACE):  # ESPACE: r.count holds the records needed
                raise RuntimeError(f"shockidx_idx_range: {rc} {r.message!r}")
            recs_cap = max(int(r.count), 1)
            own = self.alloc(16 * recs_cap + 64)
            d_recs = own.ptr
        rc = self._lib.shockidx_idx_range(self._h, d_rows, nrows, part.encode(), int(idx_length), d_recs, recs_cap,
                                          ctypes.byref(r))
        if rc == L.EFORMAT:
            if own is not None:
                own.free()
            return (np.zeros((0, 2), np.int64) if own is not None else 0), r.message
        if rc != L.OK:
            raise RuntimeError(f"shockidx_idx_range: {rc} {r.message!r}")
        if own is None:
            return int(r.count), None
        out = own.rows(int(r.count)).view(np.int64) if r.count else np.zeros((0, 2), np.int64)
        own.free()
        return out, None

    # -- download filters (node/filter/) -------------------------------------------------------
    def filter_device(self, name: str, d_data: int, n: int, d_out: int, out_cap: int) -> SubsetResult:
        """fq2fa / anonymize over a FASTQ section in HBM (count = records, size = bytes out)."""
        r = L.SubsetResult()
        rc = self._lib.shockidx_filter_device(self._h, name.encode(), d_data, n, d_out, out_cap, ctypes.byref(r))
        return _sub_result(r, rc)

    def filter_host(self, name: str, data) -> SubsetResult:
        """Host-memory convenience: upload, filter on the device, download (r.gathered = bytes)."""
        data = bytes(data)
        d_in = self.alloc(len(data) + 64)
        d_in.upload(data)
        cap = 2 * len(data) + 64  # anonymize may lengthen short records (counter digits)
        d_out = self.alloc(cap)
        try:
            r = self.filter_device(name, d_in.ptr, len(data), d_out.ptr, cap)
            if r.status == L.ESPACE:  # many tiny FASTA records: r.size holds the bytes needed
                d_out.free()
                cap = int(r.size) + 64
                d_out = self.alloc(cap)
                r = self.filter_device(name, d_in.ptr, len(data), d_out.ptr, cap)
            if r.status in (L.OK, L.EFORMAT):
                r.gathered = d_out.download(r.size).tobytes() if r.size else b""
        finally:
            d_in.free()
            d_out.free()
        return r

    def detect(self, data):
        buf = np.frombuffer(bytes(data[:32768]), dtype=np.uint8)
        f = ctypes.c_int(0)
        m = ctypes.c_int(0)
        rc = self._lib.shockidx_detect(self._h, buf.ctypes.data if buf.size else None, buf.size,
                                       ctypes.byref(f), ctypes.byref(m))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_detect failed")
        return L.FMT_NAMES.get(f.value), m.value


@dataclass
class SubsetResult:
    count: int        # oCount (rows before an error)
    runs: int         # coCount
    size: int         # oSize
    status: int
    err: bytes | None
    kernel_ms: float = 0.0
    total_ms: float = 0.0
    gather_ms: float = 0.0  # subset_node: device time of the gather
    rows: np.ndarray | None = None
    run_rows: np.ndarray | None = None
    gathered: bytes | None = None

    @property
    def ok(self) -> bool:
        return self.status == L.OK


def _sub_result(r: L.SubsetResult, rc: int) -> SubsetResult:
    if rc < 0 and rc not in (L.EINVAL, L.ESPACE):
        raise L.ShockIdxError(rc, r.message.decode("utf-8", "replace"))
    return SubsetResult(count=int(r.count), runs=int(r.runs), size=int(r.size), status=rc,
                        err=r.message if rc != L.OK else None, kernel_ms=r.kernel_ms, total_ms=r.total_ms,
                        gather_ms=r.gather_ms)


class DeviceBuffer:
    """HBM allocation on a Context's device (libshockidx's HIP runtime; torch's bundled HIP
    runtime is a different library and is not mixed into the same process)."""

    def __init__(self, ctx: Context, nbytes: int, node: bool = False):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        fn = ctx._lib.shockidx_dev_alloc_node if node else ctx._lib.shockidx_dev_alloc
        rc = fn(ctx._h, self.nbytes, ctypes.byref(p))
        if rc != L.OK:
            raise L.ShockIdxError(rc, f"device allocation of {nbytes} bytes failed")
        self.ptr = p.value

    def upload(self, data, offset: int = 0):
        buf = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray)
                                   else data).view(np.uint8).reshape(-1)
        assert offset + buf.size <= self.nbytes
        if buf.size:
            rc = self.ctx._lib.shockidx_memcpy_h2d(self.ctx._h, self.ptr + offset, buf.ctypes.data, buf.size)
            if rc != L.OK:
                raise L.ShockIdxError(rc, "h2d copy failed")

    def download(self, nbytes: int | None = None, offset: int = 0) -> np.ndarray:
        nbytes = self.nbytes - offset if nbytes is None else int(nbytes)
        out = np.empty(nbytes, dtype=np.uint8)
        if nbytes:
            rc = self.ctx._lib.shockidx_memcpy_d2h(self.ctx._h, out.ctypes.data, self.ptr + offset, nbytes)
            if rc != L.OK:
                raise L.ShockIdxError(rc, "d2h copy failed")
        return out

    def rows(self, count: int) -> np.ndarray:
        return self.download(16 * count).view(np.uint64).reshape(count, 2)

    def fill(self, value: int, nbytes: int | None = None, offset: int = 0):
        rc = self.ctx._lib.shockidx_memset(self.ctx._h, self.ptr + offset, value,
                                           self.nbytes - offset if nbytes is None else nbytes)
        if rc != L.OK:
            raise L.ShockIdxError(rc, "memset failed")

    def free(self):
        if self.ptr:
            self.ctx._lib.shockidx_dev_free(self.ctx._h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def write_idx(rows: np.ndarray, tmpdir: str, outpath: str) -> None:
    """The .idx output protocol (record.go:35-41,65-87) through libshockidx."""
    lib = L.lib()
    r = np.ascontiguousarray(rows, dtype=np.uint64)
    err = ctypes.create_string_buffer(256)
    rc = lib.shockidx_write_idx(r.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), r.shape[0],
                                os.fsencode(tmpdir), os.fsencode(outpath), err, 256)
    if rc != L.OK:
        raise L.ShockIdxError(rc, err.value.decode("utf-8", "replace"))


class MultiContext:
    """Several GPUs building one node file from this process (shockidx_multi_*): byte slabs,
    one per device, summaries all-gathered over RCCL (host memory when a device repeats).
    Same results as Context.build_host / build_fd / create."""

    def __init__(self, devices):
        self._lib = L.lib()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        rc = self._lib.shockidx_multi_create(devs, len(devices), ctypes.byref(h))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_multi_create failed")
        self._h = h
        self.devices = list(devices)
        self._fin = weakref.finalize(self, self._lib.shockidx_multi_destroy, h)

    @property
    def rccl(self) -> bool:
        return bool(self._lib.shockidx_multi_rccl(self._h))

    def close(self):
        self._fin()

    def build_host(self, data, kind="record", fmt=None) -> IndexResult:
        if isinstance(data, np.ndarray):
            buf = np.ascontiguousarray(data, dtype=np.uint8)
        else:
            buf = np.frombuffer(bytes(data), dtype=np.uint8)
        ptr = buf.ctypes.data if buf.size else None
        res = L.Result()
        rows_p = ctypes.POINTER(ctypes.c_uint64)()
        rc = self._lib.shockidx_multi_build_host(self._h, ptr, buf.size, _kind(kind), _fmt(fmt),
                                                 ctypes.byref(rows_p), ctypes.byref(res))
        rows = _take_rows(rows_p, int(res.count)) if rows_p else None
        return _result(res, rc, rows)

    def build_fd(self, fd: int, size: int, kind="record", fmt=None) -> IndexResult:
        res = L.Result()
        rows_p = ctypes.POINTER(ctypes.c_uint64)()
        rc = self._lib.shockidx_multi_build_fd(self._h, fd, size, _kind(kind), _fmt(fmt),
                                               ctypes.byref(rows_p), ctypes.byref(res))
        rows = _take_rows(rows_p, int(res.count)) if rows_p else None
        return _result(res, rc, rows)

    def create(self, fd: int, size: int, kind, tmpdir: str, outpath: str) -> IndexResult:
        res = L.Result()
        rc = self._lib.shockidx_multi_create_index(self._h, fd, size, _kind(kind), os.fsencode(tmpdir),
                                                   os.fsencode(outpath), ctypes.byref(res))
        return _result(res, rc)

    def plan(self, size: int):
        """[(lo, hi, wlo, whi)] per slab: slab k owns [lo, hi) and is held as [wlo, whi)."""
        n = len(self.devices)
        arr = [(ctypes.c_uint64 * n)() for _ in range(4)]
        rc = self._lib.shockidx_multi_plan(self._h, size, *arr)
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_multi_plan failed")
        return [tuple(int(a[k]) for a in arr) for k in range(n)]

    def build_resident(self, size: int, d_win, d_rows, row_cap, kind="record", fmt=None):
        """Windows already in HBM (d_win[k] on devices[k], per plan()); rows stay on the devices.
        Returns (IndexResult, first_record[], rows_owned[])."""
        n = len(self.devices)
        win = (ctypes.c_void_p * n)(*d_win)
        rws = (ctypes.c_void_p * n)(*d_rows)
        cap = (ctypes.c_uint64 * n)(*row_cap)
        first, owned = (ctypes.c_uint64 * n)(), (ctypes.c_uint64 * n)()
        res = L.Result()
        rc = self._lib.shockidx_multi_build_resident(self._h, size, _kind(kind), _fmt(fmt), win, rws, cap, first,
                                                     owned, ctypes.byref(res))
        return _result(res, rc), [int(x) for x in first], [int(x) for x in owned]
