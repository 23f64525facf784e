"""Host-side mirror of Shock's indexer plug-in surface, backed by libshockidx.

Reference interface (paths relative to /root/reference/shock-server/):
    node/file/index/index.go:19   type indexerFunc func(*os.File, string, string, string) Indexer
    node/file/index/index.go:21   var Indexers = map[string]indexerFunc{...}
    node/file/index/index.go:30   type Indexer interface { Create(string) (int64, string, error); Close() error }
    node/file/index/record.go:23  NewRecordIndexer      node/file/index/line.go:25  NewLineIndexer

Same names, argument meaning and error behaviour: create(out_path) returns
(count, "array", err) where err is None or a ShockIndexError carrying Go's exact message and
count is the number of records produced before the error; on error nothing is written to
out_path.  The temp file lives in <PATH_DATA>/temp like record.go:35.
"""
from __future__ import annotations

import os

from . import _lib as L
import numpy as np

from .core import Context, write_idx

PATH_DATA = os.environ.get("SHOCK_PATH_DATA", "/tmp/shock-data")  # conf.PATH_DATA

_ctx: Context | None = None


def context() -> Context:
    global _ctx
    if _ctx is None:
        _ctx = Context(int(os.environ.get("SHOCKIDX_DEVICE", "0")))
    return _ctx


class ShockIndexError(Exception):
    """A Go `error` value returned by Create (message = Go's error string, bytes)."""

    def __init__(self, msg: bytes):
        super().__init__(msg.decode("utf-8", "replace"))
        self.msg = msg


class _GPUIndexer:
    kind = "record"

    def __init__(self, f, n_type: str = "", sn_format: str = "", sn_index_path: str = ""):
        self.f = f
        self.t = n_type
        self.snf = sn_format
        self.snp = sn_index_path

    def create(self, file: str):
        """Indexer.Create(outPath) -> (count int64, format string, err error)."""
        fd = self.f.fileno()
        size = os.fstat(fd).st_size
        tmpdir = os.path.join(PATH_DATA, "temp")
        os.makedirs(tmpdir, exist_ok=True)
        r = context().create(fd, size, self.kind, tmpdir, file)
        if r.status == L.OK:
            return r.count, "array", None
        if r.status == L.EFORMAT:
            return r.count, "array", ShockIndexError(r.err)
        raise L.ShockIdxError(r.status, (r.err or b"").decode("utf-8", "replace"))

    def close(self):
        # record.go:92-95 closes the file; AsyncIndexer never calls it (node/index.go:113)
        self.f.close()


class RecordIndexer(_GPUIndexer):
    kind = "record"


class LineIndexer(_GPUIndexer):
    kind = "line"


class ChunkRecordIndexer(_GPUIndexer):
    """chunkRecord.Create (index/chunkrecord.go:41-228).  Non-subset nodes (:41-99): the file goes
    to HBM and shockidx_chunkrecord_fd builds the table.  Subset nodes (:100-228): the subset
    node's record index file (sn_index_path) is read whole rows at a time and its rows are
    grouped on the device (shockidx_chunkrecord_subset_device) into the "matrix" index.  Either
    way write_idx renames the table into place."""
    kind = "chunkrecord"

    def _create_subset(self, file: str):
        if self.snf == "matrix":  # chunkrecord.go:101-103
            return 0, "", ShockIndexError(b"Shock does not currently support the creation of chunkrecord "
                                          b"indices for subset nodes derived from a matrix formatted index.")
        try:
            with open(self.snp, "rb") as rfh:  # :107-111 os.Open(i.snrp)
                raw = rfh.read()
        except OSError as e:
            return 0, "", ShockIndexError(str(e).encode())
        k = len(raw) // 16  # ReadAt of a partial last row is io.EOF: the loop ends (:146-153)
        ri = np.frombuffer(raw[: 16 * k], dtype="<u8").reshape(-1, 2)
        r = context().chunkrecord_subset(ri)
        if r.status != L.OK:
            raise L.ShockIdxError(r.status, (r.err or b"").decode("utf-8", "replace"))
        tmpdir = os.path.join(PATH_DATA, "temp")
        os.makedirs(tmpdir, exist_ok=True)
        write_idx(r.rows, tmpdir, file)
        return r.count, "matrix", None

    def create(self, file: str):
        if self.t == "subset":
            return self._create_subset(file)
        fd = self.f.fileno()
        size = os.fstat(fd).st_size
        # the whole file goes to HBM through libshockidx's pread staging (short reads retried)
        r = context().chunkrecord_fd(fd, size)
        if r.status == L.EFORMAT:
            return r.count, "array", ShockIndexError(r.err)
        if r.status != L.OK:
            raise L.ShockIdxError(r.status, (r.err or b"").decode("utf-8", "replace"))
        tmpdir = os.path.join(PATH_DATA, "temp")
        os.makedirs(tmpdir, exist_ok=True)
        write_idx(r.rows if r.rows is not None else np.zeros((0, 2), np.uint64), tmpdir, file)
        return r.count, "array", None


def NewChunkRecordIndexer(f, n_type="", sn_format="", sn_index_path=""):  # noqa: N802
    return ChunkRecordIndexer(f, n_type, sn_format, sn_index_path)


def NewRecordIndexer(f, n_type="", sn_format="", sn_index_path=""):  # noqa: N802 (reference name)
    return RecordIndexer(f, n_type, sn_format, sn_index_path)


def NewLineIndexer(f, n_type="", sn_format="", sn_index_path=""):  # noqa: N802
    return LineIndexer(f, n_type, sn_format, sn_index_path)


# index.go:21-28 -- the GPU path serves the scanning indexers; "size" (no scan) is not provided.
Indexers = {
    "chunkrecord": NewChunkRecordIndexer,
    "line": NewLineIndexer,
    "record": NewRecordIndexer,
}
