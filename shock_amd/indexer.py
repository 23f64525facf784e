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
from .core import Context

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


def NewRecordIndexer(f, n_type="", sn_format="", sn_index_path=""):  # noqa: N802 (reference name)
    return RecordIndexer(f, n_type, sn_format, sn_index_path)


def NewLineIndexer(f, n_type="", sn_format="", sn_index_path=""):  # noqa: N802
    return LineIndexer(f, n_type, sn_format, sn_index_path)


# index.go:21-28 -- the GPU path serves the two scanning indexers; "chunkrecord" and "size"
# are outside this hot path and are not provided here.
Indexers = {
    "line": NewLineIndexer,
    "record": NewRecordIndexer,
}
