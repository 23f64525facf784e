"""Host-side mirror of Shock's index read path (Idx.Part / Idx.Range), backed by libshockidx.

Reference interface (paths relative to /root/reference/shock-server/):
    node/file/index/index.go:35-41    type Index interface { ...; Part(...); Range(...) }
    node/file/index/index.go:43-65    type Idx struct { T string; Length int }, New, Set, Type, GetLength
    node/file/index/index.go:67-117   Idx.Part(part, idxFilePath, idxLength) (pos, length int64, err error)
    node/file/index/index.go:119-193  Idx.Range(part, idxFilePath, idxLength) (recs [][]int64, err error)
    callers: controller/node/single.go:391-508 (?index=..&part=.. downloads, subset nodes),
             controller/preauth/preauth.go:84

Same names, argument meaning and error behaviour: errors are ShockIndexError carrying Go's
text (IndexNoFile "Index file is missing", InvalidIndexRange "Invalid index record range",
IndexOutBounds "Index record out of bounds"); Range returns an int64[k, 2] array of
{pos, length} (empty for Go's nil slice).  The .idx file is read into HBM once and served from
there (shockidx_idx_part / shockidx_idx_range); a table is reloaded when the file's size or
mtime changes, and the least recently used tables are dropped past SHOCKIDX_IDX_CACHE_BYTES
(default 4 GiB).
"""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np

from .indexer import ShockIndexError, context

_CACHE_BYTES = int(os.environ.get("SHOCKIDX_IDX_CACHE_BYTES", str(4 << 30)))


class _Tables:
    """Device-resident .idx tables keyed by path (LRU, bounded)."""

    def __init__(self):
        self._t: OrderedDict[str, tuple] = OrderedDict()  # path -> (key, buffer, nrows, bytes)
        self._bytes = 0

    def get(self, path: str):
        """(device pointer, nrows) of the file's whole rows, or None when it cannot be opened."""
        try:
            st = os.stat(path)
            key = (st.st_size, st.st_mtime_ns, st.st_ino)
            hit = self._t.get(path)
            if hit is not None and hit[0] == key:
                self._t.move_to_end(path)
                return hit[1].ptr, hit[2]
            with open(path, "rb") as f:  # os.Open (index.go:70, :122)
                raw = f.read()
        except OSError:
            return None
        self.drop(path)
        nrows = len(raw) // 16  # binary.Read of a row past the end fails
        buf = context().alloc(16 * nrows + 64)
        if nrows:
            buf.upload(raw[: 16 * nrows])
        self._t[path] = (key, buf, nrows, 16 * nrows)
        self._bytes += 16 * nrows
        while self._bytes > _CACHE_BYTES and len(self._t) > 1:
            self.drop(next(iter(self._t)))
        return buf.ptr, nrows

    def drop(self, path: str):
        old = self._t.pop(path, None)
        if old is not None:
            self._bytes -= old[3]
            old[1].free()


_tables = _Tables()


class Idx:
    """index.go:43-53 (T "file", Length 0)."""

    def __init__(self):
        self.T = "file"
        self.Length = 0

    def Set(self, inter):  # noqa: N802  (index.go:55-57: a no-op)
        return

    def Type(self) -> str:  # noqa: N802
        return self.T

    def GetLength(self) -> int:  # noqa: N802
        return int(self.Length)

    def Part(self, part: str, idx_file_path: str, idx_length: int):  # noqa: N802
        """-> (pos, length, err): one record "N", or "N-M" as one contiguous span."""
        t = _tables.get(idx_file_path)
        d_rows, nrows = t if t is not None else (None, 0)
        pos, length, err = context().idx_part(d_rows, nrows, part, idx_length)
        return pos, length, (ShockIndexError(err) if err is not None else None)

    def Range(self, part: str, idx_file_path: str, idx_length: int):  # noqa: N802
        """-> (recs int64[k, 2], err): the maximal runs of contiguous records of the range."""
        t = _tables.get(idx_file_path)
        d_rows, nrows = t if t is not None else (None, 0)
        recs, err = context().idx_range(d_rows, nrows, part, idx_length)
        return recs, (ShockIndexError(err) if err is not None else None)


def New() -> Idx:  # noqa: N802  (index.go:48-53)
    return Idx()
