"""Host-side mirror of Shock's subset-node index builder, backed by libshockidx.

Reference (paths relative to /root/reference/shock-server/):
    node/file/index/subset.go:133-303  CreateSubsetNodeIndexes(s, cofile, ofile, ifile, iformat, ilength)
        -> (coCount, oCount, oSize int64, err error)
    node/file/index/subset.go:36-128   CreateSubsetIndex(s, oifile, ifile, iformat, ilength)
        -> (count, size int64, err error); (-1, -1, err) on every error (caller node/index.go:103)
    node/fs.go:52-126                  SetFileFromSubset (the caller: paths, counts -> IdxInfo)

Same argument meaning and error behaviour: the uploaded id list is parsed and checked on the
device (shockidx_subset_index); on success the compressed index is renamed into `cofile`
first, then the subset index into `ofile` (subset.go:293-297); on an error nothing is renamed
and the counts are the ones Go returns at that point.
"""
from __future__ import annotations

import os

import numpy as np

from .core import write_idx
from .indexer import PATH_DATA, ShockIndexError, context


def _read(f) -> bytes:
    if hasattr(f, "read"):
        return f.read()
    with open(f, "rb") as fh:
        return fh.read()


def CreateSubsetNodeIndexes(ids, cofile: str, ofile: str, ifile: str, iformat: str, ilength: int):  # noqa: N802
    """ids: the uploaded subset_indices file (path or binary file object)."""
    if iformat != "array":  # subset.go:298-300
        return 0, 0, 0, ShockIndexError(
            b"Subset node does not currently support the format of your parent index: " + iformat.encode())
    text = _read(ids)
    raw = _read(ifile)
    parent = np.frombuffer(raw[: len(raw) // 16 * 16], dtype="<u8").reshape(-1, 2)  # ReadAt of whole rows
    r = context().subset_host(text, parent, ilength)
    if not r.ok:
        return r.runs, r.count, r.size, ShockIndexError(r.err)
    tmpdir = os.path.join(PATH_DATA, "temp")
    os.makedirs(tmpdir, exist_ok=True)
    write_idx(r.run_rows, tmpdir, cofile)
    write_idx(r.rows, tmpdir, ofile)
    return r.runs, r.count, r.size, None


def CreateSubsetIndex(ids, oifile: str, ifile: str, iformat: str, ilength: int):  # noqa: N802
    """ids: the uploaded subset_indices file (path or binary file object).  On success the
    subset index is renamed into `oifile`; on any error (-1, -1, err) and nothing is renamed."""
    if iformat != "array":  # subset.go:125-127
        return -1, -1, ShockIndexError(
            b"Subset index does not currently support the format of your parent index: " + iformat.encode())
    try:
        raw = _read(ifile)  # os.Open(ifile) (:40-43)
    except OSError as e:
        return -1, -1, ShockIndexError(str(e).encode())
    text = _read(ids)
    parent = np.frombuffer(raw[: len(raw) // 16 * 16], dtype="<u8").reshape(-1, 2)
    ctx = context()
    n = parent.shape[0]
    d_ids = ctx.alloc(len(text) + 64)
    d_ids.upload(text)
    d_par = ctx.alloc(16 * n + 64)
    if n:
        d_par.upload(parent.tobytes())
    cap = max(1, len(text) // 2 + 2)  # one row per non-blank line: at most len/2 + 1
    d_rows = ctx.alloc(16 * cap)
    try:
        r = ctx.create_subset_index(d_ids.ptr, len(text), d_par.ptr, n, int(ilength), d_rows.ptr, cap)
        if not r.ok:
            return -1, -1, ShockIndexError(r.err)
        rows = d_rows.rows(r.count) if r.count else np.zeros((0, 2), np.uint64)
    finally:
        for b in (d_ids, d_par, d_rows):
            b.free()
    tmpdir = os.path.join(PATH_DATA, "temp")
    os.makedirs(tmpdir, exist_ok=True)
    write_idx(rows, tmpdir, oifile)  # temp file + os.Rename (:38, :122)
    return int(r.count), int(r.size), None
