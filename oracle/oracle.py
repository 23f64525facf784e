"""ctypes wrapper over the C restatement (oracle/build/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
See shockidx_oracle.h for what is restated and how parity is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
if os.environ.get("ORACLE_VARIANT"):  # e.g. "san": the ASan + UBSan build (tools/sanitize.sh)
    _LIB_PATH = os.path.join(_HERE, "build", f"liboracle_{os.environ['ORACLE_VARIANT']}.so")
_lib = None

FMT = {"fasta": 1, "fastq": 2, "sam": 3}
FMT_NAME = {0: None, 1: "fasta", 2: "fastq", 3: "sam"}


def build():
    subprocess.run(["make", "-s", "-C", _HERE] + (["san"] if os.environ.get("ORACLE_VARIANT") == "san" else []),
                   check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_detect.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
        L.oracle_detect.restype = ctypes.c_int
        L.oracle_regex_match.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_regex_match.restype = ctypes.c_int
        L.oracle_record_index.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p,
                                          ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_record_index.restype = ctypes.c_int
        L.oracle_line_index.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                        ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_line_index.restype = ctypes.c_int
        L.oracle_trim_space.argtypes = [ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        PP = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64))
        Pu = ctypes.POINTER(ctypes.c_uint64)
        L.oracle_subset.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint64,
                                    ctypes.c_int64, PP, Pu, PP, Pu, Pu, ctypes.c_char_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_subset.restype = ctypes.c_int
        I64P = ctypes.POINTER(ctypes.c_int64)
        L.oracle_idx_part.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int64, I64P, I64P,
                                      ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_idx_part.restype = ctypes.c_int
        L.oracle_idx_range.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int64,
                                       ctypes.POINTER(ctypes.POINTER(ctypes.c_int64)), ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_idx_range.restype = ctypes.c_int
        L.oracle_create_subset_index.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_int64, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                                 I64P, I64P, ctypes.c_char_p, ctypes.c_size_t,
                                                 ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_create_subset_index.restype = ctypes.c_int
        L.oracle_filter_fastq.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                          ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_filter_fastq.restype = ctypes.c_int
        L.oracle_go_quote.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_go_quote.restype = ctypes.c_size_t
        L.oracle_chunkrecord.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64, PP, Pu,
                                         ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_chunkrecord.restype = ctypes.c_int
        L.oracle_chunkrecord_subset.argtypes = [ctypes.c_void_p, ctypes.c_uint64, PP, Pu]
        L.oracle_chunkrecord_subset.restype = ctypes.c_int
        L.oracle_fq_record_at.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_long]
        L.oracle_fq_record_at.restype = ctypes.c_long
        _lib = L
    return _lib


def _ptr(data):
    if isinstance(data, np.ndarray):
        assert data.dtype == np.uint8 and data.flags["C_CONTIGUOUS"]
        return data.ctypes.data, data.size, data
    buf = ctypes.create_string_buffer(bytes(data), len(data)) if len(data) else ctypes.create_string_buffer(1)
    return ctypes.addressof(buf), len(data), buf


def detect(data):
    p, n, keep = _ptr(data)
    mask = ctypes.c_int(0)
    f = lib().oracle_detect(p, n, ctypes.byref(mask))
    del keep
    return FMT_NAME[f], mask.value


def regex_match(data):
    """Regex.MatchString(data) for fasta.Regex / fastq.Regex / sam.Regex (no padding):
    the list of matching names in the order fasta, fastq, sam."""
    p, n, keep = _ptr(data)
    m = lib().oracle_regex_match(p, n)
    del keep
    return [name for i, name in enumerate(("fasta", "fastq", "sam")) if m >> i & 1]


def _take_rows(rows_p, count):
    n = int(count.value)
    if n == 0:
        out = np.zeros((0, 2), dtype=np.uint64)
    else:
        out = np.ctypeslib.as_array(rows_p, shape=(n * 2,)).copy().reshape(n, 2)
    lib().oracle_free(ctypes.cast(rows_p, ctypes.c_void_p))
    return out


def record_index(data, fmt=None):
    """Returns (rows uint64[count,2], err bytes|None)."""
    p, n, keep = _ptr(data)
    rows_p = ctypes.POINTER(ctypes.c_uint64)()
    count = ctypes.c_uint64(0)
    err = ctypes.create_string_buffer(512)
    errn = ctypes.c_size_t(0)
    rc = lib().oracle_record_index(p, n, -1 if fmt is None else FMT[fmt], ctypes.byref(rows_p),
                                   ctypes.byref(count), err, 512, ctypes.byref(errn))
    del keep
    if rc < 0:
        raise MemoryError("oracle_record_index")
    rows = _take_rows(rows_p, count)
    return rows, (err.raw[:errn.value] if rc == 1 else None)


def line_index(data):
    p, n, keep = _ptr(data)
    rows_p = ctypes.POINTER(ctypes.c_uint64)()
    count = ctypes.c_uint64(0)
    rc = lib().oracle_line_index(p, n, ctypes.byref(rows_p), ctypes.byref(count))
    del keep
    if rc < 0:
        raise MemoryError("oracle_line_index")
    return _take_rows(rows_p, count), None


def trim_space(s: bytes):
    p, n, keep = _ptr(s)
    lo = ctypes.c_size_t(0)
    hi = ctypes.c_size_t(0)
    lib().oracle_trim_space(p, n, ctypes.byref(lo), ctypes.byref(hi))
    del keep
    return bytes(s[lo.value:hi.value])


def subset(ids, parent_rows, ilength=None):
    """index/subset.go:133-303 CreateSubsetNodeIndexes ("array" parent index).
    Returns (rows uint64[k,2], runs uint64[c,2], size, err bytes|None)."""
    p, n, keep = _ptr(ids)
    par = np.ascontiguousarray(parent_rows, dtype=np.uint64).reshape(-1, 2)
    if ilength is None:
        ilength = par.shape[0]
    rows_p = ctypes.POINTER(ctypes.c_uint64)()
    runs_p = ctypes.POINTER(ctypes.c_uint64)()
    count, nruns, size = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    err = ctypes.create_string_buffer(256)
    errn = ctypes.c_size_t(0)
    rc = lib().oracle_subset(p, n, par.ctypes.data if par.size else None, par.shape[0], int(ilength),
                             ctypes.byref(rows_p), ctypes.byref(count), ctypes.byref(runs_p), ctypes.byref(nruns),
                             ctypes.byref(size), err, 256, ctypes.byref(errn))
    del keep
    if rc < 0:
        raise MemoryError("oracle_subset")
    rows = _take_rows(rows_p, count)
    runs = _take_rows(runs_p, nruns)
    return rows, runs, int(size.value), (err.raw[:errn.value] if rc == 1 else None)


CHUNK_SIZE = 1048576  # conf/conf.go:138


def chunkrecord(data, fmt=None, chunk=CHUNK_SIZE):
    """index/chunkrecord.go:41-99 (non-subset node).  Returns (rows uint64[k,2], err bytes|None);
    err is b"Invalid file type for filter" when detection fails and raises RuntimeError for a
    SAM file (the reference never terminates there, sam.go:100-102)."""
    p, n, keep = _ptr(data)
    rows_p = ctypes.POINTER(ctypes.c_uint64)()
    count = ctypes.c_uint64(0)
    err = ctypes.create_string_buffer(256)
    rc = lib().oracle_chunkrecord(p, n, -1 if fmt is None else FMT[fmt], int(chunk), ctypes.byref(rows_p),
                                  ctypes.byref(count), err, 256)
    del keep
    if rc < 0:
        raise MemoryError("oracle_chunkrecord")
    if rc == 2:
        raise RuntimeError(err.value.decode())
    return _take_rows(rows_p, count), (err.value if rc == 1 else None)


def fq_record_at(buf: bytes, s: int) -> int:
    """End of the leftmost-first `Record` match anchored at s in buf (fastq.go:23), or -1."""
    p, n, keep = _ptr(buf)
    e = lib().oracle_fq_record_at(p, n, s)
    del keep
    return e


def go_quote(s: bytes) -> bytes:
    p, n, keep = _ptr(s)
    out = ctypes.create_string_buffer(8 * len(s) + 8)
    k = lib().oracle_go_quote(p, n, out, len(out))
    del keep
    return out.raw[:k]


def _idx_rows(rows):
    if rows is None:
        return None, 0, None  # the .idx file is missing
    r = np.ascontiguousarray(rows, dtype=np.uint64).reshape(-1, 2)
    return (r.ctypes.data if r.size else ctypes.c_void_p(16)), r.shape[0], r


def idx_part(rows, part: str, idx_length: int):
    """index/index.go:67-117 Idx.Part over the .idx rows (None: file missing).
    Returns (pos, length, err bytes|None)."""
    p, n, keep = _idx_rows(rows)
    pos, length = ctypes.c_int64(0), ctypes.c_int64(0)
    err = ctypes.create_string_buffer(128)
    rc = lib().oracle_idx_part(p, n, part.encode(), int(idx_length), ctypes.byref(pos), ctypes.byref(length), err, 128)
    del keep
    return pos.value, length.value, (err.value if rc == 1 else None)


def idx_range(rows, part: str, idx_length: int):
    """index/index.go:119-193 Idx.Range.  Returns (recs int64[k,2], err bytes|None)."""
    p, n, keep = _idx_rows(rows)
    recs_p = ctypes.POINTER(ctypes.c_int64)()
    nrecs = ctypes.c_uint64(0)
    err = ctypes.create_string_buffer(128)
    rc = lib().oracle_idx_range(p, n, part.encode(), int(idx_length), ctypes.byref(recs_p), ctypes.byref(nrecs),
                                err, 128)
    del keep
    if rc < 0:
        raise MemoryError("oracle_idx_range")
    k = nrecs.value
    out = np.ctypeslib.as_array(recs_p, shape=(k * 2,)).copy().reshape(k, 2) if k else np.zeros((0, 2), np.int64)
    if recs_p:
        lib().oracle_free(ctypes.cast(recs_p, ctypes.c_void_p))
    return out, (err.value if rc == 1 else None)


def create_subset_index(ids, parent_rows, ilength=None):
    """index/subset.go:36-128 CreateSubsetIndex ("array").  Returns (rows uint64[k,2], count,
    size, err bytes|None); count = size = -1 on an error."""
    p, n, keep = _ptr(ids)
    par = np.ascontiguousarray(parent_rows, dtype=np.uint64).reshape(-1, 2)
    if ilength is None:
        ilength = par.shape[0]
    rows_p = ctypes.POINTER(ctypes.c_uint64)()
    count, size = ctypes.c_int64(0), ctypes.c_int64(0)
    err = ctypes.create_string_buffer(256)
    errn = ctypes.c_size_t(0)
    rc = lib().oracle_create_subset_index(p, n, par.ctypes.data if par.size else None, par.shape[0], int(ilength),
                                          ctypes.byref(rows_p), ctypes.byref(count), ctypes.byref(size), err, 256,
                                          ctypes.byref(errn))
    del keep
    if rc < 0:
        raise MemoryError("oracle_create_subset_index")
    rows = _take_rows(rows_p, ctypes.c_uint64(max(count.value, 0))) if rc == 0 else np.zeros((0, 2), np.uint64)
    if rc == 1 and rows_p:
        lib().oracle_free(ctypes.cast(rows_p, ctypes.c_void_p))
    return rows, count.value, size.value, (err.raw[:errn.value] if rc == 1 else None)


FILTERS = {"fq2fa": 1, "anonymize": 2}


def filter_fastq(data, name: str):
    """node/filter/{fq2fa,anonymize} over a FASTQ section.  Returns (out bytes, count, err|None)."""
    p, n, keep = _ptr(data)
    out_p = ctypes.POINTER(ctypes.c_uint8)()
    outlen, count = ctypes.c_size_t(0), ctypes.c_uint64(0)
    err = ctypes.create_string_buffer(256)
    rc = lib().oracle_filter_fastq(p, n, FILTERS[name], ctypes.byref(out_p), ctypes.byref(outlen), ctypes.byref(count),
                                   err, 256)
    del keep
    if rc < 0:
        raise MemoryError("oracle_filter_fastq")
    if rc == 2:
        raise NotImplementedError("anonymize of a non-FASTQ section")
    out = ctypes.string_at(out_p, outlen.value) if outlen.value else b""
    if out_p:
        lib().oracle_free(ctypes.cast(out_p, ctypes.c_void_p))
    return out, count.value, (err.value if rc == 1 else None)


def chunkrecord_subset(ri):
    """index/chunkrecord.go:100-228 (subset node, not "matrix"): the subset node's record index
    rows (uint64[k,2]) grouped into chunks; returns uint64[m,2] of (16 * first row, 16 * rows)."""
    ri = np.ascontiguousarray(ri, dtype=np.uint64).reshape(-1, 2)
    rows_p = ctypes.POINTER(ctypes.c_uint64)()
    count = ctypes.c_uint64(0)
    rc = lib().oracle_chunkrecord_subset(ri.ctypes.data if ri.size else None, len(ri), ctypes.byref(rows_p),
                                         ctypes.byref(count))
    if rc < 0:
        raise MemoryError("oracle_chunkrecord_subset")
    return _take_rows(rows_p, count)
