"""Synthetic node files generated on the device (libshocksynth.so) -- benchmark / large-size
parity infrastructure, not part of the index path.

A SynthFile is a virtual FASTQ or FASTA file of `size` bytes:
whole records generated from (seed, record index), then '\n' padding up to `size` (trailing
blank lines are legal and unindexed in FASTQ; in FASTA they belong to the last record).
Any byte window can be materialised in HBM, so one GPU's slab of a larger file is produced
without the rest, and the expected index table is known by construction.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .core import Context, DeviceBuffer

HERE = os.path.dirname(os.path.abspath(__file__))
SYNTH_PATH = os.path.join(HERE, "libshocksynth.so")
SEED = 0x5EED
_slib = None


def slib():
    global _slib
    if _slib is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError(f"{SYNTH_PATH} not built (make -C shock_amd/csrc)")
        L = ctypes.CDLL(SYNTH_PATH)
        u64, vp, i32 = ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int
        L.synth_lengths.argtypes = [i32, u64, u64, u64, vp, vp]
        L.synth_offsets.argtypes = [vp, u64, u64, vp, vp]
        L.synth_fill.argtypes = [i32, vp, u64, u64, vp, u64, u64, u64, vp]
        L.synth_find.argtypes = [vp, u64, u64, vp, vp]
        L.synth_check_rows.argtypes = [vp, vp, vp, u64, vp, vp]
        L.synth_stream_floor.argtypes = [vp, u64, i32, vp, vp, vp]
        L.synth_run_hash.argtypes = [vp, vp, u64, vp, vp]
        for f in (L.synth_lengths, L.synth_offsets, L.synth_fill, L.synth_find, L.synth_check_rows,
                  L.synth_stream_floor, L.synth_run_hash):
            f.restype = i32
        _slib = L
    return _slib


def _ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"libshocksynth {what} failed ({rc})")


def run_hashes(ctx: Context, d_data: int, d_runs: int, nruns: int) -> np.ndarray:
    """A 64-bit hash of each byte run (rows of u64 offset, length at d_runs) of d_data, computed on
    the device (k_run_hash) -- test support for whole-output checks of gathered bytes."""
    out = ctx.alloc(8 * max(1, nruns))
    try:
        _ck(slib().synth_run_hash(d_data, d_runs, nruns, out.ptr, ctx.stream), "run_hash")
        ctx.sync()
        return out.download(8 * nruns).view(np.uint64).copy()
    finally:
        out.free()


# smallest possible record of each generator (bounds the record count for a given size)
MIN_REC = {"fastq": 125, "fasta": 30 + 16}


class SynthFile:
    def __init__(self, ctx: Context, fmt: str, size: int, seed: int = SEED):
        assert fmt in ("fastq", "fasta")
        self.ctx, self.fmt, self.size, self.seed = ctx, fmt, int(size), seed
        self.fasta = 1 if fmt == "fasta" else 0
        L = slib()
        n_est = self.size // MIN_REC[fmt] + 2
        self.n_est = n_est
        self.d_len = ctx.alloc(4 * n_est + 64)
        self.d_off = ctx.alloc(8 * (n_est + 1) + 64)
        self._tmp = ctx.alloc(64)
        s = ctx.stream
        _ck(L.synth_lengths(self.fasta, 0, n_est, seed, self.d_len.ptr, s), "lengths")
        _ck(L.synth_offsets(self.d_len.ptr, n_est, 0, self.d_off.ptr, s), "offsets")
        ctx.sync()
        # records wholly inside [0, size)
        self.nrec = self._count_le(self.size) - 1
        self.covered = int(self.d_off.download(8, 8 * self.nrec).view(np.uint64)[0])

    def _count_le(self, pos: int) -> int:
        """number of offsets off[0..n_est] <= pos"""
        L = slib()
        _ck(L.synth_find(self.d_off.ptr, self.n_est + 1, pos, self._tmp.ptr, self.ctx.stream), "find")
        self.ctx.sync()
        return int(self._tmp.download(8).view(np.uint64)[0])

    def record_range(self, lo: int, hi: int):
        """indices [k0, k1) of the records (of the first nrec) that overlap [lo, hi)"""
        k0 = max(self._count_le(lo) - 1, 0)
        k1 = min(self._count_le(hi - 1) if hi > 0 else 0, self.nrec)
        return k0, max(k1, k0)

    def window(self, lo: int, hi: int, pad: int = 64) -> DeviceBuffer:
        """HBM buffer holding bytes [lo, hi) of the virtual file."""
        lo, hi = int(lo), int(min(hi, self.size))
        buf = self.ctx.alloc(hi - lo + pad, node=True)  # a node body resident in HBM
        buf.fill(0x0A)  # '\n' padding beyond the last whole record
        k0, k1 = self.record_range(lo, hi)
        L = slib()
        _ck(L.synth_fill(self.fasta, buf.ptr, lo, hi, self.d_off.ptr + 8 * k0, k0, k1 - k0, self.seed,
                         self.ctx.stream), "fill")
        self.ctx.sync()
        return buf

    def expected_count(self) -> int:
        return self.nrec

    def check_rows(self, rows: DeviceBuffer, k0: int, count: int, row_index0: int = 0) -> int:
        """Mismatching rows among rows[row_index0 : row_index0+count] vs records k0.. (device)."""
        L = slib()
        self._tmp.fill(0, 8)
        _ck(L.synth_check_rows(rows.ptr + 16 * row_index0, self.d_off.ptr + 8 * k0, self.d_len.ptr + 4 * k0,
                               count, self._tmp.ptr, self.ctx.stream), "check")
        self.ctx.sync()
        return int(self._tmp.download(8).view(np.uint64)[0])

    def stream_floor(self, data: DeviceBuffer, n: int, reps: int = 20) -> float:
        """Average ms of the tile passes' staging skeleton alone over data[0, n) (no parsing, no
        per-tile stores): this box's HBM floor for their read pattern (bench context)."""
        ms = ctypes.c_float(0.0)
        _ck(slib().synth_stream_floor(data.ptr, n, reps, self._tmp.ptr, ctypes.byref(ms), self.ctx.stream), "floor")
        return float(ms.value)

    def free(self):
        for b in (self.d_len, self.d_off, self._tmp):
            b.free()
