"""CPU test double of DeviceSlabEngine (shock_amd/dist.py) for FASTQ and line indexes.

TEST INFRASTRUCTURE: lets the multi-process slab protocol (guess -> index -> exchange ->
combine -> rerun) run under gloo on a machine without a GPU.  It restates, for one slab,
what k_index / k_finalize / k_slab_guess / k_slab_combine compute (sidx_kernels.hip), with
each record validated by the oracle (oracle/shockidx_oracle.c) on the record's own bytes.
Only well-formed inputs plus single injected errors are exercised through it; the kernels'
own multi-slab parity is tested on the GPU against the oracle (tests/test_gpu_slabs.py).
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle  # noqa: E402

from shock_amd.dist import KEY_NONE, Plan  # noqa: E402

FASTQ, LINE = 2, 4
# oracle error text -> device status (sidx_common.hpp Status)
_ST = {b"Invalid format: truncated fastq record": 2, b"Invalid format: empty line(s) between records": 3,
       b"Invalid format: id line does not start with @": 4, b"Invalid format: missing sequence ID": 5,
       b"Invalid format: empty sequence": 6, b"Invalid format: plus line does not start with +": 7,
       b"Invalid format: quality ID does not match sequence ID": 8,
       b"Invalid format: length of sequence and quality lines do not match": 9}


class HostSlabEngine:
    def __init__(self, rank: int, world: int, wrong_guess: bool = False):
        self.rank, self.world, self.wrong_guess = rank, world, wrong_guess

    def set_slab(self, window: bytes, wlo: int, lo: int, hi: int, whi: int, size: int):
        self.win, self.wlo, self.lo, self.hi, self.whi = window, wlo, lo, hi, whi
        self.is_first, self.is_last = lo == 0 and self.rank == 0, whi == size
        self.row_base = 0 if self.is_first else 1
        self.f = lo - wlo  # slab byte 0 inside the window

    def _slab(self, a, b):
        return self.win[self.f + a:self.f + b]

    def guess(self, fmt: int) -> int:
        if self.is_first or fmt != FASTQ:
            g = 0
        else:  # k_slab_guess: first '@' line with '+' two lines later and equal seq/qual lengths
            head = self._slab(0, min(4096, self.hi - self.lo))
            nl = [i for i, c in enumerate(head) if c == 0x0A]
            g = 0
            for i in range(len(nl) - 4):
                s, e0, e1, e2, e3 = nl[i] + 1, nl[i + 1], nl[i + 2], nl[i + 3], nl[i + 4]
                if head[s] == 0x40 and e0 > s + 1 and head[e1 + 1] == 0x2B and e1 - e0 == e3 - e2 and e1 > e0 + 1:
                    g = (3 - (i & 3)) & 3
                    break
        if self.wrong_guess and fmt == FASTQ and not self.is_first:
            g = (g + 1) & 3
        return g

    def _record(self, fmt: int, s: int):
        """(status, length) of the record starting at slab offset s."""
        end = self.whi - self.lo
        if s >= end:  # line.go emits the final (empty) entry at EOF; FASTQ ends cleanly
            return ((0 if fmt == LINE else 1) if self.is_last else 12), 0
        rest = self._slab(s, end)
        if fmt == LINE:
            j = rest.find(b"\n")
            return 0, (j + 1 if j >= 0 else len(rest))
        cut, k = 0, 0
        while k < 4:  # exactly one FASTQ record's lines for the oracle
            j = rest.find(b"\n", cut)
            if j < 0:
                cut = len(rest)
                break
            cut, k = j + 1, k + 1
        if k < 4 and not self.is_last:
            return 12, 0
        rows, err = oracle.record_index(rest[:cut], "fastq")
        if err is not None and len(rows) == 0:
            return _ST[err], 0
        if len(rows) == 0:
            return 1, 0
        return 0, int(rows[0][1])

    def index(self, fmt: int, state_in: int, seq: int = 0):
        self.seq = seq
        n = self.hi - self.lo
        nl = np.flatnonzero(np.frombuffer(self._slab(0, n), dtype=np.uint8) == 0x0A)
        self.agg = len(nl)
        recs = [(0, 0)] if self.is_first else []
        for j, p in enumerate(nl.tolist()):
            if fmt == LINE:
                recs.append((state_in + j + 1, p + 1))
            elif (state_in + j) % 4 == 3:
                recs.append(((state_in + j + 1) >> 2, p + 1))
        self.key = KEY_NONE
        self.rows = []
        for k, s in recs:
            st, ln = self._record(fmt, s)
            if st == 0:
                self.rows.append((self.lo + s, ln))
            else:
                self.key = min(self.key, (k << 28) | st)
                break
        fin = state_in + self.agg
        self.natural = (fin >> 2) + 1 if fmt == FASTQ else fin + 1
        self.local_count = (self.key >> 28) if self.key != KEY_NONE else self.natural
        self.state_in = state_in
        self.local_flags = 0
        self.rows = self.rows[:max(0, self.local_count - self.row_base)]

    def summary_bytes(self) -> bytes:
        return struct.pack("<7Q2HI", self.agg, self.state_in, self.key, self.natural, self.row_base, 0, 0, 0, 0,
                           self.seq)

    def load_all(self, blobs):
        self.all = [struct.unpack("<7Q2HI", b) for b in blobs]

    def combine(self, fmt: int, expect=None) -> Plan:
        """slab_combine<F> for the count monoid (sidx_kernels.hip)."""
        s, done = 0, False
        pl = Plan(0, 0, 0, 0, 0, 0, -1, 0, 0)
        for q, (agg, sin, key, natural, row_base, _, _, _, _, seq) in enumerate(self.all):
            if expect is not None and seq != expect[q]:
                pl.flags |= 32
            ok = (s & 3) == (sin & 3) if fmt == FASTQ else True
            if not ok:
                pl.inconsistent |= 1 << q
            delta = (s - (sin & 3)) >> 2 if fmt == FASTQ else s - sin
            if q == self.rank:
                pl.state_in, pl.first_record = s, delta + row_base
            if not done and ok:
                if key != KEY_NONE:
                    pl.count, pl.code, done = (key >> 28) + delta, key & 15, True
                elif q == len(self.all) - 1:
                    pl.count = natural + delta
            s += agg
        return pl
