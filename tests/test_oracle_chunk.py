"""chunkrecord oracle (oracle/chunk_oracle.c) pinned against an independent restatement.

The reference (index/chunkrecord.go:41-99, fastq.go:216-243, fasta.go:143-173) cannot run here
(no Go toolchain) and its tests hold no chunkrecord vectors.  The second restatement below uses
Python's backtracking `re` for fastq.Record (fastq.go:23): leftmost-first like Go's RE2, with
RE2's ASCII \\s = [\\t\\n\\f\\r ] spelled out (Python's bytes \\s also holds \\v).
"""
import os
import random
import zlib
import re
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import oracle  # noqa: E402

WIN = 32768
RECORD = re.compile(rb"@[^\t\n\f\r ](.*)?[\n\r]+[A-Za-z\-]+[\n\r]+\+(.*)?[\n\r]+([^\t\n\f\r ]+)[\n\r]+")


def py_seek_chunk(data, fmt, chunk, off, last):
    """fastq.go:216-243 / fasta.go:143-173 with the recursion unrolled; returns (n, eof)."""
    acc = 0
    while True:
        w = off + chunk - WIN
        if w + WIN > len(data):
            return acc, True
        buf = data[w:w + WIN]
        if fmt == "fastq":
            ms = list(RECORD.finditer(buf)) if last else [m for m in [RECORD.search(buf)] if m]
            if ms:
                loc = ms[-1] if last else ms[0]
                return acc + chunk - WIN + min(loc.end(), WIN - 1), False
        else:
            find = buf.rfind if last else buf.find
            pos = find(b"\n>")
            if pos == -1:
                pos = find(b"\r>")
            if pos != -1:
                return acc + chunk - WIN + pos + 1, False
        acc += WIN
        off += WIN
        last = False


def py_chunkrecord(data, fmt, chunk=oracle.CHUNK_SIZE):
    rows, curr = [], 0
    while True:
        n, eof = py_seek_chunk(data, fmt, chunk, curr, True)
        rows.append((curr, len(data) - curr if eof else n))
        curr += n
        if eof:
            return np.array(rows, dtype=np.uint64).reshape(-1, 2)


def fastq_records(rng, k, crlf=False, at_qual=0.0, long_every=0):
    out = []
    nl = b"\r\n" if crlf else b"\n"
    for i in range(k):
        L = rng.randint(1, 300)
        if long_every and i % long_every == long_every - 1:
            L = rng.randint(40000, 70000)
        seq = bytes(rng.choice(b"ACGTN") for _ in range(min(L, 64))) * (L // 64 + 1)
        seq = seq[:L]
        q = bytes(rng.randint(33, 74) for _ in range(min(L, 64))) * (L // 64 + 1)
        q = q[:L]
        if rng.random() < at_qual:
            q = b"@" + q[1:]
        plus = b"+" if rng.random() < 0.8 else b"+r%d" % i
        out.append(b"@r%d x" % i + nl + seq + nl + plus + nl + q + nl)
    return b"".join(out)


def fasta_records(rng, k, crlf=False, long_every=0):
    out = []
    nl = b"\r\n" if crlf else b"\n"
    for i in range(k):
        L = rng.randint(1, 3000)
        if long_every and i % long_every == long_every - 1:
            L = rng.randint(40000, 90000)
        body = bytes(rng.choice(b"ACGT") for _ in range(min(L, 80))) * (L // 80 + 1)
        body = body[:L]
        lines = nl.join(body[j:j + 70] for j in range(0, L, 70))
        out.append(b">c%d d" % i + nl + lines + nl)
    return b"".join(out)


def check(data, fmt, chunk):
    got, err = oracle.chunkrecord(data, fmt, chunk)
    assert err is None
    exp = py_chunkrecord(data, fmt, chunk)
    assert np.array_equal(got, exp), (fmt, chunk, got[:4], exp[:4])
    assert got[0, 0] == 0 and int(got[-1, 0] + got[-1, 1]) == len(data)
    assert np.all(got[1:, 0] == np.cumsum(got[:-1, 1])[: len(got) - 1])
    return got


@pytest.mark.parametrize("chunk", [WIN + 1, 40000, 65536, 1 << 20])
@pytest.mark.parametrize("variant", ["plain", "crlf", "atqual", "long"])
def test_fastq_vs_python_re(chunk, variant):
    seed = zlib.crc32(f"{chunk}/{variant}".encode()) & 0xFFFF
    k = 6000 if chunk < (1 << 20) else 15000
    data = fastq_records(random.Random(seed), k, crlf=variant == "crlf", at_qual=0.3 if variant == "atqual" else 0.0,
                         long_every=700 if variant == "long" else 0)
    try:
        check(data, "fastq", chunk)
    except AssertionError as e:
        raise AssertionError(f"seed={seed}: {e}") from e


@pytest.mark.parametrize("chunk", [WIN + 1, 50000, 1 << 20])
@pytest.mark.parametrize("variant", ["plain", "crlf", "long"])
def test_fasta_vs_python(chunk, variant):
    rng = random.Random(7 + chunk)
    data = fasta_records(rng, 3000, crlf=variant == "crlf", long_every=50 if variant == "long" else 0)
    check(data, "fasta", chunk)


def test_fastq_fuzz_bytes():
    """Random bytes over the regex alphabet: every choice point of Record exercised."""
    rng = random.Random(99)
    alpha = b"@@@++\n\n\r\r ACGTacgt-\t!I"
    for t in range(40):
        data = bytes(rng.choice(alpha) for _ in range(WIN * 3 + rng.randint(0, 5000)))
        check(data, "fastq", WIN + 1 + rng.randint(0, 3000))


def test_record_at_choice_points():
    # header `.*` stops at an inner '\r' (the line's '\n' fails: the plus line is not next)
    b = b"@x\rACGT\n+\nIIII\n"
    assert oracle.fq_record_at(b, 0) == len(b) == RECORD.match(b).end()
    # plus-line `.*` stops at an inner '\r' when the quality line holds a space
    b = b"@r1\nACGT\n+a\rIIII\nII II\n"
    assert oracle.fq_record_at(b, 0) == RECORD.match(b).end()
    # \v is not RE2 whitespace: @\v starts a record
    b = b"@\vid\nAC\n+\n!!\n"
    assert oracle.fq_record_at(b, 0) == len(b)
    assert oracle.fq_record_at(b"@ id\nAC\n+\n!!\n", 0) == -1
    # trailing newline runs are consumed greedily
    b = b"@a\nAC\n+\n!!\n\r\n\n@b"
    assert oracle.fq_record_at(b, 0) == len(b) - 2


def test_match_at_window_end_is_clamped():
    """A last match ending exactly at the window end gives pos = len(buf)-1 (fastq.go:241)."""
    chunk = WIN + 100
    rec = b"@a\nAC\n+\n!!\n"
    head = b"@h\nA\n+\n!\n"
    pad_len = chunk - len(head) - len(rec)
    filler = (b"A" * 60 + b"\n") * (pad_len // 61) + b"A" * (pad_len % 61)
    data = head + filler + rec + b"@z\nA\n+\n!\n" * 4000
    rows = check(data, "fastq", chunk)
    assert rows[0, 1] == chunk - 1


def test_exact_eof_boundaries():
    rng = random.Random(3)
    base = fastq_records(rng, 500)
    for size in (WIN - 1, WIN, WIN + 1, 2 * WIN, len(base)):
        check(base[:size], "fastq", WIN)


def test_detection_and_sam():
    rows, err = oracle.chunkrecord(b"hello world\n" * 10000)
    assert err == b"Invalid file type for filter" and len(rows) == 0
    with pytest.raises(RuntimeError):
        oracle.chunkrecord(b"@HD\tVN:1.0\n" + b"r\t0\t*\n" * 10000, "sam")
