"""GPU: the drop-in fd build with a bounded device footprint.

record.go streams any node through a 4 KiB bufio.Reader (record.go:51-83, fastq.go:136); the fd
build holds the whole node in HBM only when its one-pass build fits the device budget.  With a
cap (shockidx_ctx_set_dev_cap / SHOCKIDX_DEV_CAP) below that, slabs go through two slot buffers
sized to the cap.  A Go error inside a slab ends the build there (the slab was indexed with its
exact incoming state, so its error is the file's first).  A record longer than the halo across a
slab end ends the walk there, and the rest of the file is walked again from the first record not
yet emitted (its first slab starting there); only a record longer than a slab takes the one-pass
build of the rest.  Every case is compared with the C oracle
(rows, count, Go error text) and create's .idx is byte-identical."""
import os
import random

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

CAP = 300 << 20      # 64 MiB slabs (the smallest the ring takes)
SIZE = (600 << 20) + 4321


@pytest.fixture
def capped():
    from shock_amd import Context
    ctx = Context(0)
    ctx.set_dev_cap(CAP)
    yield ctx


def _synth_host(ctx, fmt, size):
    from shock_amd.synth import SynthFile
    sf = SynthFile(ctx, fmt, size)
    data = sf.window(0, size)
    host = data.download(size)
    data.free()
    sf.free()
    return host


def _run(ctx, host, tmp_path, kind="record"):
    path = tmp_path / "node.data"
    host.tofile(path)
    fd = os.open(path, os.O_RDONLY)
    try:
        r = ctx.build_fd(fd, host.size, kind=kind)
        out = tmp_path / "idx" / f"{kind}.idx"
        out.parent.mkdir(exist_ok=True)
        (tmp_path / "temp").mkdir(exist_ok=True)
        c = ctx.create(fd, host.size, kind, str(tmp_path / "temp"), str(out))
        idx = np.fromfile(out, dtype=np.uint64).reshape(-1, 2) if out.exists() else None
        if out.exists():
            out.unlink()
        left = os.listdir(tmp_path / "temp")
    finally:
        os.close(fd)
        path.unlink()
    return r, c, idx, left


def _check(oracle_lib, host, r, c, idx, left, kind="record"):
    exp, err = oracle_lib.line_index(host) if kind == "line" else oracle_lib.record_index(host)
    assert r.count == len(exp) and r.err == err, (r.count, len(exp), r.err, err)
    assert c.count == len(exp) and c.err == err
    assert left == []
    assert r.path == 4 and c.path == 4, (r.path, c.path)  # the slab pipeline through two slots
    if err is None:
        assert r.ok and np.array_equal(r.rows, exp)
        assert idx is not None and np.array_equal(idx, exp)
    else:
        assert idx is None
        if r.rows is not None and len(exp):
            assert np.array_equal(r.rows[:len(exp)], exp)
    return exp


@pytest.mark.parametrize("fmt,kind", [("fastq", "record"), ("fasta", "record"), ("fastq", "line")])
def test_ring_clean(capped, oracle_lib, tmp_path, fmt, kind):
    host = _synth_host(capped, fmt, SIZE)
    r, c, idx, left = _run(capped, host, tmp_path, kind)
    _check(oracle_lib, host, r, c, idx, left, kind)
    assert r.reruns == 0  # every slab clean: no fallback
    assert capped.workspace_bytes() <= CAP  # what the context keeps after the build


@pytest.mark.parametrize("case", ["fastq_plus", "fastq_blank_tail", "fasta_gt_in_seq", "fastq_trunc_end"])
def test_ring_errors(capped, oracle_lib, tmp_path, case):
    """A Go error, blank lines right before a slab boundary (fastq.go:161-163: an error mid-file),
    a '>' inside a sequence line, a truncated last record: the rows of the clean slabs before it
    and the error, from the slab that holds it (no re-read)."""
    fmt = "fasta" if case.startswith("fasta") else "fastq"
    b = _synth_host(capped, fmt, SIZE)
    at = 520 << 20  # late enough that the rest fits the cap (one_pass_bytes: ~1.8 x the rest + 64 MiB)
    if case == "fastq_plus":
        w = b[at:at + 8192]
        p = int(np.flatnonzero((w[1:] == ord("+")) & (w[:-1] == ord("\n")))[0]) + at + 1
        b[p] = ord("x")
    elif case == "fastq_blank_tail":
        p = (576 << 20) - 2000  # a blank group right before a slab boundary (64 MiB slabs)
        s = int(np.flatnonzero(b[p:p + 4096] == ord("@"))[0]) + p
        e = int(np.flatnonzero(b[s + 1:s + 8192] == ord("@"))[0]) + s + 1
        while b[e - 1] != ord("\n"):
            e = int(np.flatnonzero(b[e + 1:e + 8192] == ord("@"))[0]) + e + 1
        b[s:e] = ord("\n")
    elif case == "fasta_gt_in_seq":
        g = int(np.flatnonzero(b[at:at + 65536] == ord(">"))[0]) + at
        nl = int(np.flatnonzero(b[g:g + 65536] == ord("\n"))[0]) + g
        b[nl + 3] = ord(">")
    elif case == "fastq_trunc_end":
        b = b[:-100].copy()
    r, c, idx, left = _run(capped, b, tmp_path)
    exp = _check(oracle_lib, b, r, c, idx, left)
    assert r.reruns == 0 and len(exp) > 0
    if case in ("fastq_plus", "fastq_blank_tail"):  # (the others: as the oracle decides)
        assert r.err is not None


def _fq_record(b, at):
    """The four line starts of the first FASTQ record starting at or after byte `at`."""
    p = at
    while True:
        p = int(np.flatnonzero(b[p:p + 65536] == ord("@"))[0]) + p
        if p == 0 or b[p - 1] == ord("\n"):
            ls = [p]
            for _ in range(4):
                ls.append(int(np.flatnonzero(b[ls[-1]:ls[-1] + 65536] == ord("\n"))[0]) + ls[-1] + 1)
            if b[ls[2]] == ord("+") and ls[4] - ls[3] == ls[2] - ls[1]:
                return ls
        p += 1


def _fa_record(b, at):
    """The header start and the first sequence line start of the first FASTA record at or after `at`."""
    g = int(np.flatnonzero(b[at:at + (1 << 20)] == ord(">"))[0]) + at
    while g and b[g - 1] != ord("\n"):
        g = int(np.flatnonzero(b[g + 1:g + 1 + (1 << 20)] == ord(">"))[0]) + g + 1
    return g, int(np.flatnonzero(b[g:g + 65536] == ord("\n"))[0]) + g + 1


# in the first slab (its one-pass fallback would need the whole node: more than the cap), across
# the first slab boundary (the record starts in slab 0 and ends in its halo), in a middle slab, in
# the last slab
SWEEP_AT = [3000, (64 << 20) - 200, 200 << 20, SIZE - (1 << 20)]
FQ_KINDS = ["no_at", "no_plus", "empty_seq", "len_mismatch", "missing_id", "id_mismatch"]
FA_KINDS = ["gt_in_seq", "header_header"]


def _fq_corrupt(b, at, kind):
    ls = _fq_record(b, at)
    if kind == "no_at":
        b = b.copy(); b[ls[0]] = ord("X")
    elif kind == "no_plus":
        b = b.copy(); b[ls[2]] = ord("-")
    elif kind == "empty_seq":
        b = np.concatenate([b[:ls[1]], b[ls[2] - 1:]])
    elif kind == "len_mismatch":
        b = np.concatenate([b[:ls[4] - 1], np.frombuffer(b"I", np.uint8), b[ls[4] - 1:]])
    elif kind == "missing_id":
        b = np.concatenate([b[:ls[0] + 1], b[ls[1] - 1:]])
    elif kind == "id_mismatch":
        b = np.concatenate([b[:ls[2] + 1], np.frombuffer(b"zz", np.uint8), b[ls[2] + 1:]])
    return b


@pytest.mark.parametrize("kind", FQ_KINDS + FA_KINDS)
def test_ring_error_sweep(capped, oracle_lib, tmp_path, kind):
    """Every FASTQ / FASTA corruption kind at four places of a capped build (ADVICE r5 / VERDICT
    r5 #3): Go's error and the rows before it, reported by the slab that holds it, even in the
    first slab, where the one-pass fallback of round 5 refused the node with SHOCKIDX_ENOMEM."""
    fmt = "fasta" if kind in FA_KINDS else "fastq"
    base = _synth_host(capped, fmt, SIZE)
    for at in SWEEP_AT:
        if fmt == "fastq":
            b = _fq_corrupt(base, at, kind)
        else:
            g, s = _fa_record(base, at)
            if kind == "gt_in_seq":
                b = np.concatenate([base[:s + 2], np.frombuffer(b">", np.uint8), base[s + 2:]])
            else:  # a header line followed by another header line
                b = np.concatenate([base[:s], np.frombuffer(b">hdr\n", np.uint8), base[s:]])
        r, c, idx, left = _run(capped, b, tmp_path)
        exp = _check(oracle_lib, b, r, c, idx, left)
        if r.err is not None:
            assert r.reruns == 0, (kind, at, r.err)  # from the slab, no re-read


def test_ring_long_records(capped, oracle_lib, tmp_path):
    """A FASTA record longer than the 4 MiB halo across a slab boundary (a chromosome-sized
    contig): the slab before it cannot close it (ST_NEEDMORE), so the walk ends there and the
    rest of the node is walked again from the contig's start."""
    rng = random.Random(61)
    head = gen.fasta(rng, 2000)
    reps = (380 << 20) // len(head)
    line = b"ACGT" * 20 + b"\n"
    long_rec = b">contig1 len=16777216\n" + line * ((16 << 20) // len(line))
    tail = gen.fasta(rng, 4000)
    host = np.frombuffer(head * reps + long_rec + tail, np.uint8).copy()
    start = len(head) * reps
    assert start < (384 << 20) and start + len(long_rec) > (384 << 20) + (5 << 20)  # past the halo
    r, c, idx, left = _run(capped, host, tmp_path)
    _check(oracle_lib, host, r, c, idx, left)
    assert r.reruns >= 1  # the walk ended at the long record and restarted there


def test_ring_many_long_records(capped, oracle_lib, tmp_path):
    """Contigs of 6-40 MiB all through a 600 MiB node, the first one in the first slab: every slab
    end a contig crosses past the halo restarts the walk at that contig (no one-pass of the rest,
    which would not fit the cap this early)."""
    rng = random.Random(63)
    line = b"ACGT" * 20 + b"\n"
    parts, size, i = [], 0, 0
    while size < SIZE:
        head = gen.fasta(rng, rng.randint(50, 400))
        L = rng.randint(6, 40) << 20
        rec = b">contig%d len=%d\n" % (i, L) + line * (L // len(line))
        parts += [head, rec]
        size += len(head) + len(rec)
        i += 1
    host = np.frombuffer(b"".join(parts)[:SIZE], np.uint8).copy()
    r, c, idx, left = _run(capped, host, tmp_path)
    _check(oracle_lib, host, r, c, idx, left)
    assert r.reruns >= 3


def _dense(kind, R):
    """R bytes of 8-byte lines (kind line) or 9-byte FASTQ records (record), the last one
    stretched so that they end exactly at R."""
    if kind == "line":
        m = R // 8
        return b"abcdefg\n" * m + (b"x" * (R - 8 * m - 1) + b"\n" if R - 8 * m else b"")
    m = (R - 10) // 9
    last = R - 9 * m  # 10..18 bytes: "@a\n" + k + "\n+\n" + k + "\n" (7 + 2k) or "@ab\n"... (8 + 2k)
    idl = b"@a\n" if last % 2 else b"@ab\n"
    k = (last - len(idl) - 4) // 2
    return b"@a\nA\n+\nI\n" * m + idl + b"A" * k + b"\n+\n" + b"I" * k + b"\n"


@pytest.mark.parametrize("kind", ["line", "record"])
def test_ring_dense_rows(capped, oracle_lib, tmp_path, kind):
    """A ~64 MiB stretch of 8-byte lines / 9-byte FASTQ records inside a capped node: that slab
    holds more rows than its share (16 B of rows per 32 input bytes), so it runs again into rows
    grown to its count, in its slot -- no restart, no one-pass of the rest."""
    host = _synth_host(capped, "fastq", SIZE)
    lo = _fq_record(host, 128 << 20)[0]
    hi = _fq_record(host, lo + (64 << 20))[0]
    d = _dense(kind, hi - lo)
    assert len(d) == hi - lo
    host[lo:hi] = np.frombuffer(d, np.uint8)
    r, c, idx, left = _run(capped, host, tmp_path, kind)
    exp = _check(oracle_lib, host, r, c, idx, left, kind)
    assert r.err is None and r.reruns == 0 and len(exp) > (6 << 20)


def test_ring_junk(capped, oracle_lib, tmp_path):
    """An undetectable node: Go's detection error, as the one-pass build reports it."""
    junk = np.frombuffer(b"xy" * (SIZE // 2), np.uint8).copy()
    r, c, idx, left = _run(capped, junk, tmp_path)
    assert r.err == b"Invalid file type for filter" and c.err == r.err and r.count == 0 and idx is None


def test_ring_early_long_restart(capped, oracle_lib, tmp_path):
    """A 16 MiB contig across the FIRST slab end: the walk restarts at the contig (the one-pass
    build of the rest would need more than the cap)."""
    rng = random.Random(62)
    head = gen.fasta(rng, 2000)
    line = b"ACGT" * 20 + b"\n"
    long_rec = b">contig1 len=16777216\n" + line * ((16 << 20) // len(line))
    head = head * ((60 << 20) // len(head))
    tail = gen.fasta(rng, 4000)
    body = head + long_rec
    body += tail * ((SIZE - len(body)) // len(tail) + 1)
    b = np.frombuffer(body[:SIZE], np.uint8).copy()
    r, c, idx, left = _run(capped, b, tmp_path)
    _check(oracle_lib, b, r, c, idx, left)
    assert r.reruns == 1


def test_ring_early_huge_enomem(capped, oracle_lib, tmp_path):
    """A 72 MiB contig (longer than a 64 MiB slab and its halo) early in the node: no walk can
    close it from its own start, and the one-pass build of the rest needs more than the cap --
    refused with SHOCKIDX_ENOMEM (never a short table)."""
    from shock_amd import _lib as L
    rng = random.Random(64)
    head = gen.fasta(rng, 2000)
    line = b"ACGT" * 20 + b"\n"
    long_rec = b">chr1 len=75497472\n" + line * ((72 << 20) // len(line))
    head = head * ((60 << 20) // len(head))
    tail = gen.fasta(rng, 4000)
    body = head + long_rec
    body += tail * ((SIZE - len(body)) // len(tail) + 1)
    b = np.frombuffer(body[:SIZE], np.uint8).copy()
    path = tmp_path / "early.data"
    b.tofile(path)
    fd = os.open(path, os.O_RDONLY)
    try:
        with pytest.raises(L.ShockIdxError) as e:
            capped.build_fd(fd, b.size)
        assert e.value.code == L.ENOMEM and "does not fit" in str(e.value)
    finally:
        os.close(fd)


def test_ring_pin_budget(capped, oracle_lib, tmp_path, monkeypatch):
    """A process-wide pin budget below the node (SHOCKIDX_PIN_CAP_GIB=0.3): the slab
    walk unpins the page-cache chunks behind its current slab to pin the next ones, and whatever
    does not get a reservation goes through the staging buffers -- the same table."""
    monkeypatch.setenv("SHOCKIDX_PIN_CAP_GIB", "0.3")
    host = _synth_host(capped, "fastq", SIZE)
    r, c, idx, left = _run(capped, host, tmp_path)
    _check(oracle_lib, host, r, c, idx, left)
    monkeypatch.setenv("SHOCKIDX_PIN_CAP_GIB", "-1")  # (clamped: nothing pinned, all staged)
    r, c, idx, left = _run(capped, host, tmp_path)
    _check(oracle_lib, host, r, c, idx, left)
