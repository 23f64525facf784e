"""GPU: the slab-pipelined drop-in path -- shockidx_build_fd / shockidx_create over a node file of
two or more 1 GiB slabs (node.AsyncIndexer hands the opened node file to Create,
shock-server/node/index.go:107-121).  Slabs are indexed while later slabs are still read and
their rows go to the caller's table / the temp .idx file as they arrive; anything but a clean slab
falls back to the one-pass build.  Every case is compared with the C oracle (rows, count, format,
Go error text) and with the one-pass build (SHOCKIDX_NO_FD_PIPE); create's .idx is byte-identical
and nothing is renamed on an error."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZE = (5 << 29) + 12345  # 2.5 GiB: three slabs, the last one short


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


def _check(oracle_lib, host, r, c, idx, left, kind="record", piped=True):
    exp, err = oracle_lib.line_index(host) if kind == "line" else oracle_lib.record_index(host)
    assert r.count == len(exp) and r.err == err, (r.count, len(exp), r.err, err)
    assert c.count == len(exp) and c.err == err
    assert left == []  # the temp file was renamed or removed
    if err is None:
        assert r.ok and np.array_equal(r.rows, exp)
        assert idx is not None and np.array_equal(idx, exp)
        if piped:
            assert r.path == 3 and c.path == 3, (r.path, c.path)
    else:
        assert idx is None  # nothing renamed into outPath on an error
        if r.rows is not None and len(exp):
            assert np.array_equal(r.rows[:len(exp)], exp)
    return exp


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_fd_pipeline_clean_gpu(gpu_ctx, oracle_lib, tmp_path, monkeypatch, fmt):
    host = _synth_host(gpu_ctx, fmt, SIZE)
    r, c, idx, left = _run(gpu_ctx, host, tmp_path)
    assert r.fmt == fmt and c.fmt == fmt
    exp = _check(oracle_lib, host, r, c, idx, left)
    monkeypatch.setenv("SHOCKIDX_NO_FD_PIPE", "1")
    r2, c2, idx2, left2 = _run(gpu_ctx, host, tmp_path)
    assert r2.path != 3 and r2.ok and np.array_equal(r2.rows, exp) and np.array_equal(idx2, exp)


def test_fd_pipeline_line_gpu(gpu_ctx, oracle_lib, tmp_path):
    host = _synth_host(gpu_ctx, "fastq", SIZE)
    r, c, idx, left = _run(gpu_ctx, host, tmp_path, kind="line")
    _check(oracle_lib, host, r, c, idx, left, kind="line")


@pytest.mark.parametrize("case", ["fastq_plus", "fastq_blank_tail", "fasta_gt_in_seq", "junk"])
def test_fd_pipeline_fallback_gpu(gpu_ctx, oracle_lib, tmp_path, case):
    """A Go error in the second slab, a blank group before a slab boundary (legal only at the
    end), a FASTA '>' inside a sequence line, an undetectable file: the one-pass result."""
    fmt = "fasta" if case.startswith("fasta") else "fastq"
    if case == "junk":
        host = np.frombuffer(b"xy" * (SIZE // 2), np.uint8).copy()
    else:
        host = _synth_host(gpu_ctx, fmt, SIZE)
    b = host
    if case == "fastq_plus":
        p = (1 << 30) + (300 << 20)
        w = b[p:p + 8192]
        p = int(np.flatnonzero((w[1:] == ord("+")) & (w[:-1] == ord("\n")))[0]) + p + 1
        b[p] = ord("x")  # a plus line that does not start with '+'
    elif case == "fastq_blank_tail":
        p = (1 << 30) - 2000
        s = int(np.flatnonzero(b[p:p + 4096] == ord("@"))[0]) + p
        e = int(np.flatnonzero(b[s + 1:s + 8192] == ord("@"))[0]) + s + 1
        while b[e - 1] != ord("\n"):
            e = int(np.flatnonzero(b[e + 1:e + 8192] == ord("@"))[0]) + e + 1
        b[s:e] = ord("\n")
    elif case == "fasta_gt_in_seq":
        p = (2 << 30) + (100 << 20)
        g = int(np.flatnonzero(b[p:p + 65536] == ord(">"))[0]) + p
        nl = int(np.flatnonzero(b[g:g + 65536] == ord("\n"))[0]) + g
        b[nl + 3] = ord(">")  # inside the record's first sequence line
    r, c, idx, left = _run(gpu_ctx, b, tmp_path)
    _check(oracle_lib, b, r, c, idx, left, piped=False)
    if case != "fasta_gt_in_seq":  # (a '>' after a '\n' is a boundary; the slab may stay clean)
        assert r.err is not None


def test_fd_pipeline_pin_cap_gpu(gpu_ctx, oracle_lib, tmp_path, monkeypatch):
    """A pin cap below the file (SHOCKIDX_PIN_CAP_GIB): the first 0.75 GiB from the
    pinned page cache, the rest through the staging buffers -- the same table."""
    host = _synth_host(gpu_ctx, "fastq", SIZE)
    monkeypatch.setenv("SHOCKIDX_PIN_CAP_GIB", "0.75")
    r, c, idx, left = _run(gpu_ctx, host, tmp_path)
    _check(oracle_lib, host, r, c, idx, left)
