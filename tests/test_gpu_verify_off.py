"""GPU parity with the whole-table check OFF: the suite runs with SHOCKIDX_VERIFY=1
(tests/conftest.py), which adds k_verify_rows to every build; production runs without it.  These
cases build with it off -- the default build, as Shock runs it -- and compare rows, count and Go
error text with the oracle: single-slab builds of every format and the line index, a multi-slab
FASTQ / FASTA file through the fd pipeline, and corrupted FASTQ."""
import os
import random
import zlib

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

CASES = {
    "fastq": lambda r: gen.fastq(r, 20000, plus_id=0.1),
    "fastq_crlf": lambda r: gen.fastq(r, 8000, crlf=1.0),
    "fasta": lambda r: gen.fasta(r, 3000),
    "fasta_long": lambda r: gen.fasta(r, 200, long_every=40, long_len=90000),
    "sam": lambda r: gen.sam(r, 5000, headers=300),
    "lines": lambda r: gen.lines(r, 20000),
}


@pytest.fixture
def verify_off(monkeypatch):
    monkeypatch.setenv("SHOCKIDX_VERIFY", "0")  # (read by every build: sidx_capi.cpp verify_rows)


def _cmp(ctx, oracle_lib, data, mode, tag):
    if mode == "line":
        r = ctx.build_host(data, kind="line")
        exp, err = oracle_lib.line_index(data)
    else:
        r = ctx.build_host(data, kind="record", fmt=None if mode == "auto" else mode)
        exp, err = oracle_lib.record_index(data, None if mode == "auto" else mode)
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    assert r.count == len(exp) and r.err == err, (tag, mode, r.count, len(exp), r.err, err)
    assert np.array_equal(got, exp), (tag, mode)


@pytest.mark.parametrize("case", sorted(CASES))
def test_verify_off_generated(gpu_ctx, oracle_lib, verify_off, case):
    seed = zlib.crc32(f"verify_off/{case}".encode()) & 0xFFFF
    data = CASES[case](random.Random(seed))
    for mode in ("auto", "fastq", "fasta", "line"):
        _cmp(gpu_ctx, oracle_lib, data, mode, f"{case} seed={seed}")


@pytest.mark.parametrize("kind", gen.FASTQ_CORRUPTIONS)
def test_verify_off_fastq_corruptions(gpu_ctx, oracle_lib, verify_off, kind):
    seed = zlib.crc32(f"verify_off/corrupt/{kind}".encode()) & 0xFFFF
    rng = random.Random(seed)
    data = gen.fastq_corrupt(rng, gen.fastq(rng, 3000), kind)
    _cmp(gpu_ctx, oracle_lib, data, "auto", f"{kind} seed={seed}")


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_verify_off_fd_pipeline(gpu_ctx, oracle_lib, verify_off, tmp_path, fmt):
    """A 2.5 GiB node through the slab-pipelined fd build (slab walks with exact incoming states)."""
    from shock_amd.synth import SynthFile
    size = (5 << 29) + 777
    sf = SynthFile(gpu_ctx, fmt, size)
    buf = sf.window(0, size)
    host = buf.download(size)
    buf.free()
    sf.free()
    path = tmp_path / "node.data"
    host.tofile(path)
    fd = os.open(path, os.O_RDONLY)
    try:
        r = gpu_ctx.build_fd(fd, size)
    finally:
        os.close(fd)
    exp, err = oracle_lib.record_index(host)
    assert r.ok and err is None and r.path == 3 and np.array_equal(r.rows, exp)
