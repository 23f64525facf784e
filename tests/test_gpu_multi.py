"""GPU: one node file built across several devices from one process (shockidx_multi_*,
SURVEY.md §8(e) for a single Shock server process, node/index.go:107-121).  The pool gives one
MI355X per box, so the group lists device 0 several times: its slabs then run one after another
and the summaries go through host memory; a group of one device exercises the RCCL path (a
world-1 communicator from ncclCommInitAll).  Bar: rows, count and Go error text equal the
oracle's single pass over the whole file and the one-device build, bit for bit."""
import os
import random

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def multi3():
    from shock_amd import MultiContext
    m = MultiContext([0, 0, 0])
    yield m
    m.close()


def _expect(oracle_lib, data, kind, fmt):
    if kind == "line":
        return oracle_lib.line_index(data)
    return oracle_lib.record_index(data, fmt) if fmt else oracle_lib.record_index(data)


def _check(r, rows, err):
    assert r.err == err, (r.err, err)
    assert r.count == len(rows), (r.count, len(rows))
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    if not np.array_equal(got, rows):
        bad = np.nonzero((got != rows).any(axis=1))[0][:5]
        raise AssertionError(f"rows {bad.tolist()}: gpu {got[bad].tolist()} oracle {rows[bad].tolist()}")


def _data(fmt, seed, n):
    rng = random.Random(seed)
    return {"fastq": lambda: gen.fastq(rng, n, at_qual=0.3, plus_id=0.3), "fasta": lambda: gen.fasta(rng, n),
            "sam": lambda: gen.sam(rng, n), "line": lambda: gen.lines(rng, n)}[fmt]()


def test_multi_exchange_kind():
    from shock_amd import MultiContext
    m = MultiContext([0, 0])
    assert not m.rccl  # a device listed twice: host exchange
    m.close()
    m1 = MultiContext([0])
    assert m1.rccl     # one device: a world-1 RCCL communicator
    m1.close()


@pytest.mark.parametrize("fmt", ["fastq", "fasta", "sam", "line"])
def test_multi_clean(multi3, gpu_ctx, oracle_lib, fmt):
    n = {"fastq": 20000, "fasta": 3000, "sam": 20000, "line": 40000}[fmt]
    data = _data(fmt, 31, n)
    kind = "line" if fmt == "line" else "record"
    rows, err = _expect(oracle_lib, data, kind, None if fmt == "line" else fmt)
    r = multi3.build_host(data, kind=kind, fmt=None if fmt == "line" else fmt)
    _check(r, rows, err)
    assert r.path == (2 if fmt == "sam" else 1), r.path
    if fmt != "line":  # format detection on the head (DetermineFormat): as the one-device build
        r1 = gpu_ctx.build_host(data, kind=kind)
        r2 = multi3.build_host(data, kind=kind)
        assert (r2.fmt, r2.status, r2.err, r2.count) == (r1.fmt, r1.status, r1.err, r1.count)
        if r1.ok:
            assert r1.fmt == fmt
            _check(r2, rows, err)


@pytest.mark.parametrize("kind", gen.FASTQ_CORRUPTIONS)
def test_multi_fastq_errors(multi3, oracle_lib, kind):
    data = _data("fastq", 3, 6000)
    rng = random.Random(kind)
    for _ in range(3):
        bad = gen.fastq_corrupt(rng, data, kind)
        rows, err = oracle_lib.record_index(bad, "fastq")
        _check(multi3.build_host(bad, fmt="fastq"), rows, err)


@pytest.mark.parametrize("kind", ["header_only", "gt_in_seq", "lead_newline", "trail_header"])
def test_multi_fasta_errors(multi3, oracle_lib, kind):
    data = _data("fasta", 5, 1500)
    rng = random.Random(kind)
    for _ in range(3):
        bad = gen.fasta_corrupt(rng, data, kind)
        rows, err = oracle_lib.record_index(bad, "fasta")
        _check(multi3.build_host(bad, fmt="fasta"), rows, err)


@pytest.mark.parametrize("fmt", ["fastq", "fasta", "sam", "line"])
def test_multi_tiny_files(oracle_lib, fmt):
    from shock_amd import MultiContext
    rng = random.Random(7)
    groups = [MultiContext([0, 0]), MultiContext([0, 0, 0, 0, 0])]
    kind = "line" if fmt == "line" else "record"
    for _ in range(30):
        d = gen.tiny(rng)
        rows, err = _expect(oracle_lib, d, kind, None if fmt == "line" else fmt)
        for m in groups:
            _check(m.build_host(d, kind=kind, fmt=None if fmt == "line" else fmt), rows, err)
    for m in groups:
        m.close()


def test_multi_halo_exhausted_falls_back(multi3, oracle_lib):
    """A FASTA record longer than the 4 MiB halo across the slab ends: rebuilt on one device."""
    rng = random.Random(11)
    data = gen.fasta(rng, 40) + b">huge\n" + gen._big_seq(rng, 12 << 20) + b"\n" + gen.fasta(rng, 40)
    rows, err = oracle_lib.record_index(data, "fasta")
    _check(multi3.build_host(data, fmt="fasta"), rows, err)


def test_multi_fd_and_create(multi3, gpu_ctx, oracle_lib, tmp_path):
    from shock_amd.synth import SynthFile
    size = (96 << 20) + 4321
    sf = SynthFile(gpu_ctx, "fastq", size)
    buf = sf.window(0, size)
    host = buf.download(size)
    buf.free()
    sf.free()
    rows, err = oracle_lib.record_index(host)
    assert err is None
    f = tmp_path / "node.data"
    host.tofile(f)
    fd = os.open(f, os.O_RDONLY)
    try:
        r = multi3.build_fd(fd, size)
        _check(r, rows, None)
        out = tmp_path / "record.idx"
        r2 = multi3.create(fd, size, "record", str(tmp_path), str(out))
        assert r2.ok and r2.count == len(rows)
        assert out.read_bytes() == rows.astype("<u8").tobytes()
    finally:
        os.close(fd)


def test_multi_resident_rccl_world1(gpu_ctx, oracle_lib):
    """The device-resident form through a world-1 RCCL communicator: windows per plan(), rows
    left on the device, the global first record and the owned count per slab."""
    from shock_amd import MultiContext
    data = _data("fastq", 9, 5000)
    rows, err = oracle_lib.record_index(data, "fastq")
    m = MultiContext([0])
    assert m.rccl
    (lo, hi, wlo, whi), = m.plan(len(data))
    assert (lo, hi, wlo, whi) == (0, len(data), 0, len(data))
    win = gpu_ctx.alloc(len(data) + 64)
    win.upload(np.frombuffer(data, np.uint8))
    d_rows = gpu_ctx.alloc(16 * (len(rows) + 64))
    r, first, owned = m.build_resident(len(data), [win.ptr], [d_rows.ptr], [len(rows) + 64], fmt="fastq")
    assert r.ok and r.count == len(rows) and first == [0] and owned == [len(rows)]
    assert np.array_equal(d_rows.rows(len(rows)), rows)
    win.free()
    d_rows.free()
    m.close()


def test_multi_resident_slabs(gpu_ctx, oracle_lib):
    """Device-resident slabs (4 windows on device 0): owned rows concatenate to the table."""
    from shock_amd import MultiContext
    data = _data("fasta", 13, 4000)
    rows, err = oracle_lib.record_index(data, "fasta")
    m = MultiContext([0, 0, 0, 0])
    plan = m.plan(len(data))
    wins, outs, caps = [], [], []
    for lo, hi, wlo, whi in plan:
        w = gpu_ctx.alloc(whi - wlo + 64)
        w.upload(np.frombuffer(data[wlo:whi], np.uint8))
        cap = (hi - lo) // 8 + 64
        wins.append(w)
        outs.append(gpu_ctx.alloc(16 * cap))
        caps.append(cap)
    r, first, owned = m.build_resident(len(data), [w.ptr for w in wins], [o.ptr for o in outs], caps, fmt="fasta")
    assert r.ok and r.count == len(rows)
    table = np.concatenate([o.rows(k) if k else np.zeros((0, 2), np.uint64) for o, k in zip(outs, owned)])
    assert first == [0] + list(np.cumsum(owned)[:-1])
    assert np.array_equal(table, rows)
    for b in wins + outs:
        b.free()
    m.close()
