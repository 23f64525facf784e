"""GPU parity of the chunkrecord index (index/chunkrecord.go:41-99 with fastq.go:216-243 /
fasta.go:143-173 SeekChunk): shockidx_chunkrecord_device through the C ABI against the C
oracle (itself pinned to a Python `re` restatement in test_oracle_chunk.py).  Bar: identical
rows, identical count, Go's detection error, SAM refused."""
import random
import zlib

import numpy as np
import pytest

from test_oracle_chunk import WIN, fasta_records, fastq_records

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["spec", "serial"])
def chunk_mode(request, monkeypatch):
    """The speculative build (default) and the serial walk (SHOCKIDX_CHUNK_MODE=serial, the
    definition it is verified against on the device) must both equal the oracle."""
    if request.param == "serial":
        monkeypatch.setenv("SHOCKIDX_CHUNK_MODE", "serial")
    else:
        monkeypatch.delenv("SHOCKIDX_CHUNK_MODE", raising=False)
    return request.param


def _run(ctx, data, fmt=None, chunk=0, cap=None):
    n = len(data)
    buf = ctx.alloc(n + 64)
    if n:
        buf.upload(data)
    cap = ctx.chunkrecord_capacity(n, chunk) if cap is None else cap
    rows = ctx.alloc(16 * max(cap, 1))
    r = ctx.chunkrecord_buffer(buf, n, rows, fmt=fmt, chunk=chunk)
    got = rows.rows(min(r.count, cap)) if r.count else np.zeros((0, 2), np.uint64)
    buf.free()
    rows.free()
    return r, got


def _cmp(ctx, oracle_lib, data, fmt, chunk):
    exp, err = oracle_lib.chunkrecord(data, fmt, chunk or oracle_lib.CHUNK_SIZE)
    assert err is None
    r, got = _run(ctx, data, fmt, chunk)
    assert r.ok, r
    assert r.count == len(exp), (r.count, len(exp))
    assert np.array_equal(got, exp), (got[:4], exp[:4])


@pytest.mark.parametrize("chunk", [WIN + 1, 40000, 0])
@pytest.mark.parametrize("variant", ["plain", "crlf", "atqual", "long"])
def test_chunk_fastq_gpu(gpu_ctx, oracle_lib, chunk, variant, chunk_mode):
    seed = zlib.crc32(f"{chunk}/{variant}/1".encode()) & 0xFFFF
    data = fastq_records(random.Random(seed), 6000 if chunk else 15000, crlf=variant == "crlf",
                         at_qual=0.3 if variant == "atqual" else 0.0, long_every=700 if variant == "long" else 0)
    try:
        _cmp(gpu_ctx, oracle_lib, data, "fastq", chunk)
    except AssertionError as e:
        raise AssertionError(f"seed={seed}: {e}") from e


@pytest.mark.parametrize("chunk", [WIN + 1, 50000, 0])
@pytest.mark.parametrize("variant", ["plain", "crlf", "long"])
def test_chunk_fasta_gpu(gpu_ctx, oracle_lib, chunk, variant, chunk_mode):
    rng = random.Random(11 + chunk)
    data = fasta_records(rng, 3000, crlf=variant == "crlf", long_every=50 if variant == "long" else 0)
    _cmp(gpu_ctx, oracle_lib, data, "fasta", chunk)


def test_chunk_fuzz_bytes_gpu(gpu_ctx, oracle_lib, chunk_mode):
    rng = random.Random(5)
    alpha = b"@@@++\n\n\r\r ACGTacgt-\t!I>"
    for _ in range(20):
        data = bytes(rng.choice(alpha) for _ in range(WIN * 3 + rng.randint(0, 5000)))
        chunk = WIN + 1 + rng.randint(0, 3000)
        _cmp(gpu_ctx, oracle_lib, data, "fastq", chunk)
        _cmp(gpu_ctx, oracle_lib, data, "fasta", chunk)


def test_chunk_dense_at_runs_gpu(gpu_ctx, oracle_lib):
    """Windows where thousands of overlapping '@' starts all match (serial-walk fallback)."""
    rec = b"@" * 6000 + b"\nA\n+\n!\n"
    _cmp(gpu_ctx, oracle_lib, rec * 40, "fastq", WIN + 7)
    rec = b"@@@@@@@@x\nAC\n+\n!!\n"
    _cmp(gpu_ctx, oracle_lib, rec * 20000, "fastq", WIN + 3)


def test_chunk_cr_runs_linear_gpu(gpu_ctx, oracle_lib):
    """'@' starts whose header `.*` can stop at any of thousands of '\r's, all of
    which fail: one evaluation per [\n\r]+ run, so such windows cost no more than plain ones.
    Byte-exact against the oracle where the oracle (quadratic there) finishes, then a
    time-bounded window the oracle could not finish (no match anywhere: one row)."""
    import time
    pats = [
        b"@" * 50 + b"x" + b"\r" * 3000 + b"\n1\n" + b"@r\nAC\n+\n!!\n" * 20,
        b"@@@@x" + b"\rA" * 1500 + b"\n+" + b"\r!" * 700 + b"\n",
        (b"@q" + b"\r" * 50 + b"AC\r+" + b"\r" * 40 + b"!!\n") * 600,
    ]
    for pat in pats:
        data = pat * (3 * WIN // len(pat) + 2)
        _cmp(gpu_ctx, oracle_lib, data, "fastq", WIN + 5)
    data = (b"@" * 1000 + b"x" + b"\r" * 30000 + b"\n1\n") * 64  # ~2 MiB
    n = len(data)
    buf = gpu_ctx.alloc(n + 64)
    buf.upload(data)
    rows = gpu_ctx.alloc(16 * gpu_ctx.chunkrecord_capacity(n, WIN + 5))
    t0 = time.perf_counter()
    r = gpu_ctx.chunkrecord_buffer(buf, n, rows, fmt="fastq", chunk=WIN + 5)
    dt = time.perf_counter() - t0
    assert r.ok and dt < 2.0, dt
    assert r.count == 1 and rows.rows(1).tolist() == [[0, n]]  # no Record match: SeekChunk to EOF
    buf.free()
    rows.free()


def test_chunk_edges_gpu(gpu_ctx, oracle_lib, chunk_mode):
    rng = random.Random(3)
    base = fastq_records(rng, 500)
    for size in (1, WIN - 1, WIN, WIN + 1, 2 * WIN, len(base)):
        _cmp(gpu_ctx, oracle_lib, base[:size], "fastq", WIN)
    # a last match ending exactly at the window end (pos clamped to 32767)
    chunk = WIN + 100
    rec, head = b"@a\nAC\n+\n!!\n", b"@h\nA\n+\n!\n"
    pad = chunk - len(head) - len(rec)
    data = head + (b"A" * 60 + b"\n") * (pad // 61) + b"A" * (pad % 61) + rec + b"@z\nA\n+\n!\n" * 4000
    _cmp(gpu_ctx, oracle_lib, data, "fastq", chunk)


def test_chunk_detect_and_errors_gpu(gpu_ctx, oracle_lib):
    rng = random.Random(9)
    fq = fastq_records(rng, 8000)
    exp, _ = oracle_lib.chunkrecord(fq, None)
    r, got = _run(gpu_ctx, fq, None)
    assert r.ok and r.fmt == "fastq" and np.array_equal(got, exp)
    r, _ = _run(gpu_ctx, b"hello world\n" * 10000, None)
    assert not r.ok and r.err == b"Invalid file type for filter"
    r, _ = _run(gpu_ctx, b"@HD\tVN:1.0\n" + b"r\t0\t*\n" * 10000, "sam")
    assert not r.ok and b"sam.SeekChunk" in r.err
    r, _ = _run(gpu_ctx, fq, "fastq", WIN, cap=2)
    assert not r.ok and r.count == len(oracle_lib.chunkrecord(fq, "fastq", WIN)[0])


def _fixed_fastq(nrec, L, crlf=False):
    nl = b"\r\n" if crlf else b"\n"
    recs = []
    for i in range(nrec):
        h = b"@r%07d" % i
        body = L - len(h) - 4 * len(nl) - 1
        recs.append(h + nl + b"A" * (body // 2) + nl + b"+" + nl + b"I" * (body - body // 2) + nl)
    out = b"".join(recs)
    return out


@pytest.mark.parametrize("crlf", [False, True])
def test_chunk_spec_exact_boundaries_gpu(gpu_ctx, oracle_lib, crlf):
    """Fixed-length records with chunk a multiple of the record length: every window ends on
    a record boundary (the match clamped to 32767, the chain continuing from window end - 1,
    and for CRLF from the '\r'), so the path runs through the delta = 1 / 2 nodes."""
    L = 200 if not crlf else 202
    data = _fixed_fastq(30000, L, crlf)
    for chunk in (L * 200, L * 171 + 1, L * 164 - 1):
        _cmp(gpu_ctx, oracle_lib, data, "fastq", chunk)


def test_chunk_spec_mispredictions_gpu(gpu_ctx, oracle_lib):
    """Files where the predicted path is wrong or absent part of the way: a FASTQ record index
    that fails half-way (no nodes after the error), blank lines and '@' quality lines (matches
    the record table does not predict), records longer than a window, CR-only FASTA pairs
    ("\r>") and '>' split across windows.  The result is the serial walk's either way."""
    rng = random.Random(77)
    good = fastq_records(rng, 9000)
    bad = good[: len(good) // 2] + b"@broken\nACGT\n+\nII\n" + good[len(good) // 2:]
    for chunk in (WIN + 1, 40000, 70001):
        _cmp(gpu_ctx, oracle_lib, bad, "fastq", chunk)
    blank = good.replace(b"\n@r1", b"\n\n\n@r1")
    _cmp(gpu_ctx, oracle_lib, blank, "fastq", 40000)
    atq = fastq_records(rng, 9000, at_qual=0.5, long_every=900)
    _cmp(gpu_ctx, oracle_lib, atq, "fastq", 40000)
    fa = fasta_records(rng, 2500, long_every=40)
    fa_cr = fa.replace(b"\n>c1", b"\r>c1")
    for chunk in (WIN + 1, 50000):
        _cmp(gpu_ctx, oracle_lib, fa_cr, "fasta", chunk)


def test_chunk_spec_many_chunks_gpu(gpu_ctx, oracle_lib):
    """Thousands of chunks per build (the jump table's levels > 0 and more than one path
    round: chunk just above the window on a 96 MiB file)."""
    rng = random.Random(5)
    base = fastq_records(rng, 20000)
    data = (base * (96 * 2**20 // len(base) + 1))[: 96 * 2**20]
    for chunk in (WIN + 1, 45000):
        _cmp(gpu_ctx, oracle_lib, data, "fastq", chunk)
    fa = fasta_records(rng, 3000)
    data = (fa * (64 * 2**20 // len(fa) + 1))[: 64 * 2**20]
    _cmp(gpu_ctx, oracle_lib, data, "fasta", WIN + 1)


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_chunk_synth_64mib_gpu(gpu_ctx, oracle_lib, fmt):
    from shock_amd.synth import SynthFile
    size = 64 << 20
    sf = SynthFile(gpu_ctx, fmt, size)
    data = sf.window(0, size)
    host = data.download(size)
    exp, err = oracle_lib.chunkrecord(host, fmt)
    assert err is None
    cap = gpu_ctx.chunkrecord_capacity(size)
    rows = gpu_ctx.alloc(16 * cap)
    r = gpu_ctx.chunkrecord_buffer(data, size, rows, fmt=fmt)
    assert r.ok and r.count == len(exp)
    assert np.array_equal(rows.rows(r.count), exp)


def test_chunk_indexer_mirror_gpu(oracle_lib, tmp_path, monkeypatch):
    """Indexers["chunkrecord"](f).Create(outPath) writes the oracle's table as the .idx file."""
    from shock_amd import indexer
    monkeypatch.setattr(indexer, "PATH_DATA", str(tmp_path))
    data = fastq_records(random.Random(21), 9000)
    src = tmp_path / "node.fastq"
    src.write_bytes(data)
    out = tmp_path / "chunkrecord.idx"
    with open(src, "rb") as f:
        count, fmt, err = indexer.Indexers["chunkrecord"](f).create(str(out))
    exp, _ = oracle_lib.chunkrecord(data)
    assert err is None and fmt == "array" and count == len(exp)
    assert out.read_bytes() == exp.astype("<u8").tobytes()


def test_chunk_indexer_file_over_2gib_gpu(gpu_ctx, oracle_lib, tmp_path, monkeypatch):
    """A node file larger than one read(2) can return (Linux caps a read at 0x7ffff000 bytes):
    Indexers["chunkrecord"] stages every byte through shockidx_chunkrecord_fd's pread loop
    (a single os.pread left the tail of the HBM buffer uninitialised)."""
    from shock_amd import indexer
    from shock_amd.synth import SynthFile
    monkeypatch.setattr(indexer, "PATH_DATA", str(tmp_path))
    size = (2 << 30) + (200 << 20)
    sf = SynthFile(gpu_ctx, "fasta", size)
    data = sf.window(0, size)
    host = data.download(size)
    data.free()
    sf.free()
    src = tmp_path / "node.fasta"
    host.tofile(src)
    exp, err = oracle_lib.chunkrecord(host, "fasta")
    assert err is None and int(exp[-1, 0]) > 0x7FFFF000
    out = tmp_path / "chunkrecord.idx"
    with open(src, "rb") as f:
        count, fmt, err = indexer.Indexers["chunkrecord"](f).create(str(out))
    assert err is None and count == len(exp)
    assert out.read_bytes() == exp.astype("<u8").tobytes()


# ---- subset nodes (index/chunkrecord.go:100-228) -------------------------------------------
def test_chunk_subset_kats_gpu(gpu_ctx, oracle_lib):
    from test_oracle_chunk_subset import KATS, _rows
    for lengths, exp in KATS:
        r = gpu_ctx.chunkrecord_subset(_rows(lengths))
        assert r.ok and r.count == len(exp), (lengths, r)
        assert [tuple(map(int, x)) for x in r.rows] == exp


def test_chunk_subset_random_gpu(gpu_ctx, oracle_lib):
    from test_oracle_chunk_subset import _rows
    rng = np.random.default_rng(11)
    MIB = 1 << 20
    for trial in range(120):
        n = int(rng.integers(0, 3000))
        kind = trial % 4
        if kind == 0:
            L = rng.integers(0, 400000, n)
        elif kind == 1:
            L = rng.choice([0, 1, 1000, MIB - 1, MIB, 3 * MIB, 300000], n)
        elif kind == 2:
            L = rng.integers(0, 2 * MIB, n) * (rng.random(n) < 0.8)
        else:
            L = rng.integers(100, 700, n * 20)
        ri = _rows([int(x) for x in L])
        exp = oracle_lib.chunkrecord_subset(ri)
        r = gpu_ctx.chunkrecord_subset(ri)
        assert r.ok and r.count == len(exp)
        assert np.array_equal(r.rows, exp)


def test_chunk_subset_large_gpu(gpu_ctx, oracle_lib):
    """The record index of a 2 GiB FASTQ node (6.2 M rows) grouped on the device straight from
    HBM (levels > 0 of the jump table), against the oracle on the same rows."""
    from shock_amd.synth import SynthFile
    size = 2 << 30
    sf = SynthFile(gpu_ctx, "fastq", size)
    data = sf.window(0, size)
    R = sf.expected_count()
    ri = gpu_ctx.alloc(16 * (R + 64))
    r = gpu_ctx.build_buffer(data, size, ri, kind="record", fmt="fastq")
    assert r.ok and r.count == R
    out = gpu_ctx.alloc(16 * R)
    c = gpu_ctx.chunkrecord_subset_device(ri.ptr, R, out.ptr, R)
    exp = oracle_lib.chunkrecord_subset(ri.rows(R))
    assert c.ok and c.count == len(exp) > 1000
    assert np.array_equal(out.rows(c.count), exp)
    for b in (ri, out, data):
        b.free()
    sf.free()


def test_chunk_subset_indexer_mirror_gpu(oracle_lib, tmp_path, monkeypatch):
    """Indexers["chunkrecord"](f, "subset", snFormat, snRecordIndexPath).Create(outPath): the
    "matrix" table from the subset node's record index file (a partial last row ignored, as
    ReadAt's io.EOF ends the Go loop); snFormat "matrix" is Go's error."""
    from shock_amd import indexer
    from test_oracle_chunk_subset import _rows
    monkeypatch.setattr(indexer, "PATH_DATA", str(tmp_path))
    rng = np.random.default_rng(3)
    ri = _rows([int(x) for x in rng.integers(0, 500000, 5000)])
    snp = tmp_path / "record.idx"
    snp.write_bytes(ri.astype("<u8").tobytes() + b"\x01\x02\x03")
    node = tmp_path / "node.fastq"
    node.write_bytes(b"")
    out = tmp_path / "chunkrecord.idx"
    with open(node, "rb") as f:
        count, fmt, err = indexer.Indexers["chunkrecord"](f, "subset", "array", str(snp)).create(str(out))
    exp = oracle_lib.chunkrecord_subset(ri)
    assert err is None and fmt == "matrix" and count == len(exp)
    assert out.read_bytes() == exp.astype("<u8").tobytes()
    with open(node, "rb") as f:
        count, fmt, err = indexer.Indexers["chunkrecord"](f, "subset", "matrix", str(snp)).create(str(tmp_path / "m"))
    assert count == 0 and err is not None and b"matrix formatted index" in err.msg
