"""GPU parity: the HIP path (through the C ABI) against the golden vectors and the oracle.

Bar: bit-exact rows, identical record count and identical Go error text."""
import hashlib
import json
import os
import random
import zlib

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
KATS = json.load(open(os.path.join(GOLD, "kats.json")))
MANIFEST = json.load(open(os.path.join(GOLD, "expected", "manifest.json")))


def _gpu(ctx, data, mode):
    if mode == "line":
        return ctx.build_host(data, kind="line")
    return ctx.build_host(data, kind="record", fmt=None if mode == "auto" else mode)


def _check(ctx, oracle_lib, data, mode):
    r = _gpu(ctx, data, mode)
    if mode == "line":
        rows, err = oracle_lib.line_index(data)
    else:
        rows, err = oracle_lib.record_index(data, None if mode == "auto" else mode)
    assert r.count == len(rows), (mode, r.count, len(rows), r.err, err)
    assert r.err == err, (mode, r.err, err)
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    assert got.shape == rows.shape
    if not np.array_equal(got, rows):
        bad = np.nonzero((got != rows).any(axis=1))[0][:5]
        raise AssertionError(f"{mode}: first mismatching rows {bad.tolist()}: gpu {got[bad].tolist()} "
                             f"oracle {rows[bad].tolist()}")
    return r


@pytest.mark.parametrize("kat", KATS["record_kats"], ids=lambda k: k["id"])
def test_kat_gpu(gpu_ctx, kat):
    data = bytes.fromhex(kat["input_hex"])
    r = _gpu(gpu_ctx, data, kat["mode"])
    assert r.rows.tolist() == kat["rows"]
    assert (r.err.hex() if r.err is not None else None) == kat["err_hex"]


@pytest.mark.parametrize("kat", KATS["detect_kats"], ids=lambda k: k["id"])
def test_detect_gpu(gpu_ctx, kat):
    data = bytes.fromhex(kat["input_hex"])
    _, mask = gpu_ctx.detect(data)
    assert [n for i, n in enumerate(("fasta", "fastq", "sam")) if mask >> i & 1] == kat["matches"]


@pytest.mark.parametrize("name", sorted(MANIFEST))
@pytest.mark.parametrize("mode", ("auto", "fasta", "fastq", "sam", "line"))
def test_fixture_gpu(gpu_ctx, name, mode):
    data = open(os.path.join(GOLD, "fixtures", name), "rb").read()
    exp = MANIFEST[name]["modes"][mode]
    r = _gpu(gpu_ctx, data, mode)
    idx = (r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)).astype("<u8").tobytes()
    assert r.count == exp["count"]
    assert (r.err.hex() if r.err is not None else None) == exp["err_hex"]
    assert hashlib.sha256(idx).hexdigest() == exp["idx_sha256"]


def test_tiny_fuzz_gpu(gpu_ctx, oracle_lib):
    rng = random.Random(1234)
    for _ in range(400):
        d = gen.tiny(rng)
        for mode in ("fasta", "fastq", "sam", "line"):
            _check(gpu_ctx, oracle_lib, d, mode)


CASES = {
    "fastq_plain": lambda r: gen.fastq(r, 30000, plus_id=0.1),
    "fastq_crlf_uni": lambda r: gen.fastq(r, 5000, crlf=0.3, uni=0.05, at_qual=0.3),
    "fastq_long": lambda r: gen.fastq(r, 400, long_every=7, long_len=90000),
    "fastq_nofinal_nl": lambda r: gen.fastq(r, 3000, final_nl=False),
    "fastq_trailing_blank": lambda r: gen.fastq(r, 3000, trail_blank=70000),
    "fasta_plain": lambda r: gen.fasta(r, 5000),
    "fasta_long": lambda r: gen.fasta(r, 300, long_every=5, long_len=200000, embedded_gt=0.2),
    "fasta_crlf_uni": lambda r: gen.fasta(r, 2000, crlf=0.3, uni=0.1, blank=0.2),
    "fasta_nofinal": lambda r: gen.fasta(r, 2000, final_nl=False),
    "fasta_lead_cr": lambda r: gen.fasta(r, 500, lead=b"\r\n\r"),
    "sam": lambda r: gen.sam(r, 20000, headers=3000),
    "lines": lambda r: gen.lines(r, 50000, long_every=997, long_len=120000),
    "lines_nofinal": lambda r: gen.lines(r, 20000, final_nl=False),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_generated_gpu(gpu_ctx, oracle_lib, case):
    seed = zlib.crc32(case.encode()) & 0xFFFF  # (not hash(): str hashes are salted per process)
    data = CASES[case](random.Random(seed))
    for mode in ("auto", "fasta", "fastq", "sam", "line"):
        try:
            _check(gpu_ctx, oracle_lib, data, mode)
        except AssertionError as e:
            raise AssertionError(f"case={case} seed={seed} mode={mode}: {e}") from e


def _fastq_seg(rng, nrec, lmin, lmax, idlen):
    out = []
    for _ in range(nrec):
        L = rng.randint(lmin, lmax)
        rid = b"r" + bytes(rng.choice(b"0123456789") for _ in range(idlen))
        out.append(b"@" + rid + b"\n" + bytes(rng.choice(b"ACGT") for _ in range(L)) + b"\n+\n" +
                   bytes(rng.randint(33, 74) for _ in range(L)) + b"\n")
    return b"".join(out)


def test_fastq_density_mix_gpu(gpu_ctx, oracle_lib):
    """Tiles of every record density back to back in one file: records of about 320 bytes (about
    50 per 16 KiB tile), of about 140 (past the 64 one wave certifies in one step), of about 14
    (more than the 256 starts a tile keeps: the tile goes to k_fixup whole) -- so the tile pass's
    packed per-workgroup start arrays hold arrays of every length, and empty ones, at every
    offset next to each other (round 5, SIDX_FQ_PACK)."""
    rng = random.Random(77)
    segs = []
    for i in range(24):
        kind = i % 3
        if kind == 0:
            segs.append(_fastq_seg(rng, rng.randint(50, 400), 1, 300, 6))
        elif kind == 1:
            segs.append(_fastq_seg(rng, rng.randint(100, 900), 50, 70, 4))
        else:
            segs.append(_fastq_seg(rng, rng.randint(500, 3000), 1, 3, 2))
    # 40 copies: more tiles than the tile pass has workgroups, so workgroups append several
    # arrays (the copies' offsets relative to the tiles all differ: 952,820 bytes each)
    data = b"".join(segs) * 40
    for mode in ("fastq", "auto"):
        _check(gpu_ctx, oracle_lib, data, mode)


@pytest.mark.parametrize("kind", gen.FASTQ_CORRUPTIONS)
def test_fastq_corruptions_gpu(gpu_ctx, oracle_lib, kind):
    for seed in range(3):
        rng = random.Random(seed * 100 + len(kind))
        data = gen.fastq_corrupt(rng, gen.fastq(rng, 4000), kind)
        r = _check(gpu_ctx, oracle_lib, data, "fastq")
        if kind not in ("trail_partial",):
            assert r.err is not None or kind == "truncate"


@pytest.mark.parametrize("kind", ("header_only", "gt_in_seq", "lead_newline", "trail_header"))
def test_fasta_corruptions_gpu(gpu_ctx, oracle_lib, kind):
    for seed in range(3):
        rng = random.Random(seed * 10 + len(kind))
        data = gen.fasta_corrupt(rng, gen.fasta(rng, 1500), kind)
        _check(gpu_ctx, oracle_lib, data, "fasta")


def test_blank_runs_gpu(gpu_ctx, oracle_lib):
    """Long runs of blank lines straddling tiles (the FASTQ DONTCARE rule)."""
    rng = random.Random(5)
    base = gen.fastq(rng, 200)
    for tail in (b"\n" * 100000, b"\n" * 100000 + b"X", b"\n" * 70001 + b"@r\nA\n+\nI\n", b"\n" * 3 + b"Y\n"):
        _check(gpu_ctx, oracle_lib, base + tail, "fastq")
    _check(gpu_ctx, oracle_lib, b"\n" * 200000, "fastq")
    _check(gpu_ctx, oracle_lib, b"\n" * 200000, "line")


def test_huge_single_line_gpu(gpu_ctx, oracle_lib):
    rng = random.Random(9)
    one = gen._big_seq(rng, 3_000_000, b"ACGT")
    for d in (b">h\n" + one + b"\n", b"@h\n" + one + b"\n+\n" + one + b"\n", one, one + b"\n"):
        for mode in ("auto", "fasta", "fastq", "sam", "line"):
            _check(gpu_ctx, oracle_lib, d, mode)


def test_device_resident_api(gpu_ctx, oracle_lib):
    rng = random.Random(3)
    data = gen.fastq(rng, 20000)
    d = gpu_ctx.alloc(len(data) + 64)
    d.upload(data)
    rows = gpu_ctx.alloc(16 * (len(data) // 16 + 16))
    r = gpu_ctx.build_buffer(d, len(data), rows, kind="record", fmt="fastq")
    exp, err = oracle_lib.record_index(data, "fastq")
    assert r.ok and err is None and r.count == len(exp)
    assert np.array_equal(rows.rows(r.count), exp)
    # auto-detection on device-resident data
    r = gpu_ctx.build_buffer(d, len(data), rows, kind="record", fmt=None)
    assert r.ok and r.fmt == "fastq" and r.count == len(exp)
    # too-small table: reports the required count, writes nothing beyond capacity
    small = gpu_ctx.alloc(16 * 11)
    small.fill(0xFF)
    r2 = gpu_ctx.build_device(d.ptr, len(data), small.ptr, 10, kind="record", fmt="fastq")
    assert r2.status == -6 and r2.count == len(exp)  # SHOCKIDX_ESPACE
    got = small.download().view(np.uint64).reshape(11, 2)
    assert np.array_equal(got[:10], exp[:10]) and (got[10] == np.uint64(2 ** 64 - 1)).all()


def test_create_writes_idx(gpu_ctx, oracle_lib, tmp_path):
    from shock_amd import indexer
    indexer.PATH_DATA = str(tmp_path)
    rng = random.Random(4)
    data = gen.fastq(rng, 5000)
    f = tmp_path / "node.data"
    f.write_bytes(data)
    out = tmp_path / "record.idx"
    with open(f, "rb") as fh:
        count, fmt, err = indexer.Indexers["record"](fh, "basic", "", "").create(str(out))
    exp, _ = oracle_lib.record_index(data)
    assert err is None and fmt == "array" and count == len(exp)
    assert out.read_bytes() == exp.astype("<u8").tobytes()
    # error: nothing renamed into place, count = records before the error
    bad = gen.fastq_corrupt(rng, data, "len_mismatch")
    f.write_bytes(bad)
    out2 = tmp_path / "bad.idx"
    with open(f, "rb") as fh:
        count, fmt, err = indexer.Indexers["record"](fh, "basic", "", "").create(str(out2))
    exp2, e2 = oracle_lib.record_index(bad)
    assert err is not None and err.msg == e2 and count == len(exp2)
    assert not out2.exists()
    # line index
    out3 = tmp_path / "line.idx"
    with open(f, "rb") as fh:
        count, fmt, err = indexer.Indexers["line"](fh, "basic", "", "").create(str(out3))
    exp3, _ = oracle_lib.line_index(bad)
    assert err is None and out3.read_bytes() == exp3.astype("<u8").tobytes()


REGEX = json.load(open(os.path.join(GOLD, "regex_corpora.json")))["entries"]


@pytest.mark.parametrize("e", REGEX, ids=lambda e: e["id"])
def test_regex_corpora_gpu(gpu_ctx, oracle_lib, e):
    """k_detect on the reference's labelled regex corpora (fastq_test.go / fasta_test.go) as
    DetermineFormat sees them (zero-padded 32 KiB head): same match mask as the oracle, which
    tests/test_oracle_regex.py pins to the literal Go regexes and the labels."""
    s = bytes.fromhex(e["text_hex"])
    fmt, mask = gpu_ctx.detect(s)
    ofmt, omask = oracle_lib.detect(s)
    assert (fmt, mask) == (ofmt, omask)
    r = gpu_ctx.build_host(s, kind="record", fmt=None)
    rows, err = oracle_lib.record_index(s)
    assert r.err == err and r.count == len(rows)
    assert np.array_equal(r.rows if r.rows is not None else np.zeros((0, 2), np.uint64), rows)


def test_workspace_trim_gpu(oracle_lib, monkeypatch):
    """shockidx_ctx_trim frees the grow-only caches; builds after a trim, and
    under SHOCKIDX_WORKSPACE_CAP, stay correct."""
    import random as _r
    from shock_amd import Context
    import gen
    data = gen.fastq(_r.Random(4), 20000)
    exp, _ = oracle_lib.record_index(data, "fastq")
    with Context(0) as ctx:
        r = ctx.build_host(data)
        assert r.ok and np.array_equal(r.rows, exp)
        assert ctx.workspace_bytes() > len(data)
        ctx.trim(0)
        assert ctx.workspace_bytes() == 0
        r = ctx.build_host(data)
        assert r.ok and np.array_equal(r.rows, exp)
    monkeypatch.setenv("SHOCKIDX_WORKSPACE_CAP", str(1 << 20))
    with Context(0) as ctx:
        for _ in range(2):
            r = ctx.build_host(data)
            assert r.ok and np.array_equal(r.rows, exp)
            assert ctx.workspace_bytes() <= 1 << 20


def test_format_speculation_gpu(gpu_ctx, oracle_lib):
    """AUTO builds speculate the context's last detected format (one host round trip): a file of
    another format (FASTA after FASTQ, SAM, undetectable bytes) is gated off on the device and
    re-run with the detected format -- rows, count, format and Go's error text as without it."""
    rng = random.Random(21)
    fq = gen.fastq(rng, 9000)
    fa = gen.fasta(rng, 1200)
    sam = b"RG\tID:x\n" + gen.sam(rng, 9000)
    junk = b"xy" * (1 << 20)
    assert min(map(len, (fq, fa, sam, junk))) >= 1 << 20
    seq = [fq, fa, fq, sam, junk, fa, fa, junk, fq, fq]
    fmts = {id(fq): "fastq", id(fa): "fasta", id(sam): "sam", id(junk): None}
    prev = None
    for i, data in enumerate(seq):
        exp, err = oracle_lib.record_index(data)
        if i % 2:
            r = gpu_ctx.build_host(np.frombuffer(data, np.uint8), kind="record")
            got = r.rows
        else:
            d = gpu_ctx.alloc(len(data) + 64)
            d.upload(data)
            rows = gpu_ctx.alloc(16 * (len(data) // 16 + 16))
            r = gpu_ctx.build_buffer(d, len(data), rows, kind="record", fmt=None)
            got = rows.rows(r.count) if r.count else np.zeros((0, 2), np.uint64)
        assert r.count == len(exp), (i, r.count, len(exp), r.err, err)
        assert r.err == err, (i, r.err, err)
        # the format reported after a failed speculation is the detected one
        assert r.fmt == fmts[id(data)], (i, r.fmt, fmts[id(data)])
        # a speculation that failed re-ran the build (the previous detection was another format)
        if i and len(data) >= 1 << 20 and prev in ("fastq", "fasta") and fmts[id(data)] not in (prev, None):
            assert r.reruns >= 1, (i, r.reruns)
        prev = fmts[id(data)]  # the context speculates the last detected format (none after junk)
        if exp is not None and len(exp):
            assert np.array_equal(got[:len(exp)], exp), i
