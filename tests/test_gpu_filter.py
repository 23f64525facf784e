"""GPU: the download filters fq2fa / anonymize (node/filter/) on the device -- anonymize over
FASTQ, FASTA and SAM sections -- byte-exact against the oracle (oracle/filter_oracle.c; parity unpinned by reference-held vectors, see
tests/test_oracle_filter.py)."""
import os
import random

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "fixtures")

KATS = [
    b"@r1 x\nACGT\n+\nIIII\n@r2\nAC\n+r2\nII\n",
    b"@r1\nAC\n+\nII",
    b"@r1\nAC\n+\nII\n@r2\nA\n+\nI",
    b"@ \nAC\n+\nII\n",
    b"@r1\n \n+\nI\n",
    b"@r1\r\nAC\r\n+r1\r\nII\r\n",
    b"@r1\nAC\n+\nII\n\n\n",
    b"@r1\nAC\n+\nII\n\n@r2\nA\n+\nI\n",
    b"@r1\nAC\n+r2\nII\n",
    b"@r1\nAC\n+\nII\n@ \t\nAC\n+\nII\n",
    b"@r1\nAC\n+\nII\n@r2\n\xc2\xa0\n+\n\n",
    b"",
]


def _check(ctx, oracle_lib, data, name):
    r = ctx.filter_host(name, data)
    out, n, err = oracle_lib.filter_fastq(data, name)
    assert r.status in (0, 1), (r.status, r.err)
    assert (r.count, r.err) == (n, err), (r, n, err)
    assert r.gathered == out


@pytest.mark.parametrize("name", ["fq2fa", "anonymize"])
def test_filter_kats_gpu(gpu_ctx, oracle_lib, name):
    for d in KATS:  # anonymize detects the format first (multi.go:43-62): "" and "@ \n..." fail it
        _check(gpu_ctx, oracle_lib, d, name)


@pytest.mark.parametrize("seed", range(16))
def test_filter_random_gpu(gpu_ctx, oracle_lib, seed):
    rng = random.Random(100 + seed)
    data = gen.fastq(rng, rng.randint(1, 3000), crlf=0.3 if seed % 3 == 0 else 0.0, plus_id=0.3,
                     long_every=97 if seed % 4 == 3 else 0, final_nl=seed % 4 != 1,
                     uni=0.1 if seed % 5 == 2 else 0.0)
    if seed % 2:
        data = gen.fastq_corrupt(rng, data, rng.choice(gen.FASTQ_CORRUPTIONS))
    for name in ("fq2fa", "anonymize"):
        _check(gpu_ctx, oracle_lib, data, name)


def test_filter_fixture_gpu(gpu_ctx, oracle_lib):
    data = open(os.path.join(FIX, "sample1.fq"), "rb").read()
    for name in ("fq2fa", "anonymize"):
        _check(gpu_ctx, oracle_lib, data, name)


def test_filter_multigeneration_gpu(gpu_ctx, oracle_lib):
    """A 1 GiB section (hundreds of grid-stride passes of the record index) through both filters, byte-exact."""
    from shock_amd.synth import SynthFile
    size = 1 << 30
    sf = SynthFile(gpu_ctx, "fastq", size)
    data = sf.window(0, size)
    host = data.download(size).tobytes()
    for name in ("fq2fa", "anonymize"):
        cap = 2 * size
        d_out = gpu_ctx.alloc(cap)
        r = gpu_ctx.filter_device(name, data.ptr, size, d_out.ptr, cap)
        out, n, err = oracle_lib.filter_fastq(host, name)
        assert r.ok and err is None and r.count == n == sf.expected_count()
        assert r.size == len(out)
        got = d_out.download(r.size)
        assert np.array_equal(got, np.frombuffer(out, dtype=np.uint8))
        d_out.free()
    data.free()
    sf.free()


def test_filter_reader_mirror(gpu_ctx):
    """filter.NewReader: the bytes, then the reader's error (what io.Copy sees)."""
    from shock_amd.filter import Filter, Has, NewReader
    from shock_amd.indexer import ShockIndexError
    assert Has("fq2fa") and Has("anonymize") and not Has("gzip") and Filter("x") is None
    rd = NewReader("fq2fa", b"@r1\nAC\n+\nII\n@r2\nA\n+\nIX\n")
    assert rd.read(3) == b">r1" and rd.read() == b"\nAC\n"
    with pytest.raises(ShockIndexError, match="length of sequence and quality"):
        rd.read()
    assert Filter("anonymize")(b"@a\nA\n+\nI\n").read() == b"@1\nA\n+\nI\n"
    assert Filter("anonymize")(b">c1 x\nAC\nGT\n>c2\nA\n").read() == b">1\nACGT\n"


# ---- anonymize over FASTA and SAM sections (fasta.go:40-88, sam.go:44-81) --------------------
def test_anonymize_fasta_sam_kats_gpu(gpu_ctx, oracle_lib):
    from test_oracle_anonymize import FASTA_KATS, SAM_KATS
    for data, exp, err in FASTA_KATS + SAM_KATS:
        r = gpu_ctx.filter_host("anonymize", data)
        assert (r.gathered or b"", r.err) == (exp, err), data
        _check(gpu_ctx, oracle_lib, data, "anonymize")


def test_anonymize_fasta_sam_random_gpu(gpu_ctx, oracle_lib):
    from test_oracle_anonymize import _fasta_corpus, _sam_corpus
    rng = random.Random(12)
    for _ in range(150):
        _check(gpu_ctx, oracle_lib, _fasta_corpus(rng), "anonymize")
        d = _sam_corpus(rng)
        if oracle_lib.detect(d)[0] == "sam":
            _check(gpu_ctx, oracle_lib, d, "anonymize")


def test_anonymize_fasta_boundary_sources_gpu(gpu_ctx, oracle_lib, monkeypatch):
    """FASTA boundaries come from the record index when it builds without error, else from the
    unvalidated scan (forced here with SHOCKIDX_ANON_SCAN): both byte-exact on the same corpus,
    which holds sections whose index fails where Read goes on (a header ending in '>')."""
    from test_oracle_anonymize import _fasta_corpus
    rng = random.Random(77)
    corpus = [_fasta_corpus(rng) for _ in range(60)]
    corpus += [b">a>\nAC\n>b\nGT\n>c\nA\n", b">x\nAC\n>>\n>y\nG\n>z\nT\n",
               open(os.path.join(FIX, "nr_subset1.fa"), "rb").read()]
    for scan in (False, True):
        if scan:
            monkeypatch.setenv("SHOCKIDX_ANON_SCAN", "1")
        for d in corpus:
            _check(gpu_ctx, oracle_lib, d, "anonymize")


def test_anonymize_fasta_fixtures_gpu(gpu_ctx, oracle_lib):
    for f in ("10kb.fna", "40kb.fna", "nr_subset1.fa", "nr_subset2.fa"):
        _check(gpu_ctx, oracle_lib, open(os.path.join(FIX, f), "rb").read(), "anonymize")


def test_anonymize_fasta_large_gpu(gpu_ctx, oracle_lib):
    """A 1 GiB FASTA section (6 k tiles, most boundaries from the per-tile slots), plus one with
    short records (every tile re-read in the second pass), byte-exact."""
    from shock_amd.synth import SynthFile
    size = 1 << 30
    sf = SynthFile(gpu_ctx, "fasta", size)
    data = sf.window(0, size)
    host = data.download(size).tobytes()
    cap = size + (64 << 20)
    d_out = gpu_ctx.alloc(cap)
    r = gpu_ctx.filter_device("anonymize", data.ptr, size, d_out.ptr, cap)
    out, n, err = oracle_lib.filter_fastq(host, "anonymize")
    assert r.ok and err is None and r.count == n == sf.expected_count() - 1
    assert r.size == len(out)
    assert np.array_equal(d_out.download(r.size), np.frombuffer(out, dtype=np.uint8))
    for b in (d_out, data):
        b.free()
    sf.free()
    short = b"".join(b">s%d\nACGTACGTAC\nGG\n" % i for i in range(400000))
    _check(gpu_ctx, oracle_lib, short, "anonymize")


def test_anonymize_fasta_long_sequences_gpu(gpu_ctx, oracle_lib):
    """k_fa_anon_write's steps (several 1 KiB chunks each, the kept-byte counts of every chunk in
    one packed scan): bodies from empty to many steps long, with lines from 1 byte ('\\n'-dense
    chunks that keep little) to longer than a step (chunks that keep everything), each sequence at
    every 16-byte phase of the output."""
    rng = random.Random(31)
    parts = []
    for i in range(600):
        body = rng.choice([0, 1, 15, 16, 17, 1023, 1024, 1025, 4095, 4096, 4097, 9000, 20000,
                           rng.randint(0, 30000)])
        width = rng.choice([1, 2, 7, 60, 80, 1000, 5000, 1 << 20])
        seq = bytes(rng.choices(b"ACGT", k=body))
        lines = b"\n".join(seq[j:j + width] for j in range(0, len(seq), width))
        parts.append(b">s" + b"x" * (i % 16) + b"\n" + lines + b"\n")
    _check(gpu_ctx, oracle_lib, b"".join(parts), "anonymize")


def test_anonymize_fasta_tiny_records_gpu(gpu_ctx, oracle_lib):
    """1.2 M minimal sequences (">a\\nA\\n", 5 bytes): with 7-digit counters the anonymized
    section is 2.2 x its input, past filter_host's first output guess -- the call reports the
    bytes it needs (SHOCKIDX_ESPACE) and the mirror retries with that size."""
    data = b">a\nA\n" * 1_200_000
    r = gpu_ctx.filter_host("anonymize", data)
    out, n, err = oracle_lib.filter_fastq(data, "anonymize")
    assert len(out) > 2 * len(data) + 64
    assert r.status == 0 and (r.count, r.err) == (n, err), (r, n, err)
    assert r.gathered == out
