"""GPU: the download filters fq2fa / anonymize (node/filter/) on the device, byte-exact against
the oracle (oracle/filter_oracle.c; parity unpinned by reference-held vectors, see
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
        if name == "anonymize" and oracle_lib.detect(data)[0] not in ("fastq", None):
            continue  # FASTA / SAM sections are not filtered on the device
        _check(gpu_ctx, oracle_lib, data, name)


def test_filter_fixture_gpu(gpu_ctx, oracle_lib):
    data = open(os.path.join(FIX, "sample1.fq"), "rb").read()
    for name in ("fq2fa", "anonymize"):
        _check(gpu_ctx, oracle_lib, data, name)


def test_filter_multigeneration_gpu(gpu_ctx, oracle_lib):
    """A 1 GiB section (hundreds of k_pipe generations) through both filters, byte-exact."""
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
    r = gpu_ctx.filter_host("anonymize", b">c1\nACGT\n")  # FASTA sections stay on the host path
    assert r.status == -1  # SHOCKIDX_EINVAL
