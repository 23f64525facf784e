"""GPU parity of the subset path (index/subset.go:133-303; the subset node's bytes per
controller/node/single.go:500-517): shockidx_subset_index / shockidx_subset_gather through
the C ABI against the oracle.  Bar: identical rows, runs, oSize and Go error text; gathered
bytes equal to the concatenated runs of the parent file."""
import random

import numpy as np
import pytest

import gen
from test_oracle_subset import KATS, PARENT

pytestmark = pytest.mark.gpu


def _cmp(ctx, oracle_lib, ids, parent, ilength=None, data=None):
    rows, runs, size, err = oracle_lib.subset(ids, parent, ilength)
    r = ctx.subset_host(ids, parent, ilength, data=data)
    assert r.err == err, (ids[:80], r.err, err)
    assert r.count == len(rows)
    assert np.array_equal(r.rows, rows)
    if err is None:
        assert r.size == size and r.runs == len(runs)
        assert np.array_equal(r.run_rows, runs)
        if data is not None:
            exp = b"".join(bytes(data[int(o):int(o) + int(n)]) for o, n in runs)
            assert r.gathered == exp
    return r


@pytest.mark.parametrize("kat", KATS, ids=[repr(k[0])[:30] for k in KATS])
def test_subset_kat_gpu(gpu_ctx, oracle_lib, kat):
    _cmp(gpu_ctx, oracle_lib, kat[0], PARENT)


def test_subset_read_past_parent_gpu(gpu_ctx, oracle_lib):
    _cmp(gpu_ctx, oracle_lib, b"1\n8\n", PARENT, ilength=10)


def _sample(rng, n, frac):
    k = max(1, int(n * frac))
    return sorted(rng.sample(range(1, n + 1), k))


def test_subset_fastq_fuzz_gpu(gpu_ctx, oracle_lib):
    rng = random.Random(11)
    data = gen.fastq(rng, 20000)
    parent, err = oracle_lib.record_index(data, "fastq")
    assert err is None
    n = len(parent)
    for frac in (0.01, 0.2, 0.9, 1.0):
        ids = _sample(rng, n, frac)
        text = b"".join(b"%d\n" % i for i in ids)
        _cmp(gpu_ctx, oracle_lib, text, parent, data=data)
    # blank lines, sign, no final newline, CRLF, errors placed at random lines
    ids = _sample(rng, n, 0.3)
    lines = [b"%d" % i for i in ids]
    for variant in range(8):
        ls = list(lines)
        if variant == 1:
            ls = [x + (b"\n" if rng.random() < 0.2 else b"") for x in ls]
        if variant == 2:
            ls[rng.randrange(len(ls))] = b"abc"
        if variant == 3:
            j = rng.randrange(1, len(ls))
            ls[j] = ls[j - 1]
        if variant == 4:
            ls[rng.randrange(len(ls))] = b"%d" % (n + 5)
        if variant == 5:
            ls[rng.randrange(len(ls))] += b"\r"
        if variant == 6:
            ls = [b"+" + x for x in ls]
        if variant == 7:
            ls[rng.randrange(len(ls))] = b"1" * 25
        text = b"\n".join(ls) + (b"\n" if variant != 0 else b"")
        _cmp(gpu_ctx, oracle_lib, text, parent, data=data)


def test_subset_lines_and_zero_lengths_gpu(gpu_ctx, oracle_lib):
    # a line index parent (ends with a (size, 0) row) and tiny runs: the gather's byte path
    rng = random.Random(12)
    data = gen.lines(rng, 5000)
    parent, _ = oracle_lib.line_index(data)
    n = len(parent)
    for frac in (0.05, 0.5, 1.0):
        ids = _sample(rng, n, frac)
        _cmp(gpu_ctx, oracle_lib, b"".join(b"%d\n" % i for i in ids), parent, data=data)
    _cmp(gpu_ctx, oracle_lib, b"%d\n" % n, parent, data=data)  # only the empty final row


def test_subset_gather_large_gpu(gpu_ctx, oracle_lib):
    """Long contiguous runs (many 16 KiB output blocks) and runs shorter than 16 bytes."""
    rng = random.Random(13)
    data = bytes(rng.getrandbits(8) for _ in range(3_000_000))
    cuts = sorted(rng.sample(range(1, len(data)), 20000))
    offs = [0] + cuts
    parent = np.array([[offs[i], (offs[i + 1] if i + 1 < len(offs) else len(data)) - offs[i]]
                       for i in range(len(offs))], dtype=np.uint64)
    for frac in (0.02, 0.5, 0.97):
        ids = _sample(rng, len(parent), frac)
        _cmp(gpu_ctx, oracle_lib, b"".join(b"%d\n" % i for i in ids), parent, data=data)


def test_subset_create_files(gpu_ctx, oracle_lib, tmp_path):
    from shock_amd import indexer, subset
    indexer.PATH_DATA = str(tmp_path)
    idx = tmp_path / "record.idx"
    idx.write_bytes(PARENT.astype("<u8").tobytes())
    ids = tmp_path / "ids.txt"
    ids.write_bytes(b"1\n3\n4\n6\n")
    co, o = tmp_path / "n.subset.idx", tmp_path / "record_sub.idx"
    coc, oc, osz, err = subset.CreateSubsetNodeIndexes(str(ids), str(co), str(o), str(idx), "array", 6)
    assert err is None and (coc, oc, osz) == (3, 4, 31)
    assert o.read_bytes() == np.array([[0, 10], [30, 5], [35, 7], [43, 9]], dtype="<u8").tobytes()
    assert co.read_bytes() == np.array([[0, 10], [30, 12], [43, 9]], dtype="<u8").tobytes()
    ids.write_bytes(b"3\n1\n")
    co2 = tmp_path / "bad.subset.idx"
    coc, oc, osz, err = subset.CreateSubsetNodeIndexes(str(ids), str(co2), str(o) + "2", str(idx), "array", 6)
    assert err is not None and err.msg.startswith(b"Subset indices must be") and not co2.exists()
    coc, oc, osz, err = subset.CreateSubsetNodeIndexes(str(ids), str(co2), str(o) + "2", str(idx), "matrix", 6)
    assert err.msg == b"Subset node does not currently support the format of your parent index: matrix"
