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


def _node(ctx, ids, parent, ilength=None, data=b"", rows_cap=None, runs_cap=None, out_cap=None, pad=0):
    """shockidx_subset_node (index + gather in one call) on device copies of the inputs; `pad`
    rows of 0xAB sentinel past each table (an overflow would overwrite them)."""
    par = np.ascontiguousarray(parent, dtype=np.uint64).reshape(-1, 2)
    n = par.shape[0]
    d_ids = ctx.alloc(len(ids) + 64)
    d_ids.upload(ids)
    d_par = ctx.alloc(16 * n + 64)
    d_par.upload(par.tobytes())
    cap = max(1, len(ids) // 2 + 2)
    rows_cap = cap if rows_cap is None else rows_cap
    runs_cap = cap if runs_cap is None else runs_cap
    d_rows, d_runs = ctx.alloc(16 * (rows_cap + pad) + 16), ctx.alloc(16 * (runs_cap + pad) + 16)
    d_rows.fill(0xAB)
    d_runs.fill(0xAB)
    d_data = ctx.alloc(len(data) + 64)
    d_data.upload(data)
    out_cap = len(data) + 64 if out_cap is None else out_cap
    d_out = ctx.alloc(out_cap + 16 * pad + 64)
    d_out.fill(0xAB)
    r = ctx.subset_node(d_ids.ptr, len(ids), d_par.ptr, n, n if ilength is None else ilength, d_rows.ptr, rows_cap,
                        d_runs.ptr, runs_cap, d_data.ptr, len(data), d_out.ptr, out_cap)
    return r, d_rows, d_runs, d_out


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
    # the same through the one-call node build (index + gather, counts kept on the device)
    if data is None:  # a parent file for the gather: zeros covering every parent row
        par = np.asarray(parent, dtype=np.uint64).reshape(-1, 2)
        data = bytes(int((par[:, 0] + par[:, 1]).max()) if len(par) else 0)
        exp = b"".join(bytes(data[int(o):int(o) + int(n)]) for o, n in runs) if err is None else b""
    nd, d_rows, d_runs, d_out = _node(ctx, ids, parent, ilength, bytes(data))
    assert nd.err == err and nd.count == len(rows)
    assert np.array_equal(d_rows.rows(nd.count) if nd.count else np.zeros((0, 2), np.uint64), rows)
    if err is None:
        assert nd.size == size and nd.runs == len(runs)
        assert np.array_equal(d_runs.rows(nd.runs) if nd.runs else np.zeros((0, 2), np.uint64), runs)
        assert d_out.download(size).tobytes() == exp
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
    """Long contiguous runs (many 32 KiB output blocks) and runs shorter than 16 bytes."""
    rng = random.Random(13)
    data = bytes(rng.getrandbits(8) for _ in range(3_000_000))
    cuts = sorted(rng.sample(range(1, len(data)), 20000))
    offs = [0] + cuts
    parent = np.array([[offs[i], (offs[i + 1] if i + 1 < len(offs) else len(data)) - offs[i]]
                       for i in range(len(offs))], dtype=np.uint64)
    for frac in (0.02, 0.5, 0.97):
        ids = _sample(rng, len(parent), frac)
        _cmp(gpu_ctx, oracle_lib, b"".join(b"%d\n" % i for i in ids), parent, data=data)


@pytest.mark.parametrize("maxlen", [3, 40, 700])
def test_gather_host_runs_gpu(gpu_ctx, maxlen):
    """The standalone gather of host-given runs, in any order: runs of 1..maxlen bytes (with 3 and
    40, far more runs per output block than the workgroup stages), every one of them
    unaligned, runs that end at the file's last byte (the file's length not a multiple of 16)."""
    rng = np.random.default_rng(maxlen)
    n = 1_000_003
    data = rng.integers(0, 256, n, dtype=np.uint8)
    k = n // maxlen  # the gather refuses more bytes than the parent holds (subset.go: a subset of it)
    lens = rng.integers(1, maxlen + 1, k).astype(np.uint64)
    offs = (rng.integers(0, n, k).astype(np.uint64) % (n - lens + 1)).astype(np.uint64)
    offs[::97] = n - lens[::97]  # the file's end
    runs = np.stack([offs, lens], axis=1).astype(np.uint64)
    size = int(lens.sum())
    exp = np.concatenate([data[int(o):int(o) + int(m)] for o, m in runs])
    d_data = gpu_ctx.alloc(n + 64)
    d_data.upload(data)
    d_runs = gpu_ctx.alloc(16 * k + 16)
    d_runs.upload(runs.tobytes())
    d_o = gpu_ctx.alloc(size + 64)
    g = gpu_ctx.subset_gather(d_data.ptr, n, d_runs.ptr, k, d_o.ptr, size)
    assert g.ok and g.size == size and g.runs == k
    assert np.array_equal(d_o.download(size), exp)


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


def test_subset_capacities_gpu(gpu_ctx, oracle_lib):
    """Short row / run / output capacities: the counts needed come back (ESPACE, like every
    capacity error of the C ABI) and nothing is written past any capacity (sentinels intact)."""
    rng = random.Random(14)
    data = gen.fastq(rng, 3000)
    parent, _ = oracle_lib.record_index(data, "fastq")
    ids = _sample(rng, len(parent), 0.3)
    text = b"".join(b"%d\n" % i for i in ids)
    rows, runs, size, err = oracle_lib.subset(text, parent, None)
    assert err is None and len(runs) > 20
    pad = 64
    r, d_rows, _, _ = _node(gpu_ctx, text, parent, data=data, rows_cap=10, pad=pad)
    assert r.status == -6 and r.count == len(rows)
    assert np.all(d_rows.download(16 * pad, 16 * 10) == 0xAB)
    r, _, d_runs, _ = _node(gpu_ctx, text, parent, data=data, runs_cap=5, pad=pad)
    assert r.status == -6 and r.count == len(rows) and r.runs == len(runs)
    assert np.all(d_runs.download(16 * pad, 16 * 5) == 0xAB)
    r, _, _, d_out = _node(gpu_ctx, text, parent, data=data, out_cap=size - 1, pad=pad)
    assert r.status == -6 and r.size == size
    assert np.all(d_out.download(size + 16 * pad) == 0xAB)  # nothing gathered
    r, _, _, d_out = _node(gpu_ctx, text, parent, data=data, out_cap=size)
    assert r.ok and r.size == size and r.runs == len(runs)
    # the standalone gather with a short output buffer
    d_data = gpu_ctx.alloc(len(data) + 64)
    d_data.upload(data)
    d_runs = gpu_ctx.alloc(16 * len(runs) + 16)
    d_runs.upload(np.ascontiguousarray(runs, dtype=np.uint64).tobytes())
    d_o = gpu_ctx.alloc(size + 64)
    g = gpu_ctx.subset_gather(d_data.ptr, len(data), d_runs.ptr, len(runs), d_o.ptr, size - 1)
    assert g.status == -6 and g.size == size
    g = gpu_ctx.subset_gather(d_data.ptr, len(data), d_runs.ptr, len(runs), d_o.ptr, size)
    assert g.ok and g.size == size
    assert d_o.download(size).tobytes() == b"".join(bytes(data[int(o):int(o) + int(n)]) for o, n in runs)
