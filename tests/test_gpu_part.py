"""GPU: the index read path (Idx.Part / Idx.Range, index/index.go:67-193) and
CreateSubsetIndex (index/subset.go:36-128) served from HBM, bit-exact against the oracle
(oracle/part_oracle.c; parity unpinned by reference-held vectors, see tests/test_oracle_part.py).
"""
import os
import random

import numpy as np
import pytest

from test_oracle_part import ROWS, _random_part, _random_rows

pytestmark = pytest.mark.gpu
GIB = 1 << 30


def _dev_rows(ctx, rows):
    rows = np.ascontiguousarray(rows, dtype=np.uint64).reshape(-1, 2)
    buf = ctx.alloc(16 * rows.shape[0] + 64)
    if rows.size:
        buf.upload(rows.tobytes())
    return buf, rows.shape[0]


def _check_table(ctx, oracle_lib, rows, parts, idx_length):
    buf, n = _dev_rows(ctx, rows)
    try:
        for part in parts:
            assert ctx.idx_part(buf.ptr, n, part, idx_length) == oracle_lib.idx_part(rows, part, idx_length), part
            recs, err = ctx.idx_range(buf.ptr, n, part, idx_length)
            erecs, eerr = oracle_lib.idx_range(rows, part, idx_length)
            assert err == eerr, part
            assert np.array_equal(recs, erecs), part
    finally:
        buf.free()


def test_part_range_kats_gpu(gpu_ctx, oracle_lib):
    parts = ["1", "6", "2-3", "1-6", "3-2", "6-1", "0", "7", "x", "+2", "0-2", "1-7", "-2", "2-", "2-3-9",
             "1-1", "1-3", "3-4", "4-5", "5-4"]
    _check_table(gpu_ctx, oracle_lib, ROWS, parts, 6)
    _check_table(gpu_ctx, oracle_lib, ROWS[:3], ["5", "2-5", "2-6", "5-6", "1-3"], 6)  # short file


def test_missing_file_gpu(gpu_ctx):
    assert gpu_ctx.idx_part(None, 0, "1", 5) == (0, 0, b"Index file is missing")
    recs, err = gpu_ctx.idx_range(None, 0, "1-2", 5)
    assert err == b"Index file is missing" and recs.shape == (0, 2)


def test_random_tables_gpu(gpu_ctx, oracle_lib):
    rng = random.Random(7)
    for _ in range(30):
        n = rng.randrange(1, 3000)
        rows = _random_rows(rng, n)
        il = n if rng.random() < 0.8 else n + rng.randrange(1, 5)
        _check_table(gpu_ctx, oracle_lib, rows, [_random_part(rng, il) for _ in range(8)] + [f"1-{il}"], il)


def test_create_subset_index_gpu(gpu_ctx, oracle_lib):
    rng = np.random.default_rng(11)
    parent = _random_rows(random.Random(3), 5000)
    d_par, n = _dev_rows(gpu_ctx, parent)
    cases = []
    ids = np.sort(rng.choice(n, size=700, replace=False) + 1)
    cases.append(("\n".join(map(str, ids.tolist())) + "\n").encode())
    cases.append(b"1\n2\n\n5\n")
    cases.append(b"2\n1\n")
    cases.append(b"4\n5001\n")
    cases.append(b"1\n+3\nx7\n")
    cases.append(b"")
    cases.append(b"9")  # last line without '\n' is dropped (ReadLine EOF)
    try:
        for text in cases:
            d_ids = gpu_ctx.alloc(len(text) + 64)
            d_ids.upload(text)
            cap = len(text) // 2 + 2
            d_rows = gpu_ctx.alloc(16 * cap)
            r = gpu_ctx.create_subset_index(d_ids.ptr, len(text), d_par.ptr, n, n, d_rows.ptr, cap)
            erows, ecount, esize, eerr = oracle_lib.create_subset_index(text, parent, n)
            if eerr is None:
                assert r.ok and (r.count, r.size) == (ecount, esize)
                got = d_rows.rows(r.count) if r.count else np.zeros((0, 2), np.uint64)
                assert np.array_equal(got, erows)
            else:
                assert not r.ok and r.err == eerr
                assert (r.count, r.size) == ((1 << 64) - 1, (1 << 64) - 1)  # Go's (-1, -1)
            d_ids.free()
            d_rows.free()
    finally:
        d_par.free()


def test_idx_class_files(gpu_ctx, oracle_lib, tmp_path):
    """The host mirror: Idx().Part / .Range on an .idx file (loaded into HBM once, reloaded
    when the file changes), and shock_amd.subset.CreateSubsetIndex writing one."""
    from shock_amd.core import write_idx
    from shock_amd.index import New
    from shock_amd.subset import CreateSubsetIndex
    p = str(tmp_path / "record.idx")
    write_idx(ROWS, str(tmp_path), p)
    idx = New()
    assert idx.Type() == "file" and idx.GetLength() == 0
    pos, length, err = idx.Part("2-3", p, 6)
    assert (pos, length, err) == (10, 12, None)
    recs, err = idx.Range("1-6", p, 6)
    assert err is None and recs.tolist() == [[0, 22], [40, 5], [100, 1]]
    _, _, err = idx.Part("9", p, 6)
    assert str(err) == "Index record out of bounds"
    _, err = idx.Range("1", str(tmp_path / "missing.idx"), 6)
    assert str(err) == "Index file is missing"
    rows2 = ROWS.copy()
    rows2[1, 0] = 11  # breaks the first run
    write_idx(rows2, str(tmp_path), p)
    recs, err = idx.Range("1-3", p, 6)
    assert recs.tolist() == oracle_lib.idx_range(rows2, "1-3", 6)[0].tolist()
    ids = tmp_path / "ids.txt"
    ids.write_bytes(b"1\n2\n\n5\n")
    out = str(tmp_path / "sub.idx")
    assert CreateSubsetIndex(str(ids), out, p, "array", 6) == (3, 10 + 5 + 2, None)
    assert np.fromfile(out, dtype="<u8").reshape(-1, 2).tolist() == [[0, 10], [11, 5], [43, 2]]
    ids.write_bytes(b"3\n2\n")
    c, s, err = CreateSubsetIndex(str(ids), str(tmp_path / "bad.idx"), p, "array", 6)
    assert (c, s) == (-1, -1) and not os.path.exists(tmp_path / "bad.idx")
    assert CreateSubsetIndex(str(ids), out, p, "matrix", 6)[:2] == (-1, -1)


def test_range_10gib_node(gpu_ctx, oracle_lib):
    """A part=N-M request on a 10 GiB FASTQ node (configs[1]), served from the record index the
    device just built, and the full-file Range a subset download does (single.go:388-399)."""
    from shock_amd.synth import SynthFile
    size = 10 * GIB
    sf = SynthFile(gpu_ctx, "fastq", size)
    data = sf.window(0, size)
    R = sf.expected_count()
    rows = gpu_ctx.alloc(16 * (R + 1024))
    r = gpu_ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
    assert r.ok and r.count == R
    data.free()
    sf.free()
    tab = rows.rows(R)
    rng = random.Random(99)
    parts = [f"1-{R}", "1", str(R), f"{R // 3}-{R // 2}", f"{R}-1", f"{R + 1}", f"1-{R + 1}"]
    parts += [f"{a}-{a + rng.randrange(0, 100000)}" for a in (rng.randrange(1, R - 100000) for _ in range(4))]
    for part in parts:
        assert gpu_ctx.idx_part(rows.ptr, R, part, R) == oracle_lib.idx_part(tab, part, R), part
        recs, err = gpu_ctx.idx_range(rows.ptr, R, part, R)
        erecs, eerr = oracle_lib.idx_range(tab, part, R)
        assert err == eerr and np.array_equal(recs, erecs), part
    # the whole node is one contiguous run (up to the generator's trailing '\n' padding)
    recs, _ = gpu_ctx.idx_range(rows.ptr, R, f"1-{R}", R)
    assert recs.tolist() == [[0, int(tab[-1, 0] + tab[-1, 1])]]
    # a 1 % subset index of it: Range over the subset rows coalesces like the .subset.idx runs
    ids = np.sort(np.random.default_rng(5).choice(R, size=R // 100, replace=False) + 1)
    sub = np.ascontiguousarray(tab[ids - 1])
    d_sub, k = _dev_rows(gpu_ctx, sub)
    recs, err = gpu_ctx.idx_range(d_sub.ptr, k, f"1-{k}", k)
    erecs, _ = oracle_lib.idx_range(sub, f"1-{k}", k)
    assert err is None and np.array_equal(recs, erecs)
    text = ("\n".join(map(str, ids.tolist())) + "\n").encode()
    _, runs, _, _ = oracle_lib.subset(text, tab, R)
    assert np.array_equal(recs.view(np.uint64), runs)
    d_sub.free()
    rows.free()
