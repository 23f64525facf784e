"""GPU parity at the sizes the hot path runs at (BASELINE.json configs[0..4]).

* The tile passes (k_fq_tiles, k_fa_tiles, k_line_tiles) walk the tiles grid-stride: tile
  t, t + G, ... with G = the persistent grid (CUs x co-resident workgroups).  Their provisional
  rows, the device-wide scan (k_scan_excl: several look-back blocks), the placement kernels and
  the fix-up queues only meet every case when a build spans many passes of G tiles: these
  FASTQ and FASTA inputs span >= 16 of them and are compared bit for bit (rows, count, Go
  error text) with the C oracle, clean and with errors injected in the first, a middle and
  the last pass, in CRLF form and with long blank-line tails.  Inputs >= 64 MiB also cross
  the 64 MiB pinned-staging chunks of shockidx_build_host.
* configs[1] / configs[2]: 10 GiB FASTQ and FASTA at full size, every row checked on the device
  against the synthetic generator (which knows each record's offset and length).
* configs[3]: a 50 GiB FASTQ node, its device-resident index, a random 1 % subset node (rows,
  coalesced runs, bytes) checked against the parent table.
* configs[0]: 64 MiB and 200 MiB FASTQ files through shockidx_create(fd) -> record.idx, byte
  identical to the oracle's table.
* configs[4]: the 80 GiB node whole and as 8 slabs through the slab protocol on one device.
* Two contexts building different files on one GPU from two threads at once.
"""
import ctypes
import os
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GIB = 1 << 30
MIB = 1 << 20
TILE = 16384


def _tiles_grid(ctx):
    lib = ctx._lib
    lib.shockidx_debug_tiles_grid.argtypes = [ctypes.c_void_p]
    lib.shockidx_debug_tiles_grid.restype = ctypes.c_int
    return lib.shockidx_debug_tiles_grid(ctx._h)


def _check(r, exp, err):
    assert r.err == err, (r.err, err)
    assert r.count == len(exp), (r.count, len(exp))
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    if not np.array_equal(got, exp):
        bad = np.nonzero((got != exp).any(axis=1))[0][:5]
        raise AssertionError(f"rows differ at {bad.tolist()}: gpu {got[bad].tolist()} oracle {exp[bad].tolist()}")


@pytest.fixture(scope="module")
def big_fastq(gpu_ctx):
    """A synthetic FASTQ (configs[1] generator) spanning >= 16 grid-stride passes, on the host."""
    from shock_amd.synth import SynthFile
    G = _tiles_grid(gpu_ctx)
    assert G > 0
    size = max(256 * MIB, (16 * G + 5) * TILE + 12345)
    sf = SynthFile(gpu_ctx, "fastq", size)
    buf = sf.window(0, size)
    host = buf.download(size)
    buf.free()
    sf.free()
    return host, G


def crlf(host: np.ndarray) -> np.ndarray:
    """every '\\n' of host becomes "\\r\\n" (byte i moves right by the newlines before it)"""
    isnl = host == 10
    pos = np.arange(host.size, dtype=np.int64)
    pos[1:] += np.cumsum(isnl[:-1])
    out = np.empty(host.size + int(isnl.sum()), np.uint8)
    out[pos + isnl] = host
    out[pos[isnl]] = 13
    return out


def _gen_bounds(G, k, n):
    lo = k * G * TILE
    return lo, min(n, lo + G * TILE)


def test_fastq_generations_clean(gpu_ctx, oracle_lib, big_fastq):
    host, G = big_fastq
    ntiles = (host.size + TILE - 1) // TILE
    assert ntiles // G >= 16, (ntiles, G)
    exp, err = oracle_lib.record_index(host, "fastq")
    assert err is None
    d = gpu_ctx.alloc(host.size + 64)
    d.upload(host)
    rows = gpu_ctx.alloc(16 * (len(exp) + 64))
    r = gpu_ctx.build_buffer(d, host.size, rows, kind="record", fmt=None)
    assert r.ok and r.fmt == "fastq" and r.count == len(exp), r
    assert np.array_equal(rows.rows(r.count), exp)
    # repeated builds on the same context (epoch tags, alternating first-bad slots)
    for _ in range(3):
        r = gpu_ctx.build_buffer(d, host.size, rows, kind="record", fmt="fastq")
        assert r.ok and r.count == len(exp)
    assert np.array_equal(rows.rows(r.count), exp)
    d.free()
    rows.free()


def _record_in(exp, lo, hi, frac=0.5):
    """index of a record starting inside [lo, hi), near lo + frac*(hi-lo)"""
    target = lo + int(frac * (hi - lo))
    k = int(np.searchsorted(exp[:, 0], target))
    k = min(max(k, 0), len(exp) - 2)
    assert lo <= int(exp[k, 0]) < hi
    return k


def _lines(host, off):
    """(start, end) of the 4 lines of the record at byte offset off (end = index of '\\n')"""
    out, p = [], off
    for _ in range(4):
        e = int(np.argmax(host[p:p + (1 << 20)] == 10)) + p
        out.append((p, e))
        p = e + 1
    return out


def _corrupt(host, exp, k, kind):
    h = host.copy()
    (i0, i1), (s0, s1), (p0, p1), (q0, q1) = _lines(h, int(exp[k, 0]))
    if kind == "noplus":
        h[p0] = ord("-")
    elif kind == "noat":
        h[i0] = ord("X")
    elif kind == "lenmismatch":  # trailing space in the sequence line: TrimSpace shortens it
        h[s1 - 1] = ord(" ")
    elif kind == "emptyseq":     # "\n\n" in place of the sequence line: shifts the line phase
        h = np.concatenate([h[:s0], np.frombuffer(b"\n", np.uint8), h[s1 + 1:]])
    elif kind == "blank":        # a blank line between records
        h = np.concatenate([h[:i0], np.frombuffer(b"\n", np.uint8), h[i0:]])
    else:
        raise ValueError(kind)
    return h


@pytest.mark.parametrize("where", ["first", "middle", "last", "boundary", "two"])
def test_fastq_generation_errors(gpu_ctx, oracle_lib, big_fastq, where):
    host, G = big_fastq
    exp0, _ = oracle_lib.record_index(host, "fastq")
    ntiles = (host.size + TILE - 1) // TILE
    ngen = (ntiles + G - 1) // G
    if where == "first":
        lo, hi = _gen_bounds(G, 0, host.size)
        h = _corrupt(host, exp0, _record_in(exp0, lo, hi, 0.7), "noplus")
    elif where == "middle":
        lo, hi = _gen_bounds(G, ngen // 2, host.size)
        h = _corrupt(host, exp0, _record_in(exp0, lo, hi, 0.3), "lenmismatch")
    elif where == "last":
        lo, hi = _gen_bounds(G, ngen - 1, host.size)
        h = _corrupt(host, exp0, _record_in(exp0, lo, int(exp0[-1, 0]) + 1, 0.6), "blank")
    elif where == "boundary":  # the record straddling the first generation boundary
        b = G * TILE
        k = int(np.searchsorted(exp0[:, 0], b)) - 1
        assert int(exp0[k, 0]) < b <= int(exp0[k, 0] + exp0[k, 1])
        h = _corrupt(host, exp0, k, "noat")
    else:  # errors in a middle and the last generation: the earlier one is reported
        lo, hi = _gen_bounds(G, ngen - 1, host.size)
        h = _corrupt(host, exp0, _record_in(exp0, lo, int(exp0[-1, 0]) + 1, 0.2), "noat")
        lo, hi = _gen_bounds(G, ngen - 2, host.size)
        h = _corrupt(h, exp0, _record_in(exp0, lo, hi, 0.5), "emptyseq")
    exp, err = oracle_lib.record_index(h, "fastq")
    assert err is not None
    r = gpu_ctx.build_host(h, kind="record", fmt=None)  # > 64 MiB: several pinned stages
    _check(r, exp, err)


def test_fastq_generations_crlf(gpu_ctx, oracle_lib, big_fastq):
    host, G = big_fastq
    exp0, _ = oracle_lib.record_index(host, "fastq")
    cut = int(exp0[-1, 0] + exp0[-1, 1])  # records in CRLF form, the '\n' padding kept as is
    out = np.concatenate([crlf(host[:cut]), host[cut:]])
    assert out.size > 256 * MIB
    exp, err = oracle_lib.record_index(out, "fastq")
    assert err is None and len(exp) > 1000
    r = gpu_ctx.build_host(out, kind="record", fmt=None)
    assert r.fmt == "fastq"
    _check(r, exp, err)


@pytest.mark.parametrize("tail", [b"\n" * 200000, b"\n" * 100001 + b"@x\nA\n+\nI\n", b"\n" * 70000 + b"Z",
                                  b"\r\n" * 40000], ids=["blank200k", "blank_then_record", "blank_then_byte", "crlf_lines"])
def test_fastq_generations_blank_tail(gpu_ctx, oracle_lib, big_fastq, tail):
    host, _ = big_fastq
    h = np.concatenate([host, np.frombuffer(tail, np.uint8)])
    exp, err = oracle_lib.record_index(h, "fastq")
    r = gpu_ctx.build_host(h, kind="record", fmt="fastq")
    _check(r, exp, err)


def test_line_index_generations(gpu_ctx, oracle_lib, big_fastq):
    host, _ = big_fastq
    exp, _ = oracle_lib.line_index(host)
    r = gpu_ctx.build_host(host, kind="line")
    _check(r, exp, None)


# ---- FASTA tile pass (k_fa_tiles / k_fa_place / k_fa_fixup) over >= 16 grid-stride passes -----------
@pytest.fixture(scope="module")
def big_fasta(gpu_ctx):
    """A synthetic FASTA (configs[2] generator: wrapped sequences, 1 % headers holding '>')
    spanning >= 16 grid-stride passes of k_fa_tiles, on the host."""
    from shock_amd.synth import SynthFile
    G = _tiles_grid(gpu_ctx)
    assert G > 0
    size = max(256 * MIB, (16 * G + 5) * TILE + 12345)
    sf = SynthFile(gpu_ctx, "fasta", size)
    buf = sf.window(0, size)
    host = buf.download(size)
    buf.free()
    sf.free()
    return host, G


def _fa_record(host, exp, k):
    """(start, header '\n', next record start) of FASTA record k"""
    st = int(exp[k, 0])
    e = int(np.argmax(host[st:st + (1 << 20)] == 10)) + st
    return st, e, st + int(exp[k, 1])


def _fa_corrupt(host, exp, k, kind):
    st, he, nx = _fa_record(host, exp, k)
    if kind == "hdronly":      # header without sequence: the piece "ctg.. len=..\n" trims to one line
        return np.concatenate([host[:he + 1], host[nx:]])
    if kind == "blankhdr":     # a record of whitespace only: ">   \n", TrimSpace leaves nothing
        return np.concatenate([host[:st], np.frombuffer(b">   \n", np.uint8), host[nx:]])
    if kind == "gtseq":        # '>' inside a sequence line: a '\n' came before it, so a boundary
        h = host.copy()
        h[he + 7] = ord(">")
        return h
    if kind == "crhdr":        # header ending "\r\n" then its sequence: valid, the CR is trimmed
        return np.concatenate([host[:he], np.frombuffer(b"\r", np.uint8), host[he:]])
    raise ValueError(kind)


def test_fasta_passes_clean(gpu_ctx, oracle_lib, big_fasta):
    host, G = big_fasta
    ntiles = (host.size + TILE - 1) // TILE
    assert ntiles // G >= 16, (ntiles, G)
    exp, err = oracle_lib.record_index(host, "fasta")
    assert err is None
    r = gpu_ctx.build_host(host, kind="record", fmt=None)
    assert r.fmt == "fasta"
    _check(r, exp, err)


@pytest.mark.parametrize("where", ["first", "middle", "last", "boundary", "two", "gtseq", "leadnl"])
def test_fasta_pass_errors(gpu_ctx, oracle_lib, big_fasta, where):
    """An invalid piece (fasta.go:111-121) in the first, a middle and the last grid-stride pass,
    across a pass boundary, two of them (the earlier one is reported), a '>' inside a sequence
    line (more records, no error) and a file that starts with a blank line (an empty record 0)."""
    host, G = big_fasta
    exp0, _ = oracle_lib.record_index(host, "fasta")
    ntiles = (host.size + TILE - 1) // TILE
    npass = (ntiles + G - 1) // G
    if where == "first":
        lo, hi = _gen_bounds(G, 0, host.size)
        h = _fa_corrupt(host, exp0, _record_in(exp0, lo, hi, 0.6), "hdronly")
    elif where == "middle":
        lo, hi = _gen_bounds(G, npass // 2, host.size)
        h = _fa_corrupt(host, exp0, _record_in(exp0, lo, hi, 0.4), "blankhdr")
    elif where == "last":
        lo, hi = _gen_bounds(G, npass - 1, host.size)
        h = _fa_corrupt(host, exp0, _record_in(exp0, lo, int(exp0[-2, 0]) + 1, 0.5), "hdronly")
    elif where == "boundary":  # the record straddling the first pass boundary
        b = G * TILE
        k = int(np.searchsorted(exp0[:, 0], b)) - 1
        assert int(exp0[k, 0]) < b <= int(exp0[k, 0] + exp0[k, 1])
        h = _fa_corrupt(host, exp0, k, "hdronly")
    elif where == "two":
        lo, hi = _gen_bounds(G, npass - 1, host.size)
        h = _fa_corrupt(host, exp0, _record_in(exp0, lo, int(exp0[-2, 0]) + 1, 0.3), "blankhdr")
        lo, hi = _gen_bounds(G, npass - 2, host.size)
        h = _fa_corrupt(h, exp0, _record_in(exp0, lo, hi, 0.5), "hdronly")
    elif where == "gtseq":
        h = host
        for q in range(0, npass, max(1, npass // 5)):
            lo, hi = _gen_bounds(G, q, host.size)
            h = _fa_corrupt(h, exp0, _record_in(exp0, lo, hi, 0.5), "gtseq")
    else:  # a leading '\n': the file no longer starts with '>'
        h = np.concatenate([np.frombuffer(b"\n", np.uint8), host])
    exp, err = oracle_lib.record_index(h, "fasta")
    if where == "gtseq":
        assert err is None and len(exp) > len(exp0)
    else:  # leadnl: record 0 is the piece "\n" before the first '>', which trims to nothing
        assert err is not None and err.startswith(b"Invalid fasta entry")
    r = gpu_ctx.build_host(h, kind="record", fmt="fasta")
    _check(r, exp, err)


def test_fasta_passes_crlf(gpu_ctx, oracle_lib, big_fasta):
    host, _ = big_fasta
    out = crlf(host)
    exp, err = oracle_lib.record_index(out, "fasta")
    assert err is None and len(exp) > 1000
    r = gpu_ctx.build_host(out, kind="record", fmt=None)
    assert r.fmt == "fasta"
    _check(r, exp, err)


@pytest.mark.parametrize("tail", [b"\n" * 200000, b"\n" * 100001 + b">x\nACGT\n", b"\r\n" * 40000 + b">y\n"],
                         ids=["blank200k", "blank_then_record", "crlf_then_header_only"])
def test_fasta_passes_blank_tail(gpu_ctx, oracle_lib, big_fasta, tail):
    host, _ = big_fasta
    h = np.concatenate([host, np.frombuffer(tail, np.uint8)])
    exp, err = oracle_lib.record_index(h, "fasta")
    r = gpu_ctx.build_host(h, kind="record", fmt="fasta")
    _check(r, exp, err)


# ---- configs[1] / configs[2] at full size ---------------------------------------------------
@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_full_size_10gib(gpu_ctx, oracle_lib, fmt):
    """configs[1] / configs[2]: the whole 10 GiB table against the generator AND against the C
    oracle run over the same 10 GiB (rows, count, SHA-256 of the .idx bytes)."""
    import hashlib
    from shock_amd.synth import SynthFile
    size = 10 * GIB
    sf = SynthFile(gpu_ctx, fmt, size)
    data = sf.window(0, size)
    R = sf.expected_count()
    rows = gpu_ctx.alloc(16 * (R + 1024))
    r = gpu_ctx.build_buffer(data, size, rows, kind="record", fmt=None)
    assert r.ok and r.fmt == fmt and r.count == R, r
    if fmt == "fastq":
        assert sf.check_rows(rows, 0, R) == 0
    else:  # the '\n' padding belongs to the last FASTA record (fasta.go EOF piece)
        assert sf.check_rows(rows, 0, R - 1) == 0
        last = rows.download(16, 16 * (R - 1)).view(np.uint64)
        off = int(sf.d_off.download(8, 8 * (R - 1)).view(np.uint64)[0])
        assert int(last[0]) == off and int(last[1]) == size - off
    # rows tile the covered bytes: off[k+1] == off[k] + len[k] (checked on the host)
    tab = rows.rows(R)
    assert int(tab[0, 0]) == 0 and bool(np.all(tab[1:, 0] == tab[:-1, 0] + tab[:-1, 1]))
    # oracle identity at full size: the C restatement over the same bytes, in host memory
    host = data.download(size)
    for b in (data, rows):
        b.free()
    sf.free()
    exp, err = oracle_lib.record_index(host, fmt)
    del host
    assert err is None and len(exp) == R
    assert hashlib.sha256(tab.tobytes()).hexdigest() == hashlib.sha256(exp.tobytes()).hexdigest()
    assert np.array_equal(tab, exp)


# ---- configs[3]: 50 GiB parent + 1 % subset ------------------------------------------------------
def test_subset_50gib(gpu_ctx):
    from shock_amd.synth import SynthFile
    size = 50 * GIB
    sf = SynthFile(gpu_ctx, "fastq", size)
    data = sf.window(0, size)
    R = sf.expected_count()
    rows = gpu_ctx.alloc(16 * (R + 1024))
    r = gpu_ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
    assert r.ok and r.count == R
    assert sf.check_rows(rows, 0, R) == 0
    rng = np.random.default_rng(0x5EED)
    k = R // 100
    ids = np.sort(rng.choice(R, size=k, replace=False) + 1)
    text = ("\n".join(map(str, ids.tolist())) + "\n").encode()
    d_ids = gpu_ctx.alloc(len(text) + 64)
    d_ids.upload(text)
    d_sub = gpu_ctx.alloc(16 * (k + 16))
    d_runs = gpu_ctx.alloc(16 * (k + 16))
    res = gpu_ctx.subset_index(d_ids.ptr, len(text), rows.ptr, R, R, d_sub.ptr, k + 16, d_runs.ptr, k + 16)
    assert res.ok and res.count == k, res
    parent = rows.rows(R)
    got = d_sub.rows(k)
    assert np.array_equal(got, parent[ids - 1])
    # runs: maximal contiguous pieces of the selected rows (subset.go:245), same total bytes
    runs = d_runs.rows(res.runs)
    brk = np.flatnonzero(got[1:, 0] != got[:-1, 0] + got[:-1, 1]) + 1
    starts = np.concatenate([[0], brk])
    ends = np.concatenate([brk, [k]])
    exp_runs = np.stack([got[starts, 0], np.add.reduceat(got[:, 1], starts)], axis=1)
    assert res.runs == len(exp_runs) and np.array_equal(runs, exp_runs)
    assert res.size == int(got[:, 1].sum())
    d_out = gpu_ctx.alloc(res.size + 64)
    g = gpu_ctx.subset_gather(data.ptr, size, d_runs.ptr, res.runs, d_out.ptr, res.size)
    assert g.ok and g.size == res.size
    # the whole gathered output: each run's bytes hashed on the device from the
    # parent at its offset and from the output at its place there (k_run_hash, libshocksynth)
    from shock_amd.synth import run_hashes
    outoff = np.concatenate([[0], np.cumsum(runs[:, 1])]).astype(np.uint64)
    oruns = np.stack([outoff[:-1], runs[:, 1]], axis=1).astype(np.uint64)
    d_oruns = gpu_ctx.alloc(16 * len(oruns))
    d_oruns.upload(oruns)
    h_parent = run_hashes(gpu_ctx, data.ptr, d_runs.ptr, res.runs)
    h_out = run_hashes(gpu_ctx, d_out.ptr, d_oruns.ptr, res.runs)
    assert len(h_parent) == res.runs and np.array_equal(h_parent, h_out), int(np.argmin(h_parent == h_out))
    assert len(np.unique(h_parent)) > res.runs * 0.99  # (the hashes tell runs apart)
    for i in (0, res.runs // 2, res.runs - 1):  # and a few runs byte for byte
        o, n = int(runs[i, 0]), int(runs[i, 1])
        assert data.download(n, o).tobytes() == d_out.download(n, int(outoff[i])).tobytes()
    del ends
    for b in (data, rows, d_ids, d_sub, d_runs, d_out, d_oruns):
        b.free()
    sf.free()


# ---- configs[0]: files through shockidx_create ----------------------------------------------------
@pytest.mark.parametrize("mib", [64, 200])
def test_create_fd_large(gpu_ctx, oracle_lib, big_fastq, tmp_path, mib):
    host, _ = big_fastq
    exp_all, _ = oracle_lib.record_index(host, "fastq")
    cut = int(exp_all[np.searchsorted(exp_all[:, 0], mib * MIB) - 1, 0])  # whole records
    h = host[:cut]
    if mib == 64:  # exactly 64 MiB: pad with trailing blank lines (legal, unindexed)
        h = np.concatenate([h, np.full(64 * MIB - h.size, 10, np.uint8)])
        assert h.size == 64 * MIB
    f = tmp_path / "node.data"
    h.tofile(f)
    exp, err = oracle_lib.record_index(h)
    assert err is None
    out = tmp_path / "record.idx"
    fd = os.open(f, os.O_RDONLY)
    try:
        r = gpu_ctx.create(fd, h.size, "record", str(tmp_path), str(out))
    finally:
        os.close(fd)
    assert r.ok and r.count == len(exp), r
    assert out.read_bytes() == exp.astype("<u8").tobytes()


# ---- reentrancy: two contexts, two threads, one GPU ----------------------------------------------
def test_two_contexts_concurrent(gpu_ctx, oracle_lib, big_fastq):
    from shock_amd import Context
    host, _ = big_fastq
    a = host
    ea, _ = oracle_lib.record_index(a, "fastq")
    b = host[: int(ea[len(ea) // 2, 0])]  # the first half of the records
    eb, _ = oracle_lib.record_index(b)
    ca, cb = Context(0), Context(0)
    bufs = {}
    for name, ctx, h in (("a", ca, a), ("b", cb, b)):
        d = ctx.alloc(h.size + 64)
        d.upload(h)
        rows = ctx.alloc(16 * (h.size // 32 + 4096))
        bufs[name] = (ctx, d, rows, h.size)

    def build(name, reps, out):
        ctx, d, rows, n = bufs[name]
        t0 = time.perf_counter()
        for _ in range(reps):
            r = ctx.build_buffer(d, n, rows, kind="record", fmt=None)
            assert r.ok, r
        out[name] = (time.perf_counter() - t0) / reps
        out[name + "_rows"] = rows.rows(r.count)

    reps = 20
    solo = {}
    build("a", 3, {})
    build("b", 3, {})
    build("a", reps, solo)
    build("b", reps, solo)
    both = {}
    ths = [threading.Thread(target=build, args=(n, reps, both)) for n in ("a", "b")]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    wall = time.perf_counter() - t0
    assert np.array_equal(both["a_rows"], ea) and np.array_equal(both["b_rows"], eb)
    # the device work of the two builds is serialised per GPU: neither build exceeds twice its
    # solo time by more than the other build's share, and the pair takes no longer than the sum
    total_solo = (solo["a"] + solo["b"]) * reps
    assert wall < 1.5 * total_solo + 0.5, (wall, total_solo)
    assert both["a"] < 2 * (solo["a"] + solo["b"]) + 0.05 and both["b"] < 2 * (solo["a"] + solo["b"]) + 0.05
    print(f"solo a {solo['a']*1e3:.2f} ms b {solo['b']*1e3:.2f} ms; concurrent a {both['a']*1e3:.2f} "
          f"b {both['b']*1e3:.2f} ms, wall {wall*1e3:.1f} ms for {reps}+{reps}")
    for ctx, d, rows, _ in bufs.values():
        d.free()
        rows.free()
    ca.close()
    cb.close()


# ---- configs[4]: 80 GiB FASTQ, one GPU and 8 slabs --------------------------------------------
def test_c5_80gib_one_gpu_and_8_slabs(gpu_ctx):
    """C5 at full size on one MI355X: the 80 GiB node indexed whole (the strong-scaling 1-GPU
    point) and as 8 slabs of 10 GiB through the multi-GPU protocol (guess, slab index, summary
    fold, rows owned) with every slab on this device -- both checked row by row against the
    generator."""
    from shock_amd import dist
    from shock_amd.synth import SynthFile
    size = 80 * GIB
    sf = SynthFile(gpu_ctx, "fastq", size)
    R = sf.expected_count()
    data = sf.window(0, size)
    rows = gpu_ctx.alloc(16 * (R + 1024))
    r = gpu_ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
    assert r.ok and r.count == R, r
    assert sf.check_rows(rows, 0, R) == 0
    for b in (data, rows):
        b.free()
    world = 8
    engines, bufs = [], []
    for rk, (lo, hi) in enumerate(dist.plan_slabs(size, world)):
        wlo, whi = dist.slab_window(size, lo, hi)
        buf = sf.window(wlo, whi)
        k0, k1 = sf.record_range(lo, hi)
        cap = (k1 - k0) + 1024
        srows = gpu_ctx.alloc(16 * cap)
        e = dist.DeviceSlabEngine(gpu_ctx, rk, world)
        e.set_slab(buf, wlo, lo, hi, whi, size, srows, cap)
        engines.append(e)
        bufs.append((buf, srows))
    outs = dist.run_protocol(engines, dist.LocalExchange(), 2)
    assert outs[0].plan.count == R and outs[0].rounds == 1
    total = 0
    for e, o in zip(engines, outs):
        assert sf.check_rows(e.rows, o.plan.first_record, o.rows_owned) == 0
        total += o.rows_owned
    assert total == R
    for e in engines:
        e.free()
    for b, sr in bufs:
        b.free()
        sr.free()
    sf.free()


def test_c3_fasta_10gib_as_8_slabs(gpu_ctx):
    """C3 (10 GiB FASTA) cut into 8 slabs through the slab protocol on this device: every slab
    runs the FASTA tile pass (the armed bit carried in, the first piece left to the previous
    slab, the last record closed in the halo) and the owned rows equal the whole-file build."""
    from shock_amd import dist
    from shock_amd.synth import SynthFile
    size = 10 * GIB
    sf = SynthFile(gpu_ctx, "fasta", size)
    R = sf.expected_count()
    data = sf.window(0, size)
    rows = gpu_ctx.alloc(16 * (R + 1024))
    r = gpu_ctx.build_buffer(data, size, rows, kind="record", fmt="fasta")
    assert r.ok and r.count == R and r.path == 1, r
    whole = rows.rows(R)
    for b in (data, rows):
        b.free()
    world = 8
    engines, bufs = [], []
    for rk, (lo, hi) in enumerate(dist.plan_slabs(size, world)):
        wlo, whi = dist.slab_window(size, lo, hi)
        buf = sf.window(wlo, whi)
        k0, k1 = sf.record_range(lo, hi)
        cap = (k1 - k0) + 1024
        srows = gpu_ctx.alloc(16 * cap)
        e = dist.DeviceSlabEngine(gpu_ctx, rk, world)
        e.set_slab(buf, wlo, lo, hi, whi, size, srows, cap)
        engines.append(e)
        bufs.append((buf, srows))
    outs = dist.run_protocol(engines, dist.LocalExchange(), 1)
    assert outs[0].plan.count == R and outs[0].rounds == 1
    assert all(int(e.res.path) == 1 for e in engines)
    total = 0
    for e, o in zip(engines, outs):
        got = e.rows.rows(o.rows_owned)
        assert np.array_equal(got, whole[o.plan.first_record:o.plan.first_record + o.rows_owned]), e.rank
        total += o.rows_owned
    assert total == R
    for e in engines:
        e.free()
    for b, sr in bufs:
        b.free()
        sr.free()
    sf.free()


# ---- the drop-in with a bounded device footprint -------------------------------
def test_create_10gib_with_2gib_cap(gpu_ctx, oracle_lib, tmp_path):
    """configs[1]'s 10 GiB FASTQ node through shockidx_create with the context capped at 2 GiB of
    device memory: the slabs go through two slot buffers sized to the cap, the .idx is
    byte-identical to the oracle's, and the device memory the build took (hipMemGetInfo polled
    during the build) stays under the cap."""
    from shock_amd import Context
    from shock_amd.synth import SynthFile
    size, cap = 10 * GIB, 2 * GIB
    sf = SynthFile(gpu_ctx, "fastq", size)
    data = sf.window(0, size)
    R = sf.expected_count()
    host = data.download(size)
    data.free()
    sf.free()
    f = tmp_path / "node.data"
    host.tofile(f)
    exp, err = oracle_lib.record_index(host, "fastq")
    del host
    assert err is None and len(exp) == R
    ctx = Context(0)
    ctx.set_dev_cap(cap)
    hip = ctypes.CDLL("libamdhip64.so")
    free0, tot = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free0), ctypes.byref(tot)) == 0
    low = [free0.value]
    stop = threading.Event()

    def poll():
        fr = ctypes.c_size_t()
        while not stop.is_set():
            if hip.hipMemGetInfo(ctypes.byref(fr), ctypes.byref(tot)) == 0:
                low[0] = min(low[0], fr.value)
            time.sleep(0.0005)

    th = threading.Thread(target=poll)
    out = tmp_path / "record.idx"
    fd = os.open(f, os.O_RDONLY)
    th.start()
    try:
        r = ctx.create(fd, size, "record", str(tmp_path), str(out))
    finally:
        stop.set()
        th.join()
        os.close(fd)
    assert r.ok and r.count == R and r.path == 4, r  # (4: the slab pipeline through two slots)
    peak = free0.value - low[0]
    assert peak <= cap, (peak, cap)
    assert out.read_bytes() == exp.astype("<u8").tobytes()
    gib_s = size / (r.timings["total_ms"] * 1e-3) / GIB
    print(f"create 10 GiB under a 2 GiB cap: {gib_s:.1f} GiB/s end to end, peak device {peak / GIB:.2f} GiB")
