"""GPU parity of the multi-slab path: a file cut into W slabs, each indexed
by the HIP kernels against a guessed incoming state (shockidx_slab_guess / _index), the
64-byte summaries folded on the device (shockidx_slab_combine), wrong guesses re-run.  One
process drives all W slabs (dist.LocalExchange) -- the same protocol bench.py --gpus N runs
with one GPU per slab and RCCL for the exchange.  Bar: the concatenated row table, count
and Go error text equal the oracle's single pass over the whole file, bit for bit."""
import random

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

FMT = {"fasta": 1, "fastq": 2, "sam": 3, "line": 4}


def _slabbed(ctx, data, fmt, world, front=64 << 10, halo=1 << 20, wrong=()):
    from shock_amd import dist
    size = len(data)
    engines, bufs = [], []
    for r, (lo, hi) in enumerate(dist.plan_slabs(size, world)):
        wlo, whi = dist.slab_window(size, lo, hi, front, halo)
        buf = ctx.alloc(whi - wlo + 64)
        buf.upload(np.frombuffer(data[wlo:whi], dtype=np.uint8))
        cap = (hi - lo) + 64
        rows = ctx.alloc(16 * cap)
        e = dist.DeviceSlabEngine(ctx, r, world)
        e.set_slab(buf, wlo, lo, hi, whi, size, rows, cap)
        if r in wrong:  # force a wrong guess: the fold must flag it and the re-run fix it
            g0 = e.guess
            e.guess = (lambda g0: lambda f: (g0(f) + 1) % {1: 2, 2: 4, 3: 3, 4: 1}[f])(g0)
        engines.append(e)
        bufs.append((buf, rows))
    outs = dist.run_protocol(engines, dist.LocalExchange(), FMT[fmt])
    table = np.concatenate([e.rows.rows(o.rows_owned) if o.rows_owned else np.zeros((0, 2), np.uint64)
                            for e, o in zip(engines, outs)])
    plan = outs[0].plan
    by_rank = {e.rank: e for e in engines}
    err = dist.error_text(plan, lambda pos, n: by_rank[plan.err_rank].error_bytes(pos, n))
    for e, o in zip(engines, outs):  # which build indexed each non-empty slab (1: tile pass)
        o.path = int(e.res.path) if e.slab.n else 0
    for e in engines:
        e.free()
    for b, r in bufs:
        b.free()
        r.free()
    return plan, table, err, outs


def _expect(oracle_lib, data, fmt):
    if fmt == "line":
        return oracle_lib.line_index(data)
    return oracle_lib.record_index(data, fmt)


def _cmp(ctx, oracle_lib, data, fmt, world, **kw):
    plan, table, err, outs = _slabbed(ctx, data, fmt, world, **kw)
    # FASTQ, FASTA and line slabs run the one-read tile passes; SAM the two-pass build
    want = 2 if fmt == "sam" else 1
    assert all(o.path in (0, want) for o in outs), (fmt, [o.path for o in outs])
    rows, oerr = _expect(oracle_lib, data, fmt)
    assert plan.count == len(rows), (fmt, world, plan, len(rows), oerr)
    assert err == oerr, (fmt, world, err, oerr)
    assert table.shape == rows.shape, (table.shape, rows.shape)
    if not np.array_equal(table, rows):
        bad = np.nonzero((table != rows).any(axis=1))[0][:5]
        raise AssertionError(f"{fmt} W={world}: rows {bad.tolist()} gpu {table[bad].tolist()} "
                             f"oracle {rows[bad].tolist()}")
    return outs


def _data(fmt, seed, n):
    rng = random.Random(seed)
    if fmt == "fastq":
        return gen.fastq(rng, n, at_qual=0.3, plus_id=0.3)
    if fmt == "fasta":
        return gen.fasta(rng, n)
    if fmt == "sam":
        return gen.sam(rng, n)
    return gen.lines(rng, n)


@pytest.mark.parametrize("fmt", ["fastq", "fasta", "sam", "line"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_slabs_clean(gpu_ctx, oracle_lib, fmt, world):
    n = {"fastq": 20000, "fasta": 3000, "sam": 20000, "line": 40000}[fmt]
    outs = _cmp(gpu_ctx, oracle_lib, _data(fmt, 100 + world, n), fmt, world)
    assert outs[0].rounds == 1  # the guesses were right


@pytest.mark.parametrize("fmt", ["fastq", "fasta", "sam"])
def test_slabs_wrong_guess(gpu_ctx, oracle_lib, fmt):
    n = {"fastq": 8000, "fasta": 2000, "sam": 8000}[fmt]
    outs = _cmp(gpu_ctx, oracle_lib, _data(fmt, 7, n), fmt, 4, wrong=(1, 3))
    assert outs[0].rounds == 2 and sum(o.reruns for o in outs[:1]) == 2


@pytest.mark.parametrize("fmt", ["fastq", "fasta", "sam", "line"])
def test_slabs_tiny_files(gpu_ctx, oracle_lib, fmt):
    rng = random.Random(99)
    for _ in range(40):
        d = gen.tiny(rng)
        for world in (2, 3):
            _cmp(gpu_ctx, oracle_lib, d, fmt, world, front=64, halo=4096)


@pytest.mark.parametrize("kind", ["no_at", "no_plus", "len_mismatch", "id_mismatch", "empty_seq", "blank_between", "truncate",
                                  "missing_id", "trail_partial"])
def test_slabs_fastq_errors(gpu_ctx, oracle_lib, kind):
    data = _data("fastq", 3, 6000)
    rng = random.Random(kind)
    for _ in range(3):
        bad = gen.fastq_corrupt(rng, data, kind)
        _cmp(gpu_ctx, oracle_lib, bad, "fastq", 3)


@pytest.mark.parametrize("kind", ["header_only", "gt_in_seq", "lead_newline", "trail_header"])
def test_slabs_fasta_errors(gpu_ctx, oracle_lib, kind):
    data = _data("fasta", 5, 1500)
    rng = random.Random(kind)
    for _ in range(3):
        bad = gen.fasta_corrupt(rng, data, kind)
        _cmp(gpu_ctx, oracle_lib, bad, "fasta", 3)


def test_slabs_long_records_cross_slabs(gpu_ctx, oracle_lib):
    rng = random.Random(17)
    for fmt, d in (("fastq", gen.fastq(rng, 400, long_every=50, long_len=60000)),
                   ("fasta", gen.fasta(rng, 300, long_every=40, long_len=120000)),
                   ("line", gen.lines(rng, 2000, long_every=300, long_len=90000))):
        _cmp(gpu_ctx, oracle_lib, d, fmt, 5)


def test_rccl_exchange_world1(gpu_ctx):
    """RCCL communicator of one rank: unique id, init, all-gather of a 64-byte summary."""
    from shock_amd import dist
    g = dist.SocketGroup(0, 1)
    ex = dist.RcclExchange(gpu_ctx, g)
    e = dist.DeviceSlabEngine(gpu_ctx, 0, 1)
    e.d_summary.upload(np.arange(64, dtype=np.uint8))
    ex.gather([e])
    gpu_ctx.sync()
    assert e.d_all.download(64).tolist() == list(range(64))
    assert ex.nranks == 1 and ex.gathers == 1  # ncclCommCount: what bench.py reports as rccl_ranks
    assert dist.rccl_report(ex, g) == (1, [1])
    ex.close()
    e.free()
