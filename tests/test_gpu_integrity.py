"""GPU: a build never returns a wrong table as success.

record.go:51-83 writes row i + 1 at the offset where row i ends, starting at 0, so a table is
contiguous by construction and a successful FASTA / SAM / line build ends at the file end
(FASTQ: before trailing blank lines only, fastq.go:141-156).  The library checks that of its
own output -- in the finalize of every whole-file build, at every slab seam of the pipelined and
multi-GPU builds, and (SHOCKIDX_VERIFY, set for this suite in conftest.py) over the whole table --
and tags every multi-GPU slab summary with the caller's build / round, refusing stale ones.

The hooks below (shockidx_debug_inject / shockidx_multi_debug_inject, exported but not in the
public header) recreate the failure modes deterministically:
  * a freshly grown status array full of published look-back words of the next build's epoch,
    written before it is zeroed on the build stream: the build must be exact (the zeroing is
    ordered before the kernels);
  * the same words written after the zeroing (a zeroing that lost a race): exact or an internal
    error, never a different table with OK;
  * a finalize that reports one record short: an internal error for every format;
  * a multi-GPU exchange whose copy into the gathered buffers never lands (the r4 flake's
    mechanism: the fold read the previous build's summaries): an internal error.
"""
import os

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

EINTERNAL = -5


def _lib():
    from shock_amd import _lib as L
    return L.lib()


def _inject(ctx, flags):
    return _lib().shockidx_debug_inject(ctx._h, flags)


def _synth(ctx, fmt, size):
    from shock_amd.synth import SynthFile
    sf = SynthFile(ctx, fmt, size)
    host = sf.window(0, size).download(size)
    return host, sf.expected_count()


@pytest.fixture(scope="module")
def files(gpu_ctx, oracle_lib):
    out = {}
    for fmt in ("fastq", "fasta"):
        host, _ = _synth(gpu_ctx, fmt, 96 << 20)  # 6144 tiles: three look-back scan blocks
        rows, err = oracle_lib.record_index(host.tobytes(), fmt)
        assert err is None
        out[fmt] = (host, rows)
    return out


def _build(ctx, host, fmt):
    from shock_amd import _lib as L
    try:
        return ctx.build_host(host, kind="record", fmt=fmt), None
    except L.ShockIdxError as e:
        return None, e


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_poisoned_status_zeroed_before_build(fmt, files):
    from shock_amd import Context
    host, rows = files[fmt]
    for _ in range(3):  # a fresh context: its first build grows (and zeroes) the status array
        ctx = Context(0)
        _inject(ctx, 1)
        r, e = _build(ctx, host, fmt)
        ctx.close()
        assert e is None and r.ok and r.count == len(rows) and np.array_equal(r.rows, rows)


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_poisoned_status_after_zeroing_never_silent(fmt, files):
    from shock_amd import Context
    host, rows = files[fmt]
    for _ in range(3):
        ctx = Context(0)
        _inject(ctx, 2)
        r, e = _build(ctx, host, fmt)
        ctx.close()
        if e is None:  # every look-back read found its predecessor already published
            assert r.ok and r.count == len(rows) and np.array_equal(r.rows, rows)
        else:
            assert e.code == EINTERNAL, e


@pytest.mark.parametrize("mode", ["fastq", "fasta", "sam", "line", "fastq_blank_tail"])
def test_short_count_refused(gpu_ctx, oracle_lib, mode):
    import random
    from shock_amd import _lib as L
    rng = random.Random(17)
    if mode.startswith("fastq"):
        data = gen.fastq(rng, 300) + (b"\n\n\n" if mode == "fastq_blank_tail" else b"")
    elif mode == "fasta":
        data = gen.fasta(rng, 300)
    elif mode == "sam":
        data = gen.sam(rng, 300)
    else:
        data = gen.fastq(rng, 300)
    kind = "line" if mode == "line" else "record"
    fmt = None if kind == "line" else mode.split("_")[0]
    r = gpu_ctx.build_host(data, kind=kind, fmt=fmt)  # untouched: exact and OK
    exp = oracle_lib.line_index(data)[0] if kind == "line" else oracle_lib.record_index(data, fmt)[0]
    assert r.ok and np.array_equal(r.rows, exp)
    _inject(gpu_ctx, 4)
    try:
        with pytest.raises(L.ShockIdxError) as ei:
            gpu_ctx.build_host(data, kind=kind, fmt=fmt)
    finally:
        _inject(gpu_ctx, 0)
    assert ei.value.code == EINTERNAL
    r = gpu_ctx.build_host(data, kind=kind, fmt=fmt)  # the context is usable again
    assert r.ok and np.array_equal(r.rows, exp)


def test_short_count_refused_device_resident(gpu_ctx, files):
    """The device-resident entry point (what bench.py times) checks the same invariants."""
    from shock_amd import _lib as L
    host, rows = files["fastq"]
    d = gpu_ctx.alloc(host.size + 64, node=True)
    d.upload(host)
    out = gpu_ctx.alloc(16 * (len(rows) + 64))
    r = gpu_ctx.build_buffer(d, host.size, out, kind="record", fmt="fastq")
    assert r.ok and r.count == len(rows) and np.array_equal(out.rows(r.count), rows)
    _inject(gpu_ctx, 4)
    try:
        with pytest.raises(L.ShockIdxError) as ei:
            gpu_ctx.build_buffer(d, host.size, out, kind="record", fmt="fastq")
    finally:
        _inject(gpu_ctx, 0)
    assert ei.value.code == EINTERNAL
    d.free()
    out.free()


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_multi_stale_gathered_summaries_refused(gpu_ctx, oracle_lib, fmt):
    """Four slabs on device 0 with the host exchange: a build whose exchange does not land reads
    the previous build's summaries -- refused by their tags (r4: 3868 of 4000 rows with OK)."""
    import random
    from shock_amd import MultiContext, _lib as L
    rng = random.Random(13)
    data = gen.fasta(rng, 4000) if fmt == "fasta" else gen.fastq(rng, 4000)
    rows, err = oracle_lib.record_index(data, fmt)
    m = MultiContext([0, 0, 0, 0])
    try:
        r = m.build_host(data, fmt=fmt)
        assert r.ok and np.array_equal(r.rows, rows)
        assert _lib().shockidx_multi_debug_inject(m._h, 1) == 0
        with pytest.raises(L.ShockIdxError) as ei:
            m.build_host(data, fmt=fmt)  # the same bytes: only the tags tell the summaries apart
        assert ei.value.code == EINTERNAL and "stale slab summary" in ei.value.msg
        _lib().shockidx_multi_debug_inject(m._h, 0)
        r = m.build_host(data, fmt=fmt)
        assert r.ok and np.array_equal(r.rows, rows)
    finally:
        m.close()


def test_multi_resident_short_slab_refused(gpu_ctx, oracle_lib):
    """A slab that reports one record short breaks the seam with the next slab."""
    import random
    from shock_amd import MultiContext, _lib as L
    data = gen.fasta(random.Random(13), 4000)
    m = MultiContext([0, 0, 0, 0])
    plan = m.plan(len(data))
    wins, outs, caps = [], [], []
    for lo, hi, wlo, whi in plan:
        w = gpu_ctx.alloc(whi - wlo + 64)
        w.upload(np.frombuffer(data[wlo:whi], np.uint8))
        wins.append(w)
        caps.append((hi - lo) // 8 + 64)
        outs.append(gpu_ctx.alloc(16 * caps[-1]))
    try:
        r, first, owned = m.build_resident(len(data), [w.ptr for w in wins], [o.ptr for o in outs], caps, fmt="fasta")
        rows, _ = oracle_lib.record_index(data, "fasta")
        assert r.ok and r.count == len(rows)
        # every slab context of the group gets the hook
        for k in range(4):
            ctxp = _lib().shockidx_multi_debug_ctx(m._h, k)
            _lib().shockidx_debug_inject(ctxp, 4)
        with pytest.raises(L.ShockIdxError) as ei:
            m.build_resident(len(data), [w.ptr for w in wins], [o.ptr for o in outs], caps, fmt="fasta")
        assert ei.value.code == EINTERNAL
    finally:
        for b in wins + outs:
            b.free()
        m.close()


def test_pipelined_fd_short_slab_refused(gpu_ctx, oracle_lib, tmp_path):
    """The slab-pipelined fd build (>= 2 GiB): a slab one record short breaks the next seam."""
    from shock_amd import _lib as L
    from shock_amd.synth import SynthFile
    size = (5 << 29) + 12345
    sf = SynthFile(gpu_ctx, "fastq", size)
    host = sf.window(0, size).download(size)
    path = tmp_path / "node.data"
    host.tofile(path)
    del host
    fd = os.open(path, os.O_RDONLY)
    try:
        r = gpu_ctx.build_fd(fd, size)
        assert r.ok and r.path == 3 and r.count == sf.expected_count()
        _inject(gpu_ctx, 4)
        try:
            with pytest.raises(L.ShockIdxError) as ei:
                gpu_ctx.build_fd(fd, size)
        finally:
            _inject(gpu_ctx, 0)
        assert ei.value.code == EINTERNAL, ei.value
    finally:
        os.close(fd)
        path.unlink()
