"""GPU: shockidx_build_host from a pinned (hipHostRegister'ed) node body: the direct-DMA input
path (1 GiB pieces) gives the same table as the pageable staging path and the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fmt", ["fastq", "fasta"])
def test_build_host_pinned_gpu(gpu_ctx, oracle_lib, fmt):
    from shock_amd.synth import SynthFile
    size = (1 << 30) + (96 << 20) + 12345  # crosses the 1 GiB DMA piece
    sf = SynthFile(gpu_ctx, fmt, size)
    data = sf.window(0, size)
    host = data.download(size)
    data.free()
    sf.free()
    exp, err = oracle_lib.record_index(host)
    assert err is None
    gpu_ctx.host_register(host)
    try:
        r = gpu_ctx.build_host(host, kind="record")
    finally:
        gpu_ctx.host_unregister(host)
    assert r.ok and r.fmt == fmt and r.count == len(exp)
    assert np.array_equal(r.rows, exp)
    r2 = gpu_ctx.build_host(host, kind="record")  # pageable: through the staging buffers
    assert r2.ok and np.array_equal(r2.rows, exp)


def test_build_host_pinned_small_gpu(gpu_ctx, oracle_lib):
    rec = b"@r1 x\nACGT\n+\nIIII\n@r2\nAC\n+r2\nII\n"
    host = np.frombuffer(rec * 5000 + b"@bad\nAC\n+\nI\n", np.uint8).copy()
    exp, err = oracle_lib.record_index(host.tobytes())
    gpu_ctx.host_register(host)
    try:
        r = gpu_ctx.build_host(host, kind="record")
    finally:
        gpu_ctx.host_unregister(host)
    assert not r.ok and r.err == err and r.count == len(exp)


def _synth_host(ctx, fmt, size):
    from shock_amd.synth import SynthFile
    sf = SynthFile(ctx, fmt, size)
    data = sf.window(0, size)
    host = data.download(size)
    data.free()
    sf.free()
    return host


def _pinned_build(ctx, host):
    ctx.host_register(host)
    try:
        return ctx.build_host(host, kind="record")
    finally:
        ctx.host_unregister(host)


def test_build_host_slab_pipeline_gpu(gpu_ctx, oracle_lib, monkeypatch):
    """A pinned FASTQ body of 2.5 GiB takes the slab-pipelined build (1 GiB slabs indexed while
    later slabs cross PCIe, rows copied out per slab): the table equals the oracle's and the
    plain one-pass build's (SHOCKIDX_NO_HOST_PIPE)."""
    size = (5 << 29) + 777
    host = _synth_host(gpu_ctx, "fastq", size)
    exp, err = oracle_lib.record_index(host)
    assert err is None
    r = _pinned_build(gpu_ctx, host)
    assert r.ok and r.fmt == "fastq" and r.count == len(exp)
    assert np.array_equal(r.rows, exp)
    monkeypatch.setenv("SHOCKIDX_NO_HOST_PIPE", "1")
    r2 = _pinned_build(gpu_ctx, host)
    assert r2.ok and np.array_equal(r2.rows, exp)


@pytest.mark.parametrize("where", ["error", "blank"])
def test_build_host_slab_pipeline_fallback_gpu(gpu_ctx, oracle_lib, where):
    """A slab that is not clean (a Go error in the second slab; a blank group right before the
    first slab boundary, legal only at the end of a file) sends the pipelined build back to the
    one-pass build of the whole body: count, rows and error text as the oracle's."""
    size = (5 << 29) + 12345
    host = _synth_host(gpu_ctx, "fastq", size)
    b = host
    if where == "error":
        p = (1 << 30) + (300 << 20)
        w = b[p:p + 8192]
        p = int(np.flatnonzero((w[1:] == ord("+")) & (w[:-1] == ord("\n")))[0]) + p + 1
        b[p] = ord("x")  # a plus line that does not start with '+'
    else:
        p = (1 << 30) - 2000
        s = int(np.flatnonzero(b[p:p + 4096] == ord("@"))[0]) + p  # a record start ...
        e = int(np.flatnonzero(b[s + 1:s + 8192] == ord("@"))[0]) + s + 1
        while b[e - 1] != ord("\n"):  # ... to the next record start
            e = int(np.flatnonzero(b[e + 1:e + 8192] == ord("@"))[0]) + e + 1
        b[s:e] = ord("\n")  # the record becomes blank lines
    exp, err = oracle_lib.record_index(b)
    assert err is not None
    r = _pinned_build(gpu_ctx, b)
    assert not r.ok and r.err == err and r.count == len(exp)
    assert np.array_equal(r.rows, exp)


def test_build_host_partly_registered_gpu(gpu_ctx, oracle_lib):
    """Only the first half of the body is registered: the build must not DMA past the pinned
    range (it takes the pageable staging path) and gives the oracle's table."""
    host = _synth_host(gpu_ctx, "fastq", (96 << 20) + 777)
    exp, err = oracle_lib.record_index(host)
    assert err is None
    half = host[: host.size // 2]
    gpu_ctx.host_register(half)
    try:
        r = gpu_ctx.build_host(host, kind="record")
    finally:
        gpu_ctx.host_unregister(half)
    assert r.ok and r.count == len(exp)
    assert np.array_equal(r.rows, exp)


def test_failed_build_then_builds_gpu(gpu_ctx, oracle_lib, monkeypatch):
    """a build that fails after taking its epoch (here: a forced error after the
    newline scan, before k_fq_place / k_finalize) leaves its scan tickets and first-bad key
    unreset.  The next builds on the same context -- both slot parities -- must still be exact
    (without the reset the third build's scan would wait on look-back words nobody writes)."""
    from shock_amd import _lib as L
    rec = b"@r1 x\nACGT\n+\nIIII\n@r2\nAC\n+r2\nII\n"
    good = np.frombuffer(rec * 200000, np.uint8).copy()
    bad = np.frombuffer(rec * 200000 + b"@bad\nAC\n+\nI\n", np.uint8).copy()
    exp_g, _ = oracle_lib.record_index(good.tobytes())
    exp_b, err_b = oracle_lib.record_index(bad.tobytes())
    monkeypatch.setenv("SHOCKIDX_DEBUG", "4096")
    with pytest.raises(L.ShockIdxError):
        gpu_ctx.build_host(good, kind="record", fmt="fastq")
    monkeypatch.delenv("SHOCKIDX_DEBUG")
    for _ in range(2):
        r = gpu_ctx.build_host(good, kind="record", fmt="fastq")
        assert r.ok and np.array_equal(r.rows, exp_g)
        r = gpu_ctx.build_host(bad, kind="record", fmt="fastq")
        assert not r.ok and r.err == err_b and r.count == len(exp_b)
