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
