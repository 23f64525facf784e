"""Line index tile pass (k_line_tiles / k_line_place / k_line_final) against the oracle's
line.go restatement and against the two-pass build (SHOCKIDX_LINE_MODE=two).

Cases: tile-aligned sizes, tiles denser than the per-tile position capacity (lines under
16 bytes, rescanned from global memory), no '\\n' at all, '\\n'-only input, long lines
spanning many tiles, a missing or present trailing '\\n', '\\n's exactly 255 / 256 / 257
bytes apart and lines over 255 bytes among short ones.  Bar: bit-exact rows and counts."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TILE = 16384


def _lines(rng, n, lo, hi):
    out = bytearray()
    while len(out) < n:
        k = int(rng.integers(lo, hi + 1))
        out += b"x" * k + b"\n"
    return bytes(out[:n])


def _cases():
    rng = np.random.default_rng(77)
    yield "one_byte", b"a"
    yield "one_nl", b"\n"
    yield "nl_only_2tiles", b"\n" * (2 * TILE)
    yield "nl_only_ragged", b"\n" * (3 * TILE + 17)
    yield "no_nl_5tiles", b"y" * (5 * TILE + 3)
    yield "tile_aligned", _lines(rng, 8 * TILE, 20, 200)
    yield "tile_aligned_nl_end", _lines(rng, 8 * TILE - 1, 20, 200) + b"\n"
    yield "dense", _lines(rng, 6 * TILE + 999, 0, 14)
    yield "mixed_density", (_lines(rng, 3 * TILE, 0, 6) + _lines(rng, 3 * TILE, 100, 3000)
                            + _lines(rng, 2 * TILE + 5, 0, 30))
    yield "long_lines", _lines(rng, 20 * TILE, 5 * TILE, 7 * TILE)
    yield "boundary_nl", b"".join(b"z" * (TILE - 1) + b"\n" for _ in range(9))
    yield "random_bytes", rng.integers(0, 256, 4 * TILE + 1234, dtype=np.uint8).tobytes()
    yield "big_mixed", _lines(rng, 24 << 20, 0, 400)
    # '\n' gaps around one byte's range
    yield "delta_255", b"".join(b"d" * 254 + b"\n" for _ in range(700))
    yield "delta_256", b"".join(b"e" * 255 + b"\n" for _ in range(700))
    yield "delta_257", b"".join(b"f" * 256 + b"\n" for _ in range(700))
    yield "wide_mix", b"".join((b"w" * 300 if i % 37 == 5 else b"s" * (20 + i % 180)) + b"\n" for i in range(60000))


CASES = dict(_cases())


@pytest.mark.parametrize("name", sorted(CASES))
def test_line_tiles_vs_oracle(gpu_ctx, oracle_lib, name):
    data = CASES[name]
    r = gpu_ctx.build_host(data, kind="line")
    rows, err = oracle_lib.line_index(data)
    assert err is None and r.err is None
    assert r.count == len(rows)
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    if not np.array_equal(got, rows):
        bad = np.nonzero((got != rows).any(axis=1))[0][:5]
        raise AssertionError(f"{name}: rows {bad.tolist()}: gpu {got[bad].tolist()} oracle {rows[bad].tolist()}")


@pytest.mark.parametrize("name", ["dense", "mixed_density", "big_mixed", "wide_mix"])
def test_line_tiles_vs_two_pass(gpu_ctx, name, monkeypatch):
    data = CASES[name]
    a = gpu_ctx.build_host(data, kind="line")
    monkeypatch.setenv("SHOCKIDX_LINE_MODE", "two")
    b = gpu_ctx.build_host(data, kind="line")
    assert a.count == b.count
    assert np.array_equal(a.rows, b.rows)


def test_line_tiles_row_cap_retry(gpu_ctx, oracle_lib):
    """More rows than the first row buffer guess: the host retries with the exact count."""
    data = b"\n" * (40 * TILE)
    r = gpu_ctx.build_host(data, kind="line")
    assert r.count == 40 * TILE + 1
    rows, _ = oracle_lib.line_index(data)
    assert np.array_equal(r.rows, rows)
