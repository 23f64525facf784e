"""SAM tile pass (k_sam_tiles / k_sam_resolve / k_line_place<F_SAM> / k_sam_final) against the
oracle's restatement of sam.go:83-98 GetReadOffset + record.go:51-83 Create, and against the
two-pass build (SHOCKIDX_SAM_MODE=two).

A record ends at the '\\n' of a terminator line (longer than the '\\n' alone, first byte not
'@'); header and blank lines go to the record after them; the bytes after the last terminator
are one more record when there are any.  The cases aim at what a tile cannot see by itself: the
first '\\n' of a tile, whose line starts in an earlier tile (a data or a header line crossing
the boundary) or exactly at the tile start (first byte '@', '\\n', '\\r' or data); tiles without
a terminator; header-only and '\\n'-only stretches over many tiles; every kind of tail; tiles
with more terminators than the per-tile position capacity (records under 16 bytes: the build
re-runs two-pass).
Bar: bit-exact rows and counts."""
import functools
import random

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

TILE = 16384


def _boundaries():
    """Twelve tiles; around every tile boundary a different situation."""
    rng = random.Random(3)
    out = bytearray()
    kinds = [b"@", b"\n", b"\r", b"x", b"hdr_cross", b"data_cross", b"nl_last", b"at_last"]
    for k in range(12):
        kind = kinds[k % len(kinds)]
        end = (k + 1) * TILE
        while len(out) < end - 400:
            L = rng.randint(20, 300)
            out += (b"@CO\t" if rng.random() < 0.2 else b"r") + b"x" * L + b"\n"
        if kind in (b"@", b"\n", b"\r", b"x"):  # a line ends exactly at the tile end
            out += b"y" * (end - 1 - len(out)) + b"\n" + kind + b"z" * 30 + b"\n"
        elif kind == b"hdr_cross":  # a header line across the boundary
            out += b"\n@SQ\t" + b"h" * (end - len(out) + 40) + b"\n"
        elif kind == b"data_cross":  # a data line across the boundary
            out += b"\nread\t" + b"d" * (end - len(out) + 40) + b"\n"
        elif kind == b"nl_last":  # '\n' as the tile's last byte after a lone '\n' line
            out += b"q" * (end - 2 - len(out)) + b"\n\n" + b"w" * 10 + b"\n"
        else:  # '@' as the tile's last byte, starting a header
            out += b"q" * (end - 2 - len(out)) + b"\n@" + b"v" * 10 + b"\n"
    return bytes(out)


def _fuzz(seed, n):
    rng = np.random.default_rng(seed)
    alph = np.frombuffer(b"\n@x\r\t", np.uint8)
    p = np.array([0.04, 0.04, 0.84, 0.04, 0.04])  # lines of ~25 bytes: under the per-tile capacity
    return alph[rng.choice(len(alph), size=n, p=p)].tobytes()


@functools.lru_cache(maxsize=1)
def _sam():
    return gen.sam(random.Random(11), 60000, headers=500)


def _cases():
    sam = _sam()
    yield "tiny_a", b"a"
    yield "tiny_at", b"@"
    yield "tiny_nl", b"\n"
    yield "tiny_term", b"ab\n"
    yield "tiny_header", b"@a\n"
    yield "tiny_mix", b"\n\n@h\nx\ny\n\n"
    yield "nl_only", b"\n" * (3 * TILE + 5)
    yield "no_nl", b"x" * (4 * TILE + 7)
    yield "headers_only", b"".join(b"@SQ\tSN:" + str(i).encode() + b"\tLN:1000\n" for i in range(20000))
    yield "headers_then_data", b"@H\t" + b"h" * (5 * TILE) + b"\n" + sam
    yield "boundaries", _boundaries()
    yield "sam_nl_end", sam
    yield "sam_no_final_nl", sam.rstrip(b"\n")
    yield "sam_trailing_blank", sam + b"\n" * 5000
    yield "sam_trailing_header", sam + b"@CO\tend"
    yield "sam_crlf", sam.replace(b"\n", b"\r\n")
    yield "fuzz", _fuzz(5, 6 * TILE + 321)
    yield "dense", b"".join(b"r" + b"x" * (i % 9) + b"\n" for i in range(40000))
    yield "mixed_density", sam[: 3 * TILE] + b"".join(b"a\n" for _ in range(20000)) + sam[3 * TILE:]
    yield "big", gen.sam(random.Random(12), 80000, headers=20000, blank=0.1)


NAMES = ["tiny_a", "tiny_at", "tiny_nl", "tiny_term", "tiny_header", "tiny_mix", "nl_only", "no_nl",
         "headers_only", "headers_then_data", "boundaries", "sam_nl_end", "sam_no_final_nl",
         "sam_trailing_blank", "sam_trailing_header", "sam_crlf", "fuzz", "dense", "mixed_density", "big"]


def _case(name):  # generated when a test asks (not at collection: the CPU suite collects this file)
    for k, v in _cases():
        if k == name:
            return v
    raise KeyError(name)


def _check(r, rows, err, name):
    assert err is None and r.err is None, (name, r.err, err)
    assert r.count == len(rows), (name, r.count, len(rows))
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    if not np.array_equal(got, rows):
        bad = np.nonzero((got != rows).any(axis=1))[0][:5]
        raise AssertionError(f"{name}: rows {bad.tolist()}: gpu {got[bad].tolist()} oracle {rows[bad].tolist()}")


@pytest.mark.parametrize("name", NAMES)
def test_sam_tiles_vs_oracle(gpu_ctx, oracle_lib, name):
    data = _case(name)
    r = gpu_ctx.build_host(data, kind="record", fmt="sam")
    rows, err = oracle_lib.record_index(data, "sam")
    _check(r, rows, err, name)
    assert r.fmt == "sam"
    if name not in ("dense", "mixed_density"):
        assert r.path == 1, (name, r.path)  # the tile pass, not the two-pass build
    else:
        assert r.path == 2, (name, r.path)  # over LCAP terminators in a tile: re-run two-pass


@pytest.mark.parametrize("name", ["boundaries", "fuzz", "big", "sam_crlf"])
def test_sam_tiles_vs_two_pass(gpu_ctx, name, monkeypatch):
    data = _case(name)
    a = gpu_ctx.build_host(data, kind="record", fmt="sam")
    monkeypatch.setenv("SHOCKIDX_SAM_MODE", "two")
    b = gpu_ctx.build_host(data, kind="record", fmt="sam")
    assert a.path == 1 and b.path == 2
    assert a.count == b.count and np.array_equal(a.rows, b.rows)


def test_sam_tiles_fuzz_many_gpu(gpu_ctx, oracle_lib):
    """Short random '\\n' / '@' / data / '\\r' / tab strings over one to three tiles."""
    for seed in range(40):
        n = 1 + (seed * 7919) % (3 * TILE)
        data = _fuzz(100 + seed, n)
        r = gpu_ctx.build_host(data, kind="record", fmt="sam")
        rows, err = oracle_lib.record_index(data, "sam")
        _check(r, rows, err, f"seed {seed}")
