"""GPU parity of the FASTA tile pass (k_fa_tiles / k_fa_place / k_fa_fixup) against the oracle.

The tile pass decides each '>' inside its 16 KiB tile, validates a record at the tile that
holds its closing '>', and sends what a tile cannot decide alone to k_fa_fixup: the tile's
conditional first '>', pieces that start in an earlier tile without a local witness, non-ASCII
bytes at a trimmed edge, tiles with more candidates than the table holds.  These cases put
exactly those situations on tile edges (fasta.go:93-140 semantics, oracle/shockidx_oracle.c
fasta_get)."""
import os
import random

import numpy as np
import pytest

import gen

pytestmark = pytest.mark.gpu

TILE = 16384


def _check(ctx, oracle_lib, data):
    r = ctx.build_host(data, kind="record", fmt="fasta")
    rows, err = oracle_lib.record_index(data, "fasta")
    assert r.count == len(rows), (r.count, len(rows), r.err, err)
    assert r.err == err, (r.err, err)
    got = r.rows if r.rows is not None else np.zeros((0, 2), np.uint64)
    if not np.array_equal(got, rows):
        bad = np.nonzero((got != rows).any(axis=1))[0][:5]
        raise AssertionError(f"first mismatching rows {bad.tolist()}: gpu {got[bad].tolist()} "
                             f"oracle {rows[bad].tolist()}")
    return r


_TOKS = [b"ACGTACGTACGTACGT", b"\n", b">", b" ", b"\r\n", b"\t", b"\xc2\xa0", b"\xe3\x80\x80",
         b"\x85", b"x", b"\n\n", b">>", b"\n>", b"\n>id desc\n"]
_W = [40, 10, 3, 3, 2, 1, 1, 1, 1, 3, 2, 1, 5, 6]


def _noise(rng, n):
    out = bytearray()
    while len(out) < n:
        out += rng.choices(_TOKS, _W)[0]
    return bytes(out[:n])


def test_fasta_tiles_fuzz_gpu(gpu_ctx, oracle_lib):
    rng = random.Random(77)
    for _ in range(160):
        n = rng.choice([1, 2, 3, 100, 5000, TILE - 1, TILE, TILE + 1, 3 * TILE + 17, 70000])
        _check(gpu_ctx, oracle_lib, _noise(rng, n))


def test_fasta_tiles_edges_gpu(gpu_ctx, oracle_lib):
    """A '>' at tile offsets 0..5 after assorted line ends, followed by assorted pieces."""
    rng = random.Random(3)
    body = gen.fasta(rng, 60)[: 2 * TILE - 300]
    rest = gen.fasta(rng, 20)
    for d in range(6):
        for pre in (b"ACGT\n", b"\n", b"AC", b" \n", b"\xc2\xa0\n", b"\n \n", b">", b"\n>"):
            for post in (b"id\nACGT\n", b"\nACGT\n", b"x>y\nA\n", b"", b">\n", b" \n \n"):
                fill = 2 * TILE + d - len(body) - len(pre)
                filler = (b"ACGTACGTAC\n" * (fill // 11 + 1))[:fill]
                head = body + filler + pre
                assert len(head) == 2 * TILE + d
                for tail in (b"", rest):
                    _check(gpu_ctx, oracle_lib, head + b">" + post + tail)


def test_fasta_tiles_dense_gpu(gpu_ctx, oracle_lib):
    """Tiles with more candidates than the table holds (k_fa_fixup walks them whole)."""
    rng = random.Random(11)
    recs = b">a\nC\n" * 20000
    normal = gen.fasta(rng, 80)
    cases = [
        recs,
        normal + recs + normal,
        recs[:50001] + b">b\n\n" + recs,                 # an invalid piece inside a dense tile
        normal[: TILE + 7] + b"\n" + recs + b"\n",
        b"AC" + recs,                                   # record 0 without a '>'
        recs + b"\n>tail",                              # EOF piece without '\n'
        recs + b"\n>\n",                                # EOF piece that fails validation
        b">" * 40000 + b"\nAC\n" + recs,                # '>' runs: embedded, not boundaries
    ]
    for d in cases:
        _check(gpu_ctx, oracle_lib, d)


def test_fasta_tiles_long_records_gpu(gpu_ctx, oracle_lib):
    """Records spanning many tiles; closing pieces with and without a witness in their tile."""
    rng = random.Random(5)
    seq = gen._big_seq(rng, 200000, b"ACGT")
    for d in (
        b">h\n" + seq + b"\n>h2\nAC\n",
        b">h\n" + seq + b"\n>",
        b">h\n" + seq + b">h2\nAC\n",                    # '>' with no '\n' since the last '>'... embedded
        b">h" + seq + b"\n>h2\nAC\n",                    # header line the size of the record: invalid
        b">h\n" + b" " * 100000 + b"\n>x\nA\n",           # whitespace piece tail
        b">h\n" + seq + b"\n" + b" " * 40000 + b"\n",     # EOF piece ending in a long blank run
        b"\n" * 50000 + b">a\nC\n",
        seq,
    ):
        _check(gpu_ctx, oracle_lib, d)


def test_fasta_tiles_vs_two_pass_gpu(gpu_ctx, oracle_lib, monkeypatch):
    """The tile pass and the two-pass build agree on a multi-MiB synthetic FASTA."""
    rng = random.Random(21)
    data = gen.fasta(rng, 3000, long_every=40, long_len=60000, embedded_gt=0.1, crlf=0.1, uni=0.02)
    a = gpu_ctx.build_host(data, kind="record", fmt="fasta")
    monkeypatch.setenv("SHOCKIDX_FA_MODE", "two")
    b = gpu_ctx.build_host(data, kind="record", fmt="fasta")
    assert a.count == b.count and a.err == b.err
    assert np.array_equal(a.rows, b.rows)
    _check(gpu_ctx, oracle_lib, data)


def test_fasta_tile_certificate_gpu(gpu_ctx, oracle_lib):
    """The piece a tile's first '>' closes began in the previous tile: k_fa_place settles it with
    the previous tile's certificate (a '\\n' between two ASCII non-space bytes in the piece's part
    there) instead of k_fa_fixup.  Each case puts one piece across a tile edge with that part
    certifying it or not: valid and invalid pieces alike must come out as the oracle says."""
    rng = random.Random(31)
    tails = [
        b"hdr\nACGT",            # certified in the previous tile
        b"hdr   ",               # no '\n' there: the closing tile decides (or k_fa_fixup)
        b"hdr\n   ",             # '\n' followed by spaces only: not a certificate
        b"   \nA",               # leading spaces, then a witness
        b"hdr\xc2\xa0\nA",       # a non-ASCII byte before the '\n': not a certificate
        b"\n\n\nx",              # blank lines then a byte: '\n' between '\n' and 'x' is no witness
        b"h",                    # one byte before the edge
    ]
    heads = [b"CGTA\n>", b"   \n>", b"\n>", b">", b"  >", b"ACGT\r\n>", b"\xe3\x80\x80\n>"]
    for tail in tails:
        for head in heads:
            pre = gen.fasta(rng, 5)[: TILE - len(tail) - 1]
            body = pre + b"A" * (TILE - len(tail) - 1 - len(pre)) + b">"  # the piece starts after this '>'
            data = body + tail + head + b"id2\nACGT\n>id3\nGG\n"
            assert data[TILE:TILE + len(head)] == head  # the closing '>' is in the second tile
            _check(gpu_ctx, oracle_lib, data)
            # the same two tiles further into a longer file (tiles with t > 0 on both sides)
            lead = gen.fasta(rng, 40)[: 3 * TILE - 1] + b"\n"
            _check(gpu_ctx, oracle_lib, lead + data)
