"""CPU: the subset-node chunkrecord (index/chunkrecord.go:100-228) -- the C oracle against
known answers read off the Go loop, a literal Python transcription of that loop, and the
"fresh start" formulation the GPU build evaluates in parallel (every chunk's end found from
prefix sums, the chain of chunk starts by pointer jumping): all three agree on random tables."""
import numpy as np
import pytest

import oracle

MIB = 1048576


def go_loop(lengths):
    """chunkrecord.go:140-216, transcribed."""
    out = []
    ri = po = pl = acc = 0
    for L in lengths:
        ri += 1
        if acc == 0:
            po, pl = (ri - 1) * 16, 16
        else:
            pl += 16
        if acc + L >= MIB:
            if acc == 0:
                out.append((po, pl))
                acc, pl = 0, 0
            else:
                out.append((po, pl - 16))
                acc, po, pl = L, (ri - 1) * 16, 16
        else:
            acc += L
    if acc != 0:
        out.append((po, pl))
    return out


def fresh_starts(lengths):
    """The parallel form: from a fresh start a, skip zero-length rows (a'), a row of >= 1 MiB is
    a chunk alone, else the chunk runs to the last row b - 1 whose running sum stays < 1 MiB;
    the next fresh start is a' + 1 or b."""
    L = list(lengths)
    R = len(L)
    P = np.concatenate([[0], np.cumsum(np.array(L, dtype=np.uint64))]).astype(np.uint64) if R else np.zeros(1, np.uint64)
    out, a = [], 0
    while a < R:
        a1 = a
        while a1 < R and L[a1] == 0:
            a1 += 1
        if a1 == R:
            break
        if L[a1] >= MIB:
            out.append((16 * a1, 16))
            a = a1 + 1
            continue
        q = int(np.searchsorted(P, P[a1] + MIB, side="left"))  # first q with P[q] >= P[a'] + 1 MiB
        b = q - 1 if q <= R else R
        out.append((16 * a1, 16 * (b - a1)))
        a = b
    return out


KATS = [
    ([100, 200], [(0, 32)]),
    ([600000, 600000], [(0, 16), (16, 16)]),
    ([2000000], [(0, 16)]),
    ([0, 5], [(16, 16)]),
    ([MIB - 1, 1], [(0, 16), (16, 16)]),
    ([], []),
    ([5, 0, 0], [(0, 48)]),
    ([2000000, 0, 7], [(0, 16), (32, 16)]),
    ([MIB // 2] * 5, [(0, 16), (16, 16), (32, 16), (48, 16), (64, 16)]),  # ">=": two halves never share a chunk
    ([MIB // 2 - 1] * 3, [(0, 32), (32, 16)]),
]


def _rows(lengths):
    L = np.array(lengths, dtype=np.uint64)
    off = np.concatenate([[0], np.cumsum(L)[:-1]]).astype(np.uint64) if len(L) else np.zeros(0, np.uint64)
    return np.stack([off, L], axis=1) if len(L) else np.zeros((0, 2), np.uint64)


@pytest.mark.parametrize("lengths,exp", KATS)
def test_kats(lengths, exp):
    assert go_loop(lengths) == exp
    assert fresh_starts(lengths) == exp
    got = oracle.chunkrecord_subset(_rows(lengths))
    assert [tuple(map(int, r)) for r in got] == exp


def test_random_tables_agree():
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(0, 400))
        kind = trial % 4
        if kind == 0:
            L = rng.integers(0, 400000, n)
        elif kind == 1:
            L = rng.choice([0, 1, 1000, MIB - 1, MIB, 3 * MIB, 300000], n)
        elif kind == 2:
            L = rng.integers(0, 2 * MIB, n) * (rng.random(n) < 0.8)
        else:
            L = rng.integers(100, 700, n * 20)
        L = [int(x) for x in L]
        exp = go_loop(L)
        assert fresh_starts(L) == exp
        got = oracle.chunkrecord_subset(_rows(L))
        assert [tuple(map(int, r)) for r in got] == exp
