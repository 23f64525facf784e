"""CPU: the Idx.Part / Idx.Range / CreateSubsetIndex restatements (oracle/part_oracle.c).

Reference: shock-server/node/file/index/index.go:67-193 and subset.go:36-128.  The reference
holds no tests or vectors for these functions, so parity is unpinned by reference-held
outputs: the C oracle is checked against hand-derived known answers (read off the Go code
line by line, cited per case) and against `go_part` / `go_range` below, a literal transcription
of the Go control flow (same loop, same reused `rec` slice, same int64 wrap-around), over
random tables and part strings.
"""
import random

import numpy as np
import pytest

M64 = (1 << 64) - 1


def _i64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def _parse_int(s):
    """strconv.ParseInt(s, 10, 64) -> int or None (any error)."""
    if not s:
        return None
    neg = s[0] == "-"
    body = s[1:] if s[0] in "+-" else s
    if not body or any(c not in "0123456789" for c in body):
        return None
    v = int(body)
    if v > (1 << 63) - (0 if neg else 1):
        return None
    return -v if neg else v


def _read(rows, i):
    return (int(rows[i][0]), int(rows[i][1])) if 0 <= i < len(rows) else None


def go_part(rows, part, idx_length):
    if rows is None:
        return 0, 0, b"Index file is missing"
    if "-" in part:
        se = part.split("-")
        start, end = _parse_int(se[0]), _parse_int(se[1])
        if start is None or end is None or start <= 0 or start > idx_length or end <= 0 or end > idx_length:
            return 0, 0, b"Invalid index record range"
        s = _read(rows, start - 1) or (0, 0)
        e = _read(rows, end - 1) or (0, 0)
        return _i64(s[0]), _i64((e[0] - s[0]) + e[1]), None
    p = _parse_int(part)
    if p is None or p <= 0 or p > idx_length:
        return 0, 0, b"Index record out of bounds"
    r = _read(rows, p - 1) or (0, 0)
    return _i64(r[0]), _i64(r[1]), None


def go_range(rows, part, idx_length):
    if rows is None:
        return [], b"Index file is missing"
    recs = []
    rec = [0, 0]

    def read(i):
        r = _read(rows, i)
        if r is not None:
            rec[0], rec[1] = r

    if "-" in part:
        se = part.split("-")
        start, end = _parse_int(se[0]), _parse_int(se[1])
        if start is None or end is None or start <= 0 or start > idx_length or end <= 0 or end > idx_length:
            return [], b"Invalid index record range"
        read(start - 1)
        cur_pos, cur_len = rec[0], rec[1]
        if start == end:
            return [[_i64(cur_pos), _i64(cur_len)]], None
        x = start
        while x <= end - 1:
            read(x)
            next_pos, next_len = rec[0], rec[1]
            if x == end - 1:
                if (cur_len - (next_pos - cur_pos)) & M64 == 0:
                    recs.append([cur_pos, cur_len + next_len])
                else:
                    recs.append([cur_pos, cur_len])
                    recs.append([next_pos, next_len])
                break
            if (cur_len - (next_pos - cur_pos)) & M64 == 0:
                cur_len = cur_len + next_len
                x += 1
                continue
            recs.append([cur_pos, cur_len])
            cur_pos, cur_len = next_pos, next_len
            x += 1
        return [[_i64(a), _i64(b)] for a, b in recs], None
    p = _parse_int(part)
    if p is None or p <= 0 or p > idx_length:
        return [], b"Index record out of bounds"
    read(p - 1)
    return [[_i64(rec[0]), _i64(rec[1])]], None


# rows: 3 contiguous records, a gap, 2 contiguous, a gap, 1
ROWS = np.array([[0, 10], [10, 5], [15, 7], [40, 3], [43, 2], [100, 1]], dtype=np.uint64)


@pytest.mark.parametrize("part,exp", [
    ("1", (0, 10, None)),                              # index.go:100-115 single record
    ("6", (100, 1, None)),
    ("2-3", (10, 12, None)),                            # :98-99 pos = s.pos, len = e.pos - s.pos + e.len
    ("1-6", (0, 101, None)),                            # spans the gaps: Part does not care
    ("3-2", (15, -5 + 5, None)),                        # end < start is not rejected: (10-15)+5 = 0
    ("6-1", (100, -100 + 10, None)),                    # negative length, as Go computes it
    ("0", (0, 0, b"Index record out of bounds")),       # :102 p <= 0
    ("7", (0, 0, b"Index record out of bounds")),       # :102 p > idxLength
    ("x", (0, 0, b"Index record out of bounds")),       # ParseInt error
    ("+2", (10, 5, None)),                              # ParseInt accepts a sign
    ("0-2", (0, 0, b"Invalid index record range")),     # :81 start <= 0
    ("1-7", (0, 0, b"Invalid index record range")),     # :81 end > idxLength
    ("-2", (0, 0, b"Invalid index record range")),      # Split: ["", "2"] -> ParseInt("") fails
    ("2-", (0, 0, b"Invalid index record range")),
    ("2-3-9", (10, 12, None)),                          # Split: the third field is ignored
    ("2-3-x", (10, 12, None)),
    ("1 -2", (0, 0, b"Invalid index record range")),    # no trimming
    ("99999999999999999999-2", (0, 0, b"Invalid index record range")),  # range error
])
def test_part_kats(oracle_lib, part, exp):
    assert oracle_lib.idx_part(ROWS, part, 6) == exp
    assert go_part(ROWS, part, 6) == exp


@pytest.mark.parametrize("part,exp", [
    ("1", [[0, 10]]),                                   # :178-192
    ("1-1", [[0, 10]]),                                 # :146-150 start == end
    ("1-3", [[0, 22]]),                                 # :152-177 coalesced
    ("1-6", [[0, 22], [40, 5], [100, 1]]),              # runs split at the gaps
    ("3-4", [[15, 7], [40, 3]]),                        # :161-168 last pair not contiguous
    ("4-5", [[40, 5]]),                                 # :161-163 last pair contiguous
    ("5-4", []),                                        # end < start: the loop never runs, nil
    ("6-1", []),
    ("0-1", b"Invalid index record range"),
    ("7", b"Index record out of bounds"),
])
def test_range_kats(oracle_lib, part, exp):
    recs, err = oracle_lib.idx_range(ROWS, part, 6)
    if isinstance(exp, bytes):
        assert err == exp and recs.shape == (0, 2)
    else:
        assert err is None and recs.tolist() == exp
    assert go_range(ROWS, part, 6) == ((exp, None) if not isinstance(exp, bytes) else ([], exp))


def test_missing_file(oracle_lib):
    assert oracle_lib.idx_part(None, "1", 5) == (0, 0, b"Index file is missing")
    recs, err = oracle_lib.idx_range(None, "1-2", 5)
    assert err == b"Index file is missing" and recs.shape == (0, 2)


def test_short_file_reads(oracle_lib):
    """idxLength larger than the file: Part reads zeros past the end; Range keeps the last row read."""
    rows = ROWS[:3]
    assert oracle_lib.idx_part(rows, "5", 6) == (0, 0, None)
    assert oracle_lib.idx_part(rows, "2-5", 6) == (10, _i64(0 - 10 + 0), None)
    recs, err = oracle_lib.idx_range(rows, "2-6", 6)
    # rows 2,3 then rows 4,5,6 all read as row 3 again: (15,7) after (15,7) is not contiguous
    assert err is None and recs.tolist() == go_range(rows, "2-6", 6)[0]
    assert recs.tolist() == [[10, 12], [15, 7], [15, 7], [15, 7]]
    recs, err = oracle_lib.idx_range(rows, "5-6", 6)  # even row 5 is past the end: zeros
    assert recs.tolist() == [[0, 0]] and go_range(rows, "5-6", 6)[0] == [[0, 0]]


def _random_rows(rng, n):
    rows = np.zeros((n, 2), dtype=np.uint64)
    pos = rng.randrange(0, 1000)
    for i in range(n):
        ln = rng.choice([0, 1, rng.randrange(1, 500)])
        rows[i] = (pos, ln)
        pos += ln + (0 if rng.random() < 0.7 else rng.randrange(1, 50))
        if rng.random() < 0.05:
            pos = rng.randrange(0, 1 << 63)  # jumps backwards / far: 64-bit wrap cases
    return rows


def _random_part(rng, n):
    c = rng.random()
    if c < 0.2:
        return str(rng.randrange(-2, n + 3))
    a, b = rng.randrange(-1, n + 3), rng.randrange(-1, n + 3)
    if c < 0.3:
        return f"{a}-{b}-{rng.randrange(0, 9)}"
    if c < 0.35:
        return f"+{a}-{b}"
    return f"{a}-{b}"


def test_random_against_transcription(oracle_lib):
    rng = random.Random(20261016)
    for _ in range(400):
        n = rng.randrange(1, 60)
        rows = _random_rows(rng, n)
        il = n if rng.random() < 0.8 else n + rng.randrange(1, 5)  # short files too
        part = _random_part(rng, il)
        assert oracle_lib.idx_part(rows, part, il) == go_part(rows, part, il), part
        recs, err = oracle_lib.idx_range(rows, part, il)
        exp, eerr = go_range(rows, part, il)
        assert err == eerr and recs.tolist() == exp, part


def test_create_subset_index(oracle_lib):
    """subset.go:36-128: the subset rows and (count, size); every error (-1, -1)."""
    parent = ROWS
    rows, count, size, err = oracle_lib.create_subset_index(b"1\n2\n\n5\n", parent, 6)
    assert err is None and count == 3 and size == 10 + 5 + 2
    assert rows.tolist() == [[0, 10], [10, 5], [43, 2]]
    for ids, msg in [
        (b"2\n1\n", b"Subset indices must be numerically sorted and non-redundant, found value 1 after value 2"),
        (b"7\n", b"Subset index: 7 does not exist in parent index file."),
        (b"1\nx\n", b'strconv.Atoi: parsing "x": invalid syntax'),
    ]:
        rows, count, size, err = oracle_lib.create_subset_index(ids, parent, 6)
        assert (count, size, err) == (-1, -1, msg)
    # the node-index builder on the same ids agrees on the rows (:133-303 vs :36-128)
    r2, runs, size2, err2 = oracle_lib.subset(b"1\n2\n\n5\n", parent, 6)
    assert err2 is None and r2.tolist() == [[0, 10], [10, 5], [43, 2]] and size2 == 17
