"""CPU: the subset oracle (oracle/subset_oracle.c) against known answers derived by reading
index/subset.go:133-303 line by line (no reference fixture covers subset nodes: parity of
the restatement rests on these vectors)."""
import numpy as np
import pytest

PARENT = np.array([[0, 10], [10, 20], [30, 5], [35, 7], [42, 1], [43, 9]], dtype=np.uint64)

SORT = b"Subset indices must be numerically sorted and non-redundant, found value %d after value %d"

KATS = [
    # ids, rows, runs, size, err
    (b"1\n2\n3\n", [[0, 10], [10, 20], [30, 5]], [[0, 35]], 35, None),
    (b"1\n3\n5\n6", [[0, 10], [30, 5], [42, 1]], [[0, 10], [30, 5], [42, 1]], 16, None),  # last line w/o \n dropped
    (b"1\n3\n4\n6\n", [[0, 10], [30, 5], [35, 7], [43, 9]], [[0, 10], [30, 12], [43, 9]], 31, None),
    (b"\n\n2\n\n5\n", [[10, 20], [42, 1]], [[10, 20], [42, 1]], 21, None),           # blank lines skipped
    (b"+3\n", [[30, 5]], [[30, 5]], 5, None),                                         # Atoi accepts a sign
    (b"", [], [], 0, None),
    (b"\n", [], [], 0, None),
    (b"2\n2\n", [[10, 20]], [], 20, SORT % (2, 2)),
    (b"3\n1\n", [[30, 5]], [], 5, SORT % (1, 3)),
    (b"-1\n", [], [], 0, SORT % (-1, 0)),
    (b"0\n", [], [], 0, SORT % (0, 0)),
    (b"7\n", [], [], 0, b"Subset index: 7 does not exist in parent index file."),
    (b"x1\n", [], [], 0, b'strconv.Atoi: parsing "x1": invalid syntax'),
    (b"1\r\n", [], [], 0, b'strconv.Atoi: parsing "1\\r": invalid syntax'),
    (b" 1\n", [], [], 0, b'strconv.Atoi: parsing " 1": invalid syntax'),
    (b"-\n", [], [], 0, b'strconv.Atoi: parsing "-": invalid syntax'),
    (b"99999999999999999999\n", [], [], 0, b'strconv.Atoi: parsing "99999999999999999999": value out of range'),
    (b"9223372036854775808\n", [], [], 0, b'strconv.Atoi: parsing "9223372036854775808": value out of range'),
    (b"-9223372036854775809\n", [], [], 0, b'strconv.Atoi: parsing "-9223372036854775809": value out of range'),
    (b"12345678901234567890x\n", [], [], 0, b'strconv.Atoi: parsing "12345678901234567890x": invalid syntax'),
    (b"99999999999999999999x\n", [], [], 0, b'strconv.Atoi: parsing "99999999999999999999x": value out of range'),
    (b"9223372036854775807\n", [], [], 0, b"Subset index: 9223372036854775807 does not exist in parent index file."),
    (b"1\n2\nx\n", [[0, 10], [10, 20]], [], 30, b'strconv.Atoi: parsing "x": invalid syntax'),
    (b'\x01"\\\n', [], [], 0, b'strconv.Atoi: parsing "\\x01\\"\\\\": invalid syntax'),
]


@pytest.mark.parametrize("kat", KATS, ids=[repr(k[0])[:30] for k in KATS])
def test_subset_kat(oracle_lib, kat):
    ids, rows, runs, size, err = kat
    r, c, sz, e = oracle_lib.subset(ids, PARENT)
    assert e == err
    assert r.tolist() == rows
    if err is None:
        assert c.tolist() == runs and sz == size


def test_subset_read_past_parent(oracle_lib):
    # TotalUnits larger than the rows present: ReadAt fails (subset.go:218-223)
    r, c, sz, e = oracle_lib.subset(b"1\n8\n", PARENT, ilength=10)
    assert e == b"Subset index could not read parent index file for part: 8" and r.tolist() == [[0, 10]]


def test_subset_zero_length_final_run(oracle_lib):
    # oSize == 0: the final compressed row is never written (subset.go:285-291)
    par = np.array([[5, 0], [9, 0]], dtype=np.uint64)
    r, c, sz, e = oracle_lib.subset(b"1\n2\n", par)
    assert e is None and sz == 0 and r.tolist() == [[5, 0], [9, 0]] and c.tolist() == [[5, 0]]


def test_go_quote(oracle_lib):
    assert oracle_lib.go_quote(b"a\tb\x7f\xff\xc3\xa9") == b'"a\\tb\\x7f\\xff\xc3\xa9"'
    assert oracle_lib.go_quote("  ".encode()) == b'"\\u00a0\\u2028"'
