"""CPU: the oracle (C restatement + Python restatement) against the golden vectors.

Pins the oracle before it is trusted as the GPU checker: SURVEY.md Appendix B KATs (plus
hand-derived edge cases, tests/golden/kats.json), the reference's own fixture files
(tests/golden/fixtures/ copied from /root/reference/test/testdata/) with their expected index
tables (tests/golden/expected/, written by make_golden.py from the Python restatement), and a
C-vs-Python differential fuzz."""
import hashlib
import json
import os
import random

import pytest

import gen
import pyref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
KATS = json.load(open(os.path.join(GOLD, "kats.json")))
MANIFEST = json.load(open(os.path.join(GOLD, "expected", "manifest.json")))


def _rows(r):
    return [list(map(int, x)) for x in (r.tolist() if hasattr(r, "tolist") else r)]


@pytest.mark.parametrize("kat", KATS["record_kats"], ids=lambda k: k["id"])
def test_kat_c_oracle(oracle_lib, kat):
    data = bytes.fromhex(kat["input_hex"])
    rows, err = (oracle_lib.line_index(data) if kat["mode"] == "line"
                 else oracle_lib.record_index(data, kat["mode"]))
    assert _rows(rows) == kat["rows"]
    assert (err.hex() if err is not None else None) == kat["err_hex"]


@pytest.mark.parametrize("kat", KATS["record_kats"], ids=lambda k: k["id"])
def test_kat_pyref(kat):
    data = bytes.fromhex(kat["input_hex"])
    rows, err = pyref.line_index(data) if kat["mode"] == "line" else pyref.record_index(data, kat["mode"])
    assert _rows(rows) == kat["rows"]
    assert (err.hex() if err is not None else None) == kat["err_hex"]


@pytest.mark.parametrize("kat", KATS["detect_kats"], ids=lambda k: k["id"])
def test_detect_kat(oracle_lib, kat):
    data = bytes.fromhex(kat["input_hex"])
    assert pyref.detect_all(data) == kat["matches"]
    _, mask = oracle_lib.detect(data)
    assert [n for i, n in enumerate(("fasta", "fastq", "sam")) if mask >> i & 1] == kat["matches"]


FIXTURES = sorted(MANIFEST)
MODES = ("auto", "fasta", "fastq", "sam", "line")


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("mode", MODES)
def test_fixture_golden_c_oracle(oracle_lib, name, mode):
    data = open(os.path.join(GOLD, "fixtures", name), "rb").read()
    ent = MANIFEST[name]
    assert hashlib.sha256(data).hexdigest() == ent["sha256"]
    exp = ent["modes"][mode]
    if mode == "line":
        rows, err = oracle_lib.line_index(data)
    else:
        rows, err = oracle_lib.record_index(data, None if mode == "auto" else mode)
    idx = rows.astype("<u8").tobytes()
    assert len(rows) == exp["count"]
    assert (err.hex() if err is not None else None) == exp["err_hex"]
    assert hashlib.sha256(idx).hexdigest() == exp["idx_sha256"]
    assert idx == open(os.path.join(GOLD, "expected", f"{name}.{mode}.idx"), "rb").read()


def test_fixture_facts():
    """Appendix C facts that pin the restatement on the reference's own fixtures."""
    m = MANIFEST
    assert m["sample1.fq"]["modes"]["auto"]["count"] == 25
    assert m["10kb.fna"]["modes"]["auto"]["count"] == 80
    assert m["40kb.fna"]["modes"]["auto"]["count"] == 280
    assert m["nr_subset1.fa"]["modes"]["auto"]["count"] == 5
    assert m["sample1.fq"]["modes"]["line"]["count"] == 101
    assert m["10kb.fna"]["modes"]["line"]["count"] == 160
    # sample1.sam matches no validator (sam.go:17 needs whitespace as the third char);
    # nr_subset2.fa's 355 KB header never ends inside the 32 KiB detection window.
    for name in ("sample1.sam", "nr_subset2.fa"):
        assert m[name]["detect"] == []
        assert bytes.fromhex(m[name]["modes"]["auto"]["err_hex"]) == b"Invalid file type for filter"
    assert m["nr_subset2.fa"]["modes"]["fasta"]["count"] == 5
    assert m["sample1.sam"]["modes"]["sam"]["count"] == 47


def test_c_vs_python_fuzz(oracle_lib):
    rng = random.Random(7)
    for _ in range(1500):
        d = gen.tiny(rng)
        for f in ("fasta", "fastq", "sam"):
            r1, e1 = oracle_lib.record_index(d, f)
            r2, e2 = pyref.record_index(d, f)
            assert e1 == e2 and _rows(r1) == _rows(r2), (d, f)
        assert _rows(oracle_lib.line_index(d)[0]) == _rows(pyref.line_index(d)[0])
        assert oracle_lib.trim_space(d) == pyref.trim_space(d)
        _, mask = oracle_lib.detect(d)
        assert [n for i, n in enumerate(("fasta", "fastq", "sam")) if mask >> i & 1] == pyref.detect_all(d)


def test_c_vs_python_generated(oracle_lib):
    rng = random.Random(11)
    cases = [gen.fastq(rng, 200, crlf=0.1, uni=0.05), gen.fasta(rng, 50, embedded_gt=0.2, uni=0.05),
             gen.sam(rng, 100), gen.lines(rng, 300)]
    for kind in gen.FASTQ_CORRUPTIONS:
        cases.append(gen.fastq_corrupt(rng, gen.fastq(rng, 50), kind))
    for kind in ("header_only", "gt_in_seq", "lead_newline", "trail_header"):
        cases.append(gen.fasta_corrupt(rng, gen.fasta(rng, 20), kind))
    for d in cases:
        for f in (None, "fasta", "fastq", "sam"):
            r1, e1 = oracle_lib.record_index(d, f)
            r2, e2 = pyref.record_index(d, f)
            assert e1 == e2 and _rows(r1) == _rows(r2)


@pytest.mark.parametrize("s,exp", [
    (b"  a b \n", b"a b"), (b"\xc2\xa0x\xc2\xa0", b"x"), (b"x\xa0", b"x\xa0"), (b"\xe2\x80\x80", b""),
    (b"\x85x", b"\x85x"), (b"a\xc2\x85", b"a"), (b"\v\fz\r\n", b"z"), (b"", b""),
])
def test_trim_space(oracle_lib, s, exp):
    assert pyref.trim_space(s) == exp
    assert oracle_lib.trim_space(s) == exp
