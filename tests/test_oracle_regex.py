"""CPU: the detector restatements against the reference's own labelled regex corpora.

tests/golden/regex_corpora.json holds the `valid` / `invalid` strings of
shock-server/node/file/format/fastq/fastq_test.go:19-72 and fasta/fasta_test.go:19-169
(extracted by tests/golden/make_regex_corpora.py).  The reference's TestRegex prints
Regex.MatchString(s) for each; the labels are its authors' expectations.  These are the only
reference-held expectations on this path, so they pin the hand-written matchers of
fasta.go:22 / fastq.go:22 / sam.go:17 (oracle/shockidx_oracle.c, oracle/pyref.py, and on the
GPU k_detect, tests/test_gpu_parity.py::test_regex_corpora_gpu).

Two entries carry a label that the regex itself contradicts (Go RE2 would print the same
as we do; recorded in DESIGN.md §5):
  fasta_valid_2   "> S1 rank=..." -- fasta.go:22 needs \\S right after '>' (label: valid, no match)
  fasta_invalid_4 "$%#%" inside a sequence line -- the regex inspects only the first
                  sequence character (label: invalid, matches)
"""
import json
import os
import re

import pytest

import pyref

HERE = os.path.dirname(os.path.abspath(__file__))
CORPORA = json.load(open(os.path.join(HERE, "golden", "regex_corpora.json")))["entries"]

# The three regexes exactly as written in the Go source, Go's \s = [\t\n\f\r ] (RE2, no \v),
# translated to Python byte regexes.  re.match = anchored at 0, unanchored end = MatchString.
_S, _SST = rb"[^\t\n\f\r ]", rb"[^\n\f\r]"  # \S and [\S\t ]
FULL = {
    "fasta": re.compile(rb"^[\n\r]*>" + _S + rb"+" + _SST + rb"*[\n\r]+[A-Za-z\- ]+"),         # fasta.go:22
    "fastq": re.compile(rb"^[\n\r]*@" + _S + rb"+" + _SST + rb"*[\n\r]+[A-Za-z\-]+[\n\r]+\+"    # fastq.go:22
                        + _SST + rb"*[\n\r]+" + _S + rb"*[\n\r]+"),
    "sam": re.compile(rb"^[\n\r]*[@\[A-Z][A-Z][ \t]+" + _SST + rb"+[\n\r]\]*"),                 # sam.go:17
}
LABEL_CONTRADICTED = {"fasta_valid_2", "fasta_invalid_4"}


def _names(mask):
    return [n for i, n in enumerate(("fasta", "fastq", "sam")) if mask >> i & 1]


@pytest.mark.parametrize("e", CORPORA, ids=lambda e: e["id"])
def test_regex_corpus_matchstring(oracle_lib, e):
    """MatchString semantics (the reference test's own call): oracle == the literal regex."""
    s = bytes.fromhex(e["text_hex"])
    full = [n for n in ("fasta", "fastq", "sam") if FULL[n].match(s)]
    assert oracle_lib.regex_match(s) == full
    matched = e["regex"] in full
    assert matched == (e["label"] == "valid") or e["id"] in LABEL_CONTRADICTED
    assert (e["id"] in LABEL_CONTRADICTED) == (matched != (e["label"] == "valid"))


@pytest.mark.parametrize("e", CORPORA, ids=lambda e: e["id"])
def test_regex_corpus_detect(oracle_lib, e):
    """DetermineFormat semantics (multi.go:43-62: 32 KiB zero-padded head): C oracle, the
    Python restatement and the literal regexes over the padded buffer agree."""
    s = bytes.fromhex(e["text_hex"])
    pad = s[:32768] + b"\x00" * (32768 - min(len(s), 32768))
    full = [n for n in ("fasta", "fastq", "sam") if FULL[n].match(pad)]
    assert _names(oracle_lib.detect(s)[1]) == full == pyref.detect_all(s)


def test_regex_corpora_complete():
    """All 17 literals of the two TestRegex functions are present."""
    ids = {e["id"] for e in CORPORA}
    assert len(ids) == 17
    assert sum(e["regex"] == "fastq" for e in CORPORA) == 6
    assert sum(e["regex"] == "fasta" for e in CORPORA) == 11
