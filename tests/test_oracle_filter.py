"""CPU: the fq2fa / anonymize restatement (oracle/filter_oracle.c) over FASTQ sections.

Reference: shock-server/node/filter/fq2fa/fq2fa.go:58-84, anonymize/anonymize.go:28-56 and
fastq.Reader.Read (node/file/format/fastq/fastq.go:50-132).  The reference holds no tests for
the filters, so parity is unpinned by reference-held outputs: the C oracle is checked against
known answers read off the Go code (cited per case) and against `go_filter` below, a literal
transcription of fastq.Reader.Read + the filter loops, on seeded inputs with CRLF, plus-line
IDs, Unicode spaces, corruptions and missing final newlines.
"""
import random

import pytest

import gen

ASCII_SPACE = b" \t\n\v\f\r"
UNI = (b"\xc2\x85", b"\xc2\xa0")  # the Unicode spaces gen.py can put at an edge besides >U+00FF ones


def _trim(b: bytes) -> bytes:
    """bytes.TrimSpace for the inputs gen.py makes (ASCII + Unicode spaces of UNI_SPACES)."""
    spaces = [bytes([c]) for c in ASCII_SPACE] + list(gen.UNI_SPACES)
    changed = True
    while changed and b:
        changed = False
        for s in spaces:
            if b.startswith(s):
                b, changed = b[len(s):], True
            if b.endswith(s):
                b, changed = b[:-len(s)], True
    return b


def go_filter(data: bytes, name: str):
    pos = 0
    out = []
    k = 0

    def read_bytes():
        nonlocal pos
        j = data.find(b"\n", pos)
        if j < 0:
            s, pos = data[pos:], len(data)
            return s, True
        s, pos = data[pos:j + 1], j + 1
        return s, False

    while True:
        empty = False
        while True:  # fastq.go:56-66
            seq_id, eof = read_bytes()
            if eof or len(seq_id) > 1:
                break
            empty = True
        if eof:
            if seq_id:
                return b"".join(out), k, b"Invalid format: truncated fastq record"
            return b"".join(out), k, None
        if empty:
            return b"".join(out), k, b"Invalid format: empty line(s) between records"
        if not seq_id.startswith(b"@"):
            return b"".join(out), k, b"Invalid format: id line does not start with @"
        seq_id = _trim(seq_id[1:])
        if not seq_id:
            return b"".join(out), k, b"Invalid format: missing sequence ID"
        body, eof = read_bytes()
        if eof:
            return b"".join(out), k, b"Invalid format: truncated fastq record"
        body = _trim(body)
        if not body:
            return b"".join(out), k, b"Invalid format: empty sequence"
        qid, eof = read_bytes()
        if eof:
            return b"".join(out), k, b"Invalid format: truncated fastq record"
        if not qid.startswith(b"+"):
            return b"".join(out), k, b"Invalid format: plus line does not start with +"
        qid = _trim(qid)
        if len(qid) > 1 and seq_id != qid[1:]:
            return b"".join(out), k, b"Invalid format: quality ID does not match sequence ID"
        qual, eof = read_bytes()
        qual = _trim(qual)
        if len(body) != len(qual):
            return b"".join(out), k, b"Invalid format: length of sequence and quality lines do not match"
        if eof:  # Read returned (seq, io.EOF): the filter loop breaks before formatting it
            return b"".join(out), k, None
        k += 1
        if name == "fq2fa":
            out.append(b">" + seq_id + b"\n" + body + b"\n")
        else:
            out.append(b"@" + str(k).encode() + b"\n" + body + b"\n+\n" + qual + b"\n")


@pytest.mark.parametrize("name", ["fq2fa", "anonymize"])
@pytest.mark.parametrize("data,exp_n,exp_err", [
    (b"@r1 x\nACGT\n+\nIIII\n@r2\nAC\n+r2\nII\n", 2, None),
    (b"@r1\nAC\n+\nII", 0, None),                                      # :117-121 EOF record dropped
    (b"@r1\nAC\n+\nII\n@r2\nA\n+\nI", 1, None),
    (b"@ \nAC\n+\nII\n", 0, b"Invalid format: missing sequence ID"),    # :83-87 after TrimSpace
    (b"@r1\n \n+\nI\n", 0, b"Invalid format: empty sequence"),           # :96-100 after TrimSpace
    (b"@r1\r\nAC\r\n+r1\r\nII\r\n", 1, None),                           # CRLF trimmed
    (b"@r1\nAC\n+\nII\n\n\n", 1, None),                                 # blank lines at EOF
    (b"@r1\nAC\n+\nII\n\n@r2\nA\n+\nI\n", 1, b"Invalid format: empty line(s) between records"),
    (b"@r1\nAC\n+r2\nII\n", 0, b"Invalid format: quality ID does not match sequence ID"),
    (b"", 0, None),
])
def test_filter_kats(oracle_lib, name, data, exp_n, exp_err):
    out, n, err = oracle_lib.filter_fastq(data, name)
    if name == "anonymize" and oracle_lib.detect(data)[0] is None:  # multi.go:61 DetermineFormat fails
        assert (out, n, err) == (b"", 0, b"Invalid file type for filter")
        return
    assert (n, err) == (exp_n, exp_err)
    assert (out, n, err) == go_filter(data, name)


def test_filter_formats(oracle_lib):
    d = b"@r1 x\nACGT\n+\nIIII\n@r2\nAC\n+r2\nII\n"
    assert oracle_lib.filter_fastq(d, "fq2fa")[0] == b">r1 x\nACGT\n>r2\nAC\n"            # fasta.go:216-218
    assert oracle_lib.filter_fastq(d, "anonymize")[0] == b"@1\nACGT\n+\nIIII\n@2\nAC\n+\nII\n"  # fastq.go:283-285


@pytest.mark.parametrize("seed", range(12))
def test_filter_random(oracle_lib, seed):
    rng = random.Random(seed)
    data = gen.fastq(rng, rng.randint(1, 300), crlf=0.2 if seed % 3 == 0 else 0.0, plus_id=0.3,
                     final_nl=seed % 4 != 1, uni=0.1 if seed % 5 == 2 else 0.0)
    if seed % 2:
        data = gen.fastq_corrupt(rng, data, rng.choice(gen.FASTQ_CORRUPTIONS))
    for name in ("fq2fa", "anonymize"):
        if name == "anonymize" and oracle_lib.detect(data)[0] != "fastq":
            continue
        assert oracle_lib.filter_fastq(data, name) == go_filter(data, name)
