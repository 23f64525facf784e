"""CPU: ?filter=anonymize over FASTA and SAM sections (anonymize.go:28-56 through
multi.Reader): the C oracle against known answers read off fasta.go:40-88 / sam.go:44-81 and
their Format functions, and against a literal Python transcription of those loops on random
sections.  Where Go's fasta Read loops forever (an EOF read without '\\n') both end the stream."""
import random

import pytest

import oracle


def trim_space(b: bytes) -> bytes:
    """bytes.TrimSpace for the ASCII inputs used here."""
    return b.strip(b" \t\n\v\f\r")


class Reader:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def read_bytes(self, delim: bytes):
        i = self.d.find(delim, self.p)
        if i < 0:
            out, self.p = self.d[self.p:], len(self.d)
            return out, True
        out, self.p = self.d[self.p:i + 1], i + 1
        return out, False


def fasta_read(r: Reader):
    """fasta.go:40-88; returns ("ok", label, body) | ("eof",) | ("err",)."""
    prev = b""
    while True:
        read, eof = r.read_bytes(b">")
        if prev:
            read = prev + read
        if len(read) == 1:
            if eof:
                return ("eof",)
            continue
        if b"\n" not in read:
            if eof:
                return ("eof",)  # Go: endless loop
            prev = read
            continue
        t = trim_space(read.rstrip(b">"))
        lines = t.split(b"\n")
        label = body = b""
        if len(lines) > 1:
            label, body = lines[0], b"".join(lines[1:])
        if eof:
            return ("eof",)
        return ("ok", label, body) if label and body else ("err",)


def sam_read(r: Reader):
    while True:
        line, eof = r.read_bytes(b"\n")
        if eof:
            return ("eof",)
        if line and line[-1:] == b"\r":
            line = line[:-1]
        line = trim_space(line)
        if not line or line[:1] == b"@":
            continue
        if len(line.split(b"\t")) < 11:
            return ("err",)
        return ("ok", line.split(b"\t")[0], line)


def anonymize(data: bytes, fmt: str):
    r, out, k = Reader(data), [], 0
    while True:
        s = fasta_read(r) if fmt == "fasta" else sam_read(r)
        if s[0] == "eof":
            return b"".join(out), k, None
        if s[0] == "err":
            return b"".join(out), k, (b"Invalid fasta entry" if fmt == "fasta" else b"sam alignment fields less than 11")
        k += 1
        out.append(b">%d\n%s\n" % (k, s[2]) if fmt == "fasta" else s[2] + b"\n")


FASTA_KATS = [
    (b">a\nAC\n>b\nGG\n", b">1\nAC\n", None),
    (b">a\nAC\nGT\n>b x\nG\n>c\nTT", b">1\nACGT\n>2\nG\n", None),
    (b">a\nAC\n>b\n>c\nA\n", b">1\nAC\n", b"Invalid fasta entry"),
    (b">a x>y\nAC\n>b\nGG\n", b">1\nAC\n", None),
    (b">h>\nAC\n>b\nG\n>c\n", b">1\nAC\n>2\nG\n", None),
    (b">a\r\nAC\r\nGT\r\n>b\r\n", b">1\nAC\rGT\n", None),
    (b">>a\nAC\n>b\nC\n", b">1\nAC\n", None),
    (b">a\nAC\n>", b">1\nAC\n", None),
    (b">a\nAC\n>b", b">1\nAC\n", None),
]

SAM_HEAD = b"@A x\n"  # sam.go:17 needs [@A-Z[][A-Z][ \t]+ at the head ("@HD\t" does not match)
ALN = b"r1\t0\tchr1\t1\t60\t4M\t*\t0\t0\tACGT\tIIII"
SAM_KATS = [
    (SAM_HEAD + ALN + b"\n" + ALN + b"\n", ALN + b"\n" + ALN + b"\n", None),
    (SAM_HEAD + ALN + b"\n\n @x\n" + ALN, ALN + b"\n", None),
    (SAM_HEAD + ALN + b"\r\n" + b"r2\t0\t*\n" + ALN + b"\n", ALN + b"\n", b"sam alignment fields less than 11"),
    (SAM_HEAD + b"  " + ALN + b" \t\n", ALN + b"\n", None),
]


@pytest.mark.parametrize("data,exp,err", FASTA_KATS + SAM_KATS)
def test_kats(data, exp, err):
    fmt = "fasta" if data[:1] == b">" else "sam"
    assert oracle.detect(data)[0] == fmt
    out, k, e = anonymize(data, fmt)
    assert (out, e) == (exp, err)
    got, gk, ge = oracle.filter_fastq(data, "anonymize")
    assert (got, gk, ge) == (exp, k, err)


def _fasta_corpus(rng):
    parts = []
    for i in range(rng.randint(0, 40)):
        nl = b"\r\n" if rng.random() < 0.2 else b"\n"
        head = b">" * rng.choice([1, 1, 1, 2]) + b"s%d" % i + (b" d>x" if rng.random() < 0.2 else b"")
        if rng.random() < 0.1:
            head += b">"
        body = nl.join(bytes(rng.choice(b"ACGT ") for _ in range(rng.randint(0, 90))) for _ in range(rng.randint(0, 4)))
        parts.append(head + nl + body + (nl if rng.random() < 0.9 else b""))
    return b">x\nA\n" + b"".join(parts)


def _sam_corpus(rng):
    lines = [SAM_HEAD]
    for i in range(rng.randint(0, 40)):
        c = rng.random()
        if c < 0.1:
            lines.append(b"@CO\tx\n")
        elif c < 0.2:
            lines.append(b" \n")
        elif c < 0.25:
            lines.append(b"r%d\t0\t*\n" % i)
        else:
            lines.append(b"r%d\t0\tc\t1\t60\t4M\t*\t0\t0\tACGT\tIIII" % i + (b"\r\n" if c > 0.9 else b"\n"))
    data = b"".join(lines)
    return data if rng.random() < 0.7 else data[: rng.randint(len(SAM_HEAD), len(data))]


def test_random_sections_agree():
    rng = random.Random(12)
    for _ in range(300):
        data = _fasta_corpus(rng)
        exp = anonymize(data, "fasta")
        got = oracle.filter_fastq(data, "anonymize")
        assert got == exp, data
        data = _sam_corpus(rng)
        if oracle.detect(data)[0] != "sam":
            continue
        assert oracle.filter_fastq(data, "anonymize") == anonymize(data, "sam"), data
