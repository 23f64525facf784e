"""Pure-Python restatement of Shock's record/line indexers -- TEST INFRASTRUCTURE ONLY.

This module is the slow, line-by-line restatement of the reference Go code used to
generate and pin golden vectors (tests/golden/) and to cross-check the C restatement
(oracle/shockidx_oracle.c).  Nothing in the product path (shock_amd/, libshockidx)
may import it; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.

Parity status: the reference's own tests pin no index results, and
the reference (Go) cannot be built here (no Go toolchain).  This restatement is pinned by
the known-answer vectors of SURVEY.md Appendix B and by the fixture tables of Appendix C
(tests/golden/), i.e. "parity pinned by restatement + KATs", not by running the reference.

Every function cites the Go source (paths relative to /root/reference/shock-server/).
"""
from __future__ import annotations

import re

# --------------------------------------------------------------------------------------
# Error strings (errors/errors.go:20, node/file/format/fastq/fastq.go:156-207,
# node/file/format/fasta/fasta.go:120)
# --------------------------------------------------------------------------------------
ERR_INVALID_FILE_TYPE = b"Invalid file type for filter"
ERR_FQ_TRUNCATED = b"Invalid format: truncated fastq record"
ERR_FQ_EMPTY_LINES = b"Invalid format: empty line(s) between records"
ERR_FQ_NO_AT = b"Invalid format: id line does not start with @"
ERR_FQ_MISSING_ID = b"Invalid format: missing sequence ID"
ERR_FQ_EMPTY_SEQ = b"Invalid format: empty sequence"
ERR_FQ_NO_PLUS = b"Invalid format: plus line does not start with +"
ERR_FQ_ID_MISMATCH = b"Invalid format: quality ID does not match sequence ID"
ERR_FQ_LEN_MISMATCH = b"Invalid format: length of sequence and quality lines do not match"
ERR_FA_PREFIX = b"Invalid fasta entry: "


class GoError(Exception):
    """A non-EOF error returned by a reader (message = the Go error string)."""

    def __init__(self, msg: bytes):
        super().__init__(msg)
        self.msg = msg


# --------------------------------------------------------------------------------------
# Go stdlib pieces: unicode/utf8 DecodeRune / DecodeLastRune, unicode.IsSpace,
# bytes.TrimSpace (Go >= 1.13 semantics)
# --------------------------------------------------------------------------------------
RUNE_ERROR = 0xFFFD
_ASCII_SPACE = frozenset(b"\t\n\v\f\r ")


def _first_info(b0: int):
    """(size, lo, hi) of the accept range for lead byte b0, or None if invalid lead."""
    if 0xC2 <= b0 <= 0xDF:
        return 2, 0x80, 0xBF
    if b0 == 0xE0:
        return 3, 0xA0, 0xBF
    if 0xE1 <= b0 <= 0xEC or 0xEE <= b0 <= 0xEF:
        return 3, 0x80, 0xBF
    if b0 == 0xED:
        return 3, 0x80, 0x9F
    if b0 == 0xF0:
        return 4, 0x90, 0xBF
    if 0xF1 <= b0 <= 0xF3:
        return 4, 0x80, 0xBF
    if b0 == 0xF4:
        return 4, 0x80, 0x8F
    return None


def decode_rune(p: bytes):
    """Go unicode/utf8.DecodeRune."""
    n = len(p)
    if n < 1:
        return RUNE_ERROR, 0
    p0 = p[0]
    if p0 < 0x80:
        return p0, 1
    info = _first_info(p0)
    if info is None:
        return RUNE_ERROR, 1
    sz, lo, hi = info
    if n < sz:
        return RUNE_ERROR, 1
    b1 = p[1]
    if b1 < lo or hi < b1:
        return RUNE_ERROR, 1
    if sz == 2:
        return ((p0 & 0x1F) << 6) | (b1 & 0x3F), 2
    b2 = p[2]
    if b2 < 0x80 or 0xBF < b2:
        return RUNE_ERROR, 1
    if sz == 3:
        return ((p0 & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (b2 & 0x3F), 3
    b3 = p[3]
    if b3 < 0x80 or 0xBF < b3:
        return RUNE_ERROR, 1
    return ((p0 & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((b2 & 0x3F) << 6) | (b3 & 0x3F), 4


def decode_last_rune(p: bytes):
    """Go unicode/utf8.DecodeLastRune."""
    end = len(p)
    if end == 0:
        return RUNE_ERROR, 0
    start = end - 1
    r = p[start]
    if r < 0x80:
        return r, 1
    lim = max(end - 4, 0)
    start -= 1
    while start >= lim:
        if (p[start] & 0xC0) != 0x80:
            break
        start -= 1
    if start < 0:
        start = 0
    r, size = decode_rune(p[start:end])
    if start + size != end:
        return RUNE_ERROR, 1
    return r, size


def is_space(r: int) -> bool:
    """Go unicode.IsSpace."""
    if r <= 0xFF:
        return r in (0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0)
    return r == 0x1680 or 0x2000 <= r <= 0x200A or r in (0x2028, 0x2029, 0x202F, 0x205F, 0x3000)


def trim_space(s: bytes) -> bytes:
    """Go bytes.TrimSpace: ASCII fast path, Unicode TrimFunc fallback on a byte >= 0x80."""
    start = 0
    n = len(s)
    while start < n:
        c = s[start]
        if c >= 0x80:
            return _trim_func_space(s[start:])
        if c not in _ASCII_SPACE:
            break
        start += 1
    stop = n
    while stop > start:
        c = s[stop - 1]
        if c >= 0x80:
            return _trim_func_space(s[start:stop])
        if c not in _ASCII_SPACE:
            break
        stop -= 1
    return s[start:stop]


def _trim_func_space(s: bytes) -> bytes:
    # TrimLeftFunc
    i = 0
    while i < len(s):
        r, w = decode_rune(s[i:])
        if not is_space(r):
            break
        i += w
    s = s[i:]
    # TrimRightFunc (lastIndexFunc + forward width of the rune found)
    i = len(s)
    found = -1
    while i > 0:
        r, size = s[i - 1], 1
        if r >= 0x80:
            r, size = decode_last_rune(s[:i])
        i -= size
        if not is_space(r):
            found = i
            break
    if found >= 0 and s[found] >= 0x80:
        _, wid = decode_rune(s[found:])
        end = found + wid
    else:
        end = found + 1
    return s[:end]


# --------------------------------------------------------------------------------------
# bufio.Reader subset used by the readers (ReadBytes / UnreadByte), over a bytes object.
# --------------------------------------------------------------------------------------
class BufReader:
    def __init__(self, data: bytes):
        self.d = data
        self.p = 0

    def read_bytes(self, delim: int):
        """Returns (bytes, eof).  Mirrors bufio.Reader.ReadBytes: on EOF returns the rest."""
        i = self.d.find(bytes([delim]), self.p)
        if i < 0:
            b = self.d[self.p:]
            self.p = len(self.d)
            return b, True
        b = self.d[self.p:i + 1]
        self.p = i + 1
        return b, False

    def unread_byte(self):
        self.p -= 1


# --------------------------------------------------------------------------------------
# Readers: GetReadOffset() -> (n, eof) or raise GoError
# --------------------------------------------------------------------------------------
class FastqReader:
    """node/file/format/fastq/fastq.go:134-213 (GetReadOffset)."""

    def __init__(self, data: bytes):
        self.r = BufReader(data)

    def get_read_offset(self):
        r = self.r
        curr = 0
        empty = False
        while True:  # :143-152 skip empty lines
            seq_id, eof = r.read_bytes(0x0A)
            if eof:
                break
            if len(seq_id) > 1:
                break
            empty = True
        if eof:  # :154-158
            if len(seq_id) > 0:
                raise GoError(ERR_FQ_TRUNCATED)
            return 0, True
        if empty:  # :161-163
            raise GoError(ERR_FQ_EMPTY_LINES)
        if seq_id[:1] != b"@":  # :164-166
            raise GoError(ERR_FQ_NO_AT)
        if len(seq_id) == 2:  # :167-169
            raise GoError(ERR_FQ_MISSING_ID)
        curr += len(seq_id)
        seq_body, eof = r.read_bytes(0x0A)  # :173-182
        if eof:
            raise GoError(ERR_FQ_TRUNCATED)
        if len(seq_body) == 1:
            raise GoError(ERR_FQ_EMPTY_SEQ)
        curr += len(seq_body)
        qual_id, eof = r.read_bytes(0x0A)  # :185-199
        if eof:
            raise GoError(ERR_FQ_TRUNCATED)
        if qual_id[:1] != b"+":
            raise GoError(ERR_FQ_NO_PLUS)
        qt = trim_space(qual_id)
        if len(qt) > 1 and trim_space(seq_id[1:]) != qt[1:]:
            raise GoError(ERR_FQ_ID_MISMATCH)
        curr += len(qual_id)
        qual_body, eof = r.read_bytes(0x0A)  # :202-209
        if len(trim_space(seq_body)) != len(trim_space(qual_body)):
            raise GoError(ERR_FQ_LEN_MISMATCH)
        return curr + len(qual_body), eof  # :211


class FastaReader:
    """node/file/format/fasta/fasta.go:93-140 (GetReadOffset)."""

    def __init__(self, data: bytes):
        self.r = BufReader(data)

    def get_read_offset(self):
        r = self.r
        n = 0
        while True:
            read, eof = r.read_bytes(0x3E)
            if len(read) > 1 and b"\n" in read:  # :111
                core = trim_space(read.rstrip(b">"))
                lines = core.split(b"\n")
                if len(b"".join(lines[1:])) == 0:  # :113-121
                    raise GoError(ERR_FA_PREFIX + read[:50])
                if eof:  # :123-125
                    return n + len(read), True
                r.unread_byte()  # :126-128
                return n + len(read) - 1, False
            n += len(read)  # :131-132
            if eof:  # :134-136
                return n, True


class SamReader:
    """node/file/format/sam/sam.go:83-98 (GetReadOffset)."""

    def __init__(self, data: bytes):
        self.r = BufReader(data)

    def get_read_offset(self):
        n = 0
        while True:
            read, eof = self.r.read_bytes(0x0A)
            n += len(read)
            if len(read) > 1:
                if read[0] == 0x40:  # '@'
                    continue
                return n, False  # err stays nil even at EOF (sam.go:92-93)
            elif eof:
                return n, True


class LineReader:
    """node/file/format/line/line.go:37-45."""

    def __init__(self, data: bytes):
        self.r = BufReader(data)

    def get_read_offset(self):
        p, eof = self.r.read_bytes(0x0A)
        return len(p), eof


# --------------------------------------------------------------------------------------
# Format detection (node/file/format/multi/multi.go:43-62) with the three regexes
# translated to explicit RE2 classes: Go \s = [\t\n\f\r ] (no \v!), so \S = [^\t\n\f\r ].
# --------------------------------------------------------------------------------------
_S = rb"[^\t\n\f\r ]"
_SST = rb"[^\n\f\r]"  # [\S\t ]  (and [\S \t])
# `\S+[\S\t ]*` is rewritten to the equivalent `\S[\S\t ]*` (\S is a subset of [\S\t ]) so
# that Python's backtracking engine stays linear on the zero-padded 32 KiB buffer.
FASTA_RE = re.compile(rb"^[\n\r]*>" + _S + _SST + rb"*[\n\r]+[A-Za-z\- ]")  # fasta.go:22
FASTQ_RE = re.compile(rb"^[\n\r]*@" + _S + _SST + rb"*[\n\r]+[A-Za-z\-]+[\n\r]+\+"
                      + _SST + rb"*[\n\r]+" + _S + rb"*[\n\r]")  # fastq.go:22
SAM_RE = re.compile(rb"^[\n\r]*[@\[A-Z][A-Z][ \t]" + _SST + rb"+[\n\r]")  # sam.go:17

# Go ranges over a map (random order, multi.go:54); we fix the source order fasta, fastq, sam.
DETECT_ORDER = (("fasta", FASTA_RE), ("fastq", FASTQ_RE), ("sam", SAM_RE))


def detect_format(data: bytes):
    """Returns 'fasta' | 'fastq' | 'sam' | None (None -> ERR_INVALID_FILE_TYPE)."""
    buf = data[:32768]
    buf = buf + b"\x00" * (32768 - len(buf))  # zero padding of make([]byte, 32768)
    for name, rx in DETECT_ORDER:
        if rx.match(buf):
            return name
    return None


def detect_all(data: bytes):
    buf = data[:32768]
    buf = buf + b"\x00" * (32768 - len(buf))
    return [name for name, rx in DETECT_ORDER if rx.match(buf)]


READERS = {"fasta": FastaReader, "fastq": FastqReader, "sam": SamReader}


# --------------------------------------------------------------------------------------
# Drivers
# --------------------------------------------------------------------------------------
def record_index(data: bytes, fmt: str | None = None):
    """index/record.go:34-90 over multi.NewReader (fmt=None -> auto-detect like multi.go).

    Returns (rows, err): rows = list of (offset, length); err = None or bytes message.
    On error, rows holds the records emitted before the error (the Go driver's `count`).
    """
    if fmt is None:
        fmt = detect_format(data)
        if fmt is None:
            return [], ERR_INVALID_FILE_TYPE
    rd = READERS[fmt](data)
    rows = []
    curr = 0
    while True:
        try:
            n, eof = rd.get_read_offset()
        except GoError as e:
            return rows, e.msg
        if eof and n == 0:
            break
        rows.append((curr, n))
        curr += n
        if eof:
            break
    return rows, None


def line_index(data: bytes):
    """index/line.go:33-85 -- note: no `eof && n == 0` break, final entry always emitted."""
    rd = LineReader(data)
    rows = []
    curr = 0
    while True:
        n, eof = rd.get_read_offset()
        rows.append((curr, n))
        curr += n
        if eof:
            break
    return rows, None


def rows_to_idx(rows) -> bytes:
    """record.go:74-75: little-endian u64 offset, u64 length, no header."""
    import struct
    return b"".join(struct.pack("<QQ", o, n) for o, n in rows)
