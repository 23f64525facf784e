"""Seeded generators of FASTQ / FASTA / SAM / line inputs with the edge cases the reference
readers care about (tile- and slab-crossing records, long lines, CRLF, blank lines, embedded
'>', '@' in quality strings, Unicode whitespace, missing final newline, corrupt records)."""
from __future__ import annotations

import random

ALNUM = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789._:|-"
UNI_SPACES = [b"\xc2\xa0", b"\xc2\x85", b"\xe2\x80\x80", b"\xe3\x80\x80", b"\xe2\x80\xa8"]


def _word(rng, lo, hi):
    return bytes(rng.choice(ALNUM) for _ in range(rng.randint(lo, hi)))


def _seq(rng, n, alphabet=b"ACGT"):
    return bytes(rng.choice(alphabet) for _ in range(n))


def _big_seq(rng, n, alphabet=b"ACGT"):
    # fast long sequence: repeat a random block
    blk = _seq(rng, 257, alphabet)
    return (blk * (n // 257 + 1))[:n]


def fastq(rng: random.Random, nrec: int, *, long_every=0, long_len=70000, crlf=0.0, plus_id=0.1,
          at_qual=0.05, trail_blank=0, final_nl=True, uni=0.0) -> bytes:
    out = []
    for i in range(nrec):
        rid = b"r" + str(i).encode() + b" " + _word(rng, 0, 12)
        if long_every and i % long_every == long_every - 1:
            L = rng.randint(long_len // 2, long_len)
            s = _big_seq(rng, L)
            q = _big_seq(rng, L, b"!#$%&'()*+ABCDEFGHIJ")
        else:
            L = rng.randint(1, 300)
            s = _seq(rng, L, b"ACGTN")
            q = bytes(rng.randint(33, 74) for _ in range(L))
        if rng.random() < at_qual:
            q = b"@" + q[1:]
        eol = b"\r\n" if rng.random() < crlf else b"\n"
        if rng.random() < uni:
            s = s + rng.choice(UNI_SPACES)
        plus = b"+" + rid if rng.random() < plus_id else b"+"
        out.append(b"@" + rid + eol + s + eol + plus + eol + q + eol)
    data = b"".join(out)
    if not final_nl and data.endswith(b"\n"):
        data = data[:-1]
        if data.endswith(b"\r"):
            data = data[:-1]
    return data + b"\n" * trail_blank


FASTQ_CORRUPTIONS = ("no_at", "empty_seq", "no_plus", "id_mismatch", "len_mismatch", "blank_between",
                     "truncate", "missing_id", "blank_lead", "trail_partial")


def fastq_corrupt(rng: random.Random, data: bytes, kind: str) -> bytes:
    """Corrupt one record of a well-formed FASTQ (records start at every 4th line)."""
    lines = data.split(b"\n")
    nrec = (len(lines) - 1) // 4
    if nrec == 0:
        return data
    r = rng.randrange(nrec)
    b = 4 * r
    if kind == "no_at":
        lines[b] = b"X" + lines[b][1:]
    elif kind == "empty_seq":
        lines[b + 1] = b""
    elif kind == "no_plus":
        lines[b + 2] = b"-" + lines[b + 2][1:]
    elif kind == "id_mismatch":
        lines[b + 2] = b"+zz" + lines[b][1:]
    elif kind == "len_mismatch":
        lines[b + 3] = lines[b + 3] + b"I"
    elif kind == "blank_between":
        lines.insert(b, b"")
    elif kind == "truncate":
        return b"\n".join(lines[:b + rng.randint(1, 3)])
    elif kind == "missing_id":
        lines[b] = b"@"
    elif kind == "blank_lead":
        return b"\n" + data
    elif kind == "trail_partial":
        return data + b"\n\nXY"
    return b"\n".join(lines)


def fasta(rng: random.Random, nrec: int, *, long_every=0, long_len=150000, crlf=0.0, embedded_gt=0.05,
          blank=0.05, final_nl=True, uni=0.0, lead=b"") -> bytes:
    out = [lead]
    for i in range(nrec):
        eol = b"\r\n" if rng.random() < crlf else b"\n"
        hdr = b">ctg" + str(i).encode() + b" " + _word(rng, 0, 20)
        if rng.random() < embedded_gt:
            hdr += b" a>b"
        if long_every and i % long_every == long_every - 1:
            L = rng.randint(long_len // 2, long_len)
            body = _big_seq(rng, L)
        else:
            L = rng.randint(1, 3000)
            body = _seq(rng, L, b"ACGTNacgt")
        w = rng.choice((60, 70, 80, 1000000))
        seq_lines = [body[k:k + w] for k in range(0, len(body), w)]
        rec = hdr + eol + eol.join(seq_lines) + eol
        if rng.random() < blank:
            rec += eol
        if rng.random() < uni:
            rec = rec[:-len(eol)] + rng.choice(UNI_SPACES) + eol
        out.append(rec)
    data = b"".join(out)
    if not final_nl:
        data = data.rstrip(b"\r\n")
    return data


def fasta_corrupt(rng: random.Random, data: bytes, kind: str) -> bytes:
    idx = [i for i in range(len(data)) if data[i] == 0x3E]
    if not idx:
        return data
    g = rng.choice(idx)
    if kind == "header_only":   # drop the sequence lines of one record
        nxt = data.find(b"\n", g)
        end = data.find(b">", nxt) if nxt >= 0 else -1
        if nxt < 0 or end < 0:
            return data + b">x\n"
        return data[:nxt + 1] + data[end:]
    if kind == "gt_in_seq":     # '>' inside a sequence line
        nl = data.find(b"\n", g)
        if nl < 0 or nl + 3 >= len(data):
            return data
        return data[:nl + 2] + b">" + data[nl + 2:]
    if kind == "lead_newline":
        return b"\n" + data
    if kind == "trail_header":
        return data + (b"" if data.endswith(b"\n") else b"\n") + b">last\n"
    return data


def sam(rng: random.Random, nrec: int, *, headers=5, blank=0.05, final_nl=True) -> bytes:
    out = [b"@HD\tVN:1.6\tSO:unsorted\n"]
    for i in range(headers):
        out.append(b"@SQ\tSN:chr" + str(i).encode() + b"\tLN:" + str(rng.randint(1000, 10 ** 8)).encode() + b"\n")
    for i in range(nrec):
        if rng.random() < blank:
            out.append(b"\n")
        if rng.random() < 0.02:
            out.append(b"@CO\tcomment " + _word(rng, 0, 30) + b"\n")
        L = rng.randint(20, 250)
        fields = [b"read" + str(i).encode(), b"0", b"chr1", str(rng.randint(1, 10 ** 6)).encode(), b"60",
                  str(L).encode() + b"M", b"*", b"0", b"0", _seq(rng, L), bytes(rng.randint(33, 74) for _ in range(L))]
        out.append(b"\t".join(fields) + b"\n")
    data = b"".join(out)
    return data if final_nl else data.rstrip(b"\n")


def lines(rng: random.Random, nlines: int, *, long_every=0, long_len=100000, empty=0.1, final_nl=True) -> bytes:
    out = []
    for i in range(nlines):
        if long_every and i % long_every == long_every - 1:
            out.append(_big_seq(rng, rng.randint(long_len // 2, long_len), b"xyz ") + b"\n")
        elif rng.random() < empty:
            out.append(b"\n")
        else:
            out.append(_word(rng, 1, 120) + b"\n")
    data = b"".join(out)
    return data if final_nl else data[:-1]


ALPH = [b"\n", b"\r", b">", b"@", b"+", b" ", b"\t", b"A", b"C", b"x", b"\xc2\xa0", b"\xc2\x85",
        b"\xe2\x80\x80", b"\x85", b"\xc2", b"\v", b"\f", b"I", b"[", b"H", b"D"]


def tiny(rng: random.Random) -> bytes:
    """Small adversarial inputs (random tokens, FASTQ-ish, FASTA-ish)."""
    c = rng.randrange(3)
    if c == 0:
        return b"".join(rng.choice(ALPH) for _ in range(rng.randint(0, 40)))
    if c == 1:
        recs = []
        for _ in range(rng.randint(0, 5)):
            sid = b"".join(rng.choice(ALPH) for _ in range(rng.randint(0, 4)))
            seq = b"".join(rng.choice(ALPH) for _ in range(rng.randint(0, 5)))
            q = b"".join(rng.choice(ALPH) for _ in range(rng.randint(0, 5)))
            plus = rng.choice([b"+", b"+" + sid, b"+ " + sid, b"".join(rng.choice(ALPH) for _ in range(2))])
            recs.append(b"@" + sid + b"\n" + seq + b"\n" + plus + b"\n" + q + rng.choice([b"\n", b"", b"\n\n"]))
        return b"".join(recs)
    return b"".join(rng.choice([b">", b"\n", b">a\n", b"AC", b" ", b"\r\n", b"\xc2\xa0", b"x>y"])
                    for _ in range(rng.randint(0, 14)))
