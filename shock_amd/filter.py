"""Host-side mirror of Shock's download filters, backed by libshockidx.

Reference interface (paths relative to /root/reference/shock-server/):
    node/filter/filter.go:11-32             type FilterFunc func(file.SectionReader) io.Reader;
                                            filters = {"anonymize", "fq2fa"}; Has, Filter, NewReader
    node/filter/fq2fa/fq2fa.go:18-84        fq2fa.NewReader / Reader.Read
    node/filter/anonymize/anonymize.go:20-56  anonymize.NewReader / Reader.Read
    caller: request/streamer.go:80-95 (io.Copy of each section through the filter)

Same names and behaviour: NewReader(name, section) returns a reader whose read() yields the
filtered stream of one section (a path, a bytes-like object or a binary file object) and
raises ShockIndexError (Go's text) once the bytes delivered before a reader error are
consumed -- what io.Copy sees.  The transform runs on the device (shockidx_filter_device):
the section is staged into HBM, indexed, and formatted record-parallel.
"""
from __future__ import annotations

from . import _lib as L
from .indexer import ShockIndexError, context

FILTERS = ("anonymize", "fq2fa")


def Has(f: str) -> bool:  # noqa: N802  (filter.go:20-25)
    return f in FILTERS


def Filter(f: str):  # noqa: N802  (filter.go:27-29): the FilterFunc, None when unknown
    return (lambda section: NewReader(f, section)) if Has(f) else None


class FilterReader:
    """io.Reader over the filtered section: bytes first, then the reader's error (if any)."""

    def __init__(self, out: bytes, err: bytes | None):
        self._out = out
        self._pos = 0
        self._err = err

    def read(self, n: int = -1) -> bytes:
        if self._pos >= len(self._out):
            if self._err is not None:
                raise ShockIndexError(self._err)
            return b""
        end = len(self._out) if n is None or n < 0 else min(len(self._out), self._pos + n)
        b = self._out[self._pos:end]
        self._pos = end
        return b

    def close(self):
        return None


def _section_bytes(section) -> bytes:
    if isinstance(section, (bytes, bytearray, memoryview)):
        return bytes(section)
    if hasattr(section, "read"):
        return section.read()
    with open(section, "rb") as f:
        return f.read()


def NewReader(f: str, section) -> FilterReader:  # noqa: N802  (filter.go:31-33)
    if not Has(f):
        raise KeyError(f)
    r = context().filter_host(f, _section_bytes(section))
    if r.status not in (L.OK, L.EFORMAT):
        raise RuntimeError(f"shockidx_filter_device: {r.status} {r.err!r}")
    return FilterReader(r.gathered or b"", r.err if r.status == L.EFORMAT else None)
