"""CPU: the C-ABI library builds, loads and exports every symbol include/shockidx.h declares.
No compute call is made (no GPU here)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "shockidx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(shockidx_[a-z_]+)\s*\(", src)))


def test_header_declares_expected():
    names = _declared()
    for n in ("shockidx_ctx_create", "shockidx_build_device", "shockidx_build_host", "shockidx_build_fd",
              "shockidx_create", "shockidx_write_idx", "shockidx_detect", "shockidx_free"):
        assert n in names


def test_library_exports_every_declared_symbol(shockidx_so):
    out = subprocess.run(["nm", "-D", "--defined-only", shockidx_so], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (shockidx_\w+)", out))
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(shockidx_so)
    for n in _declared():
        assert getattr(lib, n)


def test_abi_version_and_strerror(shockidx_so):
    from shock_amd import _lib
    L = _lib.lib()
    assert L.shockidx_abi_version() == 5
    assert L.shockidx_strerror(_lib.EFORMAT) == b"format error"


def test_gfx950_code_object(shockidx_so):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", shockidx_so], capture_output=True,
                         text=True)
    blob = open(shockidx_so, "rb").read()
    assert b"gfx950" in blob or "gfx950" in out.stdout


def test_indexer_registry_mirrors_reference():
    from shock_amd import indexer
    assert set(indexer.Indexers) == {"record", "line", "chunkrecord"}
    idx = indexer.Indexers["record"](open(__file__, "rb"), "basic", "", "")
    assert hasattr(idx, "create") and hasattr(idx, "close")
    idx.close()


def test_write_idx_protocol(shockidx_so, tmp_path):
    """record.go:35-41,65-87: LE {u64 off, u64 len} rows, temp file + rename."""
    import numpy as np
    from shock_amd.core import write_idx
    rows = np.array([[0, 16], [16, 14], [30, 2 ** 40 + 5]], dtype=np.uint64)
    tmpdir = tmp_path / "temp"
    tmpdir.mkdir()
    out = tmp_path / "record.idx"
    write_idx(rows, str(tmpdir), str(out))
    b = out.read_bytes()
    assert b == rows.astype("<u8").tobytes()
    assert list(tmpdir.iterdir()) == []
