"""shock_amd -- MI355X-native record indexing for MG-RAST/Shock.

The hot path of Shock's index build (record / line index of a node's file,
shock-server/node/file/index/{record,line}.go over the readers in
shock-server/node/file/format/) re-implemented as gfx950 HIP kernels behind a C ABI
(include/shockidx.h, built as shock_amd/libshockidx.so).  This package is the host-side
mirror of the reference's plug-in interface:

    from shock_amd.indexer import Indexers
    idxer = Indexers["record"](f, n_type, "", "")
    count, fmt, err = idxer.create(out_path)       # Indexer.Create (index/index.go:30-33)

See DESIGN.md and INTEGRATION.md.
"""
from ._lib import ShockIdxError, lib  # noqa: F401
from .core import Context, IndexResult, MultiContext  # noqa: F401

__all__ = ["Context", "IndexResult", "MultiContext", "ShockIdxError", "lib"]
