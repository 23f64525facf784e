"""ctypes binding of libshockidx.so (include/shockidx.h) -- the product path.

The library is loaded from this package directory (built in-tree by
shock_amd/csrc/Makefile).  There is no fallback: if the shared object is missing or no GPU
is usable, calls raise ShockIdxError.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libshockidx.so")
if os.environ.get("SHOCKIDX_VARIANT"):  # profiling A/B builds (shock_amd/variants/, built by csrc/Makefile)
    LIB_PATH = os.path.join(HERE, "variants", f"libshockidx_{os.environ['SHOCKIDX_VARIANT']}.so")

RECORD, LINE = 0, 1
FMT_AUTO, FMT_NONE, FMT_FASTA, FMT_FASTQ, FMT_SAM, FMT_LINE = -1, 0, 1, 2, 3, 4
FMT_NAMES = {FMT_NONE: None, FMT_FASTA: "fasta", FMT_FASTQ: "fastq", FMT_SAM: "sam", FMT_LINE: "line"}
FMT_CODES = {"fasta": FMT_FASTA, "fastq": FMT_FASTQ, "sam": FMT_SAM, "line": FMT_LINE, None: FMT_AUTO,
             "auto": FMT_AUTO}

OK, EFORMAT, EINVAL, EHIP, ENOMEM, EIO, EINTERNAL, ESPACE = 0, 1, -1, -2, -3, -4, -5, -6

EXPORTS = ("shockidx_ctx_create", "shockidx_ctx_destroy", "shockidx_build_device",
           "shockidx_build_host", "shockidx_host_register", "shockidx_host_unregister", "shockidx_build_fd", "shockidx_create", "shockidx_write_idx",
           "shockidx_detect", "shockidx_free", "shockidx_strerror", "shockidx_abi_version",
           "shockidx_dev_alloc", "shockidx_dev_alloc_node", "shockidx_dev_free", "shockidx_memcpy_h2d", "shockidx_memcpy_d2h",
           "shockidx_memset", "shockidx_sync", "shockidx_stream", "shockidx_slab_guess",
           "shockidx_slab_index", "shockidx_slab_combine", "shockidx_comm_unique_id", "shockidx_comm_init",
           "shockidx_comm_allgather", "shockidx_comm_destroy", "shockidx_comm_count", "shockidx_subset_index", "shockidx_subset_gather",
           "shockidx_subset_node",
           "shockidx_chunkrecord_device", "shockidx_chunkrecord_fd", "shockidx_chunkrecord_subset_device", "shockidx_create_subset_index",
           "shockidx_idx_part", "shockidx_idx_range", "shockidx_filter_device", "shockidx_ctx_trim",
           "shockidx_ctx_workspace_bytes", "shockidx_ctx_set_dev_cap", "shockidx_multi_create", "shockidx_multi_destroy", "shockidx_multi_rccl",
           "shockidx_multi_build_host", "shockidx_multi_build_fd", "shockidx_multi_create_index", "shockidx_multi_plan",
           "shockidx_multi_build_resident", "shockidx_device_count")


class ShockIdxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"shockidx error {code}: {msg}")
        self.code = code
        self.msg = msg


class Result(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("format", ctypes.c_int32), ("status", ctypes.c_int32),
                ("err_len", ctypes.c_uint64), ("err", ctypes.c_char * 256),
                ("kernel_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("d2h_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("path", ctypes.c_uint32), ("reruns", ctypes.c_uint32),
                ("index_ms", ctypes.c_double), ("state_out", ctypes.c_uint64), ("term_code", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("fixups", ctypes.c_uint32), ("fix_tiles", ctypes.c_uint32)]

    @property
    def message(self) -> bytes:
        return bytes(self.err.raw[:self.err_len]) if hasattr(self.err, "raw") else bytes(self.err)[:self.err_len]


class Slab(ctypes.Structure):
    """mirrors shockidx_slab (include/shockidx.h)"""
    _fields_ = [("d_data", ctypes.c_void_p), ("n", ctypes.c_uint64), ("end", ctypes.c_uint64),
                ("front", ctypes.c_uint64), ("base", ctypes.c_uint64), ("is_first", ctypes.c_int32),
                ("is_last", ctypes.c_int32), ("seq", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class SlabSummary(ctypes.Structure):
    _fields_ = [("agg", ctypes.c_uint64), ("state_in", ctypes.c_uint64), ("key", ctypes.c_uint64),
                ("natural", ctypes.c_uint64), ("row_base", ctypes.c_uint64), ("err_pos", ctypes.c_uint64),
                ("err_len", ctypes.c_uint64), ("fmt", ctypes.c_uint16), ("flags", ctypes.c_uint16),
                ("seq", ctypes.c_uint32)]


class SlabPlan(ctypes.Structure):
    _fields_ = [("state_in", ctypes.c_uint64), ("first_record", ctypes.c_uint64), ("count", ctypes.c_uint64),
                ("err_pos", ctypes.c_uint64), ("err_len", ctypes.c_uint64), ("code", ctypes.c_uint32),
                ("err_rank", ctypes.c_int32), ("inconsistent", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class SubsetResult(ctypes.Structure):
    """mirrors shockidx_subset_result (include/shockidx.h)"""
    _fields_ = [("count", ctypes.c_uint64), ("runs", ctypes.c_uint64), ("size", ctypes.c_uint64),
                ("status", ctypes.c_int32), ("pad", ctypes.c_uint32), ("err_len", ctypes.c_uint64),
                ("err", ctypes.c_char * 256), ("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("gather_ms", ctypes.c_double)]

    @property
    def message(self) -> bytes:
        return ctypes.string_at(ctypes.addressof(self) + SubsetResult.err.offset, self.err_len)


assert ctypes.sizeof(SlabSummary) == 64
assert ctypes.sizeof(Slab) == 56

_lib = None


def lib():
    """Load libshockidx.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ShockIdxError(EINVAL, f"{LIB_PATH} not built (run __graft_entry__.build() or make -C shock_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    PRes = ctypes.POINTER(Result)
    PPu64 = ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64))
    L.shockidx_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.shockidx_ctx_create.restype = i32
    L.shockidx_ctx_destroy.argtypes = [vp]
    L.shockidx_ctx_destroy.restype = None
    L.shockidx_build_device.argtypes = [vp, vp, u64, i32, i32, vp, u64, vp, PRes]
    L.shockidx_build_device.restype = i32
    L.shockidx_chunkrecord_device.argtypes = [vp, vp, u64, i32, u64, vp, u64, PRes]
    L.shockidx_chunkrecord_device.restype = i32
    L.shockidx_chunkrecord_fd.argtypes = [vp, i32, u64, i32, u64, PPu64, PRes]
    L.shockidx_chunkrecord_fd.restype = i32
    L.shockidx_chunkrecord_subset_device.argtypes = [vp, vp, u64, vp, u64, PRes]
    L.shockidx_chunkrecord_subset_device.restype = i32
    L.shockidx_build_host.argtypes = [vp, vp, u64, i32, i32, PPu64, PRes]
    L.shockidx_build_host.restype = i32
    L.shockidx_host_register.argtypes = [vp, vp, u64]
    L.shockidx_host_register.restype = i32
    L.shockidx_host_unregister.argtypes = [vp, vp]
    L.shockidx_host_unregister.restype = i32
    L.shockidx_build_fd.argtypes = [vp, i32, u64, i32, i32, PPu64, PRes]
    L.shockidx_build_fd.restype = i32
    L.shockidx_create.argtypes = [vp, i32, u64, i32, ctypes.c_char_p, ctypes.c_char_p, PRes]
    L.shockidx_create.restype = i32
    L.shockidx_write_idx.argtypes = [ctypes.POINTER(ctypes.c_uint64), u64, ctypes.c_char_p, ctypes.c_char_p,
                                     ctypes.c_char_p, ctypes.c_size_t]
    L.shockidx_write_idx.restype = i32
    L.shockidx_detect.argtypes = [vp, vp, u64, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.shockidx_detect.restype = i32
    L.shockidx_dev_alloc.argtypes = [vp, u64, ctypes.POINTER(vp)]
    L.shockidx_dev_alloc.restype = i32
    L.shockidx_dev_alloc_node.argtypes = [vp, u64, ctypes.POINTER(vp)]
    L.shockidx_dev_alloc_node.restype = i32
    L.shockidx_dev_free.argtypes = [vp, vp]
    L.shockidx_dev_free.restype = i32
    L.shockidx_memcpy_h2d.argtypes = [vp, vp, vp, u64]
    L.shockidx_memcpy_h2d.restype = i32
    L.shockidx_memcpy_d2h.argtypes = [vp, vp, vp, u64]
    L.shockidx_memcpy_d2h.restype = i32
    L.shockidx_memset.argtypes = [vp, vp, i32, u64]
    L.shockidx_memset.restype = i32
    L.shockidx_sync.argtypes = [vp]
    L.shockidx_sync.restype = i32
    L.shockidx_stream.argtypes = [vp]
    L.shockidx_stream.restype = vp
    PSlab = ctypes.POINTER(Slab)
    L.shockidx_slab_guess.argtypes = [vp, PSlab, i32, ctypes.POINTER(u64)]
    L.shockidx_slab_index.argtypes = [vp, PSlab, i32, u64, vp, u64, vp, PRes]
    L.shockidx_slab_combine.argtypes = [vp, vp, i32, i32, i32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(SlabPlan)]
    L.shockidx_comm_unique_id.argtypes = [vp]
    L.shockidx_comm_init.argtypes = [vp, i32, i32, vp, ctypes.POINTER(vp)]
    L.shockidx_comm_allgather.argtypes = [vp, vp, vp, u64]
    L.shockidx_comm_destroy.argtypes = [vp]
    L.shockidx_comm_count.argtypes = [vp, ctypes.POINTER(i32)]
    for f in (L.shockidx_slab_guess, L.shockidx_slab_index, L.shockidx_slab_combine, L.shockidx_comm_unique_id,
              L.shockidx_comm_init, L.shockidx_comm_allgather, L.shockidx_comm_destroy, L.shockidx_comm_count):
        f.restype = i32
    Pu64 = ctypes.POINTER(ctypes.c_uint64)
    L.shockidx_multi_create.argtypes = [ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.shockidx_device_count.argtypes = []
    L.shockidx_device_count.restype = i32
    L.shockidx_multi_destroy.argtypes = [vp]
    L.shockidx_multi_destroy.restype = None
    L.shockidx_multi_rccl.argtypes = [vp]
    L.shockidx_multi_build_host.argtypes = [vp, vp, u64, i32, i32, PPu64, PRes]
    L.shockidx_multi_build_fd.argtypes = [vp, i32, u64, i32, i32, PPu64, PRes]
    L.shockidx_multi_create_index.argtypes = [vp, i32, u64, i32, ctypes.c_char_p, ctypes.c_char_p, PRes]
    L.shockidx_multi_plan.argtypes = [vp, u64, Pu64, Pu64, Pu64, Pu64]
    L.shockidx_multi_build_resident.argtypes = [vp, u64, i32, i32, ctypes.POINTER(vp), ctypes.POINTER(vp), Pu64,
                                                Pu64, Pu64, PRes]
    for f in (L.shockidx_multi_create, L.shockidx_multi_rccl, L.shockidx_multi_build_host, L.shockidx_multi_build_fd,
              L.shockidx_multi_create_index, L.shockidx_multi_plan, L.shockidx_multi_build_resident):
        f.restype = i32
    PSub = ctypes.POINTER(SubsetResult)
    L.shockidx_subset_index.argtypes = [vp, vp, u64, vp, u64, ctypes.c_int64, vp, u64, vp, u64, PSub]
    L.shockidx_subset_index.restype = i32
    L.shockidx_subset_gather.argtypes = [vp, vp, u64, vp, u64, vp, u64, PSub]
    L.shockidx_subset_gather.restype = i32
    L.shockidx_subset_node.argtypes = [vp, vp, u64, vp, u64, ctypes.c_int64, vp, u64, vp, u64, vp, u64, vp, u64, PSub]
    L.shockidx_subset_node.restype = i32
    L.shockidx_create_subset_index.argtypes = [vp, vp, u64, vp, u64, ctypes.c_int64, vp, u64, PSub]
    L.shockidx_create_subset_index.restype = i32
    L.shockidx_idx_part.argtypes = [vp, vp, u64, ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                    ctypes.POINTER(ctypes.c_int64), PSub]
    L.shockidx_idx_part.restype = i32
    L.shockidx_idx_range.argtypes = [vp, vp, u64, ctypes.c_char_p, ctypes.c_int64, vp, u64, PSub]
    L.shockidx_idx_range.restype = i32
    L.shockidx_filter_device.argtypes = [vp, ctypes.c_char_p, vp, u64, vp, u64, PSub]
    L.shockidx_filter_device.restype = i32
    L.shockidx_ctx_trim.argtypes = [vp, u64]
    L.shockidx_ctx_trim.restype = i32
    L.shockidx_ctx_workspace_bytes.argtypes = [vp]
    L.shockidx_ctx_workspace_bytes.restype = u64
    L.shockidx_ctx_set_dev_cap.argtypes = [vp, u64]
    L.shockidx_ctx_set_dev_cap.restype = i32
    L.shockidx_free.argtypes = [vp]
    L.shockidx_free.restype = None
    L.shockidx_strerror.argtypes = [i32]
    L.shockidx_strerror.restype = ctypes.c_char_p
    L.shockidx_abi_version.argtypes = []
    L.shockidx_abi_version.restype = i32
    # test hooks (exported, not in the public header): shockidx_ctx::inject / shockidx_multi::inject
    L.shockidx_debug_inject.argtypes = [vp, ctypes.c_uint32]
    L.shockidx_debug_inject.restype = i32
    L.shockidx_multi_debug_inject.argtypes = [vp, ctypes.c_uint32]
    L.shockidx_multi_debug_inject.restype = i32
    L.shockidx_multi_debug_ctx.argtypes = [vp, i32]
    L.shockidx_multi_debug_ctx.restype = vp
    _lib = L
    return L
