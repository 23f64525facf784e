"""Dev probe: k_fq_tiles time by HBM allocation method of the 10 GiB input (hipMalloc vs
hipExtMallocWithFlags(hipDeviceMallocContiguous) vs VMM hipMemCreate in 1 GiB physical chunks);
several allocations each, kept alive so each lands elsewhere."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shock_amd import Context  # noqa: E402
from shock_amd.synth import SynthFile  # noqa: E402

os.environ.setdefault("SHOCKIDX_CONTIG", "none")  # the library's own buffers: plain hipMalloc
hip = ctypes.CDLL("libamdhip64.so")
size = 10 << 30
ctx = Context(0)
sf = SynthFile(ctx, "fastq", size)
src = sf.window(0, size)
rows = ctx.alloc(16 * (sf.expected_count() + 1024))
cap = sf.expected_count() + 1024


def alloc_flags(flag):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(size + 4096), ctypes.c_uint(flag))
    if rc != 0:
        print(f"   hipExtMallocWithFlags(flag {flag}) rc {rc}", flush=True)
    return p.value if rc == 0 else None


class Prop(ctypes.Structure):  # hipMemAllocationProp
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("loc_type", ctypes.c_int),
                ("loc_id", ctypes.c_int), ("win32", ctypes.c_void_p), ("compType", ctypes.c_ubyte),
                ("gpuDirect", ctypes.c_ubyte), ("usage", ctypes.c_ushort), ("reserved", ctypes.c_ubyte * 4)]


class Access(ctypes.Structure):  # hipMemAccessDesc
    _fields_ = [("loc_type", ctypes.c_int), ("loc_id", ctypes.c_int), ("flags", ctypes.c_int)]


def alloc_vmm(chunk):
    prop = Prop(1, 0, 1, 0, None, 0, 0, 0)
    g = ctypes.c_size_t()
    if hip.hipMemGetAllocationGranularity(ctypes.byref(g), ctypes.byref(prop), 1) != 0:
        return None
    total = ((size + 4096 + chunk - 1) // chunk) * chunk
    va = ctypes.c_void_p()
    if hip.hipMemAddressReserve(ctypes.byref(va), ctypes.c_size_t(total), ctypes.c_size_t(chunk), None, ctypes.c_ulonglong(0)) != 0:
        return None
    for off in range(0, total, chunk):
        h = ctypes.c_void_p()
        if hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(chunk), ctypes.byref(prop), ctypes.c_ulonglong(0)) != 0:
            return None
        if hip.hipMemMap(ctypes.c_void_p(va.value + off), ctypes.c_size_t(chunk), ctypes.c_size_t(0), h, ctypes.c_ulonglong(0)) != 0:
            return None
    acc = Access(1, 0, 3)
    if hip.hipMemSetAccess(va, ctypes.c_size_t(total), ctypes.byref(acc), ctypes.c_size_t(1)) != 0:
        return None
    print(f"   vmm granularity {g.value}", flush=True)
    return va.value


keep = []
plan = [("malloc", 0), ("contig", 4), ("vmm1g", 1 << 30)] * 3
for name, arg in plan:
    p = alloc_vmm(arg) if name.startswith("vmm") else alloc_flags(arg)
    if not p:
        print(f"{name}: allocation failed", flush=True)
        continue
    hip.hipMemcpy(ctypes.c_void_p(p), ctypes.c_void_p(src.ptr), ctypes.c_size_t(size), 3)
    hip.hipDeviceSynchronize()
    t = []
    k = []
    for i in range(6):
        r = ctx.build_device(p, size, rows.ptr, cap, kind="record", fmt="fastq")
        t.append(r.timings["index_ms"])
        k.append(r.timings["kernel_ms"])
    t.sort(); k.sort()
    print(f"{name:7s} ptr {p:#x} index_ms min {t[0]:.3f} med {t[3]:.3f} max {t[-1]:.3f} build med {k[3]:.3f} ok {r.ok}", flush=True)
    keep.append(p)
