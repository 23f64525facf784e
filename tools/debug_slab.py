"""Debug harness: runs the internal slab launcher (sidx_launch_index) on a file and dumps the
per-tile look-back words, first-bad key and rows next to the oracle.  Development tool."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle

class SlabParams(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("n", ctypes.c_uint64), ("end", ctypes.c_uint64), ("base", ctypes.c_uint64),
                ("state_in", ctypes.c_uint64), ("row_base", ctypes.c_uint64), ("row_cap", ctypes.c_uint64),
                ("rows", ctypes.c_void_p), ("status", ctypes.c_void_p), ("badkey", ctypes.c_void_p),
                ("detail", ctypes.c_void_p), ("counters", ctypes.c_void_p), ("badkey_next", ctypes.c_void_p), ("counters_next", ctypes.c_void_p), ("ntiles", ctypes.c_uint32), ("epoch", ctypes.c_uint32),
                ("eof", ctypes.c_int), ("file_start", ctypes.c_int), ("timing", ctypes.c_void_p), ("debug", ctypes.c_uint32)]
class DevResult(ctypes.Structure):
    _fields_ = [("count", ctypes.c_uint64), ("state_out", ctypes.c_uint64), ("err_pos", ctypes.c_uint64),
                ("err_len", ctypes.c_uint64), ("code", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("selfhelp", ctypes.c_uint32), ("fmt", ctypes.c_uint32)]

def run(data: bytes, fmt: int, tile=32768):
    L = ctypes.CDLL(os.path.join(ROOT, "shock_amd", "libshockidx.so"))
    n = len(data)
    nt = max(1, (n + tile - 1) // tile)
    d = torch.zeros(n + 64, dtype=torch.uint8, device="cuda")
    if n: d[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cap = n // 4 + 64
    rows = torch.zeros((cap, 2), dtype=torch.int64, device="cuda")
    status = torch.zeros(nt + 8, dtype=torch.int64, device="cuda")
    small = torch.zeros(64, dtype=torch.int64, device="cuda")
    detail = torch.zeros(2 * nt + 8, dtype=torch.int64, device="cuda")
    res = torch.zeros(8, dtype=torch.int64, device="cuda")
    p = SlabParams(d.data_ptr(), n, n, 0, 0, 0, cap, rows.data_ptr(), status.data_ptr(), small.data_ptr(),
                   detail.data_ptr(), small.data_ptr() + 64, nt, 1, 1)
    L.sidx_launch_index.argtypes = [ctypes.c_int, ctypes.POINTER(SlabParams), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    rc = L.sidx_launch_index(fmt, ctypes.byref(p), res.data_ptr(), None, None, None)
    torch.cuda.synchronize()
    r = DevResult.from_buffer_copy(res.cpu().numpy().tobytes()[:ctypes.sizeof(DevResult)])
    return rc, r, status[:nt].cpu().numpy().view(np.uint64), rows.cpu().numpy().view(np.uint64), small.cpu().numpy().view(np.uint64)

if __name__ == "__main__":
    path, fmt = sys.argv[1], int(sys.argv[2])
    data = open(path, "rb").read()
    rc, r, st, rows, small = run(data, fmt)
    print("rc", rc, "count", r.count, "code", r.code, "flags", r.flags, "state_out", r.state_out, "badkey", hex(int(small[0])))
    for i, w in enumerate(st.tolist()):
        print("tile", i, "flag", w >> 62, "payload", w & ((1 << 62) - 1), "->", (w & ((1 << 62) - 1)) >> 1, (w & 1))
    name = {1: "fasta", 2: "fastq", 3: "sam"}.get(fmt)
    exp, err = oracle.line_index(data) if fmt == 4 else oracle.record_index(data, name)
    print("oracle count", len(exp), err)
    k = min(len(exp), r.count)
    bad = np.nonzero((rows[:k] != exp[:k]).any(axis=1))[0]
    print("first mismatches", bad[:10].tolist())
    for b in bad[:5]:
        print(b, rows[b].tolist(), exp[b].tolist())
