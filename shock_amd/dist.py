"""Multi-GPU slab indexing of one node file.

One process per GPU.  The file is cut into byte slabs, one per rank (`plan_slabs`); each rank
holds its slab in HBM plus up to FRONT bytes before it and HALO bytes after it (records that
start in the slab and end past it are validated in place).  The protocol per build:

  1. guess the slab's incoming reader state from its first bytes (shockidx_slab_guess);
  2. index the slab against the guess (shockidx_slab_index): rows of the records the slab
     owns + a 64-byte summary (slab aggregate, first-bad key, natural count, ...);
  3. all-gather the summaries (RCCL over xGMI: `RcclExchange`; 64 B x world, the only data
     that crosses GPUs);
  4. fold them in slab order on the device (shockidx_slab_combine): the true incoming state,
     the global number of the slab's first record, the global count / error;
  5. a slab whose guess disagrees with the fold is re-indexed with the true state and the
     summaries exchanged again (never needed on well-formed data).

The reference has no multi-node index build (record.Create is one sequential pass,
index/record.go:34-90); the result of this protocol equals that pass byte for byte: the
global row table is the concatenation of each rank's first `rows_owned` rows.

The control plane (unique-id broadcast, barriers, timing max) runs over a `HostGroup`:
torch.distributed (gloo) where torch is safe to import, or plain sockets in GPU processes
(torch's bundled HIP runtime shares the soname of the system ROCm runtime that
libshockidx.so links, so GPU processes never import torch).
"""
from __future__ import annotations

import ctypes
import json
import os
import socket
import struct
import time
from dataclasses import dataclass

import numpy as np

from . import _lib as L

FRONT = 64 << 10        # bytes kept before a slab (state guess + trim look-behind)
HALO = 4 << 20          # bytes kept after a slab (records crossing the slab end)
ALIGN = 16              # slab cuts are 16-byte aligned (device loads are 16 B per lane)
ST_NEEDMORE = 12        # device status: slab halo exhausted (sidx_common.hpp)
ST_FA_INVALID = 10
KEY_NONE = (1 << 64) - 1


def plan_slabs(size: int, world: int, align: int = ALIGN):
    """[(lo, hi)] byte ranges, one per rank, 16-byte aligned cuts, equal up to alignment.
    Only slab 0 starts at offset 0 (it owns record 0); empty slabs, if any, come last."""
    cuts = [0] + [min(size, max(align, (size * r // world + align - 1) // align * align))
                  for r in range(1, world)] + [size]
    return [(cuts[r], max(cuts[r], cuts[r + 1])) for r in range(world)]


def slab_window(size: int, lo: int, hi: int, front: int = FRONT, halo: int = HALO):
    """Bytes [wlo, whi) a rank keeps in HBM for slab [lo, hi)."""
    wlo = max(0, lo - front) // ALIGN * ALIGN
    whi = min(size, hi + halo)
    return wlo, whi


# ---------------------------------------------------------------------------------------------
# Control plane
# ---------------------------------------------------------------------------------------------
class HostGroup:
    rank: int
    world: int

    def allgather(self, blob: bytes) -> list:
        raise NotImplementedError

    def barrier(self):
        self.allgather(b"")

    def max(self, x: float) -> float:
        return max(struct.unpack("<d", b)[0] for b in self.allgather(struct.pack("<d", float(x))))

    def close(self):
        pass


class TorchGroup(HostGroup):
    """torch.distributed CPU group (gloo).  Only for processes that do not use libshockidx's
    GPU path (CPU tests); see the module docstring."""

    def __init__(self, pg=None):
        import torch.distributed as tdist
        self._d = tdist
        self._pg = pg
        self.rank = tdist.get_rank(pg)
        self.world = tdist.get_world_size(pg)

    def allgather(self, blob: bytes) -> list:
        out = [None] * self.world
        self._d.all_gather_object(out, bytes(blob), group=self._pg)
        return out

    def barrier(self):
        self._d.barrier(group=self._pg)


def _send(sock, blob: bytes):
    sock.sendall(struct.pack("<Q", len(blob)) + blob)


def _recv_exact(sock, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        part = sock.recv(n - len(buf))
        if not part:
            raise ConnectionError("peer closed the control connection")
        buf += part
    return bytes(buf)


def _recv(sock) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class SocketGroup(HostGroup):
    """Star-shaped control plane over TCP on 127.0.0.1 (one node).  Rank 0 listens on an
    ephemeral port and publishes it in a rendezvous file keyed by MASTER_PORT + run id."""

    def __init__(self, rank: int, world: int, key: str | None = None, timeout: float = 300.0):
        self.rank, self.world = rank, world
        self._peers = []
        self._sock = None
        if world == 1:
            return
        if key is None:
            if "MASTER_PORT" not in os.environ:
                raise ValueError("SocketGroup: pass a key or set MASTER_PORT (the rendezvous file name)")
            key = "%s_%s" % (os.environ["MASTER_PORT"], os.environ.get("TORCHELASTIC_RUN_ID", "x"))
        path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"shockidx_rdzv_{key}.json")
        # handshake: rank 0 publishes (port, world, nonce); a peer answers with (rank, world,
        # nonce) and waits for an ack.  A stale or foreign rendezvous file, a duplicate or an
        # out-of-range rank is refused, so two jobs can never be folded together.
        if rank == 0:
            nonce = os.urandom(16)
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(world)
            tmp = path + ".%d.tmp" % os.getpid()
            with open(tmp, "w") as f:
                json.dump({"port": srv.getsockname()[1], "pid": os.getpid(), "world": world, "nonce": nonce.hex()}, f)
            os.replace(tmp, path)
            srv.settimeout(timeout)
            peers = {}
            while len(peers) < world - 1:
                c, _ = srv.accept()
                c.settimeout(timeout)
                try:
                    r, w = struct.unpack("<ii", _recv_exact(c, 8))
                    good = _recv_exact(c, 16) == nonce and w == world and 1 <= r < world and r not in peers
                except (OSError, struct.error):
                    good = False
                if not good:
                    c.close()
                    continue
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.sendall(b"\x01")
                c.settimeout(None)  # the handshake timeout does not apply to the collectives
                peers[r] = c
            srv.close()
            self._peers = [peers[r] for r in range(1, world)]
            try:
                os.unlink(path)
            except OSError:
                pass
        else:
            t0 = time.time()
            while True:
                try:
                    info = json.load(open(path))
                    if int(info["world"]) != world:
                        raise ValueError("rendezvous file of another job")
                    s = socket.create_connection(("127.0.0.1", int(info["port"])), timeout=timeout)
                    s.sendall(struct.pack("<ii", rank, world) + bytes.fromhex(info["nonce"]))
                    if _recv_exact(s, 1) != b"\x01":
                        raise ConnectionError("rendezvous refused")
                    break
                except (OSError, ValueError, KeyError, ConnectionError):
                    if time.time() - t0 > timeout:
                        raise TimeoutError(f"rank {rank}: no rendezvous at {path}")
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            self._sock = s

    def allgather(self, blob: bytes) -> list:
        if self.world == 1:
            return [bytes(blob)]
        if self.rank == 0:
            parts = [bytes(blob)] + [_recv(c) for c in self._peers]
            packed = b"".join(struct.pack("<Q", len(p)) + p for p in parts)
            for c in self._peers:
                _send(c, packed)
            return parts
        _send(self._sock, bytes(blob))
        packed = _recv(self._sock)
        out, o = [], 0
        for _ in range(self.world):
            (n,) = struct.unpack_from("<Q", packed, o)
            out.append(packed[o + 8:o + 8 + n])
            o += 8 + n
        return out

    def close(self):
        for c in self._peers:
            c.close()
        if self._sock is not None:
            self._sock.close()
        self._peers, self._sock = [], None


# ---------------------------------------------------------------------------------------------
# Device engine (one slab on one GPU) and summary exchanges
# ---------------------------------------------------------------------------------------------
@dataclass
class Plan:
    state_in: int
    first_record: int
    count: int
    err_pos: int
    err_len: int
    code: int
    err_rank: int
    inconsistent: int
    flags: int

    @classmethod
    def from_struct(cls, p: L.SlabPlan) -> "Plan":
        return cls(*(int(getattr(p, f)) for f, _ in L.SlabPlan._fields_))


class DeviceSlabEngine:
    """One rank's slab on its GPU: wraps shockidx_slab_{guess,index,combine}."""

    def __init__(self, ctx, rank: int, world: int):
        self.ctx, self.rank, self.world = ctx, rank, world
        self._lib = L.lib()
        self.d_summary = ctx.alloc(64)
        self.d_all = ctx.alloc(64 * world)
        self.res = L.Result()
        self.slab = None

    def set_slab(self, buf, wlo: int, lo: int, hi: int, whi: int, size: int, rows, row_cap: int):
        """buf holds file bytes [wlo, whi); the slab owns [lo, hi)."""
        s = L.Slab()
        s.d_data = buf.ptr + (lo - wlo)
        s.n = hi - lo
        s.end = whi - lo
        s.front = lo - wlo
        s.base = lo
        s.is_first = int(lo == 0 and self.rank == 0)
        s.is_last = int(whi == size)
        self.slab, self.buf, self.wlo = s, buf, wlo
        self.rows, self.row_cap = rows, row_cap
        self.row_base = 0 if s.is_first else 1

    def guess(self, fmt: int) -> int:
        g = ctypes.c_uint64(0)
        rc = self._lib.shockidx_slab_guess(self.ctx._h, ctypes.byref(self.slab), fmt, ctypes.byref(g))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_slab_guess failed")
        return g.value

    def index(self, fmt: int, state_in: int, seq: int = 0):
        self.slab.seq = seq  # stamped into the slab's summary (the fold checks it)
        rc = self._lib.shockidx_slab_index(self.ctx._h, ctypes.byref(self.slab), fmt, state_in, self.rows.ptr,
                                           self.row_cap, self.d_summary.ptr, ctypes.byref(self.res))
        if rc != L.OK:
            raise L.ShockIdxError(rc, bytes(self.res.err)[:self.res.err_len].decode("utf-8", "replace"))
        self.local_count = int(self.res.count)
        self.local_flags = int(self.res.flags)
        return self.res

    def summary_bytes(self) -> bytes:
        return self.d_summary.download(64).tobytes()

    def load_all(self, blobs):
        self.d_all.upload(b"".join(blobs))

    def combine(self, fmt: int, expect=None) -> Plan:
        p = L.SlabPlan()
        ex = (ctypes.c_uint32 * self.world)(*expect) if expect is not None else None
        rc = self._lib.shockidx_slab_combine(self.ctx._h, self.d_all.ptr, self.world, self.rank, fmt, ex,
                                             ctypes.byref(p))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "shockidx_slab_combine failed")
        return Plan.from_struct(p)

    def error_bytes(self, pos: int, n: int) -> bytes:
        return self.buf.download(n, pos - self.wlo).tobytes()

    def head(self, n: int = 32768) -> bytes:
        """first bytes of the file (rank 0: format detection, multi.go:43-62)"""
        return self.buf.download(min(n, self.slab.end + self.slab.front)).tobytes()

    def free(self):
        self.d_summary.free()
        self.d_all.free()


class HostExchange:
    """Summaries through the host control plane (64 B per rank)."""

    def __init__(self, group: HostGroup):
        self.group = group

    def gather(self, engines):
        mine = b"".join(e.summary_bytes() for e in engines)
        allb = self.group.allgather(mine)
        blobs = [b[i:i + 64] for b in allb for i in range(0, len(b), 64)]
        for e in engines:
            e.load_all(blobs)


class LocalExchange:
    """All slabs driven by one process (tests, single-GPU rehearsal of the protocol)."""

    def gather(self, engines):
        blobs = [e.summary_bytes() for e in sorted(engines, key=lambda e: e.rank)]
        for e in engines:
            e.load_all(blobs)


class RcclExchange:
    """Summaries all-gathered device-to-device over RCCL (one communicator per process)."""

    @staticmethod
    def prepare(rank: int) -> bytes:
        """The part of setup that is not collective: the library and its RCCL entry points load,
        and rank 0 draws the unique id (ncclGetUniqueId).  Raises on failure."""
        lib = L.lib()
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            rc = lib.shockidx_comm_unique_id(uid)
            if rc != L.OK:
                raise L.ShockIdxError(rc, "ncclGetUniqueId failed")
            return uid.raw
        return b""

    def __init__(self, ctx, group: HostGroup, uid: bytes | None = None):
        lib = L.lib()
        if uid is None:  # (one call does both phases: tests, world 1)
            ids = group.allgather(self.prepare(group.rank))
            uid = ids[0]
        buf = ctypes.create_string_buffer(uid, 128)
        h = ctypes.c_void_p()
        rc = lib.shockidx_comm_init(ctx._h, group.world, group.rank, buf, ctypes.byref(h))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "ncclCommInitRank failed")
        self._h, self._lib = h, lib
        n = ctypes.c_int(0)
        rc = lib.shockidx_comm_count(h, ctypes.byref(n))
        if rc != L.OK:
            raise L.ShockIdxError(rc, "ncclCommCount failed")
        self.nranks = n.value  # the ranks the communicator spans (bench: "rccl_ranks")
        self.gathers = 0       # all-gathers issued over it

    def gather(self, engines):
        (e,) = engines
        rc = self._lib.shockidx_comm_allgather(self._h, e.d_summary.ptr, e.d_all.ptr, 64)
        if rc != L.OK:
            raise L.ShockIdxError(rc, "ncclAllGather failed")
        self.gathers += 1

    def close(self):
        if self._h:
            self._lib.shockidx_comm_destroy(self._h)
            self._h = None


# ---------------------------------------------------------------------------------------------
# The protocol
# ---------------------------------------------------------------------------------------------
class HaloExhausted(RuntimeError):
    """A record starting in some slab runs past that slab's halo: re-run with a larger halo."""


@dataclass
class SlabOutcome:
    plan: Plan
    rank: int
    rows_owned: int      # this rank's rows[0:rows_owned] are global records first_record..
    rounds: int          # summary exchanges (1 unless a guess was wrong)
    reruns: int          # slabs of this process re-indexed


def rows_owned(plan: Plan, local_count: int, row_base: int) -> int:
    delta = plan.first_record - row_base  # global - local record numbers
    local_end = min(local_count, plan.count - delta) if plan.count >= delta else 0
    return max(0, local_end - row_base)


def local_state(fmt: int, s: int) -> int:
    """A state with its record count dropped: what a slab is indexed against (guesses have
    this form; the fold adds the count back as the slab's record-number delta)."""
    if fmt == L.FMT_FASTQ or fmt == L.FMT_SAM:
        return s & 3
    if fmt == L.FMT_FASTA:
        return s & 1
    return 0


def run_protocol(engines, exchange, fmt: int, max_rounds: int = 4, times: dict | None = None):
    """Index the slabs of `engines` (this process's ranks) and fold the global result.
    Every process calls this collectively with the same fmt.  `times` (optional) accumulates
    wall-clock ms per phase: guess, index, exchange, combine (each call returns synchronised)."""
    clock = time.perf_counter

    def tick(key, t0):
        if times is not None:
            times[key] = times.get(key, 0.0) + (clock() - t0) * 1e3

    # Every summary carries a tag: the build (counted alike by every process, the protocol being
    # collective) << 4 | the round its slab was last indexed in.  The fold refuses a summary with
    # any other tag -- one left from an earlier build or round by an exchange that did not land.
    for e in engines:
        e.builds = getattr(e, "builds", 0) + 1
    build = engines[0].builds
    expect = [build << 4] * engines[0].world
    for e in engines:
        t0 = clock()
        g = e.guess(fmt)
        tick("guess", t0)
        t0 = clock()
        e.index(fmt, g, expect[e.rank])
        tick("index", t0)
    reruns = 0
    for rounds in range(1, max_rounds + 1):
        t0 = clock()
        exchange.gather(engines)
        tick("exchange", t0)
        t0 = clock()
        plans = [e.combine(fmt, expect) for e in engines]
        tick("combine", t0)
        if any(p.flags & 32 for p in plans):
            raise L.ShockIdxError(L.EINTERNAL, "internal error: stale slab summary")
        bad = plans[0].inconsistent
        if not bad:
            break
        for q in range(len(expect)):
            if (bad >> q) & 1:
                expect[q] = (build << 4) | rounds
        for e, p in zip(engines, plans):
            if (bad >> e.rank) & 1:
                t0 = clock()
                e.index(fmt, local_state(fmt, p.state_in), expect[e.rank])
                tick("index", t0)
                reruns += 1
    else:
        raise RuntimeError("slab states did not converge")
    out = []
    for e, p in zip(engines, plans):
        if p.code == ST_NEEDMORE or (p.flags & 4):
            raise HaloExhausted(f"record crosses the halo of a slab (plan {p})")
        if p.flags & 2:
            raise L.ShockIdxError(L.EINTERNAL, "internal error: device invariant violated")
        if e.local_flags & 1:
            raise L.ShockIdxError(L.ENOMEM, f"slab {e.rank}: row table capacity {e.row_cap} exceeded")
        out.append(SlabOutcome(p, e.rank, rows_owned(p, e.local_count, e.row_base), rounds, reruns))
    return out


_STATUS_TEXT = {
    2: "Invalid format: truncated fastq record", 3: "Invalid format: empty line(s) between records",
    4: "Invalid format: id line does not start with @", 5: "Invalid format: missing sequence ID",
    6: "Invalid format: empty sequence", 7: "Invalid format: plus line does not start with +",
    8: "Invalid format: quality ID does not match sequence ID",
    9: "Invalid format: length of sequence and quality lines do not match",
}


def error_text(plan: Plan, fetch) -> bytes | None:
    """Go's error text for the global result (None on success).  `fetch(pos, n)` returns file
    bytes from the rank that holds them (plan.err_rank)."""
    if plan.code in (0, 1, 13):  # OK, END, ABSENT
        return None
    if plan.code == ST_FA_INVALID:
        n = min(50, plan.err_len)
        return b"Invalid fasta entry: " + (fetch(plan.err_pos, n) if n else b"")
    return _STATUS_TEXT.get(plan.code, "internal error: status %d" % plan.code).encode()


def open_summary_exchange(ctx, group: HostGroup, want_host: bool, rccl=None):
    """The bench's summary exchange and its label for the JSON line: RCCL unless `want_host`.
    Communicator setup is collective: a failure that hits every rank alike (library or transport
    unavailable) is agreed on over the control plane and the run continues on the host exchange,
    labelled as such -- the summaries are 64 B per slab, so the step time barely moves, but the
    label never claims RCCL it did not use.  `rccl` (tests): the RCCL exchange's constructor.

    Two agreements: first every rank reports whether the non-collective part of setup
    worked (the library loads; rank 0 has a unique id), and only if all did does any rank enter
    the collective ncclCommInitRank -- so a rank that fails early never leaves the others blocked
    inside init; then every rank reports whether init worked, catching every exception, so each
    rank reaches that all-gather.  (A rank that fails INSIDE init while the others wait there is
    RCCL's own failure mode and is not covered.)"""
    import sys
    if want_host:
        return HostExchange(group), "host all-gather of 64-B slab summaries (TCP control plane)"
    make = rccl or RcclExchange
    prep = getattr(make, "prepare", None)
    ex, err = None, ""
    try:
        mine = b"1" + (prep(group.rank) if prep else b"")
    except Exception as e:  # noqa: BLE001 (every failure must reach the agreement below)
        mine = b"0" + str(e).encode()[:300]
    pre = group.allgather(mine)
    if any(p[:1] != b"1" for p in pre):
        why = next(p[1:].decode("utf-8", "replace") for p in pre if p[:1] != b"1")
        return HostExchange(group), f"host all-gather of 64-B slab summaries (RCCL setup failed: {why})"
    # RCCL prints its version banner on stdout when setup fails; the driver reads rank 0's
    # stdout as the one JSON line, so the library's fd 1 points at stderr while it sets up
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        ex = make(ctx, group, pre[0][1:]) if prep else make(ctx, group)
    except Exception as e:  # noqa: BLE001
        err = str(e) or type(e).__name__
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    flags = group.allgather(b"1" if ex is not None else b"0")
    if all(f == b"1" for f in flags):
        return ex, "RCCL all-gather of 64-B slab summaries"
    if ex is not None:
        ex.close()
    return HostExchange(group), f"host all-gather of 64-B slab summaries (RCCL setup failed: {err or 'on another rank'})"


# ---------------------------------------------------------------------------------------------
# bench.py --gpus N (one process per GPU, launched by torch.distributed.run)
# ---------------------------------------------------------------------------------------------
def bench_main(a, rank: int, world: int, local: int) -> int:
    """Weak scaling (default): the node file is world x size-gib; rank r indexes slab r.
    Strong scaling (--scaling strong, BASELINE configs[4] / SURVEY §8(d) C5): one file of
    total-gib (80 GiB) cut into world slabs; the 1-GPU point indexes all of it."""
    import sys
    from .core import Context
    from .synth import SynthFile

    GIB = 1 << 30
    group = SocketGroup(rank, world)
    # rehearsal knobs (one-GPU boxes): every rank on one device, summaries over the host plane
    dev = int(os.environ.get("SHOCKIDX_BENCH_DEVICE", local))
    ctx = Context(dev)
    strong = getattr(a, "scaling", "weak") == "strong"
    if strong:
        size = int(a.total_gib * GIB)
        per = size // world
    else:
        per = int(a.size_gib * GIB)
        size = per * world
    sf = SynthFile(ctx, a.fmt, size)
    lo, hi = plan_slabs(size, world)[rank]
    wlo, whi = slab_window(size, lo, hi)
    buf = sf.window(wlo, whi)
    k0, k1 = sf.record_range(lo, hi)
    row_cap = (k1 - k0) + 1024
    rows = ctx.alloc(16 * row_cap)
    eng = DeviceSlabEngine(ctx, rank, world)
    eng.set_slab(buf, wlo, lo, hi, whi, size, rows, row_cap)
    ex, exchange_label = open_summary_exchange(ctx, group, os.environ.get("SHOCKIDX_BENCH_EXCHANGE") == "host")
    fmt = L.FMT_CODES[a.fmt]
    phase_ms: dict = {}

    def step(times=None):
        return run_protocol([eng], ex, fmt, times=times)[0]

    for _ in range(a.warmup):
        step()
    ctx.sync()
    group.barrier()
    t0 = time.perf_counter()
    idx_ms = []
    for _ in range(a.steps):
        o = step(phase_ms)
        idx_ms.append(eng.res.index_ms)
    ctx.sync()
    dt = time.perf_counter() - t0
    group.barrier()
    dt_max = group.max(dt)
    ms = dt_max / a.steps * 1e3
    R = sf.expected_count()
    ok = o.plan.count == R
    mism = -1
    if a.check and a.fmt == "fastq":
        mism = sf.check_rows(rows, o.plan.first_record, o.rows_owned)
        ok = ok and mism == 0
    mism_all = group.allgather(struct.pack("<q", mism))
    k_ms = group.max(float(np.mean(idx_ms)))
    rccl_ranks, rccl_gathers = rccl_report(ex, group)
    phases = {k: round(group.max(phase_ms.get(k, 0.0) / a.steps), 4) for k in ("guess", "index", "exchange", "combine")}
    if rank == 0:
        alg = per + 16 * (R // world)
        achieved = alg / (k_ms * 1e-3) / 1e9
        out = {
            "metric": "device-resident index-build GiB/s + Mrecords/s, 10 GiB FASTQ, 1/2/4/8 GPU",
            "value": round(size / (ms * 1e-3) / GIB, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (device-generated, seed 0x5EED, SURVEY.md §8(d))",
            "config": {"workload": (f"{a.fmt} record index, one {size / GIB:g} GiB node file cut into {world} slabs "
                                    "(BASELINE configs[4])" if strong else
                                    f"{a.fmt} record index, {world} x {a.size_gib:g} GiB node file, one slab per GPU"),
                       "records": R, "bytes": size, "tile": 16384, "parallelism": f"slab{world}",
                       "exchange": exchange_label},
            "rccl_ranks": rccl_ranks, "rccl_allgathers_per_rank": rccl_gathers,
            "index_kernel_ms": round(k_ms, 4), "rounds": o.rounds,
            # per-step wall-clock ms of each protocol phase, max over ranks: the slab guess,
            # the slab index (kernels), the summary exchange and the combine
            "protocol_ms": phases,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": 8000.0, "unit": "GB/s",
                         "frac": round(achieved / 8000.0, 4), "traffic": None},
            "parity": {"count_ok": ok, "mismatches": [struct.unpack("<q", m)[0] for m in mism_all]},
        }
        print(json.dumps(out))
        sys.stdout.flush()
    if hasattr(ex, "close"):
        ex.close()
    group.close()
    return 0 if ok else 1


def rccl_report(ex, group: HostGroup):
    """(rccl_ranks, all-gathers per rank): the ranks every rank's communicator spans
    (ncclCommCount; 0 when any rank used the host exchange) and how many summary all-gathers each
    rank issued over RCCL -- so a scaling line shows the collective it ran, not only that it ran."""
    mine = struct.pack("<ii", int(getattr(ex, "nranks", 0)), int(getattr(ex, "gathers", 0)))
    got = [struct.unpack("<ii", b) for b in group.allgather(mine)]
    ranks = min(n for n, _ in got)
    return (ranks if all(n == ranks for n, _ in got) else 0), [g for _, g in got]
