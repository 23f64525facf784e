"""Multi-process slab protocol on CPU (world_size 2 and 3, gloo and socket control planes).

Each rank holds only its slab window of the file (FRONT bytes before, HALO after), runs
shock_amd.dist.run_protocol with the CPU engine double (tests/slab_double.py), and rank 0
compares the concatenated global row table, count and error with the oracle over the whole
file (index/record.go:34-90 / index/line.go:33-85 semantics)."""
from __future__ import annotations

import multiprocessing as mp
import os
import random
import socket
import sys
import traceback

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import gen  # noqa: E402

FASTQ, LINE = 2, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, data, fmt, front, halo, wrong, backend, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, HERE)
        from shock_amd import dist
        from slab_double import HostSlabEngine
        if backend == "gloo":
            import torch.distributed as tdist
            tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
            group = dist.TorchGroup()
        else:
            os.environ["MASTER_PORT"] = str(port)
            group = dist.SocketGroup(rank, world, key=f"test_{port}", timeout=60)
        size = len(data)
        lo, hi = dist.plan_slabs(size, world)[rank]
        wlo, whi = dist.slab_window(size, lo, hi, front, halo)
        eng = HostSlabEngine(rank, world, wrong_guess=(rank in wrong))
        eng.set_slab(data[wlo:whi], wlo, lo, hi, whi, size)  # a rank sees only its window
        out = dist.run_protocol([eng], dist.HostExchange(group), fmt)[0]
        rows = np.array(eng.rows[:out.rows_owned], dtype=np.uint64).reshape(-1, 2)
        allrows = group.allgather(rows.tobytes())
        res = None
        if rank == 0:
            table = np.frombuffer(b"".join(allrows), dtype=np.uint64).reshape(-1, 2)
            res = (out.plan.count, out.plan.code, table, out.rounds)
        group.barrier()
        group.close()
        if backend == "gloo":
            tdist.destroy_process_group()
        q.put((rank, "ok", res, out.reruns))
    except Exception:
        q.put((rank, "err", traceback.format_exc(), 0))


def _run(data, fmt, world=2, front=256, halo=4096, wrong=(), backend="gloo"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, data, fmt, front, halo, set(wrong), backend, q))
          for r in range(world)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(30)
    errs = [o[2] for o in outs if o[1] == "err"]
    assert not errs, errs[0]
    res = [o for o in outs if o[0] == 0][0][2]
    reruns = sum(o[3] for o in outs)
    return res, reruns


def _oracle(data, fmt):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    if fmt == LINE:
        return oracle.line_index(data)
    return oracle.record_index(data, "fastq")


@pytest.mark.parametrize("backend", ["gloo", "socket"])
def test_fastq_two_slabs(backend):
    data = gen.fastq(random.Random(7), 120)
    (count, code, table, rounds), reruns = _run(data, FASTQ, backend=backend)
    rows, err = _oracle(data, FASTQ)
    assert err is None and code in (0, 1)
    assert count == len(rows) and rounds == 1 and reruns == 0
    np.testing.assert_array_equal(table, rows)


@pytest.mark.parametrize("wrong", [(1,), (1, 2)])
def test_fastq_wrong_guess_rerun(wrong):
    data = gen.fastq(random.Random(11), 150)
    (count, code, table, rounds), reruns = _run(data, FASTQ, world=3, wrong=wrong)
    rows, err = _oracle(data, FASTQ)
    assert count == len(rows) and rounds == 2 and reruns == len(wrong)
    np.testing.assert_array_equal(table, rows)


def test_fastq_error_in_second_slab():
    data = bytearray(gen.fastq(random.Random(5), 100))
    # corrupt a '+' line in the second half
    pos = data.index(b"\n+", len(data) * 3 // 4) + 1
    data[pos] = ord("-")
    data = bytes(data)
    (count, code, table, rounds), _ = _run(data, FASTQ)
    rows, err = _oracle(data, FASTQ)
    assert err == b"Invalid format: plus line does not start with +" and code == 7
    assert count == len(rows)
    np.testing.assert_array_equal(table, rows)


def test_line_three_slabs():
    data = gen.lines(random.Random(3), 400) if hasattr(gen, "lines") else b"".join(
        b"x" * random.Random(i).randint(0, 40) + b"\n" for i in range(400))
    (count, code, table, rounds), _ = _run(data, LINE, world=3)
    rows = _oracle(data, LINE)
    rows = rows[0] if isinstance(rows, tuple) else rows
    assert count == len(rows)
    np.testing.assert_array_equal(table, rows)


def _stale_worker(rank, world, port, data, q):
    """Two builds; in the second the exchange runs its collective but no rank takes what it
    gathered (its gathered buffer still holds the first build's summaries), as when a copy into
    the gathered buffer has not landed.  The fold must refuse them."""
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, HERE)
        from shock_amd import dist, _lib as L
        from slab_double import HostSlabEngine
        import torch.distributed as tdist
        tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        group = dist.TorchGroup()

        class StaleExchange(dist.HostExchange):
            def gather(self, engines):
                self.group.allgather(b"".join(e.summary_bytes() for e in engines))

        size = len(data)
        lo, hi = dist.plan_slabs(size, world)[rank]
        wlo, whi = dist.slab_window(size, lo, hi, 256, 4096)
        eng = HostSlabEngine(rank, world)
        eng.set_slab(data[wlo:whi], wlo, lo, hi, whi, size)
        first = dist.run_protocol([eng], dist.HostExchange(group), FASTQ)[0]
        try:
            dist.run_protocol([eng], StaleExchange(group), FASTQ)
            out = ("accepted", None)
        except L.ShockIdxError as e:
            out = ("refused", (e.code, e.msg))
        group.barrier()
        tdist.destroy_process_group()
        q.put((rank, "ok", (first.plan.count, out), 0))
    except Exception:
        q.put((rank, "err", traceback.format_exc(), 0))


def test_stale_summaries_refused():
    from shock_amd import _lib as L
    data = gen.fastq(random.Random(9), 120)
    rows, err = _oracle(data, FASTQ)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_stale_worker, args=(r, 2, port, data, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(30)
    errs = [o[2] for o in outs if o[1] == "err"]
    assert not errs, errs[0]
    for _, _, (count, (verdict, info)), _ in outs:
        assert count == len(rows)
        assert verdict == "refused" and info == (L.EINTERNAL, "internal error: stale slab summary"), info


def test_plan_slabs_cover():
    from shock_amd import dist
    for size in (0, 1, 15, 16, 17, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            sl = dist.plan_slabs(size, world)
            assert sl[0][0] == 0 and sl[-1][1] == size
            for (a, b), (c, d) in zip(sl, sl[1:]):
                assert b == c and (c % 16 == 0 or c == size)
            assert all(lo > 0 for lo, _ in sl[1:]) or size == 0  # only slab 0 owns record 0


def _rdzv_worker(rank, world, key, q):
    try:
        from shock_amd import dist
        g = dist.SocketGroup(rank, world, key=key, timeout=30)
        got = g.allgather(bytes([rank]))
        g.close()
        q.put((rank, got))
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_socket_rendezvous_refuses_foreign_peers(tmp_path, monkeypatch):
    """A stale rendezvous file of another job and a peer with the wrong nonce / rank are
    refused (jobs must never be folded together)."""
    import json
    import struct
    import threading
    import time
    from shock_amd import dist
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    key = "rdzv_test"
    path = tmp_path / f"shockidx_rdzv_{key}.json"
    path.write_text(json.dumps({"port": 1, "pid": 1, "world": 5, "nonce": "00" * 16}))  # stale, other job
    monkeypatch.delenv("MASTER_PORT", raising=False)
    with pytest.raises(ValueError):  # no key and no MASTER_PORT: no shared default file
        dist.SocketGroup(1, 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    os.environ["TMPDIR"] = str(tmp_path)
    peer = ctx.Process(target=_rdzv_worker, args=(1, 2, key, q))
    peer.start()
    time.sleep(1.0)  # the peer polls the stale file meanwhile

    def intruder():  # connects to rank 0 with a wrong nonce and a duplicate-free bogus rank
        for _ in range(200):
            try:
                info = json.load(open(path))
                if info["world"] != 2:
                    raise ValueError
                s = socket.create_connection(("127.0.0.1", info["port"]), timeout=5)
                s.sendall(struct.pack("<ii", 1, 2) + b"\x00" * 16)
                assert s.recv(1) == b""  # refused: closed without an ack
                s.close()
                return
            except (OSError, ValueError, KeyError):
                time.sleep(0.02)

    t = threading.Thread(target=intruder)
    t.start()
    g = dist.SocketGroup(0, 2, key=key, timeout=30)
    got = g.allgather(b"\x00")
    g.close()
    t.join()
    rank, peer_got = q.get(timeout=60)
    peer.join(timeout=30)
    assert got == [b"\x00", b"\x01"] and peer_got == [b"\x00", b"\x01"], peer_got


def test_bench_gpus_without_launcher_spawns_ranks(monkeypatch):
    """`python bench.py --gpus 4` run directly starts the one-process-per-GPU launch (never a
    silent one-GPU measurement); nothing touches a GPU in the parent."""
    import subprocess
    import sys as _sys
    import bench
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(_sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    assert bench.main() == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]


def _exchange_worker(rank, world, key, mode, q):
    try:
        from shock_amd import _lib as L
        from shock_amd import dist

        class FakeRccl:  # stands in for RcclExchange: fails on the ranks `mode` names
            closed = False
            inits = 0

            def __init__(self, ctx, group, uid=None):
                FakeRccl.inits += 1
                if mode in ("prep_fail_one", "prep_raise"):
                    assert uid == b"UID", uid  # rank 0's id reached every rank
                if mode == "fail_all" or (mode == "fail_one" and group.rank == 1):
                    raise L.ShockIdxError(-2, "ncclCommInitRank failed")
                if mode == "init_raise" and group.rank == 1:
                    raise RuntimeError("transport exploded")  # not a ShockIdxError: still agreed on
                self.nranks, self.gathers = group.world, 3 + group.rank

            def close(self):
                FakeRccl.closed = True

        if mode in ("prep_fail_one", "prep_raise"):
            def prepare(r):
                if mode == "prep_fail_one" and r == 1:
                    raise OSError("librccl.so: cannot open shared object file")
                return b"UID" if r == 0 else b""
            FakeRccl.prepare = staticmethod(prepare)

        g = dist.SocketGroup(rank, world, key=key, timeout=30)
        ex, label = dist.open_summary_exchange(None, g, mode == "host", rccl=FakeRccl)
        report = dist.rccl_report(ex, g)
        got = g.allgather(bytes([rank]))  # the control plane still works afterwards
        g.close()
        q.put((rank, type(ex).__name__, label, (FakeRccl.closed, FakeRccl.inits, report), got))
    except Exception:
        q.put((rank, "err", traceback.format_exc(), False, None))


@pytest.mark.parametrize("mode", ["ok", "fail_all", "fail_one", "host", "prep_fail_one", "prep_raise", "init_raise"])
def test_bench_exchange_fallback(mode):
    """bench --gpus N's summary exchange (dist.open_summary_exchange): RCCL when its setup works
    on every rank; the host exchange, labelled with the failure, when it fails on any rank (the
    ranks that did set up close their communicator); the host exchange when asked for."""
    world, key = 2, f"exch_{mode}_{os.getpid()}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_exchange_worker, args=(r, world, key, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
    for rank, kind, label, info, got in out:
        assert kind != "err", label
        closed, inits, (rccl_ranks, gathers) = info
        assert got == [b"\x00", b"\x01"]
        if mode in ("ok", "prep_raise"):
            assert kind == "FakeRccl" and label.startswith("RCCL") and not closed
            assert rccl_ranks == world and gathers == [3, 4]  # bench.py's "rccl_ranks"
        elif mode == "host":
            assert kind == "HostExchange" and "TCP control plane" in label
        else:
            assert kind == "HostExchange" and "RCCL setup failed" in label
            assert rccl_ranks == 0 and gathers == [0, 0]
            if mode == "fail_one":
                assert closed == (rank == 0)  # rank 0 had set up, then closed on the agreement
                assert ("ncclCommInitRank" in label) == (rank == 1)
            if mode == "prep_fail_one":  # agreed BEFORE the collective init: no rank entered it
                assert inits == 0 and "cannot open shared object" in label
            if mode == "init_raise":
                assert closed == (rank == 0) and ("transport exploded" in label) == (rank == 1)
