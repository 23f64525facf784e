"""bench.py -- device-resident record-index build throughput (BASELINE.json metric).

Workload (N=1): BASELINE.json configs[1] -- a 10 GiB synthetic FASTQ node file resident in
HBM, record index built by libshockidx exactly as Shock's
index/record.go would (auto-detected format, full validation, offset table left in HBM).
A "step" is one complete build: detect + index kernel + finalize.  N>1: the file is
N x 10 GiB, one slab per GPU (weak scaling), with one RCCL all-gather of slab summaries.

Prints one JSON line (rank 0).  --check verifies every row against the generator.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = 1 << 30
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
METRIC = "device-resident index-build GiB/s + Mrecords/s, 10 GiB FASTQ, 1/2/4/8 GPU"  # BASELINE.json
TILE = 16384  # bytes per workgroup tile (sidx_common.hpp SIDX_TILE)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    # ~0.25 s of builds before the timed region: the first builds of a process run up to ~10 %
    # slower while the device's clocks ramp (profiles/r04/placement2c.txt, warmup 3 / 30 / 300:
    # k_fq_tiles 1.88 / 1.87 / 1.86 ms on one box)
    ap.add_argument("--warmup", type=int, default=None, help="default: 100 for the device-resident builds, 3 otherwise")
    ap.add_argument("--fmt", default="fastq", choices=("fastq", "fasta"))
    ap.add_argument("--size-gib", type=float, default=10.0)
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="N>1: weak = N x size-gib; strong = one total-gib file cut into N slabs (configs[4])")
    ap.add_argument("--total-gib", type=float, default=80.0, help="--scaling strong: the node file size")
    ap.add_argument("--cpu-sec", type=float, default=10.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--cpu-sample-gib", type=float, default=1.0)
    ap.add_argument("--check", action="store_true", default=True)
    ap.add_argument("--no-check", dest="check", action="store_false")
    ap.add_argument("--no-floor", dest="floor", action="store_false", default=True,
                    help="skip the box's streaming floor (k_stream_floor) printed beside record / line builds")
    ap.add_argument("--pmc", default=None, help="rocprofv3 PMC summary (default: the newest profiles/r*/pmc_<fmt>.json on these sources)")
    ap.add_argument("--filter", default="fq2fa", choices=("fq2fa", "anonymize"), help="--kind filter: which filter")
    ap.add_argument("--kind", default="record", choices=("record", "line", "chunkrecord", "filter"),
                    help="line: the line indexer (index/line.go) over the same synthetic file")
    ap.add_argument("--subset", action="store_true",
                    help="BASELINE configs[3]: subset node of a random 1%% of the records (default 50 GiB FASTQ)")
    ap.add_argument("--subset-frac", type=float, default=0.01)
    ap.add_argument("--pinned", action="store_true", help="--e2e from a host buffer registered for DMA")
    ap.add_argument("--fd", action="store_true",
                    help="--e2e from a page-cached node file through shockidx_build_fd / shockidx_create")
    ap.add_argument("--trim", type=float, default=None, metavar="GIB",
                    help="--e2e --fd: trim the context to GIB after every call, as the Go shim's pool does "
                         "(gpurecord.go gpuCtxPool.put: shockidx_ctx_trim(ctx, 1 GiB)); the next call regrows")
    ap.add_argument("--dev-cap", type=float, default=None, metavar="GIB",
                    help="--e2e --fd: cap the device bytes one build may hold (shockidx_ctx_set_dev_cap); a node "
                         "whose one-pass build does not fit goes through two slab slots sized to the cap")
    ap.add_argument("--e2e", action="store_true",
                    help="host-memory build (POSTed body): pinned H2D staging + kernel + table D2H")
    a = ap.parse_args()
    if a.warmup is None:
        a.warmup = 100 if (a.kind in ("record", "line") and not a.e2e and not a.subset) else 3
    return a


def cpu_threads(sample: np.ndarray, cuts, fmt: str, budget_s: float, oracle):
    """The same restatement on every host core the GPU box leases (16): the sample cut at record
    boundaries into one piece per thread (independent, as the multi-GPU slabs are), each piece
    indexed by its own thread (ctypes releases the GIL for the C call).  The all-cores CPU bar."""
    from concurrent.futures import ThreadPoolExecutor
    pieces = [sample[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    with ThreadPoolExecutor(len(pieces)) as ex:
        reps, t_total = 0, 0.0
        while t_total < budget_s or reps == 0:
            t0 = time.perf_counter()
            list(ex.map(lambda x: oracle.record_index(x, fmt), pieces))
            t_total += time.perf_counter() - t0
            reps += 1
    return reps * sample.size / t_total / GIB, len(pieces)


def cpu_baseline(sample: np.ndarray, fmt: str, budget_s: float, cuts=None):
    """Oracle (C restatement of the Go path) on a bounded sample: one thread, then (cuts: record
    boundaries) one piece per leased core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only
    oracle.build()
    reps, t_total, nrec = 0, 0.0, 0
    while t_total < budget_s or reps == 0:
        t0 = time.perf_counter()
        rows, err = oracle.record_index(sample, fmt)
        t_total += time.perf_counter() - t0
        reps += 1
        nrec = len(rows)
    gibs = reps * sample.size / t_total / GIB
    # the same sample from a page-cached file (read(2) into a buffer, then the scan), as the Go
    # reader consumes the node file (BASELINE.md "CPU baseline plan")
    import tempfile
    fgibs, freps = None, 0
    with tempfile.NamedTemporaryFile(dir="/tmp", suffix=".sample") as tf:
        sample.tofile(tf.name)
        np.fromfile(tf.name, dtype=np.uint8)  # warm the page cache
        f_total = 0.0
        while f_total < budget_s / 2 or freps == 0:
            t0 = time.perf_counter()
            buf = np.fromfile(tf.name, dtype=np.uint8)
            oracle.record_index(buf, fmt)
            f_total += time.perf_counter() - t0
            freps += 1
            del buf
        fgibs = freps * sample.size / f_total / GIB
    out = {"value": round(gibs, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
           "mrec_per_s": round(reps * nrec / t_total / 1e6, 3),
           "page_cached_file_value": round(fgibs, 3),
           "sample": f"first {sample.size / GIB:.2f} GiB of the same synthetic {fmt} file, "
                     f"{reps} passes in {t_total:.1f} s from memory ({freps} more from a page-cached file: "
                     f"page_cached_file_value), oracle/shockidx_oracle.c (C restatement of "
                     f"index/record.go + format/{fmt}), 1 thread"}
    if cuts is not None and len(cuts) > 2:
        tg, nt = cpu_threads(sample, cuts, fmt, budget_s / 2, oracle)
        out["all_cores"] = {"value": round(tg, 3), "unit": "GiB/s", "cores": nt,
                            "sample": f"the same sample cut at record boundaries into {nt} pieces, one thread each"}
    return out


def kernel_source_sha() -> str:
    """sha256 of the kernel sources: a PMC summary counts only for the code it was taken on."""
    h = hashlib.sha256()
    for f in ("sidx_kernels.hip", "sidx_common.hpp", "sidx_device.hpp"):
        with open(os.path.join(ROOT, "shock_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def load_pmc(path, cfg, kernel):
    """HBM bytes per launch of `kernel` from a rocprofv3 PMC summary (tools/pmc_summary.py) taken
    on this same kernel source and config, else None (never a stale number)."""
    try:
        d = json.load(open(path))
    except Exception:
        return None
    if d.get("config") != cfg or d.get("kernel") != kernel or d.get("source_sha") != kernel_source_sha():
        return None
    return d.get("hbm_bytes_per_launch")


def fastq_kernel() -> str:
    """The FASTQ build's dominant kernel."""
    return "k_fq_tiles"


def fasta_kernel() -> str:
    """The FASTA build's dominant kernel (SHOCKIDX_FA_MODE=two: the two-pass build)."""
    return "k_index1" if os.environ.get("SHOCKIDX_FA_MODE", "") in ("two", "0") else "k_fa_tiles"


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start the one-process-per-GPU launch the
    driver uses (torch.distributed.run, rendezvous on 127.0.0.1) as a child -- before this
    process touches a GPU -- and return its exit code.  Never measures fewer GPUs than asked."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(a.gpus)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:  # the launcher's world is authoritative; say so instead of measuring silently
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: measuring {world} GPU(s)", file=sys.stderr)
        a.gpus = world
    if world > 1 or a.scaling == "strong":
        from shock_amd import dist
        return dist.bench_main(a, rank, world, local)

    from shock_amd import Context
    from shock_amd.synth import SynthFile

    ctx = Context(local)
    if a.subset and a.size_gib == 10.0:
        a.size_gib = 50.0  # configs[3]
    size = int(a.size_gib * GIB)
    sf = SynthFile(ctx, a.fmt, size)
    data = sf.window(0, size)
    R = sf.expected_count()
    if a.e2e:
        return e2e(a, ctx, sf, data, size, R)
    if a.subset:
        return subset_bench(a, ctx, sf, data, size, R)
    rows = ctx.alloc(16 * (R + 1024))

    if a.kind == "line":
        return line_bench(a, ctx, sf, data, size)
    if a.kind == "chunkrecord":
        return chunk_bench(a, ctx, sf, data, size)
    if a.kind == "filter":
        return filter_bench(a, ctx, sf, data, size)
    for _ in range(a.warmup):
        r = ctx.build_buffer(data, size, rows, kind="record", fmt=None)
        assert r.ok or os.environ.get("SHOCKIDX_DEBUG"), r
    ctx.sync()
    idx_ms, build_ms_l = [], []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = ctx.build_buffer(data, size, rows, kind="record", fmt=None)
        idx_ms.append(r.timings["index_ms"])
        build_ms_l.append(r.timings["kernel_ms"])
    ctx.sync()
    dt = time.perf_counter() - t0
    ms = dt / a.steps * 1e3
    count = r.count

    ok = (count == R and r.fmt == a.fmt)
    mism = -1
    if a.check:
        if a.fmt == "fastq":
            mism = sf.check_rows(rows, 0, count)
        else:  # FASTA: the '\n' padding belongs to the last record (fasta.go EOF piece)
            mism = sf.check_rows(rows, 0, count - 1)
            last = rows.download(16, 16 * (count - 1)).view(np.uint64)
            off_last = int(sf.d_off.download(8, 8 * (count - 1)).view(np.uint64)[0])
            mism += int(not (last[0] == off_last and last[1] == size - off_last))
        ok = ok and mism == 0

    k_ms = float(np.mean(idx_ms))
    build_ms = float(np.mean(build_ms_l))
    ntiles = (size + TILE - 1) // TILE
    kernel = fastq_kernel() if a.fmt == "fastq" else fasta_kernel()
    # algorithmic bytes of ONE launch of the dominant kernel: the input once, plus what it writes
    # -- the tile passes write one packed u64 per tile and a u16 per record (FASTQ: + the end of
    # the tile's last record; FASTA: one per boundary candidate, about one per record); the
    # two-pass kernel writes the final 16-B rows
    if kernel == "k_fq_tiles":
        alg_bytes = size + 2 * count + 10 * ntiles
    elif kernel == "k_fa_tiles":
        alg_bytes = size + 2 * count + 8 * ntiles
    else:
        alg_bytes = size + 16 * count
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    build_bytes = size + 16 * count  # the whole build: input read once, final rows written
    cfg = {"workload": f"{a.fmt} record index, {a.size_gib:g} GiB synthetic node file in HBM (BASELINE configs[1])"
           if a.fmt == "fastq" else f"fasta record index, {a.size_gib:g} GiB (BASELINE configs[2])",
           "records": count, "bytes": size, "tile": TILE, "parallelism": "single slab",
           "exchange": "none (one slab: no collective)"}
    traffic = None  # the newest round's summary taken on these kernel sources (--pmc: that file only)
    for path in ([a.pmc] if a.pmc else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{a.fmt}.json")),
                                                reverse=True)):
        traffic = load_pmc(path, {"fmt": a.fmt, "bytes": size}, kernel)
        if traffic is not None:
            break
    out = {
        "metric": METRIC,
        "value": round(size / (ms * 1e-3) / GIB, 2),
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated, seed 0x5EED, SURVEY.md §8(d))",
        "config": cfg,
        "mrecords_per_s": round(count / (ms * 1e-3) / 1e6, 2),
        "index_kernel_ms": round(k_ms, 4),
        "rccl_ranks": 0,  # (N > 1: the ranks the summary all-gather's communicator spans, dist.rccl_report)
        "fixups": r.fixups, "fixup_tiles": r.fix_tiles,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": kernel, "kernel_ms": round(k_ms, 4), "algorithmic_bytes": alg_bytes},
        # every kernel of the build (scan, placement, fix-ups, finalize included), device events
        "build": {"kernel_ms": round(build_ms, 4), "bytes": build_bytes,
                  "achieved": round(build_bytes / (build_ms * 1e-3) / 1e9, 1),
                  "frac": round(build_bytes / (build_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "parity": {"rows_checked": count if a.check else 0, "mismatches": mism, "count_ok": count == R},
    }
    if a.floor:  # after the timed region: the box's own streaming floor for the tile passes' reads
        f_ms = sf.stream_floor(data, size)
        out["box_floor"] = {"kernel": "k_stream_floor (tile-pass staging alone: no parsing, no stores)",
                            "ms": round(f_ms, 4), "achieved": round(size / (f_ms * 1e-3) / 1e9, 1),
                            "frac": round(size / (f_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                            "kernel_over_floor": round(k_ms / f_ms, 4)}
    if a.cpu_sec > 0:
        sample_n = min(size, int(a.cpu_sample_gib * GIB))
        k = sf._count_le(sample_n) - 1  # cut the sample at a record boundary
        sample_n = int(sf.d_off.download(8, 8 * k).view(np.uint64)[0]) if k > 0 else sample_n
        host = data.download(sample_n)
        # one piece per leased host core (the GPU box leases 16; os.cpu_count() shows the machine)
        nth = max(1, min(16, os.cpu_count() or 1))
        kk = max(k, 1)
        idx = [int(kk * i // nth) for i in range(nth)]
        offs = sf.d_off.download(8 * (kk + 1)).view(np.uint64)
        cuts = sorted(set([int(offs[i]) for i in idx] + [sample_n]))
        out["cpu_baseline"] = cpu_baseline(host, a.fmt, a.cpu_sec, cuts)
    print(json.dumps(out))
    if not ok:
        print(f"PARITY FAILURE: count {count} expected {R}, mismatches {mism}, status {r.status} "
              f"err {r.err} state_out {r.state_out} term {r.term_code} flags {r.flags}", file=sys.stderr)
        return 1
    return 0


def line_bench(a, ctx, sf, data, size):
    """The line indexer (index/line.go:33-85) over the synthetic file: one row per '\\n' + 1."""
    host_nl = None
    cap = size // 8 + 1024
    rows = ctx.alloc(16 * cap)
    for _ in range(a.warmup):
        r = ctx.build_buffer(data, size, rows, kind="line")
    ks, bs, t0 = [], [], time.perf_counter()
    for _ in range(a.steps):
        r = ctx.build_buffer(data, size, rows, kind="line")
        ks.append(r.timings["index_ms"])
        bs.append(r.timings["kernel_ms"])
    ctx.sync()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    k_ms, b_ms = float(np.mean(ks)), float(np.mean(bs))
    tiles = os.environ.get("SHOCKIDX_LINE_MODE", "") not in ("two", "0")
    ntiles = (size + TILE - 1) // TILE
    # k_line_tiles writes 2-B '\n' positions and 16 B per tile; k_index1 the final 16-B rows
    kernel = "k_line_tiles" if tiles else "k_index1"
    alg = size + 2 * r.count + 16 * ntiles if tiles else size + 16 * r.count
    # parity (size-independent properties): rows tile the file, every row but the last ends in '\n'
    tab = rows.rows(r.count)
    ok = r.ok and int(tab[0, 0]) == 0 and bool(np.all(tab[1:, 0] == tab[:-1, 0] + tab[:-1, 1])) and \
        int(tab[-1, 0] + tab[-1, 1]) == size
    ends = tab[:-1, 0] + tab[:-1, 1] - 1
    pick = np.random.default_rng(2).choice(len(ends), size=min(2000, len(ends)), replace=False)
    ok = ok and all(data.download(1, int(ends[i]))[0] == 10 for i in pick.tolist())
    floor = None
    if a.floor:
        f_ms = sf.stream_floor(data, size)
        floor = {"kernel": "k_stream_floor (tile-pass staging alone: no parsing, no stores)", "ms": round(f_ms, 4),
                 "achieved": round(size / (f_ms * 1e-3) / 1e9, 1), "kernel_over_floor": round(k_ms / f_ms, 4)}
    print(json.dumps({"metric": "device-resident line index build (index/line.go)", "box_floor": floor, "value": round(size / (ms * 1e-3) / GIB, 2),
                      "unit": "GiB/s", "fmt": a.fmt, "bytes": size, "rows": r.count, "ms_per_step": round(ms, 4),
                      "index_kernel_ms": round(k_ms, 4), "mrows_per_s": round(r.count / (ms * 1e-3) / 1e6, 2),
                      "roofline": {"bound": "hbm", "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                   "kernel": kernel, "algorithmic_bytes": alg},
                      "build": {"kernel_ms": round(b_ms, 4), "bytes": size + 16 * r.count,
                                "frac": round((size + 16 * r.count) / (b_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                      "parity_ok": bool(ok)}))
    return 0 if ok else 1


def chunk_bench(a, ctx, sf, data, size):
    """The chunkrecord indexer (index/chunkrecord.go:41-99) over the synthetic file.  Parity: the
    whole table against the C oracle run on the downloaded file (its time is the CPU baseline)."""
    cap = ctx.chunkrecord_capacity(size)
    rows = ctx.alloc(16 * cap)
    for _ in range(a.warmup):
        r = ctx.chunkrecord_buffer(data, size, rows, fmt=a.fmt)
        assert r.ok, r
    ks, t0 = [], time.perf_counter()
    for _ in range(a.steps):
        r = ctx.chunkrecord_buffer(data, size, rows, fmt=a.fmt)
        ks.append(r.timings["index_ms"])
    ctx.sync()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    k_ms = float(np.mean(ks))
    serial = os.environ.get("SHOCKIDX_CHUNK_MODE") == "serial"
    # the reference reads one 32 KiB window and writes one row per chunk; the speculative
    # build also reads the whole file once (FASTQ record index / FASTA "\n>" positions)
    alg = r.count * (32768 + 16) + (0 if serial else size)
    tab = rows.rows(r.count)
    out = {"metric": "device-resident chunkrecord index build (index/chunkrecord.go)",
           "value": round(size / (ms * 1e-3) / GIB, 2), "unit": "GiB/s", "fmt": a.fmt, "bytes": size,
           "rows": r.count, "ms_per_step": round(ms, 4), "index_kernel_ms": round(k_ms, 4),
           "us_per_chunk": round(k_ms * 1e3 / max(r.count, 1), 3),
           "mode": "serial walk" if serial else "speculative (path over predicted chunk starts, every chunk verified)",
           "path_rounds": r.reruns,
           "roofline": {"bound": "latency (serial chunk chain)" if serial else "hbm",
                        "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes": alg}}
    ok = r.ok
    if a.check:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))
        import oracle  # checker + CPU baseline only
        host = data.download(size)
        c0 = time.perf_counter()
        exp, err = oracle.chunkrecord(host, a.fmt)
        cpu_s = time.perf_counter() - c0
        ok = ok and err is None and len(exp) == r.count and bool(np.array_equal(tab, exp))
        out["parity"] = {"rows_checked": int(len(exp)), "identical": bool(ok)}
        out["cpu_baseline"] = {"value": round(size / cpu_s / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": f"whole {size / GIB:.1f} GiB file, oracle/chunk_oracle.c, 1 thread, {cpu_s:.2f} s"}
    print(json.dumps(out))
    return 0 if ok else 1


def filter_bench(a, ctx, sf, data, size):
    """A download filter (node/filter/filter.go:13-33: fq2fa, anonymize) over the whole device-
    resident section.  Parity: the output for a prefix cut at a record boundary against the C
    oracle (the outputs of a prefix are a prefix of the outputs); its time is the CPU baseline."""
    name = a.filter
    if a.fmt == "fasta" and name != "anonymize":
        raise SystemExit("fq2fa applies to FASTQ sections only")
    cap = size + size // 2 + (64 << 20)
    d_out = ctx.alloc(cap)
    for _ in range(a.warmup):
        r = ctx.filter_device(name, data.ptr, size, d_out.ptr, cap)
        assert r.ok, r
    ks, t0 = [], time.perf_counter()
    for _ in range(a.steps):
        r = ctx.filter_device(name, data.ptr, size, d_out.ptr, cap)
        ks.append(r.kernel_ms)
    ctx.sync()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    k_ms = float(np.mean(ks))
    alg = size + r.size  # the section read once, the filtered stream written once
    out = {"metric": f"download filter {name} over a device-resident {a.fmt} section (node/filter)",
           "value": round(size / (ms * 1e-3) / GIB, 2), "unit": "GiB/s (input bytes / wall)", "fmt": a.fmt, "filter": name,
           "bytes": size, "records": r.count, "out_bytes": r.size, "ms_per_step": round(ms, 4),
           "kernel_ms": round(k_ms, 4),
           "roofline": {"bound": "hbm", "kernel": "all kernels of the filter (device events)",
                        "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes": alg}}
    ok = r.ok
    if a.check:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))
        import oracle  # checker + CPU baseline only
        k = sf._count_le(min(size, int(a.cpu_sample_gib * GIB))) - 1
        cut = int(sf.d_off.download(8, 8 * k).view(np.uint64)[0])
        host = data.download(cut).tobytes()
        c0 = time.perf_counter()
        exp, n, err = oracle.filter_fastq(host, name)
        cpu_s = time.perf_counter() - c0
        got = d_out.download(len(exp)).tobytes() if exp else b""
        ok = ok and err is None and got == exp
        out["parity"] = {"prefix_bytes": cut, "prefix_records": n, "identical": bool(got == exp)}
        out["cpu_baseline"] = {"value": round(cut / cpu_s / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": f"first {cut / GIB:.2f} GiB (cut at a record boundary), oracle/filter_oracle.c, 1 thread"}
    d_out.free()
    print(json.dumps(out))
    return 0 if ok else 1


def subset_bench(a, ctx, sf, data, size, R):
    """configs[3]: the record index of a device-resident FASTQ node, then a subset node of a
    sorted random sample of its records (index/subset.go:133-303) and its bytes (single.go:500-517)."""
    rows = ctx.alloc(16 * (R + 1024))
    r = ctx.build_buffer(data, size, rows, kind="record", fmt="fastq")
    assert r.ok and r.count == R, r
    rng = np.random.default_rng(0x5EED)
    k = max(1, int(R * a.subset_frac))
    ids = np.sort(rng.choice(R, size=k, replace=False) + 1)
    text = ("\n".join(map(str, ids.tolist())) + "\n").encode()
    d_ids = ctx.alloc(len(text) + 64)
    d_ids.upload(text)
    cap = k + 16
    d_sub = ctx.alloc(16 * cap)
    d_runs = ctx.alloc(16 * cap)
    res = None
    for _ in range(a.warmup):
        res = ctx.subset_index(d_ids.ptr, len(text), rows.ptr, R, R, d_sub.ptr, cap, d_runs.ptr, cap)
    assert res.ok, res
    d_out = ctx.alloc(res.size + 64)
    for _ in range(a.warmup):
        g = ctx.subset_gather(data.ptr, size, d_runs.ptr, res.runs, d_out.ptr, res.size)
    ti, tg, ki, kg = [], [], [], []
    for _ in range(a.steps):  # the two calls
        t0 = time.perf_counter()
        res = ctx.subset_index(d_ids.ptr, len(text), rows.ptr, R, R, d_sub.ptr, cap, d_runs.ptr, cap)
        t1 = time.perf_counter()
        g = ctx.subset_gather(data.ptr, size, d_runs.ptr, res.runs, d_out.ptr, res.size)
        t2 = time.perf_counter()
        ti.append(t1 - t0); tg.append(t2 - t1); ki.append(res.kernel_ms); kg.append(g.kernel_ms)
    tn, kn, gn = [], [], []
    for _ in range(a.steps):  # the same as one call (shockidx_subset_node: counts stay on the device)
        t0 = time.perf_counter()
        nd = ctx.subset_node(d_ids.ptr, len(text), rows.ptr, R, R, d_sub.ptr, cap, d_runs.ptr, cap, data.ptr, size,
                             d_out.ptr, res.size + 64)
        tn.append(time.perf_counter() - t0); kn.append(nd.kernel_ms); gn.append(nd.gather_ms)
    node_ok = nd.ok and nd.count == res.count and nd.size == res.size and nd.runs == res.runs
    # parity: rows = parent rows of the ids; bytes = the records' bytes (checked on a sample)
    got = d_sub.rows(res.count)
    exp = rows.rows(R)[ids - 1]
    ok = res.ok and g.ok and res.count == k and np.array_equal(got, exp) and g.size == int(exp[:, 1].sum())
    runs = d_runs.rows(res.runs)
    pick = np.random.default_rng(1).choice(res.runs, size=min(200, res.runs), replace=False)
    outoff = np.concatenate([[0], np.cumsum(runs[:, 1])])
    for i in pick.tolist():
        o, n = int(runs[i, 0]), int(runs[i, 1])
        ok = ok and data.download(n, o).tobytes() == d_out.download(n, int(outoff[i])).tobytes()
    gms = float(np.mean(gn))
    ok = ok and node_ok
    alg = 2 * g.size + 16 * res.count * 2 + 16 * res.runs  # SURVEY §8(d) C4 algorithmic bytes
    gather_bytes = 2 * g.size + 16 * res.runs
    out = {"metric": "subset node from a device-resident FASTQ index (BASELINE configs[3])",
           "value": round(g.size / float(np.mean(tn)) / GIB, 3),
           "unit": "GiB/s (subset bytes / wall of shockidx_subset_node: index + gather in one call)",
           "fmt": "fastq", "bytes": size, "records": R, "ids": k, "runs": res.runs, "subset_bytes": g.size,
           "node_ms": round(float(np.mean(tn)) * 1e3, 3), "node_index_kernel_ms": round(float(np.mean(kn)), 3),
           "two_calls_gib_s": round(g.size / (np.mean(ti) + np.mean(tg)) / GIB, 3),
           "index_ms": round(float(np.mean(ti)) * 1e3, 3), "index_kernel_ms": round(float(np.mean(ki)), 3),
           "gather_ms": round(float(np.mean(tg)) * 1e3, 3), "gather_kernel_ms": round(gms, 4),
           "gather_kernel_ms_two_calls": round(float(np.mean(kg)), 4),
           "roofline_gather": {"bound": "hbm", "achieved": round(gather_bytes / (gms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(gather_bytes / (gms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
           "algorithmic_bytes": alg, "parity_ok": bool(ok), "steps": a.steps}
    print(json.dumps(out))
    return 0 if ok else 1


def e2e(a, ctx, sf, data, size, R):
    """End-to-end rate of shockidx_build_host: the file starts and ends in host memory
    (a POSTed body): chunked H2D through pinned staging, index kernels, table D2H."""
    host = data.download(size)
    data.free()
    sf.free()
    if a.fd:
        return e2e_fd(a, ctx, host, size, R)
    if a.pinned:  # a node body kept pinned in host memory (registered once, outside the timed region)
        ctx.host_register(host)
    for _ in range(a.warmup):
        r = ctx.build_host(host, kind="record")
    t, parts, paths = [], [], []
    for _ in range(a.steps):
        r = None  # the previous table is the caller's to free, outside this build
        t0 = time.perf_counter()
        r = ctx.build_host(host, kind="record")
        t.append(time.perf_counter() - t0)
        parts.append(r.timings)
        paths.append(r.path)
    if a.pinned:
        ctx.host_unregister(host)
    ms = float(np.mean(t)) * 1e3
    avg = {k: round(float(np.mean([p[k] for p in parts])), 3) for k in parts[0]}
    print(json.dumps({"metric": "end-to-end index build from host memory (PCIe-inclusive)", "value": round(size / (ms * 1e-3) / GIB, 3),
                      "unit": "GiB/s", "ms_per_step": round(ms, 3), "steps": a.steps, "fmt": a.fmt, "bytes": size,
                      "records": r.count, "count_ok": r.count == R, "ok": r.ok, "timings_ms": avg,
                      # which build the timed calls ran (result.path 3 = the slab pipeline)
                      "pipeline": "slab" if all(p == 3 for p in paths) else "one-pass",
                      "path": ("pinned (hipHostRegister'ed) host buffer -> 1 GiB slabs H2D on a copy stream, each indexed "
                               "as soon as it and a 4 MiB halo have arrived, its rows D2H while later slabs cross PCIe; " if a.pinned else
                               "pageable host buffer -> threaded memcpy into 2 x 64 MiB pinned staging -> hipMemcpyAsync H2D (double-buffered); ")
                              + "table D2H through the pinned staging, DMA overlapped with the host copy"}))
    return 0 if (r.ok and r.count == R) else 1


def e2e_fd(a, ctx, host, size, R):
    """The drop-in path end to end: Indexers["record"](f).Create(out) -> shockidx_create(fd)
    over a page-cached node file (pread by the copy threads into pinned staging, H2D, index,
    table D2H, .idx written via temp + rename); build_fd alone (no .idx write) timed too."""
    import tempfile
    d = tempfile.mkdtemp(dir="/tmp", prefix="shockidx_e2e_")
    path = os.path.join(d, "node.fastq")
    try:
        host.tofile(path)
        del host
        fd = os.open(path, os.O_RDONLY)
        with open(path, "rb") as f:  # page-cache the node file
            while f.read(1 << 28):
                pass
        trims = []
        if a.dev_cap is not None:  # (the synthetic node was freed from HBM above)
            ctx.set_dev_cap(int(a.dev_cap * GIB))

        def trim():  # the shim's pool between builds (outside the call's time, timed apart)
            if a.trim is not None:
                t0 = time.perf_counter()
                ctx.trim(int(a.trim * GIB))
                trims.append(time.perf_counter() - t0)

        for _ in range(a.warmup):
            r = ctx.build_fd(fd, size)
            trim()
        t, parts = [], []
        for _ in range(a.steps):
            r = None
            t0 = time.perf_counter()
            r = ctx.build_fd(fd, size)
            t.append(time.perf_counter() - t0)
            parts.append(r.timings)
            trim()
        ok = r.ok and r.count == R
        r_path = r.path  # 3: the whole node in HBM, 4: two slab slots within the cap
        r = None
        tc = []
        for _ in range(max(1, a.steps // 2)):
            out = os.path.join(d, "record.idx")
            t0 = time.perf_counter()
            rc = ctx.create(fd, size, "record", d, out)
            tc.append(time.perf_counter() - t0)
            trim()
            ok = ok and rc.ok and rc.count == R and os.path.getsize(out) == 16 * R
            os.unlink(out)
        ws_after = ctx.workspace_bytes()
        os.close(fd)
    finally:
        import shutil
        shutil.rmtree(d, ignore_errors=True)
    ms = float(np.mean(t)) * 1e3
    cms = float(np.mean(tc)) * 1e3
    avg = {k: round(float(np.mean([p[k] for p in parts])), 3) for k in parts[0]}
    print(json.dumps({"metric": "end-to-end index build from a page-cached node file (PCIe-inclusive)",
                      "value": round(size / (ms * 1e-3) / GIB, 3), "unit": "GiB/s", "ms_per_step": round(ms, 3),
                      "create_ms": round(cms, 3), "create_gib_s": round(size / (cms * 1e-3) / GIB, 3),
                      "steps": a.steps, "fmt": a.fmt, "bytes": size, "records": R, "ok": ok, "timings_ms": avg,
                      "trim_gib": a.trim, "trim_ms": round(float(np.mean(trims)) * 1e3, 3) if trims else None,
                      "workspace_bytes_after_last_call": ws_after,
                      "dev_cap_gib": a.dev_cap, "build_path": int(r_path),
                      "path": ("shockidx_build_fd: 1 GiB slabs indexed as they arrive; " +
                               ("the file pread by the copy threads into 2 x 64 MiB pinned staging, then H2D"
                                if os.environ.get("SHOCKIDX_NO_MMAP_DMA") else
                                "the page-cached file mapped and pinned 256 MiB at a time, DMA'd straight to HBM") +
                               "; rows D2H per slab; create_ms: shockidx_create (the same + each slab's rows written "
                               "into the temp .idx as they come back, then renamed)")}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
