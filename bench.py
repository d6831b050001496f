#!/usr/bin/env python3
"""Benchmark: recordio v4 whole-file decode, device-resident (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): one recordio v4 file of 1,000,000 x 1 KiB Snappy
records per GPU (text-like synthetic records, seeded per rank), already in
HBM when the timed region starts. One step = one complete decode of that file: framing (header
walk + CRC-32C), scan, placement and Snappy decode into a preallocated arena — the full
rio_device_decode call. value = input file bytes decoded by all ranks / max-over-ranks time, GiB/s.

Multi-GPU: one process per GPU (torchrun); every rank decodes its own file (file sharding, no
data-path collective; the only collectives are the timing barrier and the max-over-ranks).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2r|c2x|c2g|c2l|c1|c1s|c3|c4|c5|wal|idx|enc|readat]

c5 (SSTable load + validation + scan), wal (ordered WAL replay from host files) idx (batched
DiskKeyIndex.Get) and enc (device v4 encode) print their own
metric lines; the default (c2) line is the BASELINE.json metric.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "go-sstables_amd"))

METRIC = "recordio decode GiB/s (device-resident), v4 1 KiB records, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md

# WAL replay: 8 rotated WAL files of ~128 MiB (DefaultMaxWalSize, write_ahead_log.go:9),
# 1 KiB text-like snappy records, replayed from the page cache into host memory
WAL_FILES, WAL_RECORDS_PER_FILE = 8, 230_000

CONFIGS = {
    # name: (records, record_bytes, compression, kind, description)
    "c2": (1_000_000, 1024, 2, 1, "C2: recordio v4, 1M x 1 KiB snappy records (text-like), one file per GPU"),
    "c2r": (1_000_000, 1024, 2, 0, "C2-ref-random: recordio v4, 1M x 1 KiB snappy records (incompressible)"),
    "c2x": (9_000_000, 1024, 2, 1, "C2 past 4 GiB: recordio v4, 9M x 1 KiB snappy records (text-like), a 4.6 GB file "
                                   "(the read benchmark's largest sizes, recordio_read_test.go:26-27)"),
    "c1": (100_000, 1024, 0, 0, "C1: recordio v4, 100k x 1 KiB uncompressed records (ref generator)"),
    "c1s": (32_389, 1024, 0, 0, "C1 at the read benchmark's smallest size: recordio v4, a 32 MiB file of 1 KiB "
                                "uncompressed records (recordio_read_test.go:19: records written until the file "
                                "reaches 32 MiB)"),
    "c3": (10_000_000, 64, 2, 1, "C3: recordio v4, 10M x 64 B snappy records (header-bound)"),
    "c4": (16_384, 65536, 2, 1, "C4: recordio v4, 8 files x 16384 x 64 KiB snappy records (decompress-bound), "
                                "sharded over the GPUs"),
    "c2g": (1_000_000, 1024, 1, 1, "C2-gzip: recordio v4, 1M x 1 KiB gzip records (text-like), one file per GPU"),
    "c2l": (1_000_000, 1024, 3, 1, "C2-lzw: recordio v4, 1M x 1 KiB lzw records (text-like), one file per GPU"),
    "wal": (WAL_FILES * WAL_RECORDS_PER_FILE, 1024, 2, 1, "WAL replay: 8 x ~128 MiB snappy WAL files (1 KiB "
                                                          "text-like records) per GPU, sorted, delivered in order"),
    "idx": (1_000_000, 20, 0, 0, "DiskKeyIndex Get: 1M SHA1 keys (half present) against the C5 index.rio "
                                 "(1.25M entries), one lane per key"),
    "enc": (1_000_000, 1024, 2, 1, "Encode: 1M x 1 KiB text-like records -> recordio v4 snappy file image "
                                    "(FileWriter.Write batch), device-resident"),
    "readat": (1_000_000, 1024, 2, 1, "ReadAtI: ReadNextAt / SeekNext on the C2 file from host threads "
                                      "(MMapReader, mmap_reader.go:58-203)"),
    "c5": (1_250_000, 1024, 2, 0, "C5: SSTable load + validateDataFile + full scan, 1.25M SHA1 keys x 1 KiB values "
                                  "(data.rio snappy v4 + index.rio v4), one table per GPU (10M keys over 8 GPUs)"),
}
SST_METRIC = "sstable full scan GiB/s (device-resident: index load + CRC-64 validation + data decode)"
WAL_METRIC = "wal replay GiB/s (host WAL files -> ordered host records, PCIe-inclusive)"
IDX_METRIC = "DiskKeyIndex lookups/s (device-resident index.rio, batched Get)"
ENC_METRIC = "recordio v4 encode GiB/s of records (device-resident, golang/snappy block format)"
PCIE_PEAK_GBPS = 128.0  # PCIe Gen5 x16, both directions (64 GB/s each)
DECODE_KERNEL = {0: "k_copy_records", 1: "k_gzip_inflate", 2: "k_snappy_pipe", 3: "k_lzw_decode"}
# configs decoded as a fixed file set sharded over the ranks: name -> (files, first seed)
MULTI_FILE = {"c4": (8, 100)}
SST_TABLES = 8  # C5: 10M keys in 8 tables of 1.25M


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    # rehearsal of the N-rank path on a one-GPU box: every rank decodes on device 0 (never set by the
    # driver's scaling runs, where rank i owns GPU i)
    if os.environ.get("RIO_BENCH_ONE_DEVICE") == "1":
        local = 0
    return ws, rank, local


def shard_files(n_files: int, world: int, rank: int) -> list[int]:
    """File ids this rank decodes (round-robin = LPT for equal-size files)."""
    return [f for f in range(n_files) if f % world == rank]


def reduce_max(value: float, world: int, device=None) -> float:
    """Max over ranks of a host float: gloo on the CPU (the data path has no collective at all)."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value: float, world: int, device=None) -> float:
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def job_throughput(dt: float, bytes_in: float, steps: int, world: int, device=None) -> tuple[float, float, float]:
    """Whole-job rate of a file-sharded run: every rank timed its own `steps` decodes of its own
    file (`bytes_in` per step); the job took the slowest rank's time. Returns (GiB/s, ms per step,
    max time). The two all-reduces are the job's only collectives and sit outside the timed region."""
    dt_max = reduce_max(dt, world, device)
    total_in = reduce_sum(float(bytes_in * steps), world, device)
    return total_in / 2**30 / dt_max, dt_max / steps * 1e3, dt_max


def rank_seed(rank: int) -> int:
    """Seed of the synthetic file a rank decodes: one distinct file per GPU."""
    return 1 + rank


def host_cores() -> int:
    """Host threads the CPU baseline may use: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
    GPU pool), not the machine's whole count that os.cpu_count() reports there."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = os.cpu_count() or 1
    return max(1, min(n, share) if share else n)


def device_digest(t) -> str:
    """Position-sensitive digest of a device tensor's bytes, computed on the device (int64 word sums per
    4096-word row, the row sums weighted by their index, every word weighted by its place in its row; the
    tail words and bytes separately). Used to
    show that the timed steps rebuilt exactly the bytes the warmup produced."""
    import torch

    u8 = t.contiguous().view(torch.uint8).flatten()
    n = u8.numel()
    n8 = n // 8 * 8
    w = u8[:n8].view(torch.int64)
    rows = 4096
    m = w.numel() // rows * rows
    parts = [n]
    if m:
        blk = w[:m].view(-1, rows)
        rs = blk.sum(dim=1)
        wt = torch.arange(1, rs.numel() + 1, device=t.device, dtype=torch.int64) * 2654435761
        # words weighted by their place in the row too (int64 products wrap): a permutation inside a row shows
        wr = torch.arange(1, rows + 1, device=t.device, dtype=torch.int64) * 0x9E3779B97F4A7C1
        parts += [int(rs.sum().item()), int((rs * wt).sum().item()), int((blk * wr).sum().item())]
    if w.numel() > m:
        tail = w[m:]
        wt = torch.arange(1, tail.numel() + 1, device=t.device, dtype=torch.int64) * 40503
        parts += [int(tail.sum().item()), int((tail * wt).sum().item())]
    if n > n8:
        parts += [int(x) for x in u8[n8:].cpu().tolist()]
    return "%x" % (hash(tuple(parts)) & (2**64 - 1))


def source_tree_hash(root: str = HERE) -> str:
    """sha1 of the product sources (go-sstables_amd/csrc/*.hip|*.cpp|*.h and include/*.h): the tree a
    traffic file was measured on, recorded in it by scripts/traffic.py and compared here."""
    import glob
    import hashlib

    h = hashlib.sha1()
    files = sorted(glob.glob(os.path.join(root, "go-sstables_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(root, "go-sstables_amd", "csrc", "*.cpp")) +
                   glob.glob(os.path.join(root, "go-sstables_amd", "csrc", "*.h")) +
                   glob.glob(os.path.join(root, "include", "*.h")))
    for f in files:
        h.update(os.path.relpath(f, root).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def dominant_kernel(config: str, rec_len: int | None = None) -> str:
    """The decode kernel the roofline is taken on for a decode config (rec_len: a test's override)."""
    _, rl, comp, kind, _ = CONFIGS[config]
    rec_len = rl if rec_len is None else rec_len
    batch = config in MULTI_FILE
    if comp == 2 and kind == 0:
        return "k_copy_records"  # ref-random records are each one literal: the copy path decodes them
    if comp == 2 and rec_len >= int(os.environ.get("RIO_COOP_MIN", str(1 << 56)), 0):
        return "k_snappy_coop_batch" if batch else "k_snappy_coop"  # wave-per-record decoder (opt-in)
    if comp == 2 and batch:
        return "k_snappy_pipe_batch"
    return DECODE_KERNEL[comp]


def pmc_counter(root: str, name: str, kernel: str) -> tuple[float, int]:
    """(max over dispatches, dispatch count) of one rocprofv3 counter for kernels whose name contains
    `kernel` (the first decode launch is a capacity probe that decodes nothing: the max is a real one)."""
    import csv
    import glob

    vals = []
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
                    vals.append(float(row["Counter_Value"]))
    return (max(vals), len(vals)) if vals else (float("nan"), 0)


def live_traffic(config: str, timeout_s: float = 300.0) -> dict:
    """HBM traffic of the dominant kernel measured now, on this box and this tree: two child runs of this
    script (2 timed steps) under `rocprofv3 --kernel-trace --pmc <one counter>`, FETCH_SIZE and
    WRITE_SIZE in separate passes (MI355X_MICROARCH.md, HBM / rocprofv3: KiB at the L2's memory side,
    FETCH_SIZE doubled on gfx950). Started before this process touches the GPU. Returns the traffic
    fields for `roofline`, or {"error": ...} when the profiler is missing or a pass fails."""
    import shutil
    import signal
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return {"error": "rocprofv3 not found"}
    kernel = dominant_kernel(config)
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="rio_pmc_", dir="/tmp")
        cmd = [prof, "--kernel-trace", "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv", "--",
               sys.executable, os.path.abspath(__file__), "--config", config, "--steps", "2", "--warmup", "1",
               "--no-cpu-baseline", "--no-e2e", "--traffic", "none"]
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env, cwd="/tmp",
                             start_new_session=True)
        try:
            rc = p.wait(timeout=timeout_s)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            shutil.rmtree(d, ignore_errors=True)
            return {"error": f"{ctr} pass timed out after {timeout_s:.0f} s"}
        v, k = pmc_counter(d, ctr, kernel)
        shutil.rmtree(d, ignore_errors=True)
        if rc != 0 or k == 0:
            return {"error": f"{ctr} pass rc={rc}, {k} dispatches of {kernel}"}
        vals[ctr] = v
    read_b, write_b = 2.0 * vals["FETCH_SIZE"] * 1024, vals["WRITE_SIZE"] * 1024
    return {"traffic": read_b + write_b, "traffic_read": read_b, "traffic_write": write_b,
            "traffic_source": {"kind": "live", "tree": source_tree_hash(), "kernel": kernel,
                               "method": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), max over dispatches, two "
                                         "rocprofv3 --pmc passes of this script run by this bench invocation"}}


def file_traffic(config: str, path: str | None) -> dict:
    """Traffic from a committed PMC file (scripts/traffic.py output), with the tree it was measured on and
    whether that is this tree."""
    for tpath in ([path] if path else [os.path.join(HERE, "profiles", f"traffic_{config}.json"),
                                       os.path.join(HERE, "profiles", "traffic_latest.json")]):
        if tpath and os.path.exists(tpath):
            try:
                tj = json.load(open(tpath))
            except (OSError, ValueError):
                continue
            if tj.get("config") == config:
                now = source_tree_hash()
                return {"traffic": tj.get("decode_kernel_bytes_per_launch"),
                        "traffic_source": {"kind": "file", "path": os.path.relpath(tpath, HERE),
                                           "tree": tj.get("tree"), "tree_now": now,
                                           "same_tree": tj.get("tree") == now}}
    return {"traffic": None}


def cpu_baseline(images, rec_offs=None, n_records=None, budget_s: float = 20.0, check=None) -> dict:
    """The oracle (oracle/rio_oracle.c, a C restatement of the reference reader) on host cores, timed
    on a bounded sample of the same workload:
      one core  — FileReader.ReadNext loop over one file (orc_file_reader_decode), sequential;
      all cores — MMapReader.ReadNextAt record-parallel over each file's known offset table
                  (orc_parallel_read_at), the files one after another.
    check(out, out_off, rec_off, flags): called once with the oracle's arrays of images[0] from the first
    one-core run (outside its timing), so the device result the bench timed is compared with the oracle
    on the full file (`verified` as a correctness claim, not only warmup-vs-timed reproducibility)."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import numpy as np
    import oracle_py as orc

    lib = orc.lib()
    image = images[0]
    checked = None

    def one_file(img, keep):
        nonlocal checked
        res = orc.OrcFileResult()
        t0 = time.perf_counter()
        lib.orc_file_reader_decode(img.ctypes.data, img.shape[0], ctypes.byref(res))
        dt = time.perf_counter() - t0
        n, nb = res.n_records, res.total_out_bytes
        if keep:
            def arr(ptr, cnt, dt_):
                return np.ctypeslib.as_array(ptr, shape=(cnt,)).view(dt_) if cnt else np.zeros(0, dt_)
            checked = check(arr(res.out, nb, np.uint8), arr(res.out_off, n + 1, np.uint64),
                            arr(res.rec_off, n, np.uint64), arr(res.flags, n, np.uint8))
        lib.orc_file_result_free(ctypes.byref(res))
        return n, dt

    runs, t_total = 0, 0.0
    while runs < 5 and t_total < budget_s:
        got, dt = one_file(image, check is not None and runs == 0)
        t_total += dt
        runs += 1
        if n_records is not None and got != n_records:
            raise RuntimeError("oracle baseline decoded a different record count")
    one = image.shape[0] / 2**30 * runs / t_total
    cores = host_cores()

    # all cores: MMapReader.ReadNextAt record-parallel over every file's known offset table, the files
    # one after another, so a set of fewer files than cores (C4: 8 files, 16 cores) still uses the
    # whole CPU share (one thread per file left half of it idle)
    offs = [np.ascontiguousarray(ro, dtype=np.uint64) for ro in (rec_offs if len(images) > 1 else [rec_offs])]
    runs_a, t_a = 0, 0.0
    while runs_a < 5 and t_a < budget_s:
        t0 = time.perf_counter()
        for img, ro in zip(images, offs):
            if not lib.orc_parallel_read_at(img.ctypes.data, img.shape[0], ro.ctypes.data, ro.shape[0], cores):
                raise RuntimeError("oracle parallel ReadNextAt failed")
        t_a += time.perf_counter() - t0
        runs_a += 1
    all_v = sum(img.shape[0] for img in images) / 2**30 * runs_a / t_a
    used = cores
    how = (f"ReadNextAt over the known record offsets of {len(images)} file(s) "
           f"({sum(o.shape[0] for o in offs)} records), {cores} threads, x{runs_a} runs")
    res = {"value": round(all_v, 4), "unit": "GiB/s", "cores": used, "kind": "port",
           "sample": f"{how}; {os.cpu_count()} cpus visible on the host, CPU share {cores}, {_cpu_model()}",
           "one_core": {"value": round(one, 4), "unit": "GiB/s", "cores": 1,
                        "sample": f"one file ({image.shape[0]} B) x{runs} runs, sequential FileReader.ReadNext-loop "
                                  "restatement"}}
    if check is not None:
        res["oracle_match"] = checked
    return res


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown cpu"


def e2e_rate(image, n_out_bytes: int) -> dict:
    """PCIe-inclusive rates (never `value`). GiBps_input is the path the cgo FileReader takes
    for a file of this size (rocmStreamReader, 128 MiB windows through rio_stream_*:
    one window's H2D overlapping earlier windows' decode and D2H, records handed over in place in
    page-locked memory), from a host image; beside it the same from the file in the page cache
    (rio_stream_open: pread into the staging), other window sizes, and the one-shot pair
    (rio_frame + rio_decode: the whole file's H2D, then decode + D2H)."""
    from recordio import _lib as L
    import numpy as np

    lib = L.lib()
    dev = int(os.environ.get("LOCAL_RANK", "0"))
    ctx = L.default_ctx(dev)
    fi = L.FileInfo()
    out = np.empty(n_out_bytes + 16, dtype=np.uint8)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        rc = lib.rio_frame(ctx, image.ctypes.data, image.shape[0], ctypes.byref(fi))
        n = fi.n_records
        out_off = np.empty(n + 1, dtype=np.uint64)
        rec_off = np.empty(n + 1, dtype=np.uint64)
        flags = np.empty(n + 1, dtype=np.uint8)
        rc |= lib.rio_decode(ctx, out.ctypes.data, out.shape[0], out_off.ctypes.data, rec_off.ctypes.data,
                             flags.ctypes.data, n, ctypes.byref(fi))
        times.append(time.perf_counter() - t0)
        if rc:
            return {"error": L.strerror(rc)}
    t_one = min(times)

    def stream(open_fn, wbytes):
        best, nwin = None, 0
        for rep in range(6):  # the first run warms the context pool and the page-locked block cache
            h = ctypes.c_void_p()
            t0 = time.perf_counter()
            rc = open_fn(wbytes, h)
            got, nwin = 0, 0
            while rc == 0:
                first, info = ctypes.c_uint64(), L.FileInfo()
                p = [ctypes.c_void_p() for _ in range(4)]
                rc = lib.rio_stream_next(h, ctypes.byref(first), *[ctypes.byref(x) for x in p], ctypes.byref(info))
                if rc == 0:
                    got += info.n_records
                    nwin += 1
            dt = time.perf_counter() - t0
            lib.rio_stream_free(h)
            if rc != L.RIO_EOF or got != n:
                raise RuntimeError(f"{L.strerror(rc)} after {got} records")
            if rep:
                best = dt if best is None else min(best, dt)
        return {"GiBps_input": round(image.shape[0] / 2**30 / best, 3), "windows": nwin, "seconds": round(best, 4),
                "runs": 5}

    def from_host(wbytes, h):
        return lib.rio_stream_open_host(dev, image.ctypes.data, image.shape[0], wbytes, 4, ctypes.byref(h))

    res = {}
    try:
        windowed = {f"{w}MiB": stream(from_host, w << 20) for w in (64, 128, 256)}
        # the same with the image page-locked by the caller once (rio_host_register, outside the timing):
        # each window's H2D is a DMA from the image in place, no staging copy
        if lib.rio_host_register(image.ctypes.data, image.shape[0]) == 0:
            try:
                registered = {f"{w}MiB": stream(from_host, w << 20) for w in (128, 256)}
            finally:
                lib.rio_host_unregister(image.ctypes.data)
        else:
            registered = {"error": "rio_host_register failed"}
        path = os.path.join("/dev/shm" if os.path.isdir("/dev/shm") else "/tmp", f"rio_e2e_{os.getpid()}.rio")
        try:
            image.tofile(path)
            from_file = stream(lambda wbytes, h: lib.rio_stream_open(dev, path.encode(), wbytes, 4, ctypes.byref(h)),
                               128 << 20)
        finally:
            if os.path.exists(path):
                os.unlink(path)
    except RuntimeError as e:
        return {"error": f"windowed: {e}"}
    res["GiBps_input"] = windowed["128MiB"]["GiBps_input"]
    res["path"] = ("FileReader's path for this file size: rio_stream_open_host, 128 MiB windows (ramped), "
                   "3 contexts; host image -> pinned staging H2D -> frame -> decode -> D2H into page-locked blocks")
    res["windowed"] = windowed
    res["registered_host_image"] = registered
    if "128MiB" in registered:
        res["GiBps_input_registered"] = max(v["GiBps_input"] for v in registered.values())
    res["from_file_page_cache_128MiB"] = from_file
    res["one_shot"] = {"GiBps_input": round(image.shape[0] / 2**30 / t_one, 3), "seconds": round(t_one, 4),
                       "note": "rio_frame + rio_decode: whole-file H2D, then decode + D2H into pageable arrays"}
    return res


def sstable_images(n: int, rank: int):
    """Config 5 (benchmark/sstable_read_test.go:134-158): keys = SHA1 of the big-endian u32 index,
    sorted (the memstore flush), every value the same random 1 KiB record; data.rio Snappy v4 and
    index.rio uncompressed v4 as sstable_writer.go writes them. One table per rank (disjoint keys)."""
    import hashlib
    import struct

    import numpy as np

    from sstables.proto import encode_index_entry
    from sstables.writer import _Image, crc64_iso

    keys = sorted(hashlib.sha1(struct.pack(">I", rank * n + i)).digest() for i in range(n))
    value = np.random.default_rng(rank_seed(rank)).integers(0, 256, 1024, dtype=np.uint8).tobytes()
    one = _Image(2)
    one.write(value)
    img = one.bytes()
    rec = img[8:]
    data = np.frombuffer(img[:8] + rec * n, dtype=np.uint8)
    cs = crc64_iso(value)
    # an uncompressed v4 record's header depends only on its length: encode it once per length
    hdr = {}
    parts = [_Image(0).bytes()]
    for i, k in enumerate(keys):
        e = encode_index_entry(k, 8 + i * len(rec), cs)
        h = hdr.get(len(e))
        if h is None:
            one = _Image(0)
            one.write(e)
            h = hdr[len(e)] = one.bytes()[8:-len(e)]
        parts.append(h)
        parts.append(e)
    return np.frombuffer(b"".join(parts), dtype=np.uint8), data


def run_sstable(args, world, rank, local, device):
    """One step = the device work of NewSSTableReader + Scan on every table of this rank's shard of
    the 8-table set (BASELINE configs[4]: 10M keys in 8 tables): decode index.rio, parse every
    IndexEntry, decode data.rio, CRC-64 every value against its entry (rio_sst_*)."""
    import threading

    import numpy as np
    import torch

    from recordio import _lib as L
    from recordio.device import DeviceDecoder, header_codec, to_device_file

    n = CONFIGS["c5"][0]
    mine = shard_files(SST_TABLES, world, rank)
    dec = DeviceDecoder(local)
    # data.rio on a context of its own (as the reader opens index.rio and data.rio as two files): a context picks
    # its framing walk from its previous file's record sizes, which alternating 50-byte index and 1 KiB data files
    # on one context would always get wrong for the data file
    decd = DeviceDecoder(local, own_ctx=True)
    lib = L.lib()
    i64 = dict(dtype=torch.int64, device=device)
    # a real stream: the null stream's handle (0) would send the calls to the ctx's own stream and
    # the stage events would not bracket them
    stream = torch.cuda.Stream(device=device)
    sp = ctypes.c_void_p(stream.cuda_stream)
    tables = []
    for t in mine:
        index_img, data_img = sstable_images(n, t)
        T = {"index_img": index_img, "data_img": data_img}
        T["d_index"], T["li"] = to_device_file(index_img, local)
        T["d_data"], T["ld"] = to_device_file(data_img, local)
        # the files' header codecs as decode hints: only those codecs' kernels are launched
        T["ci"], T["cd"] = header_codec(index_img), header_codec(data_img)
        T["ib"], ii = dec.decode(T["d_index"], T["li"], comp=T["ci"])
        T["db"], di = decd.decode(T["d_data"], T["ld"], comp=T["cd"])
        if ii["n_records"] != n or di["n_records"] != n:
            raise RuntimeError(f"sstable decode failed: {ii} {di}")
        T["nb_d"] = di["total_out_bytes"]
        for k in ("key_off", "key_len", "value_off", "checksum", "crc"):
            T[k] = torch.empty(n, **i64)
        T["pres"], T["vres"] = torch.empty(2, **i64), torch.empty(2, **i64)
        tables.append(T)
    torch.cuda.synchronize(device)

    def step(ev=None):
        for T in tables:
            marks = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if ev is not None else None
            if marks: marks[0].record(stream)
            dec.launch(T["d_index"], T["li"], T["ib"], stream, T["ci"])
            if marks: marks[1].record(stream)
            lib.rio_sst_index_parse(dec.ctx, T["ib"].out.data_ptr(), T["ib"].out_off.data_ptr(), n,
                                    T["key_off"].data_ptr(), T["key_len"].data_ptr(), T["value_off"].data_ptr(),
                                    T["checksum"].data_ptr(), T["pres"].data_ptr(), sp)
            if marks: marks[2].record(stream)
            decd.launch(T["d_data"], T["ld"], T["db"], stream, T["cd"])
            if marks: marks[3].record(stream)
            lib.rio_sst_validate(dec.ctx, T["db"].out.data_ptr(), T["db"].out_off.data_ptr(),
                                 T["db"].rec_off.data_ptr(), n, T["value_off"].data_ptr(), T["checksum"].data_ptr(), n,
                                 T["crc"].data_ptr(), T["vres"].data_ptr(), sp)
            if marks:
                marks[4].record(stream)
                ev.append(marks)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)

    def digests():
        # every table's parse / validation verdicts and a digest of everything the step writes (index and data
        # records, the parsed entries, every value's CRC-64)
        out = []
        for T in tables:
            pres, vres = T["pres"], T["vres"]
            if int(pres[0].item()) != -1 or int(vres[0].item()) != -1 or int(vres[1].item()) != -1:
                raise RuntimeError(f"sstable validation failed: {pres.tolist()} {vres.tolist()}")
            out.append(tuple(device_digest(x) for x in (T["ib"].out, T["ib"].out_off, T["db"].out, T["db"].out_off,
                                                       T["key_off"], T["key_len"], T["value_off"], T["checksum"],
                                                       T["crc"])))
        return out

    want = digests()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    if digests() != want:
        raise RuntimeError("sstable bench: the timed steps did not rebuild the warmup's outputs")
    if world > 1:
        torch.distributed.barrier()
    ev = []
    for _ in range(3):
        step(ev)
    torch.cuda.synchronize(device)
    names = ("decode_index", "parse_index", "decode_data", "validate")
    nt = max(1, len(tables))
    # per table (means over tables and the 3 timed passes)
    stage = {nm: float(np.mean([m[k].elapsed_time(m[k + 1]) for m in ev])) if ev else 0.0 for k, nm in enumerate(names)}
    total_in = sum(T["li"] + T["ld"] for T in tables)
    value, ms_per_step, _ = job_throughput(dt, total_in, args.steps, world, device)
    li = tables[0]["li"] if tables else 0
    ld = tables[0]["ld"] if tables else 0
    nb_d = tables[0]["nb_d"] if tables else 0
    # dominant stage: the data decode (C2-ref-random shape) or the CRC-64 pass over the values
    alg = {"decode_data": ld + nb_d + 17 * n + 8, "validate": nb_d + 8 * 5 * n}
    dom = max(alg, key=lambda k: stage[k])
    achieved = alg[dom] / (stage[dom] * 1e-3) / 1e9 if stage[dom] else 0.0
    line = {
        "metric": SST_METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic: SHA1 keys, one random 1 KiB value (benchmark/sstable_read_test.go shape), {SST_TABLES} "
                "tables sharded over the ranks",
        "config": {"workload": CONFIGS["c5"][4], "entries_per_table": n, "tables_this_rank": len(tables),
                   "index_bytes": li, "data_bytes": ld, "decoded_value_bytes": nb_d,
                   "parallelism": f"table-sharded x{world} ({SST_TABLES} tables), no data-path collectives"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None, "kernel": dom,
                     "kernel_ms": round(stage[dom], 4), "alg_bytes_per_launch": alg[dom]},
        "stages_ms_per_table": {k: round(v, 4) for k, v in stage.items()},
        # the warmup's verdicts (every key parsed, every value's CRC-64 equal to its entry's) and device digests of all
        # the step's outputs, rebuilt identically by the timed steps
        "verified": True,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and tables:
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import oracle_py as orc

        olib = orc.lib()

        def scan(T, out):
            bad = ctypes.c_uint64()
            out.append(olib.orc_sst_scan(T["index_img"].ctypes.data, T["li"], T["data_img"].ctypes.data, T["ld"],
                                         ctypes.byref(bad)))

        one, t1 = [], time.perf_counter()
        scan(tables[0], one)
        t_one = time.perf_counter() - t1
        cores = host_cores()
        # the whole CPU share: 16 concurrent scans over the 8 tables (each table twice) when the
        # share exceeds the table count
        work = (tables * -(-cores // len(tables)))[:cores]
        got, t1 = [], time.perf_counter()
        th = [threading.Thread(target=scan, args=(T, got)) for T in work]
        for x in th:
            x.start()
        for x in th:
            x.join()
        t_all = time.perf_counter() - t1
        if one != [n] or got != [n] * len(th):
            raise RuntimeError("oracle sstable scan disagreed")
        in_all = sum(T["li"] + T["ld"] for T in work)
        line["cpu_baseline"] = {
            "value": round(in_all / 2**30 / t_all, 4), "unit": "GiB/s", "cores": len(th), "kind": "port",
            "sample": f"{len(th)} table scans run concurrently over the {len(tables)} tables, one thread each (oracle "
                      f"index load + CRC-64 validation + data decode); {os.cpu_count()} cpus visible, CPU share {cores}, "
                      f"{_cpu_model()}",
            "one_core": {"value": round((tables[0]["li"] + tables[0]["ld"]) / 2**30 / t_one, 4), "unit": "GiB/s",
                         "cores": 1, "sample": f"one table ({n} entries) scanned once"}}
    if rank == 0:
        print(json.dumps(line), flush=True)


def run_wal(args, world, rank, local, device):
    """One step = Replayer.Replay's device work over one WAL directory (rio_replay_*): map each file,
    staged H2D, device framing + decode, D2H of records / offsets / flags, files handed out in order.
    The per-record `process` callback is the caller's and is not part of the step."""
    import tempfile

    import numpy as np
    import torch

    from recordio import _lib as L
    from recordio import generate

    lib = L.lib()
    tmp = tempfile.mkdtemp(prefix=f"wal_bench_r{rank}_")
    paths, total_in, total_out = [], 0, 0
    try:
        for f in range(WAL_FILES):
            img = generate(WAL_RECORDS_PER_FILE, 1024, 2, 1, seed=rank_seed(rank) * 100 + f + 1,
                           threads=min(16, os.cpu_count() or 1))
            p = os.path.join(tmp, "%06d.wal" % f)
            img.tofile(p)
            paths.append(p)
            total_in += img.shape[0]
            total_out += WAL_RECORDS_PER_FILE * 1024
        arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])

        def replay(workers, depth):
            h = ctypes.c_void_p()
            rc = lib.rio_replay_open(local, arr, len(paths), depth, workers, ctypes.byref(h))
            if rc:
                raise RuntimeError(f"rio_replay_open: {L.strerror(rc)}")
            idx, out, off, fl, info = ctypes.c_uint64(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), \
                L.FileInfo()
            got = 0
            try:
                while True:
                    rc = lib.rio_replay_next(h, ctypes.byref(idx), ctypes.byref(out), ctypes.byref(off),
                                             ctypes.byref(fl), ctypes.byref(info))
                    if rc == L.RIO_EOF:
                        break
                    if rc or info.n_records != WAL_RECORDS_PER_FILE or idx.value != got:
                        raise RuntimeError(f"replay of file {idx.value}: rc={rc} {info.as_dict()}")
                    got += 1
            finally:
                lib.rio_replay_free(h)
            return got

        def timed(workers, depth, steps):
            if world > 1:
                torch.distributed.barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                replay(workers, depth)
            return time.perf_counter() - t0

        W, D = 2, 4
        for _ in range(args.warmup):
            replay(W, D)
        dt = timed(W, D, args.steps)
        value, ms_per_step, _ = job_throughput(dt, total_in, args.steps, world, device)
        variants = {}
        if rank == 0 and world == 1:
            for w, d in ((1, 1), (1, 4), (3, 4), (4, 6)):
                variants[f"workers{w}_depth{d}"] = round(total_in * 2 / 2**30 / timed(w, d, 2), 3)
        pcie = (total_in + total_out + 9 * WAL_FILES * WAL_RECORDS_PER_FILE) * args.steps / dt / 1e9
        line = {
            "metric": WAL_METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic: seeded text-like Zipf-word records, 8 WAL files per rank in the page cache",
            "config": {"workload": CONFIGS["wal"][4], "files": WAL_FILES, "records": WAL_FILES * WAL_RECORDS_PER_FILE,
                       "file_bytes": total_in, "decoded_bytes": total_out, "workers": W, "depth": D,
                       "parallelism": f"directory per rank x{world}, no data-path collectives"},
            "roofline": {"bound": "pcie", "achieved": round(pcie, 1), "peak": PCIE_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(pcie / PCIE_PEAK_GBPS, 4), "traffic": None, "kernel": "H2D+D2H",
                         "note": "file bytes in + records, offsets and flags out per second"},
            "variants_GiBps": variants,
        }
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(HERE, "tests"))
            import oracle_py as orc

            t_total, nf = 0.0, 0
            for p in paths[:3]:
                img = np.fromfile(p, dtype=np.uint8)
                t1 = time.perf_counter()
                o = orc.file_reader_decode_arrays(img)
                t_total += time.perf_counter() - t1
                nf += 1
                if o["n_records"] != WAL_RECORDS_PER_FILE:
                    raise RuntimeError("oracle WAL decode disagreed")
            in3 = sum(os.path.getsize(p) for p in paths[:nf])
            line["cpu_baseline"] = {"value": round(in3 / 2**30 / t_total, 4), "unit": "GiB/s", "cores": 1,
                                    "kind": "port", "sample": f"{nf} of the {WAL_FILES} WAL files ({in3} B), "
                                    f"sequential FileReader.ReadNext-loop restatement, {_cpu_model()}"}
        if rank == 0:
            print(json.dumps(line), flush=True)
    finally:
        import shutil

        shutil.rmtree(tmp, ignore_errors=True)


def run_index(args, world, rank, local, device):
    """One step = DiskKeyIndex.Get for a batch of keys (disk_key_index.go:36-49) on the device: every
    lane runs the reference's binarySearch (SeekNext probes + IndexEntry parse + key compare) over
    the C5 table's index.rio, resident in HBM."""
    import hashlib
    import struct

    import numpy as np
    import torch

    from recordio import _lib as L
    from recordio.device import to_device_file

    n_entries = CONFIGS["c5"][0]
    nq = CONFIGS["idx"][0]
    index_img, _ = sstable_images(n_entries, rank)
    d_index, li = to_device_file(index_img, local)
    rng = np.random.default_rng(rank_seed(rank))
    # present keys (the table's SHA1 keys) and absent ones (SHA1 of other integers), shuffled
    ids = rng.integers(0, n_entries, nq // 2)
    keys = [hashlib.sha1(struct.pack(">I", rank * n_entries + int(i))).digest() for i in ids]
    keys += [hashlib.sha1(struct.pack(">I", 0x80000000 + rank * nq + i)).digest() for i in range(nq - nq // 2)]
    order = rng.permutation(nq)
    keys = [keys[i] for i in order]
    blob = np.frombuffer(b"".join(keys), dtype=np.uint8)
    off = np.arange(nq + 1, dtype=np.int64) * 20
    d_keys = torch.from_numpy(blob.copy()).to(device)
    d_off = torch.from_numpy(off).to(device)
    hit_sz = ctypes.sizeof(L.IndexHit)
    d_hits = torch.empty(nq * hit_sz, dtype=torch.uint8, device=device)
    lib = L.lib()
    ctx = L.default_ctx(local)
    stream = torch.cuda.Stream(device=device)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step():
        rc = lib.rio_device_index_search(ctx, d_index.data_ptr(), li, 0, d_keys.data_ptr(), d_off.data_ptr(), nq,
                                         d_hits.data_ptr(), sp)
        if rc:
            raise RuntimeError(L.strerror(rc))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    hits = (L.IndexHit * nq).from_buffer_copy(d_hits.cpu().numpy().tobytes())
    found = sum(h.found for h in hits)
    if any(h.status for h in hits) or found < nq // 2 - nq // 100:
        raise RuntimeError(f"index search: found {found} of {nq // 2} present keys")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    value, ms_per_step, _ = job_throughput(dt, nq, args.steps, world, device)
    value *= 2**30  # job_throughput reports units / 2^30 per second; here the unit is one lookup
    alg = nq * (20 + 8 + hit_sz)  # key + its offset in, one hit out
    line = {
        "metric": IDX_METRIC, "value": round(value, 1), "unit": "lookups/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: C5 table's index (SHA1 keys), half the queries present",
        "config": {"workload": CONFIGS["idx"][4], "queries": nq, "index_entries": n_entries, "index_bytes": li,
                   "found": found, "parallelism": f"index per rank x{world}, no data-path collectives"},
        "roofline": {"bound": "hbm", "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(alg / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": "k_index_search", "kernel_ms": round(kern_ms, 4), "alg_bytes_per_launch": alg,
                     "note": "dependent probe chains (~21 SeekNext probes per key): latency-bound, not bandwidth"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import oracle_py as orc

        olib = orc.lib()
        o_off, o_vo, o_cs, o_found = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        base = index_img.ctypes.data  # the index image in place: no per-query copy
        kbuf = ctypes.create_string_buffer(blob.tobytes(), len(blob))
        kaddr = ctypes.addressof(kbuf)
        t1 = time.perf_counter()
        m = 0
        while m < nq and time.perf_counter() - t1 < 10.0:
            st = olib.orc_disk_index_search(base, li, kaddr + 20 * m, 20, 4096, ctypes.byref(o_off),
                                            ctypes.byref(o_found), ctypes.byref(o_vo), ctypes.byref(o_cs))
            if st or bool(o_found.value) != bool(hits[m].found) or o_off.value != hits[m].offset:
                raise RuntimeError(f"oracle index search disagrees with the device at query {m}")
            m += 1
        t_cpu = time.perf_counter() - t1
        line["cpu_baseline"] = {"value": round(m / t_cpu, 1), "unit": "lookups/s", "cores": 1, "kind": "port",
                                "sample": f"first {m} queries, oracle binarySearch restatement (one SeekNext "
                                f"window + IndexEntry parse per probe), {_cpu_model()}"}
    if rank == 0:
        print(json.dumps(line), flush=True)


def run_encode(args, world, rank, local, device):
    """One step = FileWriter.Write for 1M records (file_writer.go:189-233) on the device: snappy
    block encoding per record, v4 headers with CRC-32C, file offsets, the file image
    (rio_device_encode). The records come from decoding the C2 file on the device, and the
    re-encoded image must equal that file byte for byte."""
    import numpy as np
    import torch

    from recordio import _lib as L
    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    n, rec_len, comp, kind, desc = CONFIGS["enc"]
    image = generate(n, rec_len, comp, kind, seed=rank_seed(rank), threads=min(16, os.cpu_count() or 1))
    d_file, flen = to_device_file(image, local)
    dec = DeviceDecoder(local)
    b, info = dec.decode(d_file, flen)
    if info["n_records"] != n:
        raise RuntimeError(f"decode of the input failed: {info}")
    total = int(info["total_out_bytes"])
    lib = L.lib()
    cap = int(lib.rio_encode_bound(n, total, comp))
    d_out = torch.empty(cap, dtype=torch.uint8, device=device)
    d_roff = torch.empty(n, dtype=torch.int64, device=device)
    d_len = torch.zeros(1, dtype=torch.int64, device=device)
    ctx = L.default_ctx(local)
    stream = torch.cuda.Stream(device=device)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step():
        rc = lib.rio_device_encode(ctx, b.out.data_ptr(), b.out_off.data_ptr(), b.flags.data_ptr(), n, total, comp,
                                   d_out.data_ptr(), cap, d_roff.data_ptr(), d_len.data_ptr(), sp)
        if rc:
            raise RuntimeError(L.strerror(rc))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    ln = int(d_len.item())
    if ln != flen or not torch.equal(d_out[:ln], d_file[:flen]):
        raise RuntimeError("device encode of the decoded records is not the original file")
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    value, ms_per_step, _ = job_throughput(dt, total, args.steps, world, device)
    alg = total + 9 * n + flen  # records + offsets/flags in, the file out
    line = {
        "metric": ENC_METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: seeded text-like Zipf-word records (the C2 file decoded on the device), one batch per rank",
        "config": {"workload": desc, "records": n, "record_bytes": rec_len, "record_total": total, "file_bytes": flen,
                   "parallelism": f"batch per rank x{world}, no data-path collectives"},
        "roofline": {"bound": "hbm", "achieved": round(alg / (step_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(alg / (step_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                     "kernel": "rio_device_encode (all launches)", "kernel_ms": round(step_ms, 4),
                     "alg_bytes_per_launch": alg,
                     "note": "dominated by k_snappy_encode<true>: one lane per record, serial golang/snappy match loop"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import oracle_py as orc

        recs = b.out[:total].cpu().numpy()
        offs = b.out_off[:n + 1].cpu().numpy().astype(np.uint64)
        flags = b.flags[:n].cpu().numpy()
        m = 100_000
        sub = np.ascontiguousarray(offs[:m + 1])
        out = np.empty(int(sub[-1]) * 2 + 64 * m, dtype=np.uint8)
        olib = orc.lib()
        runs, t_cpu = 0, 0.0
        while runs < 5 and t_cpu < 10.0:
            t1 = time.perf_counter()
            got = olib.orc_encode_file(recs.ctypes.data, sub.ctypes.data, flags.ctypes.data, m, comp, out.ctypes.data,
                                       out.shape[0], None)
            t_cpu += time.perf_counter() - t1
            runs += 1
            if not got:
                raise RuntimeError("oracle encode failed")
        line["cpu_baseline"] = {"value": round(int(sub[-1]) * runs / 2**30 / t_cpu, 4), "unit": "GiB/s", "cores": 1,
                                "kind": "port", "sample": f"first {m} records x{runs} runs, oracle FileWriter.Write "
                                f"+ golang/snappy restatement, {_cpu_model()}"}
    if rank == 0:
        print(json.dumps(line), flush=True)


def run_readat(args, world, rank, local, device):
    """ReadAtI lookups (MMapReader.ReadNextAt / SeekNext, mmap_reader.go:58-203) from host threads on
    one device-backed reader over the C2 file: the reader decodes the file once on the GPU, then
    every ReadNextAt at a record start is a binary search over the decoded record offsets on the
    calling thread (no kernel launch, no lock). Measured by go-sstables_amd/rio_readat_bench (C++
    over the C-ABI, the shape of a cgo caller); a step = one lookup."""
    import subprocess
    import tempfile

    import numpy as np

    from recordio import generate
    from recordio.device import DeviceDecoder, to_device_file

    n_rec, rec_len, comp, kind, desc = CONFIGS["readat"]
    image = generate(n_rec, rec_len, comp, kind=kind, seed=rank_seed(rank), threads=min(16, os.cpu_count() or 1))
    d_file, length = to_device_file(image, local)
    b, info = DeviceDecoder(local).decode(d_file, length)
    rec_off = b.rec_off[:info["n_records"]].cpu().numpy().astype(np.uint64)
    del d_file, b
    exe = os.path.join(HERE, "go-sstables_amd", "rio_readat_bench")
    tmp = tempfile.mkdtemp(prefix=f"readat_r{rank}_")
    try:
        fpath, opath = os.path.join(tmp, "c2.rio"), os.path.join(tmp, "offsets.u64")
        image.tofile(fpath)
        rec_off.tofile(opath)
        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(local))

        def drive(threads, k, mode):
            out = subprocess.run([exe, fpath, opath, str(threads), str(k), mode], capture_output=True, text=True,
                                 timeout=300, env=env)
            if out.returncode:
                raise RuntimeError(f"readat driver ({mode}, {threads} threads): rc {out.returncode} {out.stderr[-500:]}")
            return json.loads(out.stdout.strip().splitlines()[-1])

        per_thread = max(1, args.steps) * 10_000
        at = {t: drive(t, per_thread, "at") for t in (1, 4, 16)}
        seek = {t: drive(t, per_thread // 10, "seek") for t in (1, 16)}
    finally:
        import shutil

        shutil.rmtree(tmp, ignore_errors=True)
    best = at[16]
    line = {
        "metric": "ReadNextAt lookups/s (16 host threads, one device-decoded MMapReader)",
        "value": round(best["lookups_per_s"], 1), "unit": "lookups/s", "n_gpus": 1, "steps": int(best["lookups"]),
        "warmup": 1, "ms_per_step": round(best["seconds"] * 1e3 / best["lookups"], 6), "higher_is_better": True,
        "scaling": "replicas", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: the C2 file (1M x 1 KiB text-like snappy records), random record starts",
        "config": {"workload": desc, "records": int(info["n_records"]), "file_bytes": length,
                   "parallelism": "host threads on one reader; replicas only across GPUs"},
        "roofline": None,
        "roofline_note": "no kernel per lookup: the one-time decode is the C2 decode (see the c2 line); a "
                         "lookup is a binary search over 8-byte offsets plus a pointer into the decoded arena",
        "us_per_lookup": {f"{t}_threads": round(v["us_per_lookup_per_thread"], 4) for t, v in at.items()},
        "lookups_per_s": {f"{t}_threads": round(v["lookups_per_s"], 1) for t, v in at.items()},
        "seek_next": {f"{t}_threads": {"lookups_per_s": round(v["lookups_per_s"], 1),
                                       "us_per_lookup": round(v["us_per_lookup_per_thread"], 4)}
                      for t, v in seek.items()},
        "first_call_ms": round(at[1]["first_call_ms"], 3),
    }
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import oracle_py as orc

        olib = orc.lib()
        out, ol, nil, d0, d1 = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        rng = np.random.default_rng(5)
        picks = rec_off[rng.integers(0, len(rec_off), 200_000)]
        t1, m = time.perf_counter(), 0
        while m < len(picks) and time.perf_counter() - t1 < 10.0:
            st = olib.orc_read_next_at(image.ctypes.data, length, int(picks[m]), ctypes.byref(out), ctypes.byref(ol),
                                       ctypes.byref(nil), ctypes.byref(d0), ctypes.byref(d1))
            if st:
                raise RuntimeError("oracle ReadNextAt failed")
            olib.orc_free(out)
            m += 1
        t_cpu = time.perf_counter() - t1
        line["cpu_baseline"] = {"value": round(m / t_cpu, 1), "unit": "lookups/s", "cores": 1, "kind": "port",
                                "sample": f"{m} random record starts, oracle ReadNextAt restatement (header parse + "
                                f"snappy decode of one record per lookup, ctypes call overhead included), "
                                f"{_cpu_model()}"}
    if rank == 0:
        print(json.dumps(line), flush=True)


class DeviceBackend:
    """The device call of a decode step: rio_device_decode (one file) or rio_device_decode_batch
    (a file set) on this rank's GPU, files resident in HBM, outputs preallocated."""

    def __init__(self, local: int, device, own: bool = False):
        """own: a context and a stream of its own (in-process multi-device mode, where host threads
        drive the backends concurrently and a device may be listed twice)."""
        from recordio.device import DeviceDecoder

        self.local, self.device, self.own = local, device, own
        self.dec = DeviceDecoder(local, own_ctx=own)

    def load(self, images, batch: bool):
        import torch

        from recordio.device import to_device_file

        self.files = [to_device_file(img, self.local) for img in images]
        self.batch = batch
        # the header's compression type (the host has the image): only that codec's kernels launch
        self.comp = int(images[0][4]) if images and len(images[0]) >= 8 else None
        self.stream = torch.cuda.Stream(self.device) if self.own else torch.cuda.current_stream(self.device)
        if batch:
            self.bufs = [b for b, _ in self.dec.decode_batch(self.files)] if self.files else []
        else:
            self.bufs = [self.dec.decode(*self.files[0], comp=self.comp)[0]]
        return [ln for _, ln in self.files]

    def step(self):
        if not self.files:
            return
        if self.batch:
            self.dec.launch_batch(self.files, self.bufs, self.stream)
        else:
            self.dec.launch(self.files[0][0], self.files[0][1], self.bufs[0], self.stream, self.comp)

    def sync(self):
        import torch

        if self.own:
            self.stream.synchronize()
        else:
            torch.cuda.synchronize(self.device)

    def infos(self):
        return [self.dec.info(b) for b in self.bufs]

    def checksums(self):
        """Device digests of every file's decoded arrays (out, out_off, rec_off, flags)."""
        res = []
        for b in self.bufs:
            i = self.dec.info(b)
            n, nb = i["n_records"], i["total_out_bytes"]
            res.append((device_digest(b.out[:nb]), device_digest(b.out_off[:n + 1]), device_digest(b.rec_off[:n]),
                        device_digest(b.flags[:n])))
        self.sync()
        return res

    def set_timing(self, slots: int):
        from recordio import _lib as L

        L.lib().rio_ctx_set_timing(self.dec.ctx, slots)

    def stage_ms(self):
        return self.dec.stage_ms() if self.files else []

    def evict(self):
        """Write 1 GiB of HBM and read half of it back (pushes the decode's working set out of the MALL)."""
        import torch

        if not hasattr(self, "_evict"):
            self._evict = torch.empty(1 << 30, dtype=torch.uint8, device=self.device)
        self._evict.fill_(1)
        if os.environ.get("RIO_BENCH_EVICT", "write_read") == "write_read":
            # then read 512 MiB of it back: clean lines replace the fill's dirty ones, whose write-back would
            # otherwise run under the next decode (C1 cold walk 0.069 -> 0.045 ms, profiles/r5/r5ai_evict_ab.txt);
            # RIO_BENCH_EVICT=write: the fill alone (round 4's method)
            self._evict_sum = self._evict[: 1 << 29].view(torch.int64).sum()
        # the fill runs on torch's stream, the decode on the context's: without this wait the next decode ran
        # beside the 1 GiB write (rocprofv3 trace, profiles/r5/r5af_c1_trace.txt) and its cold stage times
        # priced the write's bandwidth in
        torch.cuda.synchronize(self.device)

    def rec_offs(self, n):
        """Record offsets of every loaded file (the CPU baseline's ReadNextAt table)."""
        out = []
        for b in self.bufs:
            k = self.dec.info(b)["n_records"]
            out.append(b.rec_off[:k].cpu().numpy())
        return out[0] if len(out) == 1 else out


def plan_files(config: str, world: int, rank: int) -> list:
    """Seeds of the files this rank decodes: C4's fixed 8-file set sharded round-robin over the
    ranks (BASELINE configs[3]), otherwise one rank-seeded file per GPU."""
    if config in MULTI_FILE:
        n_files, seed0 = MULTI_FILE[config]
        return [seed0 + f for f in shard_files(n_files, world, rank)]
    return [rank_seed(rank)]


def run_decode(args, world, rank, backend, sizes=None) -> dict:
    """One decode config on this rank: plan and generate its files, hand them to the backend (the
    device), warm up, time exactly args.steps steps between barriers, reduce over ranks (gloo) and
    build the JSON line. `sizes` = (records, record_bytes) overrides the config's (tests)."""
    from recordio import _lib as L
    from recordio import generate

    n_rec, rec_len, comp, kind, desc = CONFIGS[args.config]
    if sizes:
        n_rec, rec_len = sizes
    threads = min(16, os.cpu_count() or 1)
    batch = args.config in MULTI_FILE
    seeds = plan_files(args.config, world, rank)
    images = [generate(n_rec, rec_len, comp, kind=kind, seed=sd, threads=threads) for sd in seeds]
    lengths = backend.load(images, batch)
    for _ in range(args.warmup):
        backend.step()
    backend.sync()
    infos = backend.infos()
    for info in infos:
        if info["status"] != L.RIO_EOF or info["n_records"] != n_rec:
            raise RuntimeError(f"decode failed: {info}")
    # the warmup's result: every later pass must rebuild exactly these bytes
    digests = backend.checksums()
    length = sum(lengths)  # input bytes of this rank per step
    n = sum(i["n_records"] for i in infos)
    nb = sum(i["total_out_bytes"] for i in infos)

    backend.set_timing(args.steps)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    backend.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        backend.step()
    backend.sync()
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    stage = backend.stage_ms()  # per-stage HIP-event means over the timed steps
    backend.set_timing(0)

    def verify(what: str) -> None:
        """The decode's result struct and a device-side digest of out / out_off / rec_off / flags after
        `what`, against the warmup's: a step that went wrong fails the bench loudly."""
        now_infos, now_dig = backend.infos(), backend.checksums()
        if now_infos != infos or now_dig != digests:
            raise RuntimeError(f"bench: the {what} decoded different results from the warmup: "
                               f"{now_infos} / {now_dig} vs {infos} / {digests}")

    verify("timed steps")

    value, ms_per_step, dt_max = job_throughput(dt, length, args.steps, world)

    # when input + output fit the 256 MB MALL (C1), back-to-back steps re-read a warm
    # cache. A second pass writes 1 GiB between decodes (outside the per-stage HIP events) and
    # reports the cold-cache stage times beside the headline.
    mall_flushed, cold = None, []
    # (decided over all ranks: the reductions below are collectives every rank must join)
    if reduce_max(1.0 if lengths and length + nb < (512 << 20) else 0.0, world) > 0:
        if lengths:
            backend.set_timing(args.steps)
            for _ in range(args.steps):
                backend.evict()
                backend.step()
            backend.sync()
            cold = backend.stage_ms()
            backend.set_timing(0)
            verify("MALL-flushed steps")
        cold_ms = sum(cold) if len(cold) == 4 else 0.0
        # whole job: every rank's bytes over the slowest rank's cold step
        cold_value, cold_step_ms, _ = job_throughput(cold_ms * 1e-3, length, 1, world)
        if len(cold) == 4:
            mall_flushed = {"ms_per_step": round(cold_step_ms, 4), "value": round(cold_value, 3),
                            "unit": "GiB/s", "stages_ms": [round(x, 4) for x in cold],
                            "note": "1 GiB device write + 512 MiB read-back between steps, finished before the decode; per-stage HIP events, flush excluded"}

    # with the working set inside the MALL the warm loop would price cache hits as HBM;
    # the line then reports the cold pass (MALL evicted before every step, per-stage HIP events,
    # the eviction excluded): value, ms_per_step and the roofline; the warm wall-clock rate is kept
    # beside it as warm_value
    warm = None
    if mall_flushed and len(cold) == 4:
        warm = {"value": round(value, 3), "ms_per_step": round(ms_per_step, 4),
                "note": "back-to-back steps, input + output resident in the 256 MB MALL (wall clock)"}
        value, ms_per_step, stage = mall_flushed["value"], mall_flushed["ms_per_step"], cold

    # roofline of the dominant kernel (Snappy / copy decode): algorithmic bytes per launch =
    # input file bytes (headers + payloads read once) + decoded bytes written once
    # + 8(N+1) out_off + 8N rec_off + N flags read
    alg_bytes = length + nb + 8 * (n + len(lengths)) + 8 * n + n
    decode_ms = stage[3] if len(stage) == 4 else float("nan")
    achieved = alg_bytes / (decode_ms * 1e-3) / 1e9
    # HBM traffic of the dominant kernel: measured by this invocation (main() ran the PMC passes before
    # the GPU was touched), else the committed PMC file with the tree it was measured on, else none
    live = getattr(args, "live_traffic", None)
    if live and "traffic" in live:
        tr = live
    elif getattr(args, "traffic", "live") == "none":
        tr = {"traffic": None}
    else:
        tr = file_traffic(args.config, args.traffic_json)
        if live and "error" in live:
            tr["traffic_live_error"] = live["error"]
    traffic = tr.get("traffic")
    pipe_ms = sum(stage) if stage else float("nan")
    kernel = dominant_kernel(args.config, rec_len)
    total_files = MULTI_FILE[args.config][0] if batch else world
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if batch else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded text-like Zipf-word records (snappy ratio ~0.55)" +
                (f", {total_files} files (seeds {MULTI_FILE[args.config][1]}..) sharded over the ranks" if batch
                 else ", one file per rank"),
        "config": {"workload": desc, "records": n, "record_bytes": rec_len, "file_bytes": length,
                   "decoded_bytes": nb, "compression": {0: "none", 1: "gzip", 2: "snappy", 3: "lzw"}[comp],
                   "files_this_rank": len(lengths),
                   "parallelism": f"file-sharded x{world} ({total_files} files), no data-path collectives"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": kernel,
                     "kernel_ms": round(decode_ms, 4), "alg_bytes_per_launch": alg_bytes,
                     **{k: v for k, v in tr.items() if k != "traffic"}},
        # every pass after the warmup (the timed steps, the MALL-flushed steps) rebuilt the warmup's result
        # struct and the same device-side digest of out / out_off / rec_off / flags (verify() above); "verified" is
        # set below once the cpu_baseline leg has compared the first file with the oracle (None when it is skipped)
        "reproducible": True,
        "verified": None,
        "verify": {"method": "rio_file_info + device digest of out, out_off, rec_off, flags: warmup vs after "
                             "the timed steps (and after the MALL-flushed pass)",
                   "digest_out": digests[0][0] if digests else None},
        "stages_ms": {"walk": round(stage[0], 4), "scan": round(stage[1], 4), "place": round(stage[2], 4),
                      "decode": round(stage[3], 4)} if len(stage) == 4 else None,
        "pipeline_roofline_frac": round(alg_bytes / (pipe_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if stage else None,
        # also output GiB/s and records/s (whole job, same timed region as `value`)
        "output_GiBps": round(value * nb / length, 3) if length else None,
        "Mrecords_per_s": round(value * 2**30 / length * n / 1e6, 2) if length else None,
    }
    if mall_flushed:
        line["mall_flushed"] = mall_flushed
    if warm:
        line["warm_mall"] = warm
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        def against_oracle(out, out_off, rec_off, flags):
            """The oracle's decode of images[0] against the device arrays the timed steps left (their digests)."""
            import numpy as np
            import torch

            dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
            up = [device_digest(torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev))
                  for a in (out, out_off, rec_off, flags)]
            return tuple(up) == tuple(digests[0])

        line["cpu_baseline"] = cpu_baseline(images, backend.rec_offs(n), n_rec, check=against_oracle)
        ok = line["cpu_baseline"].get("oracle_match")
        if ok is False:
            raise RuntimeError("bench: the device decode of the first file differs from the oracle's")
        line["verified"] = bool(ok)
        line["verify"]["oracle"] = ("the oracle's FileReader loop (oracle/rio_oracle.c) over the whole first file: device "
                                    "digests of its out, out_off, rec_off, flags equal the timed decode's")
    if rank == 0 and world == 1 and not args.no_e2e and not batch:
        line["e2e"] = e2e_rate(images[0], nb)
    return line


def lpt_assign(sizes: list[int], n_dev: int) -> list[list[int]]:
    """Longest processing time first: file indices per device, each file (largest first) to the device
    with the fewest bytes so far (ties: the lower device slot). rio_fileset_decode's rule (rio.h)."""
    load = [0] * n_dev
    out: list[list[int]] = [[] for _ in range(n_dev)]
    for i in sorted(range(len(sizes)), key=lambda k: (-sizes[k], k)):
        d = min(range(n_dev), key=lambda k: (load[k], k))
        out[d].append(i)
        load[d] += sizes[i]
    return [sorted(x) for x in out]


def run_decode_inproc(args, devices: list[int], make_be, sizes=None) -> dict:
    """The in-process multi-device shape a Go caller has (rio_fileset_*): ONE process,
    one host thread and one backend (its own context and stream) per listed device, the config's files
    assigned longest-first (lpt_assign). Files are resident in HBM before the timed region, as in
    run_decode; the threads start each timed loop together (a barrier) and value = all files' bytes x
    steps / the wall time until the last thread's device is idle. Every backend's result is verified
    after the timed loop as in run_decode. A device may be listed twice (one-GPU rehearsal)."""
    import threading

    from recordio import _lib as L
    from recordio import generate

    n_rec, rec_len, comp, kind, desc = CONFIGS[args.config]
    if sizes:
        n_rec, rec_len = sizes
    threads = min(16, os.cpu_count() or 1)
    batch = args.config in MULTI_FILE
    nd = len(devices)
    seeds = ([MULTI_FILE[args.config][1] + f for f in range(MULTI_FILE[args.config][0])] if batch
             else [rank_seed(i) for i in range(nd)])
    images = [generate(n_rec, rec_len, comp, kind=kind, seed=sd, threads=threads) for sd in seeds]
    plan = lpt_assign([len(img) for img in images], nd)
    bes = [make_be(devices[k]) for k in range(nd)]
    lengths = [sum(be.load([images[i] for i in plan[k]], batch) or [0]) if plan[k] else 0 for k, be in enumerate(bes)]
    for be, part in zip(bes, plan):
        if part:
            for _ in range(args.warmup):
                be.step()
            be.sync()
    infos = [be.infos() if part else [] for be, part in zip(bes, plan)]
    for inf in infos:
        for i in inf:
            if i["status"] != L.RIO_EOF or i["n_records"] != n_rec:
                raise RuntimeError(f"decode failed: {i}")
    digests = [be.checksums() if part else [] for be, part in zip(bes, plan)]
    for be, part in zip(bes, plan):
        if part:
            be.set_timing(args.steps)
    bar = threading.Barrier(nd + 1)
    ends = [0.0] * nd
    errs: list = []

    def drive(k):
        try:
            bar.wait()
            if plan[k]:
                for _ in range(args.steps):
                    bes[k].step()
                bes[k].sync()
            ends[k] = time.perf_counter()
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)
            ends[k] = time.perf_counter()

    ths = [threading.Thread(target=drive, args=(k,)) for k in range(nd)]
    for t in ths:
        t.start()
    bar.wait()
    t0 = time.perf_counter()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]
    dt = max(ends) - t0
    stage = bes[0].stage_ms() if plan[0] else []
    for k, (be, part) in enumerate(zip(bes, plan)):
        if part:
            be.set_timing(0)
            if be.infos() != infos[k] or be.checksums() != digests[k]:
                raise RuntimeError(f"bench: device slot {k}'s timed steps decoded different results from its warmup")
    total = sum(lengths)
    value = total * args.steps / 2**30 / dt
    n = sum(i["n_records"] for inf in infos for i in inf)
    nb = sum(i["total_out_bytes"] for inf in infos for i in inf)
    return {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": nd, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if batch else "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: seeded text-like Zipf-word records (snappy ratio ~0.55)",
        "config": {"workload": desc, "records": n, "record_bytes": rec_len, "file_bytes": total, "decoded_bytes": nb,
                   "parallelism": f"in-process: one host thread + context + stream per device, {len(images)} files "
                                  f"assigned longest-first, no collectives",
                   "devices": devices, "files_per_device": [len(p) for p in plan]},
        "stages_ms_device0": ({"walk": round(stage[0], 4), "scan": round(stage[1], 4), "place": round(stage[2], 4),
                               "decode": round(stage[3], 4)} if len(stage) == 4 else None),
        "reproducible": True,
        "mode": "inproc" + (" (rehearsal: a device listed more than once)" if len(set(devices)) < nd else ""),
    }


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_contract(gpus: int, argv: list[str]) -> int | None:
    """`--gpus N` is authoritative. Runs BEFORE anything touches the GPU:
      * WORLD_SIZE unset and N > 1: no launcher started us, so start one (torch.distributed.run, one
        rank per GPU, rendezvous on 127.0.0.1) on this very script and return its exit code — the
        parent never initialises HIP, so nothing is exec'd from a GPU process;
      * WORLD_SIZE set and != N: a launcher and the flag disagree; refuse rather than report a job of
        the wrong size;
      * otherwise None: run this process as the rank the environment names (N = 1, or under a launcher).
    """
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if gpus <= 1:
            return None
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(sys.argv[0])] + argv
        print(f"bench.py: --gpus {gpus} without a launcher: starting {gpus} ranks", file=sys.stderr, flush=True)
        return subprocess.call(cmd)
    if int(ws) != gpus:
        print(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}: refusing to report a {ws}-rank job as {gpus} GPUs",
              file=sys.stderr, flush=True)
        return 2
    return None


def make_device(local: int):
    """This rank's GPU: cuda:LOCAL_RANK."""
    import torch

    torch.cuda.set_device(local)
    return torch.device(f"cuda:{local}")


def make_backend(local: int, device, own: bool = False):
    """The decode configs' device call (tests/bench_cli_oracle.py substitutes the CPU oracle)."""
    return DeviceBackend(local, device, own=own)


def make_inproc_device(local: int):
    """A device of the in-process mode (no set_device: the threads share the process)."""
    import torch

    return torch.device(f"cuda:{local}")


def main(argv: list[str] | None = None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic file (default: profiles/traffic_<config>.json, then traffic_latest.json)")
    ap.add_argument("--inproc-devices", default=None,
                    help="in-process multi-device mode: a device list (\"0,1,2,3\", or N for 0..N-1); one process, "
                         "one host thread per device (the Go caller's shape, INTEGRATION.md §2.2)")
    ap.add_argument("--traffic", default="live", choices=["live", "file", "none"],
                    help="roofline.traffic: measured by this run (two rocprofv3 --pmc passes, 1 GPU only), the "
                         "committed PMC file, or none")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)
    rc = launch_contract(args.gpus, argv)
    if rc is not None:
        sys.exit(rc)

    world, rank, local = dist_env()
    assert world == args.gpus
    import numpy as np  # noqa: F401
    import torch

    if args.inproc_devices:
        spec = args.inproc_devices
        devices = [int(x) for x in spec.split(",")] if "," in spec else list(range(int(spec)))
        line = run_decode_inproc(args, devices, lambda d: make_backend(d, make_inproc_device(d), own=True))
        print(json.dumps(line), flush=True)
        return

    # the PMC passes run as child processes before this one touches the GPU (decode configs, one GPU;
    # torch.cuda.device_count() does not initialise HIP on this image)
    args.live_traffic = None
    if (args.traffic == "live" and world == 1 and args.config not in ("c5", "wal", "idx", "enc", "readat")
            and torch.cuda.device_count() > 0):
        args.live_traffic = live_traffic(args.config)

    device = make_device(local)
    if world > 1:
        import torch.distributed as dist

        # gloo on the host: the barrier and the max/sum over ranks are the job's only collectives
        # (the decode path has none: files are sharded, north_star "no RCCL")
        dist.init_process_group(backend="gloo")

    if args.config in ("c5", "wal", "idx", "enc", "readat"):
        {"c5": run_sstable, "wal": run_wal, "idx": run_index, "enc": run_encode, "readat": run_readat}[args.config](
            args, world, rank, local, device)
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    line = run_decode(args, world, rank, make_backend(local, device))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
