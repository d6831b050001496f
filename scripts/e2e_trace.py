"""Timeline of the windowed host path (rio_stream_open_host) on the C2 file: per window the
read+H2D+frame span (driver thread) and the decode+D2H span (worker), RIO_REPLAY_TRACE=1 output on
stderr. usage: RIO_REPLAY_TRACE=1 python scripts/e2e_trace.py [window_MiB ...]"""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "go-sstables_amd"))
import torch  # noqa: F401,E402  (the HIP runtime librio binds to)

from recordio import _lib as L  # noqa: E402
from recordio import generate  # noqa: E402

img = generate(1_000_000, 1024, 2, kind=1, seed=1, threads=16)
lib = L.lib()
for wmib in [int(x) for x in sys.argv[1:]] or [128]:
    for rep in range(3):
        h = ctypes.c_void_p()
        t0 = time.perf_counter()
        rc = lib.rio_stream_open_host(0, img.ctypes.data, img.shape[0], wmib << 20, 4, ctypes.byref(h))
        n = 0
        while rc == 0:
            first, info = ctypes.c_uint64(), L.FileInfo()
            p = [ctypes.c_void_p() for _ in range(4)]
            rc = lib.rio_stream_next(h, ctypes.byref(first), *[ctypes.byref(x) for x in p], ctypes.byref(info))
            if rc == 0:
                n += info.n_records
        dt = time.perf_counter() - t0
        lib.rio_stream_free(h)
        print(f"window {wmib} MiB run {rep}: {n} records, {dt * 1e3:.2f} ms, {img.shape[0] / 2**30 / dt:.2f} GiB/s",
              file=sys.stderr, flush=True)
