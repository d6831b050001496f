"""Per-step time of the device-resident decode with the context's five per-stage timing events recorded on every call
(rio_ctx_set_timing(1)) and with none (set_timing(0), a context's default since late round 5), interleaved: what the
stage events cost a step.
usage (GPU box): python scripts/event_probe.py [steps]"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "go-sstables_amd"))

from recordio import _lib as L  # noqa: E402
from recordio import generate  # noqa: E402
from recordio.device import DeviceDecoder, to_device_file  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 50
CASES = [("c2", 1_000_000, 1024, 2, 1), ("c2r", 1_000_000, 1024, 2, 0), ("c1", 100_000, 1024, 0, 0)]

for name, n_rec, rec_len, comp, kind in CASES:
    img = generate(n_rec, rec_len, comp, kind=kind, seed=1)
    dec = DeviceDecoder(0, own_ctx=True)
    d_file, n = to_device_file(img)
    b, info = dec.decode(d_file, n, comp=comp)
    s = torch.cuda.Stream(device=0)
    res = {0: [], 1: []}
    for r in range(3):
        for slots in (1, 0):
            L.lib().rio_ctx_set_timing(dec.ctx, slots)
            for _ in range(3):
                dec.launch(d_file, n, b, s, comp)
            s.synchronize()
            t0 = time.perf_counter()
            for _ in range(STEPS):
                dec.launch(d_file, n, b, s, comp)
            s.synchronize()
            res[slots].append((time.perf_counter() - t0) / STEPS * 1e3)
    ok = dec.info(b)["n_records"] == n_rec
    print(f"{name}: with stage events {' '.join(f'{x:.4f}' for x in res[1])} ms per step, without "
          f"{' '.join(f'{x:.4f}' for x in res[0])} records ok {ok}", flush=True)
    del b, d_file, dec
    torch.cuda.empty_cache()
