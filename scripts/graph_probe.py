"""Per-step time of a device-resident decode launched call by call vs replayed from a captured HIP graph
(torch.cuda.CUDAGraph around rio_device_decode_ex): does a graph shorten the dispatch gaps between the
decode's six kernels? usage (GPU box): python scripts/graph_probe.py [steps]"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "go-sstables_amd"))

from recordio import generate  # noqa: E402
from recordio.device import DeviceDecoder, to_device_file  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 50
CASES = [("c2", 1_000_000, 1024, 2, 1, 1), ("c2r", 1_000_000, 1024, 2, 0, 1), ("c1", 100_000, 1024, 0, 0, 1),
         ("c3", 10_000_000, 64, 2, 1, 3)]

for name, n_rec, rec_len, comp, kind, seed in CASES:
    img = generate(n_rec, rec_len, comp, kind=kind, seed=seed)
    dec = DeviceDecoder(0, own_ctx=True)
    d_file, n = to_device_file(img)
    b, info = dec.decode(d_file, n, comp=comp)
    s = torch.cuda.Stream(device=0)
    for _ in range(3):
        dec.launch(d_file, n, b, s, comp)
    s.synchronize()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):  # g.replay() launches on the current stream
            for _ in range(STEPS):
                fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / STEPS * 1e3

    plain = timed(lambda: dec.launch(d_file, n, b, s, comp))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        dec.launch(d_file, n, b, s, comp)
    with torch.cuda.stream(s):
        for _ in range(3):
            g.replay()
    graph = timed(g.replay)
    plain2 = timed(lambda: dec.launch(d_file, n, b, s, comp))
    ok = dec.info(b)["n_records"] == n_rec
    print(f"{name}: plain {plain:.4f} / {plain2:.4f} ms per step, graph {graph:.4f} ms ({len(img) / 2**30 / graph * 1e3:.1f} GiB/s)"
          f" records ok {ok}", flush=True)
    del g, b, d_file, dec
    torch.cuda.empty_cache()
