"""Fused walk (RIO_FUSED=1) against the two-launch scan on growing C2-shaped files: one decode each,
timed, outputs compared. Run under `timeout`; prints a line per size as it goes.
usage: python scripts/fused_probe.py [n_records ...]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "go-sstables_amd"))
import torch  # noqa: E402

from recordio import generate  # noqa: E402
from recordio.device import DeviceDecoder, to_device_file  # noqa: E402


def ctx_decoder(fused):
    """A DeviceDecoder over a fresh rio_ctx created with RIO_FUSED=fused (read at creation)."""
    import ctypes

    from recordio import _lib as L

    os.environ["RIO_FUSED"] = fused
    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    d = DeviceDecoder.__new__(DeviceDecoder)
    d.device, d.ctx = 0, h.value
    return d


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [1000, 10000, 100000, 1000000]
    d0, d1 = ctx_decoder("0"), ctx_decoder("1")
    for n in sizes:
        img = generate(n, 1024, 2, kind=1, seed=7, threads=16)
        f, ln = to_device_file(img, 0)
        b0, i0 = d0.decode(f, ln)
        torch.cuda.synchronize()
        t = time.time()
        for rep in range(3):
            d0.decode(f, ln)
        torch.cuda.synchronize()
        base = (time.time() - t) / 3
        res = []
        for rep in range(3):
            t = time.time()
            b1, i1 = d1.decode(f, ln)
            torch.cuda.synchronize()
            res.append(time.time() - t)
        nb = i0["total_out_bytes"]
        same = (i0["status"], i0["n_records"], nb) == (i1["status"], i1["n_records"], i1["total_out_bytes"]) and \
            torch.equal(b0.out[:nb], b1.out[:nb]) and torch.equal(b0.out_off[:n + 1], b1.out_off[:n + 1])
        print(f"n={n} chunks~{len(img) // 32768} two-launch {base:.4f} s, fused s={['%.4f' % r for r in res]} same={same} "
              f"status={i1['status']} n={i1['n_records']}", flush=True)


if __name__ == "__main__":
    main()
