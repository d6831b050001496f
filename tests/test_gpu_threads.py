"""The single-process multi-device shape a Go caller has: host threads, each with its
own rio_ctx (own stream, arenas, pinned staging), decoding different files through the host C-ABI
(rio_frame + rio_decode, the cgo pair) at the same time. On the 1-GPU box the threads share device
0; every file must still be exactly the oracle's (GPU)."""
import ctypes
import threading

import numpy as np
import pytest

import oracle_py as orc
from gpu_util import assert_same_as_oracle
from recordio import _lib as L
from recordio import generate

pytestmark = pytest.mark.gpu


def host_decode(ctx, img):
    lib = L.lib()
    fi = L.FileInfo()
    rc = lib.rio_frame(ctx, img.ctypes.data, img.shape[0], ctypes.byref(fi))
    assert rc == 0, L.strerror(rc)
    n, nb = fi.n_records, fi.total_out_bytes
    out = np.zeros(nb + 16, dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    rec_off = np.zeros(n + 1, dtype=np.uint64)
    flags = np.zeros(n + 1, dtype=np.uint8)
    rc = lib.rio_decode(ctx, out.ctypes.data, nb, out_off.ctypes.data, rec_off.ctypes.data, flags.ctypes.data, n,
                        ctypes.byref(fi))
    assert rc == 0, L.strerror(rc)
    k = fi.n_records
    res = fi.as_dict()
    res.update(out=out[:fi.total_out_bytes], out_off=out_off[:k + 1].astype(np.int64),
               rec_off=rec_off[:k].astype(np.int64), flags=flags[:k])
    return res


@pytest.mark.parametrize("threads", [2, 4])
def test_threads_with_own_contexts_on_one_device(threads):
    specs = [(3000, 1024, 2, 1), (2000, 700, 0, 0), (300, 20000, 2, 1), (1500, 2048, 1, 1)]
    images = [generate(*specs[t % len(specs)][:3], kind=specs[t % len(specs)][3], seed=50 + t) for t in range(threads)]
    expect = [orc.file_reader_decode_arrays(img) for img in images]
    ctxs = []
    for _ in range(threads):
        h = ctypes.c_void_p()
        assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
        ctxs.append(h.value)
    go = threading.Barrier(threads)
    results, errors = [None] * threads, []

    def run(t):
        try:
            go.wait()
            for _ in range(3):  # repeated calls interleave with the other threads' on the device
                results[t] = host_decode(ctxs[t], images[t])
        except Exception as e:  # noqa: BLE001
            errors.append((t, repr(e)))

    th = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for h in ctxs:
        L.lib().rio_ctx_destroy(h)
    assert not errors, errors
    for t in range(threads):
        assert_same_as_oracle(results[t], expect[t], f"thread {t}")


def test_device_calls_alternating_streams_after_reserve():
    """Device-API calls of one ctx on two streams in turn, with no host synchronisation between them:
    each call waits for the previous one (they share the ctx's scratch), so every result is the
    oracle's. rio_ctx_reserve first sizes the arenas (nothing is allocated between the calls)."""
    import torch

    from recordio.device import DecodeBuffers, DeviceDecoder, to_device_file  # noqa: F401

    imgs = [generate(4000, 1024, 2, kind=1, seed=71).tobytes(), generate(9000, 300, 2, kind=1, seed=72).tobytes(),
            generate(2000, 900, 0, kind=0, seed=73).tobytes()]
    dec = DeviceDecoder(0)
    assert L.lib().rio_ctx_reserve(dec.ctx, max(len(i) for i in imgs), 20000, 2) == 0
    files = [to_device_file(i) for i in imgs]
    sized = [dec.decode(d, n)[1] for d, n in files]  # sizes (and a warm ctx)
    bufs = [dec.alloc(i["n_records"], i["total_out_bytes"]) for i in sized]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(3):
        for k, ((d, n), b) in enumerate(zip(files, bufs)):
            dec.launch(d, n, b, streams[(k + rep) % 2])
    torch.cuda.synchronize()
    for k, (img, b) in enumerate(zip(imgs, bufs)):
        info = dec.info(b)
        n, nb = info["n_records"], info["total_out_bytes"]
        g = dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:n + 1].cpu().numpy(),
                 rec_off=b.rec_off[:n].cpu().numpy(), flags=b.flags[:n].cpu().numpy())
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), f"stream file {k}")
