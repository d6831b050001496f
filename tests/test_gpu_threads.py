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
