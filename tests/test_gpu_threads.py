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


def test_host_api_waits_for_device_api_on_one_ctx():
    """A device-API decode enqueued on a torch stream and host-API calls (rio_frame / rio_decode, the
    cgo pair) on the same ctx right after it, with no host synchronisation in between: they share the
    ctx's scratch arenas, so the host calls must wait for the device call (and the next device call
    for them). Every result is the oracle's."""
    import torch

    from recordio.device import DeviceDecoder, to_device_file

    dev_imgs = [generate(20000, 1024, 2, kind=1, seed=81), generate(30000, 300, 2, kind=1, seed=82)]
    host_imgs = [generate(15000, 900, 2, kind=1, seed=83), generate(4000, 2000, 0, kind=0, seed=84)]
    dec = DeviceDecoder(0)
    files = [to_device_file(i) for i in dev_imgs]
    sized = [dec.decode(d, n)[1] for d, n in files]
    bufs = [dec.alloc(i["n_records"], i["total_out_bytes"]) for i in sized]
    s = torch.cuda.Stream()
    host_res = []
    for rep in range(2):
        for k, ((d, n), b) in enumerate(zip(files, bufs)):
            dec.launch(d, n, b, s)  # async on s
            host_res.append((k, host_decode(dec.ctx, host_imgs[k])))  # host API on the same ctx at once
    torch.cuda.synchronize()
    for k, r in host_res:
        assert_same_as_oracle(r, orc.file_reader_decode_arrays(host_imgs[k]), f"host {k}")
    for k, (img, b) in enumerate(zip(dev_imgs, bufs)):
        info = dec.info(b)
        n, nb = info["n_records"], info["total_out_bytes"]
        g = dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:n + 1].cpu().numpy(),
                 rec_off=b.rec_off[:n].cpu().numpy(), flags=b.flags[:n].cpu().numpy())
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), f"device {k}")


def test_ctx_pool_hands_back_the_same_context():
    lib = L.lib()
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.rio_ctx_acquire(0, ctypes.byref(a)) == 0 and lib.rio_ctx_device(a) == 0
    lib.rio_ctx_release(a)
    assert lib.rio_ctx_acquire(0, ctypes.byref(b)) == 0
    assert b.value == a.value  # the idle context, arenas already grown
    img = generate(2000, 1024, 2, kind=1, seed=85)
    assert_same_as_oracle(host_decode(b.value, img), orc.file_reader_decode_arrays(img), "pooled ctx")
    lib.rio_ctx_release(b)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_fileset_over_devices(tmp_path, devices):
    """rio_fileset_decode: files of different sizes and codecs assigned to the listed devices by LPT,
    one host thread + pooled context per device (two or three 'devices' map to the box's one GPU);
    every file exactly the oracle's, a missing path reported on its own."""
    lib = L.lib()
    specs = [(6000, 1024, 2, 1), (200, 30000, 2, 1), (9000, 100, 2, 1), (3000, 700, 0, 0), (500, 4096, 1, 1),
             (1, 10, 2, 1), (12000, 64, 2, 1)]
    imgs, paths = [], []
    for k, (n, ln, comp, kind) in enumerate(specs):
        img = generate(n, ln, comp, kind=kind, seed=90 + k)
        p = tmp_path / f"f{k}.rio"
        p.write_bytes(img.tobytes())
        imgs.append(img)
        paths.append(str(p))
    paths.append(str(tmp_path / "missing.rio"))
    arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
    devs = (ctypes.c_int * len(devices))(*devices)
    h = ctypes.c_void_p()
    assert lib.rio_fileset_decode(devs, len(devices), arr, len(paths), ctypes.byref(h)) == 0
    try:
        for k, img in enumerate(imgs):
            out, off, ro, fl = (ctypes.c_void_p() for _ in range(4))
            fi, dev = L.FileInfo(), ctypes.c_int()
            rc = lib.rio_fileset_get(h, k, ctypes.byref(out), ctypes.byref(off), ctypes.byref(ro), ctypes.byref(fl),
                                     ctypes.byref(fi), ctypes.byref(dev))
            assert rc == 0 and dev.value == 0
            n, nb = fi.n_records, fi.total_out_bytes
            res = fi.as_dict()
            res.update(out=np.ctypeslib.as_array((ctypes.c_uint8 * max(nb, 1)).from_address(out.value))[:nb].copy(),
                       out_off=np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(off.value)).astype(np.int64),
                       rec_off=np.ctypeslib.as_array((ctypes.c_uint64 * max(n, 1)).from_address(ro.value))[:n].astype(np.int64),
                       flags=np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(fl.value))[:n].copy())
            assert_same_as_oracle(res, orc.file_reader_decode_arrays(img), f"fileset {k}")
        fi = L.FileInfo()
        assert lib.rio_fileset_get(h, len(imgs), None, None, None, None, ctypes.byref(fi), None) == L.RIO_ERR_IO
        assert lib.rio_fileset_get(h, len(paths), None, None, None, None, None, None) == L.RIO_ERR_ARG
    finally:
        lib.rio_fileset_free(h)
