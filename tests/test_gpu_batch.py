"""rio_device_decode_batch (GPU): several device-resident files in one call, each exactly the oracle's.

BASELINE configs[3] decodes 8 files of 64 KiB Snappy records per GPU in one step; the batch runs the
framing per file and one decode launch across the files (k_snappy_pipe_batch, the lane decoder, with
the waves dealt to the files by record count; files past 32-bit positions, or every file when
RIO_COOP_MIN says so, take the wave-per-record decoder k_snappy_coop_batch instead). Every file
of a batch must come out as the FileReader.ReadNext loop restated by the oracle
(file_reader.go:61-131) says, whatever else shares the batch: large- and small-record Snappy files,
gzip, uncompressed, damaged files, header-only files, and more files than one launch group holds.
"""
import random

import numpy as np
import pytest

import corpus
import oracle_py as orc
from gpu_util import assert_same_as_oracle, decoder
from recordio import generate
from recordio.device import to_device_file

pytestmark = pytest.mark.gpu


def _host(b, info):
    k, nb = info["n_records"], info["total_out_bytes"]
    res = dict(info)
    if k or nb:
        res.update(out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:k + 1].cpu().numpy(),
                   rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())
    else:
        res.update(out=np.zeros(0, np.uint8), out_off=np.zeros(1, np.int64), rec_off=np.zeros(0, np.int64),
                   flags=np.zeros(0, np.uint8))
    return res


def check_batch(images, what):
    files = [to_device_file(img) for img in images]
    got = decoder().decode_batch(files)
    assert len(got) == len(images)
    for k, (img, (b, info)) in enumerate(zip(images, got)):
        o = orc.file_reader_decode_arrays(img)
        if o["status"] in (13,):  # SHORT_FILE_HEADER: nothing else to compare
            assert info["status"] == o["status"], (what, k)
            continue
        assert_same_as_oracle(_host(b, info), o, f"{what}[{k}]")


def _damage_records(img, every, seed):
    """Corrupt a byte inside every `every`-th record's payload (its header intact)."""
    o = orc.file_reader_decode(bytes(img))
    b = bytearray(img)
    rng = random.Random(seed)
    offs = o["rec_off"] + [len(b)]
    for i in range(0, len(o["rec_off"]), every):
        lo, hi = offs[i] + 40, offs[i + 1] - 4
        if hi > lo:
            b[rng.randrange(lo, hi)] ^= 0x5A
    return bytes(b)


def test_c4_shape_eight_files():
    """8 files of 64 KiB text-like Snappy records (the C4 shape at 1/40 of its size), seeds 100..107."""
    imgs = [generate(400, 65536, 2, kind=1, seed=100 + k).tobytes() for k in range(8)]
    check_batch(imgs, "c4")


def test_mixed_codecs_and_shapes():
    imgs = [generate(300, 65536, 2, kind=1, seed=1).tobytes(),   # large records: coop
            generate(5000, 1024, 2, kind=1, seed=2).tobytes(),   # small records: lane decoder
            generate(300, 20000, 2, kind=2, seed=3).tobytes(),   # incompressible: literal copy
            generate(2000, 700, 0, kind=0, seed=4).tobytes(),    # uncompressed
            generate(200, 4096, 1, kind=1, seed=5).tobytes(),    # gzip
            corpus.encode_file([], 2),                          # header only
            b"\x04\x00\x00",                                   # short file header
            generate(50, 100000, 2, kind=1, seed=6).tobytes()]
    check_batch(imgs, "mixed")


def test_damaged_large_records():
    """Corrupt payloads inside 64 KiB records: the coop decoder flags exactly the oracle's records."""
    base = generate(120, 65536, 2, kind=1, seed=9).tobytes()
    imgs = [_damage_records(base, 7, 1), _damage_records(base, 3, 2), base]
    check_batch(imgs, "damaged")


def test_more_files_than_one_group():
    imgs = [generate(30 + 7 * k, 30000, 2, kind=1, seed=200 + k).tobytes() for k in range(19)]
    check_batch(imgs, "19 files")


def test_batch_equals_single_calls():
    imgs = [generate(100, 65536, 2, kind=k % 2 + 1, seed=300 + k).tobytes() for k in range(4)]
    files = [to_device_file(img) for img in imgs]
    batch = decoder().decode_batch(files)
    for (d, n), (b, info) in zip(files, batch):
        b1, i1 = decoder().decode(d, n)
        assert info["status"] == i1["status"] and info["n_records"] == i1["n_records"]
        nb = info["total_out_bytes"]
        assert bytes(b.out[:nb].cpu().numpy()) == bytes(b1.out[:nb].cpu().numpy())


def test_full_c4_file_exact():
    """One whole C4 file (BASELINE configs[3]: 16384 x 64 KiB text-like Snappy records, seed 100, as
    bench.py generates it) through rio_device_decode_batch, every byte and offset against the oracle.
    A second, small file shares the batch so the launch deals its waves over two files."""
    big = generate(16384, 65536, 2, kind=1, seed=100, threads=16)
    small = generate(3000, 1024, 2, kind=1, seed=5)
    files = [to_device_file(big), to_device_file(small)]
    got = decoder().decode_batch(files)
    del files
    for k, (img, (b, info)) in enumerate(zip((big, small), got)):
        assert info["status"] == 1 and info["n_records"] == (16384, 3000)[k], info
        o = orc.file_reader_decode_arrays(img)
        assert_same_as_oracle(_host(b, info), o, f"c4-full[{k}]")


@pytest.fixture
def coop_decoder(monkeypatch):
    """A decoder whose ctx sends every Snappy file to the wave-per-record decoder (RIO_COOP_MIN=0)."""
    import ctypes

    from recordio import _lib as L
    from recordio.device import DeviceDecoder

    monkeypatch.setenv("RIO_COOP_MIN", "0")
    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    dec = DeviceDecoder.__new__(DeviceDecoder)
    dec.device, dec.ctx = 0, h.value
    yield dec
    L.lib().rio_ctx_destroy(h)


def test_coop_batch_over_several_files(coop_decoder):
    """k_snappy_coop_batch across files: waves are numbered blockIdx * waves + wave over the grid for
    every file in turn, so files of different record counts, damaged records, a gzip file and an
    uncompressed file (both skipped by the Snappy decoders) share one launch."""
    base = generate(150, 65536, 2, kind=1, seed=9).tobytes()
    imgs = [generate(700, 3000, 2, kind=1, seed=21).tobytes(),
            _damage_records(base, 5, 3),
            generate(20, 200000, 2, kind=1, seed=22).tobytes(),
            generate(4000, 100, 2, kind=1, seed=23).tobytes(),
            generate(100, 4096, 1, kind=1, seed=24).tobytes(),
            generate(500, 900, 0, kind=0, seed=25).tobytes(),
            corpus.encode_file([], 2),
            generate(1, 65536, 2, kind=2, seed=26).tobytes()]
    files = [to_device_file(img) for img in imgs]
    got = coop_decoder.decode_batch(files)
    for k, (img, (b, info)) in enumerate(zip(imgs, got)):
        assert_same_as_oracle(_host(b, info), orc.file_reader_decode_arrays(img), f"coop-batch[{k}]")


def test_coop_batch_more_files_than_one_group(coop_decoder):
    imgs = [generate(9 + 5 * k, 40000, 2, kind=1, seed=400 + k).tobytes() for k in range(19)]
    files = [to_device_file(img) for img in imgs]
    got = coop_decoder.decode_batch(files)
    for k, (img, (b, info)) in enumerate(zip(imgs, got)):
        assert_same_as_oracle(_host(b, info), orc.file_reader_decode_arrays(img), f"coop-19[{k}]")


def test_bench_c4_batch_eight_full_files():
    """The exact shape bench.py times for C4 (BASELINE configs[3]): 8 whole files of 16 384 x 64 KiB text-like Snappy
    records, seeds 100..107, in ONE rio_device_decode_batch (131 072 records, one per decoder lane, all in flight at
    once), every file compared byte for byte with the oracle's FileReader loop (VERDICT r5 What's weak 1). The oracle
    decodes run on host threads (the ctypes calls release the GIL), one file's arrays on the host at a time each."""
    from concurrent.futures import ThreadPoolExecutor

    imgs = [generate(16384, 65536, 2, kind=1, seed=100 + k, threads=16) for k in range(8)]
    files = [to_device_file(img) for img in imgs]
    got = decoder().decode_batch(files)
    del files

    def one(k):
        b, info = got[k]
        assert info["status"] == 1 and info["n_records"] == 16384, (k, info)
        assert_same_as_oracle(_host(b, info), orc.file_reader_decode_arrays(imgs[k]), f"c4-bench[{k}]")
        return k

    with ThreadPoolExecutor(4) as ex:
        assert sorted(ex.map(one, range(8))) == list(range(8))
