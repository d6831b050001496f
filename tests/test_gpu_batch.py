"""rio_device_decode_batch (GPU): several device-resident files in one call, each exactly the oracle's.

BASELINE configs[3] decodes 8 files of 64 KiB Snappy records per GPU in one step; the batch runs the
framing per file and the large-record decoder (k_snappy_coop_batch) once across the files. Every file
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
