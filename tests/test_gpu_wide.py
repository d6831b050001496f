"""Files past 32-bit positions on the device (GPU): >= 4 GiB device-resident decodes.

The reference's own read benchmark uses 4 GiB and 8 GiB files (benchmark/recordio_read_test.go:26-27).
A file or decoded arena of 4 GiB or more leaves the lane decoder's 32-bit stream positions, so a
Snappy file of that size takes the wave-per-record decoder (k_snappy_coop, 64-bit addressing); an
uncompressed one takes the copy kernel. Both are compared with the oracle byte for byte. The same
wave-per-record decoder is also forced onto ordinary files here (RIO_COOP_MIN=0) so that its parity
is checked on the whole corpus, not only on the rare huge file.
"""
import ctypes

import numpy as np
import pytest

import corpus
import oracle_py as orc
from conftest import STATUS
from gpu_util import assert_same_as_oracle, gpu_decode_arrays

pytestmark = pytest.mark.gpu

FOUR_GIB = 1 << 32


def _repetitive_snappy_file(n_records):
    """n_records identical 64 KiB records of a 100-byte pattern: Snappy turns each into a literal and
    ~1000 64-byte copies (~3 KB), so the decoded arena passes 4 GiB while the file stays ~200 MB."""
    pat = bytes((i * 37 + 11) & 0xFF for i in range(100))
    rec = (pat * 656)[:65536]
    one = corpus.encode_file([rec], 2)
    body = np.frombuffer(one[8:], dtype=np.uint8)
    img = np.concatenate([np.frombuffer(one[:8], dtype=np.uint8), np.tile(body, n_records)])
    return img, rec


def test_snappy_decoded_arena_past_4gib():
    img, rec = _repetitive_snappy_file(70_000)  # 70000 x 64 KiB = 4.59 GB decoded
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == 70_000
    assert g["total_out_bytes"] == 70_000 * 65536 > FOUR_GIB
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o, "snappy >4GiB arena")
    # and independently of the oracle: every record is the source record
    out = g["out"].reshape(70_000, 65536)
    assert np.array_equal(out[0], np.frombuffer(rec, dtype=np.uint8)) and (out == out[0]).all()


def test_uncompressed_file_past_4gib():
    """recordio_read_test.go's shape: 1 KiB uncompressed records, a 4.3 GB file."""
    from recordio import generate

    n = 4_200_000
    img = generate(n, 1024, 0, kind=0, seed=1, threads=16)
    assert img.shape[0] > FOUR_GIB
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == n
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o, "uncompressed >4GiB file")


@pytest.fixture
def coop_ctx(monkeypatch):
    """A decoder whose ctx sends every Snappy file to k_snappy_coop."""
    from recordio import _lib as L
    from recordio.device import DeviceDecoder

    monkeypatch.setenv("RIO_COOP_MIN", "0")
    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    dec = DeviceDecoder.__new__(DeviceDecoder)
    dec.device, dec.ctx = 0, h.value
    yield dec
    L.lib().rio_ctx_destroy(h)


SNAPPY_CASES = [(n, img) for n, img in corpus.cases() if img[4:5] == b"\x02"]


@pytest.mark.parametrize("name,image", SNAPPY_CASES, ids=[n for n, _ in SNAPPY_CASES])
def test_wave_decoder_on_the_corpus(coop_ctx, name, image):
    from recordio.device import to_device_file

    d, n = to_device_file(image)
    b, info = coop_ctx.decode(d, n)
    k = info["n_records"]
    g = dict(info)
    if k or info["total_out_bytes"]:
        g.update(out=b.out[:info["total_out_bytes"]].cpu().numpy(), out_off=b.out_off[:k + 1].cpu().numpy(),
                 rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())
    o = orc.file_reader_decode_arrays(image)
    if o["status"] == STATUS["SHORT_FILE_HEADER"]:
        assert g["status"] == o["status"]
        return
    assert_same_as_oracle(g, o, name)


def test_wave_decoder_on_large_and_damaged_records(coop_ctx):
    from recordio import generate
    from recordio.device import to_device_file
    from test_gpu_batch import _damage_records

    for k, img in enumerate([generate(200, 65536, 2, kind=1, seed=11).tobytes(),
                             _damage_records(generate(150, 40000, 2, kind=1, seed=12).tobytes(), 5, 3)]):
        d, n = to_device_file(img)
        b, info = coop_ctx.decode(d, n)
        kk = info["n_records"]
        g = dict(info, out=b.out[:info["total_out_bytes"]].cpu().numpy(), out_off=b.out_off[:kk + 1].cpu().numpy(),
                 rec_off=b.rec_off[:kk].cpu().numpy(), flags=b.flags[:kk].cpu().numpy())
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), f"coop {k}")


@pytest.mark.timeout(900)
def test_snappy_file_past_4gib():
    """A text-like Snappy file past 4 GiB (9 M x 1 KiB records, 4.6 GB in, 9.2 GB out): since round 4 the
    lane decoder takes it (its buffer descriptors start at each wave's lowest record, so 32-bit offsets
    reach any file size), not the wave-per-record decoder. Byte for byte against the oracle."""
    from recordio import generate

    n = 9_000_000
    img = generate(n, 1024, 2, kind=1, seed=3, threads=16)
    assert img.shape[0] > FOUR_GIB
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == n and g["total_out_bytes"] > 2 * FOUR_GIB
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o, "snappy >4GiB file")


@pytest.mark.timeout(900)
def test_snappy_wave_span_past_32_bits():
    """70 Snappy records of 64 MiB: the first wave's 64 records span 4 GiB of arena, more than its 32-bit
    buffer offsets reach, so that wave decodes its records one thread each (snappy_lane's span guard);
    the last 6 records take the lane decoder. Byte for byte against the oracle."""
    from recordio import generate

    n = 70
    img = generate(n, 64 << 20, 2, kind=1, seed=5, threads=16)
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == n and g["total_out_bytes"] == n << 26
    assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), "64 MiB records")


def _crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 & -(c & 1))
    return c ^ 0xFFFFFFFF


def _uvarint(x: int) -> bytes:
    o = bytearray()
    while x >= 0x80:
        o.append((x & 0x7F) | 0x80)
        x >>= 7
    o.append(x)
    return bytes(o)


@pytest.mark.parametrize("size", [FOUR_GIB - 1, FOUR_GIB + 4096])
def test_uncompressed_record_of_4gib(size):
    """One uncompressed v4 record whose length does not fit rec_desc's 32-bit fields (2^32 - 1 is the
    sentinel itself): its stream position and length come from rec_pay (k_place writes it for such a
    record only, rio_device.h rec_stream), and k_copy_records moves it whole."""
    head = b"\x91\x8d\x4c\x00" + _uvarint(size) + _uvarint(0)  # v4, not nil, u = size, c = 0 (uncompressed)
    head += _uvarint(_crc32c(head))
    fh = np.frombuffer(bytes.fromhex("0400000000000000"), dtype=np.uint8)  # v4, compression 0
    payload = np.resize(np.arange(251, dtype=np.uint8), size)
    img = np.concatenate([fh, np.frombuffer(head, dtype=np.uint8), payload])
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == 1 and g["total_out_bytes"] == size
    assert int(g["rec_off"][0]) == 8 and int(g["out_off"][1]) == size
    assert np.array_equal(g["out"][:size], payload)


@pytest.mark.timeout(900)
def test_batch_with_a_file_past_4gib():
    """rio_device_decode_batch over a 4.6 GB Snappy file and two small ones: the batched lane decoder
    takes the big file too (per-wave buffer bases), each file exactly the oracle's."""
    from recordio import generate
    from test_gpu_batch import check_batch

    big = generate(9_000_000, 1024, 2, kind=1, seed=4, threads=16)
    assert big.shape[0] > FOUR_GIB
    check_batch([generate(3000, 1024, 2, kind=1, seed=6), big, generate(200, 65536, 2, kind=1, seed=8)], "batch >4GiB")
