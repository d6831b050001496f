"""Device decode path vs the oracle, bit-exact (GPU).

Whole-file decode (rio_device_decode) must deliver the same records, record offsets, nil flags,
terminal status and status offset as the FileReader.ReadNext loop the oracle restates; single
records (ReadNextAt) and SeekNext must match MMapReader on every offset tried.
"""
import os

import numpy as np
import pytest

import corpus
import oracle_py as orc
from conftest import STATUS, read_fixture
from gpu_util import assert_same_as_oracle, gpu_decode_arrays

pytestmark = pytest.mark.gpu

CASES = corpus.cases()


def _fixture_images():
    from conftest import GOLDEN

    out = []
    for vd in ("v4_compat", "v3_compat"):
        for name in sorted(os.listdir(os.path.join(GOLDEN, vd))):
            out.append((f"{vd}/{name}", read_fixture(vd, name)))
    return out


UNSUPPORTED_ON_GPU = (STATUS["UNSUPPORTED"],)


@pytest.mark.parametrize("name,image", _fixture_images(), ids=[n for n, _ in _fixture_images()])
def test_fixture_whole_file(name, image):
    o = orc.file_reader_decode_arrays(image)
    g = gpu_decode_arrays(image)
    if o["status"] in (STATUS["VERSION"], STATUS["COMPRESSION_TYPE"]):
        assert g["status"] == o["status"] and g["detail0"] == o["detail0"]
        return
    assert_same_as_oracle(g, o, name)


@pytest.mark.parametrize("name,image", CASES, ids=[n for n, _ in CASES])
def test_corpus_whole_file(name, image):
    o = orc.file_reader_decode_arrays(image)
    g = gpu_decode_arrays(image)
    if o["status"] == STATUS["SHORT_FILE_HEADER"]:
        assert g["status"] == o["status"]
        return
    assert_same_as_oracle(g, o, name)


def test_repairs_happen_and_stay_exact():
    """Embedded recordio payloads put CRC-valid false headers at chunk starts: the scan must detect
    the broken speculation and re-walk, with results identical to the sequential oracle."""
    img = dict(CASES)["mixed_c0_embedded"]
    g = gpu_decode_arrays(img)
    assert g["n_repairs"] > 0
    assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), "embedded")


@pytest.mark.parametrize("chunk", [64, 256, 1024, 4096, 65536])
def test_chunk_size_independent(chunk, monkeypatch):
    """The result does not depend on the framing chunk size (speculation granularity)."""
    import ctypes

    from recordio import _lib as L
    from recordio.device import DeviceDecoder, to_device_file

    monkeypatch.setenv("RIO_CHUNK_BYTES", str(chunk))
    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    try:
        dec = DeviceDecoder.__new__(DeviceDecoder)
        dec.device, dec.ctx = 0, h.value
        for name in ("mixed_c2", "mixed_c0_embedded", "text_snappy_64k", "mixed_c2_flip"):
            img = dict(CASES)[name]
            o = orc.file_reader_decode_arrays(img)
            d_file, n = to_device_file(img)
            b, info = dec.decode(d_file, n)
            k = info["n_records"]
            g = dict(info, out=b.out[: info["total_out_bytes"]].cpu().numpy(), out_off=b.out_off[: k + 1].cpu().numpy(),
                     rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())
            assert_same_as_oracle(g, o, f"{name}@{chunk}")
    finally:
        L.lib().rio_ctx_destroy(h)


@pytest.mark.parametrize("name", ["mixed_c0", "mixed_c2", "v3_mixed_snappy", "nil_snappy", "mixed_c2_trunc3"])
def test_read_next_at_every_record_start_and_random_offsets(name, tmp_path):
    from recordio import NewMemoryMappedReaderWithPath

    img = dict(CASES)[name]
    p = tmp_path / "f"
    p.write_bytes(img)
    r, err = NewMemoryMappedReaderWithPath(str(p))
    assert err is None and r.Open() is None
    o = orc.file_reader_decode(img)
    for off, rec in list(zip(o["rec_off"], o["records"]))[::7]:
        got, err = r.ReadNextAt(off)
        assert err is None and got == rec, off
    import random

    rng = random.Random(1)
    for off in [rng.randint(0, len(img) + 3) for _ in range(150)] + [len(img), len(img) - 1, len(img) + 1]:
        st, want = orc.read_next_at(img, off)
        got, err = r.ReadNextAt(off)
        if st == 0:
            assert err is None and got == want, off
        else:
            assert err is not None, (off, st)
    r.Close()


@pytest.mark.parametrize("name", ["asc_none", "nil_snappy", "v3_mixed_none"])
def test_seek_next_matches_oracle_on_every_offset(name, tmp_path):
    from recordio import NewMemoryMappedReaderWithPath

    img = dict(CASES)[name][:6000]
    p = tmp_path / "f"
    p.write_bytes(img)
    r, _ = NewMemoryMappedReaderWithPath(str(p))
    r.Open()
    for seek_len in (4096, 10):
        r.seekLen = seek_len
        for off in range(0, len(img) + 1, 3):
            st, ro, want = orc.seek_next(img, off, seek_len)
            g_off, got, err = r.SeekNext(off)
            if st == 0:
                assert err is None and (g_off, got) == (ro, want), (off, seek_len)
            else:
                assert err is not None, (off, st)
    r.Close()


def test_full_size_headline_workload_exact():
    """C2 at full size (1M x 1 KiB snappy text-like): every byte and offset equals the oracle."""
    img = corpus.generate(1_000_000, 1024, 2, kind=1, seed=1)
    o = orc.file_reader_decode_arrays(img)
    g = gpu_decode_arrays(img)
    assert o["n_records"] == 1_000_000 and o["status"] == STATUS["EOF"]
    assert_same_as_oracle(g, o, "C2")


def test_full_size_properties_64b_records():
    """C3 shape (header-bound, 64 B records): counts, sortedness and a checksum of checksums."""
    img = corpus.generate(2_000_000, 64, 2, kind=1, seed=3)
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == 2_000_000
    assert np.all(np.diff(g["rec_off"]) > 0) and np.all(np.diff(g["out_off"]) == 64)
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o, "C3-2M")
