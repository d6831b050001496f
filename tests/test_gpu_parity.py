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
    for vd in ("v4_compat", "v3_compat", "v2_compat", "v1_compat"):
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
    for name in ("v2_embedded_same", "v1_embedded_same"):  # the older layouts' own marker bytes
        img = dict(CASES)[name]
        g = gpu_decode_arrays(img)
        assert g["n_repairs"] > 0, name
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), name)


@pytest.mark.parametrize("chunk", [64, 256, 1024, 4096, 65536])
def test_chunk_size_independent(chunk, monkeypatch):
    """The result does not depend on the framing chunk size (speculation granularity): at 64-byte
    chunks the files have thousands of chunks and speculations that break and are repaired."""
    import ctypes

    from recordio import _lib as L
    from recordio.device import DeviceDecoder, to_device_file

    monkeypatch.setenv("RIO_CHUNK_BYTES", str(chunk))
    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    try:
        dec = DeviceDecoder.__new__(DeviceDecoder)
        dec.device, dec.ctx = 0, h.value
        for name in ("mixed_c2", "mixed_c0_embedded", "text_snappy_64k", "mixed_c2_flip", "v2_embedded", "v2_empty_records",
                     "v1_mixed_c2", "v1_torn_header_12"):
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


def _big_uncompressed(seed, hi, n=3000):
    """Uncompressed records averaging >= 256 bytes: sizes around the copy's 16-byte pieces and its 1 KiB rounds
    (k_copy_records, 16-lane groups), empty and nil records."""
    import random

    rng = random.Random(seed)
    recs = []
    for _ in range(n):
        if rng.random() < 0.03:
            recs.append(None)
            continue
        ln = rng.choice([0, 1, 15, 16, 17, 255, 256, 1023, 1024, 1025, 2048, rng.randint(0, hi)])
        recs.append(rng.randbytes(ln))
    return corpus.encode_file(recs, 0)


@pytest.mark.parametrize("seed,hi", [(21, 600), (22, 3000), (23, 20000)])
def test_uncompressed_large_records_whole_file(seed, hi):
    """Whole files, a truncated end and a zero tail of large uncompressed records (the 16-lane copy groups): every
    decode is the oracle's."""
    img = _big_uncompressed(seed, hi)
    for name, im in ((f"s{seed}", img), (f"s{seed}_trunc", img[: len(img) * 2 // 3]),
                     (f"s{seed}_zero_tail", img + bytes(5000))):
        o = orc.file_reader_decode_arrays(im)
        assert o["total_out_bytes"] >= 256 * o["n_records"], name
        assert_same_as_oracle(gpu_decode_arrays(im), o, name)


@pytest.mark.parametrize("chunk", [64, 1024, 16384])
def test_uncompressed_large_records_any_chunk_size(chunk, monkeypatch):
    """The same files when records span many chunks (64-byte chunks: most own no record) or share one."""
    import ctypes

    from recordio import _lib as L
    from recordio.device import DeviceDecoder, to_device_file

    monkeypatch.setenv("RIO_CHUNK_BYTES", str(chunk))
    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    try:
        dec = DeviceDecoder.__new__(DeviceDecoder)
        dec.device, dec.ctx = 0, h.value
        img = _big_uncompressed(24, 5000, n=1500)
        o = orc.file_reader_decode_arrays(img)
        d_file, n = to_device_file(img)
        b, info = dec.decode(d_file, n)
        k = info["n_records"]
        g = dict(info, out=b.out[: info["total_out_bytes"]].cpu().numpy(), out_off=b.out_off[: k + 1].cpu().numpy(),
                 rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())
        assert_same_as_oracle(g, o, f"big_uncompressed@{chunk}")
    finally:
        L.lib().rio_ctx_destroy(h)


def _handle_read_next_at(r, off):
    """C-ABI status and details of the reader handle's ReadNextAt (rio_reader_read_next_at)."""
    import ctypes

    from recordio import _lib as L

    data, n, nil = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int()
    rc = L.lib().rio_reader_read_next_at(r._h, off, ctypes.byref(data), ctypes.byref(n), ctypes.byref(nil))
    d0, d1, eo = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    L.lib().rio_reader_last_detail(r._h, ctypes.byref(d0), ctypes.byref(d1), ctypes.byref(eo))
    return rc, d0.value, d1.value


def _handle_seek_next(r, off):
    import ctypes

    from recordio import _lib as L

    data, n, nil, ro = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64()
    rc = L.lib().rio_reader_seek_next(r._h, off, ctypes.byref(ro), ctypes.byref(data), ctypes.byref(n),
                                      ctypes.byref(nil))
    return rc, ro.value


def _offsets(img, k=150):
    """Every offset of a small file, else a seeded sample plus the boundaries."""
    import random

    if len(img) <= 8192:
        return list(range(len(img) + 3))
    rng = random.Random(1)
    return [rng.randint(0, len(img) + 3) for _ in range(k)] + [len(img), len(img) - 1, len(img) + 1, 0, 7, 8]


@pytest.mark.parametrize("name", ["mixed_c0", "mixed_c2", "v3_mixed_snappy", "nil_snappy", "mixed_c2_trunc3",
                                  "mixed_c2_flip", "damaged_small_c0", "damaged_small_c2", "header_too_long",
                                  "size_overflow", "snappy_corrupt_mid", "huge_u", "snappy_short_mid",
                                  "snappy_bad_preamble_mid", "v2_mixed_c2", "v2_mixed_c0_trunc1", "v2_embedded",
                                  "v2_empty_records", "v1_mixed_c2", "v1_mixed_c0_trunc2", "v1_torn_header_12",
                                  "v1_bad_magic_mid", "v1_huge_u"])
def test_read_next_at_every_record_start_and_random_offsets(name, tmp_path):
    """ReadNextAt at record starts and at random offsets: the record, or exactly the oracle's status
    class (and CRC details), and through the mirror the reference's error value (message, sentinel,
    wrap depth: mmap_reader.go:130-203)."""
    from go_errors import assert_go_error, expect_read_next_at
    from recordio import NewMemoryMappedReaderWithPath

    img = dict(CASES)[name]
    p = tmp_path / "f"
    p.write_bytes(img)
    r, err = NewMemoryMappedReaderWithPath(str(p))
    assert err is None and r.Open() is None
    o = orc.file_reader_decode(img)
    for k, (off, rec) in enumerate(zip(o["rec_off"], o["records"])):
        if k % 7 and not isinstance(rec, orc.BadRecord):
            continue
        got, err = r.ReadNextAt(off)
        if isinstance(rec, orc.BadRecord):  # mmap_reader.go:186-191: the codec error, wrapped once
            assert_go_error(err, expect_read_next_at(STATUS["DECOMPRESS"], off, str(p), version=img[0]))
            continue
        assert err is None and got == rec, off
    n_fail = 0
    for off in _offsets(img):
        st, want, d0, d1 = orc.read_next_at(img, off, details=True)
        rc, g0, g1 = _handle_read_next_at(r, off)
        assert rc == st, (off, rc, st)
        got, err = r.ReadNextAt(off)
        if st == 0:
            assert err is None and got == want, off
            continue
        n_fail += 1
        if st == STATUS["HEADER_CRC"]:
            assert (g0, g1) == (d0, d1), off
        assert got is None
        assert_go_error(err, expect_read_next_at(st, off, str(p), d0, d1, version=img[0]))
    assert n_fail > 0
    r.Close()


@pytest.mark.parametrize("name", ["asc_none", "nil_snappy", "v3_mixed_none", "damaged_small_c0", "damaged_small_c2",
                                  "snappy_corrupt_mid", "snappy_short_mid", "random_snappy_1k", "text_snappy_64",
                                  "v2_mixed_c2", "v2_embedded", "v2_empty_records", "v1_mixed_c0"])
def test_seek_next_matches_oracle_on_every_offset(name, tmp_path):
    """SeekNext from every third offset: the record and its offset, or exactly the oracle's status
    (with the failing trial's offset), and the reference's error value through the mirror."""
    from go_errors import assert_go_error, expect_seek_next
    from recordio import NewMemoryMappedReaderWithPath

    img = dict(CASES)[name][:6000]
    p = tmp_path / "f"
    p.write_bytes(img)
    r, _ = NewMemoryMappedReaderWithPath(str(p))
    r.Open()
    for seek_len in (4096, 10, 2):  # below 3 a marker never fits a window (the host index is not used)
        r.seekLen = seek_len
        for off in list(range(0, len(img) + 1, 3)) + [len(img) + 1]:
            st, ro, want = orc.seek_next(img, off, seek_len)
            rc, g_ro = _handle_seek_next(r, off)
            assert rc == st, (off, seek_len, rc, st)
            g_off, got, err = r.SeekNext(off)
            if st == 0:
                assert err is None and (g_off, got) == (ro, want), (off, seek_len)
                continue
            if st not in (STATUS["EOF"], STATUS["INVALID_OFFSET"]):
                assert g_ro == ro, (off, seek_len)  # the failing trial
            assert (g_off, got) == (0, None)
            if st == STATUS["UNSUPPORTED"]:  # v1: mmap_reader.go:62-64, before any scan
                assert str(err) == "unsupported on files with version lower than v2"
                continue
            assert_go_error(err, expect_seek_next(st, off, ro, str(p), version=img[0]))
    r.Close()


def test_full_size_headline_workload_exact():
    """C2 at full size (1M x 1 KiB snappy text-like): every byte and offset equals the oracle."""
    img = corpus.generate(1_000_000, 1024, 2, kind=1, seed=1)
    o = orc.file_reader_decode_arrays(img)
    g = gpu_decode_arrays(img)
    assert o["n_records"] == 1_000_000 and o["status"] == STATUS["EOF"]
    assert_same_as_oracle(g, o, "C2")


@pytest.mark.parametrize("version", [3, 2, 1])
def test_full_size_headline_workload_older_versions(version):
    """The C2 workload (1M x 1 KiB snappy text-like) re-framed with the v3 / v2 / v1 header layouts
    (readRecordHeaderV3 / V2 / V1): every byte and offset equals the oracle."""
    img = corpus.to_version(bytes(corpus.generate(1_000_000, 1024, 2, kind=1, seed=1)), version)
    o = orc.file_reader_decode_arrays(img)
    g = gpu_decode_arrays(img)
    assert o["n_records"] == 1_000_000 and o["status"] == STATUS["EOF"] and img[0] == version
    assert_same_as_oracle(g, o, f"C2 v{version}")


def test_full_size_c3_10m_64b_records_exact():
    """C3 at full size (10M x 64 B snappy text-like, seed 3 as bench.py): sortedness and sizes, then
    every byte and offset against the oracle."""
    img = corpus.generate(10_000_000, 64, 2, kind=1, seed=3)
    g = gpu_decode_arrays(img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == 10_000_000
    assert np.all(np.diff(g["rec_off"]) > 0) and np.all(np.diff(g["out_off"]) == 64)
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o, "C3-10M")


@pytest.mark.parametrize("name", ["mixed_c0", "mixed_c2", "nil_snappy", "mixed_c2_zero_tail", "v3_mixed_snappy"])
def test_compression_hint_launches_only_that_codec(name):
    """rio_device_decode_ex with the header's compression type decodes exactly as the unhinted call;
    a hint the header contradicts comes back RIO_ERR_ARG with nothing decoded."""
    from gpu_util import decoder
    from recordio import _lib as L
    from recordio.device import to_device_file

    img = dict(CASES)[name]
    comp = img[4]
    d, n = to_device_file(img)
    b, info = decoder().decode(d, n, comp=comp)
    o = orc.file_reader_decode_arrays(img)
    k, nb = info["n_records"], info["total_out_bytes"]
    g = dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:k + 1].cpu().numpy(),
             rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())
    assert_same_as_oracle(g, o, name)
    wrong = 1 if comp != 1 else 2
    _, bad = decoder().decode(d, n, comp=wrong)
    assert bad["status"] == L.RIO_ERR_ARG and bad["n_records"] == 0


@pytest.mark.parametrize("n,ln", [(1, 300), (2, 40), (63, 200), (64, 200), (65, 200), (127, 100), (4097, 64),
                                  (131071, 16), (131073, 16), (1_048_577, 24), (2_100_001, 12)])
def test_record_counts_around_decoder_chunks(n, ln):
    """Snappy files whose record counts sit on and around the lane decoder's chunk boundaries (64
    lanes x records per lane per chunk; one record per lane up to 8 x 64 x waves records, two past
    2 M), so partial chunks, idle lanes and the chunk counter's last claims are all exercised."""
    img = corpus.generate(n, ln, 2, kind=1, seed=n)
    g = gpu_decode_arrays(img)
    o = orc.file_reader_decode_arrays(img)
    assert o["n_records"] == n
    assert_same_as_oracle(g, o, f"{n} x {ln}")
