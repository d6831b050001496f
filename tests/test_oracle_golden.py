"""Pins the oracle (oracle/rio_oracle.c) to the reference's fixtures and test assertions (CPU).

Mirrors recordio/file_reader_test.go, file_reader_v{1,2,3}compat_test.go, mmap_reader_test.go,
mmap_reader_v{1,2,3}compat_test.go and checksum_byte_reader_test.go on the copied fixture files.
"""
import ctypes
import zlib

import pytest

import oracle_py as orc
from conftest import STATUS, read_fixture, spec_bytes

VERSIONS = ["v4_compat", "v3_compat", "v2_compat", "v1_compat"]


def _cases(expectations, key):
    out = []
    for vd in VERSIONS:
        for name, exp in sorted(expectations[vd].items()):
            if key in exp:
                out.append((vd, name))
    return out


def test_crc_kat(expectations):
    # checksum_byte_reader_test.go:30 — crc32c(91 8d 4c) == 0x0967294b
    assert orc.crc32c(bytes([0x91, 0x8D, 0x4C])) == expectations["kats"]["crc32c_magic"]
    # worked example: header 91 8d 4c 00 0d 00 of the SingleRecord fixture
    assert orc.crc32c(bytes([0x91, 0x8D, 0x4C, 0x00, 0x0D, 0x00])) == expectations["kats"]["single_record_header_crc"]


@pytest.mark.parametrize("vd", VERSIONS)
def test_file_reader_fixtures(vd, expectations):
    for name, exp in sorted(expectations[vd].items()):
        data = read_fixture(vd, name)
        res = orc.file_reader_decode(data)
        if "open" in exp:
            st, val = exp["open"]
            assert res["status"] == STATUS[st], name
            assert res["detail0"] == val, name
            continue
        assert res["compression"] == exp.get("compression", 0), name
        assert res["version"] == int(vd[1]), name
        if exp.get("header_only"):  # the reference checks only the header's compression type
            continue
        want = [spec_bytes(s) for s in exp["records"]]
        assert res["records"] == want, name
        assert res["status"] == STATUS[exp["end"]], (name, res["status"])


@pytest.mark.parametrize("vd", VERSIONS)
def test_mmap_read_at_fixtures(vd, expectations):
    for name, exp in sorted(expectations[vd].items()):
        data = read_fixture(vd, name)
        for off, want in exp.get("read_at", []):
            st, rec = orc.read_next_at(data, off)
            if isinstance(want, str):
                assert st == STATUS[want], (name, off, st)
            else:
                assert st == 0, (name, off, st)
                assert rec == spec_bytes(want), (name, off)


@pytest.mark.parametrize("vd", VERSIONS)
def test_read_at_every_record_start_equals_sequential(vd, expectations):
    """record_i == ReadNextAt(rec_off_i) for every record the sequential reader delivers."""
    for name, exp in sorted(expectations[vd].items()):
        if "records" not in exp:
            continue
        data = read_fixture(vd, name)
        res = orc.file_reader_decode(data)
        for off, rec in zip(res["rec_off"], res["records"]):
            st, r2 = orc.read_next_at(data, off)
            assert st == 0 and r2 == rec, (name, off)


def test_seek_next_legacy_versions():
    # mmap_reader.go:62-64: SeekNext on v1 is "unsupported on files with version lower than v2";
    # v2 has the same marker bytes and scan as v3 / v4
    v1 = read_fixture("v1_compat", "recordio_UncompressedWriterMultiRecord_asc")
    assert orc.seek_next(v1, 0)[0] == STATUS["UNSUPPORTED"]
    v2 = read_fixture("v2_compat", "recordio_UncompressedWriterMultiRecord_asc")
    res = orc.file_reader_decode(v2)
    nxt, got = 0, []
    for i in range(5):
        st, ro, rec = orc.seek_next(v2, 0 if i == 0 else nxt + 1)
        assert st == 0
        nxt = ro
        got.append((ro, rec))
    assert got == list(zip(res["rec_off"][:5], res["records"][:5]))


def test_v2_comp1_gzip_content():
    # the v2 _comp1 fixture's record is a gzip member of ascending(1337), checked with zlib
    data = read_fixture("v2_compat", "recordio_UncompressedSingleRecord_comp1")
    res = orc.file_reader_decode(data)
    asc = bytes(i & 0xFF for i in range(1337))
    gz = data.index(b"\x1f\x8b", 8)
    assert zlib.decompress(data[gz:], 16 + 15) == asc and res["records"] == [asc]


@pytest.mark.parametrize("vd", VERSIONS[:2])
def test_seek_next_magic_number_content(vd):
    # mmap_reader_test.go:244-260 / v3compat: SeekNext(0) -> rec1, SeekNext(next+1) -> ... -> EOF
    data = read_fixture(vd, "recordio_UncompressedMagicNumberContent")
    want = [bytes([0x91, 0x8D, 0x4C]), bytes([21, 8, 23]), bytes([0x91, 0x8D, 0x4C])]
    nxt = 0
    for i, w in enumerate(want):
        st, ro, rec = orc.seek_next(data, 0 if i == 0 else nxt + 1)
        assert st == 0 and rec == w
        nxt = ro
    st, _, _ = orc.seek_next(data, nxt + 1)
    assert st == STATUS["EOF"]


def test_comp1_gzip_content():
    # file_reader_generator_test.go:102-108: _comp1 holds ascending(1337) gzip-compressed
    data = read_fixture("v4_compat", "recordio_UncompressedSingleRecord_comp1")
    res = orc.file_reader_decode(data)
    asc = bytes(i & 0xFF for i in range(1337))
    assert res["records"] == [asc]
    gz = data.index(b"\x1f\x8b", 8)  # the payload is a gzip member (GZIP = 1, recordio.go:35-40)
    assert zlib.decompress(data[gz:], 16 + 15) == asc


def test_snappy_decoder_independent_check():
    """Cross-check the oracle's snappy decoder with the system libsnappy where this container has it."""
    try:
        snap = ctypes.CDLL("/opt/conda/lib/libsnappy.so")
    except OSError:
        pytest.skip("libsnappy not present")
    import random

    rng = random.Random(7)
    for n in [0, 1, 7, 64, 1000, 5000, 70000]:
        words = [bytes(rng.choice(b"abcdefgh") for _ in range(rng.randint(1, 6))) for _ in range(50)]
        src = b" ".join(rng.choice(words) for _ in range(n // 3 + 1))[:n]
        cap = ctypes.c_size_t(32 + len(src) * 2)
        out = ctypes.create_string_buffer(cap.value)
        assert snap.snappy_compress(ctypes.c_char_p(src), ctypes.c_size_t(len(src)), out, ctypes.byref(cap)) == 0
        st, dec = orc.snappy_decode(out.raw[:cap.value])
        assert st == 0 and dec == src


def test_snappy_corrupt_inputs():
    # decode.go: bad preamble, offset 0, offset beyond produced bytes, short stream => ErrCorrupt
    assert orc.snappy_decode(b"")[0] == STATUS["DECOMPRESS"]
    assert orc.snappy_decode(b"\x05\x10abcde")[0] == 0  # literal of 5
    assert orc.snappy_decode(b"\x05\x10abcd")[0] == STATUS["DECOMPRESS"]  # literal overruns src
    assert orc.snappy_decode(b"\x08\x0cabcd\x01\x00")[0] == STATUS["DECOMPRESS"]  # copy offset 0
    assert orc.snappy_decode(b"\x08\x0cabcd\x01\x05")[0] == STATUS["DECOMPRESS"]  # offset > produced
    assert orc.snappy_decode(b"\x08\x0cabcd\x01\x04")[1] == b"abcdabcd"  # overlapping-safe copy
    assert orc.snappy_decode(b"\x09\x00a\x11\x01")[1] == b"a" * 9  # copy1 len 8 offset 1 (RLE)
    assert orc.snappy_decode(b"\xff\xff\xff\xff\x1f")[0] == STATUS["DECOMPRESS"]  # > 0xffffffff
