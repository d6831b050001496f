"""The recordio reader mirror (ReaderI / ReadAtI over the device path) on the reference fixtures.

Each test restates a reference test (file:line) through the Python mirror, so the two suites can be
read side by side: recordio/file_reader_test.go, file_reader_v3compat_test.go,
mmap_reader_test.go, mmap_reader_v3compat_test.go, recordio_test.go (end-to-end).
"""
import os

import pytest

from conftest import GOLDEN, fixture_path
from recordio import (EOF, FileHeaderSizeBytes, FileWriter, HeaderChecksumMismatchErr, MagicNumberMismatchErr,
                      NewFileReader, NewFileReaderWithPath, NewMemoryMappedReaderWithPath, errors_is, errors_unwrap)

pytestmark = pytest.mark.gpu
VDS = ["v4_compat", "v3_compat"]


def asc(n):
    return bytes(i & 0xFF for i in range(n))


def opened(vd, name):
    r, err = NewFileReaderWithPath(fixture_path(vd, name))
    assert err is None
    assert r.Open() is None
    return r


def expect_eof(r):  # file_writer_test.go:424-428
    buf, err = r.ReadNext()
    assert buf is None
    assert errors_unwrap(err) is EOF


@pytest.mark.parametrize("vd", VDS)
def test_reader_happy_path_single_record(vd):  # file_reader_test.go:13-24
    r = opened(vd, "recordio_UncompressedSingleRecord")
    buf, err = r.ReadNext()
    assert err is None and buf == asc(13)
    expect_eof(r)
    assert r.Close() is None


@pytest.mark.parametrize("vd", VDS)
@pytest.mark.parametrize("name", ["recordio_UncompressedWriterMultiRecord_asc", "recordio_SnappyWriterMultiRecord_asc"])
def test_reader_happy_path_multi_record(vd, name):  # :26-52
    r = opened(vd, name)
    for n in range(255):
        buf, err = r.ReadNext()
        assert err is None and buf == asc(n)
    expect_eof(r)


@pytest.mark.parametrize("vd", VDS)
@pytest.mark.parametrize("name", ["recordio_UncompressedWriterMultiRecord_asc", "recordio_SnappyWriterMultiRecord_asc"])
def test_reader_skip_every_other(vd, name):  # :54-88
    r = opened(vd, name)
    for n in range(255):
        if n % 2 == 0:
            buf, err = r.ReadNext()
            assert err is None and buf == asc(n)
        else:
            assert r.SkipNext() is None
    expect_eof(r)


@pytest.mark.parametrize("vd", VDS)
def test_reader_skip_all(vd):  # :90-101
    r = opened(vd, "recordio_UncompressedWriterMultiRecord_asc")
    for _ in range(255):
        assert r.SkipNext() is None
    expect_eof(r)


@pytest.mark.parametrize("vd", VDS)
@pytest.mark.parametrize("name,msg", [
    ("recordio_UncompressedSingleRecord_v0", "version mismatch, expected a value from 1 to 4 but was 0"),
    ("recordio_UncompressedSingleRecord_v256", "version mismatch, expected a value from 1 to 4 but was 256"),
])
def test_reader_version_mismatch(vd, name, msg):  # :103-111
    r, _ = NewFileReaderWithPath(fixture_path(vd, name))
    err = r.Open()
    assert err is not None and msg in str(err)


@pytest.mark.parametrize("vd", VDS)
def test_reader_compression_headers(vd):  # :113-134
    for name, comp in [("recordio_UncompressedSingleRecord_comp1", 1), ("recordio_UncompressedSingleRecord_comp2", 2)]:
        r = opened(vd, name)
        assert r.header.compressionType == comp
        r.Close()
    r, _ = NewFileReaderWithPath(fixture_path(vd, "recordio_UncompressedSingleRecord_comp300"))
    assert "unknown compression type [300]" in str(r.Open())


@pytest.mark.parametrize("vd", VDS)
def test_reader_comp1_content(vd):  # file_reader_test.go:114-122: gzip payload of ascending(1337)
    r = opened(vd, "recordio_UncompressedSingleRecord_comp1")
    buf, err = r.ReadNext()
    assert err is None and buf == asc(1337)
    expect_eof(r)


@pytest.mark.parametrize("vd", VDS)
def test_reader_comp2_content(vd):
    r = opened(vd, "recordio_UncompressedSingleRecord_comp2")
    buf, err = r.ReadNext()
    assert err is None and buf == asc(1337)
    expect_eof(r)


@pytest.mark.parametrize("vd", VDS)
def test_reader_magic_number_mismatch(vd):  # :136-144
    r = opened(vd, "recordio_UncompressedSingleRecord_mnm")
    _, err = r.ReadNext()
    assert errors_is(err, MagicNumberMismatchErr)


@pytest.mark.parametrize("vd", VDS)
def test_reader_direct_io(vd):  # :146-172
    r = opened(vd, "recordio_UncompressedSingleRecord_directio")
    rec, err = r.ReadNext()
    assert err is None and rec == bytes([13, 6, 29, 7])
    _, err = r.ReadNext()
    assert errors_is(err, EOF)
    r = opened(vd, "recordio_UncompressedSingleRecord_directio_trailer")
    rec, err = r.ReadNext()
    assert err is None and rec == bytes([13, 6, 29, 7])
    _, err = r.ReadNext()
    assert errors_is(err, MagicNumberMismatchErr)


@pytest.mark.parametrize("vd", VDS)
def test_reader_magic_number_content(vd):  # :174-191
    r = opened(vd, "recordio_UncompressedMagicNumberContent")
    for want in [b"\x91\x8d\x4c", bytes([21, 8, 23]), b"\x91\x8d\x4c"]:
        buf, err = r.ReadNext()
        assert err is None and buf == want
    expect_eof(r)


def test_reader_crc_mismatch():  # :193-200
    r = opened("v4_compat", "recordio_UncompressedCrcFailure")
    _, err = r.ReadNext()
    assert errors_is(err, HeaderChecksumMismatchErr)


def test_reader_forbids_closed_and_double_open():  # :202-219
    r, _ = NewFileReaderWithPath(fixture_path("v4_compat", "recordio_UncompressedSingleRecord"))
    assert r.Close() is None
    _, err = r.ReadNext()
    assert "was either not opened yet or is closed already" in str(err)
    assert "was either not opened yet or is closed already" in str(r.SkipNext())
    assert "is already closed" in str(r.Open())
    r, _ = NewFileReaderWithPath(fixture_path("v4_compat", "recordio_UncompressedSingleRecord"))
    assert r.Open() is None
    assert "already opened" in str(r.Open())


def test_reader_init_errors():  # :221-233
    _, err = NewFileReader()
    assert str(err) == "NewFileReader: either os.File or string path must be supplied, never both"


# ---- MMapReader (mmap_reader_test.go) --------------------------------------------------------

def mm(vd, name):
    r, err = NewMemoryMappedReaderWithPath(fixture_path(vd, name))
    assert err is None and r.Open() is None
    return r


@pytest.mark.parametrize("vd", VDS)
def test_mmap_single_record_and_offsets(vd):  # :13-37, v3compat
    r = mm(vd, "recordio_UncompressedSingleRecord")
    buf, err = r.ReadNextAt(FileHeaderSizeBytes)
    assert err is None and buf == asc(13)
    _, err = r.ReadNextAt(FileHeaderSizeBytes + 1)
    assert str(errors_unwrap(err)) == "magic number mismatch"
    _, err = r.ReadNextAt(42000)
    assert str(errors_unwrap(err)) == "mmap: invalid ReadAt offset 42000"


@pytest.mark.parametrize("vd", VDS)
def test_mmap_small_varint_header_eof(vd):  # :93-106
    hl = 11 if vd == "v4_compat" else 6
    r = mm(vd, "recordio_UncompressedSingleRecord")
    b, err = r.ReadNextAt(FileHeaderSizeBytes + hl + 13)
    assert b is None and err is EOF
    # the reference's `bytes` is the nil of the EOF read above, so len(bytes) = 0: offset 18 (v4) / 13 (v3)
    b, err = r.ReadNextAt(FileHeaderSizeBytes + hl - 1 + len(b or b""))
    assert b is None and str(errors_unwrap(err)) == "magic number mismatch"
    b, err = r.ReadNextAt(FileHeaderSizeBytes + hl - 1 + 13)  # inside the payload: also a mismatch
    assert b is None and str(errors_unwrap(err)) == "magic number mismatch"


@pytest.mark.parametrize("vd", VDS)
def test_mmap_nil_and_empties(vd):  # :108-117
    r = mm(vd, "recordio_UncompressedNilAndEmptyRecord")
    b, err = r.ReadNextAt(FileHeaderSizeBytes)
    assert err is None and b is None
    b, err = r.ReadNextAt(0x13 if vd == "v4_compat" else 14)
    assert err is None and b == b""


@pytest.mark.parametrize("vd", VDS)
def test_mmap_open_errors(vd):  # :39-91
    for name, msg in [("recordio_UncompressedSingleRecord_v0", "but was 0"),
                      ("recordio_UncompressedSingleRecord_v256", "but was 256"),
                      ("recordio_UncompressedSingleRecord_comp300", "unknown compression type [300]")]:
        r, _ = NewMemoryMappedReaderWithPath(fixture_path(vd, name))
        assert msg in str(r.Open())
    r, _ = NewMemoryMappedReaderWithPath(fixture_path(vd, "recordio_UncompressedSingleRecord"))
    assert r.Close() is None
    _, err = r.ReadNextAt(100)
    assert "was either not opened yet or is closed already" in str(err)
    assert "already closed" in str(r.Open())
    r, _ = NewMemoryMappedReaderWithPath(fixture_path(vd, "recordio_UncompressedSingleRecord"))
    assert r.Open() is None
    assert "already opened" in str(r.Open())


@pytest.mark.parametrize("vd", VDS)
def test_mmap_magic_number_contents_seek_chain(vd):  # :244-260
    r = mm(vd, "recordio_UncompressedMagicNumberContent")
    nxt, rec, err = r.SeekNext(0)
    assert err is None and rec == b"\x91\x8d\x4c"
    nxt, rec, err = r.SeekNext(nxt + 1)
    assert err is None and rec == bytes([21, 8, 23])
    nxt, rec, err = r.SeekNext(nxt + 1)
    assert err is None and rec == b"\x91\x8d\x4c"
    _, _, err = r.SeekNext(nxt + 1)
    assert err is EOF


@pytest.mark.parametrize("seek_len", [4096, 10])
def test_mmap_read_sequenced_writes(tmp_path, seek_len):  # :119-242
    p = str(tmp_path / "seq")
    w = FileWriter(p)
    w.Open()
    offsets = [w.Write(bytes([i]))[0] for i in range(127)]
    w.Close()
    r, _ = NewMemoryMappedReaderWithPath(p)
    assert r.Open() is None
    r.seekLen = seek_len
    assert r.Size() == 0x5FC
    for i, off in enumerate(offsets):
        at, err = r.ReadNextAt(off)
        assert err is None and at == bytes([i])
        ofx, at, err = r.SeekNext(off)
        assert err is None and at == bytes([i]) and ofx == off
    j = 0
    for i in range(r.Size()):
        off, nxt, err = r.SeekNext(i)
        if j == len(offsets):
            assert errors_is(err, EOF)
        else:
            assert err is None and nxt == bytes([j]) and off == offsets[j]
            if i >= offsets[j]:
                j += 1


# ---- end to end (recordio_test.go:86-147) ----------------------------------------------------

@pytest.mark.parametrize("comp", [0, 2])
def test_end_to_end_berlin52(tmp_path, comp):
    lines = open(os.path.join(GOLDEN, "berlin52.tsp"), "rb").read().decode().splitlines()
    p = str(tmp_path / "e2e")
    w = FileWriter(p, comp)
    w.Open()
    for ln in lines:
        w.Write(ln.encode())
    w.Write(b"")
    w.Write(None)
    w.Close()
    r, _ = NewFileReaderWithPath(p)
    assert r.Open() is None
    for ln in lines:
        b, err = r.ReadNext()
        assert err is None and b.decode() == ln
    assert len(lines) == 59
    b, err = r.ReadNext()
    assert err is None and b == b""
    b, err = r.ReadNext()
    assert err is None and b is None
    _, err = r.ReadNext()
    assert errors_is(err, EOF)


# ---- recordio v1 / v2 files (file_reader_v{1,2}compat_test.go, mmap_reader_v{1,2}compat_test.go) ----
LEGACY = ["v2_compat", "v1_compat"]


@pytest.mark.parametrize("vd", LEGACY)
def test_legacy_reader_happy_paths(vd):  # file_reader_v2compat_test.go:13-103 / v1compat :12-102
    r = opened(vd, "recordio_UncompressedSingleRecord")
    buf, err = r.ReadNext()
    assert err is None and buf == asc(13)
    expect_eof(r)
    for name in ("recordio_UncompressedWriterMultiRecord_asc", "recordio_SnappyWriterMultiRecord_asc"):
        r = opened(vd, name)
        for n in range(255):
            buf, err = r.ReadNext()
            assert err is None and buf == asc(n), (name, n)
        expect_eof(r)
        r = opened(vd, name)
        for n in range(255):
            if n % 2 == 0:
                buf, err = r.ReadNext()
                assert err is None and buf == asc(n)
            else:
                assert r.SkipNext() is None
        expect_eof(r)
    r = opened(vd, "recordio_UncompressedWriterMultiRecord_asc")
    for _ in range(255):
        assert r.SkipNext() is None
    expect_eof(r)


@pytest.mark.parametrize("vd", LEGACY)
def test_legacy_reader_headers_and_mismatch(vd):  # v2compat :105-139 / v1compat :104-138
    for name, msg in [("recordio_UncompressedSingleRecord_v0", "version mismatch, expected a value from 1 to 4 but was 0"),
                      ("recordio_UncompressedSingleRecord_v256", "version mismatch, expected a value from 1 to 4 but was 256")]:
        r, _ = NewFileReaderWithPath(fixture_path(vd, name))
        assert msg in str(r.Open())
    for name, comp in [("recordio_UncompressedSingleRecord_comp1", 1), ("recordio_UncompressedSingleRecord_comp2", 2)]:
        r = opened(vd, name)
        assert r.header.compressionType == comp and r.header.fileVersion == int(vd[1])
    r = opened(vd, "recordio_UncompressedSingleRecord_mnm")
    _, err = r.ReadNext()
    assert str(errors_unwrap(err)) == "magic number mismatch"


def test_v2_reader_direct_io():  # file_reader_v2compat_test.go:141-167
    r = opened("v2_compat", "recordio_UncompressedSingleRecord_directio")
    rec, err = r.ReadNext()
    assert err is None and rec == bytes([13, 6, 29, 7])
    _, err = r.ReadNext()
    assert errors_is(err, EOF)
    r = opened("v2_compat", "recordio_UncompressedSingleRecord_directio_trailer")
    rec, err = r.ReadNext()
    assert err is None and rec == bytes([13, 6, 29, 7])
    _, err = r.ReadNext()
    assert errors_is(err, MagicNumberMismatchErr)


@pytest.mark.parametrize("vd", LEGACY)
def test_legacy_reader_forbids_closed_and_double_open(vd):  # v2compat :169-188 / v1compat :140-159
    r, _ = NewFileReaderWithPath(fixture_path(vd, "recordio_UncompressedSingleRecord"))
    assert r.Close() is None
    _, err = r.ReadNext()
    assert "was either not opened yet or is closed already" in str(err)
    assert "already closed" in str(r.Open())
    r, _ = NewFileReaderWithPath(fixture_path(vd, "recordio_UncompressedSingleRecord"))
    assert r.Open() is None
    assert "already opened" in str(r.Open())


@pytest.mark.parametrize("vd", LEGACY)
def test_legacy_mmap_single_record_and_offsets(vd):  # mmap_reader_v2compat_test.go:11-35 / v1compat :12-36
    r = mm(vd, "recordio_UncompressedSingleRecord")
    buf, err = r.ReadNextAt(FileHeaderSizeBytes)
    assert err is None and buf == asc(13)
    _, err = r.ReadNextAt(FileHeaderSizeBytes + 1)
    assert str(errors_unwrap(err)) == "magic number mismatch"
    _, err = r.ReadNextAt(42000)
    assert str(errors_unwrap(err)) == "mmap: invalid ReadAt offset 42000"
    assert str(err).startswith("failed reading at offset 42000 in mmap reader")  # mmap_reader.go:211 / :256
    for name, msg in [("recordio_UncompressedSingleRecord_v0", "but was 0"),
                      ("recordio_UncompressedSingleRecord_v256", "but was 256")]:
        r2, _ = NewMemoryMappedReaderWithPath(fixture_path(vd, name))
        assert msg in str(r2.Open())
    if vd == "v2_compat":
        r2, _ = NewMemoryMappedReaderWithPath(fixture_path(vd, "recordio_UncompressedSingleRecord_comp300"))
        assert "unknown compression type [300]" in str(r2.Open())


def test_v2_mmap_small_varint_header_eof():  # mmap_reader_v2compat_test.go:91-104
    r = mm("v2_compat", "recordio_UncompressedSingleRecord")
    b, err = r.ReadNextAt(FileHeaderSizeBytes)
    assert err is None and len(b) == 13
    b2, err = r.ReadNextAt(FileHeaderSizeBytes + 5 + len(b))
    assert b2 is None and err is EOF
    b2, err = r.ReadNextAt(FileHeaderSizeBytes + 4 + len(b))
    assert b2 is None and str(errors_unwrap(err)) == "magic number mismatch"


def test_v1_mmap_short_header_and_seek():
    # readNextAtV1 (mmap_reader.go:205-221): a 20-byte ReadAt past the last record fails wrapping
    # io.EOF; SeekNext on v1: "unsupported on files with version lower than v2" (:62-64)
    r = mm("v1_compat", "recordio_UncompressedSingleRecord")
    b, err = r.ReadNextAt(41)
    assert b is None and errors_is(err, EOF) and str(err).startswith("failed reading at offset 41 in mmap reader")
    b, err = r.ReadNextAt(30)
    assert b is None and errors_is(err, EOF)
    _, _, err = r.SeekNext(0)
    assert str(err) == "unsupported on files with version lower than v2"


def test_v2_mmap_seek_next():
    r = mm("v2_compat", "recordio_UncompressedWriterMultiRecord_asc")
    nxt, rec, err = r.SeekNext(0)
    assert err is None and nxt == FileHeaderSizeBytes and rec == b""
    for n in range(1, 6):
        nxt, rec, err = r.SeekNext(nxt + 1)
        assert err is None and rec == asc(n)
