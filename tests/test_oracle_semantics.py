"""Oracle behaviour on crafted edge cases, each pinned to the reference code path it follows (CPU).

These are not fixture-backed (the reference ships no such files); the expected class is read off
the reference source cited per case. The GPU suite then checks the device path equals the oracle.
"""
import pytest

import corpus
import oracle_py as orc
from conftest import STATUS

CASES = dict(corpus.cases())

EXPECT = {
    # file_reader.go:76-91: magic mismatch, remainder after the consumed magic varint all zero => EOF
    "mixed_c0_zero_tail": "EOF_ZERO_TAIL",
    "mixed_c2_zero_tail": "EOF_ZERO_TAIL",
    "v3_zero_tail": "EOF_ZERO_TAIL",
    # ... any non-zero byte => MagicNumberMismatchErr
    "mixed_c0_garbage_tail": "MAGIC",
    # a 1-byte tail 0x07 decodes as magic 7 (mismatch) and leaves an empty remainder => EOF
    "mixed_c0_one_byte_tail": "EOF_ZERO_TAIL",
    # "91 8d" then EOF: binary.ReadUvarint partial => io.ErrUnexpectedEOF
    "mixed_c0_partial_magic_tail": "UNEXPECTED_EOF",
    # checksum_byte_reader.go:25-27: 37th header byte
    "header_too_long": "HEADER_TOO_LONG",
    "header_36_exact": "EOF",
    # binary.ReadUvarint overflow (10 continuation bytes)
    "magic_overflow": "VARINT_OVERFLOW",
    "size_overflow": "VARINT_OVERFLOW",
    # snappy decode.go ErrCorrupt for one record: ReadNext returns it and goes on (file_reader.go:
    # 113-122), so the loop ends at the file's end
    "snappy_corrupt_mid": "EOF",
    "snappy_huge_preamble": "EOF",
    "snappy_empty_payload": "EOF",
    "snappy_bad_preamble_mid": "EOF",
    "snappy_short_mid": "EOF",
    "snappy_long_mid": "EOF",
    "snappy_empty_mid": "EOF",
    # io.ReadFull with a partial payload => io.ErrUnexpectedEOF (the reference would first try
    # to allocate 1 TiB in bufferPool.Get: documented divergence)
    "huge_u": "UNEXPECTED_EOF",
    # ReadUvarint accepts non-canonical encodings; the CRC covers the bytes as written
    "noncanonical_magic": "EOF",
    "nil_snappy": "EOF",
    "mixed_c0_embedded": "EOF",
    "mixed_c0_flip": "HEADER_CRC",
    "mixed_c2_flip": "HEADER_CRC",
}


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_edge_case_status(name):
    res = orc.file_reader_decode(CASES[name])
    assert res["status"] == STATUS[EXPECT[name]], (name, res["status"])


def test_every_case_decodes_without_crash():
    for name, img in CASES.items():
        res = orc.file_reader_decode_arrays(img)
        assert res["status"] >= 0, name


# name -> (indices of records that do not decompress, bytes reserved for each)
BAD = {
    "snappy_corrupt_mid": ([25], 160),
    "snappy_huge_preamble": ([3], 0),      # 5000 > 22 x 2 + 64: no stream this long reaches it
    "snappy_empty_payload": ([3], 0),      # decodedLen of an empty src: ErrCorrupt
    "snappy_bad_preamble_mid": ([30, 63], 0),
    "snappy_short_mid": ([30, 63], 170),   # 160 bytes produced, 170 announced
    "snappy_long_mid": ([30, 63], 100),    # the literal overruns the announced 100
    "snappy_empty_mid": ([30, 63], 0),
}


@pytest.mark.parametrize("name", sorted(BAD))
def test_codec_failure_is_per_record(name):
    """A record whose payload does not decompress is delivered flagged (RIO_FLAG_CORRUPT) with the
    reserved output length; the records after it decode as if it were not there."""
    res = orc.file_reader_decode(CASES[name])
    want, rsv = BAD[name]
    bad = [i for i, r in enumerate(res["records"]) if isinstance(r, orc.BadRecord)]
    assert bad == want, (name, bad)
    assert all(res["records"][i] == orc.BadRecord("corrupt") for i in bad)
    assert (res["first_bad"], res["n_bad"]) == (want[0], len(want))
    a = orc.file_reader_decode_arrays(CASES[name])
    for i in want:
        assert a["flags"][i] == 2 and a["out_off"][i + 1] - a["out_off"][i] == rsv, (name, i)
    if name.endswith("_mid") and name != "snappy_corrupt_mid":
        assert res["records"][31:63] == [bytes(j & 0xFF for j in range(60 + k)) for k in range(30)] + [None, b""]


def test_clean_files_have_no_bad_records():
    for name in ("asc_snappy", "nil_snappy", "mixed_c2_zero_tail"):
        res = orc.file_reader_decode(CASES[name])
        assert (res["first_bad"], res["n_bad"]) == (orc.NONE, 0), name


def test_noncanonical_record_delivered():
    res = orc.file_reader_decode(CASES["noncanonical_magic"])
    assert b"hello-noncanonical" in res["records"]


def test_truncation_classes():
    """A cut exactly at a payload start is io.EOF (io.ReadFull read 0 bytes, file_reader.go:104-107);
    inside a payload it is ErrUnexpectedEOF; at a record boundary it is a clean EOF."""
    img = corpus.encode_file([b"a" * 50, b"b" * 50], 0)
    h = len(corpus.header_v4(50, 0))
    first_end = 8 + h + 50
    assert orc.file_reader_decode(img[:first_end])["status"] == STATUS["EOF"]
    assert orc.file_reader_decode(img[:first_end + h])["status"] == STATUS["EOF_PAYLOAD"]
    assert orc.file_reader_decode(img[:first_end + h + 10])["status"] == STATUS["UNEXPECTED_EOF"]
    assert orc.file_reader_decode(img[:first_end + 4])["status"] == STATUS["EOF_HEADER"]  # after nil byte
    assert orc.file_reader_decode(img[:first_end + 5])["status"] == STATUS["EOF_HEADER"]  # after u
    assert orc.file_reader_decode(img[:first_end + 2])["status"] == STATUS["UNEXPECTED_EOF"]  # inside magic
