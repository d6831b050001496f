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
    # snappy decode.go ErrCorrupt
    "snappy_corrupt_mid": "DECOMPRESS",
    "snappy_huge_preamble": "DECOMPRESS",
    "snappy_empty_payload": "DECOMPRESS",
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
