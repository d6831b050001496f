"""Writes tests/golden/expectations.json: what the reference's own tests assert about each fixture.

The fixture files in v1_compat/ .. v4_compat/ are data files copied from the reference
(recordio/test_files/). The expectations below are transcribed from the reference test suite —
this script is the record of that transcription (not a copy of any reference source):
  file_reader_test.go:13-200, file_reader_v{1,2,3}compat_test.go, mmap_reader_test.go:13-117,244-260,
  mmap_reader_v{1,2,3}compat_test.go, and the generator that made the fixtures
  (file_reader_generator_test.go:37-180: contents, mutations).
Record specs: {"asc": n} = bytes 0..n-1, {"bytes": [...]} literal, null = nil record.
Status names follow include/rio.h.
"""
import json
import os

ASC_255 = [{"asc": i} for i in range(255)]


def common(v):
    # mmap_reader_test.go:93-106 (v3: mmap_reader_v3compat_test.go:91-104): EOF right after the
    # record at 8 + hl + 13; then the magic mismatch read at FileHeaderSizeBytes + (hl - 1) + len(bytes)
    # where `bytes` is the nil returned by that EOF read, i.e. offset 8 + hl - 1 (18 for v4, 13 for v3:
    # the last header byte of the record). 8 + hl - 1 + 13 (inside its payload) is checked as well.
    hl = 11 if v == 4 else 6
    eof_single = 8 + hl + 13
    d = {
        "recordio_UncompressedSingleRecord": {
            "records": [{"asc": 13}], "end": "EOF",
            "read_at": [[8, {"asc": 13}], [9, "MAGIC"], [42000, "INVALID_OFFSET"],
                        [eof_single, "EOF"], [8 + hl - 1, "MAGIC"], [eof_single - 1, "MAGIC"]],
        },
        "recordio_UncompressedWriterMultiRecord_asc": {"records": ASC_255, "end": "EOF"},
        "recordio_SnappyWriterMultiRecord_asc": {"records": ASC_255, "end": "EOF", "compression": 2},
        "recordio_UncompressedSingleRecord_v0": {"open": ["VERSION", 0]},
        "recordio_UncompressedSingleRecord_v256": {"open": ["VERSION", 256]},
        "recordio_UncompressedSingleRecord_comp1": {"compression": 1, "records": [{"asc": 1337}], "end": "EOF"},
        "recordio_UncompressedSingleRecord_comp2": {"compression": 2, "records": [{"asc": 1337}], "end": "EOF"},
        "recordio_UncompressedSingleRecord_comp300": {"open": ["COMPRESSION_TYPE", 300]},
        "recordio_UncompressedSingleRecord_mnm": {"records": [], "end": "MAGIC"},
        "recordio_UncompressedSingleRecord_directio": {"records": [{"bytes": [13, 6, 29, 7]}], "end": "EOF_ZERO_TAIL"},
        "recordio_UncompressedSingleRecord_directio_trailer": {"records": [{"bytes": [13, 6, 29, 7]}], "end": "MAGIC"},
        "recordio_UncompressedNilAndEmptyRecord": {
            "records": [None, {"bytes": []}], "end": "EOF",
            "read_at": [[8, None], [0x13 if v == 4 else 14, {"bytes": []}]],
        },
        "recordio_UncompressedMagicNumberContent": {
            "records": [{"bytes": [0x91, 0x8D, 0x4C]}, {"bytes": [21, 8, 23]}, {"bytes": [0x91, 0x8D, 0x4C]}],
            "end": "EOF", "seek_chain": True,
        },
    }
    if v == 4:
        d["recordio_UncompressedCrcFailure"] = {"records": [], "end": "HEADER_CRC"}
    return d


def legacy(v):
    # file_reader_v{1,2}compat_test.go, mmap_reader_v{1,2}compat_test.go. The _comp1 / _comp2 files
    # are checked there only for the header's compression type ("header_only").
    single = {"records": [{"asc": 13}], "end": "EOF",
              "read_at": [[8, {"asc": 13}], [9, "MAGIC"], [42000, "INVALID_OFFSET"]]}
    if v == 2:
        # mmap_reader_v2compat_test.go:91-104: header 91 8d 4c 0d 0d (5 bytes), EOF after the record,
        # magic mismatch one byte before its end
        single["read_at"] += [[8 + 5 + 13, "EOF"], [8 + 4 + 13, "MAGIC"]]
    d = {
        "recordio_UncompressedSingleRecord": single,
        "recordio_UncompressedWriterMultiRecord_asc": {"records": ASC_255, "end": "EOF"},
        "recordio_SnappyWriterMultiRecord_asc": {"records": ASC_255, "end": "EOF", "compression": 2},
        "recordio_UncompressedSingleRecord_v0": {"open": ["VERSION", 0]},
        "recordio_UncompressedSingleRecord_v256": {"open": ["VERSION", 256]},
        "recordio_UncompressedSingleRecord_comp1": {"compression": 1, "header_only": True},
        "recordio_UncompressedSingleRecord_comp2": {"compression": 2, "header_only": True},
        "recordio_UncompressedSingleRecord_mnm": {"records": [], "end": "MAGIC"},
    }
    if v == 2:
        d["recordio_UncompressedSingleRecord_comp300"] = {"open": ["COMPRESSION_TYPE", 300]}
        d["recordio_UncompressedSingleRecord_directio"] = {"records": [{"bytes": [13, 6, 29, 7]}], "end": "EOF_ZERO_TAIL"}
        d["recordio_UncompressedSingleRecord_directio_trailer"] = {"records": [{"bytes": [13, 6, 29, 7]}], "end": "MAGIC"}
    return d


def main():
    out = {"v4_compat": common(4), "v3_compat": common(3), "v2_compat": legacy(2), "v1_compat": legacy(1),
           "kats": {"crc32c_magic": 0x0967294B, "magic_uvarint": [0x91, 0x8D, 0x4C],
                    "single_record_header_crc": 0xF173A84B,
                    "writer_sizes": {"single_13": 0x20, "seq_5_10_25": [0x18, 0x2D, 0x51],
                                     "seq_127_one_byte": 0x5FC}}}
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "expectations.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", p)


if __name__ == "__main__":
    main()
