"""Oracle (CPU checker) for the SSTable load / validation / scan path, pinned by the reference's own
SSTable fixtures (sstables/test_files, copied data files) and the assertions of
sstables/sstable_reader_test.go. Also checks the mirror's writer output with the oracle."""
import os
import struct

import pytest

import oracle_py as orc
from conftest import GOLDEN, STATUS

from sstables import proto

SST = os.path.join(GOLDEN, "sstables")


def be(i):
    return struct.pack(">I", i)


@pytest.mark.parametrize("name", ["SimpleWriteHappyPathSSTableRecordIOV2", "SimpleWriteHappyPathSSTableWithCRCHashes",
                                  "SimpleWriteHappyPathSSTableWithMetaData"])
def test_fixture_seven_records(name):  # sstable_reader_test.go:28-87: keys 1..7 -> value key+1
    o = orc.sstable_oracle(os.path.join(SST, name))
    assert o["index_status"] == STATUS["EOF"] and o["bad_proto"] is None and o["unplaced"] is None
    assert [e[0] for e in o["entries"]] == [be(i) for i in range(1, 8)]
    assert o["values"] == [be(i + 1) for i in range(1, 8)]
    assert o["first_bad"] is None
    m, err = proto.read_metadata_if_exists(os.path.join(SST, name, "meta.pb.bin"))
    assert err is None and m.numRecords == 7 and m.nullValues == 0
    assert m.minKey == be(1) and m.maxKey == be(7)


def test_fixture_crc_mismatch():  # sstable_reader_test.go:89-96
    o = orc.sstable_oracle(os.path.join(SST, "SimpleWriteHappyPathSSTableWithCRCHashesMismatch"))
    i = o["first_bad"]
    assert i is not None and o["entries"][i][0] == be(4)
    k, vo, cs = o["entries"][i]
    assert vo == 41 and cs == 0x688FFFFF90000000 and o["crcs"][i] == 0x738FFFFF90000000
    assert o["values"][i] == be(0x15)  # the tampered value (:114-117)


def test_fixture_empty_values():  # sstable_reader_test.go:164-183
    o = orc.sstable_oracle(os.path.join(SST, "SimpleWriteHappyPathSSTableWithCRCHashesEmptyValues"))
    assert [e[0] for e in o["entries"]] == [be(0x2A), be(0x2D)]
    assert o["values"] == [be(0), b""] and o["first_bad"] is None  # Get(42) = 0000, Get(45) = []byte{}


def test_fixture_v0_proto_values():  # sstable_reader_test.go:11-26: no metadata -> v0 DataEntry values
    base = os.path.join(SST, "SimpleWriteHappyPathSSTable")
    m, err = proto.read_metadata_if_exists(os.path.join(base, "meta.pb.bin"))
    assert err is None and m.version == 0 and m.numRecords == 0
    o = orc.sstable_oracle(base)
    assert o["v0"] and [e[0] for e in o["entries"]] == [be(i) for i in range(1, 8)]
    # each data record is a DataEntry proto {value = 1: bytes}; the oracle unwraps it
    assert o["values"] == [be(i + 1) for i in range(1, 8)]
    raw = orc.file_reader_decode(open(os.path.join(base, "data.rio"), "rb").read())["records"]
    assert all(r == b"\x0a\x04" + v for r, v in zip(raw, o["values"]))
    assert o["first_bad"] is None and o["unplaced"] is None


def test_data_entry_wire_rules():
    de = orc.data_entry
    assert de(b"") is None                                            # no field 1: value nil
    assert de(b"\x0a\x00") == b""                                     # present and empty
    assert de(b"\x0a\x02ab\x0a\x01c") == b"c"                         # last occurrence wins
    assert de(b"\x08\x05\x0a\x01z") == b"z"                           # field 1 as varint: unknown, skipped
    assert de(b"\x08\x05") is None
    assert de(b"\x12\x01x\x0a\x01y\x25\x00\x00\x00\x00") == b"y"      # unknown bytes / fixed32 skipped
    assert de(b"\x2b\x08\x01\x2c\x0a\x01q") == b"q"                   # group skipped to its end tag
    for bad in (b"\x0a\x05ab", b"\x00", b"\x2c", b"\x0a", b"\x08" + b"\xff" * 9 + b"\x02", b"\x0e"):
        assert isinstance(de(bad), orc.BadProto), bad


def test_crc64_iso_known_answer():
    # Go: crc64.Checksum([]byte("123456789"), crc64.MakeTable(crc64.ISO)) = 0xb90956c775a41001
    assert orc.crc64_iso(b"123456789") == 0xB90956C775A41001


def test_writer_tables_check_out(tmp_path):
    from sstables import write_sstable

    items = [(be(i), None if i % 13 == 0 else bytes([i % 251]) * (i % 40)) for i in range(1, 500)]
    for comp in (0, 2):
        base = str(tmp_path / f"t{comp}")
        meta = write_sstable(base, items, comp)
        o = orc.sstable_oracle(base)
        assert o["index_status"] == STATUS["EOF"] and o["first_bad"] is None and o["unplaced"] is None
        assert [e[0] for e in o["entries"]] == [k for k, _ in items]
        assert o["values"] == [v for _, v in items]
        assert meta.numRecords == len(items) and meta.nullValues == sum(v is None for _, v in items)


def test_index_entry_wire_rules():
    ie = orc.index_entry
    assert ie(b"") == (b"", 0, 0)
    assert ie(b"\x0a\x02ab\x10\x05\x18\x07") == (b"ab", 5, 7)
    assert ie(b"\x10\x05\x10\x09") == (b"", 9, 0)                    # last occurrence wins
    assert ie(b"\x0a\x01a\x0a\x01b") == (b"b", 0, 0)
    assert ie(b"\x25\x00\x00\x00\x00\x10\x03") == (b"", 3, 0)        # unknown fixed32 skipped
    assert ie(b"\x12\x01x\x10\x04") == (b"", 4, 0)                   # field 2 as bytes: unknown, skipped
    assert ie(b"\x2b\x08\x01\x2c\x10\x02") == (b"", 2, 0)            # group 5 skipped to its end tag
    assert ie(b"\x0a\x05ab") is None                                 # truncated bytes
    assert ie(b"\x00") is None                                       # field number 0
    assert ie(b"\x2c") is None                                       # unmatched end group
    assert ie(b"\x10" + b"\xff" * 9 + b"\x02") is None               # varint overflow


@pytest.mark.parametrize("name", ["SimpleWriteHappyPathSSTable", "SimpleWriteHappyPathSSTableRecordIOV2",
                                  "SimpleWriteHappyPathSSTableWithBloom", "SimpleWriteHappyPathSSTableWithMetaData"])
def test_v0_compat_fixtures(name):  # sstable_reader_v0compat_test.go: keys 1..7 -> DataEntry value key+1
    o = orc.sstable_oracle(os.path.join(GOLDEN, "sstables_v0_compat", name))
    assert o["v0"] and o["unplaced"] is None and o["bad_proto"] is None
    assert [e[0] for e in o["entries"]] == [be(i) for i in range(1, 8)]
    assert o["values"] == [be(i + 1) for i in range(1, 8)]
