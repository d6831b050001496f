"""SSTable load / validation / full scan on the device vs the oracle (GPU).

NewSSTableReader (sstables/sstable_reader.go:250-345: index via SliceKeyIndexLoader, validateDataFile
unless SkipHashCheckOnLoad) and Scan (SSTableFullScanIterator, sstable_iterator.go:68-111) on tables
the mirror's writer produced (v4 recordio, as sstable_writer.go writes them), compared with the
oracle's restatement, and on the reference's own fixtures (recordio v2, sstable_reader_test.go's
expectations), including the v0 fixture whose values are protobuf DataEntry records."""
import os
import random
import struct

import pytest

import oracle_py as orc
from conftest import GOLDEN

import sstables as S
from sstables import proto
from sstables.writer import _Image, crc64_iso

pytestmark = pytest.mark.gpu


def be(i):
    return struct.pack(">I", i)


def write_triples(base, triples, comp=2, tamper=None):
    """Table from (key, value, checksum) triples; tamper(i, entry_bytes) may rewrite index records."""
    os.makedirs(base, exist_ok=True)
    d, ix = _Image(comp), _Image(0)
    m = proto.MetaData(version=1)
    for i, (k, v, cs) in enumerate(triples):
        off = d.write(v)
        e = proto.encode_index_entry(k, off, cs)
        if tamper is not None:
            e = tamper(i, e, off)
        ix.write(e)
        m.numRecords += 1
        m.nullValues += v is None
    m.minKey, m.maxKey = triples[0][0], triples[-1][0]
    db, ib = d.bytes(), ix.bytes()
    m.dataBytes, m.indexBytes, m.totalBytes = len(db), len(ib), len(db) + len(ib)
    for name, b in (("data.rio", db), ("index.rio", ib), ("meta.pb.bin", m.marshal())):
        with open(os.path.join(base, name), "wb") as fh:
            fh.write(b)


def triples_for(items):
    return [(k, v, crc64_iso(v or b"")) for k, v in items]


def scan_all(r):
    it, err = r.Scan()
    assert err is None
    out = []
    while True:
        k, v, err = it.Next()
        if err is S.Done:
            return out, None
        if err is not None:
            return out, err
        out.append((k, v))


def check_against_oracle(base):
    o = orc.sstable_oracle(base)
    r, err = S.NewSSTableReader(S.ReadBasePath(base))
    if o["first_bad"] is not None:
        assert r is None and err is not None
        i = o["first_bad"]
        k, vo, cs = o["entries"][i]
        msg = str(err)
        assert "validateDataFile error loading value" in msg and f"at key [{S._fmt_key(k)}]" in msg, msg
        assert f"offset [{vo}]: Checksum mismatch: expected {cs:x}, got {o['crcs'][i]:x}" in msg, msg
        return o, None
    assert err is None, err
    got, serr = scan_all(r)
    assert serr is None
    assert got == [(e[0], v) for e, v in zip(o["entries"], o["values"])]
    return o, r


def text(rng, n):
    return bytes(rng.choice(b"abcdefghij      ,.") for _ in range(n))


@pytest.mark.parametrize("comp", [0, 2])
def test_scan_matches_oracle(tmp_path, comp):
    rng = random.Random(comp)
    items = [(be(i), text(rng, rng.randint(0, 3000))) for i in range(2000)]
    base = str(tmp_path / "t")
    write_triples(base, triples_for(items), comp)
    o, r = check_against_oracle(base)
    m = r.MetaData()
    assert m.NumRecords == 2000 and m.MinKey == be(0) and m.MaxKey == be(1999)
    v, err = r.Get(be(1234))
    assert err is None and v == items[1234][1]
    assert r.Get(b"nope")[1] is S.NotFound


def test_nil_and_empty_values(tmp_path):
    items = [(be(i), None if i % 3 == 0 else (b"" if i % 3 == 1 else be(i))) for i in range(300)]
    base = str(tmp_path / "t")
    write_triples(base, triples_for(items))
    check_against_oracle(base)


def test_checksum_mismatch_on_load_and_scan(tmp_path):
    # the fixture's content (keys 1..7, value key+1) with the fourth value tampered like
    # SimpleWriteHappyPathSSTableWithCRCHashesMismatch (sstable_reader_test.go:89-162)
    tri = [(be(i), be(i + 1), crc64_iso(be(i + 1))) for i in range(1, 8)]
    tri[3] = (be(4), be(0x15), crc64_iso(be(5)))
    base = str(tmp_path / "t")
    write_triples(base, tri)
    o, _ = check_against_oracle(base)
    assert o["first_bad"] == 3
    r, err = S.NewSSTableReader(S.ReadBasePath(base), S.SkipHashCheckOnLoad(), S.EnableHashCheckOnReads())
    assert err is None
    got, serr = scan_all(r)
    assert [k for k, _ in got] == [be(1), be(2), be(3)]
    assert serr == S.ChecksumError(crc64_iso(be(0x15)), crc64_iso(be(5)))
    v, gerr = r.Get(be(4))
    assert v == be(0x15) and "Checksum mismatch" in str(gerr)


def test_zero_checksum_is_unchecked(tmp_path):
    tri = [(be(i), be(i + 1), 0 if i == 4 else crc64_iso(be(i + 1))) for i in range(1, 8)]
    tri[3] = (be(4), be(0x15), 0)
    base = str(tmp_path / "t")
    write_triples(base, tri)
    o, r = check_against_oracle(base)
    assert o["first_bad"] is None and r is not None


def _fixture(name):
    return os.path.join(GOLDEN, "sstables", name)


SEVEN = [(be(i), be(i + 1)) for i in range(1, 8)]  # TEST_ONLY_NewSkipListMapWithElements (sstable_test.go:245-258)


@pytest.mark.parametrize("name", ["SimpleWriteHappyPathSSTableRecordIOV2", "SimpleWriteHappyPathSSTableWithMetaData",
                                  "SimpleWriteHappyPathSSTableWithCRCHashes"])
def test_reference_fixtures_on_device(name):
    """sstable_reader_test.go:28-87: recordio v2 tables with metadata version 1 load on the device, with
    the tests' metadata, content (assertContentMatchesSkipList), full scan and negative lookups."""
    r, err = S.NewSSTableReader(S.ReadBasePath(_fixture(name)))
    assert err is None, err
    m = r.MetaData()
    assert (m.NumRecords, m.NullValues, m.MinKey, m.MaxKey) == (7, 0, be(1), be(7))
    for k, v in SEVEN:
        assert r.Contains(k) == (True, None)
        assert r.Get(k) == (v, None)
    assert scan_all(r) == (SEVEN, None)
    for k in (b"", b"\x01", b"\x01\x02\x03"):  # assertNegativeContains (:305-324)
        assert r.Contains(k) == (False, None)
        assert r.Get(k)[1] is S.NotFound
    assert r.t.index_info["version"] == 2 and r.t.data_info["version"] == 2
    o, _ = check_against_oracle(_fixture(name))
    assert o["first_bad"] is None


def test_reference_fixture_empty_values():
    # sstable_reader_test.go:164-183
    r, err = S.NewSSTableReader(S.ReadBasePath(_fixture("SimpleWriteHappyPathSSTableWithCRCHashesEmptyValues")))
    assert err is None, err
    m = r.MetaData()
    assert (m.NumRecords, m.NullValues, m.MinKey, m.MaxKey) == (2, 0, be(0x2A), be(0x2D))
    assert r.Get(be(45)) == (b"", None)
    assert r.Get(be(42)) == (be(0), None)


def test_reference_fixture_checksum_mismatch():
    # sstable_reader_test.go:89-162
    base = _fixture("SimpleWriteHappyPathSSTableWithCRCHashesMismatch")
    r, err = S.NewSSTableReader(S.ReadBasePath(base))
    assert r is None
    assert "offset [41]: Checksum mismatch: expected 688fffff90000000, got 738fffff90000000" in str(err)
    assert "at key [[0 0 0 4]]" in str(err)
    r, err = S.NewSSTableReader(S.ReadBasePath(base), S.SkipHashCheckOnLoad(), S.EnableHashCheckOnReads())
    assert err is None
    m = r.MetaData()
    assert (m.NumRecords, m.NullValues, m.MinKey, m.MaxKey) == (7, 0, be(1), be(7))
    for i in range(1, 8):
        v, gerr = r.Get(be(i))
        if i == 4:
            assert v == be(0x15)
            assert "offset [41]: Checksum mismatch: expected 688fffff90000000, got 738fffff90000000" in str(gerr)
        else:
            assert (v, gerr) == (be(i + 1), None)
    got, serr = scan_all(r)
    assert got == SEVEN[:3]
    assert serr == S.ChecksumError(0x738FFFFF90000000, 0x688FFFFF90000000)


def test_reference_v0_fixture_on_device():
    """sstable_reader_test.go:11-26, 185-193: SimpleWriteHappyPathSSTable (recordio v1 files, no
    meta.pb.bin: metadata version 0, every value a protobuf DataEntry) loads on the device."""
    r, err = S.NewSSTableReader(S.ReadBasePath(_fixture("SimpleWriteHappyPathSSTable")))
    assert err is None, err
    m = r.MetaData()
    assert (m.NumRecords, m.NullValues, len(m.MinKey), len(m.MaxKey), m.version) == (0, 0, 0, 0, 0)
    for k, v in SEVEN:
        assert r.Contains(k) == (True, None)
        assert r.Get(k) == (v, None)
    assert scan_all(r) == (SEVEN, None)  # V0SSTableFullScanIterator (sstable_iterator.go:34-66)
    for k in (b"", b"\x01", b"\x01\x02\x03"):
        assert r.Contains(k) == (False, None)
        assert r.Get(k)[1] is S.NotFound
    assert r.t.v0 and r.t.index_info["version"] == 1 and r.t.data_info["version"] == 1
    check_against_oracle(_fixture("SimpleWriteHappyPathSSTable"))


def data_entry(v):
    """DataEntry {value = 1} as protobuf-go marshals it (the field is omitted for nil / empty)."""
    return b"" if not v else b"\x0a" + proto_uvarint(len(v)) + v


def proto_uvarint(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def write_v0_table(base, values, comp=2, keys=None):
    """A v0 table (no meta.pb.bin): index entries without checksums, data records given raw (the
    DataEntry bytes, or anything else for malformed ones)."""
    os.makedirs(base, exist_ok=True)
    d, ix = _Image(comp), _Image(0)
    keys = keys or [be(i) for i in range(len(values))]
    for k, raw in zip(keys, values):
        ix.write(proto.encode_index_entry(k, d.write(raw), 0))
    for name, b in (("data.rio", d.bytes()), ("index.rio", ix.bytes())):
        with open(os.path.join(base, name), "wb") as fh:
            fh.write(b)


@pytest.mark.parametrize("comp", [0, 2])
def test_v0_table_matches_oracle(tmp_path, comp):
    rng = random.Random(50 + comp)
    raws = []
    for i in range(1200):
        v = text(rng, rng.randint(0, 900))
        k = rng.random()
        if k < 0.05:
            raws.append(b"")                                           # value nil (field absent)
        elif k < 0.1:
            raws.append(b"\x0a\x00")                                   # present, empty
        elif k < 0.15:
            raws.append(b"\x12\x03abc" + data_entry(v) + b"\x18\x07")  # unknown fields around it
        elif k < 0.2:
            raws.append(data_entry(b"old") + data_entry(v))            # last occurrence wins
        else:
            raws.append(data_entry(v))
    base = str(tmp_path / "t")
    write_v0_table(base, raws, comp)
    o, r = check_against_oracle(base)
    assert o["v0"]
    for i in range(0, 1200, 7):
        assert r.Get(be(i)) == (o["values"][i], None)


def test_v0_malformed_value(tmp_path):
    raws = [data_entry(be(i + 1)) for i in range(20)]
    raws[7] = b"\x0a\x09abc"  # truncated bytes field
    base = str(tmp_path / "t")
    write_v0_table(base, raws)
    o = orc.sstable_oracle(base)
    assert isinstance(o["values"][7], orc.BadProto) and o["first_bad"] is None
    r, err = S.NewSSTableReader(S.ReadBasePath(base))  # validateDataFile skips v0 tables (:205-209)
    assert err is None
    v, gerr = r.Get(be(7))
    assert v is None and str(gerr).endswith("proto: cannot parse invalid wire-format data")
    assert f"while getting value at offset {o['entries'][7][1]}" in str(gerr)
    assert r.Get(be(8)) == (be(9), None)
    got, serr = scan_all(r)
    assert got == [(be(i), be(i + 1)) for i in range(7)] and str(serr) == "proto: cannot parse invalid wire-format data"
    # the host handle with RIO_SST_V0_VALUES
    rc, info, ents = sst_open_host(base, v0=True)
    from recordio import _lib as L

    assert rc == 0 and info.first_bad_value == 7 and info.n_entries == 20
    assert [e[0] for e in ents] == [0] * 7 + [L.RIO_ERR_PROTO] + [0] * 12
    assert [e[2] for e in ents[:7] + ents[8:]] == [be(i + 1) for i in range(20) if i != 7]


def test_index_out_of_layout_is_handed_back(tmp_path):
    items = [(be(i), be(i + 1)) for i in range(50)]
    tri = triples_for(items)
    base = str(tmp_path / "t")
    # entry 10 points at record 11's value: validation (by offset) and scan (by position) disagree
    offs = {}

    def tamper(i, e, off):
        offs[i] = off
        return e

    write_triples(base, tri, tamper=tamper)
    write_triples(base, tri, tamper=lambda i, e, off: proto.encode_index_entry(tri[i][0], offs[11], tri[i][2])
                  if i == 10 else e)
    o = orc.sstable_oracle(base)
    assert o["unplaced"] == 10
    r, err = S.NewSSTableReader(S.ReadBasePath(base), S.SkipHashCheckOnLoad())
    assert r is None and isinstance(err, S.UnsupportedError)


def test_malformed_index_entry(tmp_path):
    tri = triples_for([(be(i), be(i)) for i in range(20)])
    base = str(tmp_path / "t")
    write_triples(base, tri, tamper=lambda i, e, off: b"\x0a\x7fab" if i == 6 else e)
    o = orc.sstable_oracle(base)
    assert o["bad_proto"] == 6
    r, err = S.NewSSTableReader(S.ReadBasePath(base))
    assert r is None and "error while reading index of sstable" in str(err) and "record 6" in str(err)


def test_large_table_sha1_keys(tmp_path):
    # the benchmark's shape (benchmark/sstable_read_test.go:134-158), scaled down: SHA1 keys, one
    # random 1 KiB value repeated, sorted
    import hashlib

    val = bytes(random.Random(3).getrandbits(8) for _ in range(1024))
    keys = sorted(hashlib.sha1(struct.pack(">I", i)).digest() for i in range(20000))
    base = str(tmp_path / "t")
    S.write_sstable(base, [(k, val) for k in keys])
    check_against_oracle(base)


# ---- the host-memory handle (rio_sst_open / rio_sst_entry): what the cgo NewSSTableReader binds ----
def sst_open_host(base, v0=False):
    import ctypes

    from recordio import _lib as L
    from recordio.device import DeviceDecoder

    lib = L.lib()
    dec = DeviceDecoder(0)
    imgs = [open(os.path.join(base, f), "rb").read() for f in ("index.rio", "data.rio")]
    h = ctypes.c_void_p()
    info = L.SstInfo()
    if v0:
        rc = lib.rio_sst_open_ex(dec.ctx, imgs[0], len(imgs[0]), imgs[1], len(imgs[1]), L.RIO_SST_V0_VALUES,
                                 ctypes.byref(h), ctypes.byref(info))
    else:
        rc = lib.rio_sst_open(dec.ctx, imgs[0], len(imgs[0]), imgs[1], len(imgs[1]), ctypes.byref(h), ctypes.byref(info))
    if rc:
        return rc, info, None
    ents = []
    try:
        for i in range(info.n_entries):
            k, v = ctypes.c_void_p(), ctypes.c_void_p()
            kl, vl, vo, cs, crc = (ctypes.c_uint64() for _ in range(5))
            nil = ctypes.c_int()
            st = lib.rio_sst_entry(h, i, ctypes.byref(k), ctypes.byref(kl), ctypes.byref(v), ctypes.byref(vl),
                                   ctypes.byref(nil), ctypes.byref(vo), ctypes.byref(cs), ctypes.byref(crc))
            key = ctypes.string_at(k, kl.value) if kl.value else b""
            val = None if (st or nil.value) else (ctypes.string_at(v, vl.value) if vl.value else b"")
            ents.append((st, key, val, vo.value, cs.value, crc.value))
        assert lib.rio_sst_entry(h, info.n_entries, None, None, None, None, None, None, None, None) == L.RIO_ERR_ARG
    finally:
        lib.rio_sst_free(h)
    return rc, info, ents


@pytest.mark.parametrize("comp", [0, 2])
def test_host_handle_matches_oracle(tmp_path, comp):
    rng = random.Random(10 + comp)
    items = [(be(i), None if i % 97 == 0 else text(rng, rng.randint(0, 2000))) for i in range(1500)]
    base = str(tmp_path / "t")
    write_triples(base, triples_for(items), comp)
    o = orc.sstable_oracle(base)
    rc, info, ents = sst_open_host(base)
    assert rc == 0 and info.n_entries == 1500
    none = (1 << 64) - 1
    assert (info.first_bad_proto, info.first_bad_crc, info.first_unplaced) == (none, none, none)
    for i, (st, k, v, vo, cs, crc) in enumerate(ents):
        e = o["entries"][i]
        assert st == 0 and (k, vo, cs) == tuple(e) and crc == o["crcs"][i] and v == o["values"][i]


def test_host_handle_mismatch_and_handback(tmp_path):
    tri = [(be(i), be(i + 1), crc64_iso(be(i + 1))) for i in range(1, 8)]
    tri[3] = (be(4), be(0x15), crc64_iso(be(5)))
    base = str(tmp_path / "t")
    write_triples(base, tri)
    rc, info, ents = sst_open_host(base)
    assert rc == 0 and info.first_bad_crc == 3 and ents[3][5] == crc64_iso(be(0x15))
    from recordio import _lib as L

    # the reference's v2 fixture through the host handle: the seven entries, their CRCs match
    rc, info, ents = sst_open_host(_fixture("SimpleWriteHappyPathSSTableRecordIOV2"))
    assert rc == 0 and info.n_entries == 7 and info.first_bad_crc == (1 << 64) - 1
    assert [(e[1], e[2]) for e in ents] == SEVEN and all(e[5] == e[4] for e in ents)
    rc, info, ents = sst_open_host(_fixture("SimpleWriteHappyPathSSTable"), v0=True)
    assert rc == 0 and info.n_entries == 7 and info.first_bad_value == (1 << 64) - 1
    assert [(e[1], e[2]) for e in ents] == SEVEN and all(e[0] == 0 and e[4] == 0 for e in ents)
    base2 = str(tmp_path / "m")
    write_triples(base2, triples_for([(be(i), be(i)) for i in range(20)]),
                  tamper=lambda i, e, off: b"\x0a\x7fab" if i == 6 else e)
    rc, info, _ = sst_open_host(base2)
    assert rc == 0 and info.first_bad_proto == 6


def test_full_size_c5_table_exact():
    """One whole C5 table (BASELINE configs[4]: 1.25M SHA1 keys x 1 KiB values, table 0 exactly as
    bench.py builds it) through the device calls bench.py times: decode of index.rio and data.rio,
    rio_sst_index_parse, rio_sst_validate. Decoded arenas equal the oracle's byte for byte; every
    parsed key / valueOffset / checksum equals what the writer put in; every CRC-64 equals the oracle's;
    the oracle's own scan (orc_sst_scan) accepts the same table."""
    import ctypes

    import numpy as np
    import torch

    import bench
    from gpu_util import assert_same_as_oracle, decoder
    from recordio import _lib as L
    from recordio.device import header_codec, to_device_file

    n = bench.CONFIGS["c5"][0]
    index_img, data_img = bench.sstable_images(n, 0)
    dec = decoder()
    lib = L.lib()
    host = {}
    for name, img in (("index", index_img), ("data", data_img)):
        d, ln = to_device_file(img)
        b, info = dec.decode(d, ln, comp=header_codec(img))
        assert info["status"] == 1 and info["n_records"] == n, (name, info)
        k, nb = info["n_records"], info["total_out_bytes"]
        g = dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:k + 1].cpu().numpy(),
                 rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), f"c5 {name}.rio")
        host[name] = (b, g)
    ib, gi = host["index"]
    db, gd = host["data"]
    i64 = dict(dtype=torch.int64, device="cuda:0")
    ko, kl, vo, cs, crc = (torch.empty(n, **i64) for _ in range(5))
    pres, vres = torch.empty(2, **i64), torch.empty(2, **i64)
    assert lib.rio_sst_index_parse(dec.ctx, ib.out.data_ptr(), ib.out_off.data_ptr(), n, ko.data_ptr(), kl.data_ptr(),
                                   vo.data_ptr(), cs.data_ptr(), pres.data_ptr(), None) == 0
    assert lib.rio_sst_validate(dec.ctx, db.out.data_ptr(), db.out_off.data_ptr(), db.rec_off.data_ptr(), n,
                                vo.data_ptr(), cs.data_ptr(), n, crc.data_ptr(), vres.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert pres[0].item() == -1 and vres.tolist() == [-1, -1]
    # what the writer put in (bench.sstable_images): sorted SHA1 keys, value i at data record i
    import hashlib
    import struct

    keys = np.frombuffer(b"".join(sorted(hashlib.sha1(struct.pack(">I", i)).digest() for i in range(n))),
                         np.uint8).reshape(n, 20)
    kl_h, ko_h = kl.cpu().numpy(), ko.cpu().numpy()
    assert np.all(kl_h == 20)
    got_keys = gi["out"][ko_h[:, None] + np.arange(20)[None, :]]
    np.testing.assert_array_equal(got_keys, keys)
    np.testing.assert_array_equal(vo.cpu().numpy(), gd["rec_off"])
    value = gd["out"][gd["out_off"][0]:gd["out_off"][1]].tobytes()
    want_cs = orc.crc64_iso(value)
    assert np.all(cs.cpu().numpy().astype(np.uint64) == np.uint64(want_cs))
    assert np.all(crc.cpu().numpy().astype(np.uint64) == np.uint64(want_cs))
    # the oracle's parse of a sample of index records, and its whole-table scan
    for i in range(0, n, 9973):
        a, b2 = int(gi["out_off"][i]), int(gi["out_off"][i + 1])
        k, v_off, c = orc.index_entry(gi["out"][a:b2].tobytes())
        assert (k, v_off, c) == (keys[i].tobytes(), int(gd["rec_off"][i]), want_cs), i
    bad = ctypes.c_uint64()
    assert orc.lib().orc_sst_scan(index_img.ctypes.data, len(index_img), data_img.ctypes.data, len(data_img),
                                  ctypes.byref(bad)) == n


def _table_with_index(base, items, index_img):
    """data.rio as the writer makes it for `items`, index.rio replaced by `index_img`."""
    write_triples(base, triples_for(items))
    with open(os.path.join(base, "index.rio"), "wb") as fh:
        fh.write(index_img)


@pytest.mark.parametrize("flag", ["corrupt", "eof"])
def test_flagged_index_record_comes_before_a_later_index_error(tmp_path, flag):
    """Load's ReadNext loop over index.rio (slice_key_index.go:117-126) stops at the first record that
    does not decompress: ErrCorrupt fails the load there, gzip's bare io.EOF ends the index with the
    entries before it. A later index error (a torn header at the end) is never reached."""
    import corpus
    from recordio import _lib as L

    items = [(be(i), be(i + 7)) for i in range(12)]
    base = str(tmp_path / "t")
    write_triples(base, triples_for(items))
    ents = [proto.encode_index_entry(k, off, cs) for k, off, cs in
            zip([k for k, _ in items], orc.file_reader_decode(open(os.path.join(base, "data.rio"), "rb").read())["rec_off"],
                [crc64_iso(v) for _, v in items])]
    if flag == "corrupt":
        recs = [(len(e), corpus.gzip_member(e)) for e in ents]
        recs[4] = (len(ents[4]), recs[4][1][:-8] + bytes([recs[4][1][-8] ^ 1]) + recs[4][1][-7:])  # bad CRC-32
    else:
        recs = [(len(e), corpus.gzip_member(e)) for e in ents]
        recs[4] = (len(ents[4]), b"")  # empty payload: gzip.NewReader's bare io.EOF
    index_img = corpus.gz_file(recs) + b"\x91\x8d"  # then a torn header: io.ErrUnexpectedEOF
    _table_with_index(base, items, index_img)
    rc, info, ents_got = sst_open_host(base)
    assert rc == 0 and info.n_entries == 4
    none = (1 << 64) - 1
    assert info.index_bad == (4 if flag == "corrupt" else none)
    r, err = S.NewSSTableReader(S.ReadBasePath(base))
    if flag == "corrupt":
        assert r is None and "error while reading index records" in str(err), str(err)
    else:
        assert err is None
        got, serr = scan_all(r)
        assert serr is None and got == items[:4]


V0C = os.path.join(GOLDEN, "sstables_v0_compat")


@pytest.mark.parametrize("name,meta", [("SimpleWriteHappyPathSSTable", (0, b"", b"")),
                                       ("SimpleWriteHappyPathSSTableRecordIOV2", (7, be(1), be(7))),
                                       ("SimpleWriteHappyPathSSTableWithBloom", (0, b"", b"")),
                                       ("SimpleWriteHappyPathSSTableWithMetaData", (7, be(1), be(7)))])
def test_v0_compat_fixtures_on_device(name, meta):
    """sstable_reader_v0compat_test.go:9-91: metadata version 0 tables (DataEntry values, recordio v1 /
    v2, snappy) with their metadata, content, negative lookups and full scan."""
    r, err = S.NewSSTableReader(S.ReadBasePath(os.path.join(V0C, name)))
    assert err is None, err
    m = r.MetaData()
    assert (m.NumRecords, m.MinKey, m.MaxKey, m.version) == meta + (0,)
    for k, v in SEVEN:
        assert r.Contains(k) == (True, None) and r.Get(k) == (v, None)
    for k in (b"", b"\x01", b"\x01\x02\x03"):
        assert r.Contains(k) == (False, None) and r.Get(k)[1] is S.NotFound
    assert scan_all(r) == (SEVEN, None)
    check_against_oracle(os.path.join(V0C, name))


def drain(it):
    out = []
    while True:
        k, v, err = it.Next()
        if err is S.Done:
            return out
        assert err is None
        out.append((k, v))


def test_v0_compat_scan_starting_at_and_range():  # sstable_reader_v0compat_test.go:99-160
    r, err = S.NewSSTableReader(S.ReadBasePath(os.path.join(V0C, "SimpleWriteHappyPathSSTableWithMetaData")))
    assert err is None
    it, err = r.ScanStartingAt(be(0))
    assert err is None and drain(it) == SEVEN
    for i in range(7):
        it, _ = r.ScanStartingAt(SEVEN[i][0])
        assert drain(it) == SEVEN[i:]
    it, _ = r.ScanStartingAt(be(10))
    assert it.Next() == (None, None, S.Done)
    it, err = r.ScanRange(be(0), be(10))
    assert err is None and drain(it) == SEVEN
    it, _ = r.ScanRange(be(1), be(7))
    assert drain(it) == SEVEN
    it, _ = r.ScanRange(be(4), be(4))
    assert drain(it) == [SEVEN[3]]
    _, err = r.ScanRange(be(1), be(0))
    assert err is not None
    for i in range(7):
        it, _ = r.ScanRange(SEVEN[i][0], be(10))
        assert drain(it) == SEVEN[i:]
        it, _ = r.ScanRange(be(0), SEVEN[i][0])
        assert drain(it) == SEVEN[:i + 1]
    for i in range(7):  # end crossing to the left
        it, err = r.ScanRange(SEVEN[i][0], SEVEN[6 - i][0])
        if i <= 3:
            assert err is None and drain(it) == SEVEN[i:7 - i]
        else:
            assert err is not None
    it, err = r.ScanRange(be(10), be(100))
    assert err is None and it.Next() == (None, None, S.Done)
