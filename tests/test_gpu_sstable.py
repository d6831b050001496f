"""SSTable load / validation / full scan on the device vs the oracle (GPU).

NewSSTableReader (sstables/sstable_reader.go:250-345: index via SliceKeyIndexLoader, validateDataFile
unless SkipHashCheckOnLoad) and Scan (SSTableFullScanIterator, sstable_iterator.go:68-111) on tables
the mirror's writer produced (v4 recordio, as sstable_writer.go writes them), compared with the
oracle's restatement; the reference's fixture content (sstable_reader_test.go) is re-encoded as v4,
its recordio v1/v2 originals must be handed back (UnsupportedError)."""
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


def test_reference_fixtures_are_handed_back():
    # recordio v1/v2 data files (and v0 protobuf values): the reference reader keeps them
    for name in ("SimpleWriteHappyPathSSTable", "SimpleWriteHappyPathSSTableRecordIOV2",
                 "SimpleWriteHappyPathSSTableWithCRCHashesMismatch"):
        r, err = S.NewSSTableReader(S.ReadBasePath(os.path.join(GOLDEN, "sstables", name)))
        assert r is None and isinstance(err, S.UnsupportedError), (name, err)


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
def sst_open_host(base):
    import ctypes

    from recordio import _lib as L
    from recordio.device import DeviceDecoder

    lib = L.lib()
    dec = DeviceDecoder(0)
    imgs = [open(os.path.join(base, f), "rb").read() for f in ("index.rio", "data.rio")]
    h = ctypes.c_void_p()
    info = L.SstInfo()
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

    for name in ("SimpleWriteHappyPathSSTable", "SimpleWriteHappyPathSSTableRecordIOV2"):
        rc, info, _ = sst_open_host(os.path.join(GOLDEN, "sstables", name))
        assert rc == L.RIO_ERR_UNSUPPORTED, (name, rc)
    base2 = str(tmp_path / "m")
    write_triples(base2, triples_for([(be(i), be(i)) for i in range(20)]),
                  tamper=lambda i, e, off: b"\x0a\x7fab" if i == 6 else e)
    rc, info, _ = sst_open_host(base2)
    assert rc == 0 and info.first_bad_proto == 6
