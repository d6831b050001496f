"""DiskKeyIndex lookups on the device (GPU) vs the oracle's binarySearch restatement.

rio_index_search / rio_device_index_search run sstables/disk_key_index.go:87-127 per query lane;
every hit (status, offset, found, valueOffset, checksum) must equal the oracle's on the same index
and key, on well-formed and adversarial indexes: fake record headers inside keys (SeekNext trial
candidates), the scan's skip rule (a 0x91 byte right before a header), nil records, a truncated
tail, a malformed IndexEntry, long last records (io.EOF probes), several seekLen values. The
mirror's DiskKeyIndex API is checked with sstables/sstable_index_test.go's expectations."""
import ctypes
import random
import struct

import numpy as np
import pytest

import oracle_py as orc
from recordio import _lib as L
from recordio import encode_file
from sstables import DiskIndexLoader, IndexVal
from sstables.disk_index import Done, NotFound
from sstables.proto import encode_index_entry
from corpus import header_v4

pytestmark = pytest.mark.gpu
be = lambda i: struct.pack(">I", i)  # noqa: E731


def index_image(entries, comp=0):
    return encode_file(entries, comp)


def entries_for(keys, nil_every=0):
    out = []
    for i, k in enumerate(keys):
        out.append(None if nil_every and i % nil_every == 3 else encode_index_entry(k, 8 + 17 * i, 7 * i))
    return out


def device_hits(idx_bytes, queries, seek_len=0):
    import torch

    from recordio.device import to_device_file

    d, n = to_device_file(idx_bytes, 0)
    off = np.zeros(len(queries) + 1, dtype=np.uint64)
    np.cumsum([len(q) for q in queries], out=off[1:])
    blob = np.frombuffer(b"".join(queries) + b"\0", dtype=np.uint8)
    dk = torch.from_numpy(blob.copy()).cuda()
    doff = torch.from_numpy(off.view(np.int64).copy()).cuda()
    hits = torch.empty(len(queries) * ctypes.sizeof(L.IndexHit), dtype=torch.uint8, device="cuda")
    rc = L.lib().rio_device_index_search(L.default_ctx(0), d.data_ptr(), n, seek_len, dk.data_ptr(), doff.data_ptr(),
                                         len(queries), hits.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    raw = hits.cpu().numpy().tobytes()
    arr = (L.IndexHit * len(queries)).from_buffer_copy(raw)
    return [(h.status, h.offset, bool(h.found), h.value_offset, h.checksum) for h in arr]


def check(idx_bytes, queries, seek_len=0):
    got = device_hits(idx_bytes, queries, seek_len)
    for q, g in zip(queries, got):
        o = orc.disk_index_search(idx_bytes, q, seek_len or 4096)
        if o[0] != 0:  # errors carry no offset / entry
            assert g[0] == o[0], (q, g, o)
        else:
            assert g == o, (q, g, o)
    return got


def queries_for(keys, rng, extra=200):
    qs = list(keys) + [b"", b"\x00", b"\xff" * 40]
    for _ in range(extra):
        k = rng.choice(keys) if keys else b"x"
        qs.append(k[:rng.randint(0, len(k))])  # prefixes
        qs.append(bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 24))))
    return qs


@pytest.mark.parametrize("seed", [1, 2])
def test_random_indexes_match_oracle(seed):
    rng = random.Random(seed)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 40))) for _ in range(2000)})
    idx = index_image(entries_for(keys))
    got = check(idx, queries_for(keys, rng))
    assert sum(g[2] for g in got[:len(keys)]) > len(keys) // 2


def test_long_last_records_match_oracle():
    rng = random.Random(3)
    for last in (50, 300, 2000):
        keys = [b"a" * 5 + be(i) for i in range(50)] + [b"b" * last]
        check(index_image(entries_for(keys)), queries_for(keys, rng, 20))


def test_adversarial_payloads_match_oracle():
    rng = random.Random(4)
    fake = header_v4(3, 0) + b"abc"  # a CRC-valid record header inside a key: a SeekNext candidate
    keys = []
    for i in range(400):
        k = be(i)
        r = i % 5
        if r == 1:
            k += fake
        elif r == 2:
            k += b"\x91"  # entry's last byte 0x91 right before the next header: the skip rule
        elif r == 3:
            k += b"\x91\x8d"
        elif r == 4:
            k += b"\x91\x8d\x4c\x00"
        keys.append(k)
    ents = [encode_index_entry(k, 0, 0) for k in keys]  # key-only entries end with the key's last byte
    for nil_every in (0, 9):
        e = [None if nil_every and i % nil_every == 3 else x for i, x in enumerate(ents)]
        check(index_image(e), queries_for(keys, rng, 100))


@pytest.mark.parametrize("seek_len", [1, 2, 3, 7, 64, 4096])
def test_seek_len_matches_oracle(seek_len):
    rng = random.Random(seek_len)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 12))) for _ in range(300)})
    check(index_image(entries_for(keys)), queries_for(keys, rng, 50), seek_len)


def test_damaged_indexes_match_oracle():
    rng = random.Random(5)
    keys = [be(i) for i in range(300)]
    img = bytearray(index_image(entries_for(keys)))
    check(bytes(img[:-5]), queries_for(keys, rng, 50))  # truncated last record
    bad = index_image(entries_for(keys[:150]) + [b"\x0a\x7fab"] + entries_for(keys[151:]))
    got = check(bad, queries_for(keys, rng, 50))
    assert any(g[0] == L.RIO_ERR_PROTO for g in got)


def test_compressed_index_is_handed_back():
    idx = index_image(entries_for([be(i) for i in range(10)]), comp=2)
    assert all(g[0] == L.RIO_ERR_UNSUPPORTED for g in device_hits(idx, [be(3), b""]))


def test_reference_index_api(tmp_path):
    # sstable_index_test.go:34-223 on the SimpleWriteHappyPathSSTableWithMetaData content (keys 1..7)
    p = tmp_path / "index.rio"
    p.write_bytes(index_image(entries_for([be(i) for i in range(1, 8)])))
    idx, err = DiskIndexLoader().Load(str(p), None)
    assert err is None and idx.Open() is None
    try:
        for absent in (b"", b"\x01", b"\x01\x02\x03"):
            assert idx.Contains(absent) == (False, None)
            assert idx.Get(absent) == (IndexVal(), NotFound)
        for i in range(1, 8):
            assert idx.Contains(be(i)) == (True, None)
            v, err = idx.Get(be(i))
            assert err is None and v == IndexVal(8 + 17 * (i - 1), 7 * (i - 1))

        def drain(it):
            out = []
            while True:
                k, v, err = it.Next()
                if err is Done:
                    return out
                assert err is None
                out.append(struct.unpack(">I", k)[0])

        exp = list(range(1, 8))
        assert drain(idx.Iterator()[0]) == exp
        assert drain(idx.IteratorStartingAt(be(0))[0]) == exp
        for i, s in enumerate(exp):
            assert drain(idx.IteratorStartingAt(be(s))[0]) == exp[i:]
        assert drain(idx.IteratorStartingAt(be(10))[0]) == []
        assert drain(idx.IteratorBetween(be(0), be(10))[0]) == exp
        assert drain(idx.IteratorBetween(be(4), be(4))[0]) == [4]
        assert idx.IteratorBetween(be(1), be(0))[1] is not None
        assert drain(idx.IteratorBetween(be(10), be(100))[0]) == []
        batch = idx.GetBatch([be(i) for i in range(0, 9)])
        assert [e is None for _, e in batch] == [False] + [True] * 7 + [False]
    finally:
        idx.Close()


def test_large_batch_sorted_path_matches_oracle():
    # >= 4096 keys: the device visits the queries in key-prefix order (rio_sort.hip); every hit must
    # still land at its own query index, including keys with equal 8-byte prefixes
    rng = random.Random(11)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 24))) for _ in range(3000)})
    idx = index_image(entries_for(keys, nil_every=17))
    qs = []
    for _ in range(6000):
        k = rng.choice(keys)
        r = rng.random()
        qs.append(k if r < 0.5 else (k[:8] + bytes([rng.getrandbits(8)]) if r < 0.8 else k[:rng.randint(0, len(k))]))
    check(idx, qs)


def handle_hits(idx_bytes, queries):
    """rio_index_open / rio_index_search (the cgo DiskIndexLoader binding's calls) on a host image."""
    h = ctypes.c_void_p()
    assert L.lib().rio_index_open(L.default_ctx(0), idx_bytes, len(idx_bytes), ctypes.byref(h)) == 0
    try:
        off = np.zeros(len(queries) + 1, dtype=np.uint64)
        np.cumsum([len(q) for q in queries], out=off[1:])
        blob = b"".join(queries) or b"\0"
        hits = (L.IndexHit * len(queries))()
        assert L.lib().rio_index_search(h, blob, off.ctypes.data, len(queries), hits) == 0
        return [(x.status, x.offset, bool(x.found), x.value_offset, x.checksum) for x in hits]
    finally:
        L.lib().rio_index_free(h)


@pytest.mark.parametrize("comp", [1, 2, 3])
def test_compressed_index_through_the_decoded_view(comp):
    """A gzip / snappy / lzw index.rio (rProto.NewMMapProtoReaderWithPath decompresses every record,
    disk_key_index.go:173): the handle decodes the index once and answers every probe from its records
    and SeekNext map; hits equal the oracle's binarySearch over the compressed file, adversarial keys
    (fake headers and 0x91 bytes inside entries) and nil records included."""
    rng = random.Random(20 + comp)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 40))) for _ in range(1500)})
    keys = [k + (b"\x91\x8d\x4c" if i % 7 == 1 else b"") for i, k in enumerate(keys)]
    keys = sorted(set(keys))
    for nil_every in (0, 11):
        idx = index_image(entries_for(keys, nil_every), comp)
        qs = queries_for(keys, rng, 100)
        got = handle_hits(idx, qs)
        for q, g in zip(qs, got):
            o = orc.disk_index_search(idx, q, 4096)
            if o[0] != 0:
                assert g[0] == o[0], (comp, q, g, o)
            else:
                assert g == o, (comp, q, g, o)
        assert sum(g[2] for g in got[:len(keys)]) > len(keys) // 2


@pytest.mark.parametrize("comp", [1, 2, 3])
@pytest.mark.parametrize("tail", [b"\x91", b"\x91\x8d"])
def test_compressed_index_ending_in_a_partial_marker(comp, tail):
    """A compressed index.rio whose last bytes are a cut marker (0x91, or 91 8d): SeekNext from a probe
    past the last record rewinds onto it and returns io.EOF (mmap_reader.go:88-124), so binarySearch
    reports "not found" at the end; the decoded view's SeekNext map must say the same,
    not hand the query back. Hits equal the oracle's binarySearch over the same bytes."""
    rng = random.Random(90 + comp)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 30))) for _ in range(300)})
    idx = bytes(index_image(entries_for(keys), comp)) + tail
    qs = queries_for(keys, rng, 60) + [b"\xff" * 41, keys[-1] + b"\x00"]
    got = handle_hits(idx, qs)
    for q, g in zip(qs, got):
        o = orc.disk_index_search(idx, q, 4096)
        if o[0] != 0:
            assert g[0] == o[0], (comp, q, g, o)
        else:
            assert g == o, (comp, q, g, o)
    assert all(g[0] != L.RIO_ERR_UNSUPPORTED for g in got)


@pytest.mark.parametrize("comp", [1, 2, 3])
def test_handed_back_probes_answered_on_the_host(tmp_path, comp):
    """A compressed index whose record 200 has a damaged header (its CRC no longer matches): FileReader,
    and so the handle's decoded view, stops there, while the reference's SeekNext steps over it and reads
    on (mmap_reader.go:105-110). The device hands back the probes that land past it
    (RIO_ERR_UNSUPPORTED); DiskKeyIndex answers them with the reference's binarySearch on the host
    reader, so Get / Contains / IteratorStartingAt agree with the oracle for every query."""
    rng = random.Random(40 + comp)
    keys = [be(3 * i) for i in range(400)]
    img = bytearray(index_image(entries_for(keys), comp))
    ro = orc.file_reader_decode(bytes(img))["rec_off"]
    img[ro[200] + 4] ^= 0x01  # record 200's u: its header CRC no longer matches
    img = bytes(img)
    qs = queries_for(keys, rng, 60)
    assert any(g[0] == L.RIO_ERR_UNSUPPORTED for g in handle_hits(img, qs))
    p = tmp_path / "index.rio"
    p.write_bytes(img)
    idx, err = DiskIndexLoader().Load(str(p), None)
    assert err is None and idx.Open() is None
    try:
        got = idx.lookups(qs)
        for q, (off, found, vo, cs, err), (v, gerr) in zip(qs, got, idx.GetBatch(qs)):
            o = orc.disk_index_search(img, q, 4096)  # (status, offset, found, value offset, checksum)
            if o[0] != 0:
                assert err is not None and "rio:" not in str(err), (q, o, err)
                continue
            assert err is None and (off, found) == (o[1], o[2]), (q, o, off, found)
            if found:
                assert gerr is None and v == IndexVal(o[3], o[4])
                assert idx.Contains(q) == (True, None)
            else:
                assert gerr is NotFound
        assert sum(1 for g in got if g[1]) >= 300
    finally:
        idx.Close()


@pytest.mark.parametrize("version", [3, 2, 1])
def test_older_version_indexes_match_oracle(version):
    """index.rio with the v3 / v2 / v1 header layouts: SeekNext-driven binarySearch on v3 / v2 as on v4;
    v1 fails every probe with SeekNext's "unsupported on files with version lower than v2"
    (mmap_reader.go:62-64)."""
    import corpus

    rng = random.Random(70 + version)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 30))) for _ in range(400)})
    img = corpus.to_version(bytes(index_image(entries_for(keys))), version)
    got = check(img, queries_for(keys, rng, 100))
    if version == 1:
        assert all(g[0] == L.RIO_ERR_UNSUPPORTED for g in got)
    else:
        assert sum(g[2] for g in got) >= len(keys)


def test_reference_v2_fixture_index():
    """The reference's SimpleWriteHappyPathSSTableRecordIOV2/index.rio (recordio v2): every key found at
    its IndexEntry, misses positioned as the oracle says."""
    import os

    from conftest import GOLDEN

    img = open(os.path.join(GOLDEN, "sstables", "SimpleWriteHappyPathSSTableRecordIOV2", "index.rio"), "rb").read()
    qs = [be(i) for i in range(0, 10)] + [b"", b"\x00\x00\x00\x04\x00"]
    got = check(img, qs)
    assert [g[2] for g in got[:10]] == [False] + [True] * 7 + [False, False]


def test_v1_index_through_the_api(tmp_path):
    """DiskKeyIndex over a v1 index.rio: Get / Contains fail with the reference's SeekNext error."""
    import corpus

    p = tmp_path / "index.rio"
    p.write_bytes(corpus.to_version(bytes(index_image(entries_for([be(i) for i in range(1, 8)]))), 1))
    idx, err = DiskIndexLoader().Load(str(p), None)
    assert err is None and idx.Open() is None
    try:
        v, err = idx.Get(be(3))
        assert str(err) == "unsupported on files with version lower than v2"
        assert str(idx.Contains(be(3))[1]) == "unsupported on files with version lower than v2"
    finally:
        idx.Close()
