"""MMapReader.ReadNextAt / SeekNext on gzip and lzw files at records the FileReader loop never reaches.

mmap_reader.go:130-203 decodes any record start it is pointed at. A header that fails its CRC in the
middle of a file ends FileReader's loop (and so the reader handle's decoded index) there, while the
records after it stay readable by offset: the single-record kernel locates them and the host decodes
each as a file of its own through the whole-file path (readat_expand in rio_capi.cpp). Compared with
the oracle's ReadNextAt / SeekNext (status, record, the failing trial's offset), payload damage after
the break included.
"""
import ctypes

import pytest

import corpus
import oracle_py as orc
from conftest import STATUS

pytestmark = pytest.mark.gpu


def _records(n, seed):
    return corpus.text_records(n, seed, 1, 2500)


def _gzip_image(recs):
    return corpus.gz_file([(len(r), corpus.gzip_member(r)) for r in recs])


def _lzw_image(recs):
    return corpus.lzw_file([(len(r), orc.lzw_encode(r)) for r in recs])


def _damage(img, o, k_crc, k_payload):
    """Record k_crc's header CRC no longer matches (its nil byte 0x00 -> 0x02), record k_payload's
    payload loses its last 3 bytes' meaning (they are zeroed)."""
    b = bytearray(img)
    b[int(o["rec_off"][k_crc]) + 3] ^= 0x02
    end = int(o["rec_off"][k_payload + 1])
    b[end - 3:end] = b"\0\0\0"
    return bytes(b)


def _read_next_at(h, off):
    from recordio import _lib as L

    data, n, nil = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int()
    rc = L.lib().rio_reader_read_next_at(h, off, ctypes.byref(data), ctypes.byref(n), ctypes.byref(nil))
    rec = None
    if rc == 0 and not nil.value:
        rec = ctypes.string_at(data.value, n.value) if n.value else b""
    return rc, rec


def _seek_next(h, off):
    from recordio import _lib as L

    data, n, nil, ro = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64()
    rc = L.lib().rio_reader_seek_next(h, off, ctypes.byref(ro), ctypes.byref(data), ctypes.byref(n),
                                      ctypes.byref(nil))
    rec = None
    if rc == 0 and not nil.value:
        rec = ctypes.string_at(data.value, n.value) if n.value else b""
    return rc, ro.value, rec


@pytest.mark.parametrize("codec", ["gzip", "lzw"])
def test_records_past_a_broken_header_are_read_by_offset(codec, tmp_path):
    from recordio import NewMemoryMappedReaderWithPath

    recs = _records(160, 77 if codec == "gzip" else 78)
    img = _gzip_image(recs) if codec == "gzip" else _lzw_image(recs)
    o = orc.file_reader_decode(img)
    img = _damage(img, o, 60, 100)
    o2 = orc.file_reader_decode(img)
    assert o2["status"] == STATUS["HEADER_CRC"] and o2["n_records"] == 60  # FileReader stops at record 60
    p = tmp_path / "f.rio"
    p.write_bytes(img)
    r, err = NewMemoryMappedReaderWithPath(str(p))
    assert err is None and r.Open() is None
    n_past = n_bad = 0
    for k in range(160):
        off = int(o["rec_off"][k])
        st, want = orc.read_next_at(img, off)
        rc, got = _read_next_at(r._h, off)
        assert rc == st, (codec, k, rc, st)
        if st == 0:
            assert got == want == recs[k], (codec, k)
            n_past += k > 60
        else:
            n_bad += 1
    assert n_past == 98 and n_bad == 2  # record 60 (header CRC) and record 100 (payload)
    # SeekNext from offsets before, at and after both damaged records
    lo, hi = int(o["rec_off"][55]), int(o["rec_off"][110])
    for off in list(range(lo, hi, 97)) + [int(o["rec_off"][60]) + 1, int(o["rec_off"][100]) - 1]:
        st, ro, want = orc.seek_next(img, off, 4096)
        rc, g_ro, got = _seek_next(r._h, off)
        assert rc == st, (codec, off, rc, st)
        if st == 0 or st not in (STATUS["EOF"], STATUS["INVALID_OFFSET"]):
            assert g_ro == ro, (codec, off)
        assert got == want, (codec, off)
    r.Close()


def test_empty_gzip_payload_past_the_break_continues_the_seek(tmp_path):
    """An empty gzip payload is gzip.NewReader's io.EOF: ReadNextAt reports it, SeekNext's trial
    treats it as io.EOF-class and scans on to the next record (mmap_reader.go:105-114)."""
    recs = _records(40, 79)
    items = [(len(r), corpus.gzip_member(r)) for r in recs]
    items[25] = (0, b"")
    img = corpus.gz_file(items)
    o = orc.file_reader_decode(img)
    b = bytearray(img)
    b[int(o["rec_off"][10]) + 3] ^= 0x02  # the loop stops at record 10
    img = bytes(b)
    p = tmp_path / "f.rio"
    p.write_bytes(img)
    from recordio import NewMemoryMappedReaderWithPath

    r, _ = NewMemoryMappedReaderWithPath(str(p))
    assert r.Open() is None
    for k in (11, 24, 25, 26, 39):
        off = int(o["rec_off"][k])
        st, want = orc.read_next_at(img, off)
        rc, got = _read_next_at(r._h, off)
        assert (rc, got) == (st, want), k
    for k in (24, 25):
        off = int(o["rec_off"][k]) + 1
        st, ro, want = orc.seek_next(img, off, 4096)
        assert _seek_next(r._h, off) == (st, ro, want), k
    r.Close()


def test_huge_claimed_lzw_record_past_the_break_is_a_status(tmp_path):
    """An lzw record after a broken header whose u claims 4.6 GB (lzw allows 4096x its payload): the
    expansion would be sized from that claim, so it is refused with a status, never an exception
    through the C-ABI (readat_expand): RIO_ERR_CAPACITY from the cap, or RIO_ERR_UNSUPPORTED
    when the one-record decode hands the record back first (sizes past 4 GiB), which the cgo adapter
    answers with the reference reader itself."""
    import random

    from recordio import NewMemoryMappedReaderWithPath
    from recordio import _lib as L

    recs = _records(3, 80)
    items = [(len(r), orc.lzw_encode(r)) for r in recs]
    rng = random.Random(81)
    junk = bytes(rng.getrandbits(8) for _ in range(1_200_000))
    items.append((4_600_000_000, junk))
    img = corpus.lzw_file(items)
    # record offsets from the same file with a 2-byte payload in the last record (the oracle would
    # reserve the claimed 4.6 GB); records 0..3 start at the same offsets
    o = orc.file_reader_decode(corpus.lzw_file(items[:3] + [(4_600_000_000, b"ab")]))
    b = bytearray(img)
    b[int(o["rec_off"][1]) + 3] ^= 0x02  # FileReader stops at record 1
    img = bytes(b)
    p = tmp_path / "f.rio"
    p.write_bytes(img)
    r, err = NewMemoryMappedReaderWithPath(str(p))
    assert err is None and r.Open() is None
    rc, got = _read_next_at(r._h, int(o["rec_off"][3]))
    assert rc in (L.RIO_ERR_CAPACITY, L.RIO_ERR_UNSUPPORTED) and got is None
    rc, got = _read_next_at(r._h, int(o["rec_off"][2]))  # an ordinary record past the break still reads
    assert rc == 0 and got == recs[2]
    r.Close()
