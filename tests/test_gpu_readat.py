"""ReadAtI on the device path (GPU): MMapReader.ReadNextAt / SeekNext (mmap_reader.go:58-203).

The reader decodes the file once; a ReadNextAt at a record start and a SeekNext whose scan reaches a
record header over bytes that cannot form a marker are then answered on the calling thread from the
decoded records, everything else by the single-record kernels. ReadAtI implementations must be
thread-safe (recordio.go:91-92): many host threads call one reader at once, including its first call
(the one that builds the decoded view). Every answer is checked against the oracle restatement, and
gzip files (whose payloads only the whole-file decode inflates) answer ReadNextAt / SeekNext too.
"""
import ctypes
import random
import threading

import pytest

import corpus
import oracle_py as orc
from recordio import NewMemoryMappedReaderWithPath, generate
from recordio import _lib as L

pytestmark = pytest.mark.gpu


def _call_read_at(r, off):
    data, n, nil = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int()
    rc = L.lib().rio_reader_read_next_at(r._h, off, ctypes.byref(data), ctypes.byref(n), ctypes.byref(nil))
    rec = None
    if rc == 0 and not nil.value:
        rec = ctypes.string_at(data.value, n.value) if n.value else b""
    return rc, rec


def _call_seek(r, off):
    data, n, nil, ro = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int(), ctypes.c_uint64()
    rc = L.lib().rio_reader_seek_next(r._h, off, ctypes.byref(ro), ctypes.byref(data), ctypes.byref(n),
                                      ctypes.byref(nil))
    rec = None
    if rc == 0 and not nil.value:
        rec = ctypes.string_at(data.value, n.value) if n.value else b""
    return rc, (ro.value if rc == 0 else None), rec


def _open(tmp_path, img, name="f.rio"):
    p = tmp_path / name
    p.write_bytes(bytes(img))
    r, err = NewMemoryMappedReaderWithPath(str(p))
    assert err is None and r.Open() is None
    return r, str(p)


@pytest.mark.parametrize("kind", [1, 2])
def test_many_threads_one_reader(tmp_path, kind):
    """8 threads start together on a fresh reader (racing for the one decode), then each runs a
    seeded mix of ReadNextAt at record starts, ReadNextAt inside records and SeekNext from random
    offsets; every answer equals the oracle's."""
    img = bytes(generate(3000, 700, 2, kind=kind, seed=40 + kind))
    o = orc.file_reader_decode(img)
    starts = o["rec_off"]
    rng = random.Random(7)
    plans = []
    for t in range(8):
        ops = []
        for _ in range(300):
            u = rng.random()
            if u < 0.6:
                k = rng.randrange(len(starts))
                ops.append(("at", starts[k], (0, o["records"][k])))
            elif u < 0.75:
                off = rng.randrange(len(img) + 2)
                st, rec = orc.read_next_at(img, off)
                ops.append(("at", off, (st, rec)))
            else:
                off = rng.randrange(len(img) + 2)
                st, ro, rec = orc.seek_next(img, off)
                ops.append(("seek", off, (st, ro if st == 0 else None, rec)))
        plans.append(ops)
    r, _ = _open(tmp_path, img)
    go = threading.Barrier(8)
    bad = []

    def run(ops):
        go.wait()
        for kind_, off, want in ops:
            got = _call_read_at(r, off) if kind_ == "at" else _call_seek(r, off)
            if got != want:
                bad.append((kind_, off, got[:2], want[:2]))

    th = [threading.Thread(target=run, args=(ops,)) for ops in plans]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not bad, bad[:5]
    r.Close()


def test_seek_next_fast_and_kernel_paths_agree_everywhere(tmp_path):
    """Random payloads put 0x91 bytes in most gaps: SeekNext from every offset of a small file
    (both the host answers and the kernel scans), with the default window and 5-, 4- and 3-byte
    ones (at 3 the reference ends every marker in io.EOF: mmap_reader.go:89-98)."""
    recs = [bytes(random.Random(i).getrandbits(8) for _ in range(60 + 7 * i)) for i in range(40)]
    recs[5] = b"\x91" * 30 + b"\x91\x8d\x4c\x00" + b"x" * 10  # a marker-like run inside a payload
    recs[6] = b"ab\x91"  # ends in 0x91: the scan's skip rule passes over the next record's magic
    img = corpus.encode_file(recs, 0)
    r, path = _open(tmp_path, img)
    for seek_len in (4096, 5, 4, 3):
        r.seekLen = seek_len
        for off in range(len(img) + 2):
            st, ro, rec = orc.seek_next(img, off, seek_len)
            assert _call_seek(r, off) == (st, ro if st == 0 else None, rec), (seek_len, off)
    r.Close()


GZ = {n: img for n, img, _ in corpus.gzip_cases()}


@pytest.mark.parametrize("name", ["gz_text_small", "gz_mixed_nil_empty", "gz_empty_payload", "gz_bad_crc",
                                  "gz_header_fields", "gz_v3", "gz_large", "gz_v2", "gz_v1"])
def test_gzip_read_next_at_and_seek_next(name, tmp_path):
    """gzip files through ReadAtI: every record start, offsets inside records, SeekNext from a
    sample of offsets; the oracle's status class and record, and the reference's error value."""
    from go_errors import assert_go_error, expect_read_next_at, expect_seek_next

    img = GZ[name]
    r, path = _open(tmp_path, img)
    o = orc.file_reader_decode(img)
    rng = random.Random(3)
    offs = list(o["rec_off"]) + [rng.randrange(len(img) + 2) for _ in range(200)] + [len(img), len(img) + 1]
    for off in offs:
        st, want, d0, d1 = orc.read_next_at(img, off, details=True)
        rc, got = _call_read_at(r, off)
        assert (rc, got) == (st, want), (name, off)
        if st:
            _, err = r.ReadNextAt(off)
            assert_go_error(err, expect_read_next_at(st, off, path, d0, d1, version=img[0]))
    for off in offs[::3]:
        st, ro, want = orc.seek_next(img, off)
        assert _call_seek(r, off) == (st, ro if st == 0 else None, want), (name, off)
        if st == L.RIO_ERR_UNSUPPORTED:  # v1 (mmap_reader.go:62-64)
            _, _, err = r.SeekNext(off)
            assert str(err) == "unsupported on files with version lower than v2"
        elif st:
            _, _, err = r.SeekNext(off)
            assert_go_error(err, expect_seek_next(st, off, ro, path, version=img[0]))
    r.Close()


def test_read_at_data_pointer_survives_other_calls(tmp_path):
    """A record served from the decoded view stays readable while the same and other threads go on
    (the pointer is into the reader's decoded arena, valid until rio_reader_free)."""
    img = bytes(generate(200, 300, 2, kind=1, seed=5))
    o = orc.file_reader_decode(img)
    r, _ = _open(tmp_path, img)
    data, n, nil = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int()
    assert L.lib().rio_reader_read_next_at(r._h, o["rec_off"][10], ctypes.byref(data), ctypes.byref(n),
                                           ctypes.byref(nil)) == 0
    for k in range(0, 200, 3):
        assert _call_read_at(r, o["rec_off"][k]) == (0, o["records"][k])
    assert ctypes.string_at(data.value, n.value) == o["records"][10]
    r.Close()
