"""Windowed sequential decode (GPU): rio_stream_* and the FileReader mirror over windows.

A file larger than its window is framed and decoded window by window, each window cut at a record
boundary (include/rio.h rio_stream_*). The records, their file offsets and the terminal status
(offset, details, record index) must be those of the whole-file FileReader loop: checked against
the oracle restatement (file_reader.go:61-131) on the golden fixtures, on generated workloads, on
records larger than the window (window growth), on zero tails (the DirectIO EOF reads to the end of
the file, not of the window) and on seeded random damage. Windows as small as 1 byte force a cut
inside every header and payload."""
import ctypes
import os
import random

import pytest

import oracle_py as orc
from corpus import mixed_records
from gpu_util import gpu_decode_arrays
from recordio import FileReader, encode_file, generate
from recordio import _lib as L

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = [os.path.join(HERE, "golden", d, f) for d in ("v4_compat", "v3_compat", "v2_compat", "v1_compat")
          for f in sorted(os.listdir(os.path.join(HERE, "golden", d)))]
NEVER = (1 << 64) - 1


def stream_all(data: bytes, window: int, depth: int = 2, path: str | None = None, register: bool = False):
    """Every window of rio_stream over `data` (host memory) or `path`: records, file offsets, the
    first_record of each window and the terminal info. `register`: the host image is page-locked
    (rio_host_register), so windows of 1 MiB and more are copied by DMA from it in place."""
    lib = L.lib()
    h = ctypes.c_void_p()
    buf = ctypes.create_string_buffer(data, len(data) + 1)
    if register:
        # "half": only the first half of the image is page-locked (windows past the
        # registered range must take the staging path, not a DMA past it)
        n_reg = (len(data) + 1) // 2 if register == "half" else len(data) + 1
        assert lib.rio_host_register(buf, n_reg) == 0
    try:
        return _stream_all(lib, h, buf, data, window, depth, path)
    finally:
        if register:
            assert lib.rio_host_unregister(buf) == 0


def _stream_all(lib, h, buf, data, window, depth, path):
    if path:
        rc = lib.rio_stream_open(0, path.encode(), window, depth, ctypes.byref(h))
    else:
        rc = lib.rio_stream_open_host(0, buf, len(data), window, depth, ctypes.byref(h))
    assert rc == 0, L.strerror(rc)
    recs, offs, firsts, term = [], [], [], None
    try:
        while True:
            first = ctypes.c_uint64()
            out, off, roff, fl = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
            info = L.FileInfo()
            rc = lib.rio_stream_next(h, ctypes.byref(first), ctypes.byref(out), ctypes.byref(off),
                                     ctypes.byref(roff), ctypes.byref(fl), ctypes.byref(info))
            if rc == L.RIO_EOF:
                break
            assert rc == 0, L.strerror(rc)
            assert term is None, "a window after the terminal one"
            assert first.value == len(recs)
            firsts.append(first.value)
            n = info.n_records
            o = ctypes.cast(off, ctypes.POINTER(ctypes.c_uint64))
            r = ctypes.cast(roff, ctypes.POINTER(ctypes.c_uint64))
            f = ctypes.cast(fl, ctypes.POINTER(ctypes.c_uint8))
            for i in range(n):
                lo, hi = o[i], o[i + 1]
                if f[i] & (L.RIO_FLAG_CORRUPT | L.RIO_FLAG_EOF):
                    recs.append(orc.BadRecord("corrupt" if f[i] & L.RIO_FLAG_CORRUPT else "eof"))
                elif f[i] & 1:
                    recs.append(None)
                else:
                    recs.append(ctypes.string_at(out.value + lo, hi - lo) if hi > lo else b"")
                offs.append(r[i])
            if info.status != L.RIO_OK:
                term = info.as_dict()
    finally:
        lib.rio_stream_free(h)
    assert term is not None, "no terminal window"
    return recs, offs, firsts, term


def check_stream(data: bytes, window: int, **kw):
    """Records, offsets and terminal status as the oracle's (details where the contract defines
    them: HEADER_CRC's CRCs, gpu_util.assert_same_as_oracle); every detail as the whole-file device
    decode's (the reader's error text depends on them, e.g. a payload-raised ErrUnexpectedEOF)."""
    exp = orc.file_reader_decode(data)
    recs, offs, firsts, term = stream_all(data, window, **kw)
    assert recs == exp["records"]
    assert offs == exp["rec_off"]
    assert (term["status"], term["status_offset"]) == (exp["status"], exp["status_offset"])
    if exp["status"] == L.RIO_ERR_HEADER_CRC:
        assert (term["detail0"], term["detail1"]) == (exp["detail0"], exp["detail1"])
    whole = gpu_decode_arrays(data)
    assert (term["status"], term["detail0"], term["detail1"]) == (whole["status"], whole["detail0"], whole["detail1"])
    return firsts


def reader_loop(path: str, window: int, skip_every: int = 0):
    """FileReader ReadNext (and SkipNext) loop: records and the error text."""
    r = FileReader(path, 0, window)
    err = r.Open()
    if err is not None:  # file header errors are Open's (file_reader.go:35-59)
        return ["open"], str(err)
    got, i = [], 0
    while True:
        if skip_every and i % skip_every == 1:
            err = r.SkipNext()
            if err is not None:
                return got, str(err)
            got.append("skip")
        else:
            rec, err = r.ReadNext()
            if err is not None:
                return got, str(err)
            got.append(rec)
        i += 1


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(os.path.dirname(p)) + "/" + os.path.basename(p)
                                              for p in GOLDEN])
@pytest.mark.parametrize("window", [1, 5, 13, 64, 4096])
def test_golden_fixtures(path, window):
    data = open(path, "rb").read()
    if len(data) < 8 or orc.file_reader_decode(data)["status"] == L.RIO_ERR_UNSUPPORTED:
        pytest.skip("not a device-path file")
    check_stream(data, window)
    assert reader_loop(path, window) == reader_loop(path, NEVER)
    assert reader_loop(path, window, skip_every=3) == reader_loop(path, NEVER, skip_every=3)


@pytest.mark.parametrize("n,rec_len,comp,kind,window", [
    (3000, 1024, 2, 1, 4096),
    (3000, 1024, 2, 1, 100_000),
    (3000, 1024, 0, 0, 65536),
    (600, 1024, 1, 1, 50_000),
    (20000, 64, 2, 1, 30_000),
    (40, 65536, 2, 1, 4096),  # every record larger than the window: the window doubles
    (1500, 1024, 3, 1, 40_000),  # lzw
])
def test_generated_workloads(n, rec_len, comp, kind, window):
    data = bytes(generate(n, rec_len, comp, kind=kind, seed=n + comp))
    firsts = check_stream(data, window)
    assert len(firsts) >= 2  # it really ran windowed


def test_path_source_and_depth(tmp_path):
    data = bytes(generate(5000, 1024, 2, kind=1, seed=9))
    p = tmp_path / "f.rio"
    p.write_bytes(data)
    a = stream_all(data, 50_000, depth=1, path=str(p))
    b = stream_all(data, 50_000, depth=8)
    assert a == b
    exp = orc.file_reader_decode(data)
    assert a[0] == exp["records"]


@pytest.mark.parametrize("window", [1 << 20, (3 << 20) + 17, 16 << 20, NEVER])
def test_registered_host_image(window):
    """A page-locked host image (rio_host_register): each window's bytes go to the device by DMA from
    the image in place, behind the file header copied separately (rio::frame_direct). Same records,
    offsets and status as the oracle and as the staged path."""
    data = bytes(generate(40_000, 1024, 2, kind=1, seed=31))
    check_stream(data, window, register=True)
    damaged = bytearray(data)
    damaged[len(data) // 2 + 5] ^= 0x40
    check_stream(bytes(damaged), window, register=True)


@pytest.mark.parametrize("window", [1 << 20, 3 << 20])
def test_partly_registered_host_image(window):
    """Only the first half of the image is page-locked: windows inside it are DMA'd in place, the
    ones that reach past it go through the staging pieces; records, offsets and status are those of
    the oracle either way (the whole window must be registered for the in-place copy)."""
    data = bytes(generate(12_000, 1024, 2, kind=1, seed=33))
    assert len(data) > 4 * window // 2
    check_stream(data, window, register="half")


def test_registered_image_one_shot():
    """rio_frame + rio_decode of a page-locked image equal those of the same bytes unregistered."""
    import numpy as np

    lib = L.lib()
    img = generate(20_000, 1024, 2, kind=1, seed=32)
    ctx = L.default_ctx(0)

    def one_shot():
        fi = L.FileInfo()
        assert lib.rio_frame(ctx, img.ctypes.data, img.shape[0], ctypes.byref(fi)) == 0
        n, nb = fi.n_records, fi.total_out_bytes
        out, out_off = np.empty(nb + 16, np.uint8), np.empty(n + 1, np.uint64)
        rec_off, flags = np.empty(n + 1, np.uint64), np.empty(n + 1, np.uint8)
        assert lib.rio_decode(ctx, out.ctypes.data, out.shape[0], out_off.ctypes.data, rec_off.ctypes.data,
                              flags.ctypes.data, n, ctypes.byref(fi)) == 0
        return out[:nb].tobytes(), out_off.tobytes(), rec_off[:n].tobytes(), flags[:n].tobytes(), fi.status

    plain = one_shot()
    assert lib.rio_host_register(img.ctypes.data, img.shape[0]) == 0
    try:
        assert one_shot() == plain
    finally:
        assert lib.rio_host_unregister(img.ctypes.data) == 0
    exp = orc.file_reader_decode_arrays(img)
    assert plain[0] == exp["out"].tobytes() and plain[4] == exp["status"]


def test_whole_file_when_smaller_than_window():
    data = bytes(generate(100, 1024, 2, kind=1, seed=3))
    firsts = check_stream(data, len(data))
    assert firsts == [0]


@pytest.mark.parametrize("window", [100, 1000, 20_000])
def test_zero_tail_spans_windows(tmp_path, window):
    """DirectIO padding: a magic mismatch followed only by zeros is io.EOF; the zeros reach past
    many windows, and garbage after them turns it into MagicNumberMismatch (…_directio_trailer)."""
    body = encode_file(mixed_records(60, 5, max_len=300), 0)
    for tail, trailer in ((50_000, b""), (50_000, b"\x07"), (3, b""), (0, b"\x01\x02")):
        data = body + b"\x00" * tail + trailer
        check_stream(data, window)
        p = tmp_path / "z.rio"
        p.write_bytes(data)
        assert reader_loop(str(p), window) == reader_loop(str(p), NEVER)


def test_corrupt_record_mid_file_in_any_window():
    """A header CRC failure in the middle of a long file ends the stream there with the whole-file
    status, whatever window the record falls in; a snappy ErrCorrupt is that record's alone (flagged,
    the stream goes on) in every window layout."""
    recs = mixed_records(400, 11, max_len=900)
    data = bytearray(encode_file(recs, 2))
    exp = orc.file_reader_decode(bytes(data))
    off = exp["rec_off"][250]
    data[off + 5] ^= 0x40  # inside the header: CRC or varint failure
    for w in (700, 4096, 65536):
        check_stream(bytes(data), w)
    data2 = bytearray(encode_file(recs, 2))
    end = exp["rec_off"][301]
    data2[end - 3:end] = b"\xff\xff\xff"  # last payload bytes of record 300: snappy stream corrupt
    for w in (700, 4096, 65536):
        check_stream(bytes(data2), w)


@pytest.mark.parametrize("seed", range(40))
def test_random_damage_random_windows(tmp_path, seed):
    from test_gpu_fuzz import damage

    rng = random.Random(500 + seed)
    data = encode_file(mixed_records(rng.randint(20, 300), seed, max_len=2000), rng.choice([0, 2]))
    if seed % 4 == 3:  # the older header layouts (nil records become empty ones in v1 / v2)
        import corpus

        v = rng.choice([1, 2, 3])
        data = corpus.to_version(data, 3) if v == 3 else corpus.legacy_file(
            [r or b"" for r in mixed_records(rng.randint(20, 300), seed, max_len=2000)], data[4], v)
    data = damage(rng, data)
    if rng.random() < 0.3:
        data += b"\x00" * rng.randint(1, 5000)
    window = rng.choice([1, 7, rng.randint(8, 600), rng.randint(600, 20_000)])
    check_stream(data, window, depth=rng.choice([1, 2, 4]))
    p = tmp_path / "d.rio"
    p.write_bytes(data)
    assert reader_loop(str(p), window) == reader_loop(str(p), NEVER)


def test_file_reader_windows_large_files_by_default(tmp_path):
    """Files over 256 MiB are windowed by default (FileInfo then has no whole-file totals); every
    record equals the oracle's."""
    import hashlib

    img = generate(300_000, 1024, 0, kind=1, seed=21)
    assert img.shape[0] > (256 << 20)
    p = tmp_path / "big.rio"
    img.tofile(str(p))
    exp = orc.file_reader_decode_arrays(img)
    r = FileReader(str(p))
    assert r.Open() is None
    h, n = hashlib.sha1(), 0
    while True:
        rec, err = r.ReadNext()
        if err is not None:
            break
        h.update(rec)
        n += 1
    assert r.FileInfo() is None  # windowed
    assert n == exp["n_records"] == 300_000
    assert h.digest() == hashlib.sha1(exp["out"].tobytes()).digest()
    assert "EOF" in str(err)


@pytest.mark.parametrize("seed", range(24))
def test_lzw_random_damage_random_windows(tmp_path, seed):
    """Damaged lzw files: a flipped payload byte may leave a valid stream of another length (the
    resize round), an invalid code, or a stream cut short; headers may break too."""
    from test_gpu_fuzz import damage

    rng = random.Random(900 + seed)
    recs = mixed_records(rng.randint(20, 200), seed + 70, max_len=3000)
    data = damage(rng, encode_file(recs, 3))
    window = rng.choice([7, rng.randint(8, 600), rng.randint(600, 20_000), NEVER])
    check_stream(data, window, depth=rng.choice([1, 2, 4]))
    from gpu_util import assert_same_as_oracle

    assert_same_as_oracle(gpu_decode_arrays(data), orc.file_reader_decode_arrays(data), f"lzw damage {seed}")
    p = tmp_path / "l.rio"
    p.write_bytes(data)
    assert reader_loop(str(p), window) == reader_loop(str(p), NEVER)
