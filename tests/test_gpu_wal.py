"""WAL replay on the device (GPU): wal.Replayer.Replay over the ordered replay pipeline
(rio_replay_*), checked against the oracle's FileReader loop per file and against the reference's own
loop (ReaderFactory over the FileReader mirror). Mirrors wal/appender_test.go's replay assertions
and wal/replayer_test.go."""
import os
import random
import struct

import pytest

import oracle_py as orc
from corpus import header_v4, mixed_records
import wal as W
from recordio import NewFileReaderWithPath, encode_file
from recordio.errors import EOF, GoError, errors_is

pytestmark = pytest.mark.gpu
TestMaxWalFileSize = 8 * 1024
EOF_CLASS = (0, 1, 2, 3, 4)


def replay(opts, stop_after=None):
    r, err = W.NewReplayer(opts)
    assert err is None
    got = []

    def process(rec):
        got.append(rec)
        if stop_after is not None and len(got) == stop_after:
            return GoError("test")
        return None

    return got, r.Replay(process)


def expected(base):
    """Oracle: sorted *.wal files, each decoded by the FileReader restatement; stop at a non-EOF end.
    A record that does not decompress ends the replay (its ReadNext error), or only its file when the
    error is gzip's bare io.EOF (replayer.go:59-67)."""
    recs = []
    for p in W._wal_files(base):
        o = orc.file_reader_decode(open(p, "rb").read())
        bad = [i for i, r in enumerate(o["records"]) if isinstance(r, orc.BadRecord)]
        if bad:
            recs += o["records"][:bad[0]]
            if o["records"][bad[0]].kind == "eof":
                continue
            return recs, p, o
        recs += o["records"]
        if o["status"] not in EOF_CLASS:
            return recs, p, o
    return recs, None, None


def both_paths_agree(base, **kw):
    opts, _ = W.NewWriteAheadLogOptions(W.BasePath(base), **kw) if kw else W.NewWriteAheadLogOptions(W.BasePath(base))
    dev, derr = replay(opts)
    ropts, _ = W.NewWriteAheadLogOptions(W.BasePath(base), W.ReaderFactory(NewFileReaderWithPath))
    ref, rerr = replay(ropts)
    assert dev == ref
    assert (None if derr is None else str(derr)) == (None if rerr is None else str(rerr))
    return dev, derr


def appender(tmp_path, comp=0, max_size=TestMaxWalFileSize):
    d = tmp_path / "wal"
    d.mkdir()
    opts, _ = W.NewWriteAheadLogOptions(W.BasePath(str(d)), W.MaximumWalFileSizeBytes(max_size),
                                        W.WriterFactory(lambda p: __import__("recordio").NewFileWriter(p, comp)))
    a, err = W.NewAppender(opts)
    assert err is None
    return a


def test_single_record(tmp_path):
    a = appender(tmp_path)
    assert a.AppendSync(b"\x01") is None and a.Close() is None
    got, err = replay(a.walOptions)
    assert err is None and got == [b"\x01"]


def test_rotation_happy_path(tmp_path):
    a = appender(tmp_path)
    rec = [struct.pack(">Q", i) for i in range(3 * (TestMaxWalFileSize // 8))]
    for r in rec:
        assert a.AppendSync(r) is None
    assert a.nextWriterNumber == 8 and a.Close() is None
    got, err = replay(a.walOptions)
    assert err is None and got == rec


def test_more_than_hundred_files_in_order(tmp_path):
    a = appender(tmp_path)
    rec = [struct.pack(">Q", i) for i in range(200)]
    for r in rec:
        assert a.AppendSync(r) is None
        assert a.Rotate()[1] is None
    assert a.Close() is None
    for depth in (1, 2, 7):
        opts, _ = W.NewWriteAheadLogOptions(W.BasePath(a.walOptions.basePath), W.ReplayOnDevice(0, depth))
        got, err = replay(opts)
        assert err is None and got == rec, depth


def test_bigger_record_than_max_and_forced_rotation(tmp_path):
    a = appender(tmp_path)
    big = bytes(i % 255 for i in range(TestMaxWalFileSize + 5))
    rec = [big] + [bytes([i]) for i in range(95)]
    assert a.AppendSync(big) is None
    for r in rec[1:]:
        assert a.AppendSync(r) is None
        assert a.Rotate()[1] is None
    assert a.Close() is None
    got, err = replay(a.walOptions)
    assert err is None and got == rec


def test_ignores_non_wal_files(tmp_path):
    a = appender(tmp_path)
    assert a.AppendSync(b"\x01") is None and a.Close() is None
    (tmp_path / "wal" / "some-not-so-wal-file").write_bytes(b"\x01\x02\x03")
    got, err = replay(a.walOptions)
    assert err is None and got == [b"\x01"]


def test_honors_callback_errors(tmp_path):
    a = appender(tmp_path)
    for i in range(10):
        assert a.AppendSync(bytes([i])) is None
    assert a.Close() is None
    got, err = replay(a.walOptions, stop_after=4)
    assert len(got) == 4 and err is not None
    assert str(err).startswith("error while processing WAL record under '") and str(err).endswith("': test")


@pytest.mark.parametrize("comp", [0, 2])
def test_mixed_records_large_files_match_oracle(tmp_path, comp):
    # simpledb recovery replays snappy WALs (simpledb/recovery.go:178-201); nil and empty records included
    a = appender(tmp_path, comp, max_size=1 << 20)
    rec = mixed_records(4000, seed=comp + 5, max_len=5000)
    for r in rec:
        assert (a.AppendSync(r) if r is not None else a.AppendSync(b"")) is None
    assert a.Close() is None
    exp, _, _ = expected(a.walOptions.basePath)
    got, err = both_paths_agree(a.walOptions.basePath)
    assert err is None and got == exp
    assert [x if x is not None else b"" for x in rec] == [x if x is not None else b"" for x in got]


def write_wal_dir(tmp_path, files):
    d = tmp_path / "w"
    d.mkdir()
    for i, img in enumerate(files):
        (d / (W.defaultWalFilePattern % i)).write_bytes(img)
    return str(d)


def test_nil_records(tmp_path):
    base = write_wal_dir(tmp_path, [encode_file([b"a", None, b"", None], 2), encode_file([None], 0)])
    got, err = both_paths_agree(base)
    assert err is None and got == [b"a", None, b"", None, None]


@pytest.mark.parametrize("damage", ["crc", "truncated_payload", "truncated_header", "zero_tail", "garbage_tail"])
def test_damaged_file_in_the_middle(tmp_path, damage):
    rng = random.Random(7)
    files = [encode_file([bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300))) for _ in range(50)], c)
             for c in (0, 2, 2)]
    mid = bytearray(files[1])
    if damage == "crc":
        mid[8 + 6] ^= 0x40  # first record's CRC varint
    elif damage == "truncated_payload":
        mid = mid[:-3]
    elif damage == "truncated_header":
        mid += header_v4(10, 5)[:4]
    elif damage == "zero_tail":
        mid += bytes(100)  # DirectIO padding: a clean EOF
    else:
        mid += b"\x07" * 20
    files[1] = bytes(mid)
    base = write_wal_dir(tmp_path, files)
    exp, bad, o = expected(base)
    got, err = both_paths_agree(base)
    assert got == exp
    if bad is None:
        assert err is None
    else:
        assert str(err).startswith(f"error while reading WAL records under '{bad}': ")


def test_empty_and_short_wal_files(tmp_path):
    for k, (content, inner) in enumerate(((b"", "EOF"), (b"\x04\x00\x00", "unexpected EOF"))):
        root = tmp_path / f"c{k}"
        root.mkdir()
        base = write_wal_dir(root, [encode_file([b"x"], 0), content])
        got, err = both_paths_agree(base)
        assert got == [b"x"]
        p = os.path.join(base, "000001.wal")
        assert str(err) == f"error while opening WAL reader under '{p}': error while reading header bytes of '{p}': {inner}"


def test_header_errors(tmp_path):
    base = write_wal_dir(tmp_path, [struct.pack("<II", 9, 0) + b"rest"])
    got, err = both_paths_agree(base)
    assert got == [] and "version mismatch, expected a value from 1 to 4 but was 9" in str(err)


def test_legacy_recordio_files_replay(tmp_path):
    # WAL files written by older versions of the library (recordio v2 and v1 headers) replay on the
    # device like v4 ones: readNextV2 / readNextV1 (file_reader.go:282-388)
    v2 = struct.pack("<II", 2, 0) + b"\x91\x8d\x4c\x01\x00z"
    v1 = struct.pack("<II", 1, 0) + struct.pack("<IQQ", 0x130691, 2, 0) + b"yy"
    base = write_wal_dir(tmp_path, [encode_file([b"a"], 0), v2, v1])
    got, err = both_paths_agree(base)
    assert got == [b"a", b"z", b"yy"] and err is None


def test_empty_directory(tmp_path):
    d = tmp_path / "empty"
    d.mkdir()
    opts, _ = W.NewWriteAheadLogOptions(W.BasePath(str(d)))
    assert replay(opts) == ([], None)
    assert errors_is(EOF, EOF)


@pytest.mark.parametrize("devices,workers", [([0, 0], 1), ([0, 0, 0], 2)])
def test_replay_over_a_device_list(tmp_path, devices, workers):
    """rio_replay_open_devices: workers spread over several devices (all mapped to the box's GPU),
    files still handed out in order; same records and error as the reference's loop."""
    a = appender(tmp_path, 2, max_size=64 << 10)
    rec = mixed_records(3000, seed=41, max_len=3000)
    for r in rec:
        assert (a.AppendSync(r) if r is not None else a.AppendSync(b"")) is None
    assert a.Close() is None
    exp, _, _ = expected(a.walOptions.basePath)
    opts, _ = W.NewWriteAheadLogOptions(W.BasePath(a.walOptions.basePath), W.ReplayOnDevice(devices, 3, workers))
    got, err = replay(opts)
    assert err is None and got == exp
