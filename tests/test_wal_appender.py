"""WAL options / appender / replayer construction (CPU): mirrors wal/appender_test.go and
wal/replayer_test.go for everything that does not decode. The appender writes through the
byte-identical v4 writer, so rotation points (Size() + len(record) > max) match the reference's."""
import os
import struct

import wal as W
from recordio.errors import GoError

TestMaxWalFileSize = 8 * 1024  # appender_test.go:12


def new_appender(tmp_path, name="wal"):
    d = tmp_path / name
    d.mkdir()
    opts, err = W.NewWriteAheadLogOptions(W.BasePath(str(d)), W.MaximumWalFileSizeBytes(TestMaxWalFileSize))
    assert err is None
    a, err = W.NewAppender(opts)
    assert err is None
    return a


def test_options_need_base_path():
    opts, err = W.NewWriteAheadLogOptions()
    assert opts is None and str(err) == "basePath was not supplied"
    opts, err = W.NewWriteAheadLogOptions(W.BasePath("x"))
    assert err is None and opts.maxWalFileSize == W.DefaultMaxWalSize


def test_rotation_points_match_reference(tmp_path):
    # TestSimpleWriteWithRotationHappyPath (appender_test.go:19-39): 3 x 1024 8-byte records, 8 KiB files
    a = new_appender(tmp_path)
    assert a.nextWriterNumber == 1
    for i in range(3 * (TestMaxWalFileSize // 8)):
        assert a.AppendSync(struct.pack(">Q", i)) is None
    assert a.nextWriterNumber == 8
    assert a.Close() is None
    names = sorted(os.listdir(a.walOptions.basePath))
    assert names == [W.defaultWalFilePattern % i for i in range(8)]
    # the check counts the payload only (appender.go:71-80), so a file may pass the limit by one header
    assert all(os.path.getsize(os.path.join(a.walOptions.basePath, n)) <= TestMaxWalFileSize + 36 for n in names)


def test_forced_rotation_and_more_than_hundred(tmp_path):
    a = new_appender(tmp_path)
    for i in range(200):
        assert a.AppendSync(struct.pack(">Q", i)) is None
        prev, err = a.Rotate()
        assert err is None and prev.endswith(W.defaultWalFilePattern % i)
    assert a.nextWriterNumber == 201
    assert a.Close() is None


def test_more_than_a_million_files_fails(tmp_path):
    a = new_appender(tmp_path)
    a.nextWriterNumber = 1000000
    err = a.AppendSync(bytes(TestMaxWalFileSize))
    assert "not supporting more than one million wal files at the minute. Current limit exceeded: 1000000" in str(err)


def test_bigger_record_than_max_file_size(tmp_path):
    a = new_appender(tmp_path)
    assert a.AppendSync(bytes(i % 255 for i in range(TestMaxWalFileSize + 5))) is None
    assert a.nextWriterNumber == 2  # the first WAL stays empty (header only)
    assert a.Close() is None


def test_replayer_on_file_fails(tmp_path):
    f = tmp_path / "afile"
    f.write_bytes(b"")
    opts, _ = W.NewWriteAheadLogOptions(W.BasePath(str(f)))
    r, err = W.NewReplayer(opts)
    assert r is None and str(err) == f"given base path {f} is not a directory"


def test_replayer_folder_does_not_exist():
    opts, _ = W.NewWriteAheadLogOptions(W.BasePath("somepaththathopefullydoesnotexistanywhere"))
    r, err = W.NewReplayer(opts)
    assert r is None and isinstance(err, GoError)


def test_cleaner_removes_folder(tmp_path):
    a = new_appender(tmp_path)
    assert a.Append(b"x") is None and a.Close() is None
    assert W.NewCleaner(a.walOptions).Clean() is None
    assert not os.path.exists(a.walOptions.basePath)
    assert W.NewCleaner(a.walOptions).Clean() is None  # os.RemoveAll of a missing path is nil


def test_wal_file_walk_is_sorted_and_filtered(tmp_path):
    base = tmp_path / "w"
    (base / "sub").mkdir(parents=True)
    for p in ("000002.wal", "000000.wal", "000001.wal", "sub/000000.wal", "some-not-so-wal-file", "x.wal.bak"):
        (base / p).write_bytes(b"")
    got = [os.path.relpath(p, base) for p in W._wal_files(str(base))]
    assert got == ["000000.wal", "000001.wal", "000002.wal", "sub/000000.wal"]
