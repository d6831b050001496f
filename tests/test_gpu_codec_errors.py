"""Records that do not decompress, through the ReaderI mirror and the C-ABI (GPU).

FileReader.ReadNext consumes a record's payload before the codec runs (file_reader.go:101-125 v4,
418-446 v3), so a payload that does not decompress fails that one call: ReadNext returns the codec
error unwrapped (snappy.ErrCorrupt, the gzip reader's error, or gzip.NewReader's bare io.EOF for an
empty payload) and the next call reads the record after it. SkipNext never decompresses
(:133-172) and passes over such a record without error. The expected call sequence is restated
here from the oracle's per-record flags (oracle/rio_oracle.c orc_file_reader_decode).
"""
import pytest

import corpus
import oracle_py as orc
from recordio import EOF, ErrCorrupt, FileReader
from recordio.errors import errors_is

pytestmark = pytest.mark.gpu

CASES = dict(corpus.cases())
GZ = {n: img for n, img, may in corpus.gzip_cases() if not may}
NAMES = ["snappy_corrupt_mid", "snappy_bad_preamble_mid", "snappy_short_mid", "snappy_long_mid",
         "snappy_empty_mid", "snappy_huge_preamble"]
GZ_NAMES = ["gz_bad_hcrc", "gz_bad_magic", "gz_bad_crc", "gz_isize_plus1", "gz_btype3", "gz_empty_payload"]
NEVER = (1 << 64) - 1


def _image(name):
    return CASES[name] if name in CASES else GZ[name]


def expected_calls(img, skip_every=0):
    """The reference's (value, error class) per call until the terminal error, restated from the
    oracle: bytes / None for a record, "corrupt" / "eof" for a codec failure, "skip" for SkipNext."""
    o = orc.file_reader_decode(img)
    out = []
    for i, rec in enumerate(o["records"]):
        if skip_every and i % skip_every == 1:
            out.append("skip")
        elif isinstance(rec, orc.BadRecord):
            out.append(rec.kind)
        else:
            out.append(rec)
    return out, o


def run_reader(path, n, window, skip_every=0):
    r = FileReader(path, 0, window)
    assert r.Open() is None
    got = []
    for i in range(n):
        if skip_every and i % skip_every == 1:
            assert r.SkipNext() is None, i
            got.append("skip")
            continue
        rec, err = r.ReadNext()
        if err is None:
            got.append(rec)
        elif err is ErrCorrupt:  # returned as is, no wrapping (file_reader.go:119-122)
            got.append("corrupt")
        elif err is EOF:  # gzip's bare io.EOF
            got.append("eof")
        else:
            raise AssertionError((i, str(err)))
    rec, err = r.ReadNext()  # then the file's own end
    assert rec is None and errors_is(err, EOF) and err is not EOF, str(err)
    r.Close()
    return got


@pytest.mark.parametrize("name", NAMES + GZ_NAMES)
@pytest.mark.parametrize("window", [NEVER, 700])
@pytest.mark.parametrize("skip_every", [0, 2])
def test_read_next_goes_on_after_a_codec_failure(name, window, skip_every, tmp_path):
    img = _image(name)
    want, o = expected_calls(img, skip_every)
    assert o["n_bad"] > 0
    p = tmp_path / "f.rio"
    p.write_bytes(img)
    assert run_reader(str(p), len(want), window, skip_every) == want


@pytest.mark.parametrize("name", NAMES + GZ_NAMES)
def test_file_info_counts_flagged_records(name, tmp_path):
    img = _image(name)
    o = orc.file_reader_decode(img)
    p = tmp_path / "f.rio"
    p.write_bytes(img)
    r = FileReader(str(p))
    assert r.Open() is None
    r.ReadNext()
    fi = r.FileInfo()
    assert (fi["first_bad"], fi["n_bad"], fi["n_records"]) == (o["first_bad"], o["n_bad"], o["n_records"])


def test_many_failing_records_in_one_file():
    """More failing lanes than the decoder's fail list holds (rio_device.h kFailLanes): every third
    record of 12000 is corrupt; the decode re-verifies all and flags exactly the oracle's."""
    from gpu_util import assert_same_as_oracle, gpu_decode_arrays

    lit = b"\xf0\x9f" + bytes(range(160))
    good = corpus.encode_file([bytes((i * 7 + j) & 0xFF for j in range(50 + i % 90)) for i in range(2)], 2)[8:]
    pay = corpus.uvarint(170) + lit
    bad = corpus.header_v4(160, len(pay)) + pay
    img = corpus.encode_file([], 2) + (good + bad) * 6000
    o = orc.file_reader_decode_arrays(img)
    assert o["n_bad"] == 6000
    assert_same_as_oracle(gpu_decode_arrays(img), o, "many bad")
