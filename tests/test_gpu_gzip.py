"""gzip-compressed recordio (compType 1) decoded on the device vs the oracle (GPU).

GzipCompressor.DecompressWithBuf (recordio/compressor/gzip_compression.go:54-69) per record inside
the FileReader.ReadNext loop (file_reader.go:61-131): the device path must deliver the same
records, offsets, nil flags, terminal status and status offset as the oracle, including records
of several gzip members (gzip.Reader is multistream: their outputs concatenate). Inputs marked
may_fall_back are ones the device path may hand back to the reference reader (RIO_ERR_UNSUPPORTED);
then the records before the hand-back must still match exactly.
"""
import numpy as np
import pytest

import corpus
import oracle_py as orc
from conftest import STATUS
from gpu_util import assert_same_as_oracle, gpu_decode_arrays

pytestmark = pytest.mark.gpu

CASES = corpus.gzip_cases()


@pytest.mark.parametrize("name,image,may", CASES, ids=[c[0] for c in CASES])
def test_gzip_whole_file(name, image, may):
    o = orc.file_reader_decode_arrays(image)
    g = gpu_decode_arrays(image)
    if may and g["status"] == STATUS["UNSUPPORTED"]:
        n = g["n_records"]
        assert n <= o["n_records"], name
        np.testing.assert_array_equal(g["rec_off"][:n], o["rec_off"][:n])
        np.testing.assert_array_equal(g["out_off"][:n + 1], o["out_off"][:n + 1])
        nb = int(g["out_off"][n])
        assert np.array_equal(g["out"][:nb], o["out"][:nb]), name
        return
    assert g["status"] != STATUS["UNSUPPORTED"], name
    assert_same_as_oracle(g, o, name)


@pytest.mark.parametrize("n,ln,kind", [(3000, 1024, 1), (500, 4096, 1), (300, 700, 0), (40, 70000, 1)])
def test_gzip_generated_workload(n, ln, kind):
    """rio_generate's gzip files (zlib, one member per record), text-like and random."""
    from recordio import generate

    img = generate(n, ln, 1, kind=kind, seed=3)
    o = orc.file_reader_decode_arrays(img)
    g = gpu_decode_arrays(img)
    assert o["n_records"] == n
    assert_same_as_oracle(g, o, f"gen {n}x{ln} kind {kind}")


MULTI = [c for c in CASES if any(k in c[0] for k in ("multi", "member", "trailing"))]


@pytest.mark.parametrize("name,image,may", MULTI, ids=[c[0] for c in MULTI])
def test_gzip_multi_member_host_api(name, image, may):
    """The cgo pair (rio_frame + rio_decode): the sizes rio_frame returns are the decoded ones, so a
    caller that allocates from them gets every record of several members whole."""
    import ctypes

    from recordio import _lib as L
    from test_gpu_threads import host_decode

    h = ctypes.c_void_p()
    assert L.lib().rio_ctx_create(0, ctypes.byref(h)) == 0
    try:
        g = host_decode(h.value, np.frombuffer(image, dtype=np.uint8))
    finally:
        L.lib().rio_ctx_destroy(h)
    assert_same_as_oracle(g, orc.file_reader_decode_arrays(image), name)


def _multi_file(n, seed, parts=3):
    recs = corpus.text_records(n, seed, 1, 6000)
    cuts = [sorted({len(r) * k // parts for k in range(1, parts)} - {0}) for r in recs]
    return corpus.gz_file([(len(r), corpus.gzip_members(r, c)) for r, c in zip(recs, cuts)]), recs


def test_gzip_multi_member_workload_all_paths(tmp_path):
    """3000 records of 1-3 members (every window class): device API, FileReader.ReadNext (whole
    file and 64 KiB windows), MMapReader.ReadNextAt at every record start: the source records."""
    from recordio import NewFileReaderWithPath, NewMemoryMappedReaderWithPath
    from recordio.reader import FileReader

    img, recs = _multi_file(3000, 21)
    g = gpu_decode_arrays(img)
    o = orc.file_reader_decode_arrays(img)
    assert o["n_records"] == 3000 and o["n_bad"] == 0
    assert_same_as_oracle(g, o, "multi workload")
    for k in (0, 1, 1500, 2999):
        assert bytes(g["out"][g["out_off"][k]:g["out_off"][k + 1]]) == recs[k]
    path = tmp_path / "multi.rio"
    path.write_bytes(img)
    for window in (None, 65536):
        r = FileReader(str(path), window_bytes=window) if window else NewFileReaderWithPath(str(path))[0]
        assert r.Open() is None
        for k in range(3000):
            data, err = r.ReadNext()
            assert err is None and data == recs[k], (window, k)
        _, err = r.ReadNext()
        assert err is not None
        r.Close()
    m, err = NewMemoryMappedReaderWithPath(str(path))
    assert err is None and m.Open() is None
    for k in range(0, 3000, 7):
        data, err = m.ReadNextAt(int(o["rec_off"][k]))
        assert err is None and data == recs[k], k
    m.Close()


def test_gzip_multi_member_batch():
    """rio_device_decode_batch: files with records of several members beside single-member files."""
    from recordio.device import to_device_file
    from gpu_util import decoder

    imgs = [_multi_file(400, 30 + k)[0] for k in range(3)] + [corpus.gzip_cases()[0][1]]
    got = decoder().decode_batch([to_device_file(i) for i in imgs])
    for k, (img, (b, info)) in enumerate(zip(imgs, got)):
        n, nb = info["n_records"], info["total_out_bytes"]
        g = dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:n + 1].cpu().numpy(),
                 rec_off=b.rec_off[:n].cpu().numpy(), flags=b.flags[:n].cpu().numpy())
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), f"batch {k}")


@pytest.mark.parametrize("name,image,k,go_ok", corpus.gzip_go_header_cases(), ids=lambda v: v if isinstance(v, str) else "")
def test_gzip_go_header_rules(name, image, k, go_ok):
    """Member headers on which Go's readHeader and zlib's wrapper disagree (reserved FLG bits, names
    and comments of 512+ bytes): the device and the Go-faithful oracle agree record by record."""
    g = gpu_decode_arrays(image)
    assert_same_as_oracle(g, orc.file_reader_decode_arrays(image), name)
    assert bool(g["flags"][k] & 2) == (not go_ok), name
