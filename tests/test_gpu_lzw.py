"""lzw-compressed recordio (compType 3) decoded on the device vs the oracle (GPU).

LzwCompressor.DecompressWithBuf (recordio/compressor/lzw_compressor.go:52-63: Go compress/lzw, LSB,
litWidth 8) per record inside the FileReader.ReadNext loop (file_reader.go:61-131): the device path
(k_lzw_decode, rio_lzw.hip) must deliver the same records, offsets, flags, terminal status and status
offset as the oracle's restatement of Go's reader (tests/test_oracle_lzw.py pins it). Covered: code
width steps and the writer's clear code, KwKwK chains, large records, nil / empty records, v3 files,
streams Go's writer never produces (no leading clear, double clears, bytes after eof), invalid /
truncated / empty payloads in the middle of a file, and headers whose u is not the decoded length
(the resize round).
"""
import numpy as np
import pytest

import corpus
import oracle_py as orc
from conftest import STATUS
from gpu_util import assert_same_as_oracle, gpu_decode_arrays

pytestmark = pytest.mark.gpu

CASES = corpus.lzw_cases()


@pytest.mark.parametrize("name,image", CASES, ids=[c[0] for c in CASES])
def test_lzw_whole_file(name, image):
    o = orc.file_reader_decode_arrays(image)
    g = gpu_decode_arrays(image)
    assert g["status"] != STATUS["UNSUPPORTED"], name
    assert_same_as_oracle(g, o, name)


def _text_file(n, seed, lo=1, hi=2048):
    recs = corpus.text_records(n, seed, lo, hi)
    img, _ = orc.encode_file(recs, 3)
    return img, recs


@pytest.mark.parametrize("n,lo,hi", [(3000, 1024, 1024), (2000, 1, 4096), (40, 60000, 70000)])
def test_lzw_generated_workload(n, lo, hi):
    img, recs = _text_file(n, 5 + n, lo, hi)
    o = orc.file_reader_decode_arrays(img)
    assert o["n_records"] == n and o["n_bad"] == 0
    g = gpu_decode_arrays(img)
    assert_same_as_oracle(g, o, f"lzw gen {n}")
    for k in (0, n // 2, n - 1):
        assert bytes(g["out"][g["out_off"][k]:g["out_off"][k + 1]]) == recs[k]


@pytest.mark.parametrize("name,image", [c for c in CASES if "u_" in c[0] or "clear" in c[0]],
                         ids=[c[0] for c in CASES if "u_" in c[0] or "clear" in c[0]])
def test_lzw_host_api_sizes(name, image):
    """The cgo pair (rio_frame + rio_decode): rio_frame returns the decoded sizes even where the
    header's u says otherwise, so a caller that allocates from them gets every record whole."""
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


def test_lzw_readers(tmp_path):
    """FileReader.ReadNext (whole file and 64 KiB windows), MMapReader.ReadNextAt at record starts and
    SeekNext chains over an lzw file with a corrupt record in the middle."""
    from recordio import NewFileReaderWithPath, NewMemoryMappedReaderWithPath
    from recordio.reader import FileReader

    recs = corpus.text_records(600, 41, 1, 3000)
    items = [(len(r), orc.lzw_encode(r)) for r in recs]
    items[300] = (len(recs[300]), items[300][1][:-3])  # truncated: io.ErrUnexpectedEOF
    img = corpus.lzw_file(items)
    o = orc.file_reader_decode_arrays(img)
    assert o["n_bad"] == 1 and o["first_bad"] == 300
    path = tmp_path / "f.rio"
    path.write_bytes(img)
    for window in (None, 65536):
        r = FileReader(str(path), window_bytes=window) if window else NewFileReaderWithPath(str(path))[0]
        assert r.Open() is None
        for k in range(600):
            data, err = r.ReadNext()
            if k == 300:
                assert err is not None and data is None, (window, k)
            else:
                assert err is None and data == recs[k], (window, k)
        _, err = r.ReadNext()
        assert err is not None
        r.Close()
    m, err = NewMemoryMappedReaderWithPath(str(path))
    assert err is None and m.Open() is None
    for k in range(0, 600, 3):
        data, err = m.ReadNextAt(int(o["rec_off"][k]))
        if k == 300:
            assert err is not None and data is None
        else:
            assert err is None and data == recs[k], k
    off, k = 0, 0
    while k < 300:  # SeekNext chain from the file start up to the corrupt record
        at, data, err = m.SeekNext(off)
        assert err is None and at == int(o["rec_off"][k]) and data == recs[k], k
        off, k = at + 1, k + 1
    at, data, err = m.SeekNext(off)
    assert err is not None
    m.Close()


def test_lzw_batch():
    """rio_device_decode_batch: lzw files beside snappy and gzip ones."""
    from recordio.device import to_device_file
    from gpu_util import decoder

    imgs = [_text_file(300, 60 + k)[0] for k in range(3)] + [CASES[0][1], dict(corpus.lzw_cases())["lzw_u_small"],
                                                             corpus.gzip_cases()[0][1]]
    got = decoder().decode_batch([to_device_file(i) for i in imgs])
    for k, (img, (b, info)) in enumerate(zip(imgs, got)):
        n, nb = info["n_records"], info["total_out_bytes"]
        g = dict(info, out=b.out[:nb].cpu().numpy(), out_off=b.out_off[:n + 1].cpu().numpy(),
                 rec_off=b.rec_off[:n].cpu().numpy(), flags=b.flags[:n].cpu().numpy())
        assert_same_as_oracle(g, orc.file_reader_decode_arrays(img), f"batch {k}")
