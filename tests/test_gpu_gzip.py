"""gzip-compressed recordio (compType 1) decoded on the device vs the oracle (GPU).

GzipCompressor.DecompressWithBuf (recordio/compressor/gzip_compression.go:54-69) per record inside
the FileReader.ReadNext loop (file_reader.go:61-131): the device path must deliver the same
records, offsets, nil flags, terminal status and status offset as the oracle. Inputs marked
may_fall_back are ones the device path may hand back to the reference reader
(RIO_ERR_UNSUPPORTED: a record with more than one gzip member, or one decoding past the small
window); then the records before the hand-back must still match exactly.
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
