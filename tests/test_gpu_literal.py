"""Snappy files of single-literal records (GPU): golang/snappy emits an incompressible record as
one literal element, and k_place routes a file whose every record is such to k_snappy_literal (a
cooperative copy) instead of the lane-per-record decoder. Output must match the oracle's
FileReader loop either way, including the literal-header length boundaries (1, 2, 3 bytes: lengths
60 / 61 and 256 / 257), nil and empty records, and a single compressible record that sends the whole
file back to k_snappy_pipe."""
import random

import numpy as np
import pytest

import oracle_py as orc
from gpu_util import assert_same_as_oracle, gpu_decode_arrays
from recordio import encode_file

pytestmark = pytest.mark.gpu


def rand_bytes(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def check(recs):
    img = encode_file(recs, 2)
    g = gpu_decode_arrays(np.frombuffer(img, dtype=np.uint8))
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o)
    return g


@pytest.mark.parametrize("sizes", [
    [0, 1, 2, 15, 16, 17, 59, 60, 61, 62, 255, 256, 257, 1023, 1024, 4096, 65535, 65536],
    [1024] * 3000,
])
def test_all_literal_files(sizes):
    rng = random.Random(len(sizes))
    check([rand_bytes(rng, n) for n in sizes])


def test_all_literal_with_nil_and_empty():
    rng = random.Random(7)
    recs = [None if i % 7 == 3 else (b"" if i % 11 == 5 else rand_bytes(rng, rng.randint(1, 3000)))
            for i in range(2000)]
    check(recs)


@pytest.mark.parametrize("where", [0, 777, 1999])
def test_one_compressible_record_uses_the_decoder(where):
    rng = random.Random(where)
    recs = [rand_bytes(rng, 900) for _ in range(2000)]
    recs[where] = b"abcd" * 200
    check(recs)


def test_multi_block_literal_is_not_single():
    rng = random.Random(9)
    check([rand_bytes(rng, 70000), rand_bytes(rng, 200000), rand_bytes(rng, 10)])
