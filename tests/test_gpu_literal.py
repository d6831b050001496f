"""Snappy files of single-literal records (GPU): golang/snappy emits an incompressible record as
one literal element, and k_place routes a file whose every record is such to k_snappy_literal (a
cooperative copy) instead of the lane-per-record decoder. Output must match the oracle's
FileReader loop either way, including the literal-header length boundaries (1, 2, 3 bytes: lengths
60 / 61 and 256 / 257), nil and empty records, and a single compressible record that sends the whole
file back to k_snappy_pipe."""
import random

import numpy as np
import pytest

import corpus
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


def _literal_stream(data: bytes, nb: int) -> bytes:
    """A Snappy stream that is one literal element: the decoded-length preamble, then the literal's tag with
    nb extra length bytes (0: the 1-byte form, lengths 1..60; 1..4: tag values 60..63, which golang/snappy's
    decoder accepts for any length they can hold, canonical or not), then the bytes."""
    n = len(data)
    tag = bytes([(n - 1) << 2]) if nb == 0 else bytes([(59 + nb) << 2]) + (n - 1).to_bytes(nb, "little")
    return corpus.uvarint(n) + tag + data


def test_non_canonical_literal_headers_take_the_copy():
    """Single-literal records whose literal header is 1..5 bytes for lengths that need fewer (a writer other
    than golang/snappy's): the copy path takes each record's header length from its sizes (stream length -
    record length), so every form must land the same bytes as the oracle's decoder."""
    rng = random.Random(11)
    out = bytearray(corpus.file_header(4, 2))
    for i in range(3000):
        if i % 97 == 13:
            out += corpus.header_for(4, 0, 1, nil=True)
            continue
        if i % 89 == 7:
            pay = corpus.uvarint(0)  # an empty record: the preamble alone
            out += corpus.header_for(4, 0, len(pay)) + pay
            continue
        n = rng.randint(1, 60) if i % 3 == 0 else rng.randint(61, 3000)
        nb = rng.choice([k for k in (0, 1, 2, 3, 4) if (k == 0 and n <= 60) or (k > 0 and n - 1 < 256 ** k)])
        pay = _literal_stream(rand_bytes(rng, n), nb)
        out += corpus.header_for(4, n, len(pay)) + pay
    img = bytes(out)
    g = gpu_decode_arrays(np.frombuffer(img, dtype=np.uint8))
    o = orc.file_reader_decode_arrays(img)
    assert_same_as_oracle(g, o)
    assert g["n_records"] == 3000
