"""Snappy element streams built by hand to cover the lane decoder's byte placement (GPU).

The decoder places every piece destination-aligned (bytes [d - r, d - r + 16), r = d & 3) and reads
its source from q - r: ring copies from the LDS history, literals from the input image, far copies
(offset > 192) from the arena, and far copies whose source starts in the first bytes of the arena
from q itself (the lane of a file's first record). These streams hit each source kind at every
destination alignment, overlapping copies of every short offset, long literals and copies at the
16-bit length / offset forms, against the oracle's golang/snappy restatement (decode_other.go).
"""
import random

import pytest

import corpus
import oracle_py as orc
from recordio import _lib as L
from gpu_util import assert_same_as_oracle, gpu_decode_arrays

pytestmark = pytest.mark.gpu


def lit(b: bytes) -> bytes:
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    if n < 256:
        return bytes([60 << 2, n]) + b
    return bytes([61 << 2, n & 0xFF, n >> 8]) + b


def copy(off: int, ln: int) -> bytes:
    if 4 <= ln <= 11 and off < 2048:
        return bytes([1 | ((ln - 4) << 2) | ((off >> 8) << 5), off & 0xFF])
    if off < 65536:
        return bytes([2 | ((ln - 1) << 2), off & 0xFF, off >> 8])
    return bytes([3 | ((ln - 1) << 2)]) + off.to_bytes(4, "little")


class Stream:
    """A snappy block built element by element, with the decoded bytes kept to size copies."""

    def __init__(self):
        self.els = bytearray()
        self.out = bytearray()

    def literal(self, b: bytes):
        self.els += lit(b)
        self.out += b

    def copy(self, off: int, ln: int):
        assert 1 <= off <= len(self.out) and 1 <= ln <= 64
        self.els += copy(off, ln)
        for _ in range(ln):
            self.out.append(self.out[-off])

    def payload(self) -> bytes:
        return corpus.uvarint(len(self.out)) + bytes(self.els)


def file_of(streams) -> bytes:
    img = bytearray(corpus.file_header(4, 2))
    for st in streams:
        pay = st.payload()
        img += corpus.header_v4(len(st.out), len(pay)) + pay
    return bytes(img)


def far_from_start(rng) -> Stream:
    """Far copies (offset > 192) whose source is the record's byte 0, 1 or 2, at every destination
    alignment: as record 0 of a file, 16 bytes from q - r would start below the arena."""
    st = Stream()
    st.literal(bytes(rng.randrange(256) for _ in range(250)))
    for _ in range(60):
        st.literal(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 4))))  # move d & 3
        q = rng.randrange(3)
        st.copy(len(st.out) - q, rng.choice([4, 5, 11, 16, 17, 33, 64]))
    return st


def mixed(rng, n_el) -> Stream:
    st = Stream()
    st.literal(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 300))))
    for _ in range(n_el):
        k = rng.random()
        if k < 0.3:
            st.literal(bytes(rng.randrange(256) for _ in range(rng.choice([1, 2, 3, 5, 13, 15, 16, 17, 60, 61, 200, 300]))))
        elif k < 0.55:  # overlapping copies: every short offset
            off = rng.randrange(1, min(17, len(st.out)) + 1)
            st.copy(off, rng.randrange(1, 65))
        elif k < 0.85:  # ring copies
            off = rng.randrange(1, min(192, len(st.out)) + 1)
            st.copy(off, rng.randrange(1, 65))
        else:  # far copies, including 16-bit offsets
            if len(st.out) > 193:
                st.copy(rng.randrange(193, len(st.out) + 1), rng.randrange(1, 65))
    return st


def check(img):
    o = orc.file_reader_decode_arrays(img)
    assert o["status"] == L.RIO_EOF and o["n_bad"] == 0  # the streams are valid golang/snappy blocks
    assert_same_as_oracle(gpu_decode_arrays(img), o)


@pytest.mark.parametrize("seed", range(4))
def test_far_copy_from_the_arena_start(seed):
    rng = random.Random(seed)
    check(file_of([far_from_start(rng)] + [mixed(rng, 50) for _ in range(100)]))


@pytest.mark.parametrize("seed", range(4))
def test_every_alignment_and_source_kind(seed):
    rng = random.Random(100 + seed)
    check(file_of([mixed(rng, rng.randrange(0, 400)) for _ in range(300)]))


def test_long_records_with_far_copies():
    rng = random.Random(7)
    check(file_of([far_from_start(rng)] + [mixed(rng, 3000) for _ in range(40)]))


def mutated_file(rng, n_rec):
    """Valid streams (`mixed`) with seeded damage in about a third of the records, behind valid headers
    (the v4 header CRC covers the header only, so framing keeps every record): flipped element bytes,
    a wrong decoded-length preamble, a cut element stream, or a copy offset pushed past the bytes
    produced. Records are written with the damaged payload's own length, as a writer would."""
    img = bytearray(corpus.file_header(4, 2))
    for _ in range(n_rec):
        st = mixed(rng, rng.randrange(0, 300))
        pre, els = corpus.uvarint(len(st.out)), bytearray(st.els)
        k = rng.random()
        if k < 0.15 and els:  # flipped bytes anywhere in the element stream
            for _ in range(rng.randrange(1, 4)):
                els[rng.randrange(len(els))] ^= 1 << rng.randrange(8)
        elif k < 0.22:  # preamble one off, or far off
            pre = corpus.uvarint(max(0, len(st.out) + rng.choice([-1, 1, 7, -len(st.out), 1 << 20])))
        elif k < 0.30 and els:  # the stream cut inside its last elements
            del els[len(els) - rng.randrange(1, min(6, len(els)) + 1):]
        elif k < 0.35 and els:  # a 2-byte-offset copy reaching before the record start
            els += bytes([2 | (3 << 2)]) + (len(st.out) + 1 + rng.randrange(100)).to_bytes(2, "little")
        pay = pre + bytes(els)
        img += corpus.header_v4(len(st.out), len(pay)) + pay
    return bytes(img)


@pytest.mark.parametrize("seed", range(8))
def test_damaged_streams_match_golang_snappy(seed):
    """The lane decoder flags exactly the records golang/snappy's Decode rejects (decode_other.go:
    ErrCorrupt on a tag past the stream, a literal or copy past the output, offset 0 or beyond the
    bytes produced, a decoded length other than the preamble's), with identical bytes for the rest,
    and ReadNext's status sequence is the reference loop's."""
    rng = random.Random(1000 + seed)
    img = mutated_file(rng, 400)
    o = orc.file_reader_decode_arrays(img)
    assert o["n_bad"] > 0  # the damage reaches the codec
    assert_same_as_oracle(gpu_decode_arrays(img), o, f"seed {seed}")
