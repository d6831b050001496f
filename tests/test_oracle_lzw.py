"""LZW restatement in the oracle (Go compress/lzw, LSB, litWidth 8 — LzwCompressor,
recordio/compressor/lzw_compressor.go:9-63), pinned two ways:

* the reference's own size KAT (lzw_compessor_test.go:9-16: "some data" compresses to 13 bytes,
  which fixes the writer's leading clear code) and its round trips;
* an independent decoder and encoder of the same code stream: GIF image data is variable-length
  LZW, LSB first, with 8-bit literals (clear 256, end 257, widths 9..12, no early change), which is
  exactly lzw.LSB / litWidth 8. Pillow's GIF codec (C, not derived from Go) decodes what our
  writer produces, and our reader decodes what Pillow's writer produces.
"""
import io
import random
import struct

import pytest

import oracle_py as orc
from corpus import text_records

PIL = pytest.importorskip("PIL.Image")

DECOMPRESS = 10


def gif_wrap(lzw: bytes, n: int) -> bytes:
    """A 1-row 8-bit GIF whose image data is the raw LZW stream `lzw` (n pixels)."""
    pal = bytes(range(256)) * 3
    out = [b"GIF89a", struct.pack("<HHBBB", n, 1, 0xF7, 0, 0), pal,
           b"\x2c", struct.pack("<HHHHB", 0, 0, n, 1, 0), b"\x08"]
    for i in range(0, len(lzw), 255):
        blk = lzw[i:i + 255]
        out += [bytes([len(blk)]), blk]
    out += [b"\x00", b"\x3b"]
    return b"".join(out)


def gif_unwrap(gif: bytes) -> bytes:
    """The raw LZW stream of the first image of a GIF (min code size must be 8)."""
    flags = gif[10]
    p = 13 + (3 << ((flags & 7) + 1) if flags & 0x80 else 0)
    while gif[p] == 0x21:  # extension blocks
        p += 2
        while gif[p]:
            p += gif[p] + 1
        p += 1
    assert gif[p] == 0x2C
    lf = gif[p + 9]
    p += 10 + (3 << ((lf & 7) + 1) if lf & 0x80 else 0)
    assert gif[p] == 8, "8-bit literals"
    p += 1
    data = []
    while gif[p]:
        data.append(gif[p + 1:p + 1 + gif[p]])
        p += gif[p] + 1
    return b"".join(data)


def pil_decode(lzw: bytes, n: int) -> bytes:
    im = PIL.open(io.BytesIO(gif_wrap(lzw, n)))
    im.load()
    return im.tobytes()


def pil_encode(data: bytes) -> bytes:
    im = PIL.frombytes("P", (len(data), 1), data)
    im.putpalette(list(range(256)) * 3)
    buf = io.BytesIO()
    im.save(buf, "GIF", optimize=False)
    return gif_unwrap(buf.getvalue())


def payloads():
    rnd = random.Random(11)
    text = text_records(40, 5, 1, 3000)
    return [
        b"", b"a", b"ab", b"some data", bytes(range(256)), b"a" * 5000, b"ab" * 3000,
        bytes(rnd.randrange(256) for _ in range(20000)),  # > 3838 codes: the writer's clear code
        bytes(rnd.randrange(4) for _ in range(30000)),
        b"".join(text), *text[:10],
    ]


def test_size_kat_some_data():
    # lzw_compessor_test.go:9-16 (and the three WithBuf variants, :19-50): 13 bytes
    c = orc.lzw_encode(b"some data")
    assert len(c) == 13
    assert orc.lzw_decode(c) == (0, b"some data")


def test_empty_record_is_clear_then_eof():
    c = orc.lzw_encode(b"")
    assert c == bytes([0x00, 0x03, 0x02])  # codes 256, 257 at 9 bits, LSB first
    assert orc.lzw_decode(c) == (0, b"")


@pytest.mark.parametrize("i", range(len(payloads())))
def test_round_trip(i):
    data = payloads()[i]
    c = orc.lzw_encode(data)
    assert orc.lzw_decode(c) == (0, data)


@pytest.mark.parametrize("i", range(len(payloads())))
def test_independent_decoder_reads_our_stream(i):
    data = payloads()[i]
    if not 0 < len(data) <= 65535:
        pytest.skip("GIF width")
    assert pil_decode(orc.lzw_encode(data), len(data)) == data


@pytest.mark.parametrize("i", range(len(payloads())))
def test_we_read_the_independent_encoders_stream(i):
    data = payloads()[i]
    if not 0 < len(data) <= 65535:
        pytest.skip("GIF width")
    assert orc.lzw_decode(pil_encode(data)) == (0, data)


def test_reader_errors():
    c = orc.lzw_encode(b"hello hello hello")
    assert orc.lzw_decode(b"")[0] == DECOMPRESS              # io.ErrUnexpectedEOF
    assert orc.lzw_decode(c[:-2])[0] == DECOMPRESS           # no eof code
    assert orc.lzw_decode(bytes([0x00, 0x5E, 0x04]))[0] == DECOMPRESS  # clear, then code 300 > hi
    assert orc.lzw_decode(bytes([0x02, 0x02]))[0] == DECOMPRESS  # first code 258 > hi (no clear)
    assert orc.lzw_decode(c + b"\xff\xff") == (0, b"hello hello hello")  # bytes after eof ignored
    # no leading clear: a bare literal stream is valid for the reader
    assert orc.lzw_decode(bytes([0x61, 0x02, 0x02]))[0] == 0


def test_file_reader_lzw_records():
    recs = [b"", None, b"some data", *text_records(30, 9, 1, 4000), b"z" * 9000]
    img, roff = orc.encode_file(recs, 3)
    r = orc.file_reader_decode(img)
    assert r["compression"] == 3 and r["n_records"] == len(recs)
    assert r["records"] == recs and r["rec_off"] == roff
    assert r["status"] == 1  # io.EOF at the clean end
