"""Expected Go error shapes of the reference's MMapReader, restated from its source (test helper).

For a status class the oracle reports, `expect_read_next_at` / `expect_seek_next` give the error
value MMapReader.ReadNextAt / SeekNext return: its full message, the sentinel `errors.Is` finds, and
how many `fmt.Errorf("...: %w")` wraps sit above that sentinel. The table follows the reference
(recordio/mmap_reader.go:58-203, common_reader.go:110-151, x/exp/mmap ReadAt), not the Python
mirror, so a test that compares the mirror's error with it checks the mirror's mapping too.
"""
from recordio import (EOF, ErrCorrupt, ErrUnexpectedEOF, ErrVarintOverflow, HeaderChecksumMismatchErr,
                      MagicNumberMismatchErr)
from recordio import _lib as L

# status -> (sentinel, message of the innermost error) for errors raised by readRecordHeaderV4/V3
_HEADER = {
    L.RIO_EOF_HEADER: (EOF, "EOF"),
    L.RIO_ERR_UNEXPECTED_EOF: (ErrUnexpectedEOF, "unexpected EOF"),
    L.RIO_ERR_MAGIC: (MagicNumberMismatchErr, "magic number mismatch"),
    L.RIO_ERR_VARINT_OVERFLOW: (ErrVarintOverflow, "binary: varint overflows a 64-bit integer"),
    L.RIO_ERR_HEADER_TOO_LONG: (None, "checksum byte reader out of range: 36, only have 36"),
}


def expect_read_next_at(status: int, offset: int, path: str, d0: int = 0, d1: int = 0, version: int = 4):
    """(message, sentinel or None, wraps above the sentinel) of MMapReader.ReadNextAt's error
    (readNextAtV2 / V1 for version 2 / 1: mmap_reader.go:205-296)."""
    where = f"at offset {offset} in mmap reader for '{path}'"
    if status == L.RIO_EOF:  # mmap_reader.go:150-155: 0 bytes readable -> bare io.EOF
        return "EOF", EOF, 0
    if status == L.RIO_ERR_INVALID_OFFSET:  # :156-158 wraps x/exp/mmap's error (v1 / v2: :211, :256)
        pre = "ReadNextAt failed reading" if version >= 3 else "failed reading"
        return f"{pre} {where}: mmap: invalid ReadAt offset {offset}", None, 1
    if status == L.RIO_EOF_HEADER and version == 1:  # :209-212: the 20-byte ReadAt ran short
        return f"failed reading {where}: EOF", EOF, 1
    if status == L.RIO_ERR_HEADER_CRC:  # common_reader.go:145-147 wraps the sentinel once more
        inner = f"header checksum mismatch: expected [{d0:x}], but found [{d1:x}]"
        return f"failed reading record header {where}: {inner}", HeaderChecksumMismatchErr, 2
    if status in _HEADER:  # :163-166
        sentinel, inner = _HEADER[status]
        return f"failed reading record header {where}: {inner}", sentinel, 1
    if status == L.RIO_EOF_PAYLOAD:  # :175-178: the payload ReadAt came back short (io.EOF)
        return f"failed reading record {where}: EOF", EOF, 1
    if status == L.RIO_ERR_DECOMPRESS:  # :189-191
        return f"failed decompressing record {where}: snappy: corrupt input", ErrCorrupt, 1
    if status == L.RIO_EOF_CODEC:  # :189-191 around gzip.NewReader's io.EOF (empty payload)
        return f"failed decompressing record {where}: EOF", EOF, 1
    raise AssertionError(f"status {status} is not a ReadNextAt error")


def expect_seek_next(status: int, offset: int, trial: int, path: str, version: int = 4):
    """SeekNext's error (mmap_reader.go:58-128): io.EOF and x/exp/mmap's ReadAt error come back
    unwrapped; anything else is the failing trial ReadNextAt's error at the trial offset."""
    if status == L.RIO_EOF:
        return "EOF", EOF, 0
    if status == L.RIO_ERR_INVALID_OFFSET:  # :70-83: ReadAt's own error, returned as is
        return f"mmap: invalid ReadAt offset {offset}", None, 0
    return expect_read_next_at(status, trial, path, version=version)


def wraps_above(err, sentinel) -> int:
    """Number of wrapping layers above `sentinel` in err's chain (-1 if absent)."""
    k = 0
    while err is not None:
        if err is sentinel:
            return k
        err = getattr(err, "wrapped", None)
        k += 1
    return -1


def depth(err) -> int:
    k = 0
    while getattr(err, "wrapped", None) is not None:
        err = err.wrapped
        k += 1
    return k


def assert_go_error(err, want):
    msg, sentinel, wraps = want
    assert err is not None, want
    assert str(err) == msg, (str(err), msg)
    if sentinel is not None:
        assert wraps_above(err, sentinel) == wraps, (str(err), wraps)
    else:
        assert depth(err) == wraps, (str(err), wraps)
