"""recordio.ReaderI / recordio.ReadAtI mirror over the device decode path (librio.so).

Same names, argument meaning and error behaviour as the reference:
  NewFileReader / NewFileReaderWithPath       recordio/file_reader.go:490-524
  FileReader.Open/ReadNext/SkipNext/Close     recordio/file_reader.go:26-172, 272-279
  NewMemoryMappedReaderWithPath               recordio/mmap_reader.go:364-371
  MMapReader.Open/Size/ReadNextAt/SeekNext    recordio/mmap_reader.go:25-203
Methods return Go-style `(value, err)` tuples (err is None on success). Decoding runs on the GPU
(a FileReader decodes the whole file on its first read); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_uint32, c_uint64, c_void_p

from . import _lib as L
from .errors import (EOF, ErrCorrupt, ErrUnexpectedEOF, ErrUnsupported, ErrVarintOverflow, GoError,
                     HeaderChecksumMismatchErr, MagicNumberMismatchErr, wrap)

CompressionTypeNone, CompressionTypeGZIP, CompressionTypeSnappy, CompressionTypeLzw = 0, 1, 2, 3
FileHeaderSizeBytes = 8


def _base_error(status: int, d0: int = 0, d1: int = 0) -> GoError:
    """The innermost error value the reference produces for a status class."""
    if status in (L.RIO_EOF, L.RIO_EOF_HEADER, L.RIO_EOF_PAYLOAD, L.RIO_EOF_ZERO_TAIL, L.RIO_EOF_CODEC):
        return EOF
    if status == L.RIO_ERR_UNEXPECTED_EOF:
        return ErrUnexpectedEOF
    if status == L.RIO_ERR_MAGIC:
        return MagicNumberMismatchErr
    if status == L.RIO_ERR_HEADER_CRC:
        # common_reader.go:145-147
        return GoError(f"header checksum mismatch: expected [{d0:x}], but found [{d1:x}]", HeaderChecksumMismatchErr)
    if status == L.RIO_ERR_VARINT_OVERFLOW:
        return ErrVarintOverflow
    if status == L.RIO_ERR_HEADER_TOO_LONG:
        return GoError("checksum byte reader out of range: 36, only have 36")
    if status == L.RIO_ERR_DECOMPRESS:
        return ErrCorrupt
    if status == L.RIO_ERR_UNSUPPORTED:
        return ErrUnsupported
    return GoError(L.strerror(status))


def _open_error(status: int, path: str, d0: int, what: str, size: int = -1) -> GoError:
    if status == L.RIO_ERR_VERSION:
        inner = GoError(f"version mismatch, expected a value from 1 to 4 but was {d0}")
    elif status == L.RIO_ERR_COMPRESSION_TYPE:
        inner = GoError(f"unknown compression type [{d0}]")
    elif status == L.RIO_ERR_SHORT_FILE_HEADER:
        # io.ReadFull of the 8 header bytes (file_reader.go:36-40): io.EOF when the file is empty
        return wrap(f"error while reading header bytes of '{path}'", EOF if size == 0 else ErrUnexpectedEOF)
    else:
        return GoError(f"{what}: {L.strerror(status)}")
    if what == "mmap":
        return wrap(f"failed reading header from buffer in mmap reader for '{path}'", inner)
    return wrap(f"error while parsing header of '{path}'", inner)


def read_next_error(rc: int, path: str, d0: int, d1: int, version: int = 4) -> GoError:
    """FileReader.ReadNext's error for a terminal status of the whole-file decode (file_reader.go:61-131;
    v1 files: readNextV1, :282-320)."""
    if version == 1:
        # io.ReadFull of the fixed 20-byte header, then readRecordHeaderV1; no zero-tail rule
        if rc in (L.RIO_EOF, L.RIO_ERR_UNEXPECTED_EOF) and d0 != 1:
            return wrap(f"error while reading record header of '{path}'", _base_error(rc))
        if rc == L.RIO_ERR_MAGIC:
            return wrap(f"error while parsing record header of '{path}'", MagicNumberMismatchErr)
        if rc in (L.RIO_ERR_DECOMPRESS, L.RIO_EOF_CODEC):  # :311-316 wraps the codec's error
            return wrap(f"error while decompressing record of '{path}'", ErrCorrupt if rc == L.RIO_ERR_DECOMPRESS else EOF)
    if rc in (L.RIO_EOF_ZERO_TAIL, L.RIO_EOF_CODEC):
        return EOF  # file_reader.go:89-90 (zero tail) / :119-121 (gzip's io.EOF): bare io.EOF
    if rc == L.RIO_ERR_MAGIC:
        return wrap(f"error while parsing record header for zeros towards the file end of '{path}'",
                    MagicNumberMismatchErr)
    # payload stage (io.ReadFull of the payload, file_reader.go:104-107): detail0 == 1 marks an
    # unexpected EOF raised there rather than inside a header varint
    if rc == L.RIO_EOF_PAYLOAD or (rc == L.RIO_ERR_UNEXPECTED_EOF and d0 == 1):
        return wrap(f"error while reading into record buffer of '{path}'", _base_error(rc))
    if rc == L.RIO_ERR_DECOMPRESS:
        return ErrCorrupt  # file_reader.go:119-122 returns the codec error unwrapped
    return wrap(f"error while parsing record header of '{path}'", _base_error(rc, d0, d1))


class _Reader:
    _mmap = False

    def __init__(self, path: str, device: int = 0):
        self.path = path
        self._device = device
        self._h = c_void_p()
        rc = L.lib().rio_reader_new_mmap(L.default_ctx(device), path.encode(), byref(self._h)) if self._mmap else \
            L.lib().rio_reader_new_file(L.default_ctx(device), path.encode(), byref(self._h))
        if rc != L.RIO_OK:
            raise FileNotFoundError(path)
        self.header = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            L.lib().rio_reader_free(h)
            self._h = None

    def _detail(self):
        d0, d1, off = c_uint64(), c_uint64(), c_uint64()
        L.lib().rio_reader_last_detail(self._h, byref(d0), byref(d1), byref(off))
        return d0.value, d1.value, off.value

    def Open(self):  # noqa: N802
        rc = L.lib().rio_reader_open(self._h)
        kind = "mmap reader" if self._mmap else "file reader"
        if rc == L.RIO_ERR_STATE:
            v, c = c_uint32(), c_uint32()
            opened = L.lib().rio_reader_header(self._h, byref(v), byref(c)) == L.RIO_OK
            return GoError(f"{kind} for '{self.path}' is already {'opened' if opened else 'closed'}")
        if rc != L.RIO_OK:
            d0, _, _ = self._detail()
            return _open_error(rc, self.path, d0, "mmap" if self._mmap else "file", self.Size())
        v, c = c_uint32(), c_uint32()
        L.lib().rio_reader_header(self._h, byref(v), byref(c))
        self.header = _Header(v.value, c.value)
        return None

    def Close(self):  # noqa: N802
        L.lib().rio_reader_close(self._h)
        return None

    def Size(self) -> int:  # noqa: N802
        return int(L.lib().rio_reader_size(self._h))


class _Header:
    def __init__(self, version, compression):
        self.fileVersion = version
        self.compressionType = compression


class FileReader(_Reader):
    """recordio.FileReader (ReaderI) backed by the device decode: the whole file at once, or, for
    files larger than `window_bytes` (default: files over 32 MiB in 128 MiB windows; ~0 = never),
    window by window (rio_stream_*), with the same records and errors."""

    def __init__(self, path: str, device: int = 0, window_bytes: int | None = None):
        super().__init__(path, device)
        if window_bytes is not None:
            L.lib().rio_reader_set_window(self._h, window_bytes)

    def _not_open(self):
        return GoError(f"file reader for '{self.path}' was either not opened yet or is closed already")

    def ReadNext(self):  # noqa: N802
        data, n, nil = c_void_p(), c_uint64(), c_int()
        rc = L.lib().rio_reader_read_next(self._h, byref(data), byref(n), byref(nil))
        if rc == L.RIO_OK:
            if nil.value:
                return None, None
            return (ctypes.string_at(data.value, n.value) if n.value else b""), None
        return None, self._read_error(rc)

    def SkipNext(self):  # noqa: N802
        rc = L.lib().rio_reader_skip_next(self._h)
        if rc == L.RIO_OK:
            return None
        if rc == L.RIO_ERR_STATE:
            return self._not_open()
        d0, d1, _ = self._detail()
        return wrap(f"error while reading record header of '{self.path}'", _base_error(rc, d0, d1))

    def _read_error(self, rc):
        if rc == L.RIO_ERR_STATE:
            return self._not_open()
        d0, d1, _ = self._detail()
        return read_next_error(rc, self.path, d0, d1, self.header.fileVersion if self.header else 4)

    def FileInfo(self):  # noqa: N802
        fi = L.FileInfo()
        rc = L.lib().rio_reader_file_info(self._h, byref(fi))
        return fi.as_dict() if rc == L.RIO_OK else None


class MMapReader(_Reader):
    """recordio.MMapReader (ReadAtI) backed by single-record device kernels."""

    _mmap = True

    def _not_open(self):
        return GoError(f"reader at '{self.path}' was either not opened yet or is closed already")

    def _err(self, rc, offset):
        if rc == L.RIO_ERR_STATE:
            return self._not_open()
        d0, d1, _ = self._detail()
        if rc == L.RIO_EOF:
            return EOF  # mmap_reader.go:153-155: bare io.EOF
        v = self.header.fileVersion if self.header else 4
        if rc == L.RIO_ERR_INVALID_OFFSET:  # v1 / v2: mmap_reader.go:211,256; v3 / v4: :157,312
            return wrap(f"{'ReadNextAt ' if v >= 3 else ''}failed reading at offset {offset} in mmap reader for "
                        f"'{self.path}'", GoError(f"mmap: invalid ReadAt offset {offset}"))
        if rc == L.RIO_EOF_HEADER and v == 1:  # readNextAtV1: the 20-byte ReadAt ran short (:209-212)
            return wrap(f"failed reading at offset {offset} in mmap reader for '{self.path}'", EOF)
        if rc == L.RIO_EOF_PAYLOAD:
            return wrap(f"failed reading record at offset {offset} in mmap reader for '{self.path}'", EOF)
        if rc in (L.RIO_ERR_DECOMPRESS, L.RIO_EOF_CODEC):  # mmap_reader.go:189-191
            return wrap(f"failed decompressing record at offset {offset} in mmap reader for '{self.path}'",
                        ErrCorrupt if rc == L.RIO_ERR_DECOMPRESS else EOF)
        return wrap(f"failed reading record header at offset {offset} in mmap reader for '{self.path}'",
                    _base_error(rc, d0, d1))

    def ReadNextAt(self, offset: int):  # noqa: N802
        data, n, nil = c_void_p(), c_uint64(), c_int()
        rc = L.lib().rio_reader_read_next_at(self._h, offset, byref(data), byref(n), byref(nil))
        if rc != L.RIO_OK:
            return None, self._err(rc, offset)
        if nil.value:
            return None, None
        return (ctypes.string_at(data.value, n.value) if n.value else b""), None

    def SeekNext(self, offset: int):  # noqa: N802
        data, n, nil, ro = c_void_p(), c_uint64(), c_int(), c_uint64()
        rc = L.lib().rio_reader_seek_next(self._h, offset, byref(ro), byref(data), byref(n), byref(nil))
        if rc != L.RIO_OK:
            if rc == L.RIO_EOF:
                return 0, None, EOF
            if rc == L.RIO_ERR_UNSUPPORTED:
                return 0, None, GoError("unsupported on files with version lower than v2")
            if rc == L.RIO_ERR_INVALID_OFFSET:  # mmap_reader.go:70-83: ReadAt's error, unwrapped
                return 0, None, GoError(f"mmap: invalid ReadAt offset {offset}")
            # any other error is the failing trial ReadNextAt's, at the trial offset (:105-114)
            return 0, None, self._err(rc, ro.value)
        if nil.value:
            return ro.value, None, None
        return ro.value, (ctypes.string_at(data.value, n.value) if n.value else b""), None

    @property
    def seekLen(self):  # noqa: N802
        return self._seek_len if hasattr(self, "_seek_len") else 4096

    @seekLen.setter
    def seekLen(self, v):  # noqa: N802
        self._seek_len = v
        L.lib().rio_reader_set_seek_len(self._h, v)


def NewFileReaderWithPath(path: str, device: int = 0, window_bytes: int | None = None):  # noqa: N802
    try:
        return FileReader(path, device, window_bytes), None
    except FileNotFoundError:
        return None, GoError(f"open {path}: no such file or directory")


def NewFileReader(ReaderPath: str | None = None, ReaderFile=None, device: int = 0):  # noqa: N802,N803
    if (ReaderFile is None) == (ReaderPath is None or ReaderPath == ""):
        return None, GoError("NewFileReader: either os.File or string path must be supplied, never both")
    path = ReaderPath if ReaderPath else ReaderFile.name
    return NewFileReaderWithPath(path, device)


def NewMemoryMappedReaderWithPath(path: str, device: int = 0):  # noqa: N802
    try:
        return MMapReader(path, device), None
    except FileNotFoundError:
        return None, GoError(f"error while opening mmap at '{path}': open {path}: no such file or directory")
