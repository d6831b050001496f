"""FileWriter mirror (input generator; recordio/file_writer.go:189-233). Host-side, not on the
decode path: it produces the v4 files the decode path consumes (byte-identical to the reference
writer, see tests/test_writer.py)."""
from __future__ import annotations

import ctypes
from ctypes import byref, c_uint64, c_void_p

import numpy as np

from . import _lib as L
from .errors import GoError


class FileWriter:
    def __init__(self, path: str, compression: int = 0):
        self.path = path
        self.compression = compression
        self._h = c_void_p()

    def Open(self):  # noqa: N802
        rc = L.lib().rio_writer_new(self.path.encode(), self.compression, byref(self._h))
        return None if rc == L.RIO_OK else GoError(f"open {self.path}: {L.strerror(rc)}")

    def Write(self, record):  # noqa: N802
        """record None => nil record; returns (offset, err)."""
        off = c_uint64()
        if record is None:
            rc = L.lib().rio_writer_write(self._h, None, 0, byref(off))
        else:
            buf = bytes(record)
            rc = L.lib().rio_writer_write(self._h, ctypes.c_char_p(buf) if buf else ctypes.c_char_p(b"\0"), len(buf),
                                          byref(off))
        return (off.value, None) if rc == L.RIO_OK else (0, GoError(L.strerror(rc)))

    def Size(self) -> int:  # noqa: N802
        return int(L.lib().rio_writer_size(self._h))

    def Close(self):  # noqa: N802
        rc = L.lib().rio_writer_close(self._h)
        self._h = c_void_p()
        return None if rc == L.RIO_OK else GoError(L.strerror(rc))


def NewFileWriter(path: str, compression: int = 0):  # noqa: N802
    return FileWriter(path, compression), None


def encode_file(records, compression: int = 0) -> bytes:
    """In-memory v4 file image: the same bytes FileWriter would write."""
    lib = L.lib()
    hdr = ctypes.create_string_buffer(8)
    lib.rio_encode_file_header(hdr, 4, compression)
    parts = [hdr.raw]
    for r in records:
        n = 0 if r is None else len(r)
        cap = 64 + int(lib.rio_snappy_max_encoded_len(n)) + n // 2 + 64  # lzw: <= 1.5 n + 8
        buf = ctypes.create_string_buffer(cap)
        if r is None:
            w = lib.rio_encode_record_v4(buf, cap, compression, None, 0)
        else:
            src = bytes(r)
            w = lib.rio_encode_record_v4(buf, cap, compression, ctypes.c_char_p(src) if src else ctypes.c_char_p(b"\0"),
                                         n)
        if not w:
            raise RuntimeError("rio_encode_record_v4 failed")
        parts.append(buf.raw[:w])
    return b"".join(parts)


def generate(n_records: int, record_len: int, compression: int = 2, kind: int = 1, seed: int = 1,
             threads: int = 0) -> np.ndarray:
    """Synthetic workload file image (rio_generate): kind 0 ref-random repeated record
    (benchmark/recordio_read_test.go:32-42), 1 text-like, 2 random distinct."""
    lib = L.lib()
    cap = int(lib.rio_generate_bound(compression, n_records, record_len))
    buf = np.empty(cap + L.RIO_DEVICE_PAD, dtype=np.uint8)
    n = int(lib.rio_generate(buf.ctypes.data, cap, compression, n_records, record_len, kind, seed, threads))
    if n == 0:
        raise RuntimeError("rio_generate failed")
    return buf[:n]
