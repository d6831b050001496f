"""SSTableStreamWriter mirror (sstables/sstable_writer.go:27-180): the input generator for the
device scan. data.rio = one recordio v4 record per value (Snappy by default, :219-220), index.rio =
one IndexEntry{key, valueOffset, checksum = CRC-64/ISO of the value} per key (uncompressed), and
meta.pb.bin. Host-side; the bloom filter (optional in the reference) is not written.
"""
from __future__ import annotations

import ctypes
import os

from recordio import _lib as L
from recordio.errors import GoError

from .proto import MetaData, encode_index_entry

_CRC64 = None


def crc64_iso(data: bytes) -> int:
    """hash/crc64 with crc64.ISO (what the writer stores, sstable_writer.go:120-124). Host-side
    generator helper; the read path computes it on the device."""
    global _CRC64
    if _CRC64 is None:
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ (0xD800000000000000 if c & 1 else 0)
            t.append(c)
        _CRC64 = t
    c = 0xFFFFFFFFFFFFFFFF
    for b in data:
        c = _CRC64[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFFFFFFFFFF


class _Image:
    """An in-memory recordio v4 file built with the library's record encoder."""

    def __init__(self, compression: int):
        lib = L.lib()
        self.c = compression
        hdr = ctypes.create_string_buffer(8)
        lib.rio_encode_file_header(hdr, 4, compression)
        self.parts = [hdr.raw]
        self.size = 8

    def write(self, rec):
        lib = L.lib()
        n = 0 if rec is None else len(rec)
        cap = 64 + int(lib.rio_snappy_max_encoded_len(n)) + n // 50 + 64
        buf = ctypes.create_string_buffer(cap)
        src = None if rec is None else (ctypes.c_char_p(bytes(rec)) if n else ctypes.c_char_p(b"\0"))
        w = int(lib.rio_encode_record_v4(buf, cap, self.c, src, n))
        if w == 0:
            raise GoError("record encode failed")
        off = self.size
        self.parts.append(buf.raw[:w])
        self.size += w
        return off

    def bytes(self) -> bytes:
        return b"".join(self.parts)


class SSTableStreamWriter:
    def __init__(self, base_path: str, data_compression: int = 2, index_compression: int = 0):
        self.base = base_path
        self.data = _Image(data_compression)
        self.index = _Image(index_compression)
        self.meta = MetaData(version=1)
        self.last = None
        self._crc_cache = {}

    def Open(self):  # noqa: N802
        os.makedirs(self.base, exist_ok=True)
        return None

    def WriteNext(self, key: bytes, value):  # noqa: N802
        key = bytes(key)
        if self.last is not None:
            if self.last == key:
                return GoError(f"sstables.WriteNext '{self.base}': the same key cannot be written more than once")
            if self.last > key:
                return GoError(f"sstables.WriteNext '{self.base}': non-ascending key cannot be written")
        else:
            self.meta.minKey = key
        self.last = key
        vb = b"" if value is None else bytes(value)
        cs = self._crc_cache.get(vb)
        if cs is None:
            cs = crc64_iso(vb)
            if len(self._crc_cache) < 4:
                self._crc_cache[vb] = cs
        off = self.data.write(value)
        self.index.write(encode_index_entry(key, off, cs))
        self.meta.numRecords += 1
        if value is None:
            self.meta.nullValues += 1
        return None

    def Close(self):  # noqa: N802
        from . import DataFileName, IndexFileName, MetaFileName

        d, i = self.data.bytes(), self.index.bytes()
        with open(os.path.join(self.base, DataFileName), "wb") as fh:
            fh.write(d)
        with open(os.path.join(self.base, IndexFileName), "wb") as fh:
            fh.write(i)
        self.meta.maxKey = self.last or b""
        self.meta.dataBytes, self.meta.indexBytes = len(d), len(i)
        self.meta.totalBytes = len(d) + len(i)
        with open(os.path.join(self.base, MetaFileName), "wb") as fh:
            fh.write(self.meta.marshal())
        return None


def NewSSTableStreamWriter(base_path: str, data_compression: int = 2):  # noqa: N802
    return SSTableStreamWriter(base_path, data_compression), None


def write_sstable(base_path: str, items, data_compression: int = 2) -> MetaData:
    """Write sorted (key, value) pairs as one table; returns its MetaData."""
    w = SSTableStreamWriter(base_path, data_compression)
    w.Open()
    for k, v in items:
        err = w.WriteNext(k, v)
        if err is not None:
            raise err
    w.Close()
    return w.meta
