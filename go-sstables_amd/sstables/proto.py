"""Host-side protobuf wire helpers for the SSTable mirror (sstables/proto/sstable.proto).

MetaData is one small message per table (meta.pb.bin, read on the host by the reference too,
sstable_reader.go:356-382); IndexEntry encoding is the writer side (sstable_writer.go:126-132).
IndexEntry decoding for reads runs on the device (rio_sst_index_parse).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

from recordio.errors import GoError


def put_varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _varint(b: bytes, pos: int):
    x = 0
    for i in range(10):
        if pos >= len(b):
            raise ValueError("truncated varint")
        c = b[pos]
        pos += 1
        if i == 9 and c > 1:
            raise ValueError("varint overflow")
        x |= (c & 0x7F) << (7 * i)
        if c < 0x80:
            return x, pos
    raise ValueError("varint overflow")


def encode_index_entry(key: bytes, value_offset: int, checksum: int) -> bytes:
    """proto.Marshal(&IndexEntry{...}) with proto3 defaults omitted (deterministic field order)."""
    out = bytearray()
    if key:
        out += b"\x0a" + put_varint(len(key)) + key
    if value_offset:
        out += b"\x10" + put_varint(value_offset)
    if checksum:
        out += b"\x18" + put_varint(checksum)
    return bytes(out)


def decode_index_entry(b: bytes):
    """proto.Unmarshal into a reset IndexEntry for the iterators' one-record-at-a-time path
    (DiskKeyIndexIterator.Next, disk_key_index.go:141-165): (key, valueOffset, checksum); ValueError
    on malformed input. Bulk parsing runs on the device (rio_sst_index_parse, rio_index_search)."""
    key, vo, cs = b"", 0, 0
    pos = 0
    while pos < len(b):
        tag, pos = _varint(b, pos)
        num, wt = tag >> 3, tag & 7
        if num < 1 or num > 0x1FFFFFFF:
            raise ValueError("invalid field number")
        if wt == 0:
            v, pos = _varint(b, pos)
            if num == 2:
                vo = v
            elif num == 3:
                cs = v
        elif wt == 2:
            ln, pos = _varint(b, pos)
            if ln > len(b) - pos:
                raise ValueError("truncated bytes")
            if num == 1:
                key = bytes(b[pos:pos + ln])
            pos += ln
        elif wt in (1, 5):
            w = 8 if wt == 1 else 4
            if w > len(b) - pos:
                raise ValueError("truncated fixed")
            pos += w
        elif wt == 3:
            pos = _skip_group(b, pos, num)
        else:
            raise ValueError(f"wire type {wt}")
    return key, vo, cs


def _skip_group(b: bytes, pos: int, num: int) -> int:
    """protowire.ConsumeGroup: nested start/end tags must match, depth <= 16 (as the kernels)."""
    stack = [num]
    while stack:
        tag, pos = _varint(b, pos)
        fn, t = tag >> 3, tag & 7
        if fn < 1 or fn > 0x1FFFFFFF:
            raise ValueError("invalid field number")
        if t == 4:
            if stack[-1] != fn:
                raise ValueError("mismatched end group")
            stack.pop()
        elif t == 3:
            if len(stack) == 16:
                raise ValueError("group nesting")
            stack.append(fn)
        elif t == 0:
            _, pos = _varint(b, pos)
        elif t in (1, 5):
            w = 8 if t == 1 else 4
            if w > len(b) - pos:
                raise ValueError("truncated fixed")
            pos += w
        elif t == 2:
            ln, pos = _varint(b, pos)
            if ln > len(b) - pos:
                raise ValueError("truncated bytes")
            pos += ln
        else:
            raise ValueError(f"wire type {t}")
    return pos


@dataclass
class MetaData:
    numRecords: int = 0
    minKey: bytes = b""
    maxKey: bytes = b""
    dataBytes: int = 0
    indexBytes: int = 0
    totalBytes: int = 0
    version: int = 0
    skippedRecords: int = 0
    nullValues: int = 0

    # Go accessor names used by the reference tests
    @property
    def NumRecords(self): return self.numRecords  # noqa: N802,E704
    @property
    def MinKey(self): return self.minKey  # noqa: N802,E704
    @property
    def MaxKey(self): return self.maxKey  # noqa: N802,E704
    @property
    def Version(self): return self.version  # noqa: N802,E704
    @property
    def NullValues(self): return self.nullValues  # noqa: N802,E704
    @property
    def DataBytes(self): return self.dataBytes  # noqa: N802,E704
    @property
    def IndexBytes(self): return self.indexBytes  # noqa: N802,E704
    @property
    def TotalBytes(self): return self.totalBytes  # noqa: N802,E704

    _FIELDS = {1: "numRecords", 2: "minKey", 3: "maxKey", 4: "dataBytes", 5: "indexBytes", 6: "totalBytes",
               7: "version", 8: "skippedRecords", 9: "nullValues"}

    def marshal(self) -> bytes:
        out = bytearray()
        for num, name in self._FIELDS.items():
            v = getattr(self, name)
            if not v:
                continue
            if isinstance(v, (bytes, bytearray)):
                out += put_varint(num << 3 | 2) + put_varint(len(v)) + bytes(v)
            else:
                out += put_varint(num << 3) + put_varint(v)
        return bytes(out)

    @classmethod
    def unmarshal(cls, b: bytes) -> "MetaData":
        m = cls()
        pos = 0
        while pos < len(b):
            tag, pos = _varint(b, pos)
            num, wt = tag >> 3, tag & 7
            if num < 1:
                raise ValueError("invalid field number")
            if wt == 0:
                v, pos = _varint(b, pos)
            elif wt == 2:
                ln, pos = _varint(b, pos)
                if ln > len(b) - pos:
                    raise ValueError("truncated bytes")
                v, pos = bytes(b[pos:pos + ln]), pos + ln
            elif wt in (1, 5):
                w = 8 if wt == 1 else 4
                if w > len(b) - pos:
                    raise ValueError("truncated fixed")
                v, pos = None, pos + w
            else:
                raise ValueError(f"wire type {wt}")
            name = cls._FIELDS.get(num)
            if name is None or v is None:
                continue
            want_bytes = name in ("minKey", "maxKey")
            if want_bytes == isinstance(v, bytes):
                setattr(m, name, v if want_bytes else v & (0xFFFFFFFF if name == "version" else (1 << 64) - 1))
        return m


def read_metadata_if_exists(path: str):
    """readMetaDataIfExists (sstable_reader.go:356-382): absent file -> default MetaData."""
    if not os.path.exists(path):
        return MetaData(), None
    try:
        with open(path, "rb") as fh:
            return MetaData.unmarshal(fh.read()), None
    except (OSError, ValueError) as e:
        return None, GoError(str(e))
