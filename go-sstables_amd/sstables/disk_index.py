"""DiskIndexLoader / DiskKeyIndex mirror (sstables/disk_key_index.go) over the device lookup kernel.

Load keeps index.rio resident in HBM (rio_index_open). Get / Contains / IteratorStartingAt /
IteratorBetween run the reference's binarySearch on the device (rio_index_search, one lane per
key), with the probe sequence and error rules of a freshly loaded DiskKeyIndex. GetBatch looks up
many keys in one launch, which is the path's reason to exist. The iterators walk on from the searched
offset with SeekNext through the MMapReader mirror (disk_key_index.go:141-165).
"""
from __future__ import annotations

import ctypes

import numpy as np

from recordio import _lib as L
from recordio.errors import EOF, GoError, errors_is, wrap
from recordio.reader import NewMemoryMappedReaderWithPath


NotFound = GoError("key not found")  # skiplist.NotFound (skiplist/skiplist.go)
Done = GoError("no more items in iterator")  # skiplist.Done


class IndexVal:
    """sstables.IndexVal {Offset, Checksum} (sstable_index.go)"""

    __slots__ = ("Offset", "Checksum")

    def __init__(self, offset=0, checksum=0):
        self.Offset, self.Checksum = offset, checksum

    def __eq__(self, o):
        return isinstance(o, IndexVal) and (self.Offset, self.Checksum) == (o.Offset, o.Checksum)

    def __repr__(self):
        return f"IndexVal(Offset={self.Offset}, Checksum={self.Checksum})"


def _error(status: int, version: int = 0) -> GoError:
    if status == L.RIO_ERR_PROTO:
        return GoError("proto: cannot parse invalid wire-format data")
    if status == L.RIO_ERR_UNSUPPORTED:
        if version < 2:  # a v1 index: every probe's SeekNext fails (mmap_reader.go:62-64)
            return GoError("unsupported on files with version lower than v2")
        # (v2+: DiskKeyIndex.lookups answers these probes on the host reader; this text is reached
        # only if that reader itself hands a probe back)
        return GoError("rio: SeekNext probe ends outside the decoded record sequence (unsupported on the device)")
    from recordio.reader import _base_error

    return _base_error(status)


class DiskKeyIndex:
    def __init__(self, path: str, device: int = 0):
        self.path = path
        self.device = device
        self._h = None
        self._reader = None
        self.version = 0

    def Open(self):  # noqa: N802
        with open(self.path, "rb") as fh:
            img = fh.read()
        h = ctypes.c_void_p()
        rc = L.lib().rio_index_open(L.default_ctx(self.device), img, len(img), ctypes.byref(h))
        if rc:
            return GoError(f"error while loading index '{self.path}' to the device: {L.strerror(rc)}")
        self._h, self.size = h, len(img)
        # recordio file version (common_reader.go:22-44: LE u32 at offset 0)
        self.version = int.from_bytes(img[:4], "little") if len(img) >= 4 else 0
        self._reader, err = NewMemoryMappedReaderWithPath(self.path, self.device)
        if err is not None:
            return err
        return self._reader.Open()

    def Close(self):  # noqa: N802
        if self._h is not None:
            L.lib().rio_index_free(self._h)
            self._h = None
        return self._reader.Close() if self._reader is not None else None

    def __del__(self):
        if getattr(self, "_h", None) is not None:
            L.lib().rio_index_free(self._h)
            self._h = None

    def search(self, keys) -> list:
        """One rio_index_hit per key: (offset, found, value_offset, checksum, status)."""
        keys = [bytes(k) for k in keys]
        n = len(keys)
        if n == 0:
            return []
        off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([len(k) for k in keys], out=off[1:])
        blob = b"".join(keys) or b"\0"
        hits = (L.IndexHit * n)()
        rc = L.lib().rio_index_search(self._h, blob, off.ctypes.data, n, hits)
        if rc:
            raise GoError(f"rio_index_search: {L.strerror(rc)}")
        return [(h.offset, bool(h.found), h.value_offset, h.checksum, h.status) for h in hits]

    def lookups(self, keys) -> list:
        """(offset, found, value_offset, checksum, err) per key: the device search, except that a key
        whose probe the device hands back (RIO_ERR_UNSUPPORTED on a v2+ compressed index: a SeekNext
        walk that ends outside the decoded record sequence) is searched again on the host
        reader with the reference's own loop, so Get / Contains / the iterators answer
        where the reference answers."""
        keys = [bytes(k) for k in keys]
        out = []
        for k, (off, found, vo, cs, st) in zip(keys, self.search(keys)):
            if st == L.RIO_ERR_UNSUPPORTED and self.version >= 2:
                out.append(self._host_search(k))
            else:
                out.append((off, found, vo, cs, _error(st, self.version) if st else None))
        return out

    def _host_search(self, target: bytes):
        """DiskKeyIndex.binarySearch + findAt (disk_key_index.go:88-139) with every probe a SeekNext of
        the MMapReader mirror and proto.Unmarshal of its record (mmap_proto_reader.go:26-38), as a
        freshly loaded index (no offsetCache)."""
        from .proto import decode_index_entry

        n = self.size

        def find_at(h):
            _, rec, err = self._reader.SeekNext(h)
            if err is not None:
                return None, err
            try:
                return decode_index_entry(rec or b""), None
            except ValueError:
                return None, GoError("proto: cannot parse invalid wire-format data")

        i, j = 0, n
        while i < j:
            h = (i + j) >> 1
            at, err = find_at(h)
            if err is not None:
                return (n, False, 0, 0, None) if errors_is(err, EOF) else (0, False, 0, 0, err)
            if at[0] < target:
                i = h + 1
            else:
                j = h
        at, err = find_at(i)
        if err is not None:
            return (n, False, 0, 0, None) if errors_is(err, EOF) else (0, False, 0, 0, err)
        return i, i < n and at[0] == target, at[1], at[2], None

    def GetBatch(self, keys):  # noqa: N802
        """[(IndexVal, err)] per key, Get's semantics."""
        out = []
        for off, found, vo, cs, err in self.lookups(keys):
            if err is not None:
                out.append((IndexVal(), err))
            elif not found:
                out.append((IndexVal(), NotFound))
            else:
                out.append((IndexVal(vo, cs), None))
        return out

    def Get(self, key):  # noqa: N802
        return self.GetBatch([key])[0]

    def Contains(self, key):  # noqa: N802
        off, found, _, _, err = self.lookups([key])[0]
        return (False, err) if err is not None else (found, None)

    def Iterator(self):  # noqa: N802
        return _DiskKeyIndexIterator(self._reader, 8, self.size), None

    def IteratorStartingAt(self, key):  # noqa: N802
        off, _, _, _, err = self.lookups([key])[0]
        if err is not None:
            return None, err
        return _DiskKeyIndexIterator(self._reader, off, self.size), None

    def IteratorBetween(self, lo, hi):  # noqa: N802
        if bytes(lo) > bytes(hi):
            return None, GoError("keyHigher is lower than keyLower")
        (s, _, _, _, e1), (e, found, _, _, e2) = self.lookups([lo, hi])
        if e1 is not None or e2 is not None:
            return None, e1 if e1 is not None else e2
        if not found:
            e -= 1  # keyHigher is inclusive
        return _DiskKeyIndexIterator(self._reader, s, e), None


class _DiskKeyIndexIterator:
    """disk_key_index.go:141-165: SeekNext from the current offset, then offset + 1."""

    def __init__(self, reader, offset, end):
        self.r, self.cur, self.end = reader, offset, end

    def Next(self):  # noqa: N802
        from .proto import decode_index_entry

        if self.cur > self.end:
            return None, IndexVal(), Done
        off, rec, err = self.r.SeekNext(self.cur)
        if err is not None:
            if errors_is(err, EOF):
                return None, IndexVal(), Done
            return None, IndexVal(), err
        try:
            k, vo, cs = decode_index_entry(rec or b"")
        except ValueError as e:
            return None, IndexVal(), wrap("proto", GoError(str(e)))
        self.cur = off + 1
        return k, IndexVal(vo, cs), None


class DiskIndexLoader:
    """disk_key_index.go:167-181"""

    def __init__(self, device: int = 0):
        self.device = device

    def Load(self, indexPath: str, _meta=None):  # noqa: N802,N803
        return DiskKeyIndex(indexPath, self.device), None
