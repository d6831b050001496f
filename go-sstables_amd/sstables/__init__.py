"""MI355X-native SSTable load / validation / full scan — Python mirror of
github.com/thomasjungblut/go-sstables/sstables (sstable_reader.go, sstable_iterator.go,
slice_key_index.go, sstable_writer.go).

The device does the byte work: both files are decoded by the recordio path (rio_device_decode),
the index records are parsed and every value's CRC-64/ISO is computed by the kernels of
rio_sstable.hip (rio_sst_index_parse / rio_sst_validate). This module keeps the reference's API
shape: NewSSTableReader(options...) -> (reader, err), reader.Scan() -> iterator whose Next()
returns (key, value, err) with the Done sentinel, MetaData(), Get, Contains, Close; errors carry
the reference's message texts. v0 tables (metadata version 0: every value a protobuf DataEntry,
sstable_reader.go:303-314) have their values unwrapped on the device (rio_sst_data_entries). A table
whose index is not in the writer's layout returns UnsupportedError: the adapter keeps the reference
reader for it. There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

from recordio import _lib as L
from recordio.errors import EOF, ErrCorrupt, GoError, wrap

from . import proto
from .disk_index import DiskIndexLoader, DiskKeyIndex, IndexVal  # noqa: F401
from .writer import NewSSTableStreamWriter, SSTableStreamWriter, write_sstable  # noqa: F401

IndexFileName = "index.rio"
DataFileName = "data.rio"
BloomFileName = "bloom.bf.gz"
MetaFileName = "meta.pb.bin"
Version = 1

Done = GoError("no more items in iterator")  # sstable.go:18
NotFound = GoError("key was not found")  # sstable.go:19
_NONE = 0xFFFFFFFFFFFFFFFF
ProtoWireError = GoError("proto: cannot parse invalid wire-format data")  # protobuf-go's proto.Unmarshal


class ChecksumError(GoError):
    """sstable_reader.go:22-35"""

    def __init__(self, checksum: int, expected: int):
        super().__init__(f"Checksum mismatch: expected {expected:x}, got {checksum:x}")
        self.checksum = checksum
        self.expectedChecksum = expected

    def __eq__(self, other):
        return isinstance(other, ChecksumError) and (self.checksum, self.expectedChecksum) == (
            other.checksum, other.expectedChecksum)

    __hash__ = GoError.__hash__


class UnsupportedError(GoError):
    """The device path hands this table back to the reference reader (RIO_ERR_UNSUPPORTED)."""


@dataclass
class _Opts:
    basePath: str = ""
    skipHashCheckOnLoad: bool = False  # sstable_reader.go:255-258: validate on load by default
    skipHashCheckOnRead: bool = True
    device: int = 0


def ReadBasePath(p: str):  # noqa: N802
    def f(o): o.basePath = p
    return f


def SkipHashCheckOnLoad():  # noqa: N802
    def f(o): o.skipHashCheckOnLoad = True
    return f


def EnableHashCheckOnReads():  # noqa: N802
    def f(o): o.skipHashCheckOnRead = False
    return f


def ReadWithKeyComparator(_cmp=None):  # noqa: N802
    """Bytes comparator only (skiplist.BytesComparator, the reference's default)."""
    def f(o): pass
    return f


def ReadOnDevice(device: int):  # noqa: N802
    def f(o): o.device = device
    return f


def _fmt_key(k: bytes) -> str:
    return "[" + " ".join(str(b) for b in k) + "]"  # Go's %v of a []byte


class _DeviceTable:
    """Both files decoded on the device, index parsed, every value's CRC-64 computed."""

    def __init__(self, base: str, device: int, need_crc: bool, v0: bool = False):
        import torch

        from recordio.device import DeviceDecoder, header_codec, to_device_file

        self.dec = DeviceDecoder(device)
        dev = f"cuda:{device}"
        lib = L.lib()

        def decode(name):
            with open(os.path.join(base, name), "rb") as fh:
                img = fh.read()
            d, n = to_device_file(img, device)
            # the header's codec: only that codec's kernels are launched
            b, info = self.dec.decode(d, n, comp=header_codec(img))
            return img, b, info

        self.index_img, self.ib, ii = decode(IndexFileName)
        self.data_img, self.db, di = decode(DataFileName)
        for what, info in (("index", ii), ("data", di)):
            if info["status"] == L.RIO_ERR_UNSUPPORTED:
                raise UnsupportedError(f"{what} file of '{base}' is not decoded on the device (recordio v"
                                       f"{info['version']}, compression {info['compression']})")
        self.index_info, self.data_info = ii, di
        n = ii["n_records"]
        # an index record that does not decompress: Load's ReadNext fails there, or ends the index
        # for gzip's bare io.EOF (slice_key_index.go:117-126)
        self.index_bad = _NONE
        if ii["n_bad"]:
            if int(self.ib.flags[ii["first_bad"]].item()) & L.RIO_FLAG_CORRUPT:
                self.index_bad = ii["first_bad"]
            n = ii["first_bad"]
        self.n_index = n
        self.n_data = di["n_records"]
        # first entry whose value does not decompress (entry i = data record i in the writer's layout)
        self.value_bad = di["first_bad"] if di["n_bad"] and di["first_bad"] < n else _NONE
        self.key_off = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.key_len = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.value_off = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        self.checksum = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        res = torch.empty(2, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream(device)
        rc = lib.rio_sst_index_parse(self.dec.ctx, self.ib.out.data_ptr(), self.ib.out_off.data_ptr(), n,
                                     self.key_off.data_ptr(), self.key_len.data_ptr(), self.value_off.data_ptr(),
                                     self.checksum.data_ptr(), res.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
        if rc:
            raise GoError(f"rio_sst_index_parse: {L.strerror(rc)}")
        self.crc = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        vres = torch.empty(2, dtype=torch.int64, device=dev)
        self.v0 = v0
        st = ctypes.c_void_p(stream.cuda_stream)
        if v0:
            # every value record is a DataEntry: its value's range in the data arena (MMapProtoReader /
            # ProtoReader unmarshal, recordio/proto/mmap_proto_reader.go:12-24), hashed as such
            self.view = torch.empty(2 * max(self.n_data, 1), dtype=torch.int64, device=dev)
            dres = torch.empty(1, dtype=torch.int64, device=dev)
            rc = lib.rio_sst_data_entries(self.dec.ctx, self.db.out.data_ptr(), self.db.out_off.data_ptr(), self.n_data,
                                          self.view.data_ptr(), dres.data_ptr(), st)
            if rc:
                raise GoError(f"rio_sst_data_entries: {L.strerror(rc)}")
            rc = lib.rio_sst_validate_view(self.dec.ctx, self.db.out.data_ptr(), self.db.out_off.data_ptr(),
                                           self.db.rec_off.data_ptr(), self.n_data, self.view.data_ptr(),
                                           self.value_off.data_ptr(), self.checksum.data_ptr(), n, self.crc.data_ptr(),
                                           vres.data_ptr(), st)
        else:
            rc = lib.rio_sst_validate(self.dec.ctx, self.db.out.data_ptr(), self.db.out_off.data_ptr(),
                                      self.db.rec_off.data_ptr(), self.n_data, self.value_off.data_ptr(),
                                      self.checksum.data_ptr(), n, self.crc.data_ptr(), vres.data_ptr(), st)
        if rc:
            raise GoError(f"rio_sst_validate: {L.strerror(rc)}")
        torch.cuda.synchronize(device)
        self.bad_proto = int(res[0].item()) & _NONE
        self.bad_crc, self.unplaced = (int(v) & _NONE for v in vres.cpu().tolist())
        # host views for the Python iterator (the device arrays stay resident)
        u = lambda t, k: [x & _NONE for x in t[:k].cpu().tolist()]  # noqa: E731
        self.h_key_off, self.h_key_len = u(self.key_off, n), u(self.key_len, n)
        self.h_value_off, self.h_checksum, self.h_crc = u(self.value_off, n), u(self.checksum, n), u(self.crc, n)
        nb_i, nb_d = ii["total_out_bytes"], di["total_out_bytes"]
        self.h_index = bytes(self.ib.out[:nb_i].cpu().numpy())
        self.h_data = bytes(self.db.out[:nb_d].cpu().numpy())
        self.h_data_off = u(self.db.out_off, self.n_data + 1)
        self.h_data_flags = self.db.flags[:self.n_data].cpu().tolist()
        self.h_view = u(self.view, 2 * self.n_data) if v0 else None

    def key(self, i) -> bytes:
        o = self.h_key_off[i]
        return self.h_index[o:o + self.h_key_len[i]]

    def value(self, j):
        if self.v0:  # DataEntry.value: nil when the field is absent
            b, e = self.h_view[2 * j], self.h_view[2 * j + 1]
            return None if b >= L.RIO_VALUE_BAD else self.h_data[b:e]
        if self.h_data_flags[j] & L.RIO_FLAG_NIL:
            return None
        return self.h_data[self.h_data_off[j]:self.h_data_off[j + 1]]

    def value_proto_bad(self, j) -> bool:
        """v0 tables: data record j is not a valid DataEntry (proto.Unmarshal fails)."""
        return self.v0 and self.h_view[2 * j] == L.RIO_VALUE_BAD

    def value_failed(self, j) -> bool:
        """Data record j does not decompress (RIO_FLAG_CORRUPT / RIO_FLAG_EOF)."""
        return bool(self.h_data_flags[j] & (L.RIO_FLAG_CORRUPT | L.RIO_FLAG_EOF))

    def codec_error(self, j):
        """The reader's error for data record j: snappy/gzip's error, or gzip's bare io.EOF."""
        return EOF if self.h_data_flags[j] & L.RIO_FLAG_EOF else ErrCorrupt


class SSTableReader:
    def __init__(self, opts: _Opts, meta: proto.MetaData, table: _DeviceTable):
        self.opts, self.meta, self.t = opts, meta, table
        self._keys = None

    def MetaData(self) -> proto.MetaData:  # noqa: N802
        return self.meta

    def BasePath(self) -> str:  # noqa: N802
        return self.opts.basePath

    def Scan(self):  # noqa: N802
        """SSTableFullScanIterator (sstable_iterator.go:68-111): index entries in file order paired
        with data records read sequentially."""
        # v0 tables: V0SSTableFullScanIterator (sstable_iterator.go:34-66) never checks hashes
        return _FullScanIterator(self, self.opts.skipHashCheckOnRead or self.t.v0), None

    def ScanStartingAt(self, key: bytes):  # noqa: N802
        """SSTableIterator over IteratorStartingAt (sstable_reader.go:161-167, slice_key_index.go:49-52):
        entries from the first key >= key, values by getValueAtOffset."""
        import bisect

        return _KeyRangeIterator(self, bisect.bisect_left(self._index_keys(), bytes(key)), self.t.n_index), None

    def ScanRange(self, key_lower: bytes, key_higher: bytes):  # noqa: N802
        """SSTableIterator over IteratorBetween (sstable_reader.go:169-175, slice_key_index.go:54-70):
        both ends inclusive."""
        import bisect

        lo, hi = bytes(key_lower), bytes(key_higher)
        if lo > hi:
            return None, wrap(f"error in sstable '{self.opts.basePath}' in ScanRange",
                              GoError("keyHigher is lower than keyLower"))
        ks = self._index_keys()
        start, end = bisect.bisect_left(ks, lo), bisect.bisect_left(ks, hi)
        if end < len(ks) and ks[end] <= hi:
            end += 1
        return _KeyRangeIterator(self, start, end), None

    def _value_at(self, i, skip_check):
        """getValueAtOffset (sstable_reader.go:80-117) for index entry i (the writer's layout)."""
        t = self.t
        if t.value_failed(i):  # dataReader.ReadNextAt's error (mmap_reader.go:186-191), wrapped at :90-94
            vo, path = t.h_value_off[i], os.path.join(self.opts.basePath, DataFileName)
            inner = wrap(f"failed decompressing record at offset {vo} in mmap reader for '{path}'", t.codec_error(i))
            return None, wrap(f"error in sstable '{self.opts.basePath}' while getting value at offset {vo}", inner)
        if t.value_proto_bad(i):  # v0: MMapProtoReader.ReadNextAt's proto.Unmarshal error (sstable_reader.go:79-86)
            return None, wrap(f"error in sstable '{self.opts.basePath}' while getting value at offset {t.h_value_off[i]}",
                              ProtoWireError)
        v = t.value(i)
        if skip_check:
            return v, None
        if t.h_crc[i] != t.h_checksum[i] and t.h_checksum[i] != 0:
            return v, GoError(f"error in sstable '{self.opts.basePath}' while hashing value at offset "
                              f"[{t.h_value_off[i]}]: {ChecksumError(t.h_crc[i], t.h_checksum[i])}",
                              wrapped=ChecksumError(t.h_crc[i], t.h_checksum[i]))
        return v, None

    def _index_keys(self):
        if self._keys is None:
            self._keys = [self.t.key(i) for i in range(self.t.n_index)]
        return self._keys

    def Get(self, key: bytes):  # noqa: N802
        """SliceKeyIndex.Get (sort.Search over the entries, slice_key_index.go:19-35)."""
        import bisect

        ks = self._index_keys()
        i = bisect.bisect_left(ks, bytes(key))
        if i >= len(ks) or ks[i] != bytes(key):
            return None, NotFound
        return self._value_at(i, self.opts.skipHashCheckOnRead)

    def Contains(self, key: bytes):  # noqa: N802
        import bisect

        ks = self._index_keys()
        i = bisect.bisect_left(ks, bytes(key))
        return i < len(ks) and ks[i] == bytes(key), None

    def Close(self):  # noqa: N802
        self.t = None
        return None


class _KeyRangeIterator:
    """SSTableIterator (sstable_iterator.go:11-32): index entries [i, end) with getValueAtOffset."""

    def __init__(self, r: SSTableReader, i: int, end: int):
        self.r, self.i, self.end = r, i, end

    def Next(self):  # noqa: N802
        if self.i >= self.end:
            return None, None, Done
        i = self.i
        self.i += 1
        v, err = self.r._value_at(i, self.r.opts.skipHashCheckOnRead)
        if err is not None:
            return None, None, err
        return self.r.t.key(i), v, None


class _FullScanIterator:
    def __init__(self, r: SSTableReader, skip_check: bool):
        self.r, self.skip, self.i = r, skip_check, 0

    def Next(self):  # noqa: N802
        t = self.r.t
        i = self.i
        if i >= t.n_index:
            return None, None, Done
        self.i += 1
        key = t.key(i)
        if i >= t.n_data:  # dataReader.ReadNext error (end of data file before end of index)
            return None, None, GoError(f"data file of '{self.r.opts.basePath}' ended at record {i}: "
                                       f"{L.strerror(t.data_info['status'])}")
        if t.value_failed(i):  # dataReader.ReadNext's codec error, returned as is (sstable_iterator.go:87-90)
            return None, None, t.codec_error(i)
        if t.value_proto_bad(i):  # v0: the proto reader's ReadNext, unmarshal error as is (:52-56)
            return None, None, ProtoWireError
        v = t.value(i)
        if self.skip:
            return key, v, None
        if t.h_checksum[i] != 0 and t.h_crc[i] != t.h_checksum[i]:
            return key, v, ChecksumError(t.h_crc[i], t.h_checksum[i])
        return key, v, None


def NewSSTableReader(*options):  # noqa: N802
    """sstable_reader.go:250-345: metadata, index (SliceKeyIndexLoader), data reader, then
    validateDataFile unless SkipHashCheckOnLoad."""
    o = _Opts()
    for f in options:
        f(o)
    if not o.basePath:
        return None, GoError("SSTableReader: basePath was not supplied")
    meta, err = proto.read_metadata_if_exists(os.path.join(o.basePath, MetaFileName))
    if err is not None:
        return None, GoError(f"error while reading metadata of sstable in '{o.basePath}': {err}", wrapped=err)
    v0 = meta.version == 0  # values are protobuf DataEntry records (sstable_reader.go:303-314)
    try:
        t = _DeviceTable(o.basePath, o.device, True, v0)
    except UnsupportedError as e:
        return None, e
    # a flagged index record ends Load's loop before any later terminal status is reached
    # (slice_key_index.go:117-126: ErrCorrupt returns, gzip's bare io.EOF breaks)
    if t.index_info["n_bad"] == 0 and t.index_info["status"] not in L.EOF_CLASS:
        return None, GoError(f"error while reading index of sstable in '{o.basePath}': "
                             f"{L.strerror(t.index_info['status'])}")
    if t.index_bad != _NONE and (t.bad_proto == _NONE or t.index_bad <= t.bad_proto):
        ip = os.path.join(o.basePath, IndexFileName)
        return None, wrap(f"error while reading index records of sstable in '{ip}'", ErrCorrupt)
    if t.bad_proto != _NONE:
        return None, GoError(f"error while reading index of sstable in '{o.basePath}': proto: cannot parse "
                             f"invalid wire-format data (record {t.bad_proto})")
    if t.unplaced != _NONE:
        return None, UnsupportedError(f"sstable '{o.basePath}': index entry {t.unplaced} is not in the writer's layout")
    r = SSTableReader(o, meta, t)
    # validateDataFile returns at once for v0 tables (sstable_reader.go:205-209)
    if not v0 and not o.skipHashCheckOnLoad and (t.bad_crc != _NONE or t.value_bad != _NONE):
        # validateDataFile stops at the first entry whose value fails to read or to hash; a value
        # that does not decompress has no meaningful CRC, so on a tie it is the read error
        i = min(t.bad_crc, t.value_bad)
        _, e = r._value_at(i, False)
        return None, GoError(f"validateDataFile error loading value '{o.basePath}' at key "
                             f"[{_fmt_key(t.key(i))}]: {e}", wrapped=e)
    return r, None
