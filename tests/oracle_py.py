"""ctypes binding of the oracle (oracle/librio_oracle.so) — test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, byref, c_int, c_uint8, c_uint32, c_uint64, c_void_p

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RIO_ORACLE_PATH: the sanitizer build (oracle/Makefile `asan`, scripts/asan_cpu_suite.sh)
ORACLE_SO = os.environ.get("RIO_ORACLE_PATH") or os.path.join(REPO, "oracle", "librio_oracle.so")


class OrcFileResult(ctypes.Structure):
    _fields_ = [
        ("version", c_uint32), ("compression", c_uint32), ("n_records", c_uint64), ("total_out_bytes", c_uint64),
        ("status", ctypes.c_int32), ("status_offset", c_uint64), ("detail0", c_uint64), ("detail1", c_uint64),
        ("out", POINTER(c_uint8)), ("out_off", POINTER(c_uint64)), ("rec_off", POINTER(c_uint64)),
        ("flags", POINTER(c_uint8)), ("first_bad", c_uint64), ("n_bad", c_uint64),
    ]


class BadRecord:
    """A record whose payload does not decompress: ReadNext returns the codec error (kind
    "corrupt") or gzip's bare io.EOF (kind "eof") for it, and goes on with the next record."""

    def __init__(self, kind: str):
        self.kind = kind

    def __eq__(self, other):
        return isinstance(other, BadRecord) and other.kind == self.kind

    def __hash__(self):
        return hash(self.kind)

    def __repr__(self):
        return f"BadRecord({self.kind!r})"


NONE = (1 << 64) - 1


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle")], stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_crc32c.restype = c_uint32
        L.orc_crc32c.argtypes = [c_void_p, c_uint64]
        L.orc_file_reader_decode.argtypes = [c_void_p, c_uint64, POINTER(OrcFileResult)]
        L.orc_file_result_free.argtypes = [POINTER(OrcFileResult)]
        L.orc_read_next_at.argtypes = [c_void_p, c_uint64, c_uint64, POINTER(c_void_p), POINTER(c_uint64),
                                       POINTER(c_int), POINTER(c_uint64), POINTER(c_uint64)]
        L.orc_seek_next.argtypes = [c_void_p, c_uint64, c_uint64, c_uint64, POINTER(c_uint64), POINTER(c_void_p),
                                    POINTER(c_uint64), POINTER(c_int)]
        L.orc_snappy_decode.argtypes = [c_void_p, c_uint64, POINTER(c_void_p), POINTER(c_uint64)]
        L.orc_free.argtypes = [c_void_p]
        L.orc_file_header.argtypes = [c_void_p, c_uint64, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint64)]
        L.orc_parallel_read_at.restype = c_uint64
        L.orc_parallel_read_at.argtypes = [c_void_p, c_uint64, c_void_p, c_uint64, c_int]
        L.orc_sst_scan.restype = c_uint64
        L.orc_sst_scan.argtypes = [c_void_p, c_uint64, c_void_p, c_uint64, POINTER(c_uint64)]
        L.orc_crc64_iso.restype = c_uint64
        L.orc_crc64_iso.argtypes = [c_void_p, c_uint64]
        L.orc_index_entry.argtypes = [c_void_p, c_uint64, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64),
                                      POINTER(c_uint64)]
        L.orc_disk_index_search.argtypes = [c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, POINTER(c_uint64),
                                            POINTER(c_int), POINTER(c_uint64), POINTER(c_uint64)]
        L.orc_snappy_encode.restype = c_uint64
        L.orc_snappy_encode.argtypes = [c_void_p, c_void_p, c_uint64]
        L.orc_lzw_decode.argtypes = [c_void_p, c_uint64, POINTER(c_void_p), POINTER(c_uint64)]
        L.orc_lzw_encode.restype = c_uint64
        L.orc_lzw_encode.argtypes = [c_void_p, c_void_p, c_uint64]
        L.orc_encode_file.restype = c_uint64
        L.orc_encode_file.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p]
        _lib = L
    return _lib


def _buf(data):
    b = bytes(data)
    return ctypes.create_string_buffer(b, len(b) + 1), len(b)


def crc32c(data: bytes) -> int:
    b, n = _buf(data)
    return lib().orc_crc32c(b, n)


def file_reader_decode(data: bytes) -> dict:
    """FileReader ReadNext loop: records (bytes / None for nil) + terminal status."""
    b, n = _buf(data)
    r = OrcFileResult()
    lib().orc_file_reader_decode(b, n, byref(r))
    recs, rec_off = [], []
    for i in range(r.n_records):
        lo, hi = r.out_off[i], r.out_off[i + 1]
        if r.flags[i] & 2:
            recs.append(BadRecord("corrupt"))
        elif r.flags[i] & 4:
            recs.append(BadRecord("eof"))
        elif r.flags[i] & 1:
            recs.append(None)
        elif hi > lo:
            recs.append(ctypes.string_at(ctypes.addressof(r.out.contents) + lo, hi - lo))
        else:
            recs.append(b"")
        rec_off.append(r.rec_off[i])
    res = {"version": r.version, "compression": r.compression, "n_records": r.n_records,
           "total_out_bytes": r.total_out_bytes, "status": r.status, "status_offset": r.status_offset,
           "detail0": r.detail0, "detail1": r.detail1, "records": recs, "rec_off": rec_off,
           "first_bad": r.first_bad, "n_bad": r.n_bad}
    lib().orc_file_result_free(byref(r))
    return res


def file_reader_decode_arrays(data) -> dict:
    """Same as file_reader_decode, numpy arrays instead of per-record bytes (large files)."""
    import numpy as np

    arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data
    arr = np.ascontiguousarray(arr)
    r = OrcFileResult()
    lib().orc_file_reader_decode(arr.ctypes.data, arr.shape[0], byref(r))
    n, nb = r.n_records, r.total_out_bytes

    def cp(ptr, count, dt):
        if count == 0 or not ptr:  # file-header errors leave the arrays unallocated
            return np.zeros(count, dtype=dt)
        return np.ctypeslib.as_array(ptr, shape=(count,)).astype(dt, copy=True)

    res = {"status": r.status, "status_offset": r.status_offset, "n_records": n, "total_out_bytes": nb,
           "detail0": r.detail0, "detail1": r.detail1, "first_bad": r.first_bad, "n_bad": r.n_bad,
           "out": cp(r.out, nb, np.uint8), "out_off": cp(r.out_off, n + 1, np.int64),
           "rec_off": cp(r.rec_off, n, np.int64), "flags": cp(r.flags, n, np.uint8)}
    lib().orc_file_result_free(byref(r))
    return res


def read_next_at(data: bytes, offset: int, details: bool = False):
    """(status, record) of MMapReader.ReadNextAt; with details=True also (detail0, detail1)."""
    b, n = _buf(data)
    out, ol, nil, d0, d1 = c_void_p(), c_uint64(), c_int(), c_uint64(), c_uint64()
    st = lib().orc_read_next_at(b, n, offset, byref(out), byref(ol), byref(nil), byref(d0), byref(d1))
    rec = None
    if st == 0 and not nil.value:
        rec = ctypes.string_at(out.value, ol.value) if ol.value else b""
    if out.value:
        lib().orc_free(out)
    return (st, rec, d0.value, d1.value) if details else (st, rec)


def seek_next(data: bytes, offset: int, seek_len: int = 4096):
    """(status, record offset — the failing trial's on a trial error —, record)"""
    b, n = _buf(data)
    ro, out, ol, nil = c_uint64(), c_void_p(), c_uint64(), c_int()
    st = lib().orc_seek_next(b, n, offset, seek_len, byref(ro), byref(out), byref(ol), byref(nil))
    rec = None
    if st == 0 and not nil.value:
        rec = ctypes.string_at(out.value, ol.value) if ol.value else b""
    if out.value:
        lib().orc_free(out)
    return st, ro.value, rec


def snappy_decode(data: bytes):
    b, n = _buf(data)
    out, ol = c_void_p(), c_uint64()
    st = lib().orc_snappy_decode(b, n, byref(out), byref(ol))
    rec = ctypes.string_at(out.value, ol.value) if st == 0 and ol.value else (b"" if st == 0 else None)
    if out.value:
        lib().orc_free(out)
    return st, rec


def lzw_decode(data: bytes):
    """(status, bytes) of LzwCompressor.DecompressWithBuf (Go compress/lzw, LSB, litWidth 8)."""
    b, n = _buf(data)
    out, ol = c_void_p(), c_uint64()
    st = lib().orc_lzw_decode(b, n, byref(out), byref(ol))
    rec = ctypes.string_at(out.value, ol.value) if st == 0 and ol.value else (b"" if st == 0 else None)
    if out.value:
        lib().orc_free(out)
    return st, rec


def lzw_encode(data: bytes) -> bytes:
    """LzwCompressor.Compress (lzw.NewWriter(LSB, 8) + Write + Close)."""
    b, n = _buf(data)
    out = ctypes.create_string_buffer(2 * n + 16)
    k = lib().orc_lzw_encode(out, b, n)
    return out.raw[:k]


# ---------------------------------------------------------------------------------------------
# sstables (checker for the device scan): oracle recordio decode + proto.Unmarshal + CRC-64/ISO
# ---------------------------------------------------------------------------------------------
def crc64_iso(data: bytes) -> int:
    b, n = _buf(data)
    return lib().orc_crc64_iso(b, n)


def index_entry(rec: bytes):
    """proto.Unmarshal of one IndexEntry record -> (key, valueOffset, checksum), None if malformed."""
    b, n = _buf(rec or b"")
    ko, kl, vo, cs = c_uint64(), c_uint64(), c_uint64(), c_uint64()
    if lib().orc_index_entry(b, n, byref(ko), byref(kl), byref(vo), byref(cs)):
        return None
    r = bytes(rec or b"")
    return r[ko.value:ko.value + kl.value], vo.value, cs.value


class BadProto:
    """A v0 value record that is not a valid DataEntry (proto.Unmarshal's error)."""


def data_entry(rec):
    """proto.Unmarshal of one DataEntry record -> its value (None when absent), BadProto if malformed."""
    b, n = _buf(rec or b"")
    present, vo, vl = c_int(), c_uint64(), c_uint64()
    L = lib()
    L.orc_data_entry.argtypes = [c_void_p, c_uint64, POINTER(c_int), POINTER(c_uint64), POINTER(c_uint64)]
    if L.orc_data_entry(b, n, byref(present), byref(vo), byref(vl)):
        return BadProto()
    r = bytes(rec or b"")
    return r[vo.value:vo.value + vl.value] if present.value else None


def meta_version(base: str) -> int:
    """MetaData.version (field 7, sstable.proto:16-26) of meta.pb.bin; 0 when the file is absent
    (readMetaDataIfExists, sstable_reader.go:356-377). Wire format read field by field (varints,
    length-delimited and fixed fields skipped)."""
    p = os.path.join(base, "meta.pb.bin")
    if not os.path.exists(p):
        return 0
    b, i, ver = open(p, "rb").read(), 0, 0

    def varint():
        nonlocal i
        v = s = 0
        while True:
            c = b[i]
            i += 1
            v |= (c & 0x7F) << s
            s += 7
            if c < 0x80:
                return v
    while i < len(b):
        tag = varint()
        fn, wt = tag >> 3, tag & 7
        if wt == 0:
            v = varint()
            if fn == 7:
                ver = v
        elif wt == 2:
            ln = varint()  # (not `i += varint()`: that reads i before the call advances it)
            i += ln
        elif wt in (1, 5):
            i += 8 if wt == 1 else 4
        else:
            raise ValueError("meta.pb.bin: unexpected wire type")
    return ver


def sstable_oracle(base: str) -> dict:
    """NewSSTableReader + validateDataFile + Scan restated on the host: index entries in file order
    (SliceKeyIndexLoader.Load, slice_key_index.go:91-131), value at valueOffset via ReadNextAt
    (sstable_reader.go:80-117), CRC-64/ISO vs the stored checksum (0 = unchecked), and the scan's
    positional pairing of index entries with data records (sstable_iterator.go:77-111). v0 tables
    (metadata version 0): values are DataEntry records unwrapped by proto.Unmarshal, and
    validateDataFile does not run (sstable_reader.go:205-209): first_bad / value_bad stay None."""
    v0 = meta_version(base) == 0
    idx = file_reader_decode(open(os.path.join(base, "index.rio"), "rb").read())
    data_img = open(os.path.join(base, "data.rio"), "rb").read()
    dat = file_reader_decode(data_img)
    if v0:
        dat["records"] = [r if isinstance(r, BadRecord) else data_entry(r) for r in dat["records"]]
    entries, bad_proto, index_bad = [], None, None
    for i, r in enumerate(idx["records"]):
        if isinstance(r, BadRecord):  # Load's ReadNext error; gzip's bare io.EOF ends the loop
            index_bad = i if r.kind == "corrupt" else None
            break
        e = index_entry(r)
        if e is None:
            bad_proto = i
            break
        entries.append(e)
    first_bad = unplaced = value_bad = None
    crcs = []
    at = {o: j for j, o in enumerate(dat["rec_off"])}  # ReadNextAt at a record start = that record
    for i, (k, vo, cs) in enumerate(entries):
        j = at.get(vo)
        if j != i and unplaced is None:
            unplaced = i
        val = dat["records"][j] if j is not None else None
        if isinstance(val, (BadRecord, BadProto)):  # getValueAtOffset's ReadNextAt / Unmarshal error (:79-94)
            crcs.append(None)
            if value_bad is None and not v0:
                value_bad = i
            continue
        c = crc64_iso(val or b"")
        crcs.append(c)
        if first_bad is None and cs != 0 and c != cs and not v0:
            first_bad = i
    return {"index_status": idx["status"], "data_status": dat["status"], "entries": entries,
            "bad_proto": bad_proto, "index_bad": index_bad, "values": dat["records"], "crcs": crcs,
            "first_bad": first_bad, "value_bad": value_bad, "unplaced": unplaced, "v0": v0}


def disk_index_search(index: bytes, key: bytes, seek_len: int = 4096):
    """DiskKeyIndex.binarySearch restatement on a fresh index: (status, offset, found, valueOffset, checksum)."""
    b, n = _buf(index)
    off, vo, cs = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    found = ctypes.c_int()
    kb = bytes(key) or b"\0"
    st = lib().orc_disk_index_search(b, n, kb, len(key), seek_len, byref(off), byref(found), byref(vo), byref(cs))
    return st, off.value, bool(found.value), vo.value, cs.value


def seek_next_entries(index: bytes, start: int, end: int):
    """DiskKeyIndexIterator.Next loop (disk_key_index.go:141-165) with the oracle's SeekNext: keys."""
    out, cur = [], start
    while cur <= end:
        st, ro, rec = seek_next(index, cur)
        if st != 0:
            break
        out.append(index_entry(rec or b"")[0])
        cur = ro + 1
    return out


def encode_file(records, comp):
    """FileWriter.Write over a batch (oracle restatement): (file bytes, record offsets)."""
    import numpy as np

    n = len(records)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([0 if r is None else len(r) for r in records], out=off[1:])
    blob = b"".join(r or b"" for r in records) + b"\0"
    flags = np.array([1 if r is None else 0 for r in records] + [0], dtype=np.uint8)
    cap = 8 + n * 40 + int(off[-1]) * 3 // 2 + 32 * n + 64  # lzw: <= 12 bits per byte
    out = ctypes.create_string_buffer(cap)
    roff = np.zeros(max(n, 1), dtype=np.uint64)
    ln = lib().orc_encode_file(blob, off.ctypes.data, flags.ctypes.data, n, comp, out, cap, roff.ctypes.data)
    assert ln
    return out.raw[:ln], [int(x) for x in roff[:n]]
