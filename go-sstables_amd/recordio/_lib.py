"""ctypes binding of librio.so (include/rio.h).

The library is built in-tree (go-sstables_amd/librio.so) by __graft_entry__.build() /
`make -C go-sstables_amd/csrc`. Loading it needs no GPU; every decode entry point needs one and
fails loudly (RIO_ERR_HIP) without it. There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# RIO_LIB_PATH: load an experiment build (csrc/Makefile `variant`) instead of the in-tree library
LIB_PATH = os.environ.get("RIO_LIB_PATH") or os.path.normpath(os.path.join(_HERE, "..", "librio.so"))

# status codes (rio.h rio_status)
RIO_OK = 0
RIO_EOF = 1
RIO_EOF_ZERO_TAIL = 2
RIO_EOF_HEADER = 3
RIO_EOF_PAYLOAD = 4
RIO_ERR_UNEXPECTED_EOF = 5
RIO_ERR_MAGIC = 6
RIO_ERR_HEADER_CRC = 7
RIO_ERR_VARINT_OVERFLOW = 8
RIO_ERR_HEADER_TOO_LONG = 9
RIO_ERR_DECOMPRESS = 10
RIO_ERR_VERSION = 11
RIO_ERR_COMPRESSION_TYPE = 12
RIO_ERR_SHORT_FILE_HEADER = 13
RIO_ERR_INVALID_OFFSET = 14
RIO_ERR_UNSUPPORTED = 15
RIO_ERR_CAPACITY = 16
RIO_ERR_ARG = 17
RIO_ERR_HIP = 18
RIO_ERR_STATE = 19
RIO_ERR_IO = 20
RIO_ERR_PROTO = 21
RIO_EOF_CODEC = 22

EOF_CLASS = (RIO_EOF, RIO_EOF_ZERO_TAIL, RIO_EOF_HEADER, RIO_EOF_PAYLOAD, RIO_EOF_CODEC)

RIO_FLAG_NIL = 1
RIO_FLAG_CORRUPT = 2
RIO_FLAG_EOF = 4
RIO_DEVICE_PAD = 64
RIO_VALUE_NIL = 0xFFFFFFFFFFFFFFFF  # rio_sst_data_entries: DataEntry without a value field
RIO_VALUE_BAD = 0xFFFFFFFFFFFFFFFE  # rio_sst_data_entries: not a valid DataEntry
RIO_SST_V0_VALUES = 1
RIO_COMP_UNKNOWN = 0xFFFFFFFF
COMP_NONE, COMP_GZIP, COMP_SNAPPY, COMP_LZW = 0, 1, 2, 3


class FileInfo(ctypes.Structure):
    _fields_ = [
        ("version", c_uint32),
        ("compression", c_uint32),
        ("n_records", c_uint64),
        ("total_out_bytes", c_uint64),
        ("status", ctypes.c_int32),
        ("reserved0", c_uint32),
        ("status_offset", c_uint64),
        ("detail0", c_uint64),
        ("detail1", c_uint64),
        ("n_chunks", c_uint64),
        ("n_repairs", c_uint64),
        ("first_bad", c_uint64),
        ("n_bad", c_uint64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved0"}


class SstInfo(ctypes.Structure):
    """rio_sst_info (include/rio.h)."""

    _fields_ = [
        ("index", FileInfo),
        ("data", FileInfo),
        ("n_entries", c_uint64),
        ("first_bad_proto", c_uint64),
        ("first_bad_crc", c_uint64),
        ("first_unplaced", c_uint64),
        ("index_bad", c_uint64),
        ("first_bad_value", c_uint64),
    ]


class IndexHit(ctypes.Structure):
    """rio_index_hit (include/rio.h)."""

    _fields_ = [
        ("offset", c_uint64),
        ("value_offset", c_uint64),
        ("checksum", c_uint64),
        ("status", ctypes.c_int32),
        ("found", ctypes.c_int32),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "rio_strerror": (c_char_p, [c_int]),
    "rio_status_is_eof": (c_int, [c_int]),
    "rio_build_info": (c_char_p, []),
    "rio_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "rio_ctx_destroy": (None, [c_void_p]),
    "rio_ctx_device": (c_int, [c_void_p]),
    "rio_ctx_acquire": (c_int, [c_int, POINTER(c_void_p)]),
    "rio_ctx_release": (None, [c_void_p]),
    "rio_device_count": (c_int, [POINTER(c_int)]),
    "rio_frame": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(FileInfo)]),
    "rio_host_register": (c_int, [c_void_p, c_uint64]),
    "rio_host_unregister": (c_int, [c_void_p]),
    "rio_decode": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_uint64, POINTER(FileInfo)]),
    "rio_device_decode": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p],
    ),
    "rio_device_decode_ex": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
         c_void_p],
    ),
    "rio_ctx_reserve": (c_int, [c_void_p, c_uint64, c_uint64, c_uint32]),
    "rio_ctx_arena_bytes": (c_uint64, [c_void_p]),
    "rio_device_decode_batch": (
        c_int,
        [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p],
    ),
    "rio_max_records": (c_uint64, [c_uint64]),
    "rio_ctx_last_stage_ms": (c_int, [c_void_p, POINTER(c_float), c_int]),
    "rio_ctx_set_timing": (c_int, [c_void_p, c_int]),
    "rio_device_read_at": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_uint64, POINTER(c_uint64), POINTER(c_int),
         POINTER(c_uint64), POINTER(c_uint64)],
    ),
    "rio_reader_new_file": (c_int, [c_void_p, c_char_p, POINTER(c_void_p)]),
    "rio_reader_new_mmap": (c_int, [c_void_p, c_char_p, POINTER(c_void_p)]),
    "rio_reader_open": (c_int, [c_void_p]),
    "rio_reader_close": (c_int, [c_void_p]),
    "rio_reader_free": (None, [c_void_p]),
    "rio_reader_header": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
    "rio_reader_size": (c_uint64, [c_void_p]),
    "rio_reader_last_detail": (None, [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)]),
    "rio_reader_read_next": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint64), POINTER(c_int)]),
    "rio_reader_skip_next": (c_int, [c_void_p]),
    "rio_reader_read_next_at": (c_int, [c_void_p, c_uint64, POINTER(c_void_p), POINTER(c_uint64), POINTER(c_int)]),
    "rio_reader_seek_next": (
        c_int, [c_void_p, c_uint64, POINTER(c_uint64), POINTER(c_void_p), POINTER(c_uint64), POINTER(c_int)]),
    "rio_reader_set_seek_len": (c_int, [c_void_p, c_uint64]),
    "rio_reader_file_info": (c_int, [c_void_p, POINTER(FileInfo)]),
    "rio_writer_new": (c_int, [c_char_p, c_uint32, POINTER(c_void_p)]),
    "rio_writer_write": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "rio_writer_size": (c_uint64, [c_void_p]),
    "rio_writer_close": (c_int, [c_void_p]),
    "rio_encode_record_v4": (c_uint64, [c_void_p, c_uint64, c_uint32, c_void_p, c_uint64]),
    "rio_encode_file_header": (None, [c_void_p, c_uint32, c_uint32]),
    "rio_snappy_max_encoded_len": (c_uint64, [c_uint64]),
    "rio_snappy_encode": (c_uint64, [c_void_p, c_uint64, c_void_p, c_uint64]),
    "rio_generate": (c_uint64, [c_void_p, c_uint64, c_uint32, c_uint64, c_uint64, c_int, c_uint64, c_int]),
    "rio_generate_bound": (c_uint64, [c_uint32, c_uint64, c_uint64]),
    "rio_sst_index_parse": (
        c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "rio_sst_validate": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "rio_sst_data_entries": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "rio_sst_validate_view": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p,
         c_void_p]),
    "rio_sst_open": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, POINTER(c_void_p), POINTER(SstInfo)]),
    "rio_sst_open_ex": (
        c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint32, POINTER(c_void_p), POINTER(SstInfo)]),
    "rio_sst_entry": (
        c_int,
        [c_void_p, c_uint64, POINTER(c_void_p), POINTER(c_uint64), POINTER(c_void_p), POINTER(c_uint64), POINTER(c_int),
         POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint64)]),
    "rio_sst_free": (None, [c_void_p]),
    "rio_replay_open": (c_int, [c_int, c_void_p, c_uint64, c_uint32, c_uint32, POINTER(c_void_p)]),
    "rio_replay_next": (
        c_int, [c_void_p, POINTER(c_uint64), POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p), POINTER(FileInfo)]),
    "rio_replay_free": (None, [c_void_p]),
    "rio_replay_open_devices": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64, c_uint32, c_uint32, POINTER(c_void_p)]),
    "rio_fileset_decode": (c_int, [c_void_p, c_uint32, c_void_p, c_uint64, POINTER(c_void_p)]),
    "rio_fileset_get": (c_int, [c_void_p, c_uint64, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p),
                                POINTER(c_void_p), POINTER(FileInfo), POINTER(c_int)]),
    "rio_fileset_free": (None, [c_void_p]),
    "rio_stream_open": (c_int, [c_int, c_char_p, c_uint64, c_uint32, POINTER(c_void_p)]),
    "rio_stream_open_host": (c_int, [c_int, c_void_p, c_uint64, c_uint64, c_uint32, POINTER(c_void_p)]),
    "rio_stream_next": (c_int, [c_void_p, POINTER(c_uint64), POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p),
                                POINTER(c_void_p), POINTER(FileInfo)]),
    "rio_stream_free": (None, [c_void_p]),
    "rio_reader_set_window": (c_int, [c_void_p, c_uint64]),
    "rio_encode_bound": (c_uint64, [c_uint64, c_uint64, c_uint32]),
    "rio_device_encode": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p,
                c_void_p, c_void_p]),
    "rio_encode_file": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p,
                POINTER(c_uint64)]),
    "rio_device_index_search": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "rio_index_open": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_void_p)]),
    "rio_index_search": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "rio_index_free": (None, [c_void_p]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def lib():
    """Load librio.so (in-tree). Raises if it has not been built: there is no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"librio.so not built at {LIB_PATH}: run `make -C go-sstables_amd/csrc` "
                "(or __graft_entry__.build()); the recordio GPU path has no CPU fallback")
        # One HIP runtime per process: torch bundles its own libamdhip64 under the same soname as
        # the ROCm one librio.so links. Whichever loads first is used by both; if librio's loads
        # first, torch later finds no GPU. So when torch is present (the Python mirror uses it for
        # device buffers), it is imported before the library.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("RIO_LIB_PATH") and not hasattr(L, name):
                continue  # an older experiment build (A/B timing) may predate some entry points
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def strerror(status: int) -> str:
    return lib().rio_strerror(status).decode()


_ctx = {}


def default_ctx(device: int = 0) -> int:
    """A per-device rio_ctx (created lazily; needs a GPU)."""
    if device not in _ctx:
        h = c_void_p()
        rc = lib().rio_ctx_create(device, ctypes.byref(h))
        if rc != RIO_OK:
            raise RuntimeError(f"rio_ctx_create(device={device}) failed: {strerror(rc)} "
                               "(the recordio decode path needs a HIP device)")
        _ctx[device] = h.value
    return _ctx[device]
