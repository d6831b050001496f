"""librio.so loads and exports every symbol include/rio.h declares (CPU; no compute calls)."""
import ctypes
import os
import re

from conftest import REPO

from recordio import _lib as L


def _declared():
    src = open(os.path.join(REPO, "include", "rio.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(rio_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_every_declared_symbol_exported():
    lib = ctypes.CDLL(L.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(_declared()) <= set(L.EXPORTED) | {"rio_device_count"}


def test_status_vocabulary():
    lib = L.lib()
    assert lib.rio_strerror(L.RIO_ERR_MAGIC) == b"magic number mismatch"
    assert lib.rio_strerror(L.RIO_ERR_HEADER_CRC) == b"header checksum mismatch"
    for s in (L.RIO_EOF, L.RIO_EOF_ZERO_TAIL, L.RIO_EOF_HEADER, L.RIO_EOF_PAYLOAD, L.RIO_EOF_CODEC):
        assert lib.rio_status_is_eof(s)
    for s in (L.RIO_OK, L.RIO_ERR_UNEXPECTED_EOF, L.RIO_ERR_MAGIC, L.RIO_ERR_HEADER_CRC):
        assert not lib.rio_status_is_eof(s)
    assert lib.rio_max_records(8 + 600) == 121  # 600 / 5 + 1: v2's 5-byte empty records


def test_code_object_targets_gfx950():
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_stream_and_replay_argument_errors():
    """Host-side argument and I/O errors of the windowed / replay handles come back before any
    device call (no GPU needed): null handles, a missing path, a directory."""
    lib = L.lib()
    h = ctypes.c_void_p()
    assert lib.rio_stream_open(0, None, 0, 0, ctypes.byref(h)) == L.RIO_ERR_ARG
    assert lib.rio_stream_open(0, b"/nonexistent/file.rio", 0, 0, ctypes.byref(h)) == L.RIO_ERR_IO
    assert lib.rio_stream_open(0, REPO.encode(), 0, 0, ctypes.byref(h)) == L.RIO_ERR_IO  # not a regular file
    assert not h.value
    assert lib.rio_stream_open_host(0, None, 5, 0, 0, ctypes.byref(h)) == L.RIO_ERR_ARG
    assert lib.rio_host_register(None, 5) == L.RIO_ERR_ARG
    assert lib.rio_host_unregister(None) == L.RIO_ERR_ARG
    assert lib.rio_stream_next(None, None, None, None, None, None, None) == L.RIO_ERR_ARG
    lib.rio_stream_free(None)
    assert lib.rio_replay_next(None, None, None, None, None, None) == L.RIO_ERR_ARG
    lib.rio_replay_free(None)
