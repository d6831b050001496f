"""recordio v4 encoding on the device (GPU): rio_encode_file / rio_device_encode vs the reference
writer. The reference's own v4 fixtures pin the expected bytes directly where they exist
(recordio/test_files/v4_compat, written by FileWriter with golang/snappy v1.0.0). Elsewhere the
expected bytes come from the oracle's restatement (oracle/rio_oracle.c orc_encode_file) and the host
writer, both pinned to the same fixtures by tests/test_writer.py. Plus round trips through the
device decoder."""
import ctypes
import random

import numpy as np
import pytest

import oracle_py as orc

from conftest import read_fixture
from corpus import mixed_records, text_records
from recordio import _lib as L
from recordio import encode_file
from gpu_util import gpu_decode_arrays

pytestmark = pytest.mark.gpu


def asc(n):
    return bytes(i & 0xFF for i in range(n))


def device_encode(records, comp):
    """rio_encode_file: (file image, record offsets)."""
    n = len(records)
    lens = [0 if r is None else len(r) for r in records]
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    blob = b"".join(r or b"" for r in records) + b"\0"
    flags = np.array([1 if r is None else 0 for r in records] + [0], dtype=np.uint8)
    cap = int(L.lib().rio_encode_bound(n, int(off[-1]), comp))
    out = ctypes.create_string_buffer(cap)
    roff = np.zeros(max(n, 1), dtype=np.uint64)
    ln = ctypes.c_uint64()
    rc = L.lib().rio_encode_file(L.default_ctx(0), blob, off.ctypes.data, flags.ctypes.data, n, comp, out, cap,
                                 roff.ctypes.data, ctypes.byref(ln))
    assert rc == 0, L.strerror(rc)
    return out.raw[:ln.value], [int(x) for x in roff[:n]]


@pytest.mark.parametrize("name,records,comp", [
    ("recordio_UncompressedSingleRecord", [asc(13)], 0),
    ("recordio_UncompressedWriterMultiRecord_asc", [asc(i) for i in range(255)], 0),
    ("recordio_SnappyWriterMultiRecord_asc", [asc(i) for i in range(255)], 2),
    ("recordio_UncompressedSingleRecord_comp2", [asc(1337)], 2),
    ("recordio_UncompressedNilAndEmptyRecord", [None, b""], 0),
    ("recordio_UncompressedMagicNumberContent", [b"\x91\x8d\x4c", bytes([21, 8, 23]), b"\x91\x8d\x4c"], 0),
])
def test_byte_identical_to_reference_fixtures(name, records, comp):
    img, _ = device_encode(records, comp)
    assert img == read_fixture("v4_compat", name)


@pytest.mark.parametrize("comp", [0, 2])
@pytest.mark.parametrize("kind", ["mixed", "text", "random", "tiny", "big"])
def test_byte_identical_to_writer(comp, kind):
    rng = random.Random(comp * 100 + ["mixed", "text", "random", "tiny", "big"].index(kind))
    if kind == "mixed":
        recs = mixed_records(3000, seed=11, max_len=5000)
    elif kind == "text":
        recs = text_records(2000, seed=12, lo=1, hi=3000)
    elif kind == "random":
        recs = [bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 2000))) for _ in range(300)]
    elif kind == "tiny":
        recs = [bytes(rng.getrandbits(8) % 3 for _ in range(rng.randint(0, 20))) for _ in range(2000)]
    else:  # several 64 KiB blocks per record, and the 1 KiB LDS / global table boundary
        base = b"".join(text_records(200, seed=13, lo=500, hi=1500))
        recs = [base[:1024], base[:1025], base[:65536], base[:65537], base[:200000], bytes(150000), None, b""]
    img, offs = device_encode(recs, comp)
    want, want_offs = orc.encode_file(recs, comp)
    assert len(img) == len(want)
    assert img == want
    assert img == encode_file(recs, comp)
    assert offs == want_offs


@pytest.mark.parametrize("comp", [0, 2])
def test_round_trip_through_device_decode(comp):
    recs = mixed_records(5000, seed=21, max_len=4000)
    img, _ = device_encode(recs, comp)
    g = gpu_decode_arrays(np.frombuffer(img, dtype=np.uint8))
    assert g["n_records"] == len(recs)
    out = g["out"].tobytes()
    for i, r in enumerate(recs):
        lo, hi = int(g["out_off"][i]), int(g["out_off"][i + 1])
        if r is None:
            assert g["flags"][i] & 1
        else:
            assert out[lo:hi] == r


def test_empty_batch():
    img, offs = device_encode([], 2)
    assert img == encode_file([], 2) and offs == []
