"""The lane walk (k_walk_lane, RIO_WALK_LANE=1): framing by one lane per small chunk (the serial
FileReader walk, common_reader.go:110-151 / file_reader.go:61-131, per chunk) must give exactly the
oracle's records, offsets, flags, statuses and status offsets, like the wave walk (k_walk) does:
on every fixture and corpus case at several chunk sizes (speculation granularity), with the
scan's repairs, and at the BASELINE sizes (C2, C2-ref-random, C3, one C4 file)."""
import ctypes
import os

import numpy as np
import pytest

import corpus
import oracle_py as orc
from conftest import GOLDEN, STATUS, read_fixture
from gpu_util import assert_same_as_oracle

pytestmark = pytest.mark.gpu

CASES = corpus.cases()


def _lane_decoder(monkeypatch, chunk):
    from recordio import _lib as L
    from recordio.device import DeviceDecoder

    monkeypatch.setenv("RIO_WALK_LANE", "1")
    monkeypatch.setenv("RIO_LANE_CHUNK_BYTES", str(chunk))
    dec = DeviceDecoder(0, own_ctx=True)  # the context reads the framing knobs when it is created
    assert L.lib().rio_ctx_device(dec.ctx) == 0
    return dec


def _decode(dec, img) -> dict:
    from recordio.device import to_device_file

    d_file, n = to_device_file(img)
    b, info = dec.decode(d_file, n)
    k = info["n_records"]
    return dict(info, out=b.out[: info["total_out_bytes"]].cpu().numpy(), out_off=b.out_off[: k + 1].cpu().numpy(),
                rec_off=b.rec_off[:k].cpu().numpy(), flags=b.flags[:k].cpu().numpy())


def _fixtures():
    out = []
    for vd in ("v4_compat", "v3_compat", "v2_compat", "v1_compat"):
        for name in sorted(os.listdir(os.path.join(GOLDEN, vd))):
            out.append((f"{vd}/{name}", read_fixture(vd, name)))
    return out


def _check(dec, name, img):
    o = orc.file_reader_decode_arrays(img)
    g = _decode(dec, img)
    if o["status"] in (STATUS["VERSION"], STATUS["COMPRESSION_TYPE"], STATUS["SHORT_FILE_HEADER"]):
        assert g["status"] == o["status"], name
        return g
    assert_same_as_oracle(g, o, name)
    return g


@pytest.mark.parametrize("chunk", [64, 512, 4096, 65536])
def test_fixtures_and_corpus(chunk, monkeypatch):
    """Every golden fixture (v1..v4) and every corpus case (truncations, bit flips, zero and garbage
    tails, embedded files, non-canonical varints, codec errors, nil and empty records)."""
    dec = _lane_decoder(monkeypatch, chunk)
    for name, img in _fixtures() + list(CASES):
        _check(dec, f"{name}@{chunk}", img)


def test_repairs_happen_and_stay_exact(monkeypatch):
    """CRC-valid false headers inside payloads (embedded recordio files) at chunk starts: a lane's
    speculative entry breaks, the scan repairs it, the result is the oracle's."""
    dec = _lane_decoder(monkeypatch, 4096)
    for name in ("mixed_c0_embedded", "v2_embedded_same", "v1_embedded_same"):
        g = _check(dec, name, dict(CASES)[name])
        assert g["n_repairs"] > 0, name


@pytest.mark.parametrize("n,rec,kind,seed", [(1_000_000, 1024, 1, 1), (1_000_000, 1024, 0, 1), (10_000_000, 64, 1, 3),
                                             (16_384, 65536, 1, 100)],
                         ids=["c2", "c2-ref-random", "c3", "c4-file"])
def test_baseline_sizes_exact(n, rec, kind, seed, monkeypatch):
    """The bench workloads at full size: every byte and offset equals the oracle."""
    dec = _lane_decoder(monkeypatch, 4096)
    img = corpus.generate(n, rec, 2, kind=kind, seed=seed)
    g = _check(dec, f"{n}x{rec}/{kind}", img)
    assert g["status"] == STATUS["EOF"] and g["n_records"] == n
    assert np.all(np.diff(g["rec_off"]) > 0)


@pytest.mark.parametrize("version", [3, 2, 1])
def test_older_layouts_full_size(version, monkeypatch):
    """C2 re-framed with the v3 / v2 / v1 header layouts (no header CRC below v4: more false
    candidates for the speculative entries)."""
    dec = _lane_decoder(monkeypatch, 4096)
    img = corpus.to_version(bytes(corpus.generate(200_000, 1024, 2, kind=1, seed=5)), version)
    g = _check(dec, f"C2 v{version}", img)
    assert g["n_records"] == 200_000


def test_auto_walk_follows_the_previous_decode(monkeypatch):
    """RIO_WALK_LANE unset (auto): a context's decode takes the lane walk (16 KiB chunks, info.n_chunks shows
    which) when its previous decode had records of 768 B .. 8 KiB on average and the file fills 32768 lane
    chunks, else the wave walk (32 KiB chunks; a smaller file walks the smallest 4 KiB multiple whose chunks fit one
    round of resident walk waves, at least 8 KiB: wave_cb). DeviceDecoder.decode runs a capacity probe first, which
    records the file's mean for the real decode: a fresh context's first file is framed by the wave walk in the
    probe only. Every decode is the oracle's."""
    from recordio.device import DeviceDecoder

    monkeypatch.delenv("RIO_WALK_LANE", raising=False)
    monkeypatch.delenv("RIO_LANE_CHUNK_BYTES", raising=False)
    dec = DeviceDecoder(0, own_ctx=True)
    big = corpus.generate(600_000, 1024, 2, kind=0, seed=7)  # incompressible 1 KiB records, >= 32768 lane chunks
    small = corpus.generate(200_000, 64, 2, kind=1, seed=8)
    chunks = lambda img, cb: (len(img) - 8 + cb - 1) // cb  # noqa: E731

    import torch

    slots = torch.cuda.get_device_properties(0).multi_processor_count * 4 * 5

    def wave_cb(img):  # rio_capi.cpp wave_chunk_bytes: one round of resident walk waves, 4 KiB multiples
        want = ((len(img) + slots - 1) // slots + 4095) // 4096 * 4096
        return min(32768, max(want, 8192))

    got = []
    short = corpus.generate(40_000, 1024, 2, kind=0, seed=9)  # large records, too few lane chunks
    for img in (big, big, small, small, big, short):
        g = _check(dec, "auto", img)
        got.append(g["n_chunks"])
    assert wave_cb(big) == 32768 and wave_cb(small) < 32768 and wave_cb(short) < 32768
    assert got == [chunks(big, 16384), chunks(big, 16384), chunks(small, wave_cb(small)),
                   chunks(small, wave_cb(small)), chunks(big, 16384), chunks(short, wave_cb(short))]
