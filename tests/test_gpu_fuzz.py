"""Seeded fuzz parity for the §8f components (GPU): random damage or random shapes, device result
against the oracle (or the reference's own loop) on every case.

- WAL replay: a directory of random files with one byte range overwritten at a random place; the
  device pipeline and the reference loop over the FileReader mirror must deliver the same records and
  the same error text.
- DiskKeyIndex: random bytes of an index file overwritten; every query's hit equals the oracle's.
- Encoder: random mixes of record sizes (0 .. 200 KiB) and contents; byte-identical to the oracle.
- SSTable load: random damage to data.rio / index.rio; the device reader fails or succeeds as the
  oracle's restatement says, with the same first bad entry."""
import os
import random
import struct

import pytest

import oracle_py as orc
from corpus import mixed_records
from recordio import encode_file

pytestmark = pytest.mark.gpu


def damage(rng, img, lo=8):
    b = bytearray(img)
    if len(b) <= lo + 1:
        return bytes(b)
    p = rng.randrange(lo, len(b))
    n = rng.randint(1, 6)
    kind = rng.random()
    for k in range(p, min(len(b), p + n)):
        b[k] = rng.getrandbits(8) if kind < 0.6 else (0x91 if kind < 0.8 else 0)
    if rng.random() < 0.15:
        del b[rng.randrange(lo, len(b)):]  # truncation
    return bytes(b)


@pytest.mark.parametrize("seed", range(30))
def test_wal_replay_damage(tmp_path, seed):
    import test_gpu_wal as T

    rng = random.Random(seed)
    files = [encode_file(mixed_records(rng.randint(5, 80), seed * 7 + f, max_len=700), rng.choice([0, 2]))
             for f in range(rng.randint(2, 5))]
    k = rng.randrange(len(files))
    files[k] = damage(rng, files[k])
    d = tmp_path / "w"
    d.mkdir()
    for i, img in enumerate(files):
        (d / ("%06d.wal" % i)).write_bytes(img)
    exp, _, _ = T.expected(str(d))
    got, _ = T.both_paths_agree(str(d))
    assert got == exp


@pytest.mark.parametrize("seed", range(30))
def test_disk_index_damage(seed):
    import test_gpu_disk_index as T

    rng = random.Random(100 + seed)
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 16))) for _ in range(400)})
    idx = damage(rng, T.index_image(T.entries_for(keys, nil_every=rng.choice([0, 13]))))
    T.check(idx, T.queries_for(keys, rng, 60), rng.choice([0, 3, 64]))


@pytest.mark.parametrize("seed", range(10))
def test_encoder_random_shapes(seed):
    import test_gpu_encode as T

    rng = random.Random(200 + seed)
    recs = []
    for _ in range(rng.randint(1, 400)):
        r = rng.random()
        n = rng.choice([0, 1, 16, 17, 60, 1023, 1024, 1025, rng.randint(0, 5000), rng.randint(60000, 200000)])
        if r < 0.1:
            recs.append(None)
        elif r < 0.4:
            recs.append(bytes(rng.getrandbits(8) for _ in range(min(n, 3000))))
        else:
            base = b" ".join(rng.choice([b"alpha", b"beta", b"\x91\x8d\x4c", b"zz", b"0123456789"]) for _ in range(n // 4 + 1))
            recs.append(base[:n])
    for comp in (0, 2):
        img, offs = T.device_encode(recs, comp)
        want, want_offs = orc.encode_file(recs, comp)
        assert img == want and offs == want_offs


@pytest.mark.parametrize("seed", range(30))
def test_sstable_damage(tmp_path, seed):
    import sstables as S
    import test_gpu_sstable as T
    from sstables.writer import crc64_iso

    rng = random.Random(300 + seed)
    items = [(struct.pack(">I", i), bytes(rng.getrandbits(8) % 7 + 97 for _ in range(rng.randint(0, 300))))
             for i in range(rng.randint(5, 200))]
    base = str(tmp_path / "t")
    T.write_triples(base, [(k, v, crc64_iso(v)) for k, v in items], rng.choice([0, 2]))
    which = rng.choice(["data.rio", "index.rio"])
    p = os.path.join(base, which)
    with open(p, "rb") as fh:
        img = fh.read()
    with open(p, "wb") as fh:
        fh.write(damage(rng, img))
    o = orc.sstable_oracle(base)
    r, err = S.NewSSTableReader(S.ReadBasePath(base))
    # the mirror's checks in order (sstables/__init__.py NewSSTableReader): index reading error,
    # malformed IndexEntry, index not in the writer's layout (handed back), value checksum mismatch
    fails = (o["index_status"] not in (1, 2, 3, 4) or o["bad_proto"] is not None or o["unplaced"] is not None
             or o["first_bad"] is not None or o["index_bad"] is not None or o["value_bad"] is not None)
    assert (r is None) == fails, (o["index_status"], o["bad_proto"], o["unplaced"], o["first_bad"], err)
    if fails:
        assert err is not None
        if (o["index_status"] in (1, 2, 3, 4) and o["bad_proto"] is None and o["unplaced"] is None
                and o["index_bad"] is None):
            i, vb = o["first_bad"], o["value_bad"]
            if vb is not None and (i is None or vb <= i):  # validateDataFile meets the read error first
                assert f"while getting value at offset {o['entries'][vb][1]}: failed decompressing" in str(err)
            else:
                assert f"Checksum mismatch: expected {o['entries'][i][2]:x}, got {o['crcs'][i]:x}" in str(err)
        return
    got, serr = T.scan_all(r)
    n = len(o["entries"])
    assert got == [(e[0], v) for e, v in zip(o["entries"], o["values"])][:len(got)]
    assert len(got) == min(n, len(o["values"]))


@pytest.mark.parametrize("seed", range(40))
def test_older_versions_damage(seed, tmp_path):
    """Whole-file decode of damaged v3 / v2 / v1 files (random bytes, 0x91 runs, zeros, truncation;
    the damage lands in headers and payloads alike): device == the oracle's ReadNext loop, and
    ReadNextAt / SeekNext at a sample of offsets == the oracle's."""
    import corpus
    from gpu_util import assert_same_as_oracle, gpu_decode_arrays

    rng = random.Random(500 + seed)
    version = (3, 2, 1)[seed % 3]
    comp = rng.choice([0, 2])
    recs = [r if r is not None else b"" for r in mixed_records(rng.randint(20, 400), 900 + seed, max_len=900)]
    img = corpus.legacy_file(recs, comp, version) if version < 3 else corpus.to_version(encode_file(recs, comp), 3)
    for _ in range(rng.randint(1, 3)):
        img = damage(rng, img)
    assert_same_as_oracle(gpu_decode_arrays(img), orc.file_reader_decode_arrays(img), f"v{version} seed {seed}")
    from recordio import NewMemoryMappedReaderWithPath

    p = tmp_path / "f"
    p.write_bytes(img)
    r, _ = NewMemoryMappedReaderWithPath(str(p))
    assert r.Open() is None or len(img) < 8 or img[0] not in (1, 2, 3)
    if r.header is None:
        return
    for off in [rng.randrange(len(img) + 2) for _ in range(40)]:
        st, want = orc.read_next_at(img, off)
        got, err = r.ReadNextAt(off)
        assert (err is None) == (st == 0), (off, st, err)
        if st == 0:
            assert got == want, off
        st, ro, want = orc.seek_next(img, off)
        g_off, got, err = r.SeekNext(off)
        assert (err is None) == (st == 0), (off, st, err)
        if st == 0:
            assert (g_off, got) == (ro, want), off
    r.Close()
