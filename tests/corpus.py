"""Crafted recordio files for parity tests: workloads, edge cases and corruptions.

Every case is decoded by the oracle (the checker) and by the device path; the tests compare the
two bit-exactly. Builders only produce bytes; nothing here decodes.
"""
import random
import struct

from recordio import encode_file, generate


def uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def padded_uvarint(v: int, n: int) -> bytes:
    """Non-canonical n-byte encoding of v (legal for Go's ReadUvarint)."""
    b = bytearray()
    for i in range(n):
        last = i == n - 1
        b.append((v & 0x7F) | (0 if last else 0x80))
        v >>= 7
    return bytes(b)


def crc32c(b: bytes) -> int:
    c = 0xFFFFFFFF
    for x in b:
        c ^= x
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 & -(c & 1))
    return c ^ 0xFFFFFFFF


def header_v4(u, c, nil=False, magic=b"\x91\x8d\x4c", u_bytes=None, c_bytes=None, crc_bytes=None):
    pre = magic + bytes([1 if nil else 0]) + (u_bytes or uvarint(u)) + (c_bytes or uvarint(c))
    return pre + (crc_bytes if crc_bytes is not None else uvarint(crc32c(pre)))


def header_v3(u, c, nil=False, magic=b"\x91\x8d\x4c"):
    return magic + bytes([1 if nil else 0]) + uvarint(u) + uvarint(c)


def header_v2(u, c):
    """readRecordHeaderV2 (common_reader.go:61-81): magic, u, c varints; no nil byte, no CRC."""
    return b"\x91\x8d\x4c" + uvarint(u) + uvarint(c)


def header_v1(u, c, magic=0x130691):
    """readRecordHeaderV1 (common_reader.go:46-59): LE u32 magic, LE u64 u, LE u64 c."""
    return struct.pack("<IQQ", magic, u, c)


def header_for(version, u, c, nil=False):
    if version == 4:
        return header_v4(u, c, nil=nil)
    if version == 3:
        return header_v3(u, c, nil=nil)
    assert not nil, "v1 / v2 records have no nil flag"
    return header_v2(u, c) if version == 2 else header_v1(u, c)


def file_header(version=4, comp=0):
    return struct.pack("<II", version, comp)


def v3_file(records, comp=0):
    """v3 image (no CRC) — uncompressed or snappy payloads (file_writer.go writeRecordHeaderV3)."""
    from recordio import _lib as L
    import ctypes

    out = bytearray(file_header(3, comp))
    for r in records:
        if r is None:
            c = 1 if comp == 2 else 0
            out += header_v3(0, c, nil=True)
            continue
        if comp == 2:
            cap = int(L.lib().rio_snappy_max_encoded_len(len(r)))
            buf = ctypes.create_string_buffer(cap + 1)
            n = L.lib().rio_snappy_encode(buf, cap, ctypes.c_char_p(bytes(r) or b"\0"), len(r))
            pay = buf.raw[:n]
            out += header_v3(len(r), len(pay)) + pay
        else:
            out += header_v3(len(r), 0) + bytes(r)
    return bytes(out)


def snappy_encode(r: bytes) -> bytes:
    from recordio import _lib as L
    import ctypes

    cap = int(L.lib().rio_snappy_max_encoded_len(len(r)))
    buf = ctypes.create_string_buffer(cap + 1)
    n = L.lib().rio_snappy_encode(buf, cap, ctypes.c_char_p(bytes(r) or b"\0"), len(r))
    return buf.raw[:n]


def legacy_file(records, comp=0, version=2):
    """v1 / v2 image as the old writers laid it out (uncompressed: c = 0, the fixtures' headers;
    snappy: c = the payload length). Nil records (v3+ only) are written as empty ones."""
    out = bytearray(file_header(version, comp))
    for r in records:
        r = b"" if r is None else bytes(r)
        if comp == 2:
            pay = snappy_encode(r)
            out += header_for(version, len(r), len(pay)) + pay
        else:
            out += header_for(version, len(r), 0) + r
    return bytes(out)


def to_version(img: bytes, version: int) -> bytes:
    """A v4 image re-framed as v3 / v2 / v1 (file_writer.go's older header layouts): the same payloads,
    each header rewritten; nil records need v3+."""
    assert struct.unpack_from("<I", img, 0)[0] == 4
    out = bytearray(file_header(version, struct.unpack_from("<I", img, 4)[0]))
    p, n = 8, len(img)

    def uv(i):
        v = s = 0
        while True:
            c = img[i]
            i += 1
            v |= (c & 0x7F) << s
            s += 7
            if c < 0x80:
                return v, i
    comp = struct.unpack_from("<I", img, 4)[0]
    while p < n:
        nil = img[p + 3] == 1
        u, q = uv(p + 4)
        c, q = uv(q)
        _, q = uv(q)  # header CRC
        plen = 0 if nil else (c if comp else u)
        out += header_for(version, u, c, nil=nil) + img[q:q + plen]
        p = q + plen
    return bytes(out)


def mixed_records(n, seed, max_len=3000, nil_frac=0.05):
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        if rng.random() < nil_frac:
            recs.append(None)
            continue
        L = rng.choice([0, 1, 2, 3, 7, 15, 16, 17, 63, 64, 65, rng.randint(0, max_len)])
        if rng.random() < 0.5:
            recs.append(bytes(rng.getrandbits(8) for _ in range(L)))
        else:
            words = [b"alpha", b"beta", b"gamma", b"delta", b"\x91\x8d\x4c", b"zz"]
            s = b" ".join(rng.choice(words) for _ in range(L // 4 + 1))
            recs.append(s[:L])
    return recs


def embedded_file_records(n, seed):
    """Records whose payloads are themselves valid recordio files: every chunk start inside them
    finds CRC-valid speculative headers that are not on the true chain (forces repairs)."""
    rng = random.Random(seed)
    inner = encode_file([bytes([rng.getrandbits(8)]) * rng.randint(1, 40) for _ in range(600)], 0)
    return [inner[8:] if i % 2 == 0 else b"x" * rng.randint(0, 50) for i in range(n)]


def cases():
    """(name, image) pairs covering the edge cases the reference's tests and code paths define."""
    out = []
    asc = lambda n: bytes(i & 0xFF for i in range(n))  # noqa: E731
    out.append(("empty_file_header_only", file_header()))
    out.append(("short_file_4_bytes", b"\x04\x00\x00\x00"))
    out.append(("asc_none", encode_file([asc(i) for i in range(300)], 0)))
    out.append(("asc_snappy", encode_file([asc(i) for i in range(300)], 2)))
    for comp in (0, 2):
        recs = mixed_records(2500, 11 + comp)
        img = encode_file(recs, comp)
        out.append((f"mixed_c{comp}", img))
        # truncations: inside a header, at a payload start, inside a payload, at a record boundary
        rng = random.Random(comp)
        for k in range(6):
            cut = rng.randint(9, len(img) - 1)
            out.append((f"mixed_c{comp}_trunc{k}", img[:cut]))
        # flip one CRC byte of a record in the middle (v4 header CRC mismatch)
        b = bytearray(img)
        pos = img.index(b"\x91\x8d\x4c", len(img) // 2)
        b[pos + 5] ^= 0x01
        out.append((f"mixed_c{comp}_flip", bytes(b)))
        # zero tail (DirectIO padding) short and long; non-zero garbage after zeros
        out.append((f"mixed_c{comp}_zero_tail", img + bytes(4096 * 3 + 5)))
        out.append((f"mixed_c{comp}_garbage_tail", img + bytes(5000) + b"\xb9\x0a" + bytes(10)))
        out.append((f"mixed_c{comp}_one_byte_tail", img + b"\x07"))
        out.append((f"mixed_c{comp}_partial_magic_tail", img + b"\x91\x8d"))
        out.append((f"mixed_c{comp}_embedded", encode_file(embedded_file_records(40, 5 + comp), comp)))
    # non-canonical magic / varints in a record on the chain (entry speculation cannot see it)
    pay = b"hello-noncanonical"
    h = header_v4(len(pay), 0, magic=b"\x91\x8d\xcc\x00", u_bytes=padded_uvarint(len(pay), 3))
    body = encode_file([asc(100)] * 60, 0)
    out.append(("noncanonical_magic", body + h + pay + encode_file([b"after"] * 50, 0)[8:]))
    # snappy records whose padded header varints put the payload's preamble 20..25 bytes into the
    # record (the device's 32-byte header window: the preamble fast path ends at 20)
    from recordio import _lib as L
    import ctypes

    raw = b"long-header-record " * 6
    cap = int(L.lib().rio_snappy_max_encoded_len(len(raw)))
    sbuf = ctypes.create_string_buffer(cap + 1)
    spay = sbuf.raw[: L.lib().rio_snappy_encode(sbuf, cap, ctypes.c_char_p(raw), len(raw))]
    sbody = encode_file([asc(100)] * 40, 2)
    for target in range(20, 26):
        nc = target - 9 - 8  # hl = 4 + nu (8) + nc + ncrc (5)
        pre = b"\x91\x8d\x4c\x00" + padded_uvarint(len(raw), 8) + padded_uvarint(len(spay), nc)
        hdr = pre + padded_uvarint(crc32c(pre), 5)
        out.append((f"snappy_padded_header_hl{target}", sbody + hdr + spay + encode_file([b"after"] * 30, 2)[8:]))
    # header longer than the 36-byte checksum cache
    long_pre = padded_uvarint(0x130691, 10) + b"\x00" + padded_uvarint(1, 10) + padded_uvarint(0, 10)
    long_h = long_pre + padded_uvarint(crc32c(long_pre), 6)
    out.append(("header_too_long", body + long_h + b"Z"))
    out.append(("header_36_exact", body + long_pre + padded_uvarint(crc32c(long_pre), 5) + b"Z"))
    # varint overflow in the magic / size fields
    out.append(("magic_overflow", body + b"\xff" * 10 + b"\x01" * 20))
    out.append(("size_overflow", body + b"\x91\x8d\x4c\x00" + b"\xff" * 9 + b"\x02" + b"\x00" * 20))
    # corrupt snappy: bad copy offset in a record in the middle, and a huge preamble
    recs = [b"abcdefgh" * 20 for _ in range(50)]
    img = bytearray(encode_file(recs, 2))
    p = img.index(b"\x91\x8d\x4c", len(img) // 2)
    hl = len(header_v4(160, img[p + 6]))  # u = 160 takes two varint bytes; c follows
    img[p + hl + 2] = 0x01  # first element after preamble/literal tag: turn into a copy with offset 0
    out.append(("snappy_corrupt_mid", bytes(img)))
    pre = uvarint(5000) + b"\x00a"
    out.append(("snappy_huge_preamble", encode_file([b"ok"] * 3, 2) + header_v4(5000, len(pre)) + pre))
    out.append(("snappy_empty_payload", encode_file([b"ok"] * 3, 2) + header_v4(0, 0)))
    # payloads that do not decompress in the middle of a file: ReadNext returns snappy's error for
    # that record and goes on (file_reader.go:113-122). Unusable preamble (varint overflow), preamble
    # above / below what the elements produce, empty payload; each followed by more records.
    lit160 = b"\xf0\x9f" + bytes(range(160))  # tagLiteral, 1-byte length: 160 bytes
    for name, pay in (("snappy_bad_preamble_mid", b"\xff" * 11 + b"abc"),
                      ("snappy_short_mid", uvarint(170) + lit160),
                      ("snappy_long_mid", uvarint(100) + lit160),
                      ("snappy_empty_mid", b"")):
        before = encode_file([asc(40 + i) for i in range(30)], 2)
        after = encode_file([asc(60 + i) for i in range(30)] + [None, b""], 2)[8:]
        bad = header_v4(160, len(pay)) + pay
        out.append((name, before + bad + after + bad + after))
    # nil records in a compressed file with c != 0 (file_writer.go:198-219)
    out.append(("nil_snappy", encode_file([None, b"a", None, None, b"", b"bb"] * 100, 2)))
    # payload length beyond the file (the reference would panic in bufferPool.Get; we report EOF)
    out.append(("huge_u", body + header_v4(1 << 40, 0) + b"abc"))
    # v3 files
    out.append(("v3_mixed_none", v3_file(mixed_records(1500, 3), 0)))
    out.append(("v3_mixed_snappy", v3_file(mixed_records(1500, 4), 2)))
    v3 = v3_file(mixed_records(800, 9), 0)
    out.append(("v3_zero_tail", v3 + bytes(9000)))
    out.append(("v3_trunc", v3[: len(v3) - 7]))
    # v2 / v1 files (file_reader.go:282-388: no nil byte / no CRC; v1 fixed 20-byte headers and
    # no zero-tail rule: DirectIO padding after a v1 file is a magic mismatch)
    for ver in (2, 1):
        for comp in (0, 2):
            lg = legacy_file(mixed_records(1500, 20 + ver + comp), comp, ver)
            out.append((f"v{ver}_mixed_c{comp}", lg))
            rng = random.Random(40 + ver + comp)
            for k in range(3):
                out.append((f"v{ver}_mixed_c{comp}_trunc{k}", lg[:rng.randint(9, len(lg) - 1)]))
            out.append((f"v{ver}_mixed_c{comp}_zero_tail", lg + bytes(5000)))
            out.append((f"v{ver}_mixed_c{comp}_garbage_tail", lg + bytes(300) + b"\x01" + bytes(7)))
        out.append((f"v{ver}_embedded", legacy_file(embedded_file_records(40, 9), 0, ver)))
        # payloads that are themselves files of the same version: candidate headers with this version's
        # marker bytes inside every chunk (the speculative walk has to repair)
        rng2 = random.Random(30 + ver)
        inner = legacy_file([bytes([rng2.getrandbits(8)]) * rng2.randint(1, 40) for _ in range(600)], 0, ver)[8:]
        out.append((f"v{ver}_embedded_same", legacy_file([inner if i % 2 == 0 else b"y" * rng2.randint(0, 50)
                                                          for i in range(40)], 0, ver)))
        out.append((f"v{ver}_text_snappy_1k", legacy_file(
            [bytes(r) for r in text_records(3000, 30 + ver, 900, 1100)], 2, ver)))
    # v2's smallest record (5 bytes: magic, u = 0, c = 0): more records start in a 32 KiB chunk than
    # any v3 / v4 record size allows (the framing's per-chunk slots and rio_max_records bound on it)
    out.append(("v2_empty_records", legacy_file([b""] * 30000 + [b"x"] * 5 + [b""] * 9000, 0, 2)))
    # v1 record headers cut at every length, and a wrong magic in the middle
    v1 = legacy_file([b"abc" * k for k in range(40)], 0, 1)
    for cut in (1, 4, 12, 19, 20):
        out.append((f"v1_torn_header_{cut}", v1 + header_v1(50, 0)[:cut]))
    b1 = bytearray(v1)
    b1[8 + 20 * 10 + 3 * sum(range(10)) + 1] ^= 0x40
    out.append(("v1_bad_magic_mid", bytes(b1)))
    out.append(("v1_huge_u", v1 + header_v1(1 << 40, 0) + b"abc"))
    # small files damaged in several places (every failure class of ReadNextAt / SeekNext within a
    # few KiB): a flipped CRC byte, an overflowing size varint, a header longer than 36 bytes, a
    # truncated header at the end; snappy variant with a corrupt element stream in the middle
    for comp in (0, 2):
        recs = [asc(17 * i % 200) for i in range(40)]
        img, offs = encode_file(recs, comp), []
        b = bytearray(img)
        starts = [i for i in range(8, len(b) - 2) if b[i:i + 3] == b"\x91\x8d\x4c"]
        b[starts[6] + 6] ^= 0x10  # inside record 6's header (its CRC no longer matches)
        b[starts[14] + 4:starts[14] + 14] = b"\xff" * 10  # record 14: u varint overflows
        if comp == 2:
            p0 = starts[22] + len(header_v4(len(recs[22]), 0))
            b[p0 + 3] = 0x05  # record 22: an element becomes a copy with an offset past its output
        damaged = bytes(b) + long_h + b"ZZ"
        out.append((f"damaged_small_c{comp}", damaged + header_v4(3, 0)[:5]))
    # larger synthetic workloads (several chunks / blocks)
    out.append(("text_snappy_1k", generate(3000, 1024, 2, kind=1, seed=1).tobytes()))
    out.append(("random_snappy_1k", generate(2000, 1024, 2, kind=2, seed=2).tobytes()))
    out.append(("refrandom_none_1k", generate(3000, 1024, 0, kind=0, seed=3).tobytes()))
    out.append(("text_snappy_64", generate(40000, 64, 2, kind=1, seed=4).tobytes()))
    out.append(("text_snappy_64k", generate(40, 65536, 2, kind=1, seed=5).tobytes()))
    out.append(("random_none_64k", generate(30, 65536, 0, kind=2, seed=6).tobytes()))
    return out


# ---------------------------------------------------------------------------------------------
# gzip-compressed files (compType 1, GzipCompressor: one gzip member per record)
# ---------------------------------------------------------------------------------------------
def gzip_member(data: bytes, level: int = 6, strategy: int = 0, header: bytes = None, zdict: bytes = None) -> bytes:
    """One gzip member. header=None: zlib's own 10-byte header; else `header` + raw DEFLATE + trailer.
    zdict: DEFLATE with a preset dictionary, so the body refers back past its own start."""
    import zlib

    if header is None and zdict is None:
        co = zlib.compressobj(level, zlib.DEFLATED, 31, 9, strategy)
        return co.compress(data) + co.flush()
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy, **({"zdict": zdict} if zdict else {}))
    body = co.compress(data) + co.flush()
    return ((header or gzip_header()) + body +
            struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF))


def gzip_members(data: bytes, cuts, **kw) -> bytes:
    """`data` as consecutive gzip members split at the offsets `cuts` (Go's multistream reader
    concatenates their outputs). The record header's uncompressed size is len(data)."""
    pts = [0] + list(cuts) + [len(data)]
    return b"".join(gzip_member(data[a:b], **kw) for a, b in zip(pts, pts[1:]))


def gzip_header(flg=0, extra=b"", name=b"", comment=b"", hcrc=None) -> bytes:
    """RFC 1952 header with optional FEXTRA / FNAME / FCOMMENT / FHCRC (hcrc=None: the right one)."""
    import zlib

    h = bytearray(b"\x1f\x8b\x08" + bytes([flg]) + b"\x00\x00\x00\x00\x00\xff")
    if flg & 4:
        h += struct.pack("<H", len(extra)) + extra
    if flg & 8:
        h += name + b"\x00"
    if flg & 16:
        h += comment + b"\x00"
    if flg & 2:
        v = (zlib.crc32(bytes(h)) & 0xFFFF) if hcrc is None else hcrc
        h += struct.pack("<H", v)
    return bytes(h)


def gz_file(payloads, version=4):
    """recordio image with explicit gzip payloads: (uncompressed_len, payload) or None (nil)."""
    out = bytearray(file_header(version, 1))
    for p in payloads:
        if p is None:
            out += header_for(version, 0, 0, nil=True)
            continue
        u, pay = p
        out += header_for(version, u, len(pay)) + pay
    return bytes(out)


def text_records(n, seed, lo=1, hi=1500):
    rng = random.Random(seed)
    words = ["".join(rng.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(rng.randint(2, 9)))
             for _ in range(300)]
    out = []
    for _ in range(n):
        k = rng.randint(lo, hi)
        s = b""
        while len(s) < k:
            s += (rng.choice(words) + rng.choice([" ", " ", ", ", ".\n"])).encode()
        out.append(s[:k])
    return out


def gzip_cases():
    """(name, image, may_fall_back) gzip files. may_fall_back marks inputs the device path may hand
    back to the reference reader (RIO_ERR_UNSUPPORTED); none of these does any more: records of
    several members decode on the device."""
    import zlib

    rng = random.Random(11)
    cases = []
    text = text_records(200, 5)
    cases.append(("gz_text_small", gz_file([(len(r), gzip_member(r)) for r in text]), False))
    for lvl in (0, 1, 9):
        cases.append((f"gz_level{lvl}", gz_file([(len(r), gzip_member(r, lvl)) for r in text[:60]]), False))
    for st, nm in ((zlib.Z_FIXED, "fixed"), (zlib.Z_HUFFMAN_ONLY, "huffonly"), (zlib.Z_RLE, "rle")):
        cases.append((f"gz_{nm}", gz_file([(len(r), gzip_member(r, 6, st)) for r in text[:60]]), False))
    big = [b"".join(text_records(40, 7 + i, 200, 1500)) for i in range(4)]
    rnd = [bytes(rng.getrandbits(8) for _ in range(n)) for n in (3000, 40000, 70000)]
    runs = [b"a" * 5000, b"ab" * 20000, bytes(range(256)) * 300]
    large = big + rnd + runs
    cases.append(("gz_large", gz_file([(len(r), gzip_member(r)) for r in large]), False))
    cases.append(("gz_large_stored", gz_file([(len(r), gzip_member(r, 0)) for r in large[:5]]), False))
    cases.append(("gz_mixed_nil_empty", gz_file([None, (0, gzip_member(b"")), (len(text[0]), gzip_member(text[0])),
                                                None, (0, gzip_member(b"", 0))]), False))
    hdrs = [gzip_header(8, name=b"record.txt"), gzip_header(16, comment=b"a comment"),
            gzip_header(4, extra=b"\x01\x02\x03"), gzip_header(2), gzip_header(2 | 4 | 8 | 16, b"xy", b"n", b"c")]
    cases.append(("gz_header_fields", gz_file([(len(text[i]), gzip_member(text[i], header=h))
                                              for i, h in enumerate(hdrs)]), False))
    good = [(len(r), gzip_member(r)) for r in text[:20]]

    def corrupt(name, k, pay, may=False):
        recs = list(good)
        recs[k] = (recs[k][0], pay)
        cases.append((name, gz_file(recs), may))

    p = good[7][1]
    corrupt("gz_bad_hcrc", 7, gzip_member(text[7], header=gzip_header(2, hcrc=0x1234)))
    corrupt("gz_bad_magic", 7, b"\x1f\x8c" + p[2:])
    corrupt("gz_bad_cm", 7, p[:2] + b"\x07" + p[3:])
    corrupt("gz_bad_crc", 7, p[:-8] + bytes([p[-8] ^ 1]) + p[-7:])
    corrupt("gz_isize_plus1", 7, p[:-4] + struct.pack("<I", good[7][0] + 1))
    corrupt("gz_isize_minus1", 7, p[:-4] + struct.pack("<I", good[7][0] - 1))
    corrupt("gz_isize_huge", 7, p[:-4] + struct.pack("<I", 0xFFFFFFF0))
    corrupt("gz_truncated_trailer", 7, p[:-3])
    corrupt("gz_truncated_body", 7, p[:len(p) // 2])
    corrupt("gz_tiny", 7, p[:5])
    corrupt("gz_empty_payload", 7, b"")
    corrupt("gz_btype3", 7, p[:10] + bytes([p[10] | 6]) + p[11:])
    corrupt("gz_two_members", 7, gzip_member(text[7][:100]) + gzip_member(text[7][100:]))
    corrupt("gz_trailing_garbage", 7, p + b"\x00\x01")
    corrupt("gz_trailing_header_part", 7, p + gzip_member(b"xyz")[:7])
    corrupt("gz_second_member_bad_crc", 7, gzip_member(text[7][:50]) +
            (lambda q: q[:-8] + bytes([q[-8] ^ 4]) + q[-7:])(gzip_member(text[7][50:])))
    corrupt("gz_second_member_bad_magic", 7, gzip_member(text[7][:50]) + b"\x1f\x8c" + gzip_member(text[7][50:])[2:])
    corrupt("gz_second_member_refers_back", 7, gzip_member(text[7][:80]) +
            gzip_member(text[7][80:], zdict=text[7][:80]))
    corrupt("gz_first_member_bad_isize", 7, (lambda q: q[:-4] + struct.pack("<I", 51))(gzip_member(text[7][:50])) +
            gzip_member(text[7][50:]))
    # bit flips inside the DEFLATE body (header and trailer intact)
    for j in range(12):
        q = bytearray(p)
        pos = 10 + rng.randrange(len(p) - 18)
        q[pos] ^= 1 << rng.randrange(8)
        corrupt(f"gz_flip{j}", 7, bytes(q))
    # records of several members (gzip.Reader is multistream: the outputs concatenate)
    multi = [(len(r), gzip_members(r, sorted({len(r) // 3, 2 * len(r) // 3} - {0}))) for r in text[:40]]
    cases.append(("gz_multi_three", gz_file(multi), False))
    cases.append(("gz_multi_mixed", gz_file([multi[i] if i % 3 == 0 else good[i % 20] for i in range(40)] +
                                            [None, (0, gzip_member(b"") + gzip_member(b"")), (0, b"")]), False))
    cases.append(("gz_multi_empty_members", gz_file([(len(r), gzip_member(b"") + gzip_member(r) + gzip_member(b""))
                                                    for r in text[40:60]]), False))
    cases.append(("gz_multi_header_fields", gz_file([(len(text[i]), gzip_member(text[i][:30], header=hdrs[i % 5]) +
                                                      gzip_member(text[i][30:], header=hdrs[(i + 2) % 5]))
                                                     for i in range(10)]), False))
    # sizes across the device's window classes: a small last member on a large record
    cases.append(("gz_multi_large", gz_file([(len(r), gzip_members(r, [len(r) - 500])) for r in large] +
                                            [(len(r), gzip_members(r, [100, 20000])) for r in large[4:6]]), False))
    cases.append(("gz_multi_many", gz_file([(len(r), gzip_members(r, list(range(7, len(r), 37)))) for r in text[60:70]]),
                  False))
    cases.append(("gz_multi_stored", gz_file([(len(r), gzip_members(r, [len(r) // 2], level=0)) for r in large[:3]]),
                  False))
    cases.append(("gz_v3", gz_file([(len(r), gzip_member(r)) for r in text[:30]], version=3), False))
    cases.append(("gz_v2", gz_file([(len(r), gzip_member(r)) for r in text[:30]], version=2), False))
    cases.append(("gz_v1", gz_file([(len(r), gzip_member(r)) for r in text[:30]], version=1), False))
    return cases


def gzip_go_header_cases():
    """(name, image, record index, Go accepts it) gzip headers on which zlib's wrapper and Go's
    compress/gzip readHeader disagree (gunzip.go): Go ignores FLG's reserved bits (zlib rejects them),
    and readString fails with ErrHeader once a name or comment reaches 512 bytes without its NUL
    (zlib takes any length). Record 3 of each file carries the header."""
    text = text_records(8, 12)
    cases = []

    def one(name, hdr, ok):
        recs = [(len(r), gzip_member(r)) for r in text]
        recs[3] = (len(text[3]), gzip_member(text[3], header=hdr))
        cases.append((name, gz_file(recs), 3, ok))

    one("gz_flg_reserved_bits", gzip_header(0xE0), True)
    one("gz_flg_reserved_with_name", gzip_header(0x20 | 8, name=b"n"), True)
    one("gz_name_511", gzip_header(8, name=b"a" * 511), True)
    one("gz_name_512", gzip_header(8, name=b"a" * 512), False)
    one("gz_comment_511_hcrc", gzip_header(16 | 2, comment=b"c" * 511), True)
    one("gz_comment_600", gzip_header(16, comment=b"c" * 600), False)
    return cases


# ---------------------------------------------------------------------------------------------
# lzw-compressed files (compType 3, LzwCompressor: Go compress/lzw, LSB, litWidth 8)
# ---------------------------------------------------------------------------------------------
def lzw_file(payloads, version=4):
    """recordio image with explicit lzw payloads: (header_u, payload) or None (nil)."""
    out = bytearray(file_header(version, 3))
    for p in payloads:
        if p is None:
            out += header_for(version, 0, 0, nil=True)
            continue
        u, pay = p
        out += header_for(version, u, len(pay)) + pay
    return bytes(out)


def lzw_codes(codes, width=9):
    """A raw LSB-first code stream at a fixed width (crafted streams)."""
    bits = nb = 0
    out = bytearray()
    for c in codes:
        bits |= c << nb
        nb += width
        while nb >= 8:
            out.append(bits & 0xFF)
            bits >>= 8
            nb -= 8
    if nb:
        out.append(bits & 0xFF)
    return bytes(out)


def lzw_cases():
    """(name, image) lzw files: every one decodes on the device (no hand-back)."""
    import oracle_py as orc

    enc = orc.lzw_encode
    rnd = random.Random(77)
    text = text_records(80, 13, 1, 1500)
    cases = [("lzw_text_small", lzw_file([(len(r), enc(r)) for r in text]))]
    cases.append(("lzw_text_v3", lzw_file([(len(r), enc(r)) for r in text[:40]], version=3)))
    cases.append(("lzw_text_v2", lzw_file([(len(r), enc(r)) for r in text[:40]], version=2)))
    cases.append(("lzw_text_v1", lzw_file([(len(r), enc(r)) for r in text[:40]], version=1)))
    # random bytes: about one code per byte, so these lengths sit on the width steps (255 / 767 /
    # 1791 codes) and the writer's clear at 3838 codes
    rand = [bytes(rnd.randrange(256) for _ in range(n)) for n in
            (1, 2, 253, 254, 255, 256, 257, 765, 766, 767, 768, 1789, 1790, 1791, 1792, 3837, 3838, 3839, 3840, 9000, 20000)]
    cases.append(("lzw_width_steps", lzw_file([(len(r), enc(r)) for r in rand])))
    rep = [b"a" * n for n in (1, 2, 3, 10, 100, 1000, 5000, 70000)] + [b"ab" * 3000, b"abc" * 20000,
                                                                        bytes(range(256)) * 40]
    cases.append(("lzw_repetitive", lzw_file([(len(r), enc(r)) for r in rep])))
    large = text_records(6, 17, 40000, 70000)
    cases.append(("lzw_large", lzw_file([(len(r), enc(r)) for r in large])))
    cases.append(("lzw_nil_empty", lzw_file([None, (0, enc(b"")), (len(text[0]), enc(text[0])), None,
                                             (0, enc(b""))])))
    good = [(len(r), enc(r)) for r in text[:20]]

    def with_bad(name, k, item):
        cases.append((name, lzw_file(good[:k] + [item] + good[k:])))

    p = enc(text[5])
    with_bad("lzw_truncated", 7, (len(text[5]), p[:-2]))
    with_bad("lzw_empty_payload", 7, (0, b""))
    with_bad("lzw_empty_payload_u", 7, (100, b""))
    with_bad("lzw_invalid_code", 7, (3, lzw_codes([256, 97, 300, 257])))
    with_bad("lzw_invalid_first", 7, (3, lzw_codes([258, 257])))
    with_bad("lzw_garbage", 7, (50, bytes(rnd.randrange(256) for _ in range(40))))
    # valid streams the reference's writer would not produce
    with_bad("lzw_trailing_bytes", 7, (len(text[5]), p + b"\xff\x00\x13"))
    with_bad("lzw_no_leading_clear", 7, (4, lzw_codes([104, 105, 258, 257])))
    with_bad("lzw_double_clear", 7, (2, lzw_codes([256, 256, 120, 256, 121, 257])))
    # header u that is not the decoded length: sized by the decode (resize round)
    with_bad("lzw_u_small", 7, (len(text[5]) - 10, p))
    with_bad("lzw_u_large", 7, (len(text[5]) + 300, p))
    with_bad("lzw_u_absurd", 7, (10 ** 12, p))
    cases.append(("lzw_u_zero_all", lzw_file([(0, enc(r)) for r in text[:30]])))
    return cases
