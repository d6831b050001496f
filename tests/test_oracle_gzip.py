"""Oracle (CPU checker) on the gzip corpus: valid files decode to exactly the records they were
built from; corruptions end the ReadNext loop at the damaged record with the codec-error class.
Parity for gzip is pinned by the reference's _comp1 fixture (test_oracle_golden.py); this test pins
the oracle's gzip restatement against the source records of the crafted corpus."""
import pytest

import corpus
import oracle_py as orc
from conftest import STATUS


def _records(name):
    return {n: img for n, img, _ in corpus.gzip_cases()}[name]


@pytest.mark.parametrize("name", ["gz_text_small", "gz_level0", "gz_level9", "gz_fixed", "gz_rle",
                                  "gz_large", "gz_large_stored", "gz_header_fields", "gz_v3", "gz_two_members",
                                  "gz_multi_three", "gz_multi_empty_members", "gz_multi_header_fields",
                                  "gz_multi_large", "gz_multi_many", "gz_multi_stored"])
def test_valid_gzip_files_decode_to_sources(name):
    img = _records(name)
    o = orc.file_reader_decode_arrays(img)
    assert o["status"] == STATUS["EOF"], o["status"]
    # rebuild the payloads and compare record by record with an independent decode of each payload
    out, off = o["out"], o["out_off"]
    pos, k = 8, 0
    while pos < len(img):
        pos += 4  # magic + nil byte
        vals = []
        for _ in range(3 if img[:4] == b"\x04\x00\x00\x00" else 2):
            v, sh = 0, 0
            while True:
                b = img[pos]
                pos += 1
                v |= (b & 0x7F) << sh
                sh += 7
                if b < 0x80:
                    break
            vals.append(v)
        c = vals[1]
        # every member of the payload, concatenated (gzip.Reader is multistream by default; Python's
        # gzip module is an independent decoder of the same format)
        import gzip

        want = gzip.decompress(img[pos:pos + c])
        assert bytes(out[off[k]:off[k + 1]]) == want, (name, k)
        pos += c
        k += 1
    assert k == o["n_records"]


@pytest.mark.parametrize("name", ["gz_bad_hcrc", "gz_bad_magic", "gz_bad_cm", "gz_bad_crc", "gz_isize_plus1",
                                  "gz_isize_huge", "gz_btype3", "gz_trailing_garbage", "gz_trailing_header_part",
                                  "gz_second_member_bad_crc", "gz_second_member_bad_magic",
                                  "gz_second_member_refers_back", "gz_first_member_bad_isize"])
def test_gzip_corruption_flags_the_record(name):
    """The gzip reader's error comes back for record 7 alone; ReadNext then reads record 8
    (the payload was consumed before the codec ran, file_reader.go:113-122)."""
    o = orc.file_reader_decode_arrays(_records(name))
    assert o["status"] == STATUS["EOF"] and o["n_records"] == 20
    assert o["flags"][7] == 2 and (o["first_bad"], o["n_bad"]) == (7, 1)
    full = orc.file_reader_decode_arrays(_records("gz_text_small"))
    for k in (6, 8, 19):  # neighbours decode as in the clean file (same text records)
        a, b = o["out_off"][k], full["out_off"][k]
        ln = o["out_off"][k + 1] - a
        assert bytes(o["out"][a:a + ln]) == bytes(full["out"][b:b + ln])


def test_gzip_empty_payload_is_eof_class():
    # gzip.NewReader(empty) -> bare io.EOF, returned unwrapped by ReadNext (file_reader.go:118-121);
    # the loop can go on past it
    o = orc.file_reader_decode_arrays(_records("gz_empty_payload"))
    assert o["status"] == STATUS["EOF"] and o["n_records"] == 20
    assert o["flags"][7] == 4 and o["out_off"][8] == o["out_off"][7]


@pytest.mark.parametrize("name,image,k,go_ok", corpus.gzip_go_header_cases(), ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_follows_go_gzip_header_rules(name, image, k, go_ok):
    """The oracle reads member headers as Go's readHeader does (gunzip.go), not as zlib's wrapper:
    reserved FLG bits are ignored, a name or comment of 512 bytes or more without its NUL is ErrHeader."""
    o = orc.file_reader_decode(image)
    assert o["n_records"] == 8, name
    rec = o["records"][k]
    if go_ok:
        assert not isinstance(rec, orc.BadRecord) and rec == corpus.text_records(8, 12)[k], name
    else:
        assert isinstance(rec, orc.BadRecord), name
    assert all(not isinstance(r, orc.BadRecord) for i, r in enumerate(o["records"]) if i != k), name
