/*
 * rio_oracle.c — CPU restatement of github.com/thomasjungblut/go-sstables recordio decode
 * semantics. TEST INFRASTRUCTURE ONLY (see rio_oracle.h): the parity checker for the HIP path and
 * the "port" CPU baseline of bench.py. Never linked into the product library.
 *
 * Every function cites the reference file:line it restates. Third-party algorithms restated here
 * (their code is not under /root/reference):
 *   - Go stdlib encoding/binary ReadUvarint / Uvarint (go 1.25, go.mod:27): LEB128, <=10 bytes,
 *     10th byte must be <= 1, io.EOF on 0 bytes, io.ErrUnexpectedEOF on a partial varint.
 *   - Go stdlib hash/crc32 Castagnoli (reflected poly 0x82F63B78, init/xorout 0xFFFFFFFF).
 *   - github.com/golang/snappy v1.0.0 (go.mod:6) block decoder (decode.go, decode_other.go).
 *   - golang.org/x/exp/mmap ReaderAt.ReadAt bounds semantics (go.mod:10).
 *   - Go stdlib compress/gzip reader via zlib (multistream, CRC-32 + ISIZE verified).
 *   - Go stdlib compress/lzw reader and writer (LSB, litWidth 8), restated in full.
 */
#include "rio_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "../include/rio.h"

/* ---------------------------------------------------------------------------------------- */
/* CRC-32C (hash/crc32 MakeTable(Castagnoli)); used by checksum_byte_reader.go:44-50          */
/* ---------------------------------------------------------------------------------------- */
static uint32_t crc_tab[256];
static int crc_ready = 0;

static void crc_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc_tab[i] = c;
    }
    crc_ready = 1;
}

uint32_t orc_crc32c(const uint8_t* p, uint64_t n) {
    if (!crc_ready) crc_init();
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; i++) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

void orc_free(void* p) { free(p); }

/* ---------------------------------------------------------------------------------------- */
/* io.ByteReader over a byte window, optionally teed through checksumByteReader's cache.      */
/* checksum_byte_reader.go:19-33: the underlying ReadByte error (io.EOF) wins; then the cache  */
/* bound check raises "checksum byte reader out of range".                                    */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
    const uint8_t* p;
    uint64_t avail; /* bytes the underlying reader can deliver */
    uint64_t pos;
    uint64_t cap; /* checksum cache size; UINT64_MAX = no checksum reader */
} brd;

static int brd_byte(brd* r, uint8_t* b) {
    if (r->pos >= r->avail) return RIO_EOF;
    if (r->pos >= r->cap) { r->pos++; return RIO_ERR_HEADER_TOO_LONG; }
    *b = r->p[r->pos++];
    return RIO_OK;
}

/* encoding/binary.ReadUvarint */
static int go_read_uvarint(brd* r, uint64_t* x) {
    uint64_t v = 0;
    unsigned s = 0;
    for (int i = 0; i < 10; i++) {
        uint8_t b;
        int e = brd_byte(r, &b);
        if (e) {
            if (e == RIO_EOF && i > 0) return RIO_ERR_UNEXPECTED_EOF;
            return e;
        }
        if (b < 0x80) {
            if (i == 9 && b > 1) return RIO_ERR_VARINT_OVERFLOW;
            *x = v | ((uint64_t)b << s);
            return RIO_OK;
        }
        v |= (uint64_t)(b & 0x7F) << s;
        s += 7;
    }
    return RIO_ERR_VARINT_OVERFLOW;
}

/* encoding/binary.Uvarint: returns n>0 bytes read, 0 if buf too small, <0 on overflow */
static int go_uvarint(const uint8_t* buf, uint64_t len, uint64_t* x) {
    uint64_t v = 0;
    unsigned s = 0;
    for (uint64_t i = 0; i < len; i++) {
        if (i == 10) return -(int)(i + 1);
        uint8_t b = buf[i];
        if (b < 0x80) {
            if (i == 9 && b > 1) return -(int)(i + 1);
            *x = v | ((uint64_t)b << s);
            return (int)(i + 1);
        }
        v |= (uint64_t)(b & 0x7F) << s;
        s += 7;
    }
    return 0;
}

/* a header field after the magic that hits io.EOF on its first byte returns io.EOF unchanged;
 * we tag it RIO_EOF_HEADER to keep "EOF at a record boundary" distinguishable. */
static int later_field(int e) { return e == RIO_EOF ? RIO_EOF_HEADER : e; }

typedef struct {
    uint64_t u, c;
    int nil;
    uint64_t hdr_len;
    uint64_t magic_len; /* bytes consumed by the magic varint (for the zero-tail check) */
    uint64_t exp_crc, act_crc;
} hdr_t;

/* readRecordHeaderV4 (common_reader.go:110-151) */
static int read_header_v4(brd* r, hdr_t* h) {
    uint64_t m = 0;
    int e = go_read_uvarint(r, &m);
    h->magic_len = r->pos;
    if (e) return e;
    if (m != RIO_MAGIC) return RIO_ERR_MAGIC;
    uint8_t nb;
    e = brd_byte(r, &nb);
    if (e) return later_field(e);
    e = go_read_uvarint(r, &h->u);
    if (e) return later_field(e);
    e = go_read_uvarint(r, &h->c);
    if (e) return later_field(e);
    /* checksumByteReader.Checksum over bytes cached so far (checksum_byte_reader.go:44-50) */
    h->act_crc = orc_crc32c(r->p, r->pos);
    e = go_read_uvarint(r, &h->exp_crc);
    if (e) return later_field(e);
    if (h->act_crc != h->exp_crc) return RIO_ERR_HEADER_CRC;
    h->nil = (nb == 1);
    h->hdr_len = r->pos;
    return RIO_OK;
}

/* readRecordHeaderV3 (common_reader.go:83-108) */
static int read_header_v3(brd* r, hdr_t* h) {
    uint64_t m = 0;
    int e = go_read_uvarint(r, &m);
    h->magic_len = r->pos;
    if (e) return e;
    if (m != RIO_MAGIC) return RIO_ERR_MAGIC;
    uint8_t nb;
    e = brd_byte(r, &nb);
    if (e) return later_field(e);
    e = go_read_uvarint(r, &h->u);
    if (e) return later_field(e);
    e = go_read_uvarint(r, &h->c);
    if (e) return later_field(e);
    h->nil = (nb == 1);
    h->hdr_len = r->pos;
    return RIO_OK;
}

/* readRecordHeaderV2 (common_reader.go:62-81): uvarint magic, u, c (no nil byte, no CRC) */
static int read_header_v2(brd* r, hdr_t* h) {
    uint64_t m = 0;
    int e = go_read_uvarint(r, &m);
    h->magic_len = r->pos;
    if (e) return e;
    if (m != RIO_MAGIC) return RIO_ERR_MAGIC;
    e = go_read_uvarint(r, &h->u);
    if (e) return later_field(e);
    e = go_read_uvarint(r, &h->c);
    if (e) return later_field(e);
    h->nil = 0;
    h->hdr_len = r->pos;
    return RIO_OK;
}

/* readNextV1 header (file_reader.go:282-300 + readRecordHeaderV1, common_reader.go:46-60): a
 * fixed 20-byte header read with io.ReadFull (0 bytes: io.EOF, partial: io.ErrUnexpectedEOF),
 * LE u32 magic 0x130691, LE u64 u, LE u64 c. No zero-tail rule in v1. */
static int read_header_v1(const uint8_t* f, uint64_t avail, hdr_t* h) {
    h->magic_len = 0;
    if (avail == 0) return RIO_EOF;
    if (avail < 20) return RIO_ERR_UNEXPECTED_EOF;
    uint32_t m = (uint32_t)f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
    if (m != RIO_MAGIC) return RIO_ERR_MAGIC;
    h->u = h->c = 0;
    for (int k = 7; k >= 0; k--) h->u = (h->u << 8) | f[4 + k];
    for (int k = 7; k >= 0; k--) h->c = (h->c << 8) | f[12 + k];
    h->nil = 0;
    h->hdr_len = 20;
    return RIO_OK;
}

/* ---------------------------------------------------------------------------------------- */
/* golang/snappy v1.0.0 Decode(dst, src): decodedLen (binary.Uvarint, >0xffffffff => ErrCorrupt) */
/* then decode() with its bounds checks; output length = the preamble, not the header's u.     */
/* ---------------------------------------------------------------------------------------- */
int orc_snappy_decode(const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len) {
    uint64_t dlen = 0;
    int k = go_uvarint(src, n, &dlen);
    *out = NULL;
    *out_len = 0;
    if (k <= 0 || dlen > 0xFFFFFFFFull) return RIO_ERR_DECOMPRESS;
    /* a stream of m bytes yields at most 64 bytes per 3 (tagCopy2): larger preambles cannot
     * decode (d != len(dst) at the end); refuse before allocating */
    if (dlen > 22ull * (n - (uint64_t)k) + 64) return RIO_ERR_DECOMPRESS;
    uint8_t* dst = (uint8_t*)malloc(dlen ? dlen : 1);
    const uint8_t* s0 = src + k;
    int64_t slen = (int64_t)(n - (uint64_t)k), s = 0, d = 0, dl = (int64_t)dlen;
    int64_t offset = 0, length = 0;
    while (s < slen) {
        switch (s0[s] & 3) {
        case 0: { /* tagLiteral */
            uint32_t x = s0[s] >> 2;
            if (x < 60) {
                s++;
            } else if (x == 60) {
                s += 2;
                if (s > slen) goto corrupt;
                x = s0[s - 1];
            } else if (x == 61) {
                s += 3;
                if (s > slen) goto corrupt;
                x = (uint32_t)s0[s - 2] | (uint32_t)s0[s - 1] << 8;
            } else if (x == 62) {
                s += 4;
                if (s > slen) goto corrupt;
                x = (uint32_t)s0[s - 3] | (uint32_t)s0[s - 2] << 8 | (uint32_t)s0[s - 1] << 16;
            } else {
                s += 5;
                if (s > slen) goto corrupt;
                x = (uint32_t)s0[s - 4] | (uint32_t)s0[s - 3] << 8 | (uint32_t)s0[s - 2] << 16 |
                    (uint32_t)s0[s - 1] << 24;
            }
            length = (int64_t)x + 1;
            if (length > dl - d || length > slen - s) goto corrupt;
            memcpy(dst + d, s0 + s, (size_t)length);
            d += length;
            s += length;
            continue;
        }
        case 1: /* tagCopy1 */
            s += 2;
            if (s > slen) goto corrupt;
            length = 4 + ((s0[s - 2] >> 2) & 7);
            offset = (int64_t)(((uint32_t)s0[s - 2] & 0xE0) << 3 | (uint32_t)s0[s - 1]);
            break;
        case 2: /* tagCopy2 */
            s += 3;
            if (s > slen) goto corrupt;
            length = 1 + (s0[s - 3] >> 2);
            offset = (int64_t)((uint32_t)s0[s - 2] | (uint32_t)s0[s - 1] << 8);
            break;
        default: /* tagCopy4 */
            s += 5;
            if (s > slen) goto corrupt;
            length = 1 + (s0[s - 5] >> 2);
            offset = (int64_t)((uint32_t)s0[s - 4] | (uint32_t)s0[s - 3] << 8 |
                               (uint32_t)s0[s - 2] << 16 | (uint32_t)s0[s - 1] << 24);
            break;
        }
        if (offset <= 0 || d < offset || length > dl - d) goto corrupt;
        /* forward byte copy: overlapping copies replicate the pattern (decode_other.go) */
        for (int64_t i = 0; i < length; i++) dst[d + i] = dst[d - offset + i];
        d += length;
    }
    if (d != dl) goto corrupt;
    *out = dst;
    *out_len = dlen;
    return RIO_OK;
corrupt:
    free(dst);
    return RIO_ERR_DECOMPRESS;
}

/* GzipCompressor.DecompressWithBuf (gzip_compression.go:54-69): gzip.NewReader + bytes.Buffer.ReadFrom,
 * i.e. Go's compress/gzip Reader, multistream (go 1.25 stdlib gunzip.go; not vendored). Restated:
 *   member header (readHeader): ID1 ID2 = 1f 8b, CM = 8, else ErrHeader; FLG's reserved bits are
 *   ignored; FEXTRA: 2-byte XLEN and its bytes; FNAME, FCOMMENT: readString, which reads into a
 *   512-byte buffer and fails with ErrHeader when the 512th byte is not the NUL; FHCRC: the low 16 bits
 *   of the CRC-32 of every header byte before it (strings with their NUL); a short header is
 *   io.ErrUnexpectedEOF (noEOF);
 *   body: DEFLATE (compress/flate; here zlib's raw inflate);
 *   trailer: CRC-32 and ISIZE (mod 2^32) of the member's output, else ErrChecksum; short: ErrUnexpectedEOF;
 *   after a trailer: the end of the payload ends the record (readHeader's io.EOF), anything else is the
 *   next member's header. An empty payload is gzip.NewReader's bare io.EOF.
 * zlib's own gzip wrapper differs from Go on the header (it rejects reserved FLG bits and accepts any
 * name length), so only the DEFLATE body is zlib's here. Pinned by the _comp1 fixture (Go-written). */
static uLong crc_upd(uLong c, const uint8_t* p, uint64_t n) { return crc32(c, p, (uInt)n); }

static int gz_member_header(const uint8_t* s, uint64_t n, uint64_t* hl) {
    if (n < 10 || s[0] != 0x1f || s[1] != 0x8b || s[2] != 8) return RIO_ERR_DECOMPRESS;
    const uint32_t flg = s[3];
    uLong crc = crc_upd(crc32(0L, Z_NULL, 0), s, 10);
    uint64_t p = 10;
    if (flg & 4) { /* FEXTRA */
        if (n - p < 2) return RIO_ERR_DECOMPRESS;
        const uint64_t xl = (uint64_t)s[p] | (uint64_t)s[p + 1] << 8;
        crc = crc_upd(crc, s + p, 2);
        p += 2;
        if (n - p < xl) return RIO_ERR_DECOMPRESS;
        crc = crc_upd(crc, s + p, xl);
        p += xl;
    }
    for (int f = 0; f < 2; f++) { /* FNAME, then FCOMMENT */
        if (!(flg & (f ? 16u : 8u))) continue;
        uint64_t i = 0;
        for (;;) {
            if (i >= 512) return RIO_ERR_DECOMPRESS; /* readString: ErrHeader */
            if (p + i >= n) return RIO_ERR_DECOMPRESS;
            if (s[p + i] == 0) break;
            i++;
        }
        crc = crc_upd(crc, s + p, i + 1);
        p += i + 1;
    }
    if (flg & 2) { /* FHCRC */
        if (n - p < 2) return RIO_ERR_DECOMPRESS;
        if (((uint32_t)s[p] | (uint32_t)s[p + 1] << 8) != (uint32_t)(crc & 0xFFFFu)) return RIO_ERR_DECOMPRESS;
        p += 2;
    }
    *hl = p;
    return RIO_OK;
}

static int gzip_decode(const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len) {
    *out = NULL;
    *out_len = 0;
    /* gzip.NewReader(empty) returns a bare io.EOF (gzip_compression.go:56-59), which ReadNext
     * passes through unwrapped (file_reader.go:118-121) and ReadNextAt wraps once: io.EOF class */
    if (n == 0) return RIO_EOF_CODEC;
    uint64_t cap = n * 4 + 64, used = 0, pos = 0;
    uint8_t* dst = (uint8_t*)malloc(cap);
    for (;;) { /* one member */
        uint64_t hl = 0;
        if (gz_member_header(src + pos, n - pos, &hl)) goto bad;
        pos += hl;
        z_stream z;
        memset(&z, 0, sizeof z);
        if (inflateInit2(&z, -15) != Z_OK) goto bad;
        z.next_in = (Bytef*)(src + pos);
        z.avail_in = (uInt)(n - pos);
        const uint64_t m0 = used;
        int rc;
        for (;;) {
            if (used == cap) {
                cap *= 2;
                dst = (uint8_t*)realloc(dst, cap);
            }
            z.next_out = dst + used;
            z.avail_out = (uInt)(cap - used);
            rc = inflate(&z, Z_NO_FLUSH);
            used = cap - z.avail_out;
            if (rc == Z_STREAM_END) break;
            if (rc == Z_OK) continue;
            if (rc == Z_BUF_ERROR && z.avail_out == 0) continue;
            break;
        }
        const uint64_t rest = z.avail_in;
        inflateEnd(&z);
        if (rc != Z_STREAM_END) goto bad;
        pos = n - rest;
        if (n - pos < 8) goto bad; /* trailer: io.ErrUnexpectedEOF */
        const uint8_t* t = src + pos;
        const uint32_t want_crc = (uint32_t)t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
        const uint32_t want_sz = (uint32_t)t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24;
        if ((uint32_t)crc_upd(crc32(0L, Z_NULL, 0), dst + m0, used - m0) != want_crc ||
            (uint32_t)(used - m0) != want_sz)
            goto bad; /* ErrChecksum */
        pos += 8;
        if (pos == n) break; /* readHeader's io.EOF: the stream ends cleanly */
    }
    *out = dst;
    *out_len = used;
    return RIO_OK;
bad:
    free(dst);
    return RIO_ERR_DECOMPRESS;
}


/* ---------------------------------------------------------------------------------------- */
/* LzwCompressor (lzw_compressor.go:9-63): Go stdlib compress/lzw, LSB bit order, litWidth 8.  */
/* Restated from Go's compress/lzw reader.go / writer.go (stdlib of go 1.25, go.mod:27; not   */
/* vendored under /root/reference). Pinned by lzw_compessor_test.go:9-16 ("some data" -> 13   */
/* bytes: the writer's leading clear code) and, for the decoder, by an independent decoder of */
/* the same code stream: GIF's variable-length LZW with 8-bit literals (Pillow, tests/).       */
/* ---------------------------------------------------------------------------------------- */
enum { LZW_CLEAR = 256, LZW_EOF = 257, LZW_MAXW = 12, LZW_MAXCODE = 4095, LZW_INV = 0xFFFF };

/* lzw.NewReader(src, LSB, 8) drained by bytes.Buffer.ReadFrom (lzw_compressor.go:52-63): reader.go
 * decode(). A stream that ends before the eof code is io.ErrUnexpectedEOF, a code above hi is "lzw:
 * invalid code"; both are codec errors (RIO_ERR_DECOMPRESS). Bytes after the eof code are ignored. */
int orc_lzw_decode(const uint8_t* src, uint64_t n, uint8_t** out, uint64_t* out_len) {
    static __thread uint16_t prefix[1 << LZW_MAXW];
    static __thread uint8_t suffix[1 << LZW_MAXW];
    uint8_t tmp[(1 << LZW_MAXW) + 2];
    uint64_t cap = 4 * n + 64, used = 0, ip = 0;
    uint8_t* dst = (uint8_t*)malloc(cap);
    uint32_t bits = 0, nbits = 0, width = 9, hi = LZW_EOF, overflow = 1u << 9, last = LZW_INV;
    *out = NULL;
    *out_len = 0;
    for (;;) {
        while (nbits < width) { /* readLSB */
            if (ip >= n) goto bad; /* io.EOF from ReadByte => io.ErrUnexpectedEOF */
            bits |= (uint32_t)src[ip++] << nbits;
            nbits += 8;
        }
        const uint32_t code = bits & ((1u << width) - 1u);
        bits >>= width;
        nbits -= width;
        uint64_t sl;
        const uint8_t* sp;
        if (code < LZW_CLEAR) {
            tmp[0] = (uint8_t)code;
            sp = tmp;
            sl = 1;
            if (last != LZW_INV) { suffix[hi] = (uint8_t)code; prefix[hi] = (uint16_t)last; }
        } else if (code == LZW_CLEAR) {
            width = 9;
            hi = LZW_EOF;
            overflow = 1u << 9;
            last = LZW_INV;
            continue;
        } else if (code == LZW_EOF) {
            break;
        } else if (code <= hi) {
            uint32_t c = code, i = sizeof tmp - 1;
            if (code == hi && last != LZW_INV) { /* KwKwK: last's expansion + its first byte */
                c = last;
                while (c >= LZW_CLEAR) c = prefix[c];
                tmp[i--] = (uint8_t)c;
                c = last;
            }
            while (c >= LZW_CLEAR) {
                tmp[i--] = suffix[c];
                c = prefix[c];
            }
            tmp[i] = (uint8_t)c;
            sp = tmp + i;
            sl = sizeof tmp - i;
            if (last != LZW_INV) { suffix[hi] = (uint8_t)c; prefix[hi] = (uint16_t)last; }
        } else {
            goto bad; /* "lzw: invalid code" */
        }
        if (used + sl > cap) {
            while (used + sl > cap) cap *= 2;
            dst = (uint8_t*)realloc(dst, cap);
        }
        memcpy(dst + used, sp, sl);
        used += sl;
        last = code;
        hi++;
        if (hi >= overflow) {
            if (width == LZW_MAXW) { /* table full: no new entries until a clear code */
                last = LZW_INV;
                hi--;
            } else {
                width++;
                overflow = 1u << width;
            }
        }
    }
    *out = dst;
    *out_len = used;
    return RIO_OK;
bad:
    free(dst);
    return RIO_ERR_DECOMPRESS;
}

typedef struct {
    uint8_t* dst;
    uint64_t o;
    uint32_t bits, nbits, width;
} lzw_w;
static void lzw_put(lzw_w* w, uint32_t code) { /* writer.go writeLSB */
    w->bits |= code << w->nbits;
    w->nbits += w->width;
    while (w->nbits >= 8) {
        w->dst[w->o++] = (uint8_t)w->bits;
        w->bits >>= 8;
        w->nbits -= 8;
    }
}

/* lzw.NewWriter(buf, LSB, 8) + one Write(record) + Close (lzw_compressor.go:12-26): writer.go. The
 * output is fixed by the algorithm (the hash table only implements the dictionary); dst capacity
 * >= 2 n + 16. Returns the bytes written. */
uint64_t orc_lzw_encode(uint8_t* dst, const uint8_t* src, uint64_t n) {
    enum { TSIZE = 4 << LZW_MAXW, TMASK = TSIZE - 1 };
    uint32_t* table = (uint32_t*)calloc(TSIZE, sizeof(uint32_t)); /* invalidEntry = 0 */
    lzw_w w = {dst, 0, 0, 0, 9};
    uint32_t hi = LZW_EOF, overflow = 1u << 9, code = 0xFFFFFFFFu;
    if (n) { /* first Write: the clear code, then the first byte is the pending code */
        lzw_put(&w, LZW_CLEAR);
        code = src[0];
        for (uint64_t k = 1; k < n; k++) {
            const uint32_t lit = src[k], key = code << 8 | lit, hash = (key >> 12 ^ key) & TMASK;
            int hit = 0;
            for (uint32_t h = hash, t = table[hash]; t != 0;) {
                if (key == t >> 12) { code = t & LZW_MAXCODE; hit = 1; break; }
                h = (h + 1) & TMASK;
                t = table[h];
            }
            if (hit) continue;
            lzw_put(&w, code);
            code = lit;
            /* incHi */
            if (++hi == overflow) { w.width++; overflow <<= 1; }
            if (hi == LZW_MAXCODE) { /* out of codes: clear, reset, nothing inserted */
                lzw_put(&w, LZW_CLEAR);
                w.width = 9;
                hi = LZW_EOF;
                overflow = 1u << 9;
                memset(table, 0, TSIZE * sizeof(uint32_t));
                continue;
            }
            uint32_t h = hash;
            while (table[h] != 0) h = (h + 1) & TMASK;
            table[h] = key << 12 | hi;
        }
    }
    /* Close */
    if (code != 0xFFFFFFFFu) {
        lzw_put(&w, code);
        if (++hi == overflow) { w.width++; overflow <<= 1; }
        if (hi == LZW_MAXCODE) {
            lzw_put(&w, LZW_CLEAR);
            w.width = 9;
        }
    } else {
        lzw_put(&w, LZW_CLEAR);
    }
    lzw_put(&w, LZW_EOF);
    if (w.nbits > 0) dst[w.o++] = (uint8_t)w.bits;
    free(table);
    return w.o;
}

static int decompress(uint32_t comp, const uint8_t* src, uint64_t n, uint8_t** out,
                      uint64_t* out_len) {
    if (comp == RIO_COMP_SNAPPY) return orc_snappy_decode(src, n, out, out_len);
    if (comp == RIO_COMP_GZIP) return gzip_decode(src, n, out, out_len);
    return orc_lzw_decode(src, n, out, out_len);
}

/* ---------------------------------------------------------------------------------------- */
/* readFileHeaderFromBuffer (common_reader.go:22-44); short files: io.ReadFull in Open         */
/* ---------------------------------------------------------------------------------------- */
int orc_file_header(const uint8_t* f, uint64_t len, uint32_t* version, uint32_t* compression,
                    uint64_t* detail) {
    *detail = 0;
    if (len < RIO_FILE_HEADER_BYTES) return RIO_ERR_SHORT_FILE_HEADER;
    uint32_t v = (uint32_t)f[0] | (uint32_t)f[1] << 8 | (uint32_t)f[2] << 16 | (uint32_t)f[3] << 24;
    uint32_t c = (uint32_t)f[4] | (uint32_t)f[5] << 8 | (uint32_t)f[6] << 16 | (uint32_t)f[7] << 24;
    *version = v;
    *compression = c;
    if (v > RIO_VERSION4 || v < RIO_VERSION1) { *detail = v; return RIO_ERR_VERSION; }
    if (c > RIO_COMP_LZW) { *detail = c; return RIO_ERR_COMPRESSION_TYPE; }
    return RIO_OK;
}

/* ---------------------------------------------------------------------------------------- */
/* FileReader: Open + ReadNext loop (file_reader.go:26-131 v4, 389-447 v3)                    */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
    uint8_t* out;
    uint64_t out_len, out_cap;
    uint64_t *out_off, *rec_off;
    uint8_t* flags;
    uint64_t n, cap;
} arena_t;

static void arena_push(arena_t* a, uint64_t rec_off, const uint8_t* data, uint64_t len, int nil) {
    if (a->n + 1 >= a->cap) {
        a->cap = a->cap ? a->cap * 2 : 1024;
        a->out_off = (uint64_t*)realloc(a->out_off, (a->cap + 1) * sizeof(uint64_t));
        a->rec_off = (uint64_t*)realloc(a->rec_off, a->cap * sizeof(uint64_t));
        a->flags = (uint8_t*)realloc(a->flags, a->cap);
    }
    if (a->out_len + len > a->out_cap) {
        uint64_t nc = a->out_cap ? a->out_cap * 2 : 4096;
        while (nc < a->out_len + len) nc *= 2;
        a->out = (uint8_t*)realloc(a->out, nc);
        a->out_cap = nc;
    }
    a->out_off[a->n] = a->out_len;
    a->rec_off[a->n] = rec_off;
    a->flags[a->n] = nil ? RIO_FLAG_NIL : 0;
    if (len) memcpy(a->out + a->out_len, data, len);
    a->out_len += len;
    a->n++;
    a->out_off[a->n] = a->out_len;
}

/* Output bytes reserved for a record whose payload does not decompress (the device sizes every
 * record before decoding any): snappy's preamble when decodedLen accepts it and a stream of this
 * length can reach it (orc_snappy_decode's first two checks); gzip's ISIZE trailer when the payload
 * holds a whole member (>= 18 bytes) and DEFLATE's maximum ratio (258 bytes per 2 bits) can reach
 * it; lzw: the header's u when an lzw stream of this length can reach it (ORC_LZW_MAX_RATIO bytes per
 * payload byte); otherwise 0. Not a reference behaviour: the reference returns no bytes for such a record. */
static uint64_t bad_reserve(uint32_t comp, const uint8_t* pay, uint64_t plen, uint64_t u) {
    if (comp == RIO_COMP_LZW) return u <= ORC_LZW_MAX_RATIO * plen ? u : 0;
    if (comp == RIO_COMP_SNAPPY) {
        uint64_t d = 0;
        const int k = go_uvarint(pay, plen, &d);
        if (k <= 0 || d > 0xFFFFFFFFull || d > 22ull * (plen - (uint64_t)k) + 64) return 0;
        return d;
    }
    if (plen < 18) return 0;
    const uint8_t* t = pay + plen - 4;
    const uint64_t isz = (uint64_t)t[0] | (uint64_t)t[1] << 8 | (uint64_t)t[2] << 16 | (uint64_t)t[3] << 24;
    return isz > 1032ull * plen + 64 ? 0 : isz;
}

int orc_file_reader_decode(const uint8_t* f, uint64_t len, orc_file_result* res) {
    memset(res, 0, sizeof *res);
    res->first_bad = UINT64_MAX;
    int e = orc_file_header(f, len, &res->version, &res->compression, &res->detail0);
    if (e) { res->status = e; return e; }
    arena_t a;
    memset(&a, 0, sizeof a);
    a.out_off = (uint64_t*)calloc(1, sizeof(uint64_t));
    uint64_t p = RIO_FILE_HEADER_BYTES;
    uint64_t first_bad = UINT64_MAX, n_bad = 0;
    int status = RIO_OK;
    for (;;) {
        brd r = {f + p, len - p, 0, res->version == RIO_VERSION4 ? RIO_RECORD_HEADER_V4_MAX : UINT64_MAX};
        hdr_t h;
        memset(&h, 0, sizeof h);
        switch (res->version) { /* ReadNext dispatch, file_reader.go:66-73 */
        case RIO_VERSION1: e = read_header_v1(f + p, len - p, &h); break;
        case RIO_VERSION2: e = read_header_v2(&r, &h); break;
        case RIO_VERSION3: e = read_header_v3(&r, &h); break;
        default: e = read_header_v4(&r, &h); break;
        }
        if (e) {
            if (e == RIO_ERR_MAGIC && res->version != RIO_VERSION1) {
                /* io.ReadAll of the remainder after the consumed magic varint; all zeros => EOF */
                int zero = 1;
                for (uint64_t q = p + h.magic_len; q < len; q++)
                    if (f[q]) { zero = 0; break; }
                e = zero ? RIO_EOF_ZERO_TAIL : RIO_ERR_MAGIC;
            }
            if (e == RIO_ERR_HEADER_CRC) { res->detail0 = h.exp_crc; res->detail1 = h.act_crc; }
            status = e;
            break;
        }
        if (h.nil) { /* file_reader.go:96-99: nil ⇒ no payload, whatever c says */
            arena_push(&a, p, NULL, 0, 1);
            p += h.hdr_len;
            continue;
        }
        uint64_t plen = res->compression != RIO_COMP_NONE ? h.c : h.u; /* common_reader.go:162-169 */
        uint64_t avail = len - p - h.hdr_len;
        if (plen > avail) { /* io.ReadFull: 0 bytes => io.EOF, partial => ErrUnexpectedEOF */
            status = (avail == 0) ? RIO_EOF_PAYLOAD : RIO_ERR_UNEXPECTED_EOF;
            /* detail0 = 1: raised by the payload read (file_reader.go:104-107), not inside a header
             * varint; the error's text and SkipNext's answer (:146-148 vs :157-168) differ */
            if (status == RIO_ERR_UNEXPECTED_EOF) res->detail0 = 1;
            break;
        }
        const uint8_t* pay = f + p + h.hdr_len;
        if (res->compression != RIO_COMP_NONE) {
            uint8_t* dec = NULL;
            uint64_t dlen = 0;
            e = decompress(res->compression, pay, plen, &dec, &dlen);
            if (e == RIO_ERR_DECOMPRESS || e == RIO_EOF_CODEC) {
                /* ReadNext returns the codec error; the payload is consumed and the loop goes on */
                const uint64_t rsv = bad_reserve(res->compression, pay, plen, h.u);
                uint8_t* z = (uint8_t*)calloc(rsv ? rsv : 1, 1);
                arena_push(&a, p, z, rsv, 0);
                free(z);
                a.flags[a.n - 1] = e == RIO_ERR_DECOMPRESS ? RIO_FLAG_CORRUPT : RIO_FLAG_EOF;
                if (!n_bad) first_bad = a.n - 1;
                n_bad++;
                p += h.hdr_len + plen;
                continue;
            }
            if (e) { status = e; break; }
            arena_push(&a, p, dec, dlen, 0);
            free(dec);
        } else {
            arena_push(&a, p, pay, plen, 0);
        }
        p += h.hdr_len + plen;
    }
    res->status = status;
    res->status_offset = p;
    res->n_records = a.n;
    res->total_out_bytes = a.out_len;
    res->out = a.out;
    res->out_off = a.out_off;
    res->rec_off = a.rec_off;
    res->flags = a.flags;
    res->first_bad = first_bad;
    res->n_bad = n_bad;
    return RIO_OK;
}

void orc_file_result_free(orc_file_result* res) {
    free(res->out);
    free(res->out_off);
    free(res->rec_off);
    free(res->flags);
    memset(res, 0, sizeof *res);
}

/* ---------------------------------------------------------------------------------------- */
/* MMapReader.ReadNextAt (mmap_reader.go:130-203 v4; readNextAtV3 :298-356; V2 :242-296;      */
/* V1 :205-240)                                                                              */
/* ---------------------------------------------------------------------------------------- */
int orc_read_next_at(const uint8_t* f, uint64_t len, uint64_t offset, uint8_t** out,
                     uint64_t* out_len, int* is_nil, uint64_t* detail0, uint64_t* detail1) {
    uint32_t ver, comp;
    uint64_t det;
    *out = NULL;
    *out_len = 0;
    *is_nil = 0;
    *detail0 = *detail1 = 0;
    int e = orc_file_header(f, len, &ver, &comp, &det);
    if (e) return e;
    /* x/exp/mmap ReadAt: off > len => "mmap: invalid ReadAt offset"; 0 bytes => bare io.EOF */
    if (offset > len) return RIO_ERR_INVALID_OFFSET;
    /* V1: a 20-byte ReadAt; short of it (0 bytes included) the error wraps io.EOF (:209-212) */
    if (ver == RIO_VERSION1 && len - offset < 20) return RIO_EOF_HEADER;
    uint64_t wmax = ver == RIO_VERSION4 ? RIO_RECORD_HEADER_V4_MAX : RIO_RECORD_HEADER_V3_MAX;
    uint64_t w = len - offset < wmax ? len - offset : wmax;
    if (w == 0) return RIO_EOF;
    brd r = {f + offset, w, 0, ver == RIO_VERSION4 ? RIO_RECORD_HEADER_V4_MAX : UINT64_MAX};
    hdr_t h;
    memset(&h, 0, sizeof h);
    switch (ver) {
    case RIO_VERSION1: e = read_header_v1(f + offset, len - offset, &h); break;
    case RIO_VERSION2: e = read_header_v2(&r, &h); break;
    case RIO_VERSION3: e = read_header_v3(&r, &h); break;
    default: e = read_header_v4(&r, &h); break;
    }
    if (e == RIO_EOF) e = RIO_EOF_HEADER; /* wrapped: "failed reading record header at offset" */
    if (e == RIO_ERR_HEADER_CRC) { *detail0 = h.exp_crc; *detail1 = h.act_crc; }
    if (e) return e;
    if (h.nil) { *is_nil = 1; return RIO_OK; }
    uint64_t plen = comp != RIO_COMP_NONE ? h.c : h.u;
    if (plen > len - offset - h.hdr_len) return RIO_EOF_PAYLOAD; /* short ReadAt => io.EOF */
    const uint8_t* pay = f + offset + h.hdr_len;
    if (comp != RIO_COMP_NONE) return decompress(comp, pay, plen, out, out_len);
    *out = (uint8_t*)malloc(plen ? plen : 1);
    if (plen) memcpy(*out, pay, plen);
    *out_len = plen;
    return RIO_OK;
}

/* ---------------------------------------------------------------------------------------- */
/* MMapReader.SeekNext (mmap_reader.go:58-128): windowed scan for the bytes 91 8d 4c, trial    */
/* ReadNextAt at each hit; header-CRC / magic / io.EOF-class failures continue the scan.      */
/* ---------------------------------------------------------------------------------------- */
int orc_seek_next(const uint8_t* f, uint64_t len, uint64_t offset, uint64_t seek_len,
                  uint64_t* rec_offset, uint8_t** out, uint64_t* out_len, int* is_nil) {
    static const uint8_t M[3] = {0x91, 0x8D, 0x4C};
    uint32_t ver, comp;
    uint64_t det, d0, d1;
    *out = NULL;
    *out_len = 0;
    *is_nil = 0;
    *rec_offset = 0;
    int e = orc_file_header(f, len, &ver, &comp, &det);
    if (e) return e;
    if (ver < RIO_VERSION2) return RIO_ERR_UNSUPPORTED; /* :62-64 */
    if (seek_len == 0) seek_len = 4096;
    uint64_t next = offset;
    for (;;) {
        if (next > len) return RIO_ERR_INVALID_OFFSET;
        uint64_t num = len - next < seek_len ? len - next : seek_len;
        if (num == 0) return RIO_EOF;
        const uint8_t* buf = f + next;
        uint64_t i = 0;
        int boundary = 0;
        while (i < num) {
            uint64_t ix = i;
            for (int j = 0; j < 3; j++) {
                if (buf[ix] != M[j]) break;
                ix++;
                if (ix >= num) { boundary = 1; break; }
            }
            if (boundary) break;
            if (ix - i < 3) { i = ix + 1; continue; }
            uint64_t trial = next + i;
            uint8_t* rec = NULL;
            uint64_t rl = 0;
            int nil = 0;
            e = orc_read_next_at(f, len, trial, &rec, &rl, &nil, &d0, &d1);
            if (e) {
                if (e == RIO_ERR_HEADER_CRC || e == RIO_ERR_MAGIC || rio_status_is_eof(e)) {
                    i = ix;
                    continue;
                }
                *rec_offset = trial; /* the failing trial (the reference returns 0 and its error) */
                return e;
            }
            *rec_offset = trial;
            *out = rec;
            *out_len = rl;
            *is_nil = nil;
            return RIO_OK;
        }
        if (i == 0) return RIO_EOF; /* :121-124 */
        next += i;
    }
}

/* ---------------------------------------------------------------------------------------- */
/* CPU baseline helper: record-parallel ReadNextAt over known offsets (pthreads)              */
/* ---------------------------------------------------------------------------------------- */
typedef struct {
    const uint8_t* f;
    uint64_t len;
    const uint64_t* off;
    uint64_t lo, hi;
    uint64_t bytes;
    int err;
} par_arg;

static void* par_worker(void* vp) {
    par_arg* a = (par_arg*)vp;
    for (uint64_t i = a->lo; i < a->hi; i++) {
        uint8_t* o = NULL;
        uint64_t ol = 0, d0, d1;
        int nil = 0;
        int e = orc_read_next_at(a->f, a->len, a->off[i], &o, &ol, &nil, &d0, &d1);
        if (e) a->err = e;
        a->bytes += ol;
        free(o);
    }
    return NULL;
}

uint64_t orc_parallel_read_at(const uint8_t* f, uint64_t len, const uint64_t* rec_off, uint64_t n,
                              int threads) {
    if (threads <= 0) threads = 1;
    if (!crc_ready) crc_init();
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    par_arg* args = (par_arg*)calloc((size_t)threads, sizeof(par_arg));
    for (int t = 0; t < threads; t++) {
        args[t] = (par_arg){f, len, rec_off, n * (uint64_t)t / threads, n * (uint64_t)(t + 1) / threads, 0, 0};
        pthread_create(&th[t], NULL, par_worker, &args[t]);
    }
    uint64_t total = 0;
    int err = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        total += args[t].bytes;
        if (args[t].err) err = 1;
    }
    free(th);
    free(args);
    return err ? 0 : total;
}

/* status helpers shared with the product's vocabulary (rio.h); the oracle keeps its own copy so
 * the library under test is never linked into the checker. */
int rio_status_is_eof(int s) {
    return s == RIO_EOF || s == RIO_EOF_ZERO_TAIL || s == RIO_EOF_HEADER || s == RIO_EOF_PAYLOAD || s == RIO_EOF_CODEC;
}

/* ---------------------------------------------------------------------------------------- */
/* sstables: checksumValue (sstable_reader.go:240-248) = Go hash/crc64 with crc64.ISO           */
/* (reflected poly 0xD800000000000000, init/xorout all ones)                                 */
/* ---------------------------------------------------------------------------------------- */
uint64_t orc_crc64_iso(const uint8_t* p, uint64_t n) {
    static uint64_t tab[256];
    static int init = 0;
    if (!init) {
        for (int i = 0; i < 256; i++) {
            uint64_t c = (uint64_t)i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xD800000000000000ull & (0ull - (c & 1)));
            tab[i] = c;
        }
        init = 1;
    }
    uint64_t c = ~0ull;
    for (uint64_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

/* protowire.ConsumeVarint: <= 10 bytes, the 10th <= 1 */
static int pb_varint(const uint8_t* b, uint64_t n, uint64_t* pos, uint64_t* v) {
    uint64_t x = 0;
    for (int i = 0; i < 10; i++) {
        if (*pos >= n) return -1;
        uint8_t c = b[(*pos)++];
        if (i == 9 && c > 1) return -1;
        x |= (uint64_t)(c & 0x7F) << (7 * i);
        if (c < 0x80) { *v = x; return 0; }
    }
    return -1;
}

/* skip one field value of wire type wt (protowire.ConsumeFieldValue); groups to their end tag */
static int pb_skip(const uint8_t* b, uint64_t n, uint64_t* pos, uint64_t num, int wt, int depth) {
    uint64_t v;
    switch (wt) {
    case 0: return pb_varint(b, n, pos, &v);
    case 1: if (n - *pos < 8) return -1; *pos += 8; return 0;
    case 5: if (n - *pos < 4) return -1; *pos += 4; return 0;
    case 2:
        if (pb_varint(b, n, pos, &v) || v > n - *pos) return -1;
        *pos += v;
        return 0;
    case 3: /* groups nest at most 16 deep here and on the device (protowire allows 10000) */
        if (depth >= 16) return -1;
        for (;;) {
            uint64_t tag;
            if (pb_varint(b, n, pos, &tag)) return -1;
            uint64_t fn = tag >> 3;
            int t = (int)(tag & 7);
            if (fn < 1 || fn > 0x1FFFFFFFull) return -1;
            if (t == 4) return fn == num ? 0 : -1;
            if (pb_skip(b, n, pos, fn, t, depth + 1)) return -1;
        }
    default: return -1; /* 4 (unmatched end group), 6, 7 */
    }
}

/* proto.Unmarshal into a reset IndexEntry (sstables/proto/sstable.proto:5-9): key = 1 (bytes),
 * valueOffset = 2 (varint), checksum = 3 (varint); last occurrence wins; a known field with
 * another wire type and unknown fields are skipped. Returns 0, or -1 for malformed input. */
int orc_index_entry(const uint8_t* b, uint64_t n, uint64_t* key_off, uint64_t* key_len, uint64_t* value_off,
                    uint64_t* checksum) {
    uint64_t pos = 0;
    *key_off = *key_len = *value_off = *checksum = 0;
    while (pos < n) {
        uint64_t tag, v;
        if (pb_varint(b, n, &pos, &tag)) return -1;
        uint64_t fn = tag >> 3;
        int wt = (int)(tag & 7);
        if (fn < 1 || fn > 0x1FFFFFFFull) return -1;
        if (fn == 1 && wt == 2) {
            if (pb_varint(b, n, &pos, &v) || v > n - pos) return -1;
            *key_off = pos;
            *key_len = v;
            pos += v;
        } else if ((fn == 2 || fn == 3) && wt == 0) {
            if (pb_varint(b, n, &pos, &v)) return -1;
            if (fn == 2) *value_off = v; else *checksum = v;
        } else if (pb_skip(b, n, &pos, fn, wt, 0)) {
            return -1;
        }
    }
    return 0;
}

/* proto.Unmarshal into a reset DataEntry {value = 1} (sstables/proto/sstable.proto:12-14; v0 tables'
 * values, read through MMapProtoReader.ReadNextAt, recordio/proto/mmap_proto_reader.go:12-24):
 * *present = 1 when field 1 was seen with wire type 2 (the last one wins), [value_off, + value_len).
 * Returns -1 for malformed input. */
int orc_data_entry(const uint8_t* b, uint64_t n, int* present, uint64_t* value_off, uint64_t* value_len) {
    uint64_t pos = 0;
    *present = 0;
    *value_off = *value_len = 0;
    while (pos < n) {
        uint64_t tag, v;
        if (pb_varint(b, n, &pos, &tag)) return -1;
        uint64_t fn = tag >> 3;
        int wt = (int)(tag & 7);
        if (fn < 1 || fn > 0x1FFFFFFFull) return -1;
        if (fn == 1 && wt == 2) {
            if (pb_varint(b, n, &pos, &v) || v > n - pos) return -1;
            *present = 1;
            *value_off = pos;
            *value_len = v;
            pos += v;
        } else if (pb_skip(b, n, &pos, fn, wt, 0)) {
            return -1;
        }
    }
    return 0;
}

/* NewSSTableReader (index load + validateDataFile) + Scan over in-memory data.rio / index.rio
 * images, for the CPU baseline: returns the entries scanned (0 on a decode / proto failure),
 * *first_bad = first checksum mismatch or UINT64_MAX. Values pair with entries by position after
 * checking valueOffset against the record offset (the writer's layout). */
uint64_t orc_sst_scan(const uint8_t* index, uint64_t ilen, const uint8_t* data, uint64_t dlen, uint64_t* first_bad) {
    orc_file_result ri, rd;
    *first_bad = UINT64_MAX;
    orc_file_reader_decode(index, ilen, &ri);
    orc_file_reader_decode(data, dlen, &rd);
    uint64_t n = 0;
    if (ri.status == RIO_EOF && rd.status == RIO_EOF && ri.n_records <= rd.n_records) {
        for (n = 0; n < ri.n_records; n++) {
            uint64_t ko, kl, vo, cs;
            const uint8_t* rec = ri.out + ri.out_off[n];
            if (orc_index_entry(rec, ri.out_off[n + 1] - ri.out_off[n], &ko, &kl, &vo, &cs) || vo != rd.rec_off[n]) {
                n = 0;
                break;
            }
            const uint64_t c = orc_crc64_iso(rd.out + rd.out_off[n], rd.out_off[n + 1] - rd.out_off[n]);
            if (cs != 0 && c != cs && *first_bad == UINT64_MAX) *first_bad = n;
        }
    }
    orc_file_result_free(&ri);
    orc_file_result_free(&rd);
    return n;
}

/* ---------------------------------------------------------------------------------------- */
/* DiskKeyIndex.binarySearch (sstables/disk_key_index.go:87-127) over a fresh index (empty     */
/* offsetCache): sort.Search over byte offsets [0, size) where each probe is findAt(h) =        */
/* MMapProtoReader.SeekNext(h) (recordio/proto/mmap_proto_reader.go:26-38) + proto.Unmarshal    */
/* into an IndexEntry. An io.EOF probe ends the search as "not found" at offset size; any other */
/* probe error is returned. Status: RIO_OK, the SeekNext error, or ORC_ERR_PROTO.              */
/* ---------------------------------------------------------------------------------------- */
#define ORC_ERR_PROTO 21

static int bytes_compare(const uint8_t* a, uint64_t an, const uint8_t* b, uint64_t bn) {
    uint64_t m = an < bn ? an : bn;
    int c = m ? memcmp(a, b, m) : 0;
    if (c) return c < 0 ? -1 : 1;
    return an < bn ? -1 : (an > bn ? 1 : 0);
}

/* findAt: returns 0 with the entry, or a status; *eof = the error is io.EOF-class */
static int find_at(const uint8_t* f, uint64_t len, uint64_t h, uint64_t seek_len, uint8_t** rec, uint64_t* key_off,
                   uint64_t* key_len, uint64_t* vo, uint64_t* cs) {
    uint64_t ro, rl;
    int nil;
    *rec = NULL;
    int e = orc_seek_next(f, len, h, seek_len, &ro, rec, &rl, &nil);
    if (e) return e;
    if (orc_index_entry(*rec ? *rec : (const uint8_t*)"", nil ? 0 : rl, key_off, key_len, vo, cs)) return ORC_ERR_PROTO;
    return 0;
}

int orc_disk_index_search(const uint8_t* f, uint64_t len, const uint8_t* key, uint64_t klen, uint64_t seek_len,
                          uint64_t* offset, int* found, uint64_t* value_off, uint64_t* checksum) {
    uint64_t n = len, i = 0, j = n, ko, kl, vo, cs;
    uint8_t* rec = NULL;
    *offset = 0;
    *found = 0;
    *value_off = *checksum = 0;
    while (i < j) {
        uint64_t h = (i + j) >> 1;
        int e = find_at(f, len, h, seek_len, &rec, &ko, &kl, &vo, &cs);
        if (e) {
            free(rec);
            if (rio_status_is_eof(e)) { *offset = n; return RIO_OK; }
            return e;
        }
        int c = bytes_compare(rec + ko, kl, key, klen);
        free(rec);
        rec = NULL;
        if (c < 0) i = h + 1; else j = h;
    }
    int e = find_at(f, len, i, seek_len, &rec, &ko, &kl, &vo, &cs);
    if (e) {
        free(rec);
        if (rio_status_is_eof(e)) { *offset = n; return RIO_OK; }
        return e;
    }
    *offset = i;
    *found = i < n && bytes_compare(rec + ko, kl, key, klen) == 0;
    if (*found) { *value_off = vo; *checksum = cs; }
    free(rec);
    return RIO_OK;
}

/* ---------------------------------------------------------------------------------------- */
/* Write side (checker and CPU baseline of rio_device_encode): FileWriter.Write over a batch    */
/* (recordio/file_writer.go:160-233) with golang/snappy v1.0.0's Encode (encode.go:18-41,       */
/* encode_other.go: emitLiteral, emitCopy, encodeBlock). Restated from the published Go source. */
/* ---------------------------------------------------------------------------------------- */
static uint32_t le32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t le64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t snappy_hash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

static uint64_t w_uvarint(uint8_t* b, uint64_t v) {
    uint64_t i = 0;
    for (; v >= 0x80; v >>= 7) b[i++] = (uint8_t)(v | 0x80);
    b[i++] = (uint8_t)v;
    return i;
}

static uint64_t w_literal(uint8_t* dst, const uint8_t* lit, uint64_t n) {
    uint64_t i, m = n - 1;
    if (m < 60) { dst[0] = (uint8_t)(m << 2); i = 1; }
    else if (m < 256) { dst[0] = 60 << 2; dst[1] = (uint8_t)m; i = 2; }
    else { dst[0] = 61 << 2; dst[1] = (uint8_t)m; dst[2] = (uint8_t)(m >> 8); i = 3; }
    memcpy(dst + i, lit, n);
    return i + n;
}

static uint64_t w_copy(uint8_t* dst, uint64_t offset, uint64_t length) {
    uint64_t i = 0;
    for (; length >= 68; length -= 64, i += 3) {
        dst[i] = 63 << 2 | 2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
    }
    if (length > 64) {
        dst[i] = 59 << 2 | 2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3;
        length -= 60;
    }
    if (length >= 12 || offset >= 2048) {
        dst[i] = (uint8_t)((length - 1) << 2 | 2); dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
        return i + 3;
    }
    dst[i] = (uint8_t)((offset >> 8) << 5 | (length - 4) << 2 | 1);
    dst[i + 1] = (uint8_t)offset;
    return i + 2;
}

static uint64_t w_block(uint8_t* dst, const uint8_t* src, int64_t n) {
    static uint16_t table[1 << 14];
    uint32_t shift = 24;
    for (int64_t ts = 1 << 8; ts < (1 << 14) && ts < n; ts *= 2) shift--;
    memset(table, 0, sizeof table);
    uint64_t d = 0;
    const int64_t s_limit = n - 15;
    int64_t next_emit = 0, s = 1;
    uint32_t next_hash = snappy_hash(le32(src + s), shift);
    for (;;) {
        int64_t skip = 32, next_s = s, candidate = 0;
        for (;;) {
            s = next_s;
            int64_t between = skip >> 5;
            next_s = s + between;
            skip += between;
            if (next_s > s_limit) goto remainder;
            candidate = table[next_hash];
            table[next_hash] = (uint16_t)s;
            next_hash = snappy_hash(le32(src + next_s), shift);
            if (le32(src + s) == le32(src + candidate)) break;
        }
        d += w_literal(dst + d, src + next_emit, (uint64_t)(s - next_emit));
        for (;;) {
            int64_t base = s;
            s += 4;
            for (int64_t i = candidate + 4; s < n && src[i] == src[s]; i++, s++) {}
            d += w_copy(dst + d, (uint64_t)(base - candidate), (uint64_t)(s - base));
            next_emit = s;
            if (s >= s_limit) goto remainder;
            uint64_t x = le64(src + s - 1);
            table[snappy_hash((uint32_t)x, shift)] = (uint16_t)(s - 1);
            uint32_t ch = snappy_hash((uint32_t)(x >> 8), shift);
            candidate = table[ch];
            table[ch] = (uint16_t)s;
            if ((uint32_t)(x >> 8) != le32(src + candidate)) {
                next_hash = snappy_hash((uint32_t)(x >> 16), shift);
                s++;
                break;
            }
        }
    }
remainder:
    if (next_emit < n) d += w_literal(dst + d, src + next_emit, (uint64_t)(n - next_emit));
    return d;
}

/* snappy.Encode into dst (capacity >= 32 + n + n / 6) */
uint64_t orc_snappy_encode(uint8_t* dst, const uint8_t* src, uint64_t n) {
    uint64_t d = w_uvarint(dst, n);
    while (n > 0) {
        uint64_t blk = n < 65536 ? n : 65536;
        d += blk < 17 ? w_literal(dst + d, src, blk) : w_block(dst + d, src, (int64_t)blk);
        src += blk;
        n -= blk;
    }
    return d;
}

/* The file FileWriter writes for these records (compression none, snappy or lzw): returns its length,
 * or 0 when it would exceed cap. rec_off[i] = file offset of record i (Write's return value). */
uint64_t orc_encode_file(const uint8_t* records, const uint64_t* off, const uint8_t* flags, uint64_t n, uint32_t comp,
                         uint8_t* out, uint64_t cap, uint64_t* rec_off) {
    if (cap < 8) return 0;
    uint64_t o = 8;
    out[0] = 4; out[1] = out[2] = out[3] = 0;
    out[4] = (uint8_t)comp; out[5] = out[6] = out[7] = 0;
    uint8_t* scratch = NULL;
    uint64_t scap = 0;
    for (uint64_t i = 0; i < n; i++) {
        int nil = flags && (flags[i] & 1);
        uint64_t u = nil ? 0 : off[i + 1] - off[i], c = 0;
        const uint8_t* pay = records + off[i];
        uint64_t plen = u;
        if (comp == RIO_COMP_SNAPPY) {
            if (scap < 32 + u + u / 6) {
                free(scratch);
                scap = 32 + u + u / 6;
                scratch = (uint8_t*)malloc(scap);
            }
            c = orc_snappy_encode(scratch, pay, u);
            pay = scratch;
            plen = c;
        } else if (comp == RIO_COMP_LZW) { /* nil records too: c = len(Compress(nil)), file_writer.go:198-207 */
            if (scap < 16 + 2 * u) {
                free(scratch);
                scap = 16 + 2 * u;
                scratch = (uint8_t*)malloc(scap);
            }
            c = orc_lzw_encode(scratch, pay, u);
            pay = scratch;
            plen = c;
        }
        uint8_t h[40];
        uint64_t k = w_uvarint(h, 0x130691);
        h[k++] = nil ? 1 : 0;
        k += w_uvarint(h + k, u);
        k += w_uvarint(h + k, c);
        k += w_uvarint(h + k, orc_crc32c(h, k));
        uint64_t sz = k + (nil ? 0 : plen);
        if (o + sz > cap) { free(scratch); return 0; }
        memcpy(out + o, h, k);
        if (!nil && plen) memcpy(out + o + k, pay, plen);
        if (rec_off) rec_off[i] = o;
        o += sz;
    }
    free(scratch);
    return o;
}
