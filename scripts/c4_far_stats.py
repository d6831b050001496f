# Host statistics of C4-shaped Snappy streams (far pieces, 128-B line requests of their 16-B windows, the line-shift
# and 8-byte-window counts behind profiles/r6/r6l_far_line_ab.txt). usage: python scripts/c4_far_stats.py
import sys, struct
sys.path.insert(0, 'go-sstables_amd'); sys.path.insert(0, 'tests')
from recordio import generate
img = bytes(generate(300, 65536, 2, kind=1, seed=100))
# walk v4 records: magic(3) nil(1) uvarint u, uvarint c, uvarint crc
def uv(b, p):
    v = s = 0
    while True:
        x = b[p]; p += 1; v |= (x & 0x7F) << s; s += 7
        if x < 0x80: return v, p
p = 8; streams = []
while p < len(img):
    q = p + 4
    u, q = uv(img, q); c, q = uv(img, q); _, q = uv(img, q)
    streams.append(img[q:q+c]); p = q + c
kFar = 232
stats = dict(lit_bytes=0, near_bytes=0, far_bytes=0, far_pieces16=0, far_req16=0, far_pieces32=0, far_req32=0, steps16=0, steps32=0, far_copies=0)
for st in streams[:200]:
    s = 0; _, s = uv(st, 0); d = 0
    while s < len(st):
        tag = st[s]; t = tag & 3
        if t == 0:
            x = tag >> 2
            if x < 60: L = x + 1; s += 1
            else:
                nb = x - 59; L = int.from_bytes(st[s+1:s+1+nb], 'little') + 1; s += 1 + nb
            stats['lit_bytes'] += L; s += L
            # pieces: capped at 16 - (d&3) (header piece simplification ignored)
            dd = d; rem = L
            while rem: n = min(rem, 16 - (dd & 3)); rem -= n; dd += n; stats['steps16'] += 1
            dd = d; rem = L
            while rem: n = min(rem, 32 - (dd & 3)); rem -= n; dd += n; stats['steps32'] += 1
            d += L; continue
        if t == 1: L = ((tag >> 2) & 7) + 4; off = ((tag & 0xE0) << 3) | st[s+1]; s += 2
        elif t == 2: L = (tag >> 2) + 1; off = st[s+1] | (st[s+2] << 8); s += 3
        else: L = (tag >> 2) + 1; off = struct.unpack_from('<I', st, s+1)[0]; s += 5
        if off > kFar:
            stats['far_bytes'] += L; stats['far_copies'] += 1
            for cap, kp, kr, ks in ((16, 'far_pieces16', 'far_req16', 'steps16'), (32, 'far_pieces32', 'far_req32', 'steps32')):
                dd = d; rem = L
                while rem:
                    r = dd & 3; n = min(rem, cap - r); q = dd - off
                    w0 = q - r  # window start (abs position in record; line alignment ~ arena offset: record base 64KiB aligned)
                    lines = ((w0 + cap - 1) // 128) - (w0 // 128) + 1
                    stats[kp] += 1; stats[kr] += lines; stats[ks] += 1
                    rem -= n; dd += n
        else:
            stats['near_bytes'] += L
            dd = d; rem = L; e = off
            while rem: n = min(rem, 16 - (dd & 3), e); rem -= n; dd += n; e += n if n == e else 0; stats['steps16'] += 1
            dd = d; rem = L; e = off
            while rem: n = min(rem, 32 - (dd & 3), e); rem -= n; dd += n; e += n if n == e else 0; stats['steps32'] += 1
        d += L
tot = stats['lit_bytes'] + stats['near_bytes'] + stats['far_bytes']
print({k: v for k, v in stats.items()}, 'total', tot)
print('far bytes frac %.3f, far bytes/copy %.1f, far req per 16B-piece %.3f, 32B %.3f' % (stats['far_bytes']/tot, stats['far_bytes']/stats['far_copies'], stats['far_req16']/stats['far_pieces16'], stats['far_req32']/stats['far_pieces32']))
print('steps16 %d steps32 %d ratio %.3f; far req16 %d req32 %d ratio %.3f' % (stats['steps16'], stats['steps32'], stats['steps32']/stats['steps16'], stats['far_req16'], stats['far_req32'], stats['far_req32']/stats['far_req16']))
# case analysis on 16-B pieces: straddling windows whose copy bytes fit one line (shiftable), and 8-B windows
strad = shiftable = fits8 = req8 = 0
for st in streams[:200]:
    s = 0; _, s = uv(st, 0); d = 0
    while s < len(st):
        tag = st[s]; t = tag & 3
        if t == 0:
            x = tag >> 2
            if x < 60: L = x + 1; s += 1
            else:
                nb = x - 59; L = int.from_bytes(st[s+1:s+1+nb], 'little') + 1; s += 1 + nb
            s += L; d += L; continue
        if t == 1: L = ((tag >> 2) & 7) + 4; off = ((tag & 0xE0) << 3) | st[s+1]; s += 2
        elif t == 2: L = (tag >> 2) + 1; off = st[s+1] | (st[s+2] << 8); s += 3
        else: L = (tag >> 2) + 1; off = struct.unpack_from('<I', st, s+1)[0]; s += 5
        if off > kFar:
            dd = d; rem = L
            while rem:
                r = dd & 3; n = min(rem, 16 - r); q = dd - off; w0 = q - r
                a = w0 % 128
                if a > 112:
                    strad += 1
                    if (q % 128) + n <= 128 and (q % 128) >= a: shiftable += 1   # copy within w0's line
                    elif (q // 128) != (w0 // 128) and ((q + n - 1) // 128) == (q // 128): shiftable += 1  # copy within next line (case A)
                if r + n <= 8:
                    fits8 += 1; req8 += 1 + (1 if (w0 % 128) > 120 else 0)
                else:
                    req8 += 1 + (1 if a > 112 else 0)
                rem -= n; dd += n
        d += L
print('far pieces %d straddling %d (%.3f) shiftable %d (%.3f of far req16); fits8 %d (%.3f); req with 8B loads %d (ratio %.3f)' % (
    stats['far_pieces16'], strad, strad / stats['far_pieces16'], shiftable, shiftable / stats['far_req16'], fits8, fits8 / stats['far_pieces16'], req8, req8 / stats['far_req16']))
