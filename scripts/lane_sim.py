"""Pieces per record and per lane for the C2 workload (k_snappy_pipe cost model).

Parses the snappy element streams of a generated C2-style file on the host and counts the <=16-byte
pieces the decoder emits per record (one per loop step), then groups 8 records per lane and 64 lanes
per wave to estimate the bubble fraction (lanes idle while the wave's slowest lane finishes).
usage: python scripts/lane_sim.py"""
import sys, numpy as np
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "go-sstables_amd"))
from recordio import generate
n = 64 * 64 * 8 * 4
img = bytes(generate(n, 1024, 2, 1, seed=1, threads=8))
def uv(b, p):
    r = sh = 0
    while True:
        x = b[p]; p += 1; r |= (x & 0x7F) << sh; sh += 7
        if x < 0x80: return r, p
p = 8; pieces = []; elems = []
while p < len(img) and len(pieces) < n:
    _, p = uv(img, p); p += 1; u, p = uv(img, p); c, p = uv(img, p); _, p = uv(img, p)
    s = img[p:p + c]; p += c
    _, q = uv(s, 0)  # snappy preamble: decoded length
    cnt = 0; ne = 0
    while q < len(s):
        tag = s[q]; t = tag & 3; x = tag >> 2; ne += 1
        if t == 0:
            if x < 60: L = x + 1; hl = 1
            else: k = x - 59; L = int.from_bytes(s[q+1:q+1+k], "little") + 1; hl = 1 + k
            first = min(L, 16 - hl); cnt += 1; rem = L - first; cnt += (rem + 15) // 16; q += hl + L
        else:
            if t == 1: L = ((x) & 7) + 4; off = ((tag & 0xE0) << 3) | s[q+1]; q += 2
            elif t == 2: L = x + 1; off = int.from_bytes(s[q+1:q+3], "little"); q += 3
            else: L = x + 1; off = int.from_bytes(s[q+1:q+5], "little"); q += 5
            eff = off; rem = L
            while rem:
                m = min(rem, 16, eff); cnt += 1; rem -= m
                if eff < 16 and m == eff: eff *= 2
    pieces.append(cnt); elems.append(ne)
pc = np.array(pieces)
print("records", len(pc), "pieces/record mean %.1f std %.1f" % (pc.mean(), pc.std()), "elems/record %.1f" % np.mean(elems))
for rpl in (8,):
    lanes = pc[: (len(pc) // (rpl * 64)) * rpl * 64].reshape(-1, 64, rpl).sum(2)
    print("rpl", rpl, "lane steps mean %.1f, wave max mean %.1f -> active fraction %.3f" % (lanes.mean(), lanes.max(1).mean(), lanes.mean() / lanes.max(1).mean()))
