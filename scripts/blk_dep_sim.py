"""Dependency depth of record-parallel Snappy decode on the C4 data.

A decoder that materialises one record with many lanes at once (north star's workgroup-per-record
shape) can only write a copy once the bytes it copies are final. This script parses real C4 records
(the bench generator's text-like 64 KiB records, golang/snappy-compatible encoder) into elements and
counts, for two scheduling rules, how many rounds such a decoder needs when every element whose
sources are final goes in the same round:
  rule A (frontier): a copy goes when its source ends below the first element still pending;
  rule B (byte-exact): a copy goes when every byte it reads is final.
Elements are taken in batches (consecutive elements: a wave's or workgroup's set) or in input-byte
segments. Also prints the copy-offset distribution (how far back the sources are).
usage: python scripts/blk_dep_sim.py  (about 5 minutes on one core)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "go-sstables_amd"))
from recordio import generate  # noqa: E402


def uv(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def records(img):
    i = 8
    while i + 3 <= len(img):
        i += 4  # magic + nil byte (v4)
        _, i = uv(img, i)
        c, i = uv(img, i)
        _, i = uv(img, i)
        yield img[i:i + c]
        i += c


def elems(s):
    """(input position, dst, kind 0 literal / 1 copy, length, copy offset) per element"""
    dl, i = uv(s, 0)
    d = 0
    out = []
    while i < len(s):
        t = s[i]
        k = t & 3
        if k == 0:
            n = t >> 2
            if n < 60:
                i += 1
                L = n + 1
            else:
                nb = n - 59
                L = int.from_bytes(s[i + 1:i + 1 + nb], "little") + 1
                i += 1 + nb
            out.append((i, d, 0, L, 0))
            i += L
        elif k == 1:
            L = 4 + ((t >> 2) & 7)
            out.append((i, d, 1, L, ((t & 0xE0) << 3) | s[i + 1]))
            i += 2
        elif k == 2:
            L = 1 + (t >> 2)
            out.append((i, d, 1, L, s[i + 1] | s[i + 2] << 8))
            i += 3
        else:
            L = 1 + (t >> 2)
            out.append((i, d, 1, L, int.from_bytes(s[i + 1:i + 5], "little")))
            i += 5
        d += L
    assert d == dl
    return out


def rounds(seg, rule_b):
    d0 = seg[0][1]
    fin = np.zeros(seg[-1][1] + seg[-1][3] - d0 + 1, bool)
    done = [False] * len(seg)
    r = 0
    while not all(done):
        F = min(seg[k][1] for k in range(len(seg)) if not done[k])
        go = []
        for k, e in enumerate(seg):
            if done[k]:
                continue
            if e[2] == 0:
                go.append(k)
                continue
            s0 = e[1] - e[4]
            need = min(e[1], s0 + e[3])
            if rule_b:
                lo, hi = max(s0, d0) - d0, need - d0
                if hi <= lo or fin[lo:hi].all():
                    go.append(k)
            elif need <= F:
                go.append(k)
        for k in go:
            e = seg[k]
            fin[e[1] - d0:e[1] - d0 + e[3]] = True
            done[k] = True
        r += 1
    return r


def main():
    nrec = 4
    img = bytes(generate(nrec, 65536, 2, kind=1, seed=7, threads=8))
    recs = [elems(s) for s in records(img)]
    ne = sum(len(e) for e in recs)
    print(f"{nrec} C4 records: {ne / nrec:.0f} elements per record")
    for B in (32, 64, 128):
        for rb in (False, True):
            T = sum(rounds(es[i:i + B], rb) for es in recs for i in range(0, len(es), B))
            print(f"  batches of {B:3d} elements, rule {'B' if rb else 'A'}: {T / nrec:6.0f} rounds per record "
                  f"({ne / T:.1f} elements per round)")
    for seg_in in (1024, 4096):
        for rb in (False, True):
            T = 0
            for es in recs:
                i = 0
                while i < len(es):
                    j = i
                    while j < len(es) and es[j][0] < es[i][0] + seg_in:
                        j += 1
                    T += rounds(es[i:j], rb)
                    i = j
            print(f"  input segments of {seg_in} B, rule {'B' if rb else 'A'}: {T / nrec:6.0f} rounds per record")
    offs = np.array([e[4] for es in recs for e in es if e[2]])
    lens = np.array([e[3] for es in recs for e in es if e[2]])
    print("copy offsets (fraction of copies / of copied bytes at or below):")
    for t in (64, 232, 1024, 4096, 16384, 65536):
        m = offs <= t
        print(f"  {t:6d}: {m.mean():.3f} / {lens[m].sum() / lens.sum():.3f}")


if __name__ == "__main__":
    main()
