"""Far-copy fetch model of the lane decoder (DESIGN §6, C4 / C2 traffic).

Generates the bench's records (rio_generate, kind=1 text, seed 100: C4's first file), walks every
Snappy element and counts, for the copies the lane decoder reads from the output arena (offset >
kFarOff = 208), the 64-byte and 128-byte lines its 16-byte far loads touch (one load per piece of
<= 16 bytes, at the 4-aligned source). The result, in fetched bytes per decoded byte, is what the
PMC FETCH_SIZE counts on top of the input stream when no far line survives in L2 between uses.
    python scripts/far_fetch_model.py [records] [record_len] [far threshold, default 232]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/go-sstables_amd")
from recordio.writer import generate  # noqa: E402

K_FAR = int(sys.argv[3]) if len(sys.argv) > 3 else 232  # kFarOff (rio_snappy.hip)


def uvarint(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    rl = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    img = generate(n, rl, 2, kind=1, seed=100).tobytes()
    t = dict(out=0, elements=0, pieces=0, far_elements=0, far_pieces=0, lines64=0, lines128=0)
    offs = []
    p = 8
    while p < len(img):
        assert img[p:p + 3] == b"\x91\x8d\x4c"  # v4 header: magic, nil byte, u, c, crc
        q = p + 4
        _, q = uvarint(img, q)
        c, q = uvarint(img, q)
        _, q = uvarint(img, q)
        pay = img[q:q + c]
        p = q + c
        _, i = uvarint(pay, 0)
        d = 0
        while i < len(pay):
            tag = pay[i]
            k = tag & 3
            t["elements"] += 1
            if k == 0:
                x = tag >> 2
                if x < 60:
                    ln, i = x + 1, i + 1
                else:
                    nb = x - 59
                    ln = int.from_bytes(pay[i + 1:i + 1 + nb], "little") + 1
                    i += 1 + nb
                i += ln
                t["pieces"] += (ln + 15) // 16
                d += ln
                continue
            if k == 1:
                ln, off, i = 4 + ((tag >> 2) & 7), ((tag >> 5) << 8) | pay[i + 1], i + 2
            elif k == 2:
                ln, off, i = 1 + (tag >> 2), pay[i + 1] | pay[i + 2] << 8, i + 3
            else:
                ln, off, i = 1 + (tag >> 2), int.from_bytes(pay[i + 1:i + 5], "little"), i + 5
            npc = (ln + 15) // 16
            t["pieces"] += npc
            if off > K_FAR:
                offs.append(off)
                t["far_elements"] += 1
                t["far_pieces"] += npc
                for j in range(npc):
                    a = (d - off + 16 * j) & ~3
                    t["lines64"] += (a + 15) // 64 - a // 64 + 1
                    t["lines128"] += (a + 15) // 128 - a // 128 + 1
            d += ln
        t["out"] += d
    o = np.array(offs)
    B = t["out"]
    print(t)
    print(f"bytes per element {B / t['elements']:.2f}, far elements {t['far_elements'] / t['elements']:.3f}")
    print("far offsets above: " + ", ".join(f"{x} B {float((o > x).mean()):.3f}" for x in (256, 1024, 2048, 4096, 16384)))
    print(f"far-load fetch per decoded byte: {t['lines128'] * 128 / B:.2f} B (128-B lines), {t['lines64'] * 64 / B:.2f} B (64-B)")
    print(f"input bytes per decoded byte: {len(img) / B:.3f}")


if __name__ == "__main__":
    main()
