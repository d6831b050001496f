"""Source checks on the HIP kernels (no GPU needed).

Round 3's parser/emitter hang came from `min(uint32_t, int)` resolving to HIP's `min(double, double)`
(DESIGN.md §4). Kernels use rio::umin / rio::umax (rio_dev_util.h), which static_assert that both
operands have the same integer type; this test keeps bare min( / max( calls out of csrc/*.hip.
"""
import glob
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go-sstables_amd", "csrc")
BARE = re.compile(r"(?<![\w:.])(min|max)\s*\(")


def _code(line: str) -> str:
    return line.split("//", 1)[0]


def test_no_bare_min_max_in_kernels():
    bad = []
    for path in sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "rio_dev*.h"))):
        for i, ln in enumerate(open(path), 1):
            if BARE.search(_code(ln)):
                bad.append(f"{os.path.basename(path)}:{i}: {ln.strip()}")
    assert not bad, "use rio::umin / rio::umax (same-type operands):\n" + "\n".join(bad)
