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


def test_code_prefetch_stays_inside_each_kernel(tmp_path):
    """code_pf (rio_kernels.hip) reads kPf* 64-byte lines of a kernel's code from its s_getpc_b64 on: every line
    must lie inside that kernel's own code in the built gfx950 object (a read past the code object would fault)."""
    import subprocess

    import pytest

    llvm = "/opt/rocm/llvm/bin"
    obj = os.path.join(CSRC, "build", "rio_kernels.o")
    tools = [os.path.join(llvm, t) for t in ("clang-offload-bundler", "llvm-readelf", "llvm-objdump", "llvm-objcopy")]
    if not os.path.exists(obj) or not all(os.path.exists(t) for t in tools):
        pytest.skip("no built rio_kernels.o or no ROCm LLVM tools")
    src = open(os.path.join(CSRC, "rio_kernels.hip")).read()
    lines = {k: int(v) for k, v in re.findall(r"kPf(\w+) = (\d+)", src)}
    co, fb = str(tmp_path / "k.elf"), str(tmp_path / "fatbin")
    # the host object carries the device code as an offload bundle in .hip_fatbin
    subprocess.run([tools[3], "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
    subprocess.run([tools[0], "--unbundle", "--type=o", f"--input={fb}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True)
    syms = {}
    for ln in subprocess.run([tools[1], "-s", co], check=True, capture_output=True, text=True).stdout.splitlines():
        f = ln.split()
        if len(f) >= 8 and f[3] == "FUNC":
            syms[f[7]] = (int(f[1], 16), int(f[2]))
    kernels = {"_ZN3rio13k_scan_blocksE": "Scan", "_ZN3rio7k_placeILj16E": "Place", "_ZN3rio7k_placeILj64E": "Place",
               "_ZN3rio14k_copy_recordsE": "Copy", "_ZN3rio8k_finishE": "Finish", "_ZN3rio14k_finish_batchE": "Finish",
               "_ZN3rio6k_walkE": "Walk"}
    checked = 0
    for name, (addr, size) in syms.items():
        kind = next((v for k, v in kernels.items() if name.startswith(k)), None)
        if kind is None:
            continue
        dis = subprocess.run([tools[2], "-d", f"--disassemble-symbols={name}", co], check=True, capture_output=True,
                             text=True).stdout
        m = re.search(r"s_getpc_b64.*//\s*([0-9A-Fa-f]+):", dis)
        assert m, f"{name}: no s_getpc_b64 (code_pf missing)"
        pc = int(m.group(1), 16) + 4  # s_getpc_b64 returns the next instruction's address
        last = pc + 64 * (lines[kind] - 1) + 4
        assert last <= addr + size, f"{name}: prefetch to {last:#x} past the kernel end {addr + size:#x}"
        checked += 1
    assert checked == len(kernels), checked
