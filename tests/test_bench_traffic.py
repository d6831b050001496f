"""bench.py's HBM-traffic plumbing on the CPU: the rocprofv3 counter parser (against a trimmed counter file of a
real MI355X pass, tests/data/rocprof_fetch_size_c2.csv), the live two-pass measurement driven through a stand-in
profiler on PATH (what the bench computes from the counters, and that a failed pass is reported, not guessed),
and the committed-file source with its tree check."""
import json
import math
import os
import shutil
import stat
import sys

import bench

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "data", "rocprof_fetch_size_c2.csv")


def test_pmc_counter_takes_the_max_over_the_kernel_dispatches(tmp_path):
    d = tmp_path / "pass" / "nested"
    d.mkdir(parents=True)
    shutil.copy(FIXTURE, d / "run_counter_collection.csv")
    # six k_snappy_pipe dispatches: the capacity probe (19.5 KiB) and five real launches
    assert bench.pmc_counter(str(tmp_path), "FETCH_SIZE", "k_snappy_pipe") == (1445493.375, 6)
    assert bench.pmc_counter(str(tmp_path), "FETCH_SIZE", "k_walk") == (341011.375, 2)
    v, k = bench.pmc_counter(str(tmp_path), "WRITE_SIZE", "k_snappy_pipe")
    assert k == 0 and math.isnan(v)


FAKE = r'''#!{python}
import os, sys
a = sys.argv[1:]
ctr, out = a[a.index("--pmc") + 1], a[a.index("-d") + 1]
if os.environ.get("FAKE_PROF_FAIL") == ctr:
    sys.exit(1)
val = {{"FETCH_SIZE": "100.0", "WRITE_SIZE": "50.0"}}[ctr]
os.makedirs(os.path.join(out, "host"), exist_ok=True)
with open(os.path.join(out, "host", "run_counter_collection.csv"), "w") as f:
    f.write('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n')
    f.write('1,"rio::k_snappy_pipe(rio::FrameParams)","%s",1.0\n' % ctr)
    f.write('2,"rio::k_snappy_pipe(rio::FrameParams)","%s",%s\n' % (ctr, val))
    f.write('3,"rio::k_walk(rio::FrameParams)","%s",999999.0\n' % ctr)
'''


def _stand_in(tmp_path, monkeypatch):
    b = tmp_path / "bin"
    b.mkdir()
    p = b / "rocprofv3"
    p.write_text(FAKE.format(python=sys.executable))
    p.chmod(p.stat().st_mode | stat.S_IXUSR)
    monkeypatch.setenv("PATH", str(b) + os.pathsep + os.environ.get("PATH", ""))


def test_live_traffic_from_two_counter_passes(tmp_path, monkeypatch):
    _stand_in(tmp_path, monkeypatch)
    t = bench.live_traffic("c2", timeout_s=60)
    # FETCH_SIZE doubled on gfx950, both in KiB: 2 x 100 KiB read + 50 KiB written per launch
    assert t["traffic_read"] == 2 * 100.0 * 1024 and t["traffic_write"] == 50.0 * 1024
    assert t["traffic"] == t["traffic_read"] + t["traffic_write"]
    src = t["traffic_source"]
    assert src["kind"] == "live" and src["kernel"] == "k_snappy_pipe" and src["tree"] == bench.source_tree_hash()


def test_live_traffic_reports_a_failed_pass(tmp_path, monkeypatch):
    _stand_in(tmp_path, monkeypatch)
    monkeypatch.setenv("FAKE_PROF_FAIL", "WRITE_SIZE")
    t = bench.live_traffic("c2", timeout_s=60)
    assert "traffic" not in t and "WRITE_SIZE" in t["error"]


def test_file_traffic_says_whether_it_is_this_tree(tmp_path):
    f = tmp_path / "traffic_c2.json"
    f.write_text(json.dumps({"config": "c2", "decode_kernel_bytes_per_launch": 4.0e9, "tree": "0123456789abcdef"}))
    t = bench.file_traffic("c2", str(f))
    assert t["traffic"] == 4.0e9 and t["traffic_source"]["same_tree"] is False
    f.write_text(json.dumps({"config": "c2", "decode_kernel_bytes_per_launch": 4.0e9, "tree": bench.source_tree_hash()}))
    assert bench.file_traffic("c2", str(f))["traffic_source"]["same_tree"] is True
    # another config's file is not used
    assert bench.file_traffic("c3", str(f)) == {"traffic": None}


def test_device_digest_sees_every_byte_and_its_place():
    """bench.verify's digest (the timed steps must rebuild the warmup's bytes): equal bytes give equal digests;
    a flipped bit, two words swapped inside one 4096-word row or across rows, or a changed tail byte do not."""
    import torch

    g = torch.Generator().manual_seed(5)
    base = torch.randint(0, 256, (3 * 4096 * 8 + 45,), dtype=torch.uint8, generator=g)
    d0 = bench.device_digest(base)
    assert bench.device_digest(base.clone()) == d0
    w = base[: 3 * 4096 * 8].view(torch.int64)

    def changed(edit):
        x = base.clone()
        edit(x, x[: 3 * 4096 * 8].view(torch.int64))
        return bench.device_digest(x) != d0

    assert int(w[10]) != int(w[20]) and int(w[5]) != int(w[4096 + 5])

    def swap(i, j):
        def f(x, xw):
            xw[i], xw[j] = int(w[j]), int(w[i])
        return f

    assert changed(lambda x, xw: x.__setitem__(777, int(x[777]) ^ 1))
    assert changed(swap(10, 20))  # inside one row
    assert changed(swap(5, 4096 + 5))  # the same place in two rows
    assert changed(lambda x, xw: x.__setitem__(x.numel() - 3, (int(x[-3]) + 1) % 256))
