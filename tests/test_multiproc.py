"""World-size-2 rehearsal of the file-sharded multi-GPU job on CPU (gloo backend).

The decode path shards by file with no data-path collective: every rank
decodes its own files and the job reports the slowest rank's time and the summed input bytes. These
tests run bench.py's own per-rank code (bench.run_decode: file plan, generation, warm-up, barriers,
timed steps, gloo reductions, the JSON line) in two gloo processes. The single substitution is the
device call itself: a backend with bench.DeviceBackend's interface that decodes with the CPU oracle,
because this container has no GPU (the device leg is bench.py on the GPU box).
"""
import hashlib
import os
import socket
import sys

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int):
    for p in (REPO, os.path.join(REPO, "go-sstables_amd"), os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle_py as orc
        from recordio import generate

        ws, rk, local = bench.dist_env()
        assert (ws, rk, local) == (world, rank, rank)
        # C4-style sharding: 8 equal files round-robin over the ranks, disjoint and complete
        mine = bench.shard_files(8, world, rank)
        shards = [None] * world
        dist.all_gather_object(shards, mine)
        assert sorted(f for s in shards for f in s) == list(range(8))
        # every rank decodes its own, distinct file (bench.py: rank-seeded generator)
        image = generate(2000, 256, 2, kind=1, seed=bench.rank_seed(rank), threads=1)
        res = orc.file_reader_decode(bytes(image))
        assert res["status"] == 1 and res["n_records"] == 2000  # clean io.EOF after all records
        digests = [None] * world
        dist.all_gather_object(digests, hashlib.sha256(bytes(image)).hexdigest())
        assert len(set(digests)) == world
        # whole-job rate: max time over ranks, bytes summed over ranks
        dt = 0.010 * (rank + 1)
        steps = 3
        value, ms, dt_max = bench.job_throughput(dt, image.shape[0], steps, world, torch.device("cpu"))
        sizes = [None] * world
        dist.all_gather_object(sizes, int(image.shape[0]))
        want_dt = 0.010 * world
        assert dt_max == pytest.approx(want_dt)
        assert ms == pytest.approx(want_dt / steps * 1e3)
        assert value == pytest.approx(sum(sizes) * steps / 2**30 / want_dt)
    finally:
        dist.destroy_process_group()


def test_file_sharded_job_world2():
    mp.spawn(_worker, args=(2, _free_port()), nprocs=2, join=True)


class OracleBackend:
    """bench.DeviceBackend's interface with the device call replaced by the CPU oracle."""

    def __init__(self):
        self.steps = 0

    def load(self, images, batch):
        self.images, self.batch = images, batch
        self.step()
        return [int(img.shape[0]) for img in images]

    def step(self):
        import oracle_py as orc

        self.res = [orc.file_reader_decode_arrays(img) for img in self.images]
        self.steps += 1

    def sync(self):
        pass

    def infos(self):
        return [{k: r[k] for k in ("status", "n_records", "total_out_bytes")} for r in self.res]

    def set_timing(self, slots):
        pass

    def checksums(self):
        import hashlib

        return [tuple(hashlib.sha1(r[k].tobytes()).hexdigest()[:16] for k in ("out", "out_off", "rec_off", "flags"))
                for r in self.res]

    def stage_ms(self):
        return [0.01, 0.01, 0.01, 0.1] if self.images else []

    def evict(self):
        pass

    def rec_offs(self, n):
        return self.res[0]["rec_off"][:n]


def _run_decode_worker(rank: int, world: int, port: int, config: str, q):
    for p in (REPO, os.path.join(REPO, "go-sstables_amd"), os.path.join(REPO, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import argparse

        import bench

        args = argparse.Namespace(config=config, steps=3, warmup=1, no_cpu_baseline=True, no_e2e=True,
                                  traffic_json="/nonexistent")
        be = OracleBackend()
        line = bench.run_decode(args, world, rank, be, sizes=(150, 2048))
        q.put((rank, bench.plan_files(config, world, rank), be.steps, line))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("config,files_per_rank", [("c4", 4), ("c2", 1)])
def test_bench_run_decode_world2(config, files_per_rank):
    """bench.run_decode on two gloo ranks: C4's 8 files split 4/4 with no overlap, one file per rank
    otherwise; both ranks report the same whole-job value (sum of bytes over the max time)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run_decode_worker, args=(r, 2, port, config, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict((r, (seeds, steps, line)) for r, seeds, steps, line in (q.get(timeout=300) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = [got[r][0] for r in range(2)]
    assert all(len(s) == files_per_rank for s in seeds) and not set(seeds[0]) & set(seeds[1])
    if config == "c4":
        assert sorted(seeds[0] + seeds[1]) == list(range(100, 108))
    for r in range(2):
        _, steps, line = got[r]
        # load + warm-up + exactly args.steps timed + the cold-cache (MALL-flushed) pass of small files
        assert steps == 1 + 1 + 3 + 3 and "mall_flushed" in line
        assert line["n_gpus"] == 2 and line["config"]["files_this_rank"] == files_per_rank
        assert line["config"]["records"] == 150 * files_per_rank
        assert line["reproducible"] is True and line["verify"]["digest_out"]
        assert line["verified"] is None  # the oracle comparison rides on rank 0's cpu_baseline leg at N=1 only
    assert got[0][2]["value"] == got[1][2]["value"] > 0


class _DriftingBackend(OracleBackend):
    """An oracle backend whose timed steps produce different bytes (a decode that went wrong)."""

    def step(self):
        super().step()
        if self.steps > 2:
            self.res[0]["out"][0] ^= 0xFF


def test_bench_fails_when_timed_steps_diverge():
    """The headline is self-verifying: a timed step whose output differs from the
    warmup's makes run_decode raise instead of reporting a line."""
    import argparse

    import bench

    args = argparse.Namespace(config="c2", steps=3, warmup=1, no_cpu_baseline=True, no_e2e=True,
                              traffic_json="/nonexistent")
    with pytest.raises(RuntimeError, match="different results"):
        bench.run_decode(args, 1, 0, _DriftingBackend(), sizes=(150, 2048))
    line = bench.run_decode(args, 1, 0, OracleBackend(), sizes=(150, 2048))
    assert line["reproducible"] is True and line["roofline"]["traffic"] is None


def _bench_cli(args, env_extra=None, timeout=300):
    import subprocess

    env = dict(os.environ, RIO_BENCH_TEST_SIZES="150,2048", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "tests", "bench_cli_oracle.py")] + args,
                          env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("config,files_per_rank", [("c4", 4), ("c2", 1)])
def test_bench_gpus2_without_launcher_self_launches(config, files_per_rank):
    """`bench.py --gpus 2` started bare (the way the driver starts `--gpus 1`) runs 2 ranks, not a silent
    1-rank job: the line reports n_gpus 2, each rank its own share of the files (C4: 4 of the 8)."""
    import json

    r = _bench_cli(["--gpus", "2", "--config", config, "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                    "--no-e2e", "--traffic-json", "/nonexistent"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one line
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["config"]["files_this_rank"] == files_per_rank
    assert line["config"]["records"] == 150 * files_per_rank
    assert line["value"] > 0


def test_lpt_assign():
    """Longest-first assignment (rio_fileset_decode's rule): equal files alternate, a big file gets a
    device of its own, ties go to the lower slot."""
    import bench

    assert bench.lpt_assign([10] * 8, 2) == [[0, 2, 4, 6], [1, 3, 5, 7]]
    assert bench.lpt_assign([100, 10, 10, 10, 10, 60], 2) == [[0], [1, 2, 3, 4, 5]]
    assert bench.lpt_assign([5, 5, 5], 4) == [[0], [1], [2], []]
    assert sorted(sum(bench.lpt_assign([7, 3, 9, 1, 4], 3), [])) == [0, 1, 2, 3, 4]


@pytest.mark.parametrize("config,per_dev", [("c4", [4, 4]), ("c2", [1, 1])])
def test_bench_inproc_devices(config, per_dev):
    """`bench.py --inproc-devices 0,0`: one process, one thread and backend per listed device (the Go
    caller's shape), C4's 8 files split 4 / 4, the line verified; device 0 listed twice is the
    one-GPU rehearsal and says so."""
    import json

    r = _bench_cli(["--inproc-devices", "0,0", "--config", config, "--steps", "2", "--warmup", "1",
                    "--no-cpu-baseline", "--no-e2e"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == 2 and line["config"]["devices"] == [0, 0]
    assert line["config"]["files_per_device"] == per_dev
    assert line["reproducible"] is True and "rehearsal" in line["mode"] and line["value"] > 0


def test_bench_world_size_mismatch_refused():
    """A launcher's WORLD_SIZE that disagrees with --gpus is refused (non-zero exit), not reported."""
    r = _bench_cli(["--gpus", "4", "--steps", "1", "--warmup", "0"],
                   env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_cpu_baseline_hands_the_oracle_arrays_to_the_check():
    """bench.cpu_baseline calls `check` once with the oracle's out / out_off / rec_off / flags of the first file (the
    bench compares them with the device digests of the timed decode) and reports its answer as oracle_match."""
    import numpy as np

    import bench
    import oracle_py as orc
    from recordio import generate

    img = generate(300, 1024, 2, kind=1, seed=5)
    want = orc.file_reader_decode_arrays(img)
    seen = []

    def check(out, out_off, rec_off, flags):
        seen.append(1)
        return (np.array_equal(out, want["out"]) and np.array_equal(out_off.astype(np.int64), want["out_off"]) and
                np.array_equal(rec_off.astype(np.int64), want["rec_off"]) and np.array_equal(flags, want["flags"]))

    res = bench.cpu_baseline([img], np.asarray(want["rec_off"], dtype=np.uint64), 300, budget_s=0.2, check=check)
    assert seen == [1] and res["oracle_match"] is True
    res = bench.cpu_baseline([img], np.asarray(want["rec_off"], dtype=np.uint64), 300, budget_s=0.2,
                             check=lambda *a: False)
    assert res["oracle_match"] is False
