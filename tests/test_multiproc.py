"""World-size-2 rehearsal of the file-sharded multi-GPU job on CPU (gloo backend).

The decode path shards by file with no data-path collective: every rank
decodes its own file and the job reports the slowest rank's time and the summed input bytes. This
test runs bench.py's own sharding / seeding / reduction code in two gloo processes; the per-rank
decode is the CPU oracle standing in for the device (the device leg is bench.py on the GPU box).
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
