"""bench.py's command line with the device call replaced by the CPU oracle (test infrastructure).

`python tests/bench_cli_oracle.py --gpus N ...` runs bench.main() unchanged — argument parsing, the
`--gpus` launch contract (self-launch of N ranks through torch.distributed.run when no launcher
started it), rank setup, gloo reductions and the JSON line — with two substitutions only, because
this container has no GPU: the rank's device is the CPU and the decode backend is the oracle
(tests/test_multiproc.py::OracleBackend). Records per file are cut to RIO_BENCH_TEST_SIZES
("records,record_bytes") so the run takes seconds. bench.py re-launches sys.argv[0], so every rank
runs this wrapper too.
"""
import functools
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "go-sstables_amd"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import bench  # noqa: E402
from test_multiproc import OracleBackend  # noqa: E402


def main():
    import torch

    sizes = tuple(int(x) for x in os.environ.get("RIO_BENCH_TEST_SIZES", "150,2048").split(","))
    bench.make_device = lambda local: torch.device("cpu")
    bench.make_backend = lambda local, device, own=False: OracleBackend()
    bench.make_inproc_device = lambda local: torch.device("cpu")
    bench.run_decode_inproc = functools.partial(bench.run_decode_inproc, sizes=sizes)
    bench.run_decode = functools.partial(bench.run_decode, sizes=sizes)
    bench.main()


if __name__ == "__main__":
    main()
