import gzip
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def example_paths(tmp_path_factory):
    """The reference's example data set (committed as tests/golden fixtures)."""
    d = tmp_path_factory.mktemp("example")
    csv = d / "input.csv"
    with gzip.open(os.path.join(GOLDEN, "example_input.csv.gz"), "rb") as fi, open(csv, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    return {"csv": str(csv), "config": os.path.join(GOLDEN, "example_csv_config.txt"),
            "params": os.path.join(GOLDEN, "example_parameter_file.txt")}


@pytest.fixture(scope="session")
def built():
    """Build (incrementally) the in-tree native libraries and the oracle."""
    from gfp_gaussian_process_amd import build_ext
    from oracle import oracle as O
    build_ext.build()
    O.build()
    return True
