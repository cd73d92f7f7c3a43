import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "nerf-rep_for_test_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


def golden_names(prefix=""):
    """The crop fixtures f<digit>..._<name>.npz (not the whole-frame companions)."""
    import re
    return sorted(f[:-4] for f in os.listdir(GOLDEN)
                  if re.match(r"f\d", f) and f.endswith(".npz") and f.startswith(prefix))


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
