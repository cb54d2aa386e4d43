import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "tests"))
sys.path.insert(0, str(REPO / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def pkg():
    import helpers
    return helpers.load_package()


@pytest.fixture(scope="session")
def oracle():
    import helpers
    return helpers.load_oracle()


@pytest.fixture(scope="session")
def OcpQpBatch(pkg):
    return pkg.OcpQpBatch
