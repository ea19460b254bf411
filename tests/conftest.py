import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and the HIP library")


@pytest.fixture(scope="session")
def golden_cases():
    from oracle_lib import golden_names, load_golden
    return {n: load_golden(n) for n in golden_names()}
