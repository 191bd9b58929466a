import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "styletts2-lite_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(autouse=True)
def _production_options():
    """Every test starts and ends on the production engine options (STTS_OPT_* defaults,
    automatic BiLSTM kernel choice): an A/B test cannot leak its setting into later tests."""
    from stts2_mi355x import engine
    engine.reset_options()
    yield
    engine.reset_options()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
