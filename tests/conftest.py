import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmythgpu)")


@pytest.fixture(scope="session")
def engine():
    """The HIP engine on cuda:0.  GPU tests fail (not skip) when it is
    unavailable: a silent fallback would hide a broken native path."""
    from mythril_amd.engine import get_engine
    return get_engine(0)


@pytest.fixture(autouse=True)
def _fresh_shape_statistics():
    """Each test starts with no per-shape hit statistics (model._shape_gate):
    a test's expectations must not depend on which queries earlier tests of
    the session happened to miss."""
    import mythril_amd.model as M
    M._shape_stats.clear()
    yield
