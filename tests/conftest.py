import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "default_numerics: a GPU test of the default numerics "
                            "(fast var on the register tiles), not the exact replay")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    oracle.load()
    return oracle


@pytest.fixture(autouse=True)
def exact_var_replay(request, monkeypatch):
    """GPU tests compare the moment features bit for bit with the reference, so they run
    the exact fp64 replay of var_parallel_impl (engine.EXACT_VAR); the tests of the default
    numerics (fast var, tolerance gc.FAST_VAR_RTOL) pass exact_var=False explicitly or
    carry the marker ``default_numerics``."""
    if request.node.get_closest_marker("gpu") is None or \
            request.node.get_closest_marker("default_numerics") is not None:
        return
    try:
        from pymhealth_amd import engine
    except Exception:       # torch missing: the GPU tests skip themselves
        return
    monkeypatch.setattr(engine, "EXACT_VAR", True)
