"""Shared test plumbing.

`gpu`-marked tests need a visible HIP device (run on the MI355X box); the rest
run on CPU: the oracle against the reference's known-answer tests, host logic,
and ABI loading.
"""
import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "cpu-raytracing-rt_amd")
sys.path.insert(0, REPO)


def load_package():
    """Import the product package (its directory name has dashes)."""
    if "rt_amd" in sys.modules:
        return sys.modules["rt_amd"]
    spec = importlib.util.spec_from_file_location("rt_amd", os.path.join(PKG_DIR, "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rt_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # noqa: E402
    return oracle


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); parity tests through the C ABI")


@pytest.fixture(scope="session")
def rt():
    return load_package()


@pytest.fixture(scope="session")
def orc():
    return load_oracle()


@pytest.fixture(scope="session")
def scene_text():
    def read(name):
        with open(os.path.join(REPO, "scenes", name)) as f:
            return f.read()
    return read
