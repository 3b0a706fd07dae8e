"""Shared test plumbing. `gpu`-marked tests need an MI355X (run on the GPU box); everything
else runs on CPU. The oracle (oracle/) is imported ONLY here, as the checker."""
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "ed25519-consensus_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP path, no fallback)")


def load_pkg():
    if "ed25519_consensus_amd" in sys.modules:
        return sys.modules["ed25519_consensus_amd"]
    spec = importlib.util.spec_from_file_location("ed25519_consensus_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ed25519_consensus_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ed25519_ref  # noqa: E402
    return ed25519_ref


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def edc():
    return load_pkg()


@pytest.fixture(scope="session")
def oracle():
    return load_oracle()


@pytest.fixture(scope="session")
def engine(edc):
    # GPU tests share the process with torch (device tensors): import it before the HIP
    # library is loaded so both use one HIP runtime (see load_library()).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    eng = edc.Engine(0)
    yield eng
    eng.close()
