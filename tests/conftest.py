import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

PKG_NAME = "end-to-end-image-retrieval-service-with-k8s-jenkins_amd"
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def import_pkg(sub: str | None = None):
    """Import the package (its directory name is not an identifier) or one of its submodules."""
    name = PKG_NAME if sub is None else f"{PKG_NAME}.{sub}"
    return importlib.import_module(name)


@pytest.fixture(scope="session")
def pkg():
    return import_pkg()


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    if not gpu_available():
        pytest.fail("GPU test selected but no GPU is visible")
    import torch

    return torch.device("cuda", 0)
