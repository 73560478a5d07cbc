import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native_ext():
    """The _C extension (kernels + checkpoint/bundle bindings); built in-tree if stale/missing."""
    from tools.build_ext import build_kernels
    build_kernels()
    from tensorflow_k8s_amd.ops._lib import lib
    return lib()


@pytest.fixture(scope="session")
def control_plane_bin():
    """Native control-plane binaries (cpp/ -> build/bin), built incrementally."""
    from tools.build_ext import build_control_plane
    build_control_plane()
    return os.path.join(ROOT, "build", "bin")


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
