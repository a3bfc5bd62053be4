import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libpinotgpu.so")
    # torch ships its own HIP runtime; when both are used in one process let torch initialise first
    # (libpinotgpu.so never hands its pointers or streams to torch; see pinot_amd/combine.py).
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


@pytest.fixture(scope="session")
def gpu_ctx():
    from pinot_amd.segment import GpuContext
    ctx = GpuContext(0)
    yield ctx
    ctx.close()
