import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libpinotgpu.so")


@pytest.fixture(scope="session")
def gpu_ctx():
    from pinot_amd.segment import GpuContext
    ctx = GpuContext(0)
    yield ctx
    ctx.close()
