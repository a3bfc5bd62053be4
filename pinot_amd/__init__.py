"""pinot_amd — MI355X-native segment query path for Apache Pinot (filter -> aggregate / group-by -> combine).

Host-side mirror of the reference's plan-maker / operator surface over the C ABI of libpinotgpu.so
(include/pinot_gpu.h).  See DESIGN.md for the path, the HBM layout and the kernels.
"""
from .query import parse_sql, QueryContext  # noqa: F401
