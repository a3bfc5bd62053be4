"""The partition arithmetic the two multi-GPU combines share, host only (no GPU): the reduce-scatter key slices
(pgpu_slice_of vs combine.slice_of / reduce_scatter_sections' ceil(G / world) chunks) and the hash-key owners
(pgpu_key_owner vs combine.key_owners, the routing of DistributedExecutor._hash_merge_topk), so that the node-level
combine inside the library (pgpu_node.cpp) and the one-process-per-GPU combine (combine.py) partition alike."""
import ctypes as C

import numpy as np
import pytest

from pinot_amd import _lib
from pinot_amd.combine import key_owners, slice_of


@pytest.fixture(scope="module")
def lib():
    return _lib.load()


@pytest.mark.parametrize("G", [1, 7, 64, 1000, 1 << 20, (1 << 20) + 3])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_slices(lib, G, world):
    first, count = C.c_uint64(), C.c_uint64()
    covered = 0
    for r in range(world):
        lib.pgpu_slice_of(G, world, r, C.byref(first), C.byref(count))
        assert (first.value, count.value) == slice_of(G, world, r)
        assert first.value == covered or count.value == 0
        covered += count.value
    assert covered == G


@pytest.mark.parametrize("kw", [1, 2])
@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_key_owners(lib, kw, world):
    rng = np.random.default_rng(kw * 10 + world)
    keys = rng.integers(0, 1 << 62, (500, kw), dtype=np.int64)
    keys[:5] = [[0] * kw, [1] * kw, [(1 << 63) - 1] * kw, [12345] * kw, [7] * kw]
    want = key_owners(keys, world)
    got = [lib.pgpu_key_owner(np.ascontiguousarray(k).ctypes.data_as(C.POINTER(C.c_int64)), kw, world) for k in keys]
    assert list(want) == got
    if world > 1:  # the routing spreads keys
        assert len(set(got)) == world
    assert lib.pgpu_key_owner(None, kw, world) == -1
