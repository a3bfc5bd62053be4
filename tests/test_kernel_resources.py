"""Register budget of the query kernels, read from the built code object (CPU only, no GPU needed).

The self-loading kernels' throughput rests on their occupancy: query_kernel_rdirect runs four 4-wave workgroups per
CU (<= 128 VGPRs; the aggregation-only mode three), query_kernel_direct five in its GLOBAL / HASH modes (<= 96), and
neither may use scratch.  A change to a shared device function that is inlined into them (the multi-value group-key
expansion once was: 153 VGPRs and 1.1 KB of scratch, config 5 0.35 -> 0.71 ms) shows up here, not only in a GPU
bench.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pinot_amd", "libpinotgpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"

pytestmark = pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                                reason="libpinotgpu.so not built or no ROCm LLVM tools")


def kernel_resources(path: str) -> dict:
    """{kernel symbol: {vgpr_count, sgpr_count, private_segment_fixed_size, ...}} of the gfx950 code object."""
    d = tempfile.mkdtemp()
    notes = ""
    try:
        fb = os.path.join(d, "fb")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        with open(fb, "rb") as f:
            blob = f.read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"  # one bundle per translation unit, concatenated
        starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
        for i, a in enumerate(starts):
            part, co = os.path.join(d, f"b{i}"), os.path.join(d, f"c{i}")
            with open(part, "wb") as f:
                f.write(blob[a: starts[i + 1] if i + 1 < len(starts) else len(blob)])
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                           capture_output=True)
            notes += subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                    capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(d, ignore_errors=True)
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name":
            cur = None if v.endswith(".kd") else out.setdefault(v, {})
        elif cur is not None:
            cur[k] = int(v)
    return out


@pytest.fixture(scope="module")
def res():
    r = kernel_resources(LIB)
    assert r, "no kernel metadata found"
    return r


def _mode(sym: str) -> int:
    return int(re.search(r"ILi(\d+)E", sym).group(1))


def test_register_direct_kernels_fit_four_waves_per_simd(res):
    ks = {k: v for k, v in res.items() if "query_kernel_rdirect" in k}
    assert ks
    for k, v in ks.items():
        assert v["private_segment_fixed_size"] == 0, (k, v)
        if _mode(k) != 0:  # PGPU_MODE_AGG keeps three workgroups per CU (pgpu_runtime.cpp)
            assert v["vgpr_count"] <= 128, (k, v)


def test_direct_kernels_fit_their_occupancy(res):
    ks = {k: v for k, v in res.items() if "query_kernel_direct" in k}
    assert ks
    for k, v in ks.items():
        assert v["private_segment_fixed_size"] == 0, (k, v)
        assert v["vgpr_count"] <= (96 if _mode(k) in (2, 4) else 128), (k, v)


def test_andfsm_kernels_do_not_spill(res):
    """The exact-filter-statistics transducer: no scratch in either build, and the two-sliced-leaf build (ILb1E) keeps
    four waves per SIMD."""
    ks = {k: v for k, v in res.items() if "andfsm_tile_kernel" in k}
    assert len(ks) == 2
    for k, v in ks.items():
        assert v["private_segment_fixed_size"] == 0 and v["vgpr_spill_count"] == 0, (k, v)
        if "ILb1E" in k:
            assert v["vgpr_count"] <= 128, (k, v)


def test_register_streaming_kernels_do_not_spill(res):
    """query_kernel_rstream / _rprog hold RD tiles of filter planes or bitmap words and value planes in VGPRs: no
    scratch in any variant."""
    ks = {k: v for k, v in res.items() if "query_kernel_rstream" in k or "query_kernel_rprog" in k}
    assert len(ks) == 9
    for k, v in ks.items():
        assert v["private_segment_fixed_size"] == 0 and v["vgpr_spill_count"] == 0, (k, v)
        if "rprogILi2ELi20E" in k:  # two 20-bit value columns (config 3): three waves per SIMD
            assert v["vgpr_count"] <= 168, (k, v)
