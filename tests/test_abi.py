"""The drop-in boundary: libpinotgpu.so loads and exports every entry point include/pinot_gpu.h declares (CPU)."""
import ctypes as C
import os
import re

import pytest

from pinot_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pinot_gpu.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pgpu_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "pgpu_query_launch" in names and "pgpu_segment_add_forward_index" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes signature table covers every declared function
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == declared_functions()


def test_abi_version_and_struct_sizes():
    lib = _lib.load()
    assert lib.pgpu_abi_version() == _lib.ABI_VERSION
    assert C.sizeof(_lib.FilterNode) == 48
    assert C.sizeof(_lib.Agg) == 8
    assert C.sizeof(_lib.QueryStats) == 80


def test_init_fails_loudly_without_a_gpu():
    """No CPU fallback: without a visible gfx950 device pgpu_init returns an error with a message."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib = _lib.load()
    h = C.c_void_p()
    rc = lib.pgpu_init(0, C.byref(h))
    assert rc != 0
    assert _lib.last_error()
    from pinot_amd.segment import GpuContext
    with pytest.raises(_lib.PinotGpuError):
        GpuContext(0)


def test_minmax_key_decoding():
    lib = _lib.load()
    assert lib.pgpu_decode_minmax_key(-5, _lib.PGPU_INT) == -5.0
    import struct
    for v in (-3.5, 0.0, 2.25, -1e300, 7e-310):
        b = struct.unpack("<q", struct.pack("<d", v))[0]
        key = b if b >= 0 else b ^ 0x7FFFFFFFFFFFFFFF
        assert lib.pgpu_decode_minmax_key(key, _lib.PGPU_DOUBLE) == v


def test_ctypes_structs_match_the_c_header(tmp_path):
    """Every ctypes struct mirrors include/pinot_gpu.h: sizeof and every field offset, checked by compiling the
    header with gcc (the same layout the JNI stub in INTEGRATION.md sees)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"pgpu_filter_node": _lib.FilterNode, "pgpu_agg": _lib.Agg, "pgpu_segment_plan": _lib.SegmentPlan,
               "pgpu_query_desc": _lib.QueryDesc, "pgpu_table_layout": _lib.TableLayout,
               "pgpu_query_stats": _lib.QueryStats, "pgpu_literal": _lib.Literal, "pgpu_expr_node": _lib.ExprNode}
    lines = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{ROOT}/include/pinot_gpu.h"', "int main(void){"]
    for cname, ct in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in ct._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    out = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                        text=True).stdout.splitlines())
    for cname, ct in structs.items():
        assert int(out[cname]) == C.sizeof(ct), cname
        for fname, _ in ct._fields_:
            assert int(out[f"{cname}.{fname}"]) == getattr(ct, fname).offset, (cname, fname)


def test_fixed_sum_layout_matches_restatement():
    """pgpu_fixed_sum_layout (the layout's fixed-point window) against tests/helpers.fixed_sum_layout."""
    import math
    import numpy as np
    from tests.helpers import _lsb_exp, fixed_sum_layout
    lib = _lib.load()
    rng = np.random.default_rng(3)
    cases = [np.array([0.0]), np.array([1.0, 2.0, 3.0]), np.array([0.5, 0.25]), np.array([1e-3, 1e12]),
             np.array([1e-20, 1.0]), np.array([1e-200, 1e200]), rng.normal(0, 1, 1000), np.array([-7.5, 3e9]),
             np.round(rng.normal(0, 100, 500), 2), np.array([5e-324, 1.0]), np.array([2.0 ** 61, 1.0]),
             rng.uniform(1, 2, 100).astype(np.float32).astype(np.float64)]
    for v in cases:
        nz = np.abs(v[v != 0])
        mx = float(np.abs(v).max())
        mn_exp = math.frexp(float(nz.min()))[1] - 1 if len(nz) else 2 ** 31 - 1
        mn_lsb = min(_lsb_exp(float(x)) for x in nz) if len(nz) else 2 ** 31 - 1
        e, p = C.c_int32(), C.c_int32()
        lib.pgpu_fixed_sum_layout(mx, mn_exp, mn_lsb, C.byref(e), C.byref(p))
        assert (e.value, p.value) == fixed_sum_layout(v), (v[:4], e.value, p.value, fixed_sum_layout(v))


def test_sum_layout_agree_matches_combine():
    """pgpu_sum_layout_agree (the node combine) and plan.fixed_window (combine.py over RCCL) choose one window."""
    from pinot_amd.plan import fixed_window
    lib = _lib.load()
    cases = [[(-40, 3)], [(-40, 3), (-20, 3)], [(-90, 5), (-10, 3)], [(-120, 6), (10, 3)],
             [(_lib.PGPU_SUM_EXP_ZERO, 3), (-50, 4)], [(_lib.PGPU_SUM_EXP_F64, 1), (-50, 4)],
             [(_lib.PGPU_SUM_EXP_ZERO, 3)]]
    for case in cases:
        arr = (_lib.TableLayout * len(case))()
        for i, (e, p) in enumerate(case):
            arr[i].agg_value_type[0] = _lib.PGPU_DOUBLE
            arr[i].agg_sum_exp[0] = e
            arr[i].agg_sum_parts[0] = p
        oe, op = (C.c_int32 * 1)(), (C.c_int32 * 1)()
        assert lib.pgpu_sum_layout_agree(arr, len(case), 1, oe, op) == 0
        live = [(e, p) for e, p in case if e not in (_lib.PGPU_SUM_EXP_F64, _lib.PGPU_SUM_EXP_ZERO)]
        if any(e == _lib.PGPU_SUM_EXP_F64 for e, _ in case):
            want = (_lib.PGPU_SUM_EXP_F64, 1)
        elif not live:
            want = (_lib.PGPU_SUM_EXP_ZERO, 3)
        else:
            want = fixed_window(max(e + 21 * p for e, p in live), min(e for e, _ in live))
        assert (oe[0], op[0]) == want, (case, oe[0], op[0], want)
