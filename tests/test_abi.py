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
    assert C.sizeof(_lib.QueryStats) == 72


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
