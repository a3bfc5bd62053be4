"""scripts/pmc_summarize.py: which kernels of a rocprofv3 trace belong to a query's timed region, and which one marks
a query launch (one per query), for every kernel-name shape the runtime launches -- including the phase-1 variants
whose template arguments carry the fixed-bit widths (part_scan_kernel<false, 20, 16>)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location("pmc_summarize", os.path.join(ROOT, "scripts", "pmc_summarize.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_query_launch_kernels():
    m = _mod()
    main = ["void (anonymous namespace)::query_kernel_rdirect<2, 10, 3>(DevParams)",
            "void (anonymous namespace)::part_scan_kernel<false>(DevParams)",
            "void (anonymous namespace)::part_scan_kernel<false, 20, 16>(DevParams)",
            "void (anonymous namespace)::part_scan_kernel<false, 16, 16>(DevParams)"]
    for n in main:
        assert m._is_main(n) and m._is_timed(n), n
    # the sampling pass and phase 2 are timed but are not the per-query launch marker
    for n in ["void (anonymous namespace)::part_scan_kernel<true, 0, 0>(DevParams)",
              "void (anonymous namespace)::part_reduce_kernel<2, true, 2>(DevParams, int)",
              "(anonymous namespace)::part_plan_kernel(DevParams, int)"]:
        assert m._is_timed(n) and not m._is_main(n), n
    # prologue / epilogue and PyTorch's kernels are outside the timed region
    for n in ["(anonymous namespace)::finalize_kernel(DevParams, int, long*, unsigned char*, int, long*, unsigned long)",
              "(anonymous namespace)::prologue_kernel(unsigned int __vector(4) const*, unsigned int __vector(4)*, "
              "unsigned int, int, DevParams)",
              "void at::native::vectorized_elementwise_kernel<4, at::native::FillFunctor<long>>(int, void*)"]:
        assert not m._is_timed(n), n
