"""pinot.server.query.executor.* / .gpu.* keys (pinot_amd/config.py) and the configurable server trim.  CPU only."""
import numpy as np
import pytest

from pinot_amd.config import GpuExecutorConfig, parse_devices
from pinot_amd.plan import GpuPlanMaker, table_capacity


def test_defaults_are_the_references():
    c = GpuExecutorConfig.from_properties({})
    assert (c.timeout_ms, c.num_groups_limit, c.max_init_group_holder_capacity, c.min_server_group_trim_size) == \
        (15_000, 100_000, 10_000, 5000)
    assert c.enabled and c.topk and not c.exact_filter_stats
    assert c.device_ids(8) == list(range(8))
    assert c.offload([1 << 20, 10]) == (True, "")


def test_keys_are_read():
    c = GpuExecutorConfig.from_properties({
        "pinot.server.query.executor.timeout": "2500",
        "pinot.server.query.executor.num.groups.limit": "2000000",
        "pinot.server.query.executor.max.init.group.holder.capacity": "512",
        "pinot.server.query.executor.min.server.group.trim.size": "-1",
        "pinot.server.query.executor.gpu.enabled": "TRUE",
        "pinot.server.query.executor.gpu.devices": "0x0d",
        "pinot.server.query.executor.gpu.min.segment.docs": "100000",
        "pinot.server.query.executor.gpu.min.query.docs": "1000000",
        "pinot.server.query.executor.gpu.exact.filter.stats": "true",
        "pinot.server.query.executor.gpu.topk": "false",
        "pinot.server.query.executor.pruner.class": "ColumnValueSegmentPruner",  # other executor keys pass
    })
    assert c.timeout_ms == 2500 and c.num_groups_limit == 2_000_000 and c.max_init_group_holder_capacity == 512
    assert c.min_server_group_trim_size == -1 and c.exact_filter_stats and not c.topk
    assert c.device_ids(8) == [0, 2, 3]
    assert c.resident(100_000) and not c.resident(99_999)
    ok, why = c.offload([200_000, 50_000])
    assert not ok and "min.segment.docs" in why
    ok, why = c.offload([200_000, 300_000])
    assert not ok and "min.query.docs" in why
    assert c.offload([600_000, 600_000]) == (True, "")
    pm = c.plan_maker(None)
    assert isinstance(pm, GpuPlanMaker)
    assert (pm.num_groups_limit, pm.max_init_group_holder_capacity, pm.timeout_ms, pm.exact_filter_stats,
            pm.gpu_topk, pm.min_server_group_trim_size) == (2_000_000, 512, 2500, True, False, -1)
    assert c.plan_maker(None, timeout_ms=7).timeout_ms == 7


def test_disabled_keeps_queries_on_cpu():
    c = GpuExecutorConfig.from_properties({"pinot.server.query.executor.gpu.enabled": "false"})
    assert c.offload([1 << 25]) == (False, "pinot.server.query.executor.gpu.enabled=false")
    assert not c.resident(1 << 25)


@pytest.mark.parametrize("props", [{"pinot.server.query.executor.gpu.enabled": "maybe"},
                                   {"pinot.server.query.executor.gpu.min.segment.docs": "1e5"},
                                   {"pinot.server.query.executor.gpu.devcies": "0"},
                                   {"pinot.server.query.executor.num.groups.limit": "0"}])
def test_bad_values_raise(props):
    with pytest.raises(ValueError):
        GpuExecutorConfig.from_properties(props)


def test_devices():
    assert parse_devices("all", 4) == [0, 1, 2, 3]
    assert parse_devices("3, 1,1", 4) == [1, 3]
    assert parse_devices("0x5", 4) == [0, 2]
    for bad in ("4", "0x10", "0x0", ","):
        with pytest.raises(ValueError):
            parse_devices(bad, 4)


def test_properties_file(tmp_path):
    p = tmp_path / "server.conf"
    p.write_text("# server\npinot.server.query.executor.gpu.devices = 1,2\n"
                 "! comment\npinot.server.query.executor.timeout: 900\n\n")
    c = GpuExecutorConfig.from_file(str(p))
    assert c.device_ids(4) == [1, 2] and c.timeout_ms == 900


def test_table_capacity_min_trim():
    # GroupByUtils.getTableCapacity(limit, minNumGroups); <= 0 disables the server trim
    assert table_capacity(10) == 5000
    assert table_capacity(2000) == 10000
    assert table_capacity(10, 100) == 100
    assert table_capacity(10, 0) >= 1 << 62


def test_derived_copy_columns():
    """…gpu.sliced.columns / …gpu.value.planes.columns: the GPU's IndexLoadingConfig (per-column derived copies)."""
    from pinot_amd._lib import PGPU_DERIVE_ALL, PGPU_DERIVE_SLICED, PGPU_DERIVE_VALUE_PLANES
    c = GpuExecutorConfig.from_properties({})
    assert c.derived_flags(["a", "b"]) == {"a": PGPU_DERIVE_ALL, "b": PGPU_DERIVE_ALL}
    c = GpuExecutorConfig.from_properties({
        "pinot.server.query.executor.gpu.sliced.columns": "daysSinceEpoch, accountId",
        "pinot.server.query.executor.gpu.value.planes.columns": "",
        "pinot.server.query.executor.gpu.derived.budget.bytes": "1000000"})
    f = c.derived_flags(["daysSinceEpoch", "accountId", "clicks"])
    assert f == {"daysSinceEpoch": PGPU_DERIVE_SLICED, "accountId": PGPU_DERIVE_SLICED, "clicks": 0}
    assert c.derived_budget_bytes == 1_000_000
    c = GpuExecutorConfig.from_properties({"pinot.server.query.executor.gpu.value.planes.columns": "m"})
    assert c.derived_flags(["m", "r"]) == {"m": PGPU_DERIVE_ALL, "r": PGPU_DERIVE_SLICED}
    assert PGPU_DERIVE_VALUE_PLANES | PGPU_DERIVE_SLICED == PGPU_DERIVE_ALL
