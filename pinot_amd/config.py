"""Server configuration of the GPU path: the ``pinot.server.query.executor.*`` keys the reference's plan maker reads,
plus the ``pinot.server.query.executor.gpu.*`` keys of this path.

Reference keys honoured (their defaults are the reference's):

* ``pinot.server.query.executor.timeout`` — query budget in ms when the query sets none
  (CommonConstants.java:302, DEFAULT_QUERY_EXECUTOR_TIMEOUT_MS 15,000 at :366);
* ``…num.groups.limit`` (100,000), ``…max.init.group.holder.capacity`` (10,000),
  ``…min.server.group.trim.size`` (5,000; <= 0 disables the server trim)
  (core/plan/maker/InstancePlanMakerImplV2.java:66-87).

GPU keys:

* ``…gpu.enabled`` (true): false keeps every query on the CPU plan maker;
* ``…gpu.devices`` ("all"): the devices this server drives — ``all``, a list ``0,2,5`` or a mask ``0x25``;
* ``…gpu.min.segment.docs`` (0): segments with fewer docs are not made HBM-resident (GpuIndexingOverride keeps
  the reference's readers), so a query touching one stays on the CPU;
* ``…gpu.min.query.docs`` (0): queries over fewer docs in total stay on the CPU (their launch would cost more
  than the scan);
* ``…gpu.exact.filter.stats`` (false): numEntriesScannedInFilter as the reference's iterators count it where
  they leap-frog (one more pass, PGPU_Q_EXACT_FILTER_STATS);
* ``…gpu.topk`` (true): select the ORDER BY trim on the GPU (pgpu_query_collect_topk);
* ``…gpu.sliced.columns`` / ``…gpu.value.planes.columns`` ("*"): the columns whose bit-sliced copy (filter columns)
  / value planes (metric columns) seal builds -- the GPU's IndexLoadingConfig (PhysicalColumnIndexContainer loads
  only the indexes a table names); a comma list, ``*`` = every column, empty = none;
* ``…gpu.derived.budget.bytes`` (-1 = half of the device's memory): HBM those copies may take per GPU.

INTEGRATION.md §3.3 shows the Java side reading the same keys from the server's PinotConfiguration.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

EXECUTOR_PREFIX = "pinot.server.query.executor."
GPU_PREFIX = EXECUTOR_PREFIX + "gpu."
DEFAULT_QUERY_EXECUTOR_TIMEOUT_MS = 15_000


def _bool(v: str) -> bool:
    s = str(v).strip().lower()
    if s in ("true", "1", "yes", "on"):
        return True
    if s in ("false", "0", "no", "off"):
        return False
    raise ValueError(f"not a boolean: {v!r}")


def parse_devices(spec: str, num_visible: int) -> List[int]:
    """``all`` | ``0,2,5`` | ``0x25`` → sorted device ordinals below ``num_visible``."""
    s = str(spec).strip().lower()
    if s in ("", "all", "*"):
        return list(range(num_visible))
    if s.startswith("0x"):
        mask = int(s, 16)
        ids = [i for i in range(mask.bit_length()) if (mask >> i) & 1]
    else:
        ids = sorted({int(x) for x in s.split(",") if x.strip()})
    bad = [i for i in ids if i < 0 or i >= num_visible]
    if bad:
        raise ValueError(f"{GPU_PREFIX}devices names device(s) {bad}, only {num_visible} visible")
    if not ids:
        raise ValueError(f"{GPU_PREFIX}devices selects no device")
    return ids


@dataclass
class GpuExecutorConfig:
    timeout_ms: int = DEFAULT_QUERY_EXECUTOR_TIMEOUT_MS
    num_groups_limit: int = 100_000
    max_init_group_holder_capacity: int = 10_000
    min_server_group_trim_size: int = 5000
    enabled: bool = True
    devices: str = "all"
    min_segment_docs: int = 0
    min_query_docs: int = 0
    exact_filter_stats: bool = False
    topk: bool = True
    sliced_columns: str = "*"
    value_planes_columns: str = "*"
    derived_budget_bytes: int = -1

    @classmethod
    def from_properties(cls, props: Mapping[str, str]) -> "GpuExecutorConfig":
        """Read the keys from a flat server configuration (PinotConfiguration / properties file)."""
        c = cls()

        def get(key: str, conv, attr: str):
            if key in props:
                try:
                    setattr(c, attr, conv(props[key]))
                except ValueError as e:
                    raise ValueError(f"bad value for {key}: {props[key]!r} ({e})") from None

        get(EXECUTOR_PREFIX + "timeout", int, "timeout_ms")
        get(EXECUTOR_PREFIX + "num.groups.limit", int, "num_groups_limit")
        get(EXECUTOR_PREFIX + "max.init.group.holder.capacity", int, "max_init_group_holder_capacity")
        get(EXECUTOR_PREFIX + "min.server.group.trim.size", int, "min_server_group_trim_size")
        get(GPU_PREFIX + "enabled", _bool, "enabled")
        get(GPU_PREFIX + "devices", str, "devices")
        get(GPU_PREFIX + "min.segment.docs", int, "min_segment_docs")
        get(GPU_PREFIX + "min.query.docs", int, "min_query_docs")
        get(GPU_PREFIX + "exact.filter.stats", _bool, "exact_filter_stats")
        get(GPU_PREFIX + "topk", _bool, "topk")
        get(GPU_PREFIX + "sliced.columns", str, "sliced_columns")
        get(GPU_PREFIX + "value.planes.columns", str, "value_planes_columns")
        get(GPU_PREFIX + "derived.budget.bytes", int, "derived_budget_bytes")
        unknown = [k for k in props if k.startswith(GPU_PREFIX) and k[len(GPU_PREFIX):] not in _GPU_KEYS]
        if unknown:
            raise ValueError(f"unknown GPU executor key(s): {unknown}")
        if c.num_groups_limit <= 0:
            raise ValueError(f"{EXECUTOR_PREFIX}num.groups.limit must be positive")
        return c

    @classmethod
    def from_file(cls, path: str) -> "GpuExecutorConfig":
        """A Java-style properties file (``key=value`` / ``key: value``, ``#`` / ``!`` comments)."""
        props = {}
        with open(path, encoding="utf-8") as f:
            for line in f:
                s = line.strip()
                if not s or s[0] in "#!":
                    continue
                sep = min((i for i in (s.find("="), s.find(":")) if i >= 0), default=-1)
                if sep < 0:
                    continue
                props[s[:sep].strip()] = s[sep + 1:].strip()
        return cls.from_properties(props)

    def derived_flags(self, columns: Sequence[str]) -> Dict[str, int]:
        """Column -> PGPU_DERIVE_* flags of the copies seal builds (GpuSegment(derived=...))."""
        from ._lib import PGPU_DERIVE_SLICED, PGPU_DERIVE_VALUE_PLANES

        def named(spec: str):
            s = spec.strip()
            return None if s == "*" else {c.strip() for c in s.split(",") if c.strip()}

        sl, vp = named(self.sliced_columns), named(self.value_planes_columns)
        return {c: (PGPU_DERIVE_SLICED if sl is None or c in sl else 0) |
                   (PGPU_DERIVE_VALUE_PLANES if vp is None or c in vp else 0) for c in columns}

    def apply_budget(self, ctx) -> None:
        """Set the context's derived-copy budget when the server names one."""
        if self.derived_budget_bytes >= 0:
            ctx.set_derived_budget(self.derived_budget_bytes)

    def open_context(self, device: int):
        """The GPU context of one device with this configuration's derived-copy budget applied (the server's one
        place of context creation; a budget set later governs later seals only)."""
        from .segment import GpuContext
        ctx = GpuContext(device)
        self.apply_budget(ctx)
        return ctx

    def upload(self, ctx, data, columns: Optional[Sequence[str]] = None):
        """A segment made HBM-resident under this configuration's residency policy: seal builds the bit-sliced
        copy and value planes only for the columns the table names (derived_flags)."""
        from .segment import GpuSegment
        names = list(columns) if columns is not None else list(data.columns)
        return GpuSegment(ctx, data, columns, derived=self.derived_flags(names))

    def plan_maker(self, ctx):
        """The GpuPlanMaker of a context with this configuration's query options."""
        from .plan import GpuPlanMaker
        return GpuPlanMaker(ctx, num_groups_limit=self.num_groups_limit,
                            max_init_group_holder_capacity=self.max_init_group_holder_capacity,
                            exact_filter_stats=self.exact_filter_stats, timeout_ms=self.timeout_ms,
                            gpu_topk=self.topk, min_server_group_trim_size=self.min_server_group_trim_size)

    def device_ids(self, num_visible: int) -> List[int]:
        return parse_devices(self.devices, num_visible)

    def resident(self, num_docs: int) -> bool:
        """Whether a segment of ``num_docs`` is uploaded to HBM (GpuIndexingOverride's decision)."""
        return self.enabled and num_docs >= self.min_segment_docs

    def offload(self, segment_docs: Sequence[int]) -> Tuple[bool, str]:
        """Whether a query over segments of these sizes runs on the GPU, and why not when it does not."""
        if not self.enabled:
            return False, f"{GPU_PREFIX}enabled=false"
        small = [i for i, n in enumerate(segment_docs) if not self.resident(n)]
        if small:
            return False, f"{len(small)} segment(s) below {GPU_PREFIX}min.segment.docs={self.min_segment_docs}"
        total = sum(segment_docs)
        if total < self.min_query_docs:
            return False, f"{total} docs below {GPU_PREFIX}min.query.docs={self.min_query_docs}"
        return True, ""

    def plan_maker(self, ctx, timeout_ms: Optional[int] = None):
        """A GpuPlanMaker with these settings (``timeout_ms``: the query's own budget, else the executor's)."""
        from .plan import GpuPlanMaker
        return GpuPlanMaker(ctx, num_groups_limit=self.num_groups_limit,
                            max_init_group_holder_capacity=self.max_init_group_holder_capacity,
                            exact_filter_stats=self.exact_filter_stats,
                            timeout_ms=self.timeout_ms if timeout_ms is None else timeout_ms,
                            gpu_topk=self.topk, min_server_group_trim_size=self.min_server_group_trim_size)


_GPU_KEYS = ("enabled", "devices", "min.segment.docs", "min.query.docs", "exact.filter.stats", "topk",
             "sliced.columns", "value.planes.columns", "derived.budget.bytes")
