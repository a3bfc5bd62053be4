"""Debug: the inner-segment KAT filter on the GPU under each kernel path, leaf by leaf (GPU box only)."""
import os
import sys

sys.path.insert(0, os.getcwd())
from oracle import engine  # noqa: E402
from pinot_amd.plan import GpuPlanMaker  # noqa: E402
from pinot_amd.query import parse_sql  # noqa: E402
from pinot_amd.segment import GpuContext, GpuSegment  # noqa: E402
from tests.helpers import load_kat, sv_segment  # noqa: E402

KAT = load_kat()
ctx = GpuContext(0)
seg = sv_segment()
g = GpuSegment(ctx, seg)
base = "SELECT COUNT(*) FROM testTable WHERE "
for f in ["column5 = 'gFuH'", "column1 > 100000000", "column1 > 100000000 AND column5 = 'gFuH'",
          KAT["filter"].replace(" WHERE ", "")]:
    q = parse_sql(base + f)
    ref = engine.execute(q, [seg])
    for hp in (False, True):
        r = GpuPlanMaker(ctx, host_planning=hp).execute(q, [g])
        print(f"{f[:60]:60s} host={hp} gpu={r.aggregation_result[0]} oracle={ref.aggregation_result[0]}", flush=True)
