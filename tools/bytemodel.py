"""Algorithmic bytes of a bench workload, computed from the workload itself -- the segments' dict ids
and the reference's physical filter tree -- and not from what any kernel strategy happens to read.

Measurement code only (bench.py and its tests); the product never imports it.

Per segment (every figure exact, no sampling):
  * filter: the operator tree FilterPlanNode / FilterOperatorUtils build (pinot_amd.plan.SegmentFilterPlanner, AND
    children in the reference's priority order).  A SCAN leaf with no preceding candidate set streams its forward
    index whole, ceil(N*b/8) bytes; a SCAN leaf under the docs that pass the preceding AND children (the
    SVScanDocIdIterator.applyAnd / AndDocIdIterator leap-frog of AndDocIdSet.java:87-140) reads the 32-B sectors of
    its forward index holding at least one such doc; an inverted leaf reads the serialized bitmaps of its matching
    (or, exclusive, non-matching) dict ids; a sorted leaf reads its (start, end) pairs.  OR / NOT children inherit
    their parent's candidate set.
  * aggregation and group-by columns: the whole forward index when every doc matches, else the 32-B sectors holding
    a matched doc;
  * dictionaries: per aggregated column, min(card * width, 32 B * matched docs) once per segment;
  * output: one 8-B cell per (group, section).

The dict ids are regenerated on the GPU with torch from synth.py's counter-based hash (the same function
synth.hip evaluates and synth.dict_ids_cpu restates), so the model needs no copy of the HBM segments.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

SECTOR = 32

_C1 = np.uint64(0x9E3779B97F4A7C15).astype(np.int64).item()
_C2 = np.uint64(0xBF58476D1CE4E5B9).astype(np.int64).item()
_C3 = np.uint64(0x94D049BB133111EB).astype(np.int64).item()
_CD = np.uint64(0xD1B54A32D192ED03).astype(np.int64).item()


def _to_i64(x: int) -> int:
    return np.uint64(x & ((1 << 64) - 1)).astype(np.int64).item()


def _lsr(x, s: int):
    """Logical right shift of an int64 tensor (torch's >> is arithmetic)."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def _splitmix(x):
    x = x + _C1
    x = (x ^ _lsr(x, 30)) * _C2
    x = (x ^ _lsr(x, 27)) * _C3
    return x ^ _lsr(x, 31)


def dict_ids_torch(seed: int, num_docs: int, card: int, device, cdf: Optional[np.ndarray] = None, doc0: int = 0):
    """torch twin of synth.dict_ids_cpu: int64 dict ids of docs [doc0, doc0 + num_docs)."""
    import torch

    docs = torch.arange(doc0, doc0 + num_docs, dtype=torch.int64, device=device)
    u = _lsr(_splitmix(_to_i64(seed) ^ (docs * _CD)), 32)
    del docs
    if cdf is None:
        return _lsr(u * card, 32)
    t = torch.as_tensor(cdf.astype(np.int64), device=device)
    return torch.searchsorted(t, u, right=True)


def sector_bytes(match, bits: int) -> int:
    """Bytes of the 32-B sectors of a b-bit MSB-first forward index that hold at least one doc of `match`."""
    import torch

    docs = torch.nonzero(match, as_tuple=True)[0]
    if docs.numel() == 0:
        return 0
    first = (docs * bits) >> 8                    # 256 bits per sector
    last = (docs * bits + bits - 1) >> 8          # a value may straddle two sectors
    n = int(((match.numel() * bits + 255) >> 8) + 1)
    hit = torch.zeros(n, dtype=torch.bool, device=match.device)
    hit[first] = True
    hit[last] = True
    return SECTOR * int(hit.sum().item())


class _SegmentModel:
    """One synthetic segment: lazily generated dict ids per column, the byte counters."""

    def __init__(self, w, seg_id: int, gs, num_docs: int, device):
        from pinot_amd.segment import num_bits_per_value
        from pinot_amd.synth import column_seed, zipf_cdf

        self.w, self.gs, self.n, self.device = w, gs, num_docs, device
        self._cols = {c.name: c for c in w.columns}
        self._ids: Dict[str, object] = {}
        self._seed = lambda c: column_seed(w.seed, seg_id, c)
        self._cdf = lambda c: zipf_cdf(c.cardinality, c.zipf_s) if c.dist == "zipf" else None
        self.bits = lambda c: num_bits_per_value(self._cols[c].cardinality - 1)
        self.fwd_bytes = lambda c: (num_docs * self.bits(c) + 7) // 8
        self.parts: Dict[str, int] = {"forward_full": 0, "forward_sectors": 0, "inverted_bitmaps": 0,
                                      "sorted_pairs": 0}

    def ids(self, col: str):
        if col not in self._ids:
            c = self._cols[col]
            self._ids[col] = dict_ids_torch(self._seed(col), self.n, c.cardinality, self.device, self._cdf(c))
        return self._ids[col]

    def leaf_match(self, ev, col: str):
        import torch

        ids = self.ids(col)
        if ev.kind == "RANGE":
            m = (ids >= ev.start) & (ids < ev.end)
        else:
            m = torch.isin(ids, torch.as_tensor(list(ev.ids), dtype=torch.int64, device=self.device))
            if ev.is_exclusive:
                m = ~m
        return m

    def read_column(self, col: str, cand) -> None:
        """A column read under candidate set `cand` (None: every doc, the whole forward index)."""
        if cand is None:
            self.parts["forward_full"] += self.fwd_bytes(col)
        else:
            self.parts["forward_sectors"] += sector_bytes(cand, self.bits(col))

    def eval(self, op, cand):
        """Docs the operator matches (within `cand` when given); counts the bytes it reads."""
        import torch

        k = op.kind
        if k == "ALL":
            return torch.ones(self.n, dtype=torch.bool, device=self.device) if cand is None else cand.clone()
        if k == "EMPTY":
            return torch.zeros(self.n, dtype=torch.bool, device=self.device)
        if k == "SCAN":
            self.read_column(op.column, cand)
            m = self.leaf_match(op.evaluator, op.column)
        elif k == "INV":
            ev = op.evaluator
            ids = ev.non_matching_dict_ids() if ev.is_exclusive else ev.matching_dict_ids()
            col = self.gs.column(op.column)
            offs = np.frombuffer(col.inverted, dtype=">i4", count=col.cardinality + 1).astype(np.int64)
            self.parts["inverted_bitmaps"] += int(sum(offs[i + 1] - offs[i] for i in ids))
            m = self.leaf_match(ev, op.column)
        elif k == "SORTED":
            self.parts["sorted_pairs"] += 8 * len(op.doc_ranges)
            m = torch.zeros(self.n, dtype=torch.bool, device=self.device)
            for a, b in op.doc_ranges:
                m[a:b + 1] = True
        elif k == "AND":
            m = cand
            for ch in op.children:  # each child sees the docs every preceding child passed
                m = self.eval(ch, m)
            return m
        elif k == "OR":
            m = torch.zeros(self.n, dtype=torch.bool, device=self.device)
            for ch in op.children:
                m |= self.eval(ch, cand)
        elif k == "NOT":
            m = ~self.eval(op.children[0], cand)
        else:
            raise NotImplementedError(f"byte model: filter operator {k}")
        return m if cand is None else (m & cand)


def workload_bytes(w, q, segs, num_docs: int, seg_ids: List[int], device,
                   ngroups: int = 1) -> Tuple[int, Dict[str, int], int]:
    """(algorithmic bytes per query, breakdown, matched docs) of workload `w`'s query `q` over the GPU segments
    `segs` (global segment ids `seg_ids`) with `ngroups` result groups, per the module docstring."""
    import torch

    from pinot_amd.plan import SegmentFilterPlanner

    parts = {"forward_full": 0, "forward_sectors": 0, "inverted_bitmaps": 0, "sorted_pairs": 0,
             "dictionaries": 0, "output": 0}
    matched_total = 0
    agg_cols = sorted(set(a.column for a in q.aggregations if a.column))
    read_cols = sorted(set(agg_cols) | set(q.group_by or []))
    for gs, sid in zip(segs, seg_ids):
        sm = _SegmentModel(w, sid, gs, num_docs, device)
        op = SegmentFilterPlanner(gs).build(q.filter)
        match = None if op.kind == "ALL" else sm.eval(op, None)
        matched = num_docs if match is None else int(match.sum().item())
        matched_total += matched
        for c in read_cols:
            sm.read_column(c, match)
        for c in agg_cols:
            width = {0: 4, 1: 8, 2: 4, 3: 8}.get(gs.column(c).data_type, 4)
            parts["dictionaries"] += min(gs.column(c).cardinality * width, SECTOR * matched)
        for k, v in sm.parts.items():
            parts[k] += v
        del sm, match
    parts["output"] = output_bytes(ngroups, len(q.aggregations))
    if device is not None and str(device).startswith("cuda"):
        torch.cuda.empty_cache()
    return sum(parts.values()), parts, matched_total


def output_bytes(ngroups: int, naggs: int) -> int:
    return 8 * max(1, ngroups) * (1 + naggs)
