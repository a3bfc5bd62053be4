"""Regenerate the committed golden fixtures from the reference's own test data (run here, where /root/reference
exists; the GPU box only reads the committed outputs).

Inputs (data files the reference's tests hold; nothing here executes reference code):
  pinot-core/src/test/resources/data/test_data-sv.avro        -> test_data_sv.npz  (the 11 columns that
      BaseSingleValueQueriesTest selects, qtest/BaseSingleValueQueriesTest.java:47-66,88-128)
  pinot-core/src/test/resources/data/padding{Null,Old,Percent}.tar.gz -> padding_segments.npz (real 5-doc segment
      dictionary and forward-index bytes written by the reference's segment creator)
  pinot-plugins/pinot-input-format/pinot-parquet/src/test/resources/baseballStats.snappy.parquet
      -> baseball.npz (playerID, yearID, teamID, playerName, runs; schema
      pinot-tools/src/main/resources/examples/batch/baseballStats/baseballStats_schema.json, nulls replaced by the
      FieldSpec defaults spi/data/FieldSpec.java:49-59: STRING dimension "null", INT metric 0)
  pinot-core/src/test/resources/data/simpleData200001.avro -> simple_data_200001.npz (dim0, dim1, met;
      QueryExecutorTest.java:150-185)
The known-answer values themselves are transcribed into kat.json with their file:line.
"""
from __future__ import annotations

import io
import os
import sys
import tarfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.avro import read_avro  # noqa: E402

SV_COLUMNS = {  # name -> (type, is metric)   BaseSingleValueQueriesTest.java:47-66,88-100
    "column1": ("INT", True), "column3": ("INT", True), "column5": ("STRING", False), "column6": ("INT", False),
    "column7": ("INT", False), "column9": ("INT", False), "column11": ("STRING", False),
    "column12": ("STRING", False), "column17": ("INT", True), "column18": ("INT", True),
    "daysSinceEpoch": ("INT", False),
}


def _default(t: str, metric: bool):
    if t == "STRING":
        return "null"
    return 0 if metric else -(2 ** 31)


def make_sv():
    rows = read_avro(os.path.join(REF, "pinot-core/src/test/resources/data/test_data-sv.avro"))
    out = {}
    for c, (t, metric) in SV_COLUMNS.items():
        vals = [r.get(c) for r in rows]
        vals = [_default(t, metric) if v is None else v for v in vals]
        out[c] = np.array(vals, dtype=object if t == "STRING" else np.int32)
        if t == "STRING":
            out[c] = np.array(vals, dtype=np.str_)
    np.savez_compressed(os.path.join(HERE, "test_data_sv.npz"), **out)
    print("test_data_sv.npz", len(rows), "rows")


def make_padding():
    out = {}
    for name in ("paddingNull", "paddingOld", "paddingPercent"):
        with tarfile.open(os.path.join(REF, f"pinot-core/src/test/resources/data/{name}.tar.gz")) as tf:
            for m in tf.getmembers():
                base = os.path.basename(m.name)
                if base.endswith((".dict", ".fwd", "metadata.properties")):
                    data = tf.extractfile(m).read()
                    out[f"{name}/{base}"] = np.frombuffer(data, dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "padding_segments.npz"), **out)
    print("padding_segments.npz", sorted(out))


def make_baseball():
    import pyarrow.parquet as pq
    t = pq.read_table(os.path.join(
        REF, "pinot-plugins/pinot-input-format/pinot-parquet/src/test/resources/baseballStats.snappy.parquet"))
    cols = {}
    for c in ("playerID", "teamID", "playerName"):
        cols[c] = np.array(["null" if v is None else v for v in t.column(c).to_pylist()], dtype=np.str_)
    cols["yearID"] = np.array([int(v) for v in t.column("yearID").to_pylist()], dtype=np.int32)
    cols["runs"] = np.array([0 if v is None else int(v) for v in t.column("runs").to_pylist()], dtype=np.int32)
    np.savez_compressed(os.path.join(HERE, "baseball.npz"), **cols)
    print("baseball.npz", t.num_rows, "rows")


def make_simple():
    """QueryExecutorTest.java:150-185: simpleData200001.avro (dim0, dim1, met INT columns)."""
    rows = read_avro(os.path.join(REF, "pinot-core/src/test/resources/data/simpleData200001.avro"))
    out = {c: np.array([r[c] for r in rows], dtype=np.int32) for c in ("dim0", "dim1", "met")}
    np.savez_compressed(os.path.join(HERE, "simple_data_200001.npz"), **out)
    print("simple_data_200001.npz", len(rows), "rows")


if __name__ == "__main__":
    make_simple()
    make_sv()
    make_padding()
    make_baseball()
