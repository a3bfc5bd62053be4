"""Segment loader (pinot_amd.loader): real v1 segment files from the reference's test resources, v1 / v3 round
trips through the oracle's directory writer, corruption and unsupported-shape errors, and (GPU) queries over
loaded segments against the oracle.

KATs: LoaderTest.testPadding (pinot-segment-local/src/test/java/.../segment/index/loader/LoaderTest.java:218-283)
over pinot-core/src/test/resources/data/padding{Old,Percent,Null}.tar.gz, committed as
tests/golden/padding_segments.npz (tests/golden/make_golden.py)."""
import io
import os
import struct
import tarfile

import numpy as np
import pytest

from oracle import engine
from oracle.segment_writer import unpack_fixed_bit, write_segment_dir
from pinot_amd._lib import PGPU_INT, PGPU_LONG, PGPU_STRING
from pinot_amd.loader import (MAGIC_MARKER, SegmentFormatError, UnsupportedSegmentError, load_segment,
                              read_index_map, read_properties)
from pinot_amd.predicate import SortedDictionary
from pinot_amd.query import parse_sql
from tests.helpers import GOLDEN, baseball_segment, fast_count_segment, rows_close, sv_segment

PAD = np.load(os.path.join(GOLDEN, "padding_segments.npz"))


def _padding_dir(tmp_path, name):
    d = tmp_path / name
    d.mkdir()
    for k in PAD.files:
        seg, fname = k.split("/")
        if seg == name:
            (d / fname).write_bytes(PAD[k].tobytes())
    return str(d)


def _string_dict(col):
    return SortedDictionary(col.dictionary_values(), col.data_type, pad_char=col.pad_char,
                            entry_width=col.entry_width)


# ---- LoaderTest.testPadding KATs ---------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["paddingOld", "paddingPercent"])
def test_legacy_padding_kat(tmp_path, name):
    seg = load_segment(_padding_dir(tmp_path, name))
    col = seg.column("name")
    assert col.pad_char == "%"  # LEGACY_STRING_PAD_CHAR (absent key in paddingOld, '%' in paddingPercent)
    assert col.dictionary_values() == ["lynda 2.0", "lynda"]
    d = _string_dict(col)
    assert d.index_of("lynda%") == 1
    assert d.index_of("lynda%%") == 1
    assert d.index_of("lynda") == 1  # padded to "lynda%%%%"


def test_null_padding_kat(tmp_path):
    seg = load_segment(_padding_dir(tmp_path, "paddingNull"))
    col = seg.column("name")
    assert col.pad_char == "\0"
    assert col.dictionary_values() == ["lynda", "lynda 2.0"]
    d = _string_dict(col)
    assert d.insertion_index_of("lynda\0") == -2
    assert d.insertion_index_of("lynda\0\0") == -2


@pytest.mark.parametrize("name", ["paddingNull", "paddingOld", "paddingPercent"])
def test_padding_segment_columns(tmp_path, name):
    seg = load_segment(_padding_dir(tmp_path, name))
    assert seg.num_docs == 5
    assert set(seg.columns) == {"age", "name", "percent", "outgoingName1"}
    age = seg.column("age")
    assert age.data_type == PGPU_INT and age.cardinality == 5 and age.bits_per_value == 3
    ids = unpack_fixed_bit(age.forward, 3, 5)
    assert sorted(ids.tolist()) == list(range(5))
    assert seg.column("outgoingName1").data_type == PGPU_LONG
    assert seg.column("outgoingName1").dictionary_values().tolist() == [246, 310, 336, 467, 902]


def test_tar_gz_matches_directory(tmp_path):
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for k in PAD.files:
            if k.startswith("paddingNull/"):
                data = PAD[k].tobytes()
                ti = tarfile.TarInfo(k)
                ti.size = len(data)
                tf.addfile(ti, io.BytesIO(data))
    p = tmp_path / "paddingNull.tar.gz"
    p.write_bytes(buf.getvalue())
    a = load_segment(str(p))
    b = load_segment(_padding_dir(tmp_path, "paddingNull"))
    for c in b.columns:
        assert a.column(c).dictionary == b.column(c).dictionary
        assert a.column(c).forward == b.column(c).forward


# ---- round trips through the writer --------------------------------------------------------------------------------
def _same(a, b):
    assert a.num_docs == b.num_docs and set(a.columns) == set(b.columns)
    for n, c in b.columns.items():
        x = a.column(n)
        assert (x.data_type, x.cardinality) == (c.data_type, c.cardinality), n
        if c.data_type == PGPU_STRING:
            assert list(x.dictionary) == list(c.dictionary), n
        else:
            assert bytes(x.dictionary) == bytes(c.dictionary), n
        assert (x.sorted_index is None) == (c.sorted_index is None), n
        if c.sorted_index is not None:
            assert bytes(x.sorted_index) == bytes(c.sorted_index), n
        else:
            assert bytes(x.forward) == bytes(c.forward), n
        assert (None if c.inverted is None else bytes(c.inverted)) == x.inverted, n


@pytest.mark.parametrize("version", ["v1", "v3"])
@pytest.mark.parametrize("make", [sv_segment, fast_count_segment, baseball_segment], ids=lambda f: f.__name__)
def test_round_trip(tmp_path, version, make):
    seg = make()
    write_segment_dir(seg, str(tmp_path / seg.name), version=version)
    _same(load_segment(str(tmp_path / seg.name)), seg)


def test_loaded_segment_queries_match_oracle(tmp_path):
    """The loaded bytes answer the quickstart query exactly as the in-memory segment does (CPU oracle)."""
    seg = baseball_segment()
    write_segment_dir(seg, str(tmp_path / "bb"), version="v3")
    loaded = load_segment(str(tmp_path / "bb"), columns=["playerName", "yearID", "runs"])
    q = parse_sql("SELECT playerName, SUM(runs) FROM baseballStats WHERE yearID > 2000 GROUP BY playerName "
                  "ORDER BY SUM(runs) DESC LIMIT 10")
    assert rows_close([list(r) for r in engine.execute(q, [loaded]).rows],
                      [list(r) for r in engine.execute(q, [seg]).rows])


# ---- formats and errors ------------------------------------------------------------------------------------------
def test_index_map_dotted_column_names():
    m = read_index_map("my.col.dictionary.startOffset = 0\nmy.col.dictionary.size = 20\n"
                       "x.forward_index.startOffset = 20\nx.forward_index.size = 9\n")
    assert m == {("my.col", "dictionary"): (0, 20), ("x", "forward_index"): (20, 9)}
    with pytest.raises(SegmentFormatError):
        read_index_map("x.dictionary.endOffset = 3\n")
    with pytest.raises(SegmentFormatError):
        read_index_map("x.dictionary.startOffset = 3\n")  # size missing


def test_properties_escapes():
    p = read_properties("# c\na = 1\nb: x\\,y\nsegment.padding.character = \\\\u0000\nk=v \\\n  w\n")
    assert p == {"a": "1", "b": "x,y", "segment.padding.character": "\\u0000", "k": "v w"}


def test_corrupt_magic_marker(tmp_path):
    seg = fast_count_segment()
    root = write_segment_dir(seg, str(tmp_path / "s"), version="v3")
    psf = os.path.join(root, "columns.psf")
    data = bytearray(open(psf, "rb").read())
    assert struct.unpack(">Q", bytes(data[:8]))[0] == MAGIC_MARKER
    data[0] ^= 0xFF
    open(psf, "wb").write(bytes(data))
    with pytest.raises(SegmentFormatError, match="magic marker"):
        load_segment(str(tmp_path / "s"))


def test_unsupported_columns(tmp_path):
    seg = fast_count_segment()
    root = write_segment_dir(seg, str(tmp_path / "s"), version="v1")
    meta = os.path.join(root, "metadata.properties")
    text = open(meta).read()
    open(meta, "w").write(text.replace("column.class.hasDictionary = true", "column.class.hasDictionary = false"))
    # a raw column is served now (tests/test_raw_columns.py); one whose .sv.raw.fwd file is missing is malformed
    with pytest.raises(SegmentFormatError, match="raw forward index"):
        load_segment(str(tmp_path / "s"))
    assert set(load_segment(str(tmp_path / "s"), columns=["sorted"]).columns) == {"sorted"}
    open(meta, "w").write(text.replace("column.class.dataType = INT", "column.class.dataType = BYTES"))
    with pytest.raises(UnsupportedSegmentError, match="BYTES"):
        load_segment(str(tmp_path / "s"))


def test_truncated_forward_index(tmp_path):
    seg = sv_segment()
    root = write_segment_dir(seg, str(tmp_path / "s"), version="v1")
    col = next(c for c in seg.columns.values() if c.forward is not None)
    p = os.path.join(root, col.name + ".sv.unsorted.fwd")
    open(p, "wb").write(open(p, "rb").read()[:-64])
    with pytest.raises(SegmentFormatError, match="forward index"):
        load_segment(str(tmp_path / "s"))


# ---- GPU: loaded segments through the HIP path ---------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("version", ["v1", "v3"])
def test_loaded_segments_gpu_vs_oracle(gpu_ctx, tmp_path, version):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    segs = [baseball_segment(), fast_count_segment()]
    queries = [("SELECT playerName, SUM(runs) FROM baseballStats WHERE yearID > 2000 GROUP BY playerName "
                "ORDER BY SUM(runs) DESC LIMIT 10"),
               "SELECT COUNT(*), SUM(intRangeCol) FROM t WHERE class IN (1, 3) AND sorted BETWEEN 100 AND 700"]
    for seg, sql in zip(segs, queries):
        write_segment_dir(seg, str(tmp_path / seg.name), version=version)
        loaded = load_segment(str(tmp_path / seg.name))
        g = GpuSegment(gpu_ctx, loaded)
        try:
            q = parse_sql(sql)
            res = GpuPlanMaker(gpu_ctx).execute(q, [g])
            ref = engine.execute(q, [seg])
            assert rows_close([list(r) for r in res.rows], [list(r) for r in ref.rows])
            assert res.stats.num_docs_scanned == ref.num_docs_scanned
        finally:
            g.release()


# ---- queries over the real 5-doc padding segments (string predicates under both padding conventions) ------------
PAD_QUERIES = ["SELECT COUNT(*), MAX(age), MIN(percent) FROM t WHERE name = 'lynda'",
               "SELECT COUNT(*), SUM(age) FROM t WHERE name = 'lynda%'",
               "SELECT COUNT(*), SUM(age) FROM t WHERE name IN ('lynda 2.0', 'lynda%%')",
               "SELECT COUNT(*), SUM(outgoingName1) FROM t WHERE name > 'lynda'",
               "SELECT name, COUNT(*), SUM(age) FROM t GROUP BY name ORDER BY name LIMIT 10"]


@pytest.mark.parametrize("name", ["paddingNull", "paddingOld"])
@pytest.mark.parametrize("sql", PAD_QUERIES)
def test_padding_segment_queries_oracle(tmp_path, name, sql):
    """The oracle's string predicates follow the segment's padding (padded compare for the legacy '%')."""
    seg = load_segment(_padding_dir(tmp_path, name))
    r = engine.execute(parse_sql(sql), [seg])
    if sql == PAD_QUERIES[1]:
        # LoaderTest: indexOf("lynda%") == 1 with '%' padding; with '\0' padding "lynda%" is not in the dictionary
        assert r.num_docs_scanned == (0 if name == "paddingNull" else r.num_docs_scanned)
        if name == "paddingOld":
            assert r.num_docs_scanned == engine.execute(parse_sql(PAD_QUERIES[0]), [seg]).num_docs_scanned > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["paddingNull", "paddingOld", "paddingPercent"])
def test_padding_segment_queries_gpu(gpu_ctx, tmp_path, name):
    from pinot_amd.plan import GpuPlanMaker
    from pinot_amd.segment import GpuSegment
    seg = load_segment(_padding_dir(tmp_path, name))
    g = GpuSegment(gpu_ctx, seg)
    try:
        for sql in PAD_QUERIES:
            q = parse_sql(sql)
            res = GpuPlanMaker(gpu_ctx).execute(q, [g])
            ref = engine.execute(q, [seg])
            assert rows_close([list(r) for r in res.rows], [list(r) for r in ref.rows]), sql
            assert res.stats.num_docs_scanned == ref.num_docs_scanned, sql
    finally:
        g.release()
