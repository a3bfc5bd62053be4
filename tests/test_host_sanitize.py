"""ASan / UBSan over libpinotgpu's host-side parsers of untrusted segment bytes (CPU only).

tests/sanitize/host_fuzz.cpp drives pgpu_decode_raw_forward (pgpu_rawfwd.cpp: raw forward-index chunks, snappy and
LZ4 block decoders), pgpu_parse_roaring (pgpu_roaring.cpp: inverted-index bitmaps) and reference_entries_scanned
(pgpu_iterstats.cpp: filter programs) over valid inputs -- the reference's own raw forward-index files and
oracle-written bitmaps / files -- and over every truncation and hundreds of byte-overwritten variants of each.  The
harness is built with -fsanitize=address,undefined and -fno-sanitize-recover: any out-of-bounds access, overflow
or crash fails the test; every corrupt input must come back as a status.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import rawfwd
from oracle.segment_writer import roaring_serialize
from pinot_amd._lib import PGPU_DOUBLE, PGPU_INT, PGPU_LONG

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "pinot_amd", "csrc")
SOURCES = [os.path.join(ROOT, "tests", "sanitize", "host_fuzz.cpp")] + \
          [os.path.join(CSRC, f) for f in ("pgpu_rawfwd.cpp", "pgpu_roaring.cpp", "pgpu_iterstats.cpp")]
GOLDEN = os.path.join(ROOT, "tests", "golden")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


@pytest.fixture(scope="module")
def fuzz(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("sanitize") / "host_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer"] + SOURCES + ["-o", out, "-ldl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr[-4000:])
    return out


def _run(fuzz, kind, data: bytes, tmp_path, name, variants=400):
    p = tmp_path / name
    p.write_bytes(data)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([fuzz, kind, str(p), str(variants)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (kind, name, r.stdout[-2000:], r.stderr[-6000:])
    return r.stdout


REFERENCE_FILES = [("fixedByteSVRDoubles.v1", 10009), ("fixedByteCompressed.v2", 2000), ("fixedByteRaw.v2", 2000)]


@pytest.mark.parametrize("name,n", REFERENCE_FILES)
def test_raw_forward_reference_files(fuzz, tmp_path, name, n):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        data = f.read()
    out = _run(fuzz, f"raw:8:{n}", data, tmp_path, name)
    assert "rejected" in out


@pytest.mark.parametrize("codec,version", [(rawfwd.PASS_THROUGH, 2), (rawfwd.SNAPPY, 3), (rawfwd.LZ4, 3),
                                           (rawfwd.LZ4_LENGTH_PREFIXED, 4), (rawfwd.ZSTANDARD, 2)])
@pytest.mark.parametrize("dt,width", [(PGPU_INT, 4), (PGPU_LONG, 8)])
def test_raw_forward_codecs(fuzz, tmp_path, codec, version, dt, width):
    rng = np.random.default_rng(codec * 10 + version)
    n = 3001
    vals = (rng.integers(0, 50, n) * 1000).astype(np.int32 if width == 4 else np.int64)  # compressible
    data = rawfwd.write_raw_forward(vals, dt, codec, version)
    _run(fuzz, f"raw:{width}:{n}", data, tmp_path, f"c{codec}v{version}w{width}")


@pytest.mark.parametrize("kind", ["array", "bitmap", "run", "mixed"])
def test_roaring_bitmaps(fuzz, tmp_path, kind):
    rng = np.random.default_rng(len(kind))
    if kind == "array":
        docs = np.sort(rng.choice(200_000, 3000, replace=False))
    elif kind == "bitmap":
        docs = np.flatnonzero(rng.random(140_000) < 0.3)
    elif kind == "run":
        docs = np.concatenate([np.arange(s, s + 300) for s in range(0, 250_000, 1000)])
    else:
        docs = np.concatenate([np.sort(rng.choice(65536, 100, replace=False)),
                               65536 + np.flatnonzero(rng.random(65536) < 0.5), np.arange(140_000, 150_000)])
    data = roaring_serialize(np.asarray(docs, dtype=np.int64), allow_runs=kind in ("run", "mixed"))
    _run(fuzz, "roaring", data, tmp_path, kind, variants=800)


def _program(nodes, num_docs=3000) -> bytes:
    a = [len(nodes), num_docs]
    for op, neg in nodes:
        a += [op, neg]
    return np.asarray(a, dtype=np.int32).tobytes()


def test_filter_programs(fuzz, tmp_path):
    from pinot_amd import _lib as L
    S, I, AB, AC, AE, OB, OC, OE, NOT = (L.PGPU_F_SCAN, L.PGPU_F_INVERTED, L.PGPU_F_AND_BEGIN,
                                         L.PGPU_F_AND_CHILD_END, L.PGPU_F_AND_END, L.PGPU_F_OR_BEGIN,
                                         L.PGPU_F_OR_CHILD_END, L.PGPU_F_OR_END, L.PGPU_F_NOT)
    progs = {
        "and": [(AB, 0), (S, 0), (AC, 0), (I, 1), (AC, 0), (S, 0), (AC, 0), (AE, 0)],
        "nested": [(OB, 0), (AB, 0), (S, 0), (AC, 0), (NOT, 0), (S, 1), (AC, 0), (AE, 0), (OC, 0), (I, 0), (OC, 0),
                   (OE, 0)],
    }
    for name, nodes in progs.items():
        _run(fuzz, "program", _program(nodes), tmp_path, name, variants=1500)
    # 63 nested NOTs around one leaf (the recursion is bounded at 256 levels: deeper programs are rejected)
    _run(fuzz, "program", _program([(NOT, 0)] * 63 + [(S, 0)]), tmp_path, "deep", variants=50)
