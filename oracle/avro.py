"""Minimal Avro object-container reader (null codec; int/long/string/null unions) — test infrastructure.

Used only by tests/golden/make_golden.py to turn the reference's test fixture
pinot-core/src/test/resources/data/test_data-sv.avro into committed column arrays.  Follows the Avro 1.x
specification: magic 'Obj\\x01', metadata map, 16-byte sync marker, blocks of (count, size, records, sync);
ints/longs are zig-zag varints.
"""
from __future__ import annotations

import json
from typing import Dict, List


def _varint(b: bytes, p: int):
    shift = 0
    n = 0
    while True:
        c = b[p]
        p += 1
        n |= (c & 0x7F) << shift
        shift += 7
        if c < 0x80:
            break
    return (n >> 1) ^ -(n & 1), p


def read_avro(path: str) -> List[Dict]:
    data = open(path, "rb").read()
    if data[:4] != b"Obj\x01":
        raise ValueError("not an Avro object container file")
    p = 4
    meta = {}
    while True:
        count, p = _varint(data, p)
        if count == 0:
            break
        if count < 0:
            count = -count
            _, p = _varint(data, p)
        for _ in range(count):
            kl, p = _varint(data, p)
            k = data[p:p + kl].decode()
            p += kl
            vl, p = _varint(data, p)
            meta[k] = data[p:p + vl]
            p += vl
    sync = data[p:p + 16]
    p += 16
    if meta.get("avro.codec", b"null") not in (b"null", b""):
        raise ValueError("only the null codec is supported")
    schema = json.loads(meta["avro.schema"])
    fields = schema["fields"]
    rows: List[Dict] = []
    while p < len(data):
        n, p = _varint(data, p)
        size, p = _varint(data, p)
        end = p + size
        for _ in range(n):
            r = {}
            for f in fields:
                t = f["type"]
                if isinstance(t, list):
                    idx, p = _varint(data, p)
                    t = t[idx]
                if isinstance(t, dict):
                    t = t.get("type")
                if t == "null":
                    r[f["name"]] = None
                elif t in ("int", "long"):
                    r[f["name"]], p = _varint(data, p)
                elif t == "string":
                    ln, p = _varint(data, p)
                    r[f["name"]] = data[p:p + ln].decode("utf-8")
                    p += ln
                else:
                    raise ValueError(f"unsupported Avro type {t}")
            rows.append(r)
        if p != end:
            raise ValueError("Avro block size mismatch")
        if data[p:p + 16] != sync:
            raise ValueError("Avro sync marker mismatch")
        p += 16
    return rows
