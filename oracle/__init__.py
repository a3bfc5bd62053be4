"""CPU oracle for the MI355X segment query path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may import, call, link or
run anything under ``oracle/``, and only as the checker.  The product path (``pinot_amd/`` + libpinotgpu.so) never
touches it and fails loudly when the HIP extension is missing.

Contents (each function cites the reference file:line it restates; abbreviations as in SURVEY.md):
  segment_writer.py  reference on-disk formats: dictionary creation, fixed-bit forward index, sorted index,
                     Roaring portable bitmaps, bitmap inverted index file
  engine.py          per-segment query execution (predicates, filter operators with the iterator model and its
                     numEntriesScannedInFilter accounting, SUM/COUNT/MIN/MAX/AVG, dictionary group-by with
                     numGroupsLimit first-seen semantics) and the combine / broker reduce
  avro.py            Avro object-container (null codec) reader for the reference's test_data-sv.avro fixture
  pinot_cpu.c        C restatement of the block-at-a-time CPU operators, timed as bench.py's cpu_baseline

Parity status: pinned.  The restatement reproduces the reference's own known-answer tests (tests/golden/ and
tests/test_oracle_kat.py): InnerSegment/InterSegment aggregation and group-by KATs on test_data-sv.avro, the
literal doc-id vectors of the And/Or/Not filter operator tests, FastFilteredCountTest's counts and the real
5-doc padding segments' dictionary / forward-index bytes.  Roaring serialized bytes are pinned only through
round trips and the resulting doc-id sets (the reference's tests check cardinalities, not bytes).
"""
