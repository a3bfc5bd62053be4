// Host-side parsers of the segment bytes handed to libpinotgpu (no HIP: they also build into the sanitizer harness,
// tests/sanitize/host_fuzz.cpp).  Every one treats its input as untrusted: a malformed file returns a status and a
// message, never reads or writes outside its buffers, and never allocates more than its output can hold.
#ifndef PGPU_HOST_H
#define PGPU_HOST_H

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/pinot_gpu.h"

// pgpu_rawfwd.cpp: FixedByteChunkSVForwardIndexWriter file -> num_docs little-endian values of `width` bytes.
int pgpu_decode_raw_forward(const uint8_t* b, uint64_t n, int32_t width, int32_t num_docs, std::vector<uint8_t>* out,
                            std::string* err);

// pgpu_roaring.cpp: one RoaringBitmap portable serialization (ImmutableRoaringBitmap) split into containers.
// type: 0 array (card uint16 values), 1 bitmap (1024 uint64 words), 2 run (card = runs, (start, length - 1) pairs);
// payload points into the input.  Rejects what a reader could not index safely: keys not ascending, array values
// not ascending, runs not ascending or overlapping or past 65,535, payloads past the end.
struct PgpuRoaringContainer {
  uint32_t key, type, card;
  const uint8_t* payload;
  size_t payload_bytes;
};
int pgpu_parse_roaring(const uint8_t* p, size_t n, std::vector<PgpuRoaringContainer>* out, std::string* err);

// pgpu_iterstats.cpp: numEntriesScannedInFilter of one segment's program replayed over leaf match bitmaps (-1 on a
// malformed program).
int64_t reference_entries_scanned(const pgpu_filter_node* nodes, int num_nodes, const uint32_t* const* leaf_words,
                                  int num_leaves, int32_t num_docs, const int32_t* const* leaf_offsets = nullptr);
bool pgpu_filter_count_is_reference(const pgpu_filter_node* nodes, int num_nodes);

#endif  // PGPU_HOST_H
