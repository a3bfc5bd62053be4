// RoaringBitmap portable serialization, parsed once at segment upload (pgpu_segment_add_inverted_index).
// RoaringBitmap 0.9.26 is a third-party dependency of the reference (pom.xml; not vendored): this restates its
// published format as the reference's BitmapInvertedIndexReader.getDocIds reads it
// (seglocal/segment/index/readers/BitmapInvertedIndexReader.java:45-61 -> ImmutableRoaringBitmap):
//   cookie 12346: int32 cookie, int32 size, (key, card-1) uint16 pairs, int32 offsets, containers.
//   cookie 12347: low 16 bits = 12347, high 16 bits = size-1, run-flag bitset ceil(size/8) bytes, (key, card-1)
//                 pairs, int32 offsets only when size >= 4, containers.
//   container: run (flag set) = uint16 n + n (start, length-1) pairs; else card > 4096 = bitmap 1024 x uint64;
//              else array card x uint16.  All little-endian.
#include "pgpu_host.h"

namespace {
inline uint16_t rd_le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
int bad(std::string* err, const std::string& m) {
  *err = m;
  return PGPU_E_INVALID;
}
}  // namespace

int pgpu_parse_roaring(const uint8_t* p, size_t n, std::vector<PgpuRoaringContainer>* out, std::string* err) {
  if (n < 4) return bad(err, "roaring bitmap truncated");
  const uint32_t cookie = rd_le32(p);
  size_t pos;
  uint32_t size;
  bool has_run = false;
  const uint8_t* runflags = nullptr;
  if ((cookie & 0xFFFFu) == 12347u) {
    has_run = true;
    size = (cookie >> 16) + 1;
    runflags = p + 4;
    pos = 4 + (size + 7) / 8;
    if (pos > n) return bad(err, "roaring run flags truncated");
  } else if (cookie == 12346u) {
    if (n < 8) return bad(err, "roaring bitmap truncated");
    size = rd_le32(p + 4);
    pos = 8;
  } else {
    return bad(err, "bad roaring cookie " + std::to_string(cookie));
  }
  if (size > 65536u) return bad(err, "bad roaring container count " + std::to_string(size));
  if (pos + 4ull * size > n) return bad(err, "roaring header truncated");
  const uint8_t* kc = p + pos;
  pos += 4ull * size;
  if (!has_run || size >= 4) pos += 4ull * size;  // offsets
  if (pos > n) return bad(err, "roaring offsets truncated");
  const size_t first = out->size();
  for (uint32_t i = 0; i < size; ++i) {
    PgpuRoaringContainer c;
    c.key = rd_le16(kc + 4 * i);
    const uint32_t card = (uint32_t)rd_le16(kc + 4 * i + 2) + 1;
    const bool run = has_run && ((runflags[i / 8] >> (i % 8)) & 1);
    if (run) {
      if (pos + 2 > n) return bad(err, "roaring run container truncated");
      const uint32_t nruns = rd_le16(p + pos);
      pos += 2;
      c.type = 2;
      c.card = nruns;
      c.payload = p + pos;
      c.payload_bytes = 4ull * nruns;
    } else if (card > 4096) {
      c.type = 1;
      c.card = card;
      c.payload = p + pos;
      c.payload_bytes = 8192;
    } else {
      c.type = 0;
      c.card = card;
      c.payload = p + pos;
      c.payload_bytes = 2ull * card;
    }
    if (c.payload_bytes > n - pos) return bad(err, "roaring container " + std::to_string(i) + " truncated");
    if (out->size() > first && c.key <= out->back().key) return bad(err, "roaring keys not ascending");
    // the kernels index a 65,536-bit image of each container by these values: they must stay inside it
    if (c.type == 0) {
      for (uint32_t k = 1; k < c.card; ++k)
        if (rd_le16(c.payload + 2 * k) <= rd_le16(c.payload + 2 * (k - 1)))
          return bad(err, "roaring array container " + std::to_string(i) + " not ascending");
    } else if (c.type == 2) {
      uint32_t next = 0;  // first value the next run may start at
      for (uint32_t r = 0; r < c.card; ++r) {
        const uint32_t s = rd_le16(c.payload + 4 * r), l = rd_le16(c.payload + 4 * r + 2);
        if (s < next || s + l > 65535u) return bad(err, "roaring run container " + std::to_string(i) + " malformed");
        next = s + l + 1;
      }
    }
    pos += c.payload_bytes;
    out->push_back(c);
  }
  return PGPU_OK;
}
