// Raw (no-dictionary) single-value forward index of a fixed-width column: the bytes FixedByteChunkSVForwardIndexWriter
// writes, decoded on the host at segment upload into the little-endian value array the kernels index by doc id.
//
// File layout (seglocal/io/writer/impl/BaseChunkSVForwardIndexWriter.java:125-160, read back by
// seglocal/segment/index/readers/forward/BaseChunkSVForwardIndexReader.java:56-101):
//   int32 version, int32 numChunks, int32 numDocsPerChunk, int32 lengthOfLongestEntry (= the value width)
//   version >= 2: int32 totalDocs, int32 compressionType (ChunkCompressionType ordinal), int32 dataHeaderStart
//   chunk offsets: numChunks x int32 (versions 1, 2) or int64 (versions 3, 4), absolute file positions
//   chunks: numDocsPerChunk big-endian values each (the last one may be shorter), compressed per chunk
// Version 1 has no compression field and always means SNAPPY; version 4 rounds numDocsPerChunk up to a power of two
// (FixedByteChunkSVForwardIndexWriter.normalizeDocsPerChunk) and is read by FixedBytePower2ChunkSVForwardIndexReader.
//
// Codecs (seglocal/io/compression/ChunkCompressorFactory.java): PASS_THROUGH, SNAPPY (snappy-java raw block format),
// LZ4 (lz4-java fastCompressor: raw LZ4 block), LZ4_LENGTH_PREFIXED (lz4-java LZ4CompressorWithLength: 4-byte
// little-endian decompressed length, then a raw LZ4 block).  The snappy and LZ4 libraries are third-party
// dependencies of the reference (not vendored); their published block formats are restated below.  ZSTANDARD
// (seglocal/io/compression/ZstandardDecompressor.java: zstd-jni 1.4.9-5 `Zstd.decompress`, one zstd frame per chunk)
// is decoded by the system's libzstd.so.1, loaded on first use; without it such a segment returns PGPU_E_UNSUPPORTED
// and the server keeps its CPU reader.
#include <dlfcn.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "pgpu_host.h"

namespace {

inline uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
inline uint64_t rd_be64(const uint8_t* p) { return ((uint64_t)rd_be32(p) << 32) | rd_be32(p + 4); }

// Snappy raw block: varint uncompressed length, then elements.  Tag low 2 bits: 00 literal (length-1 in the upper 6
// bits, or 60..63 = 1..4 little-endian length bytes follow), 01 copy with 1-byte offset (len 4 + 3 bits, offset 3
// high bits << 8 | next byte), 10 copy with 2-byte LE offset (len 1 + 6 bits), 11 copy with 4-byte LE offset.
// `cap`: the most bytes a chunk may decode to (its values); a longer declared or produced output is malformed.
bool snappy_decode(const uint8_t* in, size_t n, std::vector<uint8_t>* out, uint64_t cap) {
  size_t i = 0;
  uint64_t len = 0;
  for (int shift = 0;; shift += 7) {
    if (i >= n || shift > 35) return false;
    const uint8_t b = in[i++];
    len |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) break;
  }
  if (len > cap) return false;
  out->clear();
  out->reserve((size_t)std::min<uint64_t>(len, 32ull * n + 64));  // a snappy element expands at most ~22x
  while (i < n) {
    const uint8_t tag = in[i++];
    const int type = tag & 3;
    if (type == 0) {
      uint64_t l = tag >> 2;
      if (l >= 60) {
        const int nb = (int)l - 59;
        if (i + nb > n) return false;
        l = 0;
        for (int k = 0; k < nb; ++k) l |= (uint64_t)in[i + k] << (8 * k);
        i += nb;
      }
      ++l;
      if (l > n - i || out->size() + l > len) return false;
      out->insert(out->end(), in + i, in + i + l);
      i += l;
      continue;
    }
    uint64_t l, off;
    if (type == 1) {
      if (i >= n) return false;
      l = 4 + ((tag >> 2) & 7);
      off = ((uint64_t)(tag >> 5) << 8) | in[i++];
    } else if (type == 2) {
      if (i + 2 > n) return false;
      l = 1 + (tag >> 2);
      off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8);
      i += 2;
    } else {
      if (i + 4 > n) return false;
      l = 1 + (tag >> 2);
      off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8) | ((uint64_t)in[i + 2] << 16) | ((uint64_t)in[i + 3] << 24);
      i += 4;
    }
    if (off == 0 || off > out->size() || out->size() + l > len) return false;
    const size_t from = out->size() - off;
    for (uint64_t k = 0; k < l; ++k) out->push_back((*out)[from + k]);  // overlapping copies repeat the pattern
  }
  return out->size() == len;
}

// LZ4 block: sequences of token (literal length high nibble, match length - 4 low nibble; 15 = extended by 255-run
// bytes), literals, 2-byte LE match offset, extended match length.  The last sequence has literals only.
bool lz4_decode(const uint8_t* in, size_t n, std::vector<uint8_t>* out, uint64_t cap) {
  out->clear();
  size_t i = 0;
  while (i < n) {
    const uint8_t token = in[i++];
    uint64_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (i >= n) return false;
        b = in[i++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - i || out->size() + lit > cap) return false;
    out->insert(out->end(), in + i, in + i + lit);
    i += lit;
    if (i == n) break;  // last sequence
    if (i + 2 > n) return false;
    const uint64_t off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8);
    i += 2;
    uint64_t ml = token & 15;
    if (ml == 15) {
      uint8_t b;
      do {
        if (i >= n) return false;
        b = in[i++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (off == 0 || off > out->size() || out->size() + ml > cap) return false;
    const size_t from = out->size() - off;
    for (uint64_t k = 0; k < ml; ++k) out->push_back((*out)[from + k]);
  }
  return true;
}

// ZSTANDARD chunk: one zstd frame (RFC 8878) decoded by libzstd's ZSTD_decompress into at most `cap` bytes.  The
// library is resolved once; its two entry points have been ABI-stable since zstd 1.0.
struct Zstd {
  size_t (*decompress)(void*, size_t, const void*, size_t) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
};
const Zstd& zstd_lib() {
  static const Zstd z = [] {
    Zstd r;
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return r;
    r.decompress = (size_t(*)(void*, size_t, const void*, size_t))dlsym(h, "ZSTD_decompress");
    r.is_error = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
    if (!r.decompress || !r.is_error) r.decompress = nullptr;
    return r;
  }();
  return z;
}
// 1: decoded, 0: malformed (or longer than `cap`), -1: no zstd library
int zstd_decode(const uint8_t* in, size_t n, std::vector<uint8_t>* out, uint64_t cap) {
  const Zstd& z = zstd_lib();
  if (!z.decompress) return -1;
  out->resize((size_t)cap);
  const size_t r = z.decompress(out->data(), (size_t)cap, in, n);
  if (z.is_error(r)) return 0;
  out->resize(r);
  return 1;
}

}  // namespace

// Decodes the file into num_docs little-endian values of `width` bytes (out is resized to num_docs * width).
// Returns PGPU_OK, or a status with *err set.
int pgpu_decode_raw_forward(const uint8_t* b, uint64_t n, int32_t width, int32_t num_docs, std::vector<uint8_t>* out,
                            std::string* err) {
  auto bad = [&](int code, const std::string& m) {
    *err = m;
    return code;
  };
  if (n < 16) return bad(PGPU_E_INVALID, "raw forward index shorter than its header");
  const int32_t version = (int32_t)rd_be32(b);
  const int32_t num_chunks = (int32_t)rd_be32(b + 4);
  const int32_t docs_per_chunk = (int32_t)rd_be32(b + 8);
  const int32_t entry = (int32_t)rd_be32(b + 12);
  if (version < 1 || version > 4) return bad(PGPU_E_INVALID, "raw forward index version " + std::to_string(version));
  if (entry != width) return bad(PGPU_E_INVALID, "raw forward index entry length " + std::to_string(entry) +
                                                     " != value width " + std::to_string(width));
  if (num_chunks < 0 || docs_per_chunk <= 0 || (int64_t)num_chunks * docs_per_chunk < num_docs)
    return bad(PGPU_E_INVALID, "raw forward index chunk geometry does not cover numDocs");
  int32_t codec = 1;  // version 1: SNAPPY
  uint64_t data_header = 16;
  if (version > 1) {
    if (n < 28) return bad(PGPU_E_INVALID, "raw forward index header truncated");
    codec = (int32_t)rd_be32(b + 20);
    data_header = rd_be32(b + 24);
  }
  const int off_size = version >= 3 ? 8 : 4;
  if (data_header + (uint64_t)num_chunks * off_size > n) return bad(PGPU_E_INVALID, "raw forward index chunk offsets truncated");
  if (codec == 2 && !zstd_lib().decompress)
    return bad(PGPU_E_UNSUPPORTED, "ZSTANDARD raw forward index chunks need libzstd.so.1, which is not loadable");
  if (codec < 0 || codec > 4) return bad(PGPU_E_INVALID, "raw forward index compression type " + std::to_string(codec));
  auto chunk_pos = [&](int32_t c) -> uint64_t {
    const uint8_t* p = b + data_header + (uint64_t)c * off_size;
    return off_size == 8 ? rd_be64(p) : rd_be32(p);
  };
  const uint64_t chunk_bytes = (uint64_t)docs_per_chunk * width;
  out->assign((uint64_t)num_docs * width, 0);
  std::vector<uint8_t> buf;
  uint64_t done = 0;  // values decoded
  for (int32_t c = 0; c < num_chunks && done < (uint64_t)num_docs; ++c) {
    const uint64_t pos = chunk_pos(c);
    const uint64_t end = c + 1 < num_chunks ? chunk_pos(c + 1) : n;
    if (pos > end || end > n) return bad(PGPU_E_INVALID, "raw forward index chunk " + std::to_string(c) + " out of bounds");
    const uint8_t* src = b + pos;
    uint64_t len = end - pos;
    if (codec == 0) {  // PASS_THROUGH: the chunk's values as they are
      buf.assign(src, src + std::min(len, chunk_bytes));
    } else if (codec == 1) {
      if (!snappy_decode(src, len, &buf, chunk_bytes)) return bad(PGPU_E_INVALID, "bad SNAPPY chunk " + std::to_string(c));
    } else if (codec == 2) {
      if (zstd_decode(src, len, &buf, chunk_bytes) != 1) return bad(PGPU_E_INVALID, "bad ZSTANDARD chunk " + std::to_string(c));
    } else {
      if (codec == 4) {  // LZ4_LENGTH_PREFIXED
        if (len < 4) return bad(PGPU_E_INVALID, "bad LZ4 chunk " + std::to_string(c));
        const uint32_t dl = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) | ((uint32_t)src[3] << 24);
        src += 4;
        len -= 4;
        if (dl > chunk_bytes || !lz4_decode(src, len, &buf, dl) || buf.size() != dl) return bad(PGPU_E_INVALID, "bad LZ4 chunk " + std::to_string(c));
      } else if (!lz4_decode(src, len, &buf, chunk_bytes)) {
        return bad(PGPU_E_INVALID, "bad LZ4 chunk " + std::to_string(c));
      }
    }
    const uint64_t vals = std::min<uint64_t>(buf.size() / width, (uint64_t)num_docs - done);
    if (buf.size() % width || (vals < (uint64_t)docs_per_chunk && done + vals < (uint64_t)num_docs))
      return bad(PGPU_E_INVALID, "raw forward index chunk " + std::to_string(c) + " holds a partial value set");
    uint8_t* dst = out->data() + done * width;
    for (uint64_t k = 0; k < vals; ++k)  // big-endian -> little-endian
      for (int j = 0; j < width; ++j) dst[k * width + j] = buf[k * width + width - 1 - j];
    done += vals;
  }
  if (done != (uint64_t)num_docs) return bad(PGPU_E_INVALID, "raw forward index holds fewer values than numDocs");
  return PGPU_OK;
}
