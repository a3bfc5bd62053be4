// Sanitizer harness for libpinotgpu's host-side parsers of untrusted segment bytes (built with
// -fsanitize=address,undefined by tests/test_host_sanitize.py, CPU only): pgpu_decode_raw_forward (raw forward
// index chunks: PASS_THROUGH / SNAPPY / LZ4 / LZ4_LENGTH_PREFIXED / ZSTANDARD), pgpu_parse_roaring (inverted-index bitmaps)
// and reference_entries_scanned (filter programs replayed over leaf bitmaps).
//
// Usage: host_fuzz <kind> <file> [variants]   kind = raw:<width>:<num_docs> | roaring | program
// For every input it runs the parser on the file itself (which must succeed), on every truncation and on
// `variants` copies with 1-8 random bytes overwritten (deterministic xorshift): each must return a status, never
// crash, hang or touch memory outside its buffers (ASan / UBSan abort the run if it does).  A truncated or
// corrupted input may still parse when the change happens to be consistent; the harness only requires that a
// success is self-consistent.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../pinot_amd/csrc/pgpu_host.h"

namespace {
uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return g_state;
}

int run_raw(const std::vector<uint8_t>& b, int width, int ndocs) {
  std::vector<uint8_t> out;
  std::string err;
  const int rc = pgpu_decode_raw_forward(b.data(), b.size(), width, ndocs, &out, &err);
  if (rc == PGPU_OK && out.size() != (size_t)ndocs * width) {
    fprintf(stderr, "raw: success with %zu output bytes\n", out.size());
    abort();
  }
  return rc;
}

int run_roaring(const std::vector<uint8_t>& b) {
  std::vector<PgpuRoaringContainer> out;
  std::string err;
  const int rc = pgpu_parse_roaring(b.data(), b.size(), &out, &err);
  if (rc == PGPU_OK) {
    uint64_t sum = 0;  // touch every payload byte the parser vouched for
    for (const PgpuRoaringContainer& c : out) {
      if (c.payload < b.data() || c.payload + c.payload_bytes > b.data() + b.size()) abort();
      for (size_t k = 0; k < c.payload_bytes; ++k) sum += c.payload[k];
    }
    g_state += sum;
  }
  return rc;
}

// A filter program file: int32 num_nodes, num_docs, then per node {op, negate} int32 pairs (leaves = op 0).
int run_program(const std::vector<uint8_t>& b) {
  if (b.size() < 8) return PGPU_E_INVALID;
  int32_t nn, nd;
  memcpy(&nn, b.data(), 4);
  memcpy(&nd, b.data() + 4, 4);
  if (nn < 0 || nn > 64 || nd < 0 || nd > 5000 || b.size() < 8 + 8ull * nn) return PGPU_E_INVALID;
  std::vector<pgpu_filter_node> nodes(nn);
  int leaves = 0;
  for (int i = 0; i < nn; ++i) {
    memset(&nodes[i], 0, sizeof(pgpu_filter_node));
    memcpy(&nodes[i].op, b.data() + 8 + 8 * i, 4);
    memcpy(&nodes[i].negate, b.data() + 12 + 8 * i, 4);
    const int op = nodes[i].op;
    if (op == PGPU_F_SCAN || op == PGPU_F_INVERTED || op == PGPU_F_SORTED || op == PGPU_F_RAW_SCAN ||
        op == PGPU_F_RANGE_INDEX)
      ++leaves;
  }
  std::vector<std::vector<uint32_t>> words(leaves, std::vector<uint32_t>((nd + 31) / 32 + 1));
  std::vector<const uint32_t*> ptrs;
  for (auto& w : words) {
    for (auto& x : w) x = (uint32_t)rnd();
    ptrs.push_back(w.data());
  }
  const int64_t c = reference_entries_scanned(nodes.data(), nn, ptrs.data(), leaves, nd);
  (void)pgpu_filter_count_is_reference(nodes.data(), nn);
  return c < 0 ? PGPU_E_INVALID : PGPU_OK;
}

int run(const std::string& kind, const std::vector<uint8_t>& b) {
  if (kind.rfind("raw:", 0) == 0) {
    int width = 0, ndocs = 0;
    if (sscanf(kind.c_str(), "raw:%d:%d", &width, &ndocs) != 2) abort();
    return run_raw(b, width, ndocs);
  }
  if (kind == "roaring") return run_roaring(b);
  if (kind == "program") return run_program(b);
  fprintf(stderr, "unknown kind %s\n", kind.c_str());
  abort();
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string kind = argv[1];
  FILE* f = fopen(argv[2], "rb");
  if (!f) return 2;
  std::vector<uint8_t> b;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + k);
  fclose(f);
  const int variants = argc > 3 ? atoi(argv[3]) : 1000;
  g_state ^= b.size() * 0x2545F4914F6CDD1Dull;
  const bool valid_input = kind != "program";
  if (valid_input && run(kind, b) != PGPU_OK) {
    fprintf(stderr, "the unmodified input does not parse\n");
    return 1;
  }
  int rejected = 0, total = 0;
  const size_t step = b.size() > 4096 ? b.size() / 2048 : 1;
  for (size_t len = 0; len < b.size(); len += step) {  // truncations (a copy, so ASan sees the true end)
    std::vector<uint8_t> t(b.begin(), b.begin() + len);
    rejected += run(kind, t) != PGPU_OK;
    ++total;
  }
  for (int v = 0; v < variants && !b.empty(); ++v) {  // overwritten bytes
    std::vector<uint8_t> t = b;
    const int nflip = 1 + (int)(rnd() % 8);
    for (int j = 0; j < nflip; ++j) t[rnd() % t.size()] = (uint8_t)rnd();
    rejected += run(kind, t) != PGPU_OK;
    ++total;
  }
  printf("%s %s: %d variants, %d rejected\n", kind.c_str(), argv[2], total, rejected);
  return 0;
}
