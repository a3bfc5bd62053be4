// Node-level combine inside libpinotgpu: one process drives several GPUs of a node (the one-JVM Pinot server),
// and the per-GPU partial tables are merged with RCCL over xGMI inside the library -- the combine step the
// reference runs on the host (AggregationOnlyCombineOperator.mergeResultsBlocks,
// core/operator/combine/AggregationOnlyCombineOperator.java:47-57; GroupByOrderByCombineOperator's IndexedTable
// upserts, core/operator/combine/GroupByOrderByCombineOperator.java:127-248).
//
//   dense tables : every device launches its segments into its own table; one grouped ncclReduce per section
//                  (int64 SUM for counts and integer sums, float64 SUM, int64 MIN / MAX of order-preserving keys)
//                  lands the merged table on device 0, which compacts it.
//   hash tables  : slot assignments differ per device, so each device compacts its table and the rows are merged
//                  by key on the host (AggregationFunction.merge per section).
//
// RCCL is loaded with dlopen on the first pgpu_node_init, so processes that never build a node (one process per
// GPU, torch.distributed) do not load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pinot_gpu.h"

// pgpu_runtime.cpp: the calling thread's pgpu_last_error message; docs of a descriptor's segments
int pgpu_set_error(int code, const char* msg);
int64_t pgpu_desc_docs(const pgpu_query_desc* q);

namespace {

int nfail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return pgpu_set_error(code, buf);
}

// The slice of the RCCL API the node uses (rccl/rccl.h: ncclComm_t is a pointer, enums are ints).
typedef void* ncclComm_t;
typedef int ncclResult_t;
enum { ncclInt64 = 4, ncclFloat64 = 8 };
enum { ncclSum = 0, ncclMax = 2, ncclMin = 3 };

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Reduce)(const void*, void*, size_t, int, int, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  std::string error;

  bool load() {
    if (h) return true;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      error = dlerror() ? dlerror() : "librccl not found";
      return false;
    }
    CommInitAll = (decltype(CommInitAll))dlsym(h, "ncclCommInitAll");
    CommDestroy = (decltype(CommDestroy))dlsym(h, "ncclCommDestroy");
    GroupStart = (decltype(GroupStart))dlsym(h, "ncclGroupStart");
    GroupEnd = (decltype(GroupEnd))dlsym(h, "ncclGroupEnd");
    Reduce = (decltype(Reduce))dlsym(h, "ncclReduce");
    GetErrorString = (decltype(GetErrorString))dlsym(h, "ncclGetErrorString");
    if (!CommInitAll || !CommDestroy || !GroupStart || !GroupEnd || !Reduce || !GetErrorString) {
      error = "librccl lacks a required symbol";
      h = nullptr;
      return false;
    }
    return true;
  }
  const char* str(ncclResult_t r) const { return GetErrorString ? GetErrorString(r) : "rccl error"; }
};

Rccl g_rccl;
std::mutex g_rccl_mu;

struct DevBuf {
  int device = 0;
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (n >= bytes) return hipSuccess;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return e;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    e = hipMalloc(&p, bytes);
    if (e == hipSuccess) n = bytes;
    return e;
  }
};

}  // namespace

struct pgpu_node {
  std::vector<int> devices;
  std::vector<pgpu_context*> ctxs;
  std::vector<hipStream_t> streams;
  std::vector<ncclComm_t> comms;
  std::vector<DevBuf> tables;
  std::mutex mu;  // one node query at a time (the tables are node-owned)
};

namespace {

int reduce_dense(pgpu_node* nd, const pgpu_table_layout& L) {
  const size_t G = L.num_keys;
  ncclResult_t r = g_rccl.GroupStart();
  for (size_t i = 0; i < nd->devices.size() && r == 0; ++i) {
    // contiguous runs of sections with the same op go in one call
    int s = 0;
    while (s < L.num_sections && r == 0) {
      int e = s + 1;
      while (e < L.num_sections && L.section_op[e] == L.section_op[s]) ++e;
      const int op = L.section_op[s];
      const int type = op == PGPU_RED_SUM_F64 ? ncclFloat64 : ncclInt64;
      const int rop = op == PGPU_RED_MIN_I64 ? ncclMin : (op == PGPU_RED_MAX_I64 ? ncclMax : ncclSum);
      const char* src = (const char*)nd->tables[i].p + 8 * G * (size_t)s;
      char* dst = (char*)nd->tables[0].p + 8 * G * (size_t)s;  // significant on the root only
      r = g_rccl.Reduce(src, i == 0 ? dst : (void*)src, G * (size_t)(e - s), type, rop, 0, nd->comms[i],
                        nd->streams[i]);
      s = e;
    }
  }
  const ncclResult_t r2 = g_rccl.GroupEnd();
  if (r != 0 || r2 != 0) return nfail(PGPU_E_HIP, "ncclReduce: %s", g_rccl.str(r ? r : r2));
  for (size_t i = 0; i < nd->devices.size(); ++i) {
    (void)hipSetDevice(nd->devices[i]);
    const hipError_t e = hipStreamSynchronize(nd->streams[i]);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node reduce: %s", hipGetErrorString(e));
  }
  return PGPU_OK;
}

int64_t cell_merge(int op, int64_t a, int64_t b) {
  if (op == PGPU_RED_SUM_I64) return (int64_t)((uint64_t)a + (uint64_t)b);
  if (op == PGPU_RED_SUM_F64) {
    double x, y;
    memcpy(&x, &a, 8);
    memcpy(&y, &b, 8);
    x += y;
    memcpy(&a, &x, 8);
    return a;
  }
  if (op == PGPU_RED_MIN_I64) return std::min(a, b);
  return std::max(a, b);
}

}  // namespace

extern "C" {

int pgpu_node_init(const int32_t* device_ordinals, int32_t num_devices, pgpu_node** out_node) {
  if (!device_ordinals || num_devices < 1 || !out_node) return nfail(PGPU_E_INVALID, "bad node arguments");
  {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl.load()) return nfail(PGPU_E_UNSUPPORTED, "RCCL unavailable: %s", g_rccl.error.c_str());
  }
  auto* nd = new pgpu_node();
  auto bail = [&](int rc) {
    pgpu_node_shutdown(nd);
    return rc;
  };
  for (int i = 0; i < num_devices; ++i) {
    pgpu_context* ctx = nullptr;
    const int rc = pgpu_init(device_ordinals[i], &ctx);
    if (rc) return bail(rc);
    nd->devices.push_back(device_ordinals[i]);
    nd->ctxs.push_back(ctx);
    hipStream_t st = nullptr;
    (void)hipSetDevice(device_ordinals[i]);
    const hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(nfail(PGPU_E_HIP, "node stream: %s", hipGetErrorString(e)));
    nd->streams.push_back(st);
    DevBuf b;
    b.device = device_ordinals[i];
    nd->tables.push_back(b);
  }
  nd->comms.assign(num_devices, nullptr);
  const ncclResult_t r = g_rccl.CommInitAll(nd->comms.data(), num_devices, nd->devices.data());
  if (r != 0) {
    nd->comms.clear();
    return bail(nfail(PGPU_E_HIP, "ncclCommInitAll: %s", g_rccl.str(r)));
  }
  *out_node = nd;
  return PGPU_OK;
}

int pgpu_node_context(pgpu_node* node, int32_t index, pgpu_context** out_ctx) {
  if (!node || !out_ctx || index < 0 || index >= (int32_t)node->ctxs.size())
    return nfail(PGPU_E_INVALID, "bad node context index %d", index);
  *out_ctx = node->ctxs[index];
  return PGPU_OK;
}

int pgpu_node_shutdown(pgpu_node* node) {
  if (!node) return PGPU_OK;
  for (ncclComm_t c : node->comms)
    if (c) (void)g_rccl.CommDestroy(c);
  for (size_t i = 0; i < node->tables.size(); ++i) {
    (void)hipSetDevice(node->tables[i].device);
    if (node->tables[i].p) (void)hipFree(node->tables[i].p);
  }
  for (size_t i = 0; i < node->streams.size(); ++i) {
    (void)hipSetDevice(node->devices[i]);
    (void)hipStreamDestroy(node->streams[i]);
  }
  for (pgpu_context* c : node->ctxs) pgpu_shutdown(c);
  delete node;
  return PGPU_OK;
}

int pgpu_node_query(pgpu_node* node, const pgpu_query_desc* const* descs, int64_t* out_keys, int64_t* out_cells,
                    uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats,
                    pgpu_table_layout* out_layout) {
  if (!node || !descs || !out_num_groups) return nfail(PGPU_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(node->mu);
  const size_t n = node->devices.size();
  // one table layout on every device: the docs of the whole node bound the integer sums, and a split or hash
  // layout chosen by any device is taken by all
  std::vector<pgpu_query_desc> qs(n);
  std::vector<pgpu_table_layout> L(n);
  int64_t node_docs = 0;
  for (size_t i = 0; i < n; ++i) {
    if (!descs[i]) return nfail(PGPU_E_INVALID, "device %zu has no query", i);
    qs[i] = *descs[i];
    node_docs += pgpu_desc_docs(&qs[i]);
  }
  uint64_t extra = 0;
  for (size_t i = 0; i < n; ++i) {
    qs[i].reduce_docs = std::max<int64_t>(qs[i].reduce_docs, node_docs);
    const int rc = pgpu_table_layout_of(&qs[i], &L[i]);  // also validates the descriptor
    if (rc) return rc;
    for (int a = 0; a < qs[i].num_aggs; ++a)
      if (L[i].agg_sum_parts[a] == 3) extra |= PGPU_Q_SUM_SPLIT;
    if (L[i].key_kind == PGPU_KEYS_HASH) extra |= PGPU_Q_HASH;
  }
  for (size_t i = 0; i < n; ++i) {
    qs[i].flags |= extra;
    const int rc = pgpu_table_layout_of(&qs[i], &L[i]);
    if (rc) return rc;
  }
  const bool hash = L[0].key_kind == PGPU_KEYS_HASH;
  for (size_t i = 1; i < n; ++i) {
    const bool same = L[i].num_sections == L[0].num_sections && L[i].key_kind == L[0].key_kind &&
                      (hash || L[i].num_keys == L[0].num_keys) &&
                      !memcmp(L[i].section_op, L[0].section_op, sizeof(L[0].section_op));
    if (!same) return nfail(PGPU_E_INVALID, "device %zu's table layout differs from device 0's", i);
  }
  // launch every device, then wait for all
  std::vector<pgpu_query*> qq(n, nullptr);
  int rc = PGPU_OK;
  for (size_t i = 0; i < n && rc == PGPU_OK; ++i) {
    const uint64_t bytes = pgpu_table_bytes(&L[i]);
    const hipError_t e = node->tables[i].ensure(bytes);
    if (e != hipSuccess) rc = nfail(PGPU_E_HIP, "node table on device %d: %s", node->devices[i], hipGetErrorString(e));
    else rc = pgpu_query_launch(node->ctxs[i], &qs[i], node->streams[i], node->tables[i].p, bytes, &qq[i]);
  }
  pgpu_query_stats tot{};
  tot.filter_stats_exact = 1;
  for (size_t i = 0; i < n; ++i) {
    if (!qq[i]) continue;
    pgpu_query_stats st{};
    const int w = pgpu_query_wait(qq[i], &st);
    if (rc == PGPU_OK && w != PGPU_OK) rc = w;
    pgpu_query_release(qq[i]);
    tot.num_docs_scanned += st.num_docs_scanned;
    tot.num_entries_scanned_in_filter += st.num_entries_scanned_in_filter;
    tot.num_total_docs += st.num_total_docs;
    tot.num_segments_matched += st.num_segments_matched;  // the devices' segments are disjoint
    tot.num_groups_limit_reached |= st.num_groups_limit_reached;
    tot.sparse_sector_bytes += st.sparse_sector_bytes;
    tot.dense_bytes += st.dense_bytes;
    tot.kernel_ms = std::max(tot.kernel_ms, st.kernel_ms);
    tot.filter_stats_exact &= st.filter_stats_exact;
  }
  if (rc) return rc;
  if (out_stats) *out_stats = tot;
  if (out_layout) *out_layout = L[0];
  if (!hash) {
    rc = reduce_dense(node, L[0]);
    if (rc) return rc;
    return pgpu_table_compact(node->ctxs[0], &L[0], node->tables[0].p, node->streams[0], out_keys, out_cells, capacity,
                              out_num_groups);
  }
  // hash tables: compact per device, merge rows by key
  const int kw = L[0].key_words == 2 ? 2 : 1;
  const int nsec = L[0].num_sections;
  std::map<std::vector<int64_t>, std::vector<int64_t>> merged;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t cap = L[i].num_keys;
    std::vector<int64_t> keys(cap * kw + 1), cells(cap * nsec + 1);
    uint64_t got = 0;
    rc = pgpu_table_compact(node->ctxs[i], &L[i], node->tables[i].p, node->streams[i], keys.data(), cells.data(), cap,
                            &got);
    if (rc) return rc;
    for (uint64_t r = 0; r < got; ++r) {
      std::vector<int64_t> k(keys.begin() + r * kw, keys.begin() + (r + 1) * kw);
      auto it = merged.find(k);
      if (it == merged.end()) {
        merged.emplace(std::move(k), std::vector<int64_t>(cells.begin() + r * nsec, cells.begin() + (r + 1) * nsec));
      } else {
        for (int s = 0; s < nsec; ++s) it->second[s] = cell_merge(L[0].section_op[s], it->second[s], cells[r * nsec + s]);
      }
    }
  }
  *out_num_groups = merged.size();
  if (merged.size() > capacity)
    return nfail(PGPU_E_INVALID, "%zu non-empty groups exceed capacity %llu", merged.size(),
                 (unsigned long long)capacity);
  uint64_t r = 0;
  for (const auto& kv : merged) {
    for (int w = 0; w < kw; ++w) out_keys[r * kw + w] = kv.first[w];
    for (int s = 0; s < nsec; ++s) out_cells[r * nsec + s] = kv.second[s];
    ++r;
  }
  return PGPU_OK;
}

}  // extern "C"
