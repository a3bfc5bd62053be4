// Node-level combine inside libpinotgpu: one process drives several GPUs of a node (the one-JVM Pinot server),
// and the per-GPU partial tables are merged over xGMI inside the library -- the combine step the reference runs on
// the host (AggregationOnlyCombineOperator.mergeResultsBlocks, core/operator/combine/AggregationOnlyCombineOperator
// .java:47-57; GroupByOrderByCombineOperator's IndexedTable upserts and trim, core/operator/combine/
// GroupByOrderByCombineOperator.java:127-248, GroupByUtils.java:24-41).  The same collectives as the
// one-process-per-GPU combine (pinot_amd/combine.py):
//
//   dense, small (aggregation only, or < 1 MiB) : one grouped ncclReduce per run of same-op sections to device 0,
//                  which compacts (or trims by the ORDER BY key) -- combine.py's all_reduce + rank-0 compaction;
//   dense, large : a reduce-scatter -- grouped ncclReduce of each section's key slice [d*K, d*K + K) to its owner d
//                  (K = ceil(G / n), uneven G allowed) -- then every device trims ITS slice (pgpu_table_topk with
//                  key_base = d*K: every kept row is final) and the host concatenates the slices' rows;
//   hash tables  : slot assignments differ per device, so each device compacts its rows into device memory, routes
//                  every row to the owner of its key (pgpu_key_owner_of: combine.py's routing, bit for bit) over
//                  peer copies, the owner merges them into a fresh hash table (node_merge_kernel) and trims it --
//                  combine.py's all_to_all + merge_rows + per-rank top-K.
//
// RCCL is loaded with dlopen on the first pgpu_node_init, so processes that never build a node (one process per
// GPU, torch.distributed) do not load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pinot_gpu.h"
#include "pgpu_internal.h"

// pgpu_runtime.cpp: the calling thread's pgpu_last_error message; docs of a descriptor's segments; device-side
// compaction.  pgpu_kernels.hip: the hash-row routing and merge kernels.
int pgpu_set_error(int code, const char* msg);
int64_t pgpu_desc_docs(const pgpu_query_desc* q);
int pgpu_compact_to_device(pgpu_context* ctx, const pgpu_table_layout* L, const void* dev_table, hipStream_t st,
                           int64_t* dkeys, int64_t* dcells, uint64_t capacity, uint64_t* out_n);
hipError_t pgpu_launch_node_route(const int64_t* keys, const int64_t* cells, uint64_t n, int32_t kw, int32_t nsec,
                                  int32_t world, uint8_t* owner, uint32_t* counts, uint32_t* cursor, int64_t* rows,
                                  bool scatter, hipStream_t st);
hipError_t pgpu_launch_node_merge(const int64_t* rows, uint64_t n, int32_t kw, int32_t nsec, int64_t* table,
                                  uint64_t P, const NodeOps& ops, int32_t* hflag, hipStream_t st);

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
  std::vector<hipStream_t> streams;   // query kernels
  std::vector<hipStream_t> mstreams;  // merges (collectives, compaction) of a query whose kernels are done, so they
                                      // do not queue behind the kernels of queries submitted after it
  std::vector<ncclComm_t> comms;
  // per device scratch of the merges: the slice copy (dense) / compacted rows, routing, send and receive buffers and
  // the merged table (hash)
  std::vector<DevBuf> slice, rkeys, rcells, route, send, recv, merged;
  // partial-table sets (one table per device) of the queries in flight, reused
  std::vector<std::vector<DevBuf>> free_tables;
  std::mutex mu;  // submit and collect are serialised (the merge scratch is node-owned)
};

// A node query in flight: every device's launch and the table set it writes.
struct pgpu_node_pending {
  pgpu_node* node = nullptr;
  std::vector<pgpu_query*> qq;
  std::vector<pgpu_table_layout> L;
  std::vector<DevBuf> tables;
  int32_t num_group_columns = 0;
};

namespace {

int sync_all(pgpu_node* nd, const char* what) {
  for (size_t i = 0; i < nd->devices.size(); ++i) {
    (void)hipSetDevice(nd->devices[i]);
    const hipError_t e = hipStreamSynchronize(nd->mstreams[i]);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "%s: %s", what, hipGetErrorString(e));
  }
  return PGPU_OK;
}

int nccl_type(int op) { return op == PGPU_RED_SUM_F64 ? ncclFloat64 : ncclInt64; }
int nccl_op(int op) { return op == PGPU_RED_MIN_I64 ? ncclMin : (op == PGPU_RED_MAX_I64 ? ncclMax : ncclSum); }

// Whole dense tables reduced onto device 0: one grouped ncclReduce per run of same-op sections.
int reduce_dense(pgpu_node* nd, std::vector<DevBuf>& tables, const pgpu_table_layout& L) {
  const size_t G = L.num_keys;
  ncclResult_t r = g_rccl.GroupStart();
  for (size_t i = 0; i < nd->devices.size() && r == 0; ++i) {
    int s = 0;
    while (s < L.num_sections && r == 0) {
      int e = s + 1;
      while (e < L.num_sections && L.section_op[e] == L.section_op[s]) ++e;
      const int op = L.section_op[s];
      const char* src = (const char*)tables[i].p + 8 * G * (size_t)s;
      char* dst = (char*)tables[0].p + 8 * G * (size_t)s;  // significant on the root only
      r = g_rccl.Reduce(src, i == 0 ? dst : (void*)src, G * (size_t)(e - s), nccl_type(op), nccl_op(op), 0,
                        nd->comms[i], nd->mstreams[i]);
      s = e;
    }
  }
  const ncclResult_t r2 = g_rccl.GroupEnd();
  if (r != 0 || r2 != 0) return nfail(PGPU_E_HIP, "ncclReduce: %s", g_rccl.str(r ? r : r2));
  return sync_all(nd, "node reduce");
}

// Reduce-scatter of dense tables: device d ends up owning the final cells of keys [first, first + count) of
// pgpu_slice_of (in place in its own table).  One grouped ncclReduce per section and owner slice (an uneven G
// needs no padding).
int reduce_slices(pgpu_node* nd, std::vector<DevBuf>& tables, const pgpu_table_layout& L) {
  const size_t G = L.num_keys;
  const int n = (int)nd->devices.size();
  ncclResult_t r = g_rccl.GroupStart();
  for (int i = 0; i < n && r == 0; ++i)
    for (int s = 0; s < L.num_sections && r == 0; ++s)
      for (int d = 0; d < n && r == 0; ++d) {
        uint64_t first = 0, count = 0;
        pgpu_slice_of(G, n, d, &first, &count);
        if (!count) continue;
        char* p = (char*)tables[i].p + 8 * (G * (size_t)s + first);
        r = g_rccl.Reduce(p, p, count, nccl_type(L.section_op[s]), nccl_op(L.section_op[s]), d, nd->comms[i],
                          nd->mstreams[i]);
      }
  const ncclResult_t r2 = g_rccl.GroupEnd();
  if (r != 0 || r2 != 0) return nfail(PGPU_E_HIP, "ncclReduce (scatter): %s", g_rccl.str(r ? r : r2));
  return sync_all(nd, "node reduce-scatter");
}

// Rows of one device's (slice of the) result appended to the caller's buffers: compacted, or trimmed by `order`.
struct Out {
  int64_t* keys;
  int64_t* cells;
  uint64_t capacity, n = 0;
  int okw, nsec;
  bool overflow = false;
};
int append_rows(pgpu_context* ctx, const pgpu_table_layout& L, const void* table, hipStream_t st,
                const pgpu_topk* order, int64_t key_base, Out& out) {
  const uint64_t G = L.num_keys;
  std::vector<int64_t> k((size_t)G * out.okw + 1), c((size_t)G * out.nsec + 1);
  uint64_t got = 0;
  int rc;
  if (order) {
    pgpu_topk o = *order;
    o.key_base = (uint64_t)key_base;
    rc = pgpu_table_topk(ctx, &L, table, st, &o, k.data(), c.data(), G, &got);
  } else {
    rc = pgpu_table_compact(ctx, &L, table, st, k.data(), c.data(), G, &got);
  }
  if (rc) return rc;
  if (out.n + got > out.capacity) {
    out.overflow = true;
    out.n += got;
    return PGPU_OK;
  }
  const bool dense = L.key_kind != PGPU_KEYS_HASH;
  for (uint64_t r = 0; r < got; ++r) {
    for (int w = 0; w < out.okw; ++w) out.keys[(out.n + r) * out.okw + w] = k[r * out.okw + w] + (dense ? key_base : 0);
    memcpy(out.cells + (out.n + r) * out.nsec, c.data() + r * out.nsec, 8 * (size_t)out.nsec);
  }
  out.n += got;
  return PGPU_OK;
}

// Hash tables: every device's rows to the owners of their keys, merged there, trimmed there.
int merge_hash(pgpu_node* nd, std::vector<DevBuf>& tables, const std::vector<pgpu_table_layout>& L,
               const pgpu_topk* order, Out& out) {
  const int n = (int)nd->devices.size();
  const int kw = L[0].key_words == 2 ? 2 : 1, nsec = L[0].num_sections, width = kw + nsec;
  std::vector<uint64_t> rows(n, 0);
  std::vector<std::vector<uint32_t>> cnt(n, std::vector<uint32_t>(n, 0)), off(n, std::vector<uint32_t>(n, 0));
  for (int i = 0; i < n; ++i) {  // compact, count per owner
    const uint64_t G = L[i].num_keys;
    hipError_t e = hipSetDevice(nd->devices[i]);
    if (e == hipSuccess) e = nd->rkeys[i].ensure(8 * G * kw + 16);
    if (e == hipSuccess) e = nd->rcells[i].ensure(8 * G * nsec + 16);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node rows: %s", hipGetErrorString(e));
    int rc = pgpu_compact_to_device(nd->ctxs[i], &L[i], tables[i].p, nd->mstreams[i], (int64_t*)nd->rkeys[i].p,
                                    (int64_t*)nd->rcells[i].p, G, &rows[i]);
    if (rc) return rc;
    // route scratch: owner byte per row, then counts and cursors (n each)
    e = nd->route[i].ensure(rows[i] + 16 + 8 * (size_t)n + 16);
    if (e == hipSuccess) e = nd->send[i].ensure(8 * rows[i] * width + 16);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node route: %s", hipGetErrorString(e));
    uint8_t* owner = (uint8_t*)nd->route[i].p;
    uint32_t* counts = (uint32_t*)((char*)nd->route[i].p + ((rows[i] + 15) & ~15ull));
    e = hipMemsetAsync(counts, 0, 4 * (size_t)n, nd->mstreams[i]);
    if (e == hipSuccess && rows[i])
      e = pgpu_launch_node_route((const int64_t*)nd->rkeys[i].p, nullptr, rows[i], kw, nsec, n, owner, counts,
                                 nullptr, nullptr, false, nd->mstreams[i]);
    if (e == hipSuccess) e = hipMemcpyAsync(cnt[i].data(), counts, 4 * (size_t)n, hipMemcpyDeviceToHost, nd->mstreams[i]);
    if (e == hipSuccess) e = hipStreamSynchronize(nd->mstreams[i]);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node owners: %s", hipGetErrorString(e));
  }
  for (int i = 0; i < n; ++i) {  // rows grouped by owner in the send buffer
    if (!rows[i]) continue;
    uint32_t run = 0;
    for (int o = 0; o < n; ++o) {
      off[i][o] = run;
      run += cnt[i][o];
    }
    (void)hipSetDevice(nd->devices[i]);
    uint8_t* owner = (uint8_t*)nd->route[i].p;
    uint32_t* cursor = (uint32_t*)((char*)nd->route[i].p + ((rows[i] + 15) & ~15ull)) + n;
    hipError_t e = hipMemcpyAsync(cursor, off[i].data(), 4 * (size_t)n, hipMemcpyHostToDevice, nd->mstreams[i]);
    if (e == hipSuccess)
      e = pgpu_launch_node_route((const int64_t*)nd->rkeys[i].p, (const int64_t*)nd->rcells[i].p, rows[i], kw, nsec,
                                 n, owner, nullptr, cursor, (int64_t*)nd->send[i].p, true, nd->mstreams[i]);
    if (e == hipSuccess) e = hipStreamSynchronize(nd->mstreams[i]);  // (the cursors' host copy is a stack array)
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node scatter: %s", hipGetErrorString(e));
  }
  std::vector<uint64_t> incoming(n, 0);
  for (int o = 0; o < n; ++o) {  // peer copies into the owners' receive buffers
    for (int i = 0; i < n; ++i) incoming[o] += cnt[i][o];
    (void)hipSetDevice(nd->devices[o]);
    hipError_t e = nd->recv[o].ensure(8 * incoming[o] * width + 16);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node receive: %s", hipGetErrorString(e));
    uint64_t at = 0;
    for (int i = 0; i < n; ++i) {
      if (!cnt[i][o]) continue;
      (void)hipSetDevice(nd->devices[i]);
      e = hipMemcpyPeerAsync((char*)nd->recv[o].p + 8 * at * width, nd->devices[o],
                             (const char*)nd->send[i].p + 8 * (size_t)off[i][o] * width, nd->devices[i],
                             8 * (size_t)cnt[i][o] * width, nd->mstreams[i]);
      if (e != hipSuccess) return nfail(PGPU_E_HIP, "node peer copy: %s", hipGetErrorString(e));
      at += cnt[i][o];
    }
  }
  int rc = sync_all(nd, "node exchange");
  if (rc) return rc;
  NodeOps ops{};
  for (int s = 0; s < nsec; ++s) ops.op[s] = L[0].section_op[s];
  for (int o = 0; o < n; ++o) {  // merge on the owner, trim there
    uint64_t P = 64;
    while (P < 2 * incoming[o]) P <<= 1;
    (void)hipSetDevice(nd->devices[o]);
    hipError_t e = nd->merged[o].ensure(8 * P * (size_t)(nsec + 2) + 16);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node merged table: %s", hipGetErrorString(e));
    int32_t* hflag = (int32_t*)((char*)nd->merged[o].p + 8 * P * (size_t)(nsec + 2));
    e = hipMemsetAsync(hflag, 0, 4, nd->mstreams[o]);
    if (e == hipSuccess)
      e = pgpu_launch_node_merge((const int64_t*)nd->recv[o].p, incoming[o], kw, nsec, (int64_t*)nd->merged[o].p, P,
                                 ops, hflag, nd->mstreams[o]);
    if (e != hipSuccess) return nfail(PGPU_E_HIP, "node merge: %s", hipGetErrorString(e));
    pgpu_table_layout Lo = L[0];
    Lo.num_keys = P;
    rc = append_rows(nd->ctxs[o], Lo, nd->merged[o].p, nd->mstreams[o], order, 0, out);
    if (rc) return rc;
  }
  return PGPU_OK;
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
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(nfail(PGPU_E_HIP, "node stream: %s", hipGetErrorString(e)));
    nd->streams.push_back(st);
    hipStream_t ms = nullptr;
    e = hipStreamCreateWithFlags(&ms, hipStreamNonBlocking);
    if (e != hipSuccess) return bail(nfail(PGPU_E_HIP, "node merge stream: %s", hipGetErrorString(e)));
    nd->mstreams.push_back(ms);
    DevBuf b;
    b.device = device_ordinals[i];
    for (auto* v : {&nd->slice, &nd->rkeys, &nd->rcells, &nd->route, &nd->send, &nd->recv, &nd->merged})
      v->push_back(b);
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
  for (auto* v : {&node->slice, &node->rkeys, &node->rcells, &node->route, &node->send, &node->recv, &node->merged})
    for (DevBuf& b : *v) {
      (void)hipSetDevice(b.device);
      if (b.p) (void)hipFree(b.p);
    }
  for (auto& set : node->free_tables)
    for (DevBuf& b : set) {
      (void)hipSetDevice(b.device);
      if (b.p) (void)hipFree(b.p);
    }
  for (size_t i = 0; i < node->streams.size(); ++i) {
    (void)hipSetDevice(node->devices[i]);
    (void)hipStreamDestroy(node->streams[i]);
    if (i < node->mstreams.size()) (void)hipStreamDestroy(node->mstreams[i]);
  }
  for (pgpu_context* c : node->ctxs) pgpu_shutdown(c);
  delete node;
  return PGPU_OK;
}

void pgpu_slice_of(uint64_t num_keys, int32_t world, int32_t rank, uint64_t* first, uint64_t* count) {
  const uint64_t K = world > 0 ? (num_keys + (uint64_t)world - 1) / (uint64_t)world : num_keys;
  const uint64_t f = std::min<uint64_t>(num_keys, K * (uint64_t)std::max(rank, 0));
  if (first) *first = f;
  if (count) *count = std::min<uint64_t>(K, num_keys - f);
}

int32_t pgpu_key_owner(const int64_t* key_words, int32_t num_key_words, int32_t world) {
  if (!key_words || num_key_words < 1 || world < 1) return -1;
  return (int32_t)pgpu_key_owner_of(key_words, num_key_words, world);
}

int pgpu_node_query(pgpu_node* node, const pgpu_query_desc* const* descs, int64_t* out_keys, int64_t* out_cells,
                    uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats,
                    pgpu_table_layout* out_layout) {
  return pgpu_node_query_topk(node, descs, nullptr, out_keys, out_cells, capacity, out_num_groups, out_stats,
                              out_layout);
}

int pgpu_node_query_topk(pgpu_node* node, const pgpu_query_desc* const* descs, const pgpu_topk* order,
                         int64_t* out_keys, int64_t* out_cells, uint64_t capacity, uint64_t* out_num_groups,
                         pgpu_query_stats* out_stats, pgpu_table_layout* out_layout) {
  pgpu_node_pending* nq = nullptr;
  const int rc = pgpu_node_submit(node, descs, &nq);
  if (rc) return rc;
  return pgpu_node_collect(nq, order, out_keys, out_cells, capacity, out_num_groups, out_stats, out_layout);
}

int pgpu_node_submit(pgpu_node* node, const pgpu_query_desc* const* descs, pgpu_node_pending** out_query) {
  return pgpu_node_submit_expr(node, descs, nullptr, nullptr, out_query);
}

int pgpu_node_submit_expr(pgpu_node* node, const pgpu_query_desc* const* descs, const pgpu_expr_node* const* exprs,
                          const int32_t* num_nodes, pgpu_node_pending** out_query) {
  if (!node || !descs || !out_query) return nfail(PGPU_E_INVALID, "null argument");
  if (exprs && !num_nodes) return nfail(PGPU_E_INVALID, "filter expressions without their node counts");
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
  int32_t node_exp[16], node_parts[16];  // fixed-point layouts of the floating SUMs, agreed across the devices
  for (size_t i = 0; i < n; ++i) {
    qs[i].reduce_docs = std::max<int64_t>(qs[i].reduce_docs, node_docs);
    const int rc = pgpu_table_layout_of(&qs[i], &L[i]);  // also validates the descriptor
    if (rc) return rc;
    for (int a = 0; a < qs[i].num_aggs; ++a) {
      const int vt = L[i].agg_value_type[a];
      if (L[i].agg_sum_parts[a] == 3 && (vt == PGPU_INT || vt == PGPU_LONG)) extra |= PGPU_Q_SUM_SPLIT;
    }
    if (L[i].key_kind == PGPU_KEYS_HASH) extra |= PGPU_Q_HASH;
  }
  {
    const int rc = pgpu_sum_layout_agree(L.data(), (int32_t)n, qs[0].num_aggs, node_exp, node_parts);
    if (rc) return rc;
  }
  for (size_t i = 0; i < n; ++i) {
    qs[i].flags |= extra;
    qs[i].sum_exp = node_exp;
    qs[i].sum_parts = node_parts;
    const int rc = pgpu_table_layout_of(&qs[i], &L[i]);
    if (rc) return rc;
  }
  const bool hash = L[0].key_kind == PGPU_KEYS_HASH;
  for (size_t i = 1; i < n; ++i) {
    const bool same = L[i].num_sections == L[0].num_sections && L[i].key_kind == L[0].key_kind &&
                      (hash || L[i].num_keys == L[0].num_keys) &&
                      !memcmp(L[i].section_op, L[0].section_op, sizeof(L[0].section_op)) &&
                      !memcmp(L[i].agg_sum_exp, L[0].agg_sum_exp, sizeof(L[0].agg_sum_exp)) &&
                      !memcmp(L[i].agg_sum_parts, L[0].agg_sum_parts, sizeof(L[0].agg_sum_parts));
    if (!same) return nfail(PGPU_E_INVALID, "device %zu's table layout differs from device 0's", i);
  }
  auto* nq = new pgpu_node_pending();
  nq->node = node;
  nq->L = L;
  nq->num_group_columns = qs[0].num_group_columns;
  if (!node->free_tables.empty()) {
    nq->tables = std::move(node->free_tables.back());
    node->free_tables.pop_back();
  } else {
    nq->tables.resize(n);
    for (size_t i = 0; i < n; ++i) nq->tables[i].device = node->devices[i];
  }
  nq->qq.assign(n, nullptr);
  // launch every device (each query's kernels on the device's query stream; pgpu_node_collect waits for them)
  int rc = PGPU_OK;
  for (size_t i = 0; i < n && rc == PGPU_OK; ++i) {
    const uint64_t bytes = pgpu_table_bytes(&L[i]);
    const hipError_t e = nq->tables[i].ensure(bytes);
    if (e != hipSuccess) rc = nfail(PGPU_E_HIP, "node table on device %d: %s", node->devices[i], hipGetErrorString(e));
    else if (exprs && exprs[i])  // the filter planned per segment inside the library from its literals
      rc = pgpu_query_launch_expr(node->ctxs[i], &qs[i], exprs[i], num_nodes[i], node->streams[i], nq->tables[i].p,
                                  bytes, &nq->qq[i]);
    else rc = pgpu_query_launch(node->ctxs[i], &qs[i], node->streams[i], nq->tables[i].p, bytes, &nq->qq[i]);
  }
  if (rc) {
    for (pgpu_query* q : nq->qq)
      if (q) {
        (void)pgpu_query_wait(q, nullptr);
        pgpu_query_release(q);
      }
    node->free_tables.push_back(std::move(nq->tables));
    delete nq;
    return rc;
  }
  *out_query = nq;
  return PGPU_OK;
}

int pgpu_node_collect(pgpu_node_pending* nq, const pgpu_topk* order, int64_t* out_keys, int64_t* out_cells,
                      uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats,
                      pgpu_table_layout* out_layout) {
  if (!nq || !out_num_groups) return nfail(PGPU_E_INVALID, "null argument");
  if (order && order->k == 0) order = nullptr;
  pgpu_node* node = nq->node;
  std::lock_guard<std::mutex> lk(node->mu);
  const size_t n = node->devices.size();
  std::vector<pgpu_table_layout>& L = nq->L;
  const bool hash = L[0].key_kind == PGPU_KEYS_HASH;
  int rc = PGPU_OK;
  pgpu_query_stats tot{};
  tot.filter_stats_exact = 1;
  for (size_t i = 0; i < n; ++i) {
    if (!nq->qq[i]) continue;
    pgpu_query_stats st{};
    const int w = pgpu_query_wait(nq->qq[i], &st);
    if (rc == PGPU_OK && w != PGPU_OK) rc = w;
    pgpu_query_release(nq->qq[i]);
    nq->qq[i] = nullptr;
    tot.num_docs_scanned += st.num_docs_scanned;
    tot.num_entries_scanned_in_filter += st.num_entries_scanned_in_filter;
    tot.num_total_docs += st.num_total_docs;
    tot.num_segments_matched += st.num_segments_matched;  // the devices' segments are disjoint
    tot.num_groups_limit_reached |= st.num_groups_limit_reached;
    tot.sparse_sector_bytes += st.sparse_sector_bytes;
    tot.dense_bytes += st.dense_bytes;
    tot.kernel_ms = std::max(tot.kernel_ms, st.kernel_ms);
    tot.kernel_variant = std::max(tot.kernel_variant, st.kernel_variant);
    tot.filter_stats_exact &= st.filter_stats_exact;
  }
  auto done = [&](int r) {
    node->free_tables.push_back(std::move(nq->tables));
    delete nq;
    return r;
  };
  if (rc) return done(rc);
  if (out_stats) *out_stats = tot;
  if (out_layout) *out_layout = L[0];
  const int okw = L[0].key_kind == PGPU_KEYS_HASH && L[0].key_words == 2 ? 2 : 1;
  Out out{out_keys, out_cells, capacity, 0, okw, L[0].num_sections};
  std::vector<DevBuf>& tables = nq->tables;
  if (!hash) {
    const uint64_t G = L[0].num_keys;
    // PGPU_NODE_SCATTER_MIN (bytes; read per query, tests lower it to run the reduce-scatter on small tables)
    const char* sm = getenv("PGPU_NODE_SCATTER_MIN");
    const int64_t scatter_min = sm ? atoll(sm) : (int64_t)1 << 20;
    const bool scatter = nq->num_group_columns > 0 && (int64_t)(8 * G * (uint64_t)L[0].num_sections) >= scatter_min;
    if (!scatter) {
      // (one device: its table is the result -- PGPU_NODE_FORCE_RCCL=1, read per query, still reduces: tests)
      const char* fr = getenv("PGPU_NODE_FORCE_RCCL");
      if (n > 1 || (fr && atoi(fr) != 0)) rc = reduce_dense(node, tables, L[0]);
      if (rc) return done(rc);
      (void)hipSetDevice(node->devices[0]);
      rc = append_rows(node->ctxs[0], L[0], tables[0].p, node->mstreams[0], order, 0, out);
    } else {
      rc = reduce_slices(node, tables, L[0]);
      if (rc) return done(rc);
      for (size_t d = 0; d < n && rc == PGPU_OK; ++d) {  // every device trims its own slice
        uint64_t first = 0, count = 0;
        pgpu_slice_of(G, (int32_t)n, (int32_t)d, &first, &count);
        if (!count) continue;
        (void)hipSetDevice(node->devices[d]);
        hipError_t e = node->slice[d].ensure(8 * count * (size_t)L[0].num_sections + 16);
        if (e == hipSuccess)
          e = hipMemcpy2DAsync(node->slice[d].p, 8 * count, (const char*)tables[d].p + 8 * first, 8 * G, 8 * count,
                               (size_t)L[0].num_sections, hipMemcpyDeviceToDevice, node->mstreams[d]);
        if (e != hipSuccess) return done(nfail(PGPU_E_HIP, "node slice: %s", hipGetErrorString(e)));
        pgpu_table_layout Ls = L[0];
        Ls.num_keys = count;
        rc = append_rows(node->ctxs[d], Ls, node->slice[d].p, node->mstreams[d], order, (int64_t)first, out);
      }
    }
  } else {
    rc = merge_hash(node, tables, L, order, out);
  }
  if (rc) return done(rc);
  *out_num_groups = out.n;
  if (out.overflow)
    return done(nfail(PGPU_E_INVALID, "%llu result rows exceed capacity %llu", (unsigned long long)out.n,
                      (unsigned long long)capacity));
  return done(PGPU_OK);
}

}  // extern "C"
