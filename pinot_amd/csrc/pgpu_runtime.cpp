// libpinotgpu.so host runtime: the C ABI of include/pinot_gpu.h.
//
// Responsibilities (reference counterparts in parentheses):
//   * segment residency — copy each column's reference-format bytes to HBM once per segment and build the small
//     device-side directories (ImmutableSegmentLoader.load / PhysicalColumnIndexContainer reader wiring,
//     seglocal/indexsegment/immutable/ImmutableSegmentLoader.java:153-214,
//     seglocal/segment/index/column/PhysicalColumnIndexContainer.java:76-170);
//   * plan packing — turn the per-segment filter trees (already dict-id predicates, as produced by the
//     reference's PredicateEvaluators) into one flat device program with statically assigned mask slots;
//   * launch — one query kernel per query per GPU over all its segments, partial results in a dense HBM table
//     (replaces the per-segment operators + BaseCombineOperator thread pool,
//     core/operator/combine/BaseCombineOperator.java:79-227);
//   * compaction — non-empty groups back to the host (IntermediateResultsBlock payload).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pinot_gpu.h"
#include "pgpu_host.h"
#include "pgpu_internal.h"

// kernels (pgpu_kernels.hip)
hipError_t pgpu_prepare_query_kernels(size_t lds_bytes);
hipError_t pgpu_launch_table_init(const DevParams& p, hipStream_t st);
hipError_t pgpu_launch_query(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st);
hipError_t pgpu_launch_query_direct(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st);
bool pgpu_pscan_prefetch_ok(int kb, int vb);
hipError_t pgpu_launch_finalize(const DevParams& p, int nslabs, int64_t* stats_out, uint8_t* seg_out,
                                int64_t* host_table, uint64_t table_words, hipStream_t st);
hipError_t pgpu_launch_part_reduce(const DevParams& p, int nwg, hipStream_t st);
hipError_t pgpu_launch_bitslice(const uint32_t* fwd, uint32_t* out, int bits, int64_t ntiles, hipStream_t st);
hipError_t pgpu_launch_vslice(const uint32_t* fwd, const void* dict, int dict_type, int64_t vmin, int bits, int vbits,
                              uint32_t* out, int64_t ntiles, hipStream_t st);
hipError_t pgpu_launch_prologue(const DevParams& p, const void* host_arena, void* dev_arena, size_t bytes,
                                bool init_table, hipStream_t st);
hipError_t pgpu_launch_compact(const int64_t* table, uint64_t G, int32_t nsec, int32_t kw, int32_t* block_counts,
                               int64_t* total, int64_t* out_keys, int64_t* out_cells, bool count_only, hipStream_t st,
                               const uint64_t* okey = nullptr, const TopkState* ts = nullptr);
hipError_t pgpu_launch_topk(const int64_t* table, const TopkDev& s, uint64_t k, uint64_t* okey, TopkState* ts,
                            uint32_t* hist, hipStream_t st);
hipError_t pgpu_launch_segcount(const DevParams& p, int64_t* out, hipStream_t st);
hipError_t pgpu_launch_progbits(const DevParams& p, const ProgJob* jobs, int njobs, int total, hipStream_t st);
hipError_t pgpu_launch_andfsm(const DevParams& p, bool s2, uint32_t* fn, int64_t* out, hipStream_t st);
hipError_t pgpu_launch_leafbits(const DevParams& p, hipStream_t st);
hipError_t pgpu_launch_part_scan(const DevParams& p, int grid, size_t dyn_smem, hipStream_t st);
hipError_t pgpu_launch_rawpred(const RawLeaf* dev_leaves, int nleaves, int64_t max_words, hipStream_t st);
hipError_t pgpu_launch_mvpred(const MvLeaf* dev_leaves, int nleaves, int64_t max_words, hipStream_t st);
hipError_t pgpu_launch_invexp(const InvLeafX* dev_leaves, int nleaves, int64_t max_words, hipStream_t st);
hipError_t pgpu_launch_rkey_ctab(const InvLeafX* dev_leaves, int nleaves, int64_t max_pairs, DevContainer* out,
                                 hipStream_t st);
// on-the-fly group dictionaries of raw columns (pgpu_gdict.hip)
size_t pgpu_gdict_temp_bytes(int64_t n);
hipError_t pgpu_gdict_sort_unique(const void* vals, int32_t dtype, int64_t n, uint64_t* keys, uint64_t* sorted,
                                  uint64_t* uniq, uint32_t* d_card, void* temp, size_t temp_bytes, hipStream_t st);
hipError_t pgpu_gdict_encode(const uint64_t* keys, int64_t n, const uint64_t* uniq, int32_t card, int32_t dtype,
                             int bits, void* dict, uint32_t* ids, uint32_t* words, int64_t nwords, hipStream_t st);

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess) return fail(PGPU_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
inline uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
inline uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

int type_width(int32_t t) { return (t == PGPU_INT || t == PGPU_FLOAT) ? 4 : 8; }
// Running max |value| of a column (HostColumn::max_abs); a NaN or infinity makes it +inf (no fixed-point SUM).
inline double abs_bound(double m, double v) { return std::isfinite(v) ? std::max(m, std::fabs(v)) : INFINITY; }
// Magnitudes of a column's values: max |value| (integer SUM bound, fixed-point top), and for FLOAT / DOUBLE the
// smallest nonzero |value|'s binary exponent and the lowest set mantissa bit's exponent over all nonzero values --
// what the fixed-point floating SUM needs to be exact or within its per-value tolerance (pgpu_table_layout_of).
struct ValueRange {
  double max_abs = 0;
  int32_t min_exp = INT32_MAX;  // min ilogb(|v|) over nonzero values
  int32_t min_lsb = INT32_MAX;  // min exponent of the lowest set bit of v's significand over nonzero values
  void add_fp(double v) {
    max_abs = abs_bound(max_abs, v);
    if (v == 0 || !std::isfinite(v)) return;
    uint64_t b;
    memcpy(&b, &v, 8);
    const int be = (int)((b >> 52) & 0x7ff);
    const uint64_t m = be ? ((b & ((1ull << 52) - 1)) | (1ull << 52)) : (b & ((1ull << 52) - 1));
    min_exp = std::min(min_exp, (int32_t)std::ilogb(v));
    min_lsb = std::min(min_lsb, (int32_t)((be ? be : 1) - 1075 + __builtin_ctzll(m)));
  }
  void merge(const ValueRange& o) {
    max_abs = abs_bound(max_abs, o.max_abs);
    min_exp = std::min(min_exp, o.min_exp);
    min_lsb = std::min(min_lsb, o.min_lsb);
  }
};
// ValueRange of n little-endian values of type t
ValueRange value_range_of(const uint8_t* le, size_t n, int32_t t) {
  ValueRange r;
  for (size_t i = 0; i < n; ++i) {
    if (t == PGPU_INT) { int32_t x; memcpy(&x, le + 4 * i, 4); r.max_abs = std::max(r.max_abs, std::fabs((double)x)); }
    else if (t == PGPU_LONG) { int64_t x; memcpy(&x, le + 8 * i, 8); r.max_abs = std::max(r.max_abs, std::fabs((double)x)); }
    else if (t == PGPU_FLOAT) { float x; memcpy(&x, le + 4 * i, 4); r.add_fp(x); }
    else { double x; memcpy(&x, le + 8 * i, 8); r.add_fp(x); }
  }
  return r;
}

// PGPU_PROFILE=1: the query kernel records per-wave phase cycles; pgpu_query_wait prints their averages.
bool profile_enabled() {
#ifdef PGPU_PROFILE_BUILD
  static const bool on = [] {
    const char* e = getenv("PGPU_PROFILE");
    return e && e[0] == '1';
  }();
  return on;
#else
  return false;  // phase counters exist only in libpinotgpu_prof.so
#endif
}

// Device buffer that frees itself.
struct DevMem {
  void* p = nullptr;
  size_t n = 0;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  DevMem(DevMem&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  DevMem& operator=(DevMem&& o) noexcept {
    if (this != &o) {
      reset();
      p = o.p;
      n = o.n;
      o.p = nullptr;
      o.n = 0;
    }
    return *this;
  }
  ~DevMem() { reset(); }
  void reset() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  hipError_t alloc(size_t bytes) {
    reset();
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) n = bytes;
    else p = nullptr;
    return e;
  }
  hipError_t ensure(size_t bytes) { return n >= bytes ? hipSuccess : alloc(std::max(bytes, n * 3 / 2)); }
  // Query-path growth: stream-ordered, from the context's memory pool.  hipFree waits for the whole device --
  // every other query in flight -- so a workspace that grows inside pgpu_query_submit must never call it: the old
  // block goes back to the pool behind the work already queued on `s` and the new one is carved out in stream
  // order (the pool keeps its memory reserved, so steady-state growth costs nothing).
  hipError_t ensure(size_t bytes, hipMemPool_t pool, hipStream_t s) {
    if (n >= bytes) return hipSuccess;
    if (!pool) return ensure(bytes);
    size_t nb = std::max(bytes, n * 3 / 2);
    if (nb == 0) nb = 16;
    if (p) {
      const hipError_t e = hipFreeAsync(p, s);
      if (e != hipSuccess) return e;
      p = nullptr;
      n = 0;
    }
    void* q = nullptr;
    const hipError_t e = hipMallocFromPoolAsync(&q, nb, pool, s);
    if (e != hipSuccess) return e;
    p = q;
    n = nb;
    return hipSuccess;
  }
};

struct PinnedMem {
  void* p = nullptr;
  size_t n = 0;
  PinnedMem() = default;
  PinnedMem(const PinnedMem&) = delete;
  PinnedMem& operator=(const PinnedMem&) = delete;
  ~PinnedMem() { reset(); }
  void reset() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    dev = nullptr;
    n = 0;
  }
  hipError_t ensure(size_t bytes) {
    if (n >= bytes) return hipSuccess;
    reset();
    bytes = std::max(bytes, (size_t)4096);
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) n = bytes;
    else p = nullptr;
    return e;
  }
  // the buffer's device address (looked up once per allocation: a runtime call per query otherwise)
  hipError_t device_ptr(void** out) {
    if (!dev) {
      const hipError_t e = hipHostGetDevicePointer(&dev, p, 0);
      if (e != hipSuccess) {
        dev = nullptr;
        return e;
      }
    }
    *out = dev;
    return hipSuccess;
  }
  void* dev = nullptr;
};

// PGPU_HOST_TIMING=N: average host microseconds of the submit phases, printed to stderr every N submits
struct HostTiming {
  int every = 0, n = 0;
  double acc[6] = {0, 0, 0, 0, 0, 0};
  HostTiming() {
    const char* e = getenv("PGPU_HOST_TIMING");
    every = e ? atoi(e) : 0;
  }
  static double us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void add(int k, double t0, double t1) {
    if (every > 0) acc[k] += t1 - t0;
  }
  void done() {
    if (every <= 0 || ++n < every) return;
    fprintf(stderr, "[pgpu host] per submit (us): expr %.1f layout %.1f pack %.1f workspace %.1f launch %.1f total %.1f\n",
            acc[0] / n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n);
    n = 0;
    for (double& a : acc) a = 0;
  }
};
HostTiming& host_timing() {
  static HostTiming t;
  return t;
}

// System.currentTimeMillis (QueryContext end times are on this clock)
int64_t now_epoch_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

struct Workspace {
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
  DevMem arena, slab, stats, stats_out, table, cmp_counts, cmp_total, cmp_keys, cmp_cells, prof, recs, rcount;
  DevMem pcount, pcap, poff, p2work;   // PART region sizing / phase-2 plan (part_plan_kernel)
  DevMem segmask, hflag;               // HASH mode: distinct-key bitmaps of tracked segments, probe-overflow flag
  DevMem leafbits;                     // PGPU_Q_EXACT_FILTER_STATS: per-leaf match bits of every segment
  DevMem segany;                       // per-segment matched words (DevParams::segany), zero between queries
  DevMem fsmfn;                        // exact filter stats on the GPU: per-tile transducer maps (andfsm kernels)
  DevMem rawbits;                      // match bitmaps of the raw-value leaves (rawpred_kernel)
  DevMem rkctab;                       // query_kernel_rkey: container record per (leaf, id, key)
  DevMem tk_keys, tk_state;            // pgpu_table_topk: per-row order keys, radix-select state + histogram
  PinnedMem h_arena, h_stats, h_total, h_table, h_segcnt, h_leafbits, h_segany, h_fsment;
  DevMem d_cancel;                     // cancel word (DevParams::cancel): = the query's generation -> stop
  PinnedMem h_cancel;                  // its source for pgpu_query_cancel's copy-engine write
  uint32_t cancel_gen = 0;
  bool busy = false;
  ~Workspace() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

}  // namespace

struct pgpu_context {
  int device = 0;
  int num_cus = 256;
  std::mutex mu;
  std::vector<std::unique_ptr<Workspace>> pool;
  bool lds_ready = false;  // query kernels allowed the full 160 KiB of dynamic LDS
  // pgpu_query_submit: all submitted queries run back to back on one stream (each kernel fills the GPU, so
  // nothing is lost by serialising them, and their HIP events then time each kernel alone)
  hipStream_t qstream = nullptr;
  hipStream_t cstream = nullptr;  // pgpu_query_cancel: writes cancel words while the query stream is busy
  // workspace buffers grow from this pool in stream order (DevMem::ensure(bytes, pool, stream)); it never returns
  // memory to the device on its own (release threshold = max), so no query-path allocation reaches the driver
  // twice.  nullptr when the device has no memory pools: growth then falls back to hipMalloc / hipFree.
  hipMemPool_t mpool = nullptr;
  // HBM held by derived copies (bit-sliced forward indexes, value planes) of this context's segments, and the budget
  // they are built under (pgpu_context_set_derived_budget; default half of the device's memory)
  std::atomic<uint64_t> derived_bytes{0};
  // (atomic: a budget set from one thread may meet another thread's seal; a new budget governs later seals only --
  // copies already built are kept until their segment is released)
  std::atomic<uint64_t> derived_budget{UINT64_MAX};
  ~pgpu_context() {
    pool.clear();
    if (qstream) (void)hipStreamDestroy(qstream);
    if (cstream) (void)hipStreamDestroy(cstream);
    if (mpool) {
      (void)hipDeviceSynchronize();
      (void)hipMemPoolDestroy(mpool);
    }
  }
};

struct pgpu_buffer {
  pgpu_context* ctx;
  DevMem mem;
  int32_t length;
};

namespace {

struct HostColumn {
  int32_t kind = PGPU_COL_NONE;
  int32_t bits = 0;
  int32_t card = 0;
  int32_t fwd_card = 0;
  int32_t dict_type = -1;
  int32_t dict_card = 0;
  int32_t inv_card = 0;
  DevMem fwd, sorted, dict, inv_dir, inv_ct, inv_data;
  DevMem sliced;                       // bit-sliced copy of fwd (built at seal; PGPU_NO_SLICE=1 skips it)
  DevMem vsliced;                      // bit planes of the docs' values - vmin (INT / LONG dictionaries, <= 32 bits;
                                       // built at seal; PGPU_NO_VSLICE=1 skips it)
  int64_t vmin = 0;
  int32_t vbits = 0;
  uint64_t fwd_bytes = 0, dict_bytes = 0, inv_bytes = 0;
  std::vector<uint32_t> inv_cards;     // docs per dict id of the inverted index (selectivity estimates)
  std::vector<uint32_t> inv_hdir;      // its container directory (first container of each dict id, then the total):
                                       // query_kernel_cand's unit list is built on the host
  std::vector<int32_t> sorted_pairs;   // sorted index (start, end) per dict id (selectivity estimates)
  std::vector<uint8_t> hdict;          // numeric dictionary, little-endian (per-segment predicate planning)
  double max_abs = 0;                  // numeric dictionary (or raw values): largest |value| (integer SUM bound)
  int32_t derive = PGPU_DERIVE_ALL;    // derived copies seal may build (pgpu_segment_set_derived)
  int32_t min_exp = INT32_MAX;         // FLOAT / DOUBLE: ValueRange::min_exp / min_lsb (fixed-point SUM layout)
  int32_t min_lsb = INT32_MAX;
  void set_range(const ValueRange& r) {
    max_abs = r.max_abs;
    min_exp = r.min_exp;
    min_lsb = r.min_lsb;
  }
  int32_t range_index = 0;             // range index version (2 = exact bit-sliced, 1 = legacy), 0 = none
  uint64_t dict_hash[2] = {0, 0};      // two independent 64-bit hashes of the dictionary bytes (shared-dict checks)
  // INT dictionary in frame-of-reference form (phase 2 of the partitioned group-by keeps it in LDS): per block of
  // 32 ids its first value, then every id's offset from it in for_bits bits (0 = not encoded)
  DevMem for_dev;
  int32_t for_bits = 0, for_nblk = 0;
  // multi-value column (PGPU_COL_MV): fwd = the values' ids fixed-bit, mv_off = row offsets (num_docs + 1)
  DevMem mv_off;
  std::vector<int32_t> mv_offsets;     // host copy (row lengths: exact filter statistics, row columns)
  std::vector<uint8_t> mv_raw;         // host copy of the packed ids until seal (row columns)
  int64_t mv_values = 0;
};

}  // namespace

struct pgpu_segment {
  pgpu_context* ctx;
  int32_t num_docs;
  std::vector<HostColumn> cols;
  std::vector<DevColumn> dev;
  bool sealed = false;
};

struct pgpu_query {
  pgpu_context* ctx;
  Workspace* ws;
  hipStream_t stream;
  DevParams params;
  int grid;
  pgpu_query_stats stats;
  // pgpu_query_submit: the workspace owning the partial table, its layout, and whether it was copied back whole
  Workspace* tws = nullptr;
  pgpu_table_layout layout{};
  bool small = false;
  bool eager = false;  // compacted on the device at submit (enqueue_compact): collect only copies the rows out
  bool eager_ordered = false;  // ... restricted to the best groups by the order given at submit
  // HASH mode: tracked segments (query segment index) whose distinct keys are checked against the limit
  std::vector<int32_t> tracked;
  std::vector<uint8_t> tracked_map;  // per tracked segment: its holder is map-based (keys past the limit dropped)
  int64_t groups_limit = 0;
  // PGPU_Q_EXACT_FILTER_STATS: each segment's program (ids copied) and where its leaf bitmaps are
  struct FilterReplay {
    std::vector<pgpu_filter_node> nodes;
    std::vector<std::vector<int32_t>> ids;
    int32_t num_docs = 0, num_leaves = 0, ntiles = 0;
    int64_t bits_off = 0;
    std::vector<const int32_t*> leaf_off;  // per leaf: row offsets of a multi-value SCAN leaf, else null
  };
  uint8_t* matched_out = nullptr;  // pgpu_query_matched_segments: caller's per-segment flags, filled by the wait
  int64_t mv_entries = 0;  // entries of multi-value SCAN leaves that are a segment's whole filter (kernel: nostat)
  std::vector<FilterReplay> replay;
  bool exact_filter = false;
  bool exact_fsm = false;  // the reference's count per segment from the andfsm kernels (pinned h_fsment)
  hipEvent_t done = nullptr;  // submitted queries: recorded after the last copy of this query
  // deadline (ms since the epoch, 0 = none) and why the query was stopped (0 = it was not)
  int64_t deadline_ms = 0;
  std::atomic<int> stop{0};  // PGPU_E_CANCELLED / PGPU_E_TIMEOUT
};

namespace {

Workspace* acquire_ws(pgpu_context* ctx, int* err) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  for (auto& w : ctx->pool)
    if (!w->busy) {
      w->busy = true;
      return w.get();
    }
  std::unique_ptr<Workspace> w(new Workspace());
  hipError_t e = hipSetDevice(ctx->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreate(&w->ev0);
  if (e == hipSuccess) e = hipEventCreate(&w->ev1);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&w->done, hipEventDisableTiming);
  if (e != hipSuccess) {
    *err = fail(PGPU_E_HIP, "workspace creation failed: %s", hipGetErrorString(e));
    return nullptr;
  }
  w->busy = true;
  ctx->pool.push_back(std::move(w));
  return ctx->pool.back().get();
}

void release_ws(pgpu_context* ctx, Workspace* w) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  w->busy = false;
}

// Roaring portable format: pgpu_roaring.cpp (pgpu_parse_roaring)
int parse_roaring(const uint8_t* p, size_t n, std::vector<PgpuRoaringContainer>* out) {
  std::string err;
  const int rc = pgpu_parse_roaring(p, n, out, &err);
  return rc ? fail(rc, "%s", err.c_str()) : PGPU_OK;
}
using ParsedContainer = PgpuRoaringContainer;
static_assert(PGPU_CT_ARRAY == 0 && PGPU_CT_BITMAP == 1 && PGPU_CT_RUN == 2, "pgpu_parse_roaring container types");

int check_column(pgpu_segment* seg, int32_t column) {
  if (!seg) return fail(PGPU_E_INVALID, "null segment");
  if (seg->sealed) return fail(PGPU_E_INVALID, "segment already sealed");
  if (column < 0 || column >= (int32_t)seg->cols.size()) return fail(PGPU_E_INVALID, "bad column %d", column);
  return PGPU_OK;
}

// Two independent 64-bit hashes of a little-endian dictionary (shared-dictionary checks).
void dictionary_hash(const std::vector<uint8_t>& le, uint64_t* out) {
  uint64_t h1 = 1469598103934665603ull, h2 = 0x9E3779B97F4A7C15ull;  // FNV-1a, and a multiply-xorshift mix
  for (uint8_t x : le) {
    h1 = (h1 ^ x) * 1099511628211ull;
    h2 = (h2 + x + 1) * 0xBF58476D1CE4E5B9ull;
    h2 ^= h2 >> 29;
  }
  out[0] = h1;
  out[1] = h2;
}

hipError_t upload(DevMem& m, const void* src, size_t bytes, size_t alloc_bytes, int mem_kind) {
  hipError_t e = m.alloc(alloc_bytes);
  if (e != hipSuccess) return e;
  if (alloc_bytes > bytes) e = hipMemset((char*)m.p + bytes, 0, alloc_bytes - bytes);
  if (e != hipSuccess) return e;
  if (bytes)
    e = hipMemcpy(m.p, src, bytes, mem_kind == PGPU_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice);
  return e;
}

// Local cardinality product of the group columns in segment plan `sp` (saturating at 2^126).
unsigned __int128 local_key_space(const pgpu_query_desc* q, const pgpu_segment_plan& sp) {
  unsigned __int128 P = 1;
  for (int g = 0; g < q->num_group_columns; ++g) {
    const int32_t slot = sp.column_map ? sp.column_map[q->group_columns[g]] : -1;
    const pgpu_segment* sg = sp.segment;
    const int32_t card = (sg && slot >= 0 && slot < (int32_t)sg->cols.size()) ? std::max(1, sg->cols[slot].card) : 1;
    P *= (unsigned __int128)card;
    if (P > ((unsigned __int128)1 << 126)) P = (unsigned __int128)1 << 126;
  }
  return P;
}

// DictionaryBasedGroupKeyGenerator's holder choice for one segment (DictionaryBasedGroupKeyGenerator.java:137-164):
// a map-based holder (product above the array threshold) stops at num_groups_limit distinct keys, so such a
// segment whose product also exceeds the limit must have its distinct keys counted.
// PGPU_Q_EXACT_FILTER_STATS on the GPU (andfsm kernels, pgpu_kernels.hip): the segment's filter is match-all,
// empty, one SCAN leaf or one AND of 2..4 SCAN / RAW_SCAN leaves over single-value columns -- the reference then
// scans every doc (a lone leaf) or leap-frogs AndDocIdIterator over the scan iterators (AndDocIdSet.java:140-143).
bool fsm_filter(const pgpu_segment_plan& sp) {
  const int n = sp.num_filter_nodes;
  const pgpu_filter_node* f = sp.filter;
  if (n == 0) return true;
  auto scan_leaf = [&](const pgpu_filter_node& nd) {
    if (nd.op == PGPU_F_RAW_SCAN) return true;
    if (nd.op != PGPU_F_SCAN || !sp.column_map) return false;
    const int32_t slot = sp.column_map[nd.column];
    return slot >= 0 && slot < (int32_t)sp.segment->cols.size() && sp.segment->cols[slot].kind != PGPU_COL_MV;
  };
  if (n == 1) return f[0].op == PGPU_F_MATCH_ALL || f[0].op == PGPU_F_EMPTY || scan_leaf(f[0]);
  if (f[0].op != PGPU_F_AND_BEGIN || f[n - 1].op != PGPU_F_AND_END || (n - 2) % 2 != 0) return false;
  const int k = (n - 2) / 2;
  if (k < 2 || k > 4) return false;
  for (int i = 1; i + 1 < n; i += 2)
    if (!scan_leaf(f[i]) || f[i + 1].op != PGPU_F_AND_CHILD_END) return false;
  return true;
}

// numGroupsLimit: a segment's distinct group keys are counted on the GPU when they can reach the limit -- for the
// numGroupsLimitReached flag (AggregationGroupByOrderByOperator.java:111: numGroups >= numGroupsLimit) and, when
// its holder is map-based (key space above the array-based threshold, DictionaryBasedGroupKeyGenerator.java:137-164),
// for the first-seen cut of the keys past the limit (PGPU_E_GROUPS_LIMIT).
bool segment_needs_count(const pgpu_query_desc* q, const pgpu_segment_plan& sp) {
  if (q->num_group_columns == 0 || q->num_groups_limit <= 0) return false;
  return local_key_space(q, sp) >= (unsigned __int128)q->num_groups_limit;
}
bool segment_map_based(const pgpu_query_desc* q, const pgpu_segment_plan& sp) {
  return local_key_space(q, sp) > (unsigned __int128)std::max(0, q->array_based_threshold);
}

// Table shape of the group keys: dense (cell = mixed-radix key) or hash slots (key words stored per slot).
int group_key_space(const pgpu_query_desc* q, pgpu_table_layout* out) {
  out->key_kind = PGPU_KEYS_DENSE;
  out->key_words = 1;
  out->key_split = q->num_group_columns;
  out->num_keys = 1;
  if (q->num_group_columns == 0) return PGPU_OK;
  unsigned __int128 G = 1;
  const unsigned __int128 cap126 = (unsigned __int128)1 << 126;
  for (int i = 0; i < q->num_group_columns; ++i) {
    const int32_t c = q->group_cardinalities ? q->group_cardinalities[i] : 0;
    if (c < 1) return fail(PGPU_E_INVALID, "group column %d cardinality %d", i, c);
    G *= (unsigned __int128)c;
    if (G > cap126) G = cap126;
  }
  // distinct keys the launch can meet: per segment its local key space, bounded by the holder limit (a segment
  // beyond it fails the query anyway) and by its docs
  double est = 0;
  bool track = false;
  for (int s = 0; s < q->num_segments; ++s) {
    const pgpu_segment_plan& sp = q->segments[s];
    const double P = (double)local_key_space(q, sp);
    double b = P;
    if (q->num_groups_limit > 0 && P > (double)std::max(0, q->array_based_threshold)) b = std::min(P, (double)q->num_groups_limit);
    b = std::min(b, (double)(sp.segment ? sp.segment->num_docs : 0));
    est += b;
    track |= segment_needs_count(q, sp);
  }
  est = std::min(est, (double)G);
  const bool hash = (q->flags & PGPU_Q_HASH) || track || G > ((unsigned __int128)1 << 31) ||
                    ((double)G >= 65536.0 && (double)G > 8.0 * est);
  if (!hash) {
    out->num_keys = (uint64_t)G;
    return PGPU_OK;
  }
  uint64_t slots = 64;
  while ((double)slots < 2.0 * est) slots <<= 1;
  if (slots > (1ull << 31)) return fail(PGPU_E_UNSUPPORTED, "hash group-by table of %llu slots", (unsigned long long)slots);
  out->key_kind = PGPU_KEYS_HASH;
  out->num_keys = slots;
  if (G < ((unsigned __int128)1 << 63)) return PGPU_OK;
  // above 2^63 keys (the reference's ArrayMapBasedHolder): word 0 = the longest prefix of columns below 2^63,
  // word 1 = the rest, which must stay below 2^32 (the second level packs (interned word-0 slot << 32 | word 1))
  unsigned __int128 pre = 1;
  int split = 0;
  while (split < q->num_group_columns && pre * (unsigned __int128)q->group_cardinalities[split] < ((unsigned __int128)1 << 63))
    pre *= (unsigned __int128)q->group_cardinalities[split++];
  unsigned __int128 rest = 1;
  for (int i = split; i < q->num_group_columns; ++i) rest *= (unsigned __int128)q->group_cardinalities[i];
  if (split == 0 || rest >= ((unsigned __int128)1 << 32))
    return fail(PGPU_E_UNSUPPORTED, "group key of more than 95 bits");
  out->key_words = 2;
  out->key_split = split;
  return PGPU_OK;
}

}  // namespace

// =============================================================================================================
// pgpu_node.cpp's access to the thread's error message and to segment sizes
int pgpu_set_error(int code, const char* msg) { return fail(code, "%s", msg); }
int64_t pgpu_desc_docs(const pgpu_query_desc* q) {
  int64_t d = 0;
  for (int s = 0; q && s < q->num_segments; ++s)
    if (q->segments[s].segment) d += q->segments[s].segment->num_docs;
  return d;
}

extern "C" {

int pgpu_abi_version(void) { return PGPU_ABI_VERSION; }

uint64_t pgpu_table_bytes(const pgpu_table_layout* L) {
  if (!L) return 0;
  const uint64_t words = (uint64_t)L->num_sections + (L->key_kind == PGPU_KEYS_HASH ? (uint64_t)L->key_words : 0);
  return 8ull * words * L->num_keys;
}

int pgpu_last_error(char* buf, size_t len) {
  if (buf && len) {
    size_t k = std::min(len - 1, g_last_error.size());
    memcpy(buf, g_last_error.data(), k);
    buf[k] = 0;
  }
  return (int)g_last_error.size();
}

int pgpu_init(int device_ordinal, pgpu_context** out_ctx) {
  if (!out_ctx) return fail(PGPU_E_INVALID, "null out_ctx");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device_ordinal < 0 || device_ordinal >= n)
    return fail(PGPU_E_INVALID, "device %d out of range (%d devices)", device_ordinal, n);
  HIP_TRY(hipSetDevice(device_ordinal));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device_ordinal));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(PGPU_E_UNSUPPORTED, "libpinotgpu is built for gfx950 (MI355X); device is %s", prop.gcnArchName);
  auto* ctx = new pgpu_context();
  ctx->device = device_ordinal;
  ctx->num_cus = prop.multiProcessorCount;
  {  // derived copies may take up to half of the device's memory unless the server says otherwise
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) ctx->derived_budget = tot / 2;
  }
  int pools = 0;
  if (hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, device_ordinal) == hipSuccess && pools) {
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device_ordinal;
    if (hipMemPoolCreate(&ctx->mpool, &props) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      if (hipMemPoolSetAttribute(ctx->mpool, hipMemPoolAttrReleaseThreshold, &keep) != hipSuccess) {
        (void)hipMemPoolDestroy(ctx->mpool);
        ctx->mpool = nullptr;
      }
    } else {
      ctx->mpool = nullptr;
    }
  }
  *out_ctx = ctx;
  return PGPU_OK;
}

int pgpu_shutdown(pgpu_context* ctx) {
  if (!ctx) return PGPU_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipDeviceSynchronize();
  delete ctx;
  return PGPU_OK;
}

int pgpu_segment_create(pgpu_context* ctx, int32_t num_docs, int32_t num_columns, pgpu_segment** out_seg) {
  if (!ctx || !out_seg) return fail(PGPU_E_INVALID, "null argument");
  if (num_docs < 0 || num_columns < 0 || num_columns > 4096)
    return fail(PGPU_E_INVALID, "bad segment shape (%d docs, %d columns)", num_docs, num_columns);
  auto* s = new pgpu_segment();
  s->ctx = ctx;
  s->num_docs = num_docs;
  s->cols.resize(num_columns);
  *out_seg = s;
  return PGPU_OK;
}

int pgpu_segment_add_forward_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                   int32_t bits_per_value, int32_t cardinality, int32_t mem_kind) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  if (bits_per_value < 1 || bits_per_value > 31) return fail(PGPU_E_INVALID, "bits_per_value %d", bits_per_value);
  const uint64_t need = ((uint64_t)seg->num_docs * bits_per_value + 7) / 8;
  if (num_bytes < need || (!bytes && need))
    return fail(PGPU_E_INVALID, "forward index of column %d: %llu bytes < %llu needed", column,
                (unsigned long long)num_bytes, (unsigned long long)need);
  HostColumn& c = seg->cols[column];
  if (c.kind == PGPU_COL_SORTED || c.kind == PGPU_COL_RAW)
    return fail(PGPU_E_INVALID, "column %d already has a forward index", column);
  const uint64_t ntiles = ((uint64_t)seg->num_docs + PGPU_TILE - 1) / PGPU_TILE;
  const uint64_t alloc = std::max<uint64_t>(ntiles * PGPU_TILE / 8 * bits_per_value, need) + 16;
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.fwd, bytes, need, alloc, mem_kind));
  c.kind = PGPU_COL_FIXED_BIT;
  c.bits = bits_per_value;
  c.fwd_card = cardinality;
  c.fwd_bytes = need;
  return PGPU_OK;
}

int pgpu_segment_add_sorted_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                  int32_t cardinality) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  if (cardinality < 1 || num_bytes != 8ull * cardinality || !bytes)
    return fail(PGPU_E_INVALID, "sorted index of column %d: %llu bytes for cardinality %d", column,
                (unsigned long long)num_bytes, cardinality);
  HostColumn& c = seg->cols[column];
  if (c.kind == PGPU_COL_FIXED_BIT) return fail(PGPU_E_INVALID, "column %d already has a forward index", column);
  std::vector<int32_t> pairs(2 * (size_t)cardinality);
  const uint8_t* b = (const uint8_t*)bytes;
  int32_t prev_end = -1;
  for (int32_t i = 0; i < cardinality; ++i) {
    pairs[2 * i] = (int32_t)be32(b + 8 * i);
    pairs[2 * i + 1] = (int32_t)be32(b + 8 * i + 4);
    if (pairs[2 * i] != prev_end + 1 || pairs[2 * i + 1] < pairs[2 * i] - 1)
      return fail(PGPU_E_INVALID, "sorted index of column %d: ranges not contiguous at dict id %d", column, i);
    prev_end = pairs[2 * i + 1];
  }
  if (prev_end != seg->num_docs - 1)
    return fail(PGPU_E_INVALID, "sorted index of column %d ends at %d, numDocs %d", column, prev_end, seg->num_docs);
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.sorted, pairs.data(), pairs.size() * 4, pairs.size() * 4, PGPU_MEM_HOST));
  c.sorted_pairs.swap(pairs);
  c.kind = PGPU_COL_SORTED;
  c.fwd_card = cardinality;
  c.fwd_bytes = num_bytes;
  return PGPU_OK;
}

int pgpu_segment_add_dictionary(pgpu_segment* seg, int32_t column, int32_t data_type, const void* bytes,
                                uint64_t num_bytes, int32_t cardinality) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  if (data_type < PGPU_INT || data_type > PGPU_STRING || cardinality < 1)
    return fail(PGPU_E_INVALID, "dictionary of column %d: bad type %d / cardinality %d", column, data_type,
                cardinality);
  HostColumn& c = seg->cols[column];
  if (c.kind == PGPU_COL_RAW) return fail(PGPU_E_INVALID, "column %d is a raw (no-dictionary) column", column);
  c.dict_type = data_type;
  c.dict_card = cardinality;
  if (data_type == PGPU_STRING) return PGPU_OK;
  const int w = type_width(data_type);
  if (!bytes || num_bytes != (uint64_t)w * cardinality)
    return fail(PGPU_E_INVALID, "dictionary of column %d: %llu bytes, expected %llu", column,
                (unsigned long long)num_bytes, (unsigned long long)w * cardinality);
  std::vector<uint8_t> le(num_bytes);
  const uint8_t* b = (const uint8_t*)bytes;
  // Pinot dictionaries are sorted ascending (SegmentDictionaryCreator.java:92-156; BaseImmutableDictionary's
  // binary searches rely on it), and so do the kernels' MIN / MAX-on-dict-id reductions: an unsorted numeric
  // dictionary is malformed input.  Floating values compare by their order-preserving bit key (-0.0 < 0.0, as
  // Float.compare / Double.compare order them).
  auto order_key = [&](int32_t i) -> int64_t {
    if (data_type == PGPU_INT) return (int64_t)(int32_t)be32(b + 4 * i);
    if (data_type == PGPU_LONG) return (int64_t)be64(b + 8 * (size_t)i);
    int64_t k = data_type == PGPU_FLOAT ? (int64_t)(int32_t)be32(b + 4 * i) : (int64_t)be64(b + 8 * (size_t)i);
    if (data_type == PGPU_FLOAT) {  // widen the float bits' order to the int64 key space
      const int32_t f = (int32_t)k;
      return f >= 0 ? (int64_t)f : (int64_t)(f ^ 0x7FFFFFFF);
    }
    return k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFll);
  };
  int64_t prev = 0;
  for (int32_t i = 0; i < cardinality; ++i) {
    const int64_t k = order_key(i);
    if (i > 0 && k <= prev)
      return fail(PGPU_E_INVALID, "dictionary of column %d is not sorted ascending at id %d", column, i);
    prev = k;
    if (w == 4) {
      uint32_t v = be32(b + 4 * i);
      memcpy(&le[4 * i], &v, 4);
    } else {
      uint64_t v = be64(b + 8 * i);
      memcpy(&le[8 * (size_t)i], &v, 8);
    }
  }
  const ValueRange vr = value_range_of(le.data(), (size_t)cardinality, data_type);
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.dict, le.data(), le.size(), le.size(), PGPU_MEM_HOST));
  c.dict_bytes = num_bytes;
  if (data_type == PGPU_INT && cardinality >= 2048) {
    // frame of reference: sorted values differ little within a block of 32 ids
    const int32_t nblk = (cardinality + 31) / 32;
    int bits = 0;
    for (int32_t k = 0; k < nblk; ++k) {
      const int32_t first = (int32_t)be32(b + 4 * (32 * k));
      const int32_t last = (int32_t)be32(b + 4 * std::min(cardinality - 1, 32 * k + 31));
      const uint64_t span = (uint64_t)((int64_t)last - first);
      int w = 0;
      while (w < 33 && (span >> w)) ++w;
      bits = std::max(bits, w);
    }
    if (bits >= 1 && bits <= PGPU_FOR_MAX_BITS) {
      std::vector<uint32_t> img((size_t)nblk * (1 + bits) + 1, 0u);
      for (int32_t k = 0; k < nblk; ++k) img[k] = be32(b + 4 * (32 * k));
      uint32_t* words = img.data() + nblk;
      for (int32_t id = 0; id < cardinality; ++id) {
        const int32_t blk = id >> 5;
        const uint32_t off = (uint32_t)((int64_t)(int32_t)be32(b + 4 * id) - (int64_t)(int32_t)img[blk]);
        const uint32_t bit = (uint32_t)(id & 31) * bits;
        const size_t w = (size_t)blk * bits + (bit >> 5);
        words[w] |= off << (bit & 31);
        if ((bit & 31) + bits > 32) words[w + 1] |= off >> (32 - (bit & 31));
      }
      HIP_TRY(upload(c.for_dev, img.data(), img.size() * 4, img.size() * 4, PGPU_MEM_HOST));
      c.for_bits = bits;
      c.for_nblk = nblk;
    }
  }
  dictionary_hash(le, c.dict_hash);
  c.hdict = std::move(le);
  c.set_range(vr);
  return PGPU_OK;
}

int pgpu_segment_add_raw_forward_index(pgpu_segment* seg, int32_t column, int32_t data_type, const void* bytes,
                                       uint64_t num_bytes) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  if (data_type < PGPU_INT || data_type > PGPU_DOUBLE)
    return fail(PGPU_E_UNSUPPORTED, "raw forward index of column %d: type %d is not fixed-width numeric", column, data_type);
  HostColumn& c = seg->cols[column];
  if (c.kind != PGPU_COL_NONE || c.dict_card)
    return fail(PGPU_E_INVALID, "column %d already has a forward index or dictionary", column);
  if (!bytes) return fail(PGPU_E_INVALID, "null raw forward index");
  const int w = type_width(data_type);
  std::vector<uint8_t> le;
  std::string err;
  rc = pgpu_decode_raw_forward((const uint8_t*)bytes, num_bytes, w, seg->num_docs, &le, &err);
  if (rc) return fail(rc, "raw forward index of column %d: %s", column, err.c_str());
  const ValueRange vr = value_range_of(le.data(), (size_t)seg->num_docs, data_type);
  // padded to whole PGPU_TILE-doc tiles (+16 B) like a fixed-bit stream: the kernels read whole tiles of "ids"
  const uint64_t ntiles = ((uint64_t)seg->num_docs + PGPU_TILE - 1) / PGPU_TILE;
  const uint64_t alloc = std::max<uint64_t>(1, ntiles) * PGPU_TILE * w + 16;
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.dict, le.data(), le.size(), alloc, PGPU_MEM_HOST));
  c.kind = PGPU_COL_RAW;
  c.dict_type = data_type;
  c.fwd_card = seg->num_docs;
  c.fwd_bytes = num_bytes;
  c.dict_bytes = le.size();
  c.set_range(vr);
  return PGPU_OK;
}

int pgpu_segment_add_range_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  if (!bytes || num_bytes < 4) return fail(PGPU_E_INVALID, "range index of column %d: %llu bytes", column,
                                           (unsigned long long)num_bytes);
  const int32_t version = (int32_t)be32((const uint8_t*)bytes);
  if (version != 1 && version != 2) return fail(PGPU_E_INVALID, "range index of column %d: version %d", column, version);
  seg->cols[column].range_index = version;
  return PGPU_OK;
}

int pgpu_segment_add_mv_forward_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                      int32_t bits_per_value, int32_t cardinality, int64_t num_values) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  const int32_t n = seg->num_docs;
  if (bits_per_value < 1 || bits_per_value > 31 || cardinality < 1 || !bytes || n < 1 || num_values < n ||
      num_values > INT32_MAX)
    return fail(PGPU_E_INVALID, "MV forward index of column %d: bits %d, cardinality %d, %lld values, %d docs", column,
                bits_per_value, cardinality, (long long)num_values, n);
  HostColumn& c = seg->cols[column];
  if (c.kind != PGPU_COL_NONE) return fail(PGPU_E_INVALID, "column %d already has a forward index", column);
  if (c.dict_type == PGPU_STRING) return fail(PGPU_E_UNSUPPORTED, "multi-value STRING column %d", column);
  // FixedBitMVForwardIndexWriter.java:77-87: ceil(2048 / (float)(numValues / numDocs)) rows per chunk
  const float avg = (float)(num_values / n);
  const int64_t per = (int64_t)std::ceil(2048.0f / avg);
  const int64_t nchunks = (n + per - 1) / per;
  const uint64_t hdr = 4ull * nchunks, bm = ((uint64_t)num_values + 7) / 8;
  const uint64_t raw = ((uint64_t)num_values * bits_per_value + 7) / 8;
  if (num_bytes < hdr + bm + raw)
    return fail(PGPU_E_INVALID, "MV forward index of column %d: %llu bytes < %llu", column, (unsigned long long)num_bytes,
                (unsigned long long)(hdr + bm + raw));
  const uint8_t* b = (const uint8_t*)bytes;
  std::vector<int32_t> off;
  off.reserve((size_t)n + 1);
  for (int64_t v = 0; v < num_values; ++v)  // row starts: PinotDataBitSet bits, MSB first
    if ((b[hdr + (v >> 3)] >> (7 - (v & 7))) & 1) off.push_back((int32_t)v);
  if ((int64_t)off.size() != n || off[0] != 0)
    return fail(PGPU_E_INVALID, "MV forward index of column %d: %zu row starts for %d docs", column, off.size(), n);
  for (int64_t k = 0; k < nchunks; ++k)  // the chunk offsets must agree (a corrupt file fails here, not in a kernel)
    if ((int64_t)(int32_t)be32(b + 4 * k) != off[k * per])
      return fail(PGPU_E_INVALID, "MV forward index of column %d: chunk %lld offset disagrees with the bitmap", column,
                  (long long)k);
  off.push_back((int32_t)num_values);
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.fwd, b + hdr + bm, raw, raw + 16, PGPU_MEM_HOST));
  HIP_TRY(upload(c.mv_off, off.data(), off.size() * 4, off.size() * 4, PGPU_MEM_HOST));
  c.mv_raw.assign(b + hdr + bm, b + hdr + bm + raw);
  c.mv_raw.resize(raw + 8, 0);
  c.mv_offsets.swap(off);
  c.mv_values = num_values;
  c.kind = PGPU_COL_MV;
  c.bits = bits_per_value;
  c.fwd_card = cardinality;
  c.fwd_bytes = num_bytes;
  return PGPU_OK;
}

int pgpu_segment_mv_row(pgpu_segment* seg, int32_t column, int32_t doc, int32_t* out_ids, int32_t capacity,
                        int32_t* out_len) {
  if (!seg) return fail(PGPU_E_INVALID, "null segment");
  if (column < 0 || column >= (int32_t)seg->cols.size()) return fail(PGPU_E_INVALID, "bad column %d", column);
  const HostColumn& c = seg->cols[column];
  if (c.kind != PGPU_COL_MV) return fail(PGPU_E_INVALID, "column %d is not multi-value", column);
  if (doc < 0 || doc >= seg->num_docs || !out_len || (capacity > 0 && !out_ids))
    return fail(PGPU_E_INVALID, "doc %d of a %d-doc segment", doc, seg->num_docs);
  const int64_t v0 = c.mv_offsets[doc], v1 = c.mv_offsets[doc + 1];
  *out_len = (int32_t)(v1 - v0);
  const int64_t nv = std::min<int64_t>(v1 - v0, std::max(0, capacity));
  if (nv <= 0) return PGPU_OK;
  // the row's bits [v0 * b, (v0 + nv) * b) of the MSB-first packed ids (PinotDataBitSet.readInt)
  const int b = c.bits;
  const uint64_t byte0 = (uint64_t)(v0 * b) >> 3, byte1 = ((uint64_t)((v0 + nv) * b) + 7) >> 3;
  std::vector<uint8_t> raw(byte1 - byte0 + 8, 0);
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(hipMemcpy(raw.data(), (const uint8_t*)c.fwd.p + byte0, byte1 - byte0, hipMemcpyDeviceToHost));
  for (int64_t i = 0; i < nv; ++i) {
    const uint64_t bit = (uint64_t)((v0 + i) * b) - byte0 * 8;
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) w = (w << 8) | raw[(bit >> 3) + k];
    out_ids[i] = (int32_t)((w >> (64 - (bit & 7) - b)) & ((1ull << b) - 1));
  }
  return PGPU_OK;
}

namespace {
// Install host little-endian values as a raw column in `slot` (padded like a decoded raw forward index).
int install_raw(pgpu_segment* seg, int32_t slot, int32_t data_type, std::vector<uint8_t>& le, const ValueRange& vr) {
  int rc = check_column(seg, slot);
  if (rc) return rc;
  HostColumn& c = seg->cols[slot];
  if (c.kind != PGPU_COL_NONE || c.dict_card) return fail(PGPU_E_INVALID, "row column slot %d is not empty", slot);
  const int w = type_width(data_type);
  const uint64_t ntiles = ((uint64_t)seg->num_docs + PGPU_TILE - 1) / PGPU_TILE;
  const uint64_t alloc = std::max<uint64_t>(1, ntiles) * PGPU_TILE * w + 16;
  HIP_TRY(upload(c.dict, le.data(), le.size(), alloc, PGPU_MEM_HOST));
  c.kind = PGPU_COL_RAW;
  c.dict_type = data_type;
  c.fwd_card = seg->num_docs;
  c.dict_bytes = le.size();
  c.set_range(vr);
  return PGPU_OK;
}
}  // namespace

int pgpu_segment_add_mv_row_columns(pgpu_segment* seg, int32_t column, int32_t len_column, int32_t sum_column,
                                    int32_t min_column, int32_t max_column) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  const HostColumn& c = seg->cols[column];
  if (c.kind != PGPU_COL_MV || c.mv_raw.empty())
    return fail(PGPU_E_INVALID, "column %d: no multi-value forward index (or the segment is sealed)", column);
  if (c.hdict.empty() || c.dict_card != c.fwd_card)
    return fail(PGPU_E_INVALID, "column %d: row columns need the numeric dictionary first", column);
  const int32_t n = seg->num_docs, t = c.dict_type;
  const bool fp = t == PGPU_FLOAT || t == PGPU_DOUBLE;
  const int w = type_width(t);
  auto value = [&](uint32_t id, int64_t* iv, double* dv) {
    if (t == PGPU_INT) { int32_t x; memcpy(&x, &c.hdict[4 * (size_t)id], 4); *iv = x; *dv = x; }
    else if (t == PGPU_LONG) { int64_t x; memcpy(&x, &c.hdict[8 * (size_t)id], 8); *iv = x; *dv = (double)x; }
    else if (t == PGPU_FLOAT) { float x; memcpy(&x, &c.hdict[4 * (size_t)id], 4); *iv = 0; *dv = x; }
    else { double x; memcpy(&x, &c.hdict[8 * (size_t)id], 8); *iv = 0; *dv = x; }
  };
  std::vector<uint8_t> lens(4 * (size_t)n), sums(8 * (size_t)n), mins(w * (size_t)n), maxs(w * (size_t)n);
  double max_len = 0, max_sum = 0, max_val = c.max_abs;
  const uint8_t* raw = c.mv_raw.data();
  const int bits = c.bits;
  for (int32_t d = 0; d < n; ++d) {
    const int32_t s0 = c.mv_offsets[d], e0 = c.mv_offsets[d + 1];
    const int32_t len = e0 - s0;
    memcpy(&lens[4 * (size_t)d], &len, 4);
    max_len = std::max(max_len, (double)len);
    int64_t isum = 0;
    double dsum = 0;
    uint32_t lo_id = UINT32_MAX, hi_id = 0;
    for (int32_t v = s0; v < e0; ++v) {
      const uint64_t bit = (uint64_t)v * bits;
      const uint8_t* q = raw + (bit >> 3);
      uint64_t win = 0;
      for (int k = 0; k < 8; ++k) win = (win << 8) | q[k];
      const uint32_t id = (uint32_t)((win >> (64 - (int)(bit & 7) - bits)) & ((1ull << bits) - 1));
      if (id >= (uint32_t)c.dict_card) return fail(PGPU_E_INVALID, "column %d: dict id %u out of range", column, id);
      int64_t iv;
      double dv;
      value(id, &iv, &dv);
      isum += iv;   // |row sum| <= maxNumberOfMultiValues * max |value| < 2^63 for 31-bit ids of LONGs below 2^32
      dsum += dv;   // SumMVAggregationFunction: the row's values added in order, as doubles
      lo_id = std::min(lo_id, id);
      hi_id = std::max(hi_id, id);
    }
    if (fp) {
      memcpy(&sums[8 * (size_t)d], &dsum, 8);
      max_sum = abs_bound(max_sum, dsum);
    } else {
      memcpy(&sums[8 * (size_t)d], &isum, 8);
      max_sum = std::max(max_sum, std::fabs((double)isum));
    }
    // the dictionary is sorted: the row's smallest / largest value is the value of its smallest / largest id
    memcpy(&mins[w * (size_t)d], &c.hdict[w * (size_t)lo_id], w);
    memcpy(&maxs[w * (size_t)d], &c.hdict[w * (size_t)hi_id], w);
  }
  HIP_TRY(hipSetDevice(seg->ctx->device));
  ValueRange r_len, r_sum, r_val;
  r_len.max_abs = max_len;
  if (fp) r_sum = value_range_of(sums.data(), (size_t)n, PGPU_DOUBLE);  // row sums: their own fixed-point range
  r_sum.max_abs = max_sum;
  r_val.max_abs = max_val;
  r_val.min_exp = c.min_exp;  // row min / max values are dictionary values
  r_val.min_lsb = c.min_lsb;
  if (len_column >= 0 && (rc = install_raw(seg, len_column, PGPU_INT, lens, r_len))) return rc;
  if (sum_column >= 0 && (rc = install_raw(seg, sum_column, fp ? PGPU_DOUBLE : PGPU_LONG, sums, r_sum))) return rc;
  if (min_column >= 0 && (rc = install_raw(seg, min_column, t, mins, r_val))) return rc;
  if (max_column >= 0 && (rc = install_raw(seg, max_column, t, maxs, r_val))) return rc;
  return PGPU_OK;
}

int pgpu_segment_add_inverted_index(pgpu_segment* seg, int32_t column, const void* bytes, uint64_t num_bytes,
                                    int32_t cardinality) {
  int rc = check_column(seg, column);
  if (rc) return rc;
  const uint8_t* b = (const uint8_t*)bytes;
  const uint64_t hdr = 4ull * ((uint64_t)cardinality + 1);
  if (cardinality < 1 || !bytes || num_bytes < hdr)
    return fail(PGPU_E_INVALID, "inverted index of column %d: %llu bytes for cardinality %d", column,
                (unsigned long long)num_bytes, cardinality);
  // BitmapInvertedIndexReader: offsets may be absolute (writer) or bitmap-relative; subtract the first one.
  const uint32_t first = be32(b);
  std::vector<uint32_t> dir(cardinality + 1);
  std::vector<uint32_t> cards(cardinality, 0);
  std::vector<DevContainer> cts;
  std::vector<uint8_t> data;
  std::vector<ParsedContainer> parsed;
  for (int32_t i = 0; i < cardinality; ++i) {
    const uint32_t o0 = be32(b + 4ull * i), o1 = be32(b + 4ull * (i + 1));
    if (o0 < first || o1 < o0 || hdr + (o1 - first) > num_bytes)
      return fail(PGPU_E_INVALID, "inverted index of column %d: bad offsets at dict id %d", column, i);
    parsed.clear();
    rc = parse_roaring(b + hdr + (o0 - first), o1 - o0, &parsed);
    if (rc) return rc;
    dir[i] = (uint32_t)cts.size();
    for (const ParsedContainer& pc : parsed) {
      if ((uint64_t)pc.key << 16 >= (uint64_t)seg->num_docs + 65536)
        return fail(PGPU_E_INVALID, "inverted index of column %d: container key %u beyond numDocs", column, pc.key);
      size_t off = (data.size() + 7) & ~(size_t)7;
      data.resize(off + pc.payload_bytes);
      memcpy(&data[off], pc.payload, pc.payload_bytes);
      cts.push_back(DevContainer{pc.key, pc.type, pc.card, (uint32_t)off});
      if (pc.type == PGPU_CT_RUN) {
        for (uint32_t r = 0; r < pc.card; ++r) cards[i] += (uint32_t)le16(pc.payload + 4 * r + 2) + 1;
      } else {
        cards[i] += pc.card;
      }
      if (data.size() > 0xFFFFFFF0ull) return fail(PGPU_E_INVALID, "inverted index too large");
    }
  }
  dir[cardinality] = (uint32_t)cts.size();
  HostColumn& c = seg->cols[column];
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.inv_dir, dir.data(), dir.size() * 4, dir.size() * 4, PGPU_MEM_HOST));
  HIP_TRY(upload(c.inv_ct, cts.data(), cts.size() * sizeof(DevContainer), cts.size() * sizeof(DevContainer) + 16,
                 PGPU_MEM_HOST));
  HIP_TRY(upload(c.inv_data, data.data(), data.size(), data.size() + 16, PGPU_MEM_HOST));
  c.inv_card = cardinality;
  c.inv_bytes = num_bytes;
  c.inv_cards.swap(cards);
  c.inv_hdir.swap(dir);
  return PGPU_OK;
}

namespace {
// The kernels' view of column i (DevColumn), with its bit-sliced copy built first (fixed-bit columns).
// Reserve `bytes` of the context's derived-copy budget (false: over budget, the copy is not built).
bool reserve_derived(pgpu_context* ctx, uint64_t bytes) {
  uint64_t cur = ctx->derived_bytes.load();
  do {
    if (cur + bytes > ctx->derived_budget.load()) return false;
  } while (!ctx->derived_bytes.compare_exchange_weak(cur, cur + bytes));
  return true;
}

int seal_column(pgpu_segment* seg, size_t i) {
  static const bool no_slice = getenv("PGPU_NO_SLICE") && atoi(getenv("PGPU_NO_SLICE")) != 0;
  HostColumn& c = seg->cols[i];
  // derived copies (PhysicalColumnIndexContainer.java:80,151-156 loads only the indexes IndexLoadingConfig names):
  // the column's pgpu_segment_set_derived flags, within the context's budget; the kernels plan without them
  if (c.kind == PGPU_COL_FIXED_BIT && !no_slice && !c.sliced.p && (c.derive & PGPU_DERIVE_SLICED) &&
      reserve_derived(seg->ctx, c.fwd.n)) {
    // bit planes of every 2048-doc tile of the padded stream (same byte count as the packed copy)
    const int64_t ntiles = ((int64_t)seg->num_docs + PGPU_TILE - 1) / PGPU_TILE * (PGPU_TILE / PGPU_WT);
    const hipError_t ae = c.sliced.alloc(c.fwd.n);
    if (ae != hipSuccess) {
      seg->ctx->derived_bytes -= c.fwd.n;
      return fail(PGPU_E_HIP, "bit-sliced copy of column %zu: %s", i, hipGetErrorString(ae));
    }
    HIP_TRY(hipMemset(c.sliced.p, 0, c.sliced.n));
    HIP_TRY(pgpu_launch_bitslice((const uint32_t*)c.fwd.p, (uint32_t*)c.sliced.p, c.bits, ntiles, nullptr));
  }
  // value planes (bit-sliced index of the values): SUM is then sum_k 2^k popcount(plane_k & matched) per tile and
  // MIN / MAX an MSB-first selection -- no per-doc id extraction, no dictionary gather (PGPU_AM_SLICED)
  static const bool no_vslice = getenv("PGPU_NO_VSLICE") && atoi(getenv("PGPU_NO_VSLICE")) != 0;
  if (c.kind == PGPU_COL_FIXED_BIT && !no_vslice && !c.vsliced.p && c.dict.p && c.dict_card > 0 &&
      (c.dict_type == PGPU_INT || c.dict_type == PGPU_LONG) && c.hdict.size() >= (size_t)c.dict_card * type_width(c.dict_type)) {
    int64_t lo, hi;
    if (c.dict_type == PGPU_INT) {
      int32_t a, b;
      memcpy(&a, c.hdict.data(), 4);
      memcpy(&b, c.hdict.data() + 4 * (size_t)(c.dict_card - 1), 4);
      lo = a;
      hi = b;
    } else {
      memcpy(&lo, c.hdict.data(), 8);
      memcpy(&hi, c.hdict.data() + 8 * (size_t)(c.dict_card - 1), 8);
    }
    const uint64_t range = (uint64_t)hi - (uint64_t)lo;  // ascending dictionary (checked at upload)
    int vb = 0;
    while (vb < 64 && (range >> vb)) ++vb;
    const int64_t ntiles = ((int64_t)seg->num_docs + PGPU_TILE - 1) / PGPU_TILE * (PGPU_TILE / PGPU_WT);
    if (hi >= lo && vb >= 1 && vb <= 32 && (c.derive & PGPU_DERIVE_VALUE_PLANES) &&
        reserve_derived(seg->ctx, (uint64_t)ntiles * 256 * vb)) {
      const hipError_t ae = c.vsliced.alloc((size_t)ntiles * 256 * vb);
      if (ae != hipSuccess) {
        seg->ctx->derived_bytes -= (uint64_t)ntiles * 256 * vb;
        return fail(PGPU_E_HIP, "value planes of column %zu: %s", i, hipGetErrorString(ae));
      }
      HIP_TRY(pgpu_launch_vslice((const uint32_t*)c.fwd.p, c.dict.p, c.dict_type, lo, c.bits, vb,
                                 (uint32_t*)c.vsliced.p, ntiles, nullptr));
      c.vmin = lo;
      c.vbits = vb;
    }
  }
  DevColumn d{};
  d.sliced = (const uint32_t*)c.sliced.p;
  d.vsliced = (const uint32_t*)c.vsliced.p;
  d.vmin = c.vmin;
  d.vbits = c.vbits;
  d.fwd = (const uint32_t*)c.fwd.p;
  // a multi-value column's row offsets take the sorted-index slot (sparse_agg_mv; a MV column has no sorted index)
  d.sorted = (const int32_t*)(c.kind == PGPU_COL_MV ? c.mv_off.p : c.sorted.p);
  d.dict = c.dict.p;
  d.inv_dir = (const uint32_t*)c.inv_dir.p;
  d.inv_ct = (const DevContainer*)c.inv_ct.p;
  d.inv_data = (const uint8_t*)c.inv_data.p;
  d.kind = c.kind;
  d.bits = c.bits;
  d.card = c.fwd_card ? c.fwd_card : (c.dict_card ? c.dict_card : c.inv_card);
  d.dict_type = c.dict_type;
  c.card = d.card;
  if (c.dict_card && c.fwd_card && c.dict_card != c.fwd_card)
    return fail(PGPU_E_INVALID, "column %zu: dictionary cardinality %d != index cardinality %d", i, c.dict_card,
                c.fwd_card);
  seg->dev[i] = d;
  std::vector<uint8_t>().swap(c.mv_raw);
  return PGPU_OK;
}
}  // namespace

int pgpu_segment_seal(pgpu_segment* seg) {
  if (!seg) return fail(PGPU_E_INVALID, "null segment");
  seg->dev.resize(seg->cols.size());
  HIP_TRY(hipSetDevice(seg->ctx->device));
  for (size_t i = 0; i < seg->cols.size(); ++i) {
    const int rc = seal_column(seg, i);
    if (rc) return rc;
  }
  HIP_TRY(hipDeviceSynchronize());
  seg->sealed = true;
  return PGPU_OK;
}

int pgpu_segment_add_group_dictionary(pgpu_segment* seg, int32_t raw_column, int32_t dict_column,
                                      int32_t* out_cardinality) {
  if (!seg || !out_cardinality) return fail(PGPU_E_INVALID, "null argument");
  const int32_t nc = (int32_t)seg->cols.size();
  if (raw_column < 0 || raw_column >= nc || dict_column < 0 || dict_column >= nc || raw_column == dict_column)
    return fail(PGPU_E_INVALID, "bad columns %d -> %d", raw_column, dict_column);
  const HostColumn& r = seg->cols[raw_column];
  HostColumn& c = seg->cols[dict_column];
  if (r.kind != PGPU_COL_RAW) return fail(PGPU_E_INVALID, "column %d is not a raw (no-dictionary) column", raw_column);
  if (c.kind != PGPU_COL_NONE || c.dict_card) return fail(PGPU_E_INVALID, "group dictionary slot %d is not empty", dict_column);
  const int64_t n = seg->num_docs;
  if (n < 1) return fail(PGPU_E_UNSUPPORTED, "group dictionary of an empty segment");
  const int32_t t = r.dict_type;
  const int w = type_width(t);
  HIP_TRY(hipSetDevice(seg->ctx->device));
  DevMem keys, sorted, uniq, dcard, temp, ids, fwd, dict;
  const size_t tb = pgpu_gdict_temp_bytes(n);
  HIP_TRY(keys.alloc(8 * (size_t)n));
  HIP_TRY(sorted.alloc(8 * (size_t)n));
  HIP_TRY(uniq.alloc(8 * (size_t)n));
  HIP_TRY(dcard.alloc(16));
  HIP_TRY(temp.alloc(tb));
  HIP_TRY(pgpu_gdict_sort_unique(r.dict.p, t, n, (uint64_t*)keys.p, (uint64_t*)sorted.p, (uint64_t*)uniq.p,
                                 (uint32_t*)dcard.p, temp.p, tb, nullptr));
  uint32_t card = 0;
  HIP_TRY(hipMemcpy(&card, dcard.p, 4, hipMemcpyDeviceToHost));
  if (card < 1 || (int64_t)card > n) return fail(PGPU_E_INVALID, "group dictionary of column %d: cardinality %u", raw_column, card);
  sorted.reset();
  temp.reset();
  int bits = 1;  // PinotDataBitSet.getNumBitsPerValue(card - 1)
  while (bits < 31 && (1ll << bits) < (int64_t)card) ++bits;
  const uint64_t ntiles = ((uint64_t)n + PGPU_TILE - 1) / PGPU_TILE;
  const uint64_t need = ((uint64_t)n * bits + 7) / 8;
  const uint64_t alloc = std::max<uint64_t>(ntiles * PGPU_TILE / 8 * bits, need) + 16;
  HIP_TRY(fwd.alloc(alloc));
  HIP_TRY(hipMemset(fwd.p, 0, alloc));
  HIP_TRY(ids.alloc(4 * (size_t)n));
  HIP_TRY(dict.alloc((size_t)w * card));
  const int64_t nwords = (int64_t)((need + 3) / 4);
  HIP_TRY(pgpu_gdict_encode((const uint64_t*)keys.p, n, (const uint64_t*)uniq.p, (int32_t)card, t, bits, dict.p,
                            (uint32_t*)ids.p, (uint32_t*)fwd.p, nwords, nullptr));
  std::vector<uint8_t> le((size_t)w * card);
  HIP_TRY(hipMemcpy(le.data(), dict.p, le.size(), hipMemcpyDeviceToHost));
  const ValueRange vr = value_range_of(le.data(), (size_t)card, t);
  c.dict = std::move(dict);
  c.fwd = std::move(fwd);
  c.dict_type = t;
  c.dict_card = (int32_t)card;
  c.dict_bytes = le.size();
  c.kind = PGPU_COL_FIXED_BIT;
  c.bits = bits;
  c.fwd_card = (int32_t)card;
  c.fwd_bytes = need;
  c.set_range(vr);
  dictionary_hash(le, c.dict_hash);
  c.hdict = std::move(le);
  if (seg->sealed) {
    const int rc = seal_column(seg, (size_t)dict_column);
    if (rc) return rc;
  }
  HIP_TRY(hipDeviceSynchronize());
  *out_cardinality = (int32_t)card;
  return PGPU_OK;
}

int pgpu_segment_add_docid_column(pgpu_segment* seg, int32_t column) {
  if (!seg) return fail(PGPU_E_INVALID, "null segment");
  if (column < 0 || column >= (int32_t)seg->cols.size()) return fail(PGPU_E_INVALID, "bad column %d", column);
  HostColumn& c = seg->cols[column];
  if (c.kind != PGPU_COL_NONE || c.dict_card) return fail(PGPU_E_INVALID, "doc-id slot %d is not empty", column);
  const int32_t n = seg->num_docs;
  // padded to whole PGPU_TILE-doc tiles (+16 B) like any raw column: the kernels read whole tiles of "ids"
  const uint64_t ntiles = ((uint64_t)std::max(n, 1) + PGPU_TILE - 1) / PGPU_TILE;
  std::vector<int32_t> iota((size_t)ntiles * PGPU_TILE + 4, 0);
  for (int32_t i = 0; i < n; ++i) iota[(size_t)i] = i;
  HIP_TRY(hipSetDevice(seg->ctx->device));
  HIP_TRY(upload(c.dict, iota.data(), 4ull * iota.size(), 4ull * iota.size(), PGPU_MEM_HOST));
  c.kind = PGPU_COL_RAW;
  c.dict_type = PGPU_INT;
  c.fwd_card = n;
  c.dict_bytes = 4ull * (uint64_t)n;
  c.max_abs = n > 0 ? (double)(n - 1) : 0.0;
  if (seg->sealed) {
    const int rc = seal_column(seg, (size_t)column);
    if (rc) return rc;
  }
  return PGPU_OK;
}

int pgpu_segment_dictionary_values(const pgpu_segment* seg, int32_t column, void* out, uint64_t capacity_bytes,
                                   uint64_t* out_bytes) {
  if (!seg || !out_bytes) return fail(PGPU_E_INVALID, "null argument");
  if (column < 0 || column >= (int32_t)seg->cols.size()) return fail(PGPU_E_INVALID, "bad column %d", column);
  const HostColumn& c = seg->cols[column];
  if (c.hdict.empty()) return fail(PGPU_E_INVALID, "column %d has no numeric dictionary", column);
  *out_bytes = c.hdict.size();
  if (!out) return PGPU_OK;
  if (capacity_bytes < c.hdict.size()) return fail(PGPU_E_INVALID, "dictionary of column %d: %zu bytes > capacity", column,
                                                   c.hdict.size());
  memcpy(out, c.hdict.data(), c.hdict.size());
  return PGPU_OK;
}

int pgpu_segment_device_bytes(const pgpu_segment* seg, uint64_t* out_bytes) {
  pgpu_segment_bytes b;
  const int rc = pgpu_segment_device_bytes_ex(seg, &b);
  if (rc) return rc;
  if (!out_bytes) return fail(PGPU_E_INVALID, "null argument");
  *out_bytes = b.total;
  return PGPU_OK;
}

int pgpu_segment_device_bytes_ex(const pgpu_segment* seg, pgpu_segment_bytes* out) {
  if (!seg || !out) return fail(PGPU_E_INVALID, "null argument");
  memset(out, 0, sizeof(*out));
  for (const HostColumn& c : seg->cols) {
    if (c.kind == PGPU_COL_MV) out->multi_value += c.fwd.n + c.mv_off.n;
    else out->forward += c.fwd.n;
    // a raw column's values sit in the dictionary's slot (they are its forward index)
    if (c.kind == PGPU_COL_RAW) out->forward += c.dict.n;
    else out->dictionary += c.dict.n + c.for_dev.n;
    out->sorted += c.sorted.n;
    out->inverted += c.inv_dir.n + c.inv_ct.n + c.inv_data.n;
    out->sliced += c.sliced.n;
    out->value_planes += c.vsliced.n;
  }
  out->total = out->forward + out->dictionary + out->sorted + out->inverted + out->multi_value + out->sliced +
               out->value_planes;
  return PGPU_OK;
}

int pgpu_segment_set_derived(pgpu_segment* seg, int32_t column, int32_t flags) {
  const int rc = check_column(seg, column);
  if (rc) return rc;
  if (flags < 0 || flags > PGPU_DERIVE_ALL) return fail(PGPU_E_INVALID, "derived-copy flags %d", flags);
  if (seg->sealed) return fail(PGPU_E_INVALID, "segment already sealed");
  seg->cols[column].derive = flags;
  return PGPU_OK;
}

int pgpu_context_set_derived_budget(pgpu_context* ctx, uint64_t bytes) {
  if (!ctx) return fail(PGPU_E_INVALID, "null context");
  ctx->derived_budget = bytes;
  return PGPU_OK;
}

int pgpu_context_derived_bytes(pgpu_context* ctx, uint64_t* out_used, uint64_t* out_budget) {
  if (!ctx || !out_used || !out_budget) return fail(PGPU_E_INVALID, "null argument");
  *out_used = ctx->derived_bytes.load();
  *out_budget = ctx->derived_budget.load();
  return PGPU_OK;
}

int pgpu_segment_release(pgpu_segment* seg) {
  if (!seg) return PGPU_OK;
  (void)hipSetDevice(seg->ctx->device);
  uint64_t derived = 0;
  for (const HostColumn& c : seg->cols) derived += c.sliced.n + c.vsliced.n;
  seg->ctx->derived_bytes -= derived;
  delete seg;
  return PGPU_OK;
}

int pgpu_remap_upload(pgpu_context* ctx, const int32_t* map, int32_t length, pgpu_buffer** out_buf) {
  if (!ctx || !out_buf || length < 0 || (!map && length)) return fail(PGPU_E_INVALID, "bad remap arguments");
  auto* b = new pgpu_buffer();
  b->ctx = ctx;
  b->length = length;
  hipError_t e = hipSetDevice(ctx->device);
  if (e == hipSuccess) e = upload(b->mem, map, 4ull * length, 4ull * length + 16, PGPU_MEM_HOST);
  if (e != hipSuccess) {
    delete b;
    return fail(PGPU_E_HIP, "remap upload: %s", hipGetErrorString(e));
  }
  *out_buf = b;
  return PGPU_OK;
}

int pgpu_buffer_release(pgpu_buffer* buf) {
  delete buf;
  return PGPU_OK;
}

void pgpu_fixed_sum_layout(double max_abs, int32_t min_exp, int32_t min_lsb, int32_t* out_exp, int32_t* out_parts) {
  if (!(max_abs > 0)) {  // no nonzero value: any window holds the zero sums
    *out_exp = PGPU_SUM_EXP_ZERO;
    *out_parts = 3;
    return;
  }
  // every |v| < 2^top, and rint(|v| * 2^-e) <= 2^(top - 1) < 2^(21 * parts) even where rounding carries up
  const int32_t top = (int32_t)std::ilogb(max_abs) + 2;
  // the exponent each value needs: its own last bit (exact), or 41 bits below its leading bit (rounding error
  // <= 2^-41 |v|), whichever is coarser
  const int64_t need = std::max<int64_t>(min_lsb, (int64_t)min_exp - PGPU_FIXED_TOL_BITS);
  const int64_t span = (int64_t)top - need;
  const int64_t parts = std::max<int64_t>(3, (span + PGPU_PART_BITS - 1) / PGPU_PART_BITS);
  if (parts > PGPU_MAX_FIXED_PARTS) {
    *out_exp = PGPU_SUM_EXP_F64;
    *out_parts = 1;
    return;
  }
  *out_exp = top - PGPU_PART_BITS * (int32_t)parts;
  *out_parts = (int32_t)parts;
}

int pgpu_sum_layout_agree(const pgpu_table_layout* layouts, int32_t num_layouts, int32_t num_aggs, int32_t* out_exp,
                          int32_t* out_parts) {
  if (!layouts || num_layouts < 1 || num_aggs < 0 || num_aggs > 16 || !out_exp || !out_parts)
    return fail(PGPU_E_INVALID, "bad sum layout arguments");
  for (int a = 0; a < num_aggs; ++a) {
    int64_t top = INT64_MIN, bottom = INT64_MAX;
    bool f64 = false, any = false;
    for (int i = 0; i < num_layouts; ++i) {
      const pgpu_table_layout& L = layouts[i];
      const int vt = L.agg_value_type[a];
      if (vt != PGPU_FLOAT && vt != PGPU_DOUBLE) continue;
      const int32_t e = L.agg_sum_exp[a];
      if (e == PGPU_SUM_EXP_F64) f64 = true;
      if (e == PGPU_SUM_EXP_F64 || e == PGPU_SUM_EXP_ZERO || L.agg_sum_parts[a] < 1) continue;
      any = true;
      top = std::max<int64_t>(top, (int64_t)e + PGPU_PART_BITS * L.agg_sum_parts[a]);
      bottom = std::min<int64_t>(bottom, e);
    }
    out_exp[a] = 0;
    out_parts[a] = 0;
    if (f64) {
      out_exp[a] = PGPU_SUM_EXP_F64;
      out_parts[a] = 1;
    } else if (!any) {
      out_exp[a] = PGPU_SUM_EXP_ZERO;
      out_parts[a] = 3;
    } else {
      const int64_t parts = std::max<int64_t>(3, (top - bottom + PGPU_PART_BITS - 1) / PGPU_PART_BITS);
      out_parts[a] = (int32_t)std::min<int64_t>(parts, PGPU_MAX_FIXED_PARTS + 1);  // > MAX: every layout takes f64
      out_exp[a] = (int32_t)(top - PGPU_PART_BITS * parts);
    }
  }
  return PGPU_OK;
}

int pgpu_table_layout_of(const pgpu_query_desc* q, pgpu_table_layout* out) {
  if (!q || !out) return fail(PGPU_E_INVALID, "null argument");
  if (q->num_aggs < 0 || q->num_aggs > PGPU_MAX_AGGS) return fail(PGPU_E_UNSUPPORTED, "%d aggregations", q->num_aggs);
  if (q->num_group_columns < 0 || q->num_group_columns > PGPU_MAX_GCOLS)
    return fail(PGPU_E_UNSUPPORTED, "%d group-by columns", q->num_group_columns);
  if (q->num_segments < 1 || !q->segments) return fail(PGPU_E_INVALID, "no segments");
  memset(out, 0, sizeof(*out));
  const int rc = group_key_space(q, out);
  if (rc) return rc;
  out->num_sections = 1;
  out->section_op[0] = PGPU_RED_SUM_I64;
  const pgpu_segment* s0 = q->segments[0].segment;
  int64_t docs = 0;
  for (int s = 0; s < q->num_segments; ++s)
    if (q->segments[s].segment) docs += q->segments[s].segment->num_docs;
  docs = std::max<int64_t>(docs, q->reduce_docs);
  // FLOAT / DOUBLE SUM / AVG in fixed point (fx_parts[a] 21-bit part sections each, pgpu_fixed_sum_layout) when the
  // column is finite and the part count fits; otherwise that aggregation keeps a float64 section (and all of them do
  // when the part sections would not fit the table).  PGPU_NO_FIXED_SUM=1 forces float64.
  static const bool no_fixed = getenv("PGPU_NO_FIXED_SUM") && atoi(getenv("PGPU_NO_FIXED_SUM")) != 0;
  if (q->sum_exp && !q->sum_parts) return fail(PGPU_E_INVALID, "sum_exp without sum_parts");
  int32_t fx_exp[16], fx_parts[16];
  bool fixed_all = !no_fixed;
  {
    int with_fixed = 1, without = 1;  // sections of either choice
    for (int a = 0; a < q->num_aggs; ++a) {
      const pgpu_agg& ag = q->aggs[a];
      fx_exp[a] = 0;
      fx_parts[a] = 0;
      if (ag.fn == PGPU_AGG_COUNT) continue;
      int32_t vt = -1;
      ValueRange vr;
      if (ag.column >= 0 && ag.column < q->num_columns)
        for (int s = 0; s < q->num_segments; ++s) {
          const pgpu_segment* sg = q->segments[s].segment;
          const int32_t sl = q->segments[s].column_map ? q->segments[s].column_map[ag.column] : -1;
          if (!sg || sl < 0 || sl >= (int32_t)sg->cols.size()) continue;  // reported below
          if (vt < 0) vt = sg->cols[sl].dict_type;
          ValueRange c;
          c.max_abs = sg->cols[sl].max_abs;
          c.min_exp = sg->cols[sl].min_exp;
          c.min_lsb = sg->cols[sl].min_lsb;
          vr.merge(c);
        }
      const bool sum = ag.fn == PGPU_AGG_SUM || ag.fn == PGPU_AGG_AVG;
      if (sum && (vt == PGPU_FLOAT || vt == PGPU_DOUBLE)) {
        int32_t e = PGPU_SUM_EXP_F64, parts = 1;
        if (std::isfinite(vr.max_abs)) pgpu_fixed_sum_layout(vr.max_abs, vr.min_exp, vr.min_lsb, &e, &parts);
        if (q->sum_exp && e != PGPU_SUM_EXP_F64) {  // the layout agreed across launches (pgpu_sum_layout_agree)
          const int32_t ge = q->sum_exp[a], gp = q->sum_parts[a];
          if (ge == PGPU_SUM_EXP_F64) {
            e = PGPU_SUM_EXP_F64;
          } else if (ge == PGPU_SUM_EXP_ZERO) {
            if (e != PGPU_SUM_EXP_ZERO) return fail(PGPU_E_INVALID, "agg %d: agreed fixed-point layout is empty", a);
          } else if (gp > PGPU_MAX_FIXED_PARTS) {
            e = PGPU_SUM_EXP_F64;
          } else {
            // the agreed window must hold this launch's values at no less precision than its own choice
            if (gp < 3 || (e != PGPU_SUM_EXP_ZERO && (ge > e || ge + 21 * gp < e + 21 * parts)))
              return fail(PGPU_E_INVALID, "agg %d: agreed fixed-point layout (2^%d, %d parts) does not cover the launch",
                          a, ge, gp);
            e = ge;
            parts = gp;
          }
        } else if (q->sum_exp && q->sum_exp[a] != PGPU_SUM_EXP_F64) {
          return fail(PGPU_E_INVALID, "agg %d: agreed fixed-point layout for a column with NaN / infinity", a);
        }
        if (e == PGPU_SUM_EXP_F64) parts = 1;
        fx_exp[a] = e;
        fx_parts[a] = parts;
        with_fixed += parts;
        without += 1;
      } else {
        const int k = sum && ((q->flags & PGPU_Q_SUM_SPLIT) || vr.max_abs * (double)docs >= 4.611686018427388e18) ? 3 : 1;
        with_fixed += k;
        without += k;
      }
    }
    // the float64 sections when the part sections would not fit (and the integer ones would)
    if (with_fixed > PGPU_MAX_SECTIONS && without <= PGPU_MAX_SECTIONS) fixed_all = false;
  }
  for (int a = 0; a < q->num_aggs; ++a) {
    const pgpu_agg& ag = q->aggs[a];
    if (ag.fn < PGPU_AGG_COUNT || ag.fn > PGPU_AGG_AVG) return fail(PGPU_E_UNSUPPORTED, "aggregation fn %d", ag.fn);
    if (ag.fn == PGPU_AGG_COUNT) {
      out->agg_section[a] = 0;
      out->agg_value_type[a] = -1;
      continue;
    }
    if (ag.column < 0 || ag.column >= q->num_columns) return fail(PGPU_E_INVALID, "agg %d column %d", a, ag.column);
    const int32_t slot = q->segments[0].column_map[ag.column];
    if (!s0 || slot < 0 || slot >= (int32_t)s0->cols.size()) return fail(PGPU_E_INVALID, "agg %d column slot", a);
    const int32_t vt = s0->cols[slot].dict_type;
    if (vt < PGPU_INT || vt > PGPU_DOUBLE)
      return fail(PGPU_E_UNSUPPORTED, "agg %d over a non-numeric or dictionary-less column", a);
    int op;
    if (ag.fn == PGPU_AGG_MIN) op = PGPU_RED_MIN_I64;
    else if (ag.fn == PGPU_AGG_MAX) op = PGPU_RED_MAX_I64;
    else op = (vt == PGPU_INT || vt == PGPU_LONG || (fixed_all && fx_exp[a] != PGPU_SUM_EXP_F64)) ? PGPU_RED_SUM_I64
                                                                                                  : PGPU_RED_SUM_F64;
    // integer SUM: one int64 cell while max|value| x docs stays below 2^62, else three exact part sums; fixed-point
    // floating SUM: fx_parts[a] part sums
    int parts = 1;
    out->agg_sum_exp[a] = 0;
    if (op == PGPU_RED_SUM_F64) {
      out->agg_sum_exp[a] = PGPU_SUM_EXP_F64;
    } else if (op == PGPU_RED_SUM_I64 && (vt == PGPU_FLOAT || vt == PGPU_DOUBLE)) {
      out->agg_sum_exp[a] = fx_exp[a];
      parts = fx_parts[a];
    } else if (op == PGPU_RED_SUM_I64) {
      double max_abs = 0;
      for (int s = 0; s < q->num_segments; ++s) {
        const pgpu_segment* sg = q->segments[s].segment;
        const int32_t sl = q->segments[s].column_map ? q->segments[s].column_map[ag.column] : -1;
        if (!sg || sl < 0 || sl >= (int32_t)sg->cols.size()) return fail(PGPU_E_INVALID, "agg %d column slot", a);
        max_abs = std::max(max_abs, sg->cols[sl].max_abs);
      }
      if ((q->flags & PGPU_Q_SUM_SPLIT) || max_abs * (double)docs >= 4.611686018427388e18) parts = 3;
    }
    if (out->num_sections + parts > PGPU_MAX_SECTIONS)
      return fail(PGPU_E_UNSUPPORTED, "more than %d value sections", PGPU_MAX_SECTIONS - 1);
    out->agg_section[a] = out->num_sections;
    out->agg_value_type[a] = vt;
    out->agg_sum_parts[a] = parts;
    for (int k = 0; k < parts; ++k) out->section_op[out->num_sections++] = op;
  }
  return PGPU_OK;
}

double pgpu_decode_minmax_key(int64_t key, int32_t value_type) {
  if (value_type == PGPU_INT || value_type == PGPU_LONG) return (double)key;
  int64_t b = key >= 0 ? key : (key ^ 0x7FFFFFFFFFFFFFFFll);
  double d;
  memcpy(&d, &b, 8);
  return d;
}

int pgpu_kernel_geometry(pgpu_context* ctx, int32_t* out_grid, int32_t* out_tile_docs, int32_t* out_block) {
  if (!ctx) return fail(PGPU_E_INVALID, "null ctx");
  if (out_tile_docs) *out_tile_docs = PGPU_WT;
  if (out_block) *out_block = PGPU_THREADS(0);
  if (out_grid) *out_grid = ctx->num_cus;  // one 512-thread workgroup per CU
  return PGPU_OK;
}

}  // extern "C"

// ---- plan packing ---------------------------------------------------------------------------------------------
namespace {

struct Packer {
  std::vector<DevSeg> segs;
  std::vector<DevInstr> instrs;
  std::vector<DevColumn> cols;
  std::vector<int32_t> pool;
  std::vector<const int32_t*> remaps;
  int32_t slot_bytes = 0;   // largest staged region set of any segment
  int32_t max_instrs = 0;   // most DMA instructions of one tile
  int64_t tile_bytes = 0;   // largest staged bytes of one tile
  double est_matched = 0;   // estimated matched docs (LDS-table decision)
  std::vector<int32_t> tracked;  // HASH: query segments whose distinct keys are counted (bitmap row order)
  int64_t leaf_words = 0;        // PGPU_Q_EXACT_FILTER_STATS: 32-bit words of all leaf bitmaps
  bool fsm = false;              // ... computed on the GPU by the andfsm kernels (every segment fsm_filter)
  bool fsm_s2 = false;           // ... by its two-sliced-leaf build
  // raw-value leaves: until launch, RawLeaf::out holds the bitmap's word offset in Workspace::rawbits and
  // RawLeaf::vals its set's offset in rawvals; PGPU_I_BITS instructions (bits_instrs) hold the word offset in fwd
  std::vector<RawLeaf> raws;
  std::vector<int64_t> rawvals;
  int64_t raw_words = 0;
  std::vector<int> bits_instrs;
  bool legacy_range = false;     // a version-1 range-index leaf: the GPU's filter count is not the reference's
  // multi-value SCAN leaves: until launch, MvLeaf::out holds the bitmap's word offset in Workspace::rawbits and
  // MvLeaf::set its membership words' offset in mvsets
  std::vector<MvLeaf> mvs;
  std::vector<uint32_t> mvsets;
  // inverted-index leaves expanded before the query kernel (invexp_kernel): InvLeafX::out = word offset in rawbits,
  // InvLeafX::ids = offset in invids until launch
  std::vector<InvLeafX> invx;
  std::vector<ProgJob> jobs;     // index-only dense programs precomputed per query (progbits_kernel)
  int32_t job_tiles = 0;
  std::vector<int32_t> invids;
  int64_t rk_ctab_records = 0;   // query_kernel_rkey: container records of every inverted leaf (id, key)
  std::vector<uint32_t> cand;    // query_kernel_cand: {segment, container index or ~0u, first doc, last doc} per unit
};

// Inverted leaves are expanded into doc bitmaps while their words stay within this budget (per query); the rest
// are evaluated per tile (bitmap_word).  PGPU_NO_INVEXP=1 turns the expansion off.
constexpr int64_t kInvExpMaxWords = (int64_t)1 << 29;  // 2 GiB of bitmaps
// query_kernel_cand: the leading inverted leaf's ids hold at most this share of each segment's docs (above it the tile
// sweep reads the expanded bitmap at stream speed), in at most this many containers per query
constexpr double kCandDensity = 1.0 / 16;
constexpr size_t kCandMaxUnits = (size_t)1 << 24;

int64_t inv_leaf(Packer& pk, const pgpu_segment* seg, const DevColumn& dc, const pgpu_filter_node& nd) {
  InvLeafX L{};
  L.dir = dc.inv_dir;
  L.ct = dc.inv_ct;
  L.data = dc.inv_data;
  L.nids = nd.num_ids;
  L.negate = nd.negate ? 1 : 0;
  L.num_docs = seg->num_docs;
  L.words = (int32_t)(((int64_t)seg->num_docs + PGPU_WT - 1) / PGPU_WT * 64);
  L.nkeys = (L.words + 2047) / 2048;
  for (const InvLeafX& o : pk.invx) {
    if (o.dir != L.dir || o.nids != L.nids || o.negate != L.negate) continue;
    if (!std::equal(nd.ids, nd.ids + nd.num_ids, pk.invids.begin() + (intptr_t)o.ids)) continue;
    return (int64_t)(intptr_t)o.out;
  }
  if (pk.raw_words + L.words > kInvExpMaxWords) return -1;
  L.ids = (const int32_t*)(intptr_t)pk.invids.size();
  pk.invids.insert(pk.invids.end(), nd.ids, nd.ids + nd.num_ids);
  L.out = (uint32_t*)(intptr_t)pk.raw_words;
  pk.raw_words += L.words;
  pk.invx.push_back(L);
  return (int64_t)(intptr_t)L.out;
}

// The bitmap word offset of a multi-value SCAN leaf (mvpred_kernel output), shared by identical leaves.
int64_t mv_leaf(Packer& pk, const pgpu_segment* seg, const HostColumn& hc, const pgpu_filter_node& nd, int* rc) {
  *rc = PGPU_OK;
  MvLeaf L{};
  L.fwd = (const uint32_t*)hc.fwd.p;
  L.off = (const int32_t*)hc.mv_off.p;
  L.num_docs = seg->num_docs;
  L.words = (int32_t)(((int64_t)seg->num_docs + PGPU_WT - 1) / PGPU_WT * 64);
  L.bits = hc.bits;
  L.negate = nd.negate ? 1 : 0;
  const int32_t card = hc.fwd_card;
  std::vector<uint32_t> set;
  if (nd.pred == PGPU_PRED_RANGE) {
    L.lo = std::max(0, nd.lo);
    L.hi = std::max(L.lo, std::min(nd.hi, card));
  } else if (nd.pred == PGPU_PRED_SET) {
    set.assign(((size_t)card + 31) / 32 + 1, 0u);
    for (int k = 0; k < nd.num_ids; ++k) {
      const int32_t id = nd.ids[k];
      if (id < 0 || id >= card) {
        *rc = fail(PGPU_E_INVALID, "SET id %d out of range", id);
        return -1;
      }
      set[id >> 5] |= 1u << (id & 31);
    }
  } else {
    *rc = fail(PGPU_E_INVALID, "predicate kind %d", nd.pred);
    return -1;
  }
  for (const MvLeaf& o : pk.mvs) {
    if (o.off != L.off || o.negate != L.negate || o.lo != L.lo || o.hi != L.hi || (o.set == nullptr) != set.empty())
      continue;
    if (!set.empty() && !std::equal(set.begin(), set.end(), pk.mvsets.begin() + (intptr_t)o.set - 1)) continue;
    return (int64_t)(intptr_t)o.out;
  }
  // set offsets are stored + 1 so that null means "RANGE"
  L.set = set.empty() ? nullptr : (const uint32_t*)(intptr_t)(pk.mvsets.size() + 1);
  pk.mvsets.insert(pk.mvsets.end(), set.begin(), set.end());
  L.out = (uint32_t*)(intptr_t)pk.raw_words;
  pk.raw_words += L.words;
  pk.mvs.push_back(L);
  return (int64_t)(intptr_t)L.out;
}

// The bitmap word offset of a raw-value leaf (rawpred_kernel output), shared by identical leaves of one segment
// (the exact-statistics pass converts every program a second time).
int64_t raw_leaf(Packer& pk, const pgpu_segment* seg, const HostColumn& hc, const DevColumn& dc,
                 const pgpu_filter_node& nd, bool range_index, int* rc) {
  *rc = PGPU_OK;
  RawLeaf L{};
  L.values = dc.dict;
  L.num_docs = seg->num_docs;
  L.words = (int32_t)(((int64_t)seg->num_docs + PGPU_WT - 1) / PGPU_WT * 64);
  L.vtype = hc.dict_type;
  L.pred = nd.pred;
  L.negate = nd.negate ? 1 : 0;
  const bool fp = hc.dict_type == PGPU_FLOAT || hc.dict_type == PGPU_DOUBLE;
  if (!nd.values && !(nd.pred == PGPU_PRED_SET && nd.num_ids == 0)) {
    *rc = fail(PGPU_E_INVALID, "raw-value leaf on column %d without values", nd.column);
    return -1;
  }
  std::vector<int64_t> set;
  if (nd.pred == PGPU_PRED_RANGE) {
    if (range_index) {  // RangeIndexBasedFilterOperator: the evaluator's bounds, inclusive (ordinals for floats)
      L.flags = PGPU_RAW_RANGE_LO_INCL | PGPU_RAW_RANGE_HI_INCL | (fp ? PGPU_RAW_RANGE_ORDINAL : 0);
    } else {
      L.flags = (nd.lo ? PGPU_RAW_RANGE_LO_INCL : 0) | (nd.hi ? PGPU_RAW_RANGE_HI_INCL : 0);
    }
    int64_t b[2];
    memcpy(b, nd.values, 16);
    if (fp && range_index)
      for (int k = 0; k < 2; ++k) {
        double d;
        memcpy(&d, &b[k], 8);
        if (d != d) d = -INFINITY;
        memcpy(&b[k], &d, 8);
      }
    L.lo = b[0];
    L.hi = b[1];
  } else if (nd.pred == PGPU_PRED_SET) {
    if (nd.num_ids < 0) {
      *rc = fail(PGPU_E_INVALID, "raw SET of %d values", nd.num_ids);
      return -1;
    }
    set.resize(nd.num_ids);
    if (nd.num_ids) memcpy(set.data(), nd.values, 8ull * nd.num_ids);
    if (fp)  // members compare by the order-preserving key of their bits (a bijection: fastutil set semantics)
      for (int64_t& k : set) k = k >= 0 ? k : (k ^ 0x7FFFFFFFFFFFFFFFll);
    std::sort(set.begin(), set.end());
    set.erase(std::unique(set.begin(), set.end()), set.end());
    L.nvals = (int32_t)set.size();
  } else {
    *rc = fail(PGPU_E_INVALID, "raw-value predicate kind %d", nd.pred);
    return -1;
  }
  for (size_t i = 0; i < pk.raws.size(); ++i) {
    const RawLeaf& o = pk.raws[i];
    if (o.values != L.values || o.pred != L.pred || o.negate != L.negate || o.flags != L.flags || o.lo != L.lo ||
        o.hi != L.hi || o.nvals != L.nvals)
      continue;
    const int64_t vo = (int64_t)(intptr_t)o.vals;
    if (L.nvals && !std::equal(set.begin(), set.end(), pk.rawvals.begin() + vo)) continue;
    return (int64_t)(intptr_t)o.out;
  }
  L.vals = (const int64_t*)(intptr_t)pk.rawvals.size();
  pk.rawvals.insert(pk.rawvals.end(), set.begin(), set.end());
  L.out = (uint32_t*)(intptr_t)pk.raw_words;
  pk.raw_words += L.words;
  pk.raws.push_back(L);
  return (int64_t)(intptr_t)L.out;
}

// Convert one prefix-order filter program into slot-resolved device instructions appended to pk.instrs.
int convert_filter(const pgpu_query_desc* q, const pgpu_segment_plan& sp, const pgpu_filter_node* nodes, int count,
                   const pgpu_segment* seg, Packer& pk) {
  struct Frame {
    int kind;  // 0 AND, 1 OR, 2 NOT
    int slot;
    int care;  // care slot of this frame's children
    int outer_care;
    std::vector<int> patch;  // AND_CHILD instructions to patch with the AND_END index
  };
  std::vector<Frame> st;
  const int base = (int)pk.instrs.size();
  int cur = 0;     // slot the next node writes
  int care = -1;   // care slot of the next node
  auto emit = [&](DevInstr in) {
    in.stage_off = -1;
    if (in.pred != 2 && in.op != PGPU_I_SORTED)  // LIST ids and SORTED inline ranges keep theirs
      for (int k = 0; k < 8; ++k) in.ids[k] = 0xFFFFFFFFu;
    pk.instrs.push_back(in);
    return (int)pk.instrs.size() - 1 - base;
  };
  auto close_nots = [&]() {
    while (!st.empty() && st.back().kind == 2) {
      DevInstr in{};
      in.op = PGPU_I_NOT;
      in.dst = in.src = st.back().slot;
      in.care = st.back().outer_care;
      emit(in);
      cur = st.back().slot;
      care = st.back().outer_care;
      st.pop_back();
    }
  };
  auto col_of = [&](int32_t qc, const DevColumn** out) -> int {
    if (qc < 0 || qc >= q->num_columns) return fail(PGPU_E_INVALID, "filter column %d", qc);
    const int32_t slot = sp.column_map[qc];
    if (slot < 0 || slot >= (int32_t)seg->dev.size()) return fail(PGPU_E_INVALID, "filter column %d slot %d", qc, slot);
    *out = &seg->dev[slot];
    return PGPU_OK;
  };
  for (int i = 0; i < count; ++i) {
    const pgpu_filter_node& nd = nodes[i];
    if (cur >= PGPU_MAX_SLOTS - 1)
      return fail(PGPU_E_UNSUPPORTED, "filter nesting deeper than %d", PGPU_MAX_SLOTS - 1);
    DevInstr in{};
    in.col = nd.column;
    in.negate = nd.negate ? 1 : 0;
    in.dst = cur;
    in.care = care;
    switch (nd.op) {
      case PGPU_F_MATCH_ALL:
      case PGPU_F_EMPTY:
        in.op = nd.op == PGPU_F_MATCH_ALL ? PGPU_I_ALL : PGPU_I_EMPTY;
        emit(in);
        close_nots();
        break;
      case PGPU_F_SCAN: {
        const DevColumn* c;
        int rc = col_of(nd.column, &c);
        if (rc) return rc;
        if (c->kind == PGPU_COL_NONE) return fail(PGPU_E_INVALID, "SCAN on column %d without forward index", nd.column);
        if (c->kind == PGPU_COL_RAW) return fail(PGPU_E_INVALID, "SCAN on raw column %d (use RAW_SCAN)", nd.column);
        if (c->kind == PGPU_COL_MV) {
          // MVScanDocIdIterator: the applyMV bitmap, its entries (row lengths) counted on the host (nostat)
          const int64_t woff = mv_leaf(pk, seg, seg->cols[sp.column_map[nd.column]], nd, &rc);
          if (rc) return rc;
          in.op = PGPU_I_BITS;
          in.kind = PGPU_COL_MV;
          in.negate = 0;  // folded into the bitmap
          in.nostat = 1;
          in.fwd = (const uint32_t*)(intptr_t)woff;
          const int idx = emit(in);
          pk.bits_instrs.push_back(base + idx);
          close_nots();
          break;
        }
        in.op = PGPU_I_SCAN;
        in.pred = nd.pred;
        in.bits = c->bits;
        in.kind = c->kind;
        in.card = c->card;
        in.fwd = c->fwd;
        in.sorted = c->sorted;
        if (nd.pred == PGPU_PRED_RANGE) {
          in.lo = std::max(0, nd.lo);
          in.hi = std::min(nd.hi, c->card);
          if (in.hi < in.lo) in.hi = in.lo;
        } else if (nd.pred == PGPU_PRED_SET && c->card <= 64) {
          in.pred = 3;  // MASK: membership bit of a 64-bit id mask held in two SGPRs (lo, hi)
          uint64_t mask = 0;
          for (int k = 0; k < nd.num_ids; ++k) {
            const int32_t id = nd.ids[k];
            if (id < 0 || id >= c->card) return fail(PGPU_E_INVALID, "SET id %d out of range", id);
            mask |= 1ull << id;
          }
          in.lo = (int32_t)(uint32_t)mask;
          in.hi = (int32_t)(uint32_t)(mask >> 32);
        } else if (nd.pred == PGPU_PRED_SET && nd.num_ids <= 8) {
          in.pred = 2;  // LIST: compared in registers, ids inline
          in.n = nd.num_ids;
          for (int k = 0; k < 8; ++k) in.ids[k] = 0xFFFFFFFFu;
          for (int k = 0; k < nd.num_ids; ++k) {
            const int32_t id = nd.ids[k];
            if (id < 0 || id >= c->card) return fail(PGPU_E_INVALID, "SET id %d out of range", id);
            in.ids[k] = (uint32_t)id;
          }
        } else if (nd.pred == PGPU_PRED_SET) {
          in.pool_off = (int32_t)pk.pool.size();
          pk.pool.resize(pk.pool.size() + (c->card + 31) / 32 + 1, 0);
          for (int k = 0; k < nd.num_ids; ++k) {
            const int32_t id = nd.ids[k];
            if (id < 0 || id >= c->card) return fail(PGPU_E_INVALID, "SET id %d out of range", id);
            pk.pool[in.pool_off + (id >> 5)] |= (int32_t)(1u << (id & 31));
          }
        } else {
          return fail(PGPU_E_INVALID, "predicate kind %d", nd.pred);
        }
        emit(in);
        close_nots();
        break;
      }
      case PGPU_F_RAW_SCAN:
      case PGPU_F_RANGE_INDEX: {
        const DevColumn* c;
        int rc = col_of(nd.column, &c);
        if (rc) return rc;
        const HostColumn& hc = seg->cols[sp.column_map[nd.column]];
        const bool ri = nd.op == PGPU_F_RANGE_INDEX;
        if (ri && !hc.range_index) return fail(PGPU_E_INVALID, "RANGE_INDEX leaf on column %d without range index", nd.column);
        if (ri && nd.pred != PGPU_PRED_RANGE) return fail(PGPU_E_INVALID, "RANGE_INDEX leaf with a non-RANGE predicate");
        if (ri && hc.range_index == 1) pk.legacy_range = true;
        const int32_t nostat = ri && hc.range_index == 2 ? 1 : 0;
        if (c->kind != PGPU_COL_RAW) {
          if (!ri) return fail(PGPU_E_INVALID, "RAW_SCAN on dictionary-encoded column %d", nd.column);
          // range index of a dictionary column: its dict-id range evaluated like a scan leaf, counted as the index
          pgpu_filter_node sn = nd;
          sn.op = PGPU_F_SCAN;
          rc = convert_filter(q, sp, &sn, 1, seg, pk);
          if (rc) return rc;
          // convert_filter appended one SCAN leaf writing slot 0 with valid-docs care: re-target it
          DevInstr& li = pk.instrs.back();
          li.dst = cur;
          li.care = care;
          li.nostat = nostat;
          close_nots();
          break;
        }
        const int64_t woff = raw_leaf(pk, seg, hc, *c, nd, ri, &rc);
        if (rc) return rc;
        in.op = PGPU_I_BITS;
        in.kind = PGPU_COL_RAW;
        in.negate = 0;  // folded into the bitmap
        in.nostat = nostat;
        in.fwd = (const uint32_t*)(intptr_t)woff;
        const int idx = emit(in);
        pk.bits_instrs.push_back(base + idx);
        close_nots();
        break;
      }
      case PGPU_F_INVERTED: {
        const DevColumn* c;
        int rc = col_of(nd.column, &c);
        if (rc) return rc;
        if (!c->inv_dir) return fail(PGPU_E_INVALID, "INVERTED on column %d without inverted index", nd.column);
        for (int k = 0; k < nd.num_ids; ++k)
          if (nd.ids[k] < 0 || nd.ids[k] >= c->card) return fail(PGPU_E_INVALID, "bitmap id %d out of range", nd.ids[k]);
        static const bool no_invexp = getenv("PGPU_NO_INVEXP") && atoi(getenv("PGPU_NO_INVEXP")) != 0;
        if (!no_invexp && nd.num_ids > 0) {
          const int64_t woff = inv_leaf(pk, seg, *c, nd);
          if (woff >= 0) {  // the expanded bitmap as a BITS leaf (a bitmap leaf reads no entries)
            in.op = PGPU_I_BITS;
            in.kind = PGPU_COL_FIXED_BIT;
            in.negate = 0;
            in.nostat = 1;
            in.fwd = (const uint32_t*)(intptr_t)woff;
            const int idx = emit(in);
            pk.bits_instrs.push_back(base + idx);
            close_nots();
            break;
          }
        }
        in.op = PGPU_I_INV;
        in.pool_off = (int32_t)pk.pool.size();
        in.n = nd.num_ids;
        for (int k = 0; k < nd.num_ids; ++k) {
          if (nd.ids[k] < 0 || nd.ids[k] >= c->card) return fail(PGPU_E_INVALID, "bitmap id %d out of range", nd.ids[k]);
          pk.pool.push_back(nd.ids[k]);
        }
        emit(in);
        close_nots();
        break;
      }
      case PGPU_F_SORTED: {
        in.op = PGPU_I_SORTED;
        std::vector<std::pair<int32_t, int32_t>> r;
        for (int k = 0; k < nd.num_ids; ++k) {
          int32_t s = std::max(0, nd.ids[2 * k]), e = std::min(nd.ids[2 * k + 1], seg->num_docs - 1);
          if (s <= e) r.emplace_back(s, e);
        }
        std::sort(r.begin(), r.end());
        in.pool_off = (int32_t)pk.pool.size();
        int n = 0;
        for (auto& x : r) {
          if (n && x.first <= pk.pool.back() + 1) {
            pk.pool.back() = std::max(pk.pool.back(), x.second);
          } else {
            pk.pool.push_back(x.first);
            pk.pool.push_back(x.second);
            ++n;
          }
        }
        in.n = n;
        // up to four ranges also inline in the instruction (ids[2k], ids[2k + 1]): the per-tile leaf then reads no
        // memory beyond the instruction's scalar loads
        for (int k = 0; k < 8; ++k) in.ids[k] = 0xFFFFFFFFu;
        for (int k = 0; k < n && k < 4; ++k) {
          in.ids[2 * k] = (uint32_t)pk.pool[in.pool_off + 2 * k];
          in.ids[2 * k + 1] = (uint32_t)pk.pool[in.pool_off + 2 * k + 1];
        }
        emit(in);
        close_nots();
        break;
      }
      case PGPU_F_AND_BEGIN:
      case PGPU_F_OR_BEGIN: {
        const bool is_and = nd.op == PGPU_F_AND_BEGIN;
        in.op = is_and ? PGPU_I_AND_BEGIN : PGPU_I_OR_BEGIN;
        emit(in);
        Frame f;
        f.kind = is_and ? 0 : 1;
        f.slot = cur;
        f.outer_care = care;
        f.care = is_and ? cur : care;
        st.push_back(f);
        cur = f.slot + 1;
        care = f.care;
        break;
      }
      case PGPU_F_AND_CHILD_END:
      case PGPU_F_OR_CHILD_END: {
        const bool is_and = nd.op == PGPU_F_AND_CHILD_END;
        if (st.empty() || st.back().kind != (is_and ? 0 : 1)) return fail(PGPU_E_INVALID, "unbalanced filter at node %d", i);
        in.op = is_and ? PGPU_I_AND_CHILD : PGPU_I_OR_CHILD;
        in.dst = st.back().slot;
        in.src = st.back().slot + 1;
        in.care = st.back().outer_care;
        const int idx = emit(in);
        if (is_and) st.back().patch.push_back(idx);
        cur = st.back().slot + 1;
        care = st.back().care;
        break;
      }
      case PGPU_F_AND_END:
      case PGPU_F_OR_END: {
        const bool is_and = nd.op == PGPU_F_AND_END;
        if (st.empty() || st.back().kind != (is_and ? 0 : 1)) return fail(PGPU_E_INVALID, "unbalanced filter at node %d", i);
        in.op = is_and ? PGPU_I_AND_END : PGPU_I_OR_END;
        in.dst = st.back().slot;
        const int idx = emit(in);
        for (int p : st.back().patch) pk.instrs[base + p].jump = idx;
        cur = st.back().slot;
        care = st.back().outer_care;
        st.pop_back();
        close_nots();
        break;
      }
      case PGPU_F_NOT: {
        Frame f;
        f.kind = 2;
        f.slot = cur;
        f.outer_care = care;
        f.care = care;
        st.push_back(f);
        break;
      }
      default:
        return fail(PGPU_E_INVALID, "filter op %d", nd.op);
    }
  }
  if (!st.empty()) return fail(PGPU_E_INVALID, "unterminated filter program");
  if (count > 0 && cur != 0) return fail(PGPU_E_INVALID, "filter program leaves slot %d", cur);
  return PGPU_OK;
}

// ---- per-segment execution plan: which filter children stream through LDS, which run per candidate doc --------
struct SegView {
  const pgpu_query_desc* q;
  const pgpu_segment_plan* sp;
  const pgpu_segment* seg;
  const pgpu_filter_node* nd;
  int n;
  const HostColumn* host(int qc) const { return &seg->cols[sp->column_map[qc]]; }
  const DevColumn* dev(int qc) const { return &seg->dev[sp->column_map[qc]]; }
};

// Walk the subtree at node i: estimated fraction of docs it keeps (uniform-id model for scans; exact bitmap and
// sorted-range cardinalities), plus the query columns of its SCAN leaves.  Returns the index past the subtree or
// -1 on malformed input.  Estimates only steer the staging decision; results never depend on them.
int analyze(const SegView& v, int i, double* sel, std::vector<int>* scans) {
  if (i < 0 || i >= v.n) return -1;
  const pgpu_filter_node& x = v.nd[i];
  const double nd = std::max(1, v.seg->num_docs);
  auto valid_col = [&](int qc) {
    return qc >= 0 && qc < v.q->num_columns && v.sp->column_map[qc] >= 0 &&
           v.sp->column_map[qc] < (int32_t)v.seg->dev.size();
  };
  switch (x.op) {
    case PGPU_F_MATCH_ALL: *sel = 1.0; return i + 1;
    case PGPU_F_EMPTY: *sel = 0.0; return i + 1;
    case PGPU_F_RAW_SCAN:
    case PGPU_F_RANGE_INDEX:
      if (!valid_col(x.column)) return -1;
      if (v.dev(x.column)->kind == PGPU_COL_RAW) {  // a precomputed bitmap word per lane: never staged
        *sel = 0.5;
        return i + 1;
      }
      if (x.op == PGPU_F_RAW_SCAN) return -1;
      [[fallthrough]];  // range index of a dictionary column: a dict-id range scan on the GPU
    case PGPU_F_SCAN: {
      if (!valid_col(x.column)) return -1;
      if (v.dev(x.column)->kind == PGPU_COL_MV) {  // mvpred_kernel's bitmap word per lane: never staged
        *sel = 0.5;
        return i + 1;
      }
      const double card = std::max(1, v.dev(x.column)->card);
      double s = x.pred == PGPU_PRED_RANGE ? std::max(0, x.hi - x.lo) / card : std::max(0, x.num_ids) / card;
      s = std::min(1.0, s);
      *sel = x.negate ? 1.0 - s : s;
      scans->push_back(x.column);
      return i + 1;
    }
    case PGPU_F_INVERTED: {
      if (!valid_col(x.column)) return -1;
      const HostColumn* h = v.host(x.column);
      double docs = 0;
      for (int k = 0; k < x.num_ids; ++k)
        if (x.ids[k] >= 0 && x.ids[k] < (int32_t)h->inv_cards.size()) docs += h->inv_cards[x.ids[k]];
      const double s = std::min(1.0, docs / nd);
      *sel = x.negate ? 1.0 - s : s;
      return i + 1;
    }
    case PGPU_F_SORTED: {
      double docs = 0;
      for (int k = 0; k < x.num_ids; ++k) docs += std::max(0, x.ids[2 * k + 1] - x.ids[2 * k] + 1);
      const double s = std::min(1.0, docs / nd);
      *sel = x.negate ? 1.0 - s : s;
      return i + 1;
    }
    case PGPU_F_AND_BEGIN:
    case PGPU_F_OR_BEGIN: {
      const bool is_and = x.op == PGPU_F_AND_BEGIN;
      double acc = 1.0;  // AND: product of selectivities; OR: product of (1 - s)
      int j = i + 1;
      while (j < v.n && v.nd[j].op != (is_and ? PGPU_F_AND_END : PGPU_F_OR_END)) {
        double cs;
        j = analyze(v, j, &cs, scans);
        if (j < 0 || j >= v.n || v.nd[j].op != (is_and ? PGPU_F_AND_CHILD_END : PGPU_F_OR_CHILD_END)) return -1;
        acc *= is_and ? cs : 1.0 - cs;
        ++j;
      }
      if (j >= v.n) return -1;
      *sel = is_and ? acc : 1.0 - acc;
      return j + 1;
    }
    case PGPU_F_NOT: {
      double cs;
      const int j = analyze(v, i + 1, &cs, scans);
      *sel = 1.0 - cs;
      return j;
    }
    default:
      return -1;
  }
}

// Fraction of a b-bit column's 32-B sectors that hold at least one doc when docs survive with density rho.
double sector_touch(double rho, int bits) {
  if (rho >= 1.0) return 1.0;
  if (rho <= 0.0) return 0.0;
  return 1.0 - std::pow(1.0 - rho, 256.0 / bits);
}

// A column is streamed (dense) when at least half of its sectors would be read anyway.
constexpr double kDenseTouch = 0.5;
// Aggregation columns are staged densely only when nearly every 32-B sector holds a matched doc: below that the
// self-loading kernels' candidate gathers win (config 2, 9.4 % of docs, 16-bit metric, 79 % of sectors touched:
// dense 2.37 ms, candidates 1.40 ms; 50 % of docs: dense 3.0 ms, candidates 3.8 ms).  PGPU_DENSE_TOUCH overrides.
constexpr double kDenseAggTouch = 0.95;
// Aggregation-only queries: the aggregated columns are streamed bit-sliced beside the filter (PGPU_AM_SLICED) when
// at least this share of their 128-B lines holds a matched doc -- a gathered 4-B value moves a whole line
// (tools/gather_policy_bench.hip), so the candidate gathers would read those lines anyway, at gather speed.
// PGPU_SLICED_TOUCH overrides; PGPU_NO_SLICED_AGG=1 turns the mode off.
constexpr double kSlicedAggTouch = 0.5;
double line_touch(double rho, int bits) {
  if (rho >= 1.0) return 1.0;
  if (rho <= 0.0) return 0.0;
  return 1.0 - std::pow(1.0 - rho, 1024.0 / bits);
}
constexpr int kMaxSlotBytes = 27 * 1024;  // keeps >= 3 ring slots next to the consumer areas

// Prefix pre-filter for the register-direct kernel (DevSeg::pfx_*): when the residual program is one SCAN leaf on a
// fixed-bit column with a bit-sliced copy, the top PGPU_PFX_PLANES planes of that column can be streamed beside the
// fast leaf, and a candidate whose id's top bits fall outside every matching id run is rejected without its
// gather.  Each gather moves a whole 128-B line (tools/gather_policy_bench.hip: ~50 G random 4-B loads/s = 6.5 TB/s
// of lines, whatever the cache policy), a plane 256 B per 2048-doc tile: worth it when the candidates per tile x
// 128 B x the rejected share exceed the planes' bytes.  Config 5 (16 candidates per tile, accountId EQ): 4.6 ->
// 3.6 KB of DRAM traffic per tile.
void plan_prefix(const SegView& v, const Packer& pk, double rho_dense, DevSeg& ds) {
  ds.pfx_col = -1;
  ds.pfx_nr = 0;
  for (int r = 0; r < PGPU_SLICE_RANGES; ++r) ds.pfx_rng[r][0] = ds.pfx_rng[r][1] = 0;
  static const bool no_pfx = getenv("PGPU_NO_PREFIX") && atoi(getenv("PGPU_NO_PREFIX")) != 0;
  if (no_pfx || ds.rprog_len != 1) return;
  const DevInstr& in = pk.instrs[ds.rprog_begin];
  if (in.op != PGPU_I_SCAN || in.kind != PGPU_COL_FIXED_BIT || in.negate || in.nostat) return;
  const DevColumn* dc = v.dev(in.col);
  const int K = PGPU_PFX_PLANES;
  if (!dc->sliced || dc->bits <= K || dc->bits > 31) return;
  std::vector<std::pair<uint64_t, uint64_t>> runs;  // matching ids [a, b)
  if (in.pred == 0) {
    if (in.hi > in.lo) runs.emplace_back((uint64_t)(uint32_t)in.lo, (uint64_t)(uint32_t)in.hi);
  } else if (in.pred == 2) {
    for (int k = 0; k < 8; ++k)
      if (in.ids[k] != 0xFFFFFFFFu) runs.emplace_back((uint64_t)in.ids[k], (uint64_t)in.ids[k] + 1);
  } else if (in.pred == 3) {
    const uint64_t mask = (uint64_t)(uint32_t)in.lo | ((uint64_t)(uint32_t)in.hi << 32);
    for (int i = 0; i < 64; ++i)
      if ((mask >> i) & 1u) runs.emplace_back((uint64_t)i, (uint64_t)i + 1);
  } else {
    return;
  }
  const int sh = dc->bits - K;
  std::vector<std::pair<uint32_t, uint32_t>> pr;  // prefix ranges, merged
  for (auto& r : runs) pr.emplace_back((uint32_t)(r.first >> sh), (uint32_t)(((r.second - 1) >> sh) + 1));
  std::sort(pr.begin(), pr.end());
  std::vector<std::pair<uint32_t, uint32_t>> merged;
  for (auto& r : pr) {
    if (!merged.empty() && r.first <= merged.back().second) merged.back().second = std::max(merged.back().second, r.second);
    else merged.push_back(r);
  }
  if (merged.empty() || (int)merged.size() > PGPU_SLICE_RANGES) return;
  double covered = 0;
  for (auto& r : merged) covered += r.second - r.first;
  covered /= (double)(1u << K);
  const double cand = rho_dense * PGPU_WT;  // candidates per 2048-doc tile
  if (cand * 128.0 * (1.0 - covered) <= 256.0 * K) return;
  ds.pfx_col = in.col;
  ds.pfx_nr = (int32_t)merged.size();
  for (size_t r = 0; r < merged.size(); ++r) {
    ds.pfx_rng[r][0] = merged[r].first;
    ds.pfx_rng[r][1] = merged[r].second;
  }
}

int plan_segment(const pgpu_query_desc* q, const pgpu_segment_plan& sp, const pgpu_segment* seg,
                 const DevParams& p, Packer& pk, DevSeg& ds) {
  SegView v{q, &sp, seg, sp.filter, sp.num_filter_nodes};
  // top-level AND children (node ranges [begin, end))
  std::vector<std::pair<int, int>> kids;
  if (v.n > 0) {
    double s;
    std::vector<int> scans;
    const int e = analyze(v, 0, &s, &scans);
    if (e != v.n) return fail(PGPU_E_INVALID, "malformed filter program");
    if (v.nd[0].op == PGPU_F_AND_BEGIN) {
      int j = 1;
      while (v.nd[j].op != PGPU_F_AND_END) {
        const int ce = analyze(v, j, &s, &scans);
        kids.emplace_back(j, ce);
        j = ce + 1;
      }
    } else {
      kids.emplace_back(0, v.n);
    }
  }
  // dense prefix of the children: every scan column of a dense child is read with >= kDenseTouch sector density
  double rho = 1.0, rho_dense = 1.0;
  bool residual = false;
  std::vector<int> dense_kids, resid_kids, staged;
  auto add_stage = [&](int qc) {
    if (std::find(staged.begin(), staged.end(), qc) == staged.end()) staged.push_back(qc);
  };
  for (size_t k = 0; k < kids.size(); ++k) {
    double s;
    std::vector<int> scans;
    analyze(v, kids[k].first, &s, &scans);
    bool dense = !residual;
    for (int qc : scans)
      if (dense && v.dev(qc)->kind == PGPU_COL_FIXED_BIT && sector_touch(rho, v.dev(qc)->bits) < kDenseTouch)
        dense = false;
    if (dense) {
      dense_kids.push_back((int)k);
      for (int qc : scans)
        if (v.dev(qc)->kind == PGPU_COL_FIXED_BIT) add_stage(qc);
    } else {
      residual = true;
      resid_kids.push_back((int)k);
    }
    rho *= s;
    if (dense) rho_dense *= s;
  }
  const size_t nfilter_stage = staged.size();
  // aggregation plan
  std::vector<int> aggcols;
  auto add_agg = [&](int qc) {
    if (std::find(aggcols.begin(), aggcols.end(), qc) == aggcols.end()) aggcols.push_back(qc);
  };
  for (int g = 0; g < q->num_group_columns; ++g) add_agg(q->group_columns[g]);
  for (int a = 0; a < q->num_aggs; ++a)
    if (q->aggs[a].fn != PGPU_AGG_COUNT) add_agg(q->aggs[a].column);
  int agg_mode;
  static const bool no_sliced = getenv("PGPU_NO_SLICED_AGG") && atoi(getenv("PGPU_NO_SLICED_AGG")) != 0;
  static const double sliced_touch = getenv("PGPU_SLICED_TOUCH") ? atof(getenv("PGPU_SLICED_TOUCH")) : kSlicedAggTouch;
  // (aggregation-only: p.mode is still undecided for dense group-by tables here)
  // every aggregation answered from value planes (SUM of whole int64 cells, MIN, MAX over an INT / LONG dictionary
  // of <= 24 value bits: sliced_tile's bit-sliced index), or at most two over id planes of <= 16 bits (ids queued,
  // values gathered in batches)
  bool sliced = !no_sliced && !aggcols.empty() && !residual && q->num_group_columns == 0 && !p.mv_gmask;
  bool all_bsi = true;
  int nvalue = 0;
  for (int a = 0; a < q->num_aggs; ++a) {
    if (q->aggs[a].fn == PGPU_AGG_COUNT) continue;
    ++nvalue;
    const DevColumn* dc = v.dev(q->aggs[a].column);
    const bool whole_sum = q->aggs[a].fn == PGPU_AGG_SUM || q->aggs[a].fn == PGPU_AGG_AVG;
    bool split = false;  // a SUM split into 21-bit part sections (pgpu_table_layout.agg_sum_parts == 3)
    for (int i = 0; i < p.nagg; ++i) split = split || (p.aggs[i].col == q->aggs[a].column && p.aggs[i].part != 0);
    const bool bsi = dc->vsliced && dc->vbits >= 1 && dc->vbits <= 24 &&
                     ((whole_sum && (dc->dict_type == PGPU_INT || dc->dict_type == PGPU_LONG) && !split) ||
                      q->aggs[a].fn == PGPU_AGG_MIN || q->aggs[a].fn == PGPU_AGG_MAX);
    all_bsi = all_bsi && bsi;
    // (a split SUM is three device aggregations: the id path's two LDS sub-queues hold one per query aggregation)
    // value planes alone serve a value-plane aggregation; the id planes (bit-sliced copy) the others
    sliced = sliced && !split && dc->kind == PGPU_COL_FIXED_BIT && (dc->sliced || bsi) &&
             line_touch(rho, bsi ? dc->vbits : dc->bits) >= sliced_touch;
  }
  if (sliced && !all_bsi) {  // the id-plane path reads every aggregated column's bit-sliced copy
    for (int qc : aggcols) sliced = sliced && v.dev(qc)->sliced && v.dev(qc)->bits >= 1 && v.dev(qc)->bits <= 16;
    sliced = sliced && nvalue <= 2;
  }
  if (aggcols.empty()) {
    agg_mode = PGPU_AM_COUNT;
  } else if (sliced) {
    agg_mode = PGPU_AM_SLICED;  // the aggregated columns' planes load into VGPRs per matched tile: nothing staged
  } else if (residual || p.mv_gmask) {  // multi-value group keys: expanded per candidate doc (sparse_agg_mv)
    agg_mode = PGPU_AM_SPARSE;
  } else {
    // the hash group-by computes 64-bit keys and slots per doc in the candidate path only
    bool dense = p.mode != PGPU_MODE_HASH;
    static const double touch = getenv("PGPU_DENSE_TOUCH") ? atof(getenv("PGPU_DENSE_TOUCH")) : kDenseAggTouch;
    for (int qc : aggcols) {
      const DevColumn* dc = v.dev(qc);
      const int b = dc->kind == PGPU_COL_RAW ? 8 * type_width(dc->dict_type) : dc->bits;
      dense &= (dc->kind == PGPU_COL_FIXED_BIT || dc->kind == PGPU_COL_RAW) && sector_touch(rho, b) >= touch;
    }
    agg_mode = dense ? PGPU_AM_DENSE : PGPU_AM_SPARSE;
    if (dense)
      for (int qc : aggcols)
        if (v.dev(qc)->kind == PGPU_COL_FIXED_BIT) add_stage(qc);
  }
  auto fits = [&]() {
    int instrs = 0, bytes = 0;
    for (int qc : staged) {
      instrs += pgpu_stage_instrs(v.dev(qc)->bits);
      bytes += pgpu_stage_region_bytes(v.dev(qc)->bits);
    }
    return staged.size() <= PGPU_MAX_STAGE && instrs <= PGPU_MAX_STAGE_INSTRS && bytes <= kMaxSlotBytes;
  };
  if (!fits() && agg_mode == PGPU_AM_DENSE) {
    staged.resize(nfilter_stage);
    agg_mode = PGPU_AM_SPARSE;
  }
  while (!fits()) staged.pop_back();  // remaining scans read their tiles straight from HBM
  // programs
  auto build = [&](const std::vector<int>& idx, std::vector<pgpu_filter_node>& out) {
    pgpu_filter_node mark{};
    if (idx.size() > 1) {
      mark.op = PGPU_F_AND_BEGIN;
      out.push_back(mark);
    }
    for (int k : idx) {
      for (int i = kids[k].first; i < kids[k].second; ++i) out.push_back(v.nd[i]);
      if (idx.size() > 1) {
        mark.op = PGPU_F_AND_CHILD_END;
        out.push_back(mark);
      }
    }
    if (idx.size() > 1) {
      mark.op = PGPU_F_AND_END;
      out.push_back(mark);
    }
  };
  std::vector<pgpu_filter_node> dn, rn;
  build(dense_kids, dn);
  build(resid_kids, rn);
  ds.prog_begin = (int32_t)pk.instrs.size();
  int rc = convert_filter(q, sp, dn.data(), (int)dn.size(), seg, pk);
  if (rc) return rc;
  ds.prog_len = (int32_t)pk.instrs.size() - ds.prog_begin;
  ds.nbits = 0;
  for (int i = ds.prog_begin; i < ds.prog_begin + ds.prog_len; ++i) {
    DevInstr& in = pk.instrs[i];
    if (in.op != PGPU_I_BITS) continue;
    if (ds.nbits < PGPU_PREBITS) {
      in.n = ds.nbits;
      ds.bits_w[ds.nbits++] = in.fwd;  // a word offset into the workspace bitmaps until launch
    } else {
      in.n = -1;
    }
  }
  ds.rprog_begin = (int32_t)pk.instrs.size();
  rc = convert_filter(q, sp, rn.data(), (int)rn.size(), seg, pk);
  if (rc) return rc;
  ds.rprog_len = (int32_t)pk.instrs.size() - ds.rprog_begin;
  plan_prefix(v, pk, rho_dense, ds);
  auto stage_index = [&](int qc) {
    for (size_t j = 0; j < staged.size(); ++j)
      if (staged[j] == qc) return (int)j;
    return -1;
  };
  // fast dense program: one staged SCAN leaf, or AND_BEGIN (SCAN AND_CHILD){2} AND_END, RANGE / MASK predicates
  ds.fast = 0;
  ds.fast_ins[0] = ds.fast_ins[1] = -1;
  {
    int nscan = 0, nand = 0;
    bool ok = ds.prog_len > 0;
    for (int i = 0; i < ds.prog_len && ok; ++i) {
      const DevInstr& in = pk.instrs[ds.prog_begin + i];
      if (in.op == PGPU_I_SCAN) {
        ok = nscan < 2 && in.kind == PGPU_COL_FIXED_BIT && stage_index(in.col) >= 0 && (in.pred == 0 || in.pred == 3);
        if (ok) ds.fast_ins[nscan++] = i;
      } else if (in.op == PGPU_I_AND_BEGIN) {
        ok = ++nand == 1 && i == 0;
      } else {
        ok = in.op == PGPU_I_AND_CHILD || in.op == PGPU_I_AND_END;
      }
    }
    if (ok && nscan >= 1 && (nand == 0 ? ds.prog_len == 1 : ds.prog_len == 2 * nscan + 2)) ds.fast = nscan;
  }
  // bit-sliced fast leaves (kernel sliced_ranges): the column has a bit-sliced copy, only the dense filter reads
  // its staged tiles (it is not an aggregation / group column decoded from the slot, nor the other fast leaf's
  // column), and the predicate is a RANGE or a 64-id MASK whose ids (or their complement) form <= 4 runs
  ds.stage_sliced = 0;
  for (int j = 0; j < 2; ++j) {
    ds.f_nr[j] = ds.f_sneg[j] = 0;
    for (int r = 0; r < PGPU_SLICE_RANGES; ++r) ds.f_rng[j][r][0] = ds.f_rng[j][r][1] = 0;
  }
  for (int j = 0; j < ds.fast; ++j) {
    const DevInstr& in = pk.instrs[ds.prog_begin + ds.fast_ins[j]];
    const DevColumn* dc = v.dev(in.col);
    if (!dc->sliced || dc->bits < 1 || dc->bits > 31) continue;
    if (agg_mode == PGPU_AM_DENSE && std::find(aggcols.begin(), aggcols.end(), in.col) != aggcols.end()) continue;
    if (ds.fast == 2 && pk.instrs[ds.prog_begin + ds.fast_ins[1 - j]].col == in.col) continue;
    const uint64_t top = 1ull << dc->bits;
    std::vector<std::pair<uint32_t, uint32_t>> rng;
    bool neg = in.negate != 0;
    if (in.pred == 0) {
      if (in.lo < 0 || in.hi < 0 || (uint64_t)in.lo > top || (uint64_t)in.hi > top) continue;
      rng.emplace_back((uint32_t)in.lo, (uint32_t)in.hi);
    } else {
      const uint64_t mask = (uint64_t)(uint32_t)in.lo | ((uint64_t)(uint32_t)in.hi << 32);
      const int n = (int)std::min<uint64_t>(64, top);
      auto runs = [&](bool bit) {
        std::vector<std::pair<uint32_t, uint32_t>> out;
        for (int i = 0; i < n;) {
          if (((mask >> i) & 1u) != (uint64_t)bit) { ++i; continue; }
          int e = i;
          while (e < n && ((mask >> e) & 1u) == (uint64_t)bit) ++e;
          out.emplace_back((uint32_t)i, (uint32_t)e);
          i = e;
        }
        return out;
      };
      auto set = runs(true), clr = runs(false);
      if (set.size() <= clr.size()) rng = set;
      else { rng = clr; neg = !neg; }
      if (rng.empty()) rng.emplace_back(0u, 0u);  // matches no id
      if ((int)rng.size() > PGPU_SLICE_RANGES) continue;
    }
    ds.f_nr[j] = (int32_t)rng.size();
    ds.f_sneg[j] = neg ? 1 : 0;
    for (size_t r = 0; r < rng.size(); ++r) {
      ds.f_rng[j][r][0] = rng[r].first;
      ds.f_rng[j][r][1] = rng[r].second;
    }
    ds.stage_sliced |= 1 << stage_index(in.col);
  }
  // staging layout
  std::vector<int> stage_offs;
  ds.nstage = (int32_t)staged.size();
  ds.stage_instrs = 0;
  int off = 0;
  for (size_t j = 0; j < staged.size(); ++j) {
    const int b = v.dev(staged[j])->bits;
    const bool sl = (ds.stage_sliced >> j) & 1;
    ds.stage_col[j] = staged[j];
    ds.stage_off[j] = off;
    stage_offs.push_back(off);
    off += pgpu_stage_region_bytes(b, sl);
    ds.stage_instrs += pgpu_stage_instrs(b, sl);
  }
  for (int i = ds.prog_begin; i < ds.prog_begin + ds.prog_len; ++i) {
    DevInstr& in = pk.instrs[i];
    if (in.op != PGPU_I_SCAN) continue;
    const int j = stage_index(in.col);
    if (j >= 0) in.stage_off = stage_offs[j];
  }
  int64_t tb = 0;
  for (int qc : staged) tb += 256ll * v.dev(qc)->bits;
  // value planes of sliced aggregation DMA'd with the tile (DevSeg::nvstage, PGPU_VSTAGE=1): the self-loading
  // kernel's counted vmcnt then covers them too, where a plain load behind the DMAs waits for every DMA in flight.
  // Measured slower (config 2: 2.52 against 1.14 ms; config 3's query kernel 2.44 against 0.93 ms): the wider
  // slots cut the resident workgroups and the DMA depth more than the in-order waits cost, so it is opt-in.
  static const bool vstage = getenv("PGPU_VSTAGE") && atoi(getenv("PGPU_VSTAGE")) != 0;
  ds.nvstage = 0;
  if (agg_mode == PGPU_AM_SLICED && all_bsi && vstage) {
    std::vector<int> vcols;
    for (int a = 0; a < q->num_aggs; ++a)
      if (q->aggs[a].fn != PGPU_AGG_COUNT &&
          std::find(vcols.begin(), vcols.end(), q->aggs[a].column) == vcols.end())
        vcols.push_back(q->aggs[a].column);
    int vinstrs = 0, vbytes = 0;
    for (int qc : vcols) {
      vinstrs += (v.dev(qc)->vbits + 3) / 4;
      vbytes += 256 * v.dev(qc)->vbits;
    }
    if (vcols.size() <= 2 && staged.size() + vcols.size() <= PGPU_MAX_STAGE &&
        ds.stage_instrs + vinstrs <= PGPU_MAX_STAGE_INSTRS && off + vbytes <= kMaxSlotBytes) {
      for (int qc : vcols) {
        ds.vstage_col[ds.nvstage] = qc;
        ds.vstage_off[ds.nvstage++] = off;
        off += 256 * v.dev(qc)->vbits;
        tb += 256ll * v.dev(qc)->vbits;
      }
      ds.stage_instrs += vinstrs;
    }
  }
  pk.slot_bytes = std::max(pk.slot_bytes, off);
  pk.max_instrs = std::max(pk.max_instrs, ds.stage_instrs);
  pk.tile_bytes = std::max(pk.tile_bytes, tb);
  pk.est_matched += rho * seg->num_docs;
  ds.agg_mode = agg_mode;
  ds.nreg = -1;
  ds.reg_col[0] = ds.reg_col[1] = -1;
  if (agg_mode == PGPU_AM_DENSE && aggcols.size() <= 2) {
    ds.nreg = (int32_t)aggcols.size();
    for (size_t j = 0; j < aggcols.size(); ++j) ds.reg_col[j] = aggcols[j];
  }
  // An index-only dense program of several leaves (bitmap / expanded-bitmap / sorted, AND / OR / NOT) is evaluated
  // once per query for all of the segment's tiles (progbits_kernel) into a match bitmap; the query kernels then
  // read one word per lane and tile (DevSeg::single_bits).  Config 3: the interpreter's per-tile instruction
  // fetches and leaf loads were half of the query kernel.
  // Opt-in (PGPU_PROGBITS=1): measured slower on config 3 -- progbits_kernel 1.78 ms plus the query kernel's 0.92 ms
  // against 1.60 ms for the query kernel interpreting the program itself (the per-tile interpreter, not the leaf
  // loads, is the cost, and it moves with the program).
  const char* pbe = getenv("PGPU_PROGBITS");  // read per plan: tests switch it within one process
  const bool progbits = pbe && atoi(pbe) != 0;
  ds.single_bits = 0;
  if (progbits && ds.fast == 0 && ds.rprog_len == 0 && ds.prog_len > 1 && ds.ntiles > 0) {
    int leaves = 0;
    bool ok = true;
    for (int i = ds.prog_begin; i < ds.prog_begin + ds.prog_len; ++i) {
      const DevInstr& in = pk.instrs[i];
      if (in.op == PGPU_I_BITS) ok = ok && in.nostat, ++leaves;
      else if (in.op == PGPU_I_SORTED || in.op == PGPU_I_INV) ++leaves;
      else if (in.op == PGPU_I_SCAN) ok = false;
    }
    if (ok && leaves >= 2 && pk.raw_words + (int64_t)ds.ntiles * 64 <= kInvExpMaxWords) {
      ProgJob jb{};
      jb.nbits = ds.nbits;  // the leaves keep their slots: progbits loads their words together per tile
      for (int k = 0; k < ds.nbits; ++k) jb.bits_w[k] = ds.bits_w[k];
      jb.seg = (int32_t)pk.segs.size();
      jb.prog_begin = ds.prog_begin;
      jb.prog_len = ds.prog_len;
      jb.tile0 = pk.job_tiles;
      jb.ntiles = ds.ntiles;
      jb.out = (uint32_t*)(intptr_t)pk.raw_words;  // a word offset into the workspace bitmaps until launch
      pk.raw_words += (int64_t)ds.ntiles * 64;
      pk.job_tiles += ds.ntiles;
      pk.jobs.push_back(jb);
      DevInstr in{};
      in.op = PGPU_I_BITS;
      in.kind = PGPU_COL_FIXED_BIT;
      in.col = -1;
      in.care = -1;
      in.stage_off = -1;
      in.nostat = 1;
      in.n = 0;
      in.fwd = jb.out;
      for (int k = 0; k < 8; ++k) in.ids[k] = 0xFFFFFFFFu;
      pk.bits_instrs.push_back((int)pk.instrs.size());
      ds.prog_begin = (int32_t)pk.instrs.size();
      ds.prog_len = 1;
      pk.instrs.push_back(in);
      ds.nbits = 1;
      ds.bits_w[0] = jb.out;
      ds.single_bits = 1;
    }
  }
  return PGPU_OK;
}

// The index-only dense program of `ds` as a truth table over its leaves (DevSeg::ptt, query_kernel_rprog): leaves
// 0 .. nbits - 1 are its BITS slots, then up to two SORTED leaves with inline doc ranges.  False when the program
// reads anything else (SCAN / INV leaves load per tile) or counts scanned entries.  An AND's short-circuit only skips
// children whose rows nobody reads afterwards, so evaluating every instruction gives the interpreter's result.
bool program_truth_table(const Packer& pk, DevSeg& ds) {
  std::vector<int> sorted;
  int maxrow = 0;
  for (int i = ds.prog_begin; i < ds.prog_begin + ds.prog_len; ++i) {
    const DevInstr& in = pk.instrs[i];
    switch (in.op) {
      case PGPU_I_BITS:
        if (in.n < 0 || in.n >= ds.nbits || !in.nostat) return false;
        break;
      case PGPU_I_SORTED:
        if (in.n > 4) return false;
        sorted.push_back(i);
        break;
      case PGPU_I_ALL: case PGPU_I_EMPTY: case PGPU_I_AND_BEGIN: case PGPU_I_AND_CHILD: case PGPU_I_AND_END:
      case PGPU_I_OR_BEGIN: case PGPU_I_OR_CHILD: case PGPU_I_OR_END: case PGPU_I_NOT:
        break;
      default:
        return false;
    }
    maxrow = std::max({maxrow, in.dst, in.src, in.care});
  }
  if (ds.prog_len <= 0 || sorted.size() > 2 || ds.nbits + (int)sorted.size() > 5) return false;
  uint32_t tt = 0;
  std::vector<uint8_t> row((size_t)maxrow + 1);
  for (int t = 0; t < 32; ++t) {
    std::fill(row.begin(), row.end(), 0);
    for (int i = ds.prog_begin; i < ds.prog_begin + ds.prog_len; ++i) {
      const DevInstr& in = pk.instrs[i];
      const uint8_t care = in.care < 0 ? 1 : row[in.care];
      uint8_t* d = in.dst >= 0 ? &row[in.dst] : nullptr;
      switch (in.op) {
        case PGPU_I_ALL: *d = 1; break;
        case PGPU_I_EMPTY: *d = 0; break;
        case PGPU_I_BITS: *d = ((t >> in.n) & 1) & care; break;
        case PGPU_I_SORTED: {
          const int leaf = ds.nbits + (int)(std::find(sorted.begin(), sorted.end(), i) - sorted.begin());
          *d = (t >> leaf) & 1;
          break;
        }
        case PGPU_I_AND_BEGIN: *d = care; break;
        case PGPU_I_AND_CHILD: *d &= row[in.src]; break;
        case PGPU_I_OR_BEGIN: *d = 0; break;
        case PGPU_I_OR_CHILD: *d |= row[in.src]; break;
        case PGPU_I_NOT: *d = !row[in.src] & care; break;
        default: break;
      }
    }
    if (row[0]) tt |= 1u << t;
  }
  ds.ptt = tt;
  ds.pnsorted = (int32_t)sorted.size();
  for (size_t j = 0; j < 2; ++j) ds.psorted[j] = j < sorted.size() ? sorted[j] : 0;
  return true;
}

int pack_query(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_table_layout& L, Packer& pk, DevParams& p) {
  memset(&p, 0, sizeof(p));
  p.ncols = q->num_columns;
  p.ngcols = q->num_group_columns;
  p.nsec = L.num_sections;
  p.G = L.num_keys;
  p.flags = (q->flags & PGPU_Q_STATS) ? PGPU_FLAG_STATS : 0;
  if (profile_enabled()) p.flags |= PGPU_FLAG_PROFILE;
  static const int cancel_poll = getenv("PGPU_CANCEL_POLL") ? std::max(1, atoi(getenv("PGPU_CANCEL_POLL"))) : PGPU_CANCEL_POLL;
  p.cancel_poll = cancel_poll;
  // once-read tile streams take the non-temporal policy (measured on config 5: 0.407 -> 0.399 ms); PGPU_DIRECT_NT=0
  // restores the default policy
  static const bool direct_nt = !(getenv("PGPU_DIRECT_NT") && atoi(getenv("PGPU_DIRECT_NT")) == 0);
  if (direct_nt) p.flags |= PGPU_FLAG_NT;
  for (int s = 0; s < L.num_sections; ++s) p.sec_op[s] = L.section_op[s];
  uint32_t stride = 1;
  uint64_t stride64 = 1;
  if (L.key_kind == PGPU_KEYS_HASH) p.mode = PGPU_MODE_HASH;  // final; plan_segment reads it
  p.key_words = L.key_words;
  p.key_split = L.key_split;
  for (int g = 0; g < q->num_group_columns; ++g) {
    if (q->group_columns[g] < 0 || q->group_columns[g] >= q->num_columns)
      return fail(PGPU_E_INVALID, "group column %d", q->group_columns[g]);
    p.gcols[g] = q->group_columns[g];
    if (g == L.key_split) stride64 = 1;  // second key word
    p.gstride[g] = stride;
    p.gstride64[g] = stride64;
    stride *= (uint32_t)q->group_cardinalities[g];
    stride64 *= (uint64_t)q->group_cardinalities[g];
  }
  // device aggregations: one per query aggregation, or one per part section of a split integer SUM
  p.nagg = 0;
  for (int a = 0; a < q->num_aggs; ++a) {
    const int parts = q->aggs[a].fn == PGPU_AGG_COUNT ? 1 : std::max(1, L.agg_sum_parts[a]);
    for (int k = 0; k < parts; ++k) {
      if (p.nagg >= PGPU_MAX_AGGS) return fail(PGPU_E_UNSUPPORTED, "more than %d device aggregations", PGPU_MAX_AGGS);
      DevAgg& d = p.aggs[p.nagg++];
      d.fn = q->aggs[a].fn;
      d.col = q->aggs[a].column;
      d.sec = L.agg_section[a] + k;
      d.op = L.section_op[d.sec];
      d.vtype = L.agg_value_type[a];
      d.emit = 0;
      d.part = parts > 1 ? k + 1 : 0;
      d.fxe = L.agg_sum_exp[a];
    }
  }
  // multi-value group columns (every segment's column of one schema: multi-value everywhere or nowhere)
  p.mv_gmask = 0;
  for (int g = 0; g < q->num_group_columns; ++g) {
    int nmv = 0;
    for (int s = 0; s < q->num_segments; ++s) {
      const pgpu_segment_plan& sp = q->segments[s];
      const int32_t slot = sp.column_map[q->group_columns[g]];
      if (slot >= 0 && slot < (int32_t)sp.segment->dev.size() && sp.segment->dev[slot].kind == PGPU_COL_MV) ++nmv;
    }
    if (nmv && nmv != q->num_segments)
      return fail(PGPU_E_INVALID, "group column %d is multi-value in %d of %d segments", g, nmv, q->num_segments);
    if (nmv) p.mv_gmask |= 1 << g;
  }
  int64_t tiles = 0;
  for (int s = 0; s < q->num_segments; ++s) {
    const pgpu_segment_plan& sp = q->segments[s];
    const pgpu_segment* seg = sp.segment;
    if (!seg || !seg->sealed) return fail(PGPU_E_INVALID, "segment %d missing or not sealed", s);
    if (seg->ctx != ctx) return fail(PGPU_E_INVALID, "segment %d belongs to another context", s);
    if (!sp.column_map && q->num_columns) return fail(PGPU_E_INVALID, "segment %d: no column map", s);
    DevSeg ds{};
    ds.num_docs = seg->num_docs;
    ds.tile_begin = (int32_t)tiles;
    ds.ntiles = (seg->num_docs + PGPU_WT - 1) / PGPU_WT;
    ds.col_begin = (int32_t)pk.cols.size();
    ds.remap_begin = (int32_t)pk.remaps.size();
    for (int c = 0; c < q->num_columns; ++c) {
      const int32_t slot = sp.column_map[c];
      if (slot < 0 || slot >= (int32_t)seg->dev.size())
        return fail(PGPU_E_INVALID, "segment %d: column %d mapped to bad slot %d", s, c, slot);
      pk.cols.push_back(seg->dev[slot]);
    }
    // group / aggregation column checks
    for (int g = 0; g < q->num_group_columns; ++g) {
      const DevColumn& c = pk.cols[ds.col_begin + p.gcols[g]];
      if (c.kind == PGPU_COL_NONE) return fail(PGPU_E_INVALID, "segment %d: group column without forward index", s);
      if (c.kind == PGPU_COL_RAW)  // NoDictionary*GroupKeyGenerator: a value-hash path the GPU does not run
        return fail(PGPU_E_UNSUPPORTED, "segment %d: GROUP BY on a raw (no-dictionary) column", s);
      const pgpu_buffer* rb = sp.group_remap ? sp.group_remap[g] : nullptr;
      if (rb && rb->length < c.card) return fail(PGPU_E_INVALID, "segment %d: remap shorter than cardinality", s);
      if (!rb && c.card > q->group_cardinalities[g])
        return fail(PGPU_E_INVALID, "segment %d: identity group ids exceed the global cardinality", s);
      pk.remaps.push_back(rb ? (const int32_t*)rb->mem.p : nullptr);
    }
    for (int a = 0; a < q->num_aggs; ++a) {
      if (q->aggs[a].fn == PGPU_AGG_COUNT) continue;
      const DevColumn& c = pk.cols[ds.col_begin + q->aggs[a].column];
      if (c.kind == PGPU_COL_NONE || !c.dict) return fail(PGPU_E_INVALID, "segment %d: agg column not readable", s);
      if (c.kind == PGPU_COL_MV)
        return fail(PGPU_E_UNSUPPORTED, "segment %d: aggregation over a multi-value column (use its row columns)", s);
      if (c.dict_type != L.agg_value_type[a]) return fail(PGPU_E_INVALID, "segment %d: agg column type differs", s);
    }
    int rc = plan_segment(q, sp, seg, p, pk, ds);
    if (rc) return rc;
    // a filter folded to EMPTY (a literal absent from the dictionary under an AND, ...) matches nothing: the
    // reference's EmptyFilterOperator scans no doc, so the segment gets no tiles
    if (ds.prog_len == 1 && ds.rprog_len == 0 && pk.instrs[ds.prog_begin].op == PGPU_I_EMPTY) ds.ntiles = 0;
    ds.track = 0;
    if (p.mode == PGPU_MODE_HASH && segment_needs_count(q, sp)) {
      pk.tracked.push_back(s);
      ds.track = (int32_t)pk.tracked.size();
    }
    ds.leaf_len = ds.leaf_begin = 0;
    ds.leaf_bits_off = pk.leaf_words;
    if ((q->flags & PGPU_Q_EXACT_FILTER_STATS) && sp.num_filter_nodes > 0) {
      // the whole program once more, for its leaves' match bitmaps (leafbits_kernel)
      const int base = (int)pk.instrs.size();
      rc = convert_filter(q, sp, sp.filter, sp.num_filter_nodes, seg, pk);
      if (rc) return rc;
      ds.leaf_begin = (int32_t)pk.pool.size();
      for (int i = base; i < (int)pk.instrs.size(); ++i) {
        const int op = pk.instrs[i].op;
        if (op == PGPU_I_SCAN || op == PGPU_I_INV || op == PGPU_I_SORTED || op == PGPU_I_BITS) pk.pool.push_back(i);
      }
      ds.leaf_len = (int32_t)pk.pool.size() - ds.leaf_begin;
      pk.leaf_words += (int64_t)ds.leaf_len * ds.ntiles * 64;
    }
    pk.segs.push_back(ds);
    tiles += ds.ntiles;
    if (tiles > INT32_MAX / 2) return fail(PGPU_E_UNSUPPORTED, "too many docs in one launch");
  }
  p.nseg = q->num_segments;
  p.total_tiles = (int32_t)tiles;
  p.max_instrs = pk.max_instrs;
  if (q->flags & PGPU_Q_EXACT_FILTER_STATS) {
    static const bool no_fsm = getenv("PGPU_NO_ANDFSM") && atoi(getenv("PGPU_NO_ANDFSM")) != 0;
    bool fsm = !no_fsm;
    for (int s = 0; s < q->num_segments && fsm; ++s) {
      const int k = pk.segs[s].leaf_len;
      fsm = fsm_filter(q->segments[s]) && k <= 4 &&
            (k == 0 || k == (q->segments[s].num_filter_nodes == 1 ? 1 : (q->segments[s].num_filter_nodes - 2) / 2));
    }
    if (fsm) {
      pk.fsm = true;
      pk.leaf_words = 0;  // no leaf bitmaps, no host replay
      // the lean andfsm build: every segment an AND of two leaves, both read from bit planes (fsm_sliced_ok)
      pk.fsm_s2 = true;
      for (int s = 0; s < q->num_segments && pk.fsm_s2; ++s) {
        const DevSeg& ds = pk.segs[s];
        pk.fsm_s2 = ds.leaf_len == 2;
        for (int j = 0; j < 2 && pk.fsm_s2; ++j) {
          const DevInstr& in = pk.instrs[pk.pool[ds.leaf_begin + j]];
          const DevColumn& c = pk.cols[ds.col_begin + in.col];
          pk.fsm_s2 = in.op == PGPU_I_SCAN && in.kind == PGPU_COL_FIXED_BIT && c.sliced && in.bits >= 1 &&
                      in.bits <= 24 &&
                      (in.pred == 0 || in.pred == 3 || (in.pred == 2 && in.n >= 1 && in.n <= 4));  // RANGE MASK LIST
        }
      }
    }
  }
  return PGPU_OK;
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace

extern "C" {

// host_table (device-visible pointer into pinned host memory, or null): the finished table is also exported there
namespace {
int enqueue_compact(pgpu_context* ctx, Workspace* ws, const pgpu_table_layout* L, const void* dev_table,
                    hipStream_t st, const pgpu_topk* order);
}  // namespace

// eager: compact the table (only the best groups by eager_order, when given) on the query's stream right behind
// its kernels, into the workspace; pgpu_query_collect then only copies the rows out (pgpu_query_submit_ordered)
static int launch_impl(pgpu_context* ctx, const pgpu_query_desc* q, void* stream, void* dev_table,
                       uint64_t table_bytes, int64_t* host_table, pgpu_query** out_query, bool eager = false,
                       const pgpu_topk* eager_order = nullptr) {
  if (!ctx || !q || !out_query) return fail(PGPU_E_INVALID, "null argument");
  pgpu_table_layout L;
  int rc = pgpu_table_layout_of(q, &L);
  if (rc) return rc;
  const uint64_t need = pgpu_table_bytes(&L);
  if (!dev_table || table_bytes < need)
    return fail(PGPU_E_INVALID, "table buffer %llu bytes < %llu needed", (unsigned long long)table_bytes,
                (unsigned long long)need);
  Packer pk;
  DevParams p;
  const double tp0 = HostTiming::us();
  rc = pack_query(ctx, q, L, pk, p);
  host_timing().add(2, tp0, HostTiming::us());
  if (rc) return rc;
  if (pk.leaf_words > 0 && !pk.legacy_range) {
    // the reference's numEntriesScannedInFilter requested, but every segment's program is one whose GPU count IS
    // the reference's (scans driven by next(): OR / NOT trees, index merges then applyAnd, a lone multi-value scan;
    // pgpu_filter_count_is_reference): no leaf bitmaps, no copy to the host, no replay
    bool all_ref = true;
    for (int s = 0; s < q->num_segments && all_ref; ++s) {
      const pgpu_segment_plan& sp = q->segments[s];
      all_ref = pgpu_filter_count_is_reference(sp.filter, sp.num_filter_nodes);
      int nmv = 0;
      for (int i = 0; i < sp.num_filter_nodes && all_ref; ++i) {
        const pgpu_filter_node& nd = sp.filter[i];
        if (nd.op != PGPU_F_SCAN || nd.column < 0 || nd.column >= q->num_columns) continue;
        const int32_t slot = sp.column_map[nd.column];
        nmv += slot >= 0 && slot < (int32_t)sp.segment->cols.size() && sp.segment->cols[slot].kind == PGPU_COL_MV;
      }
      all_ref = all_ref && (nmv == 0 || sp.num_filter_nodes == 1);
    }
    const bool always_replay = getenv("PGPU_ALWAYS_REPLAY") && atoi(getenv("PGPU_ALWAYS_REPLAY")) != 0;  // (per plan: tests)
    if (all_ref && !always_replay) {
      pk.leaf_words = 0;
      for (DevSeg& ds : pk.segs) ds.leaf_len = 0;
    }
  }
  HIP_TRY(hipSetDevice(ctx->device));

  // mode and LDS geometry: consumer areas, optional LDS group table, then as many ring slots as fit
  const uint64_t tbytes = 8ull * L.num_sections * L.num_keys;
  const int S = (int)align16(std::max(16, pk.slot_bytes));
  bool any_dense = false;
  for (const DevSeg& ds : pk.segs) any_dense |= ds.agg_mode == PGPU_AM_DENSE;
  p.dense = any_dense ? 1 : 0;
  // mask rows per consumer: the highest filter slot any program uses, + 1 scratch row (bitmap containers)
  int max_slot = 0;
  for (const DevInstr& in : pk.instrs) max_slot = std::max({max_slot, in.dst, in.src, in.care});
  p.mask_rows = std::min(PGPU_MAX_SLOTS, max_slot + 2);
  p.cons_bytes = PGPU_CONS_BYTES(p.dense, p.mask_rows);
  const size_t fixed = pgpu_lds_fixed_bytes(p.dense, 0, p.mask_rows);
  // LDS-privatised table only when it fits next to >= 4 ring slots and enough docs are expected to match to pay
  // for initialising and flushing one table copy per workgroup
  int grid = std::max(1, std::min(ctx->num_cus, p.total_tiles));
  const bool many = pk.est_matched > 4.0 * (double)L.num_keys * grid;
  // partitioned group-by (PGPU_MODE_PART): large key spaces, at most one aggregated column of a 4-byte type
  bool part_ok = q->num_group_columns > 0 &&
                 (L.num_keys >= PGPU_PART_MIN_KEYS || (q->flags & PGPU_Q_PARTITION) != 0);
  int pcol = -1;
  for (int a = 0; a < p.nagg && part_ok; ++a) {
    if (p.aggs[a].fn == PGPU_AGG_COUNT) continue;
    if (pcol >= 0 && p.aggs[a].col != pcol) part_ok = false;
    if (p.aggs[a].vtype != PGPU_INT && p.aggs[a].vtype != PGPU_FLOAT) part_ok = false;
    if (p.aggs[a].part != 0) part_ok = false;  // records carry whole 4-byte values
    if (pcol < 0) {
      pcol = p.aggs[a].col;
      p.aggs[a].emit = 1;
    }
  }
  int pshift = 0;
  while ((8ull * L.num_sections << (pshift + 1)) <= PGPU_PART_LDS_BYTES) ++pshift;
  uint64_t nparts = (L.num_keys + (1ull << pshift) - 1) >> pshift;
  part_ok = part_ok && nparts <= PGPU_PART_MAX_PARTS && L.num_keys < (1ull << 31) &&
            L.num_sections <= PGPU_PART_MAX_SECTIONS && !p.mv_gmask;  // one record per doc: no value expansion
  if (q->num_group_columns == 0) p.mode = PGPU_MODE_AGG;
  else if (L.key_kind == PGPU_KEYS_HASH) p.mode = PGPU_MODE_HASH;
  else if (tbytes <= PGPU_LDS_TABLE_BYTES && many && !(q->flags & PGPU_Q_PARTITION) &&
           (PGPU_LDS_LIMIT - fixed - align16(tbytes)) / S >= 4)
    p.mode = PGPU_MODE_LDS;
  else if (part_ok) p.mode = PGPU_MODE_PART;
  else p.mode = PGPU_MODE_GLOBAL;
  if (p.mode != PGPU_MODE_PART)
    for (int a = 0; a < p.nagg; ++a) p.aggs[a].emit = 0;
  p.ltab_bytes = p.mode == PGPU_MODE_LDS ? (int32_t)tbytes : (p.mode == PGPU_MODE_PART ? (int32_t)(4 * nparts) : 0);
  const size_t avail = PGPU_LDS_LIMIT - fixed - align16(p.ltab_bytes);
  p.slot_bytes = S;
  p.ring_slots = (int32_t)std::min<size_t>(PGPU_RING_MAX, avail / S);
  if (p.ring_slots < 2) return fail(PGPU_E_UNSUPPORTED, "staged tile of %d bytes leaves < 2 LDS ring slots", S);
  // loader window (per loader wave): each loader publishes its oldest slot once `inflight` younger ones are
  // queued behind it.  The NLOAD windows plus one published slot per consumer (and two spare) must fit the ring,
  // otherwise consumers starve on slots that have landed but are not yet published; within that, aim for ~64 KiB
  // of DMAs in flight per CU (HBM latency x per-CU bandwidth).
  const int nload = PGPU_NLOAD_OF(p.dense), ncons = PGPU_NCONS_OF(p.dense);
  if (pk.tile_bytes == 0) {
    p.inflight = 0;
  } else {
    const int64_t by_ring = (p.ring_slots - ncons - 2) / nload;
    const int64_t by_bytes = (64 * 1024 + nload * pk.tile_bytes - 1) / (nload * pk.tile_bytes);
    p.inflight = (int32_t)std::max<int64_t>(1, std::min(by_ring, by_bytes));
  }
  size_t dyn = pgpu_lds_bytes(p.dense, p.ring_slots, S, p.ltab_bytes, p.mask_rows);
  // direct (self-loading) variant: every segment's staged columns are its bit-sliced fast leaves and no segment
  // aggregates densely; each wave streams its own tiles through two private LDS slots (query_kernel_direct)
  static const bool no_direct = getenv("PGPU_NO_DIRECT") && atoi(getenv("PGPU_NO_DIRECT")) != 0;
  p.direct = 0;
  // a segment whose dense program reads no staged column (bitmap / sorted / precomputed-bitmap leaves only) also runs
  // on self-loading waves, interpreting its program without slots: the ring's few consumer waves cannot hide the
  // candidate gathers' latency
  bool index_only = true;
  for (const DevSeg& ds : pk.segs) index_only &= ds.ntiles == 0 || (ds.nstage == 0 && ds.fast == 0);
  // (multi-value group keys expand per candidate in the ring kernel only: sparse_agg<MODE, MV>)
  if (!no_direct && !p.dense && p.mode != PGPU_MODE_PART && !p.mv_gmask && (pk.tile_bytes > 0 || index_only)) {
    bool ok = true;
    for (const DevSeg& ds : pk.segs)
      ok &= ds.ntiles == 0 || ((ds.agg_mode == PGPU_AM_COUNT || ds.agg_mode == PGPU_AM_SPARSE) &&
                               ((ds.fast >= 1 && ds.nstage == ds.fast && ds.stage_sliced == (1 << ds.nstage) - 1) ||
                                (ds.nstage == 0 && ds.fast == 0))) ||
            (ds.agg_mode == PGPU_AM_SLICED &&
             ((ds.fast >= 1 && ds.nstage == ds.fast && ds.stage_sliced == (1 << ds.nstage) - 1) ||
              (ds.nstage == 0 && ds.fast == 0)));
    // up to five 4-wave workgroups per CU (more waves hide the per-tile latency better than deeper prefetch, which
    // measured flat); each wave keeps D - 1 tiles in flight, aiming at ~12 KiB (HBM latency
    // x per-CU bandwidth), within the 6-bit vmcnt and the LDS
    int max_instrs = 1, min_instrs = 64;
    for (const DevSeg& ds : pk.segs)
      if (ds.ntiles) {
        max_instrs = std::max(max_instrs, ds.stage_instrs);
        min_instrs = std::min(min_instrs, ds.stage_instrs);
      }
    int D = (int)std::max<int64_t>(2, std::min<int64_t>(8, 1 + (12 * 1024 + pk.tile_bytes - 1) / std::max<int64_t>(1, pk.tile_bytes)));
    D = std::min(D, 1 + 63 / max_instrs);
    static const int env_slots = getenv("PGPU_DIRECT_SLOTS") ? atoi(getenv("PGPU_DIRECT_SLOTS")) : 0;
    static const int env_wgs = getenv("PGPU_DIRECT_WGS") ? atoi(getenv("PGPU_DIRECT_WGS")) : 0;  // per CU
    if (env_slots >= 2) D = std::min(env_slots, 1 + 63 / max_instrs);
    // as many 4-wave workgroups as LDS and VGPRs allow: 5 (20 waves) where the kernel fits 96 VGPRs
    // (PGPU_DIRECT_MIN_WAVES), else 4 -- a fifth workgroup that cannot be resident only adds a tail
    const int wgs = env_wgs >= 1 ? env_wgs : ((p.mode == PGPU_MODE_GLOBAL || p.mode == PGPU_MODE_HASH) ? 5 : 4);
    auto ddyn_of = [&](int d) { return (size_t)4 * p.cons_bytes + align16(p.ltab_bytes) + (size_t)4 * d * S; };
    while (D > 2 && wgs * ddyn_of(D) > PGPU_LDS_LIMIT) --D;
    const size_t ddyn = ddyn_of(D);
    if (ok && D >= 2 && ddyn <= PGPU_LDS_LIMIT) {
      const int per_cu = (int)std::min<size_t>(wgs, PGPU_LDS_LIMIT / ddyn);
      int g = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, p.total_tiles / 16));
      if (g >= 8) g &= ~7;
      p.direct = 1;
      p.dslots = D;
      p.min_instrs = std::max(1, min_instrs);
      grid = std::max(1, g);
      dyn = ddyn;
    }
    // register-direct (query_kernel_rdirect): one bit-sliced fast leaf of <= 16 bits per segment is the only staged
    // column -- its planes stream into VGPRs, no LDS slots (tools/stream_bench.hip: 5.6-6.0 TB/s)
    static const bool no_rdirect = getenv("PGPU_NO_RDIRECT") && atoi(getenv("PGPU_NO_RDIRECT")) != 0;
    bool rd = ok && !no_rdirect;
    int rd_bits = 1;
    for (const DevSeg& ds : pk.segs)
      if (ds.ntiles) {
        if (!(ds.nstage == 1 && ds.fast == 1 && ds.stage_sliced == 1) || ds.agg_mode == PGPU_AM_SLICED) {
          rd = false;
          continue;
        }
        const DevColumn& c = pk.cols[ds.col_begin + ds.stage_col[0]];
        rd &= c.bits >= 1 && c.bits <= 16;
        rd_bits = std::max(rd_bits, (int)c.bits);
      }
    const size_t rdyn = (size_t)4 * p.cons_bytes + align16(p.ltab_bytes) + 16;
    if (rd && rdyn <= PGPU_LDS_LIMIT) {
      // 104-126 VGPRs (4 waves per SIMD) except the aggregation-only mode (136-152: 3)
      const int per_cu = (int)std::min<size_t>(env_wgs >= 1 ? env_wgs : (p.mode == PGPU_MODE_AGG ? 3 : 4),
                                               PGPU_LDS_LIMIT / rdyn);
      int g = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, p.total_tiles / 16));
      if (g >= 8) g &= ~7;
      p.direct = 2;
      p.rd_planes = rd_bits <= 8 ? 8 : rd_bits <= 10 ? 10 : rd_bits <= 12 ? 12 : 16;
      // prefix pre-filter when every segment's residual leaf has one (plan_prefix)
      bool pfx = true;
      for (const DevSeg& ds : pk.segs) pfx &= ds.ntiles == 0 || ds.pfx_col >= 0;
      p.rd_pfx = pfx && p.rd_planes <= 12 ? PGPU_PFX_PLANES : 0;  // (no 16 + 3-plane variant: > 128 VGPRs)
      p.dslots = 0;
      grid = std::max(1, g);
      dyn = rdyn;
    }
    // register streaming (query_kernel_rstream): aggregation-only, every segment an AND of two bit-sliced fast
    // leaves (<= 16 and <= 8 bits) with its aggregations all answered from one column's value planes (<= 24)
    const bool no_rstream = getenv("PGPU_NO_RSTREAM") && atoi(getenv("PGPU_NO_RSTREAM")) != 0;  // per plan (tests)
    bool rs = ok && !no_rstream && p.mode == PGPU_MODE_AGG && rdyn <= PGPU_LDS_LIMIT;
    int vcol = -1, rs_narrow = 1, rs_vb = 1;
    for (int a = 0; a < p.nagg && rs; ++a) {
      const DevAgg& ag = p.aggs[a];
      if (ag.fn == PGPU_AGG_COUNT) continue;
      rs = (vcol < 0 || vcol == ag.col) && ((ag.op == PGPU_RED_SUM_I64 && ag.part == 0) ||
                                            ag.op == PGPU_RED_MIN_I64 || ag.op == PGPU_RED_MAX_I64);
      vcol = ag.col;
    }
    rs = rs && vcol >= 0;
    for (const DevSeg& ds : pk.segs) {
      if (!rs || !ds.ntiles) continue;
      rs = ds.nstage == 2 && ds.fast == 2 && ds.stage_sliced == 3 && ds.agg_mode == PGPU_AM_SLICED &&
           ds.rprog_len == 0 && ds.f_nr[0] > 0 && ds.f_nr[1] > 0;
      if (!rs) break;
      const DevColumn& vc = pk.cols[ds.col_begin + vcol];
      int b[2];
      for (int j = 0; j < 2; ++j) b[j] = pk.cols[ds.col_begin + pk.instrs[ds.prog_begin + ds.fast_ins[j]].col].bits;
      rs = vc.vsliced && vc.vbits >= 1 && vc.vbits <= 24 && std::max(b[0], b[1]) <= 16 && std::min(b[0], b[1]) >= 1 &&
           std::min(b[0], b[1]) <= 8;
      rs_narrow = std::max(rs_narrow, std::min(b[0], b[1]));
      rs_vb = std::max(rs_vb, (int)vc.vbits);
    }
    if (rs) {
      const int per_cu = (int)std::min<size_t>(env_wgs >= 1 ? env_wgs : 3, PGPU_LDS_LIMIT / rdyn);
      int g = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, p.total_tiles / 16));
      if (g >= 8) g &= ~7;
      p.direct = 3;
      p.rd_planes = rs_narrow <= 4 ? 4 : 8;
      p.rs_vplanes = rs_vb <= 16 ? 16 : 24;
      p.rd_pfx = 0;
      p.dslots = 0;
      grid = std::max(1, g);
      dyn = rdyn;
    }
  }
  // register streaming of index-only programs (query_kernel_rprog): aggregation-only, every segment's dense program
  // a truth table over <= 5 bitmap / sorted leaves, its aggregations from <= 2 columns' value planes (<= 24)
  if (p.direct == 1 && p.mode == PGPU_MODE_AGG) {
    const bool no_rprog = getenv("PGPU_NO_RPROG") && atoi(getenv("PGPU_NO_RPROG")) != 0;  // per plan (tests)
    bool rp = !no_rprog;
    int vcols[2] = {-1, -1}, nv = 0, vbmax = 1;
    for (int a = 0; a < p.nagg && rp; ++a) {
      const DevAgg& ag = p.aggs[a];
      if (ag.fn == PGPU_AGG_COUNT || ag.col == vcols[0] || ag.col == vcols[1]) continue;
      rp = nv < 2 && ((ag.op == PGPU_RED_SUM_I64 && ag.part == 0) || ag.op == PGPU_RED_MIN_I64 ||
                      ag.op == PGPU_RED_MAX_I64);
      if (rp) vcols[nv++] = ag.col;
    }
    for (int a = 0; a < p.nagg && rp; ++a)  // (every aggregation over a value column must be a value-plane one)
      if (p.aggs[a].fn != PGPU_AGG_COUNT)
        rp = (p.aggs[a].op == PGPU_RED_SUM_I64 && p.aggs[a].part == 0) || p.aggs[a].op == PGPU_RED_MIN_I64 ||
             p.aggs[a].op == PGPU_RED_MAX_I64;
    rp = rp && nv >= 1;
    for (DevSeg& ds : pk.segs) {
      if (!rp || !ds.ntiles) continue;
      rp = ds.nstage == 0 && ds.fast == 0 && ds.agg_mode == PGPU_AM_SLICED && ds.rprog_len == 0 && ds.nvstage == 0 &&
           program_truth_table(pk, ds);
      for (int c = 0; c < nv && rp; ++c) {
        const DevColumn& vc = pk.cols[ds.col_begin + vcols[c]];
        rp = vc.vsliced && vc.vbits >= 1 && vc.vbits <= 24;
        vbmax = std::max(vbmax, (int)vc.vbits);
      }
    }
    const size_t rdyn = (size_t)4 * p.cons_bytes + align16(p.ltab_bytes) + 16;
    if (rp && rdyn <= PGPU_LDS_LIMIT) {
      static const int env_wgs = getenv("PGPU_DIRECT_WGS") ? atoi(getenv("PGPU_DIRECT_WGS")) : 0;  // per CU
      const int per_cu = (int)std::min<size_t>(env_wgs >= 1 ? env_wgs : (nv > 1 && vbmax > 20 ? 2 : 3),
                                               PGPU_LDS_LIMIT / rdyn);
      int g = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, p.total_tiles / 16));
      if (g >= 8) g &= ~7;
      p.direct = 4;
      p.rd_planes = nv;
      p.rs_vplanes = vbmax <= 16 ? 16 : (vbmax <= 20 && nv > 1) ? 20 : 24;
      p.rd_pfx = 0;
      p.dslots = 0;
      grid = std::max(1, g);
      dyn = rdyn;
      // every BITS leaf an inverted one: read the containers per (segment, container key) unit into LDS instead of
      // expanding them into HBM bitmaps first (query_kernel_rkey)
      const bool no_rkey = getenv("PGPU_NO_RKEY") && atoi(getenv("PGPU_NO_RKEY")) != 0;  // per plan (tests)
      // (not under the exact-statistics replay: leafbits_kernel reads the inverted leaves as expanded bitmaps)
      bool rk = !no_rkey && !pk.invx.empty() && pk.leaf_words == 0;
      int maxbits = 0, units = 0;
      for (DevSeg& ds : pk.segs) {
        ds.unit_begin = units;
        units += (ds.ntiles + 31) / 32;
        maxbits = std::max(maxbits, (int)ds.nbits);
        int pairs = 0;
        for (int k = 0; k < ds.nbits && rk; ++k) {
          int found = -1;
          for (size_t i = 0; i < pk.invx.size() && found < 0; ++i)
            if (pk.invx[i].out == ds.bits_w[k]) found = (int)i;  // (word offsets until launch)
          rk = found >= 0;
          ds.inv_leaf[k] = found;
          if (found >= 0) pairs += pk.invx[found].nids;
        }
        rk = rk && pairs <= PGPU_RKEY_PAIRS;
      }
      // the container table (every leaf's (id, key) records) and the unit's records and leaf images in LDS
      int64_t ctab = 0;
      for (InvLeafX& x : pk.invx) {
        x.ctab_off = (int32_t)ctab;
        ctab += (int64_t)x.nids * x.nkeys;
      }
      rk = rk && ctab <= INT32_MAX;
      pk.rk_ctab_records = rk ? ctab : 0;
      const size_t kdyn = rdyn + 16 * PGPU_RKEY_PAIRS + (size_t)std::max(1, maxbits) * 8192;
      if (rk && kdyn <= PGPU_LDS_LIMIT) {
        p.direct = 5;
        p.total_units = units;
        p.rk_leaves = std::max(1, maxbits);
        // the aggregated columns' packed 16-bit ids instead of their value planes, values gathered per matched doc
        // (PGPU_RKEY_IDS, read per plan): every value column a 16-bit dictionary column, <= 2
        // non-COUNT aggregations (one queue half each)
        int nq = 0;
        for (int a = 0; a < p.nagg; ++a) nq += p.aggs[a].fn != PGPU_AGG_COUNT;
        bool ids = nq >= 1 && nq <= 2;
        for (const DevSeg& ds : pk.segs)
          for (int c = 0; c < nv && ids && ds.ntiles; ++c) {
            const DevColumn& vc = pk.cols[ds.col_begin + vcols[c]];
            ids = vc.kind == PGPU_COL_FIXED_BIT && vc.bits == 16 && vc.dict != nullptr && vc.fwd != nullptr;
          }
        const char* ev = getenv("PGPU_RKEY_IDS");
        p.rk_ids = ids && ev && atoi(ev) != 0 ? 1 : 0;
        const int per_cu = (int)std::min<size_t>(nv > 1 && vbmax > 20 ? 2 : 3, PGPU_LDS_LIMIT / kdyn);
        int gk = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, units / 2));
        if (gk >= 8) gk &= ~7;
        grid = std::max(1, gk);
        dyn = kdyn;
      }
    }
  }
  // candidate iteration from a sparse leading index leaf (query_kernel_cand; AndDocIdSet.java:87-140): every
  // segment's dense program is one inclusive inverted leaf (a BITS leaf over its expansion) or sorted leaf holding at
  // most kCandDensity of the segment's docs; the units are the inverted leaf's containers or the sorted ranges split
  // at 65,536-doc keys, so the tiles without a doc of the leaf are never visited and the leaf is not expanded.  PGPU_NO_CAND=1 / PGPU_CAND_DENSITY (read per plan: tests).
  pk.cand.clear();
  if (p.direct == 1) {
    const bool no_cand = getenv("PGPU_NO_CAND") && atoi(getenv("PGPU_NO_CAND")) != 0;
    const double cand_max = getenv("PGPU_CAND_DENSITY") ? atof(getenv("PGPU_CAND_DENSITY")) : kCandDensity;
    bool ok = !no_cand;
    std::vector<uint32_t> units;  // {segment, container index (~0u: a sorted doc range), first doc, last doc}
    std::vector<int> leaves;
    for (int s = 0; s < (int)pk.segs.size() && ok; ++s) {
      DevSeg& ds = pk.segs[s];
      ds.unit_begin = (int32_t)(units.size() / 4);
      ds.cand_leaf = -1;
      if (ds.ntiles == 0) continue;
      ok = ds.prog_len == 1 && ds.nstage == 0 && ds.fast == 0 && ds.nvstage == 0 && ds.single_bits == 0 &&
           (ds.agg_mode == PGPU_AM_COUNT || ds.agg_mode == PGPU_AM_SPARSE);
      if (!ok) break;
      const DevInstr& in = pk.instrs[ds.prog_begin];
      const pgpu_segment* sgm = q->segments[s].segment;
      if (in.op == PGPU_I_SORTED) {  // SortedIndexBasedFilterOperator: doc ranges, split at container keys
        ok = !in.negate;
        int64_t docs = 0;
        for (int k = 0; k < in.n && ok; ++k) docs += (int64_t)pk.pool[in.pool_off + 2 * k + 1] - pk.pool[in.pool_off + 2 * k] + 1;
        ok = ok && (double)docs <= cand_max * (double)sgm->num_docs;
        for (int k = 0; k < in.n && ok; ++k) {
          for (int64_t lo = pk.pool[in.pool_off + 2 * k], hi = pk.pool[in.pool_off + 2 * k + 1]; lo <= hi;) {
            const int64_t end = std::min<int64_t>(hi, (lo | 0xFFFF));
            units.insert(units.end(), {(uint32_t)s, ~0u, (uint32_t)lo, (uint32_t)end});
            lo = end + 1;
          }
        }
        ok = ok && units.size() / 4 <= kCandMaxUnits;
        continue;
      }
      ok = in.op == PGPU_I_BITS;
      if (!ok) break;
      int leaf = -1;
      for (size_t i = 0; i < pk.invx.size() && leaf < 0; ++i)
        if (pk.invx[i].out == in.fwd) leaf = (int)i;  // (word offsets until launch)
      ok = leaf >= 0 && !pk.invx[leaf].negate && in.col >= 0 && in.col < q->num_columns;
      if (!ok) break;
      const InvLeafX& x = pk.invx[leaf];
      const HostColumn& h = sgm->cols[q->segments[s].column_map[in.col]];
      const DevColumn& dc = pk.cols[ds.col_begin + in.col];
      ok = (x.nids == 1 || dc.kind == PGPU_COL_FIXED_BIT || dc.kind == PGPU_COL_RAW) &&
           h.inv_hdir.size() == (size_t)h.inv_card + 1 && h.inv_cards.size() == (size_t)h.inv_card;
      const int32_t* ids = pk.invids.data() + (intptr_t)x.ids;
      double docs = 0;
      for (int k = 0; k < x.nids && ok; ++k) {
        ok = ids[k] >= 0 && ids[k] < h.inv_card;
        if (ok) docs += h.inv_cards[ids[k]];
      }
      ok = ok && docs <= cand_max * (double)sgm->num_docs;
      // at most one container per tile of the segment: past that the tile sweep is as cheap, and a long IN list's
      // containers would cost the host more to list than the sweep costs the GPU
      uint64_t nct = 0;
      for (int k = 0; k < x.nids && ok; ++k) nct += h.inv_hdir[ids[k] + 1] - h.inv_hdir[ids[k]];
      ok = ok && nct <= (uint64_t)ds.ntiles;
      for (int k = 0; k < x.nids && ok; ++k)
        for (uint32_t c = h.inv_hdir[ids[k]]; c < h.inv_hdir[ids[k] + 1]; ++c) units.insert(units.end(), {(uint32_t)s, c, 0u, 0u});
      ok = ok && units.size() / 4 <= kCandMaxUnits;
      ds.cand_leaf = leaf;
      leaves.push_back(leaf);
    }
    // a wave's consumer area and 8 KiB container image; four waves per workgroup
    const size_t cdyn = (size_t)4 * p.cons_bytes + align16(p.ltab_bytes) + (size_t)4 * 8192;
    if (ok && cdyn <= PGPU_LDS_LIMIT) {
      const int nu = (int)(units.size() / 4);
      const int per_cu = (int)std::min<size_t>(4, PGPU_LDS_LIMIT / cdyn);
      const int g = (int)std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, (nu + 3) / 4));
      p.direct = 6;
      p.total_units = nu;
      grid = std::max(1, g);
      dyn = cdyn;
      pk.cand.swap(units);
      // the iterated leaves need no doc bitmap unless the exact-statistics replay or a residual program reads it
      std::vector<const uint32_t*> read;
      for (const DevSeg& ds : pk.segs)
        for (int i = ds.rprog_begin; i < ds.rprog_begin + ds.rprog_len; ++i)
          if (pk.instrs[i].op == PGPU_I_BITS) read.push_back(pk.instrs[i].fwd);
      if (pk.leaf_words == 0)
        for (int lf : leaves)
          if (std::find(read.begin(), read.end(), pk.invx[lf].out) == read.end()) pk.invx[lf].skip = 1;
    } else {
      for (DevSeg& ds : pk.segs) ds.cand_leaf = -1;
    }
  }
  // the reference's numEntriesScannedInFilter fused into the register stream (query_kernel_rfsm): on the
  // register-direct path with every segment an AND of two bit-sliced leaves (andfsm's two-leaf build), both leaves'
  // planes are streamed once for the query and the tile maps together (PGPU_NO_RFSM=1, read per plan: tests)
  if (p.direct == 2 && pk.fsm && pk.fsm_s2 && p.mode != PGPU_MODE_PART &&
      !(getenv("PGPU_NO_RFSM") && atoi(getenv("PGPU_NO_RFSM")) != 0)) {
    int b0 = 1, b1 = 1;
    for (const DevSeg& ds : pk.segs)
      if (ds.ntiles && ds.leaf_len == 2) {
        b0 = std::max(b0, (int)pk.instrs[pk.pool[ds.leaf_begin]].bits);
        b1 = std::max(b1, (int)pk.instrs[pk.pool[ds.leaf_begin + 1]].bits);
      }
    const size_t rdyn = (size_t)4 * p.cons_bytes + align16(p.ltab_bytes) + 16;
    if (b0 <= 16 && b1 <= 24 && rdyn <= PGPU_LDS_LIMIT) {
      const bool small = b0 <= 12 && b1 <= 20;
      // 142-167 VGPRs: three waves per SIMD; the aggregation-only mode's 183-199: two
      const int per_cu = (int)std::min<size_t>(p.mode == PGPU_MODE_AGG ? 2 : 3, PGPU_LDS_LIMIT / rdyn);
      int g = std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, p.total_tiles / 16));
      if (g >= 8) g &= ~7;
      p.direct = 8;
      p.rd_planes = small ? (b0 <= 10 ? 10 : 12) : 16;
      p.rs_vplanes = small ? 20 : 24;
      p.rd_pfx = 0;
      p.dslots = 0;
      grid = std::max(1, g);
      dyn = rdyn;
    }
  }
  // sliced aggregation runs in the self-loading kernels only (query_kernel_direct, and query_kernel_rstream with the
  // value planes in VGPRs): elsewhere its segments gather per candidate (their staged aggregation planes are then
  // only extra DMA, never read)
  if (p.direct != 1)
    for (DevSeg& ds : pk.segs) {
      if (ds.agg_mode == PGPU_AM_SLICED && p.direct != 3 && p.direct != 4) ds.agg_mode = PGPU_AM_SPARSE;
      for (int j = 0; j < ds.nvstage; ++j)  // (the ring loaders stage filter columns only)
        ds.stage_instrs -= (pk.cols[ds.col_begin + ds.vstage_col[j]].vbits + 3) / 4;
      ds.nvstage = 0;
    }
  // one-word PART records (in-partition key, dict id) when every segment holds the same dictionary for the
  // aggregated column (the common case of one table's segments sharing value sets): half the record traffic
  int part_idbits = 0;
  const void* part_pdict = nullptr;
  if (p.mode == PGPU_MODE_PART && pcol >= 0) {
    const HostColumn* h0 = &q->segments[0].segment->cols[q->segments[0].column_map[pcol]];
    bool shared = h0->dict_card > 0 && !h0->hdict.empty();
    for (int s = 1; s < q->num_segments && shared; ++s) {
      const HostColumn* h = &q->segments[s].segment->cols[q->segments[s].column_map[pcol]];
      shared = h->dict_card == h0->dict_card && h->dict_type == h0->dict_type && h->dict_hash[0] == h0->dict_hash[0] &&
               h->dict_hash[1] == h0->dict_hash[1];
    }
    int idbits = 1;
    while (idbits < 31 && (1ll << idbits) < h0->dict_card) ++idbits;
    if (shared && pshift + idbits <= 32 && !(q->flags & PGPU_Q_PART_SPILL)) {
      part_idbits = idbits;
      part_pdict = h0->dict.p;
    }
  }
  const int part_rw = pcol >= 0 && !part_idbits ? 2 : 1;
  // phase 2 reads SUM values from an LDS copy of the shared dictionary when it fits beside the partition's table,
  // instead of gathering them from L2 (one 128-B line per 4-B lookup)
  int slice_shift = 0, ldict = 0;
  uint32_t pdict_n = 0;
  int for_old_pshift = -1;
  uint64_t for_old_nparts = 0;
  const HostColumn* for_h = nullptr;
  if (part_idbits) {
    const HostColumn* h0 = &q->segments[0].segment->cols[q->segments[0].column_map[pcol]];
    pdict_n = (uint32_t)h0->dict_card;
    bool need_val = false;
    for (int s = 1; s < L.num_sections; ++s)
      need_val |= L.section_op[s] == PGPU_RED_SUM_I64 || L.section_op[s] == PGPU_RED_SUM_F64;
    while ((1ull << slice_shift) < pdict_n) ++slice_shift;
    static const bool no_ldict = getenv("PGPU_NO_LDICT") && atoi(getenv("PGPU_NO_LDICT")) != 0;
    ldict = need_val && !no_ldict && (8ull * L.num_sections << pshift) + (4ull << slice_shift) <= PGPU_LDS_LIMIT;
    // too large to copy whole: its frame-of-reference image, beside a table of fewer keys per partition
    static const bool no_for = getenv("PGPU_NO_FOR") && atoi(getenv("PGPU_NO_FOR")) != 0;
    if (need_val && !ldict && !no_for && h0->for_bits > 0 && h0->dict_type == PGPU_INT) {
      const uint64_t fb = 4ull * ((uint64_t)h0->for_nblk * (1 + h0->for_bits) + 1);
      // fewer keys per partition means more phase-1 partitions and shallower LDS rings per partition, which
      // skewed keys pay for (config 4 Zipf(1.1): 24 -> 39 ms at 2048 keys); only the unchanged geometry is used
      // unless PGPU_FOR_SHRINK=1
      // the compact phase-2 table: count and MIN / MAX ids in 4 B, SUM sections in 8 B per key
      uint64_t per_key = 4;
      for (int s = 1; s < L.num_sections; ++s)
        per_key += L.section_op[s] == PGPU_RED_SUM_I64 || L.section_op[s] == PGPU_RED_SUM_F64 ? 8 : 4;
      static const bool shrink = getenv("PGPU_FOR_SHRINK") && atoi(getenv("PGPU_FOR_SHRINK")) != 0;
      int ps = pshift;
      while (shrink && ps > 9 && (per_key << ps) + fb > PGPU_LDS_LIMIT) --ps;
      const uint64_t np2 = (L.num_keys + (1ull << ps) - 1) >> ps;
      if ((per_key << ps) + fb <= PGPU_LDS_LIMIT && np2 <= PGPU_PSCAN_MAX_PARTS &&
          np2 <= PGPU_PART_MAX_PARTS && ps + part_idbits <= 32) {
        for_old_pshift = pshift;
        for_old_nparts = nparts;
        pshift = ps;
        nparts = np2;
        ldict = 2;
        for_h = h0;
      }
    }
  }
  // partitioned group-by whose segments need no candidate queue: phase 1 by part_scan_kernel (self-loading waves,
  // records written through per-partition LDS rings of >= two 128-B lines); two workgroups per CU when the rings
  // fit, else one
  static const bool no_pscan = getenv("PGPU_NO_PSCAN") && atoi(getenv("PGPU_NO_PSCAN")) != 0;
  p.pscan = 0;
  const uint64_t ptotal = nparts;
  if (!no_pscan && p.mode == PGPU_MODE_PART && ptotal <= PGPU_PSCAN_MAX_PARTS) {
    bool ok = true;
    for (const DevSeg& ds : pk.segs) ok &= ds.rprog_len == 0;
    const size_t wave_bytes = 256 * (size_t)p.mask_rows;
    const size_t fixed_b = 16 * ((ptotal + 66) & ~1ull) + 4 * 64 * part_rw + 4 * wave_bytes;  // + caps, dummies, cancel
    const uint64_t min_rc = 64 / part_rw;  // rings of at least two 128-B lines
    for (int per_cu = 2; ok && per_cu >= 1 && !p.pscan; --per_cu) {
      const size_t budget = PGPU_LDS_LIMIT / per_cu;
      if (budget <= fixed_b) continue;
      uint64_t rc = 1;
      while (rc < 1024 && fixed_b + 4ull * ptotal * part_rw * (rc * 2) <= budget) rc *= 2;
      if (rc < min_rc) continue;
      p.pscan = (int32_t)rc;
      p.pscan_wave_bytes = (int32_t)wave_bytes;
      // the widths the prefetching phase 1 is compiled for (part_scan_kernel<false, KB, VB>)
      p.pscan_kb = p.pscan_vb = 0;
      const bool no_pfetch = getenv("PGPU_NO_PSCAN_PREFETCH") && atoi(getenv("PGPU_NO_PSCAN_PREFETCH")) != 0;
      if (!no_pfetch && p.ngcols == 1 && pcol >= 0) {
        int kb = -1, vb = -1;
        bool same = true;
        for (const DevSeg& ds : pk.segs) {
          if (!ds.ntiles) continue;
          const DevColumn& kc = pk.cols[ds.col_begin + p.gcols[0]];
          const DevColumn& vc = pk.cols[ds.col_begin + pcol];
          same = same && ds.prog_len == 0 && kc.kind == PGPU_COL_FIXED_BIT && vc.kind == PGPU_COL_FIXED_BIT &&
                 (kb < 0 || kb == kc.bits) && (vb < 0 || vb == vc.bits);
          kb = kc.bits;
          vb = vc.bits;
        }
        if (same && pgpu_pscan_prefetch_ok(kb, vb)) {
          p.pscan_kb = kb;
          p.pscan_vb = vb;
        }
      }
      int g = (int)std::min<int64_t>((int64_t)ctx->num_cus * per_cu, std::max(1, p.total_tiles / 4));
      if (g >= 8) g &= ~7;
      p.direct = 0;
      grid = std::max(1, g);
      dyn = align16(fixed_b + 4ull * ptotal * part_rw * rc);
    }
  }
  if (ldict == 2 && !p.pscan) {  // the ring's partition counters were sized for the original geometry
    pshift = for_old_pshift;
    nparts = for_old_nparts;
    ldict = 0;
    for_h = nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->lds_ready) {
      HIP_TRY(pgpu_prepare_query_kernels(PGPU_LDS_LIMIT));
      ctx->lds_ready = true;
    }
  }
  const int nwaves = grid * (p.direct || p.pscan ? 4 : PGPU_WAVES_OF(p.dense));

  static const bool trace = getenv("PGPU_PLAN_TRACE") && atoi(getenv("PGPU_PLAN_TRACE")) != 0;
  if (trace) {  // diagnostics: the plan of each segment and the kernel chosen
    fprintf(stderr, "[pgpu plan] mode %d dense %d direct %d pscan %d grid %d dyn %zu tiles %d units %d invx %zu\n",
            p.mode, p.dense, p.direct, p.pscan, grid, dyn, p.total_tiles, p.total_units, pk.invx.size());
    for (size_t i = 0; i < pk.segs.size(); ++i) {
      const DevSeg& ds = pk.segs[i];
      fprintf(stderr, "[pgpu plan]  seg %zu tiles %d prog %d (op %d) rprog %d agg_mode %d nstage %d fast %d sliced %d "
              "nvstage %d single_bits %d nbits %d\n", i, ds.ntiles, ds.prog_len,
              ds.prog_len ? pk.instrs[ds.prog_begin].op : -1, ds.rprog_len, ds.agg_mode, ds.nstage, ds.fast,
              ds.stage_sliced, ds.nvstage, ds.single_bits, ds.nbits);
    }
  }
  const double tw0 = HostTiming::us();
  Workspace* ws = acquire_ws(ctx, &rc);
  if (!ws) return rc;
  hipStream_t bail_stream = nullptr;
  auto bail = [&](int code) {
    // a bail after the query kernel was enqueued but before finalize_kernel: the matched-segment words it may
    // have set must not count towards the workspace's next query (they are zero between queries)
    if (bail_stream && ws->segany.p) (void)hipMemsetAsync(ws->segany.p, 0, ws->segany.n, bail_stream);
    release_ws(ctx, ws);
    return code;
  };
  // NULL stream: the context's query stream (queries run back to back; each has its own completion event).  The
  // cancel stream is created here too, never in pgpu_query_cancel (stream creation may wait for the device).
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!stream && !ctx->qstream) {
      const hipError_t ce = hipStreamCreateWithFlags(&ctx->qstream, hipStreamNonBlocking);
      if (ce != hipSuccess) return bail(fail(PGPU_E_HIP, "query stream: %s", hipGetErrorString(ce)));
    }
    if (!ctx->cstream) {
      const hipError_t ce = hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking);
      if (ce != hipSuccess) return bail(fail(PGPU_E_HIP, "cancel stream: %s", hipGetErrorString(ce)));
    }
  }
  hipStream_t st = stream ? (hipStream_t)stream : ctx->qstream;
  bail_stream = st;

  // arena: segs | instrs | cols | pool | remaps
  const size_t o_segs = 0;
  const size_t o_ins = align16(o_segs + pk.segs.size() * sizeof(DevSeg));
  const size_t o_cols = align16(o_ins + pk.instrs.size() * sizeof(DevInstr));
  const size_t o_pool = align16(o_cols + pk.cols.size() * sizeof(DevColumn));
  const size_t o_rem = align16(o_pool + pk.pool.size() * 4);
  const size_t o_raw = align16(o_rem + pk.remaps.size() * sizeof(void*));
  const size_t o_rvals = align16(o_raw + pk.raws.size() * sizeof(RawLeaf));
  const size_t o_mv = align16(o_rvals + pk.rawvals.size() * 8);
  const size_t o_mvset = align16(o_mv + pk.mvs.size() * sizeof(MvLeaf));
  const size_t o_inv = align16(o_mvset + pk.mvsets.size() * 4);
  const size_t o_invids = align16(o_inv + pk.invx.size() * sizeof(InvLeafX));
  const size_t o_jobs = align16(o_invids + pk.invids.size() * 4);
  const size_t o_cand = align16(o_jobs + pk.jobs.size() * sizeof(ProgJob));
  const size_t total = align16(o_cand + pk.cand.size() * 4) + 16;
  hipError_t e = ws->h_arena.ensure(total);
  if (e == hipSuccess) e = ws->arena.ensure(total, ctx->mpool, st);
  if (e == hipSuccess) e = ws->slab.ensure(8ull * nwaves * L.num_sections + 16, ctx->mpool, st);
  if (e == hipSuccess) e = ws->stats.ensure(8ull * nwaves * PGPU_NSTATS + 16, ctx->mpool, st);
  if (e == hipSuccess) e = ws->stats_out.ensure(8 * PGPU_NSTATS, ctx->mpool, st);
  if (e == hipSuccess) e = ws->h_stats.ensure(8 * PGPU_NSTATS + 16);
  // the cancel copy's pinned source is allocated here, never in pgpu_query_cancel: an allocation there could wait
  // for the device -- i.e. for the very kernel the cancel is meant to stop
  if (e == hipSuccess) e = ws->h_cancel.ensure(16);
  if (e == hipSuccess && !ws->d_cancel.p) {
    // uncached device memory: the kernels' polls read HBM, so pgpu_query_cancel's copy-engine write (which bypasses
    // the GPU's L2) is seen at the next poll
    e = hipExtMallocWithFlags(&ws->d_cancel.p, 16, hipDeviceMallocUncached);
    if (e == hipSuccess) {
      ws->d_cancel.n = 16;
      e = hipMemset(ws->d_cancel.p, 0, 16);
    } else {
      ws->d_cancel.p = nullptr;
    }
  }
  if (e == hipSuccess && (p.flags & PGPU_FLAG_PROFILE)) e = ws->prof.ensure(8ull * nwaves * PGPU_NPROF, ctx->mpool, st);
  if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "workspace allocation: %s", hipGetErrorString(e)));
  if (p.mode == PGPU_MODE_PART) {
    // region capacity: 1.25x the expected records per (partition, workgroup) + slack; full regions spill to
    // HBM atomics, so an underestimate costs time, never correctness.  Bounded by half the free HBM.
    p.pshift = pshift;
    p.nparts = (int32_t)nparts;
    p.slice_shift = slice_shift;
    p.ldict = ldict;
    p.pdict_n = pdict_n;
    p.pfor = for_h ? (const uint32_t*)for_h->for_dev.p : nullptr;
    p.for_bits = for_h ? for_h->for_bits : 0;
    p.for_nblk = for_h ? for_h->for_nblk : 0;
    p.pcol = pcol;
    p.rw = part_rw;
    p.rec_idbits = part_idbits;
    p.pdict = part_pdict;
    const double per = pk.est_matched / ((double)grid * (double)p.nparts);
    uint64_t cap = (uint64_t)(1.25 * per) + 32;
    if (q->flags & PGPU_Q_PART_SPILL) cap = 16;
    // regions of an odd number of 128-B lines: the active (partially written) line of every region then falls on
    // a different L2 set instead of all regions' cursors sharing a few sets, so lines stay resident until full
    const uint64_t per_line = 32 / p.rw;
    uint64_t lines = (cap + per_line - 1) / per_line;
    if (!(q->flags & PGPU_Q_PART_SPILL) && (lines & 1) == 0) ++lines;
    cap = lines * per_line;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    const uint64_t regions = (uint64_t)p.nparts * (uint64_t)grid;
    const uint64_t have = ws->recs.n;
    const uint64_t budget = std::max<uint64_t>(have, (uint64_t)free_b / 2);
    const uint64_t max_cap = budget / (regions * 4ull * p.rw);
    if (cap > max_cap) cap = max_cap / per_line * per_line;
    if (cap > (uint64_t)INT32_MAX) cap = (uint64_t)INT32_MAX / per_line * per_line;
    p.rcap = (int32_t)std::max<uint64_t>(cap, 16);
    e = ws->recs.ensure(regions * (uint64_t)p.rcap * 4ull * p.rw, ctx->mpool, st);
    if (e == hipSuccess) e = ws->rcount.ensure(4ull * regions, ctx->mpool, st);
    p.pblock = (uint64_t)p.nparts * (uint64_t)p.rcap;  // records per phase-1 workgroup block
    p.pcount = p.pcap = p.poff = nullptr;
    p.p2work = nullptr;
    p.p2grid = p.nparts;
    static const bool no_psize = getenv("PGPU_NO_PSIZE") && atoi(getenv("PGPU_NO_PSIZE")) != 0;
    if (p.pscan && !no_psize && !(q->flags & PGPU_Q_PART_SPILL)) {
      // regions sized from a sampled count (~8K tiles) and heavy partitions split in phase 2: skewed keys
      // (Zipf) would otherwise overflow their regions into HBM atomics and leave one phase-2 workgroup with most
      // of the records
      p.psample = std::max(1, p.total_tiles / 8192);
      p.p2grid = 2 * p.nparts;
      if (e == hipSuccess) e = ws->pcount.ensure(4ull * p.nparts, ctx->mpool, st);
      if (e == hipSuccess) e = ws->pcap.ensure(4ull * p.nparts, ctx->mpool, st);
      if (e == hipSuccess) e = ws->poff.ensure(4ull * p.nparts, ctx->mpool, st);
      if (e == hipSuccess) e = ws->p2work.ensure(16ull * p.p2grid, ctx->mpool, st);
      p.pcount = (uint32_t*)ws->pcount.p;
      p.pcap = (uint32_t*)ws->pcap.p;
      p.poff = (uint32_t*)ws->poff.p;
      p.p2work = (int32_t*)ws->p2work.p;
    }
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "group-by record buffers: %s", hipGetErrorString(e)));
    p.recs = (uint32_t*)ws->recs.p;
    p.rcount = (uint32_t*)ws->rcount.p;
  }
  if (pk.raw_words > 0 && p.direct != 5) {  // (query_kernel_rkey builds its leaf images in LDS)
    e = ws->rawbits.ensure(4ull * pk.raw_words, ctx->mpool, st);
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "raw-value leaf bitmaps: %s", hipGetErrorString(e)));
  }
  p.rk_ctab = nullptr;
  if (p.direct == 5) {
    e = ws->rkctab.ensure(sizeof(DevContainer) * (size_t)std::max<int64_t>(1, pk.rk_ctab_records), ctx->mpool, st);
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "container table: %s", hipGetErrorString(e)));
    p.rk_ctab = (const DevContainer*)ws->rkctab.p;
  }
  p.fsm_fn = nullptr;
  if (pk.fsm) {
    e = ws->fsmfn.ensure(32ull * std::max(1, p.total_tiles), ctx->mpool, st);
    if (e == hipSuccess) e = ws->h_fsment.ensure(8ull * std::max(1, p.nseg));
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "filter-statistics maps: %s", hipGetErrorString(e)));
    p.fsm_fn = (uint32_t*)ws->fsmfn.p;
  }
  if (pk.leaf_words > 0) {
    e = ws->leafbits.ensure(4ull * pk.leaf_words, ctx->mpool, st);
    if (e == hipSuccess) e = ws->h_leafbits.ensure(4ull * pk.leaf_words);
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "filter-statistics bitmaps: %s", hipGetErrorString(e)));
    p.leaf_bits = (uint32_t*)ws->leafbits.p;
  }
  {
    // numSegmentsMatched words: grown in stream order and zeroed once; finalize_kernel resets them after each query
    const size_t want = 4ull * std::max(1, p.nseg);
    if (ws->segany.n < want) {
      e = ws->segany.ensure(want, ctx->mpool, st);
      if (e == hipSuccess) e = hipMemsetAsync(ws->segany.p, 0, ws->segany.n, st);
    }
    if (e == hipSuccess) e = ws->h_segany.ensure((size_t)std::max(1, p.nseg));
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "segment match words: %s", hipGetErrorString(e)));
    p.segany = (uint32_t*)ws->segany.p;
  }
  if (p.mode == PGPU_MODE_HASH) {
    p.segmask_rows = (int32_t)pk.tracked.size();
    e = ws->hflag.ensure(16, ctx->mpool, st);
    if (e == hipSuccess && p.segmask_rows) e = ws->segmask.ensure((size_t)p.segmask_rows * (L.num_keys / 8) + 16, ctx->mpool, st);
    if (e == hipSuccess && p.segmask_rows) e = ws->h_segcnt.ensure(8 * (size_t)p.segmask_rows);
    if (e == hipSuccess) e = hipMemsetAsync(ws->hflag.p, 0, 16, st);
    if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "hash group-by buffers: %s", hipGetErrorString(e)));
    p.hflag = (int32_t*)ws->hflag.p;
    p.segmask = p.segmask_rows ? (uint32_t*)ws->segmask.p : nullptr;
  }
  char* h = (char*)ws->h_arena.p;
  char* d = (char*)ws->arena.p;
  // raw-value leaves: offsets -> device pointers (bitmaps in the workspace, set values in the arena)
  for (int idx : pk.bits_instrs)
    pk.instrs[idx].fwd = (const uint32_t*)ws->rawbits.p + (intptr_t)pk.instrs[idx].fwd;
  for (DevSeg& sg : pk.segs)
    for (int k = 0; k < sg.nbits; ++k) sg.bits_w[k] = (const uint32_t*)ws->rawbits.p + (intptr_t)sg.bits_w[k];
  int64_t max_raw_words = 0;
  for (RawLeaf& r : pk.raws) {
    r.out = (uint32_t*)ws->rawbits.p + (intptr_t)r.out;
    r.vals = (const int64_t*)(d + o_rvals) + (intptr_t)r.vals;
    max_raw_words = std::max<int64_t>(max_raw_words, r.words);
  }
  int64_t max_mv_words = 0;
  for (MvLeaf& m : pk.mvs) {
    m.out = (uint32_t*)ws->rawbits.p + (intptr_t)m.out;
    m.set = m.set ? (const uint32_t*)(d + o_mvset) + ((intptr_t)m.set - 1) : nullptr;
    max_mv_words = std::max<int64_t>(max_mv_words, m.words);
  }
  memcpy(h + o_mv, pk.mvs.data(), pk.mvs.size() * sizeof(MvLeaf));
  int64_t max_inv_words = 0;
  for (InvLeafX& x : pk.invx) {
    x.out = (uint32_t*)ws->rawbits.p + (intptr_t)x.out;
    x.ids = (const int32_t*)(d + o_invids) + (intptr_t)x.ids;
    max_inv_words = std::max<int64_t>(max_inv_words, x.words);
  }
  memcpy(h + o_inv, pk.invx.data(), pk.invx.size() * sizeof(InvLeafX));
  for (ProgJob& jb : pk.jobs) {
    jb.out = (uint32_t*)ws->rawbits.p + (intptr_t)jb.out;
    for (int k = 0; k < jb.nbits; ++k) jb.bits_w[k] = (const uint32_t*)ws->rawbits.p + (intptr_t)jb.bits_w[k];
  }
  memcpy(h + o_jobs, pk.jobs.data(), pk.jobs.size() * sizeof(ProgJob));
  memcpy(h + o_cand, pk.cand.data(), pk.cand.size() * 4);
  p.cand_ct = (const uint32_t*)(d + o_cand);
  memcpy(h + o_invids, pk.invids.data(), pk.invids.size() * 4);
  memcpy(h + o_mvset, pk.mvsets.data(), pk.mvsets.size() * 4);
  memcpy(h + o_raw, pk.raws.data(), pk.raws.size() * sizeof(RawLeaf));
  memcpy(h + o_rvals, pk.rawvals.data(), pk.rawvals.size() * 8);
  memcpy(h + o_segs, pk.segs.data(), pk.segs.size() * sizeof(DevSeg));
  memcpy(h + o_ins, pk.instrs.data(), pk.instrs.size() * sizeof(DevInstr));
  memcpy(h + o_cols, pk.cols.data(), pk.cols.size() * sizeof(DevColumn));
  memcpy(h + o_pool, pk.pool.data(), pk.pool.size() * 4);
  memcpy(h + o_rem, pk.remaps.data(), pk.remaps.size() * sizeof(void*));
  const double tl0 = HostTiming::us();
  host_timing().add(3, tw0, tl0);
  p.segs = (const DevSeg*)(d + o_segs);
  p.instrs = (const DevInstr*)(d + o_ins);
  p.cols = (const DevColumn*)(d + o_cols);
  p.pool = (const int32_t*)(d + o_pool);
  p.remaps = (const int32_t* const*)(d + o_rem);
  p.table = (int64_t*)dev_table;
  p.slab = (int64_t*)ws->slab.p;
  p.stats = (int64_t*)ws->stats.p;
  p.prof = (int64_t*)ws->prof.p;

  // metadata in and stats (and small tables) out through pinned host memory touched by kernels: no DMA-engine
  // copy sits between two queries' kernels
  void* h_arena_dev = nullptr;
  void* h_stats_dev = nullptr;
  // cancel word in HBM: a query is stopped when the word equals its generation (no reset that could race a
  // cancel issued from another stream); the kernels poll it with uncached loads
  if (++ws->cancel_gen == 0) ws->cancel_gen = 1;
  p.cancel = (const int32_t*)ws->d_cancel.p;
  p.cancel_gen = ws->cancel_gen;
  const bool expired = q->deadline_ms > 0 && now_epoch_ms() >= q->deadline_ms;
  if (expired) e = hipMemsetD32Async((hipDeviceptr_t)ws->d_cancel.p, (int)ws->cancel_gen, 1, st);
  if (e == hipSuccess) e = ws->h_arena.device_ptr(&h_arena_dev);
  if (e == hipSuccess) e = ws->h_stats.device_ptr(&h_stats_dev);
  if (e == hipSuccess) e = pgpu_launch_prologue(p, h_arena_dev, ws->arena.p, total, p.mode != PGPU_MODE_AGG, st);
  if (e == hipSuccess) e = hipEventRecord(ws->ev0, st);
  // raw-value leaves' match bitmaps (timed with the query: they are part of its filter)
  if (e == hipSuccess && !pk.raws.empty())
    e = pgpu_launch_rawpred((const RawLeaf*)(d + o_raw), (int)pk.raws.size(), max_raw_words, st);
  if (e == hipSuccess && !pk.mvs.empty())
    e = pgpu_launch_mvpred((const MvLeaf*)(d + o_mv), (int)pk.mvs.size(), max_mv_words, st);
  p.invx = (const InvLeafX*)(d + o_inv);
  bool expand = false;  // (query_kernel_rkey and query_kernel_cand read their leaves' containers themselves)
  for (const InvLeafX& x : pk.invx) expand |= !x.skip;
  if (e == hipSuccess && expand && p.direct != 5)
    e = pgpu_launch_invexp((const InvLeafX*)(d + o_inv), (int)pk.invx.size(), max_inv_words, st);
  if (e == hipSuccess && p.direct == 5) {
    int64_t max_pairs = 0;
    for (const InvLeafX& x : pk.invx) max_pairs = std::max<int64_t>(max_pairs, (int64_t)x.nids * x.nkeys);
    e = pgpu_launch_rkey_ctab((const InvLeafX*)(d + o_inv), (int)pk.invx.size(), max_pairs,
                              (DevContainer*)ws->rkctab.p, st);
  }
  if (e == hipSuccess && !pk.jobs.empty())
    e = pgpu_launch_progbits(p, (const ProgJob*)(d + o_jobs), (int)pk.jobs.size(), pk.job_tiles, st);
  if (e == hipSuccess)
    e = p.pscan ? pgpu_launch_part_scan(p, grid, dyn, st)
                : (p.direct ? pgpu_launch_query_direct(p, grid, dyn, st) : pgpu_launch_query(p, grid, dyn, st));
  if (e == hipSuccess && p.mode == PGPU_MODE_PART) e = pgpu_launch_part_reduce(p, grid, st);
  // the reference's filter statistic (andfsm maps or leaf bitmaps for the host replay) is part of the query's
  // kernels: ev0 .. ev1 spans every kernel that reads the segments, so kernel_ms prices the whole step's reads
  if (e == hipSuccess && pk.fsm) {
    void* h_ent_dev = nullptr;
    e = ws->h_fsment.device_ptr(&h_ent_dev);
    if (e == hipSuccess) e = pgpu_launch_andfsm(p, pk.fsm_s2, (uint32_t*)ws->fsmfn.p, (int64_t*)h_ent_dev, st);
  }
  if (e == hipSuccess && pk.leaf_words > 0) e = pgpu_launch_leafbits(p, st);
  if (e == hipSuccess) e = hipEventRecord(ws->ev1, st);
  // statistics, numSegmentsMatched flags and a small table into pinned host memory: one launch
  if (e == hipSuccess) {
    void* h_seg_dev = nullptr;
    e = ws->h_segany.device_ptr(&h_seg_dev);
    if (e == hipSuccess)
      e = pgpu_launch_finalize(p, nwaves, (int64_t*)h_stats_dev, (uint8_t*)h_seg_dev, host_table,
                               host_table ? pgpu_table_bytes(&L) / 8 : 0, st);
  }
  if (e == hipSuccess && p.mode == PGPU_MODE_HASH) {
    // probe-overflow flag and the tracked segments' distinct-key counts, into pinned host memory
    void* h_cnt_dev = nullptr;
    if (p.segmask_rows) {
      e = ws->h_segcnt.device_ptr(&h_cnt_dev);
      if (e == hipSuccess) e = pgpu_launch_segcount(p, (int64_t*)h_cnt_dev, st);
    }
    if (e == hipSuccess) e = hipMemcpyAsync((char*)ws->h_stats.p + 8 * PGPU_NSTATS, ws->hflag.p, 4, hipMemcpyDeviceToHost, st);
  }
  if (e == hipSuccess && pk.leaf_words > 0)
    e = hipMemcpyAsync(ws->h_leafbits.p, ws->leafbits.p, 4ull * pk.leaf_words, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && eager) {
    const int crc = enqueue_compact(ctx, ws, &L, dev_table, st, eager_order);
    if (crc) return bail(crc);
  }
  // completion of this query alone (later queries may already be queued behind it on the same stream)
  if (e == hipSuccess) e = hipEventRecord(ws->done, st);
  if (e != hipSuccess) return bail(fail(PGPU_E_HIP, "query launch: %s", hipGetErrorString(e)));

  host_timing().add(4, tl0, HostTiming::us());
  auto* qq = new pgpu_query();
  qq->ctx = ctx;
  qq->ws = ws;
  qq->done = ws->done;
  qq->eager = eager;
  qq->stream = st;
  qq->params = p;
  qq->grid = grid;
  memset(&qq->stats, 0, sizeof(qq->stats));
  int64_t tot_docs = 0;
  for (int s = 0; s < q->num_segments; ++s) tot_docs += q->segments[s].segment->num_docs;
  qq->stats.num_total_docs = tot_docs;
  qq->tracked = pk.tracked;
  for (int32_t s : pk.tracked) qq->tracked_map.push_back(segment_map_based(q, q->segments[s]) ? 1 : 0);
  qq->groups_limit = q->num_groups_limit;
  qq->exact_filter = pk.leaf_words > 0;
  qq->exact_fsm = pk.fsm;
  bool exact = true;
  for (int s = 0; s < q->num_segments; ++s) {
    const pgpu_segment_plan& sp = q->segments[s];
    exact = exact && !pk.legacy_range && pgpu_filter_count_is_reference(sp.filter, sp.num_filter_nodes);
    // multi-value SCAN leaves read row lengths, not one entry per doc: a lone one reads every row (all values);
    // elsewhere only the replay knows which rows the reference's iterators read
    std::vector<const int32_t*> leaf_off;
    int nmv = 0;
    for (int i = 0; i < sp.num_filter_nodes; ++i) {
      const pgpu_filter_node& nd = sp.filter[i];
      const bool leaf = nd.op == PGPU_F_SCAN || nd.op == PGPU_F_INVERTED || nd.op == PGPU_F_SORTED ||
                        nd.op == PGPU_F_RAW_SCAN || nd.op == PGPU_F_RANGE_INDEX;
      if (!leaf) continue;
      const HostColumn* hc = nullptr;
      if (nd.op == PGPU_F_SCAN && nd.column >= 0 && nd.column < q->num_columns) {
        const int32_t slot = sp.column_map[nd.column];
        if (slot >= 0 && slot < (int32_t)sp.segment->cols.size()) hc = &sp.segment->cols[slot];
      }
      const bool mv = hc && hc->kind == PGPU_COL_MV;
      leaf_off.push_back(mv ? hc->mv_offsets.data() : nullptr);
      nmv += mv;
    }
    if (nmv && sp.num_filter_nodes == 1) qq->mv_entries += sp.segment->cols[sp.column_map[sp.filter[0].column]].mv_values;
    else if (nmv) exact = false;
    if (!qq->exact_filter) continue;
    pgpu_query::FilterReplay r;
    r.nodes.assign(sp.filter, sp.filter + sp.num_filter_nodes);
    r.ids.resize(sp.num_filter_nodes);
    for (int i = 0; i < sp.num_filter_nodes; ++i) {
      const int k = sp.filter[i].op == PGPU_F_SORTED ? 2 * sp.filter[i].num_ids : sp.filter[i].num_ids;
      if (sp.filter[i].ids && k > 0) r.ids[i].assign(sp.filter[i].ids, sp.filter[i].ids + k);
      r.nodes[i].ids = nullptr;
    }
    r.num_docs = sp.segment->num_docs;
    r.num_leaves = pk.segs[s].leaf_len;
    r.ntiles = pk.segs[s].ntiles;
    r.bits_off = pk.segs[s].leaf_bits_off;
    r.leaf_off = std::move(leaf_off);
    qq->replay.push_back(std::move(r));
  }
  qq->stats.filter_stats_exact = exact ? 1 : 0;
  qq->deadline_ms = q->deadline_ms;
  if (expired) qq->stop = PGPU_E_TIMEOUT;
  *out_query = qq;
  return PGPU_OK;
}


int pgpu_query_launch(pgpu_context* ctx, const pgpu_query_desc* q, void* stream, void* dev_table,
                      uint64_t table_bytes, pgpu_query** out_query) {
  return launch_impl(ctx, q, stream, dev_table, table_bytes, nullptr, out_query);
}

// Write the query's generation into its cancel word from the context's side stream (the query stream is busy).
static int signal_cancel(pgpu_query* qq) {
  HIP_TRY(hipSetDevice(qq->ctx->device));
  hipStream_t cs = nullptr;
  {
    std::lock_guard<std::mutex> lk(qq->ctx->mu);
    if (!qq->ctx->cstream) HIP_TRY(hipStreamCreateWithFlags(&qq->ctx->cstream, hipStreamNonBlocking));
    cs = qq->ctx->cstream;
  }
  // A copy-engine (SDMA) write from pinned host memory: it lands while the query kernel holds every CU, where a
  // memset -- a blit kernel -- would only run after the kernel it is meant to stop.
  if (!qq->ws->h_cancel.p) return fail(PGPU_E_INVALID, "query has no cancel word");
  __atomic_store_n((volatile uint32_t*)qq->ws->h_cancel.p, qq->params.cancel_gen, __ATOMIC_SEQ_CST);
  HIP_TRY(hipMemcpyAsync((void*)qq->params.cancel, qq->ws->h_cancel.p, 4, hipMemcpyHostToDevice, cs));
  return PGPU_OK;
}

int pgpu_query_matched_segments(pgpu_query* qq, uint8_t* out, int32_t num_segments) {
  if (!qq || !out) return fail(PGPU_E_INVALID, "null argument");
  if (num_segments != qq->params.nseg)
    return fail(PGPU_E_INVALID, "matched-segment flags: %d entries for a %d-segment query", num_segments, qq->params.nseg);
  qq->matched_out = out;
  return PGPU_OK;
}

int pgpu_query_cancel(pgpu_query* qq) {
  if (!qq) return fail(PGPU_E_INVALID, "null query");
  int none = 0;
  if (!qq->stop.compare_exchange_strong(none, PGPU_E_CANCELLED)) return PGPU_OK;  // already stopped
  return signal_cancel(qq);
}

int pgpu_query_wait(pgpu_query* qq, pgpu_query_stats* out_stats) {
  if (!qq) return fail(PGPU_E_INVALID, "null query");
  HIP_TRY(hipSetDevice(qq->ctx->device));
  if (qq->deadline_ms > 0 && qq->done) {
    // BaseCombineOperator.mergeResults polls with the time left: past the deadline the query is told to stop
    // and drains (its kernels skip their remaining tiles)
    for (int spins = 0;; ++spins) {
      const hipError_t qe = hipEventQuery(qq->done);
      if (qe == hipSuccess) break;
      if (qe != hipErrorNotReady) return fail(PGPU_E_HIP, "query wait: %s", hipGetErrorString(qe));
      if (qq->stop.load() == 0 && now_epoch_ms() >= qq->deadline_ms) {
        int none = 0;
        if (qq->stop.compare_exchange_strong(none, PGPU_E_TIMEOUT)) {
          const int rc = signal_cancel(qq);
          if (rc) return rc;
        }
      }
      if (spins < 2000) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  } else if (qq->done) {
    HIP_TRY(hipEventSynchronize(qq->done));
  } else {
    HIP_TRY(hipStreamSynchronize(qq->stream));
  }
  const int64_t* s = (const int64_t*)qq->ws->h_stats.p;
  qq->stats.num_docs_scanned = s[PGPU_STAT_MATCHED];
  qq->stats.num_entries_scanned_in_filter = s[PGPU_STAT_SCANNED] + qq->mv_entries;
  qq->stats.sparse_sector_bytes = s[PGPU_STAT_SECTOR_BYTES];
  qq->stats.dense_bytes = s[PGPU_STAT_DENSE_BYTES];
  {
    const uint8_t* f = (const uint8_t*)qq->ws->h_segany.p;
    int64_t nm = 0;
    for (int i = 0; i < qq->params.nseg; ++i) nm += f[i] != 0;
    qq->stats.num_segments_matched = nm;
    if (qq->matched_out) memcpy(qq->matched_out, f, (size_t)qq->params.nseg);
  }
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, qq->ws->ev0, qq->ws->ev1));
  qq->stats.kernel_ms = ms;
  qq->stats.kernel_variant = qq->params.pscan ? PGPU_KV_PSCAN : qq->params.direct;
  if (const int st = qq->stop.load()) {
    if (out_stats) *out_stats = qq->stats;
    return fail(st, st == PGPU_E_TIMEOUT ? "query passed its deadline before it finished (EXECUTION_TIMEOUT_ERROR)"
                                         : "query cancelled");
  }
  if (qq->exact_fsm) {
    const int64_t* ent = (const int64_t*)qq->ws->h_fsment.p;
    int64_t total = 0;
    for (int i = 0; i < qq->params.nseg; ++i) total += ent[i];
    qq->stats.num_entries_scanned_in_filter = total;
    qq->stats.filter_stats_exact = 1;
  }
  if (qq->exact_filter) {
    // the reference's iterators replayed over the leaves' bitmaps (pgpu_iterstats.cpp)
    // one segment per task on up to 16 host threads (segments replay independently, as the reference's
    // per-segment operators run on its query executor's threads)
    const uint32_t* bits = (const uint32_t*)qq->ws->h_leafbits.p;
    const size_t nr = qq->replay.size();
    std::vector<int64_t> counts(nr, 0);
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t i = next++; i < nr; i = next++) {
        const pgpu_query::FilterReplay& r = qq->replay[i];
        std::vector<const uint32_t*> leaf(r.num_leaves);
        for (int k = 0; k < r.num_leaves; ++k) leaf[k] = bits + r.bits_off + (int64_t)k * r.ntiles * 64;
        counts[i] = reference_entries_scanned(r.nodes.data(), (int)r.nodes.size(), leaf.data(), r.num_leaves,
                                              r.num_docs, r.leaf_off.empty() ? nullptr : r.leaf_off.data());
      }
    };
    const size_t nthreads = std::min<size_t>({nr, 16, std::max(1u, std::thread::hardware_concurrency() / 2)});
    std::vector<std::thread> pool;
    for (size_t t = 1; t < nthreads; ++t) pool.emplace_back(work);
    work();
    for (std::thread& t : pool) t.join();
    int64_t total = 0;
    for (int64_t c : counts) {
      if (c < 0) return fail(PGPU_E_INVALID, "filter program cannot be replayed for statistics");
      total += c;
    }
    qq->stats.num_entries_scanned_in_filter = total;
    qq->stats.filter_stats_exact = 1;
  }
  if (qq->params.mode == PGPU_MODE_HASH) {
    int32_t flag = 0;
    memcpy(&flag, (const char*)qq->ws->h_stats.p + 8 * PGPU_NSTATS, 4);
    if (flag) {
      // the table holds every segment's bound (its key space, docs, and numGroupsLimit for a map-based holder): an
      // overflow means a tracked segment met more keys than numGroupsLimit
      if (out_stats) *out_stats = qq->stats;
      if (!qq->tracked.empty())
        return fail(PGPU_E_GROUPS_LIMIT, "hash group-by table overflow: a segment meets more distinct group keys than "
                    "numGroupsLimit %lld (the reference keeps the first-seen keys only)", (long long)qq->groups_limit);
      return fail(PGPU_E_UNSUPPORTED, "hash group-by table overflow (more distinct keys than the holder limits allow)");
    }
    const int64_t* cnt = (const int64_t*)qq->ws->h_segcnt.p;
    for (size_t i = 0; i < qq->tracked.size(); ++i)
      if (cnt[i] >= qq->groups_limit) qq->stats.num_groups_limit_reached = 1;
    for (size_t i = 0; i < qq->tracked.size(); ++i)
      if (cnt[i] > qq->groups_limit && qq->tracked_map[i]) {
        if (out_stats) *out_stats = qq->stats;
        return fail(PGPU_E_GROUPS_LIMIT,
                    "segment %d meets %lld distinct group keys > numGroupsLimit %lld: the reference keeps the "
                    "first-seen keys only (DictionaryBasedGroupKeyGenerator)",
                    qq->tracked[i], (long long)cnt[i], (long long)qq->groups_limit);
      }
  }
  if (qq->params.flags & PGPU_FLAG_PROFILE) {
    const int nw = qq->grid * (qq->params.direct || qq->params.pscan ? 4 : PGPU_WAVES_OF(qq->params.dense));
    std::vector<int64_t> pr((size_t)nw * PGPU_NPROF);
    HIP_TRY(hipMemcpy(pr.data(), qq->params.prof, pr.size() * 8, hipMemcpyDeviceToHost));
    double sum[PGPU_NPROF] = {0};
    int nl = 0, nc = 0;
    for (int w = 0; w < nw; ++w) {
      const bool ld = !qq->params.direct && !qq->params.pscan &&
                      (w % PGPU_WAVES_OF(qq->params.dense)) < PGPU_NLOAD_OF(qq->params.dense);
      ld ? ++nl : ++nc;
      for (int k = 0; k < PGPU_NPROF; ++k) sum[k] += (double)pr[(size_t)w * PGPU_NPROF + k];
    }
    // raw s_memtime ticks per wave (shader clock)
    fprintf(stderr,
            "[pgpu profile] kernel %.3f ms | loader/wave: total %.0f free %.0f pub %.0f issue %.0f | consumer/wave: "
            "total %.0f full %.0f filter %.0f (fetch %.0f decode %.0f) agg %.0f flush %.0f tiles %.1f\n",
            ms, sum[0] / nl, sum[1] / nl, sum[2] / nl, sum[3] / nl, sum[4] / nc, sum[5] / nc, sum[6] / nc,
            sum[10] / nc, sum[11] / nc, sum[7] / nc, sum[8] / nc, sum[9] / nc);
  }
  if (out_stats) *out_stats = qq->stats;
  return PGPU_OK;
}

int pgpu_query_release(pgpu_query* qq) {
  if (!qq) return PGPU_OK;
  // the workspaces may still be in use by queued work of this query
  if (qq->done) (void)hipEventSynchronize(qq->done);
  else (void)hipStreamSynchronize(qq->stream);
  if (qq->tws) release_ws(qq->ctx, qq->tws);
  release_ws(qq->ctx, qq->ws);
  delete qq;
  return PGPU_OK;
}

}  // extern "C"

namespace {

// The order key of a pgpu_topk over a table layout (include/pinot_gpu.h; keys in pgpu_internal.h).
int topk_spec(const pgpu_table_layout* L, const pgpu_topk* o, TopkDev* out) {
  TopkDev t{};
  t.G = L->num_keys;
  t.nsec = L->num_sections;
  t.kw = L->key_kind == PGPU_KEYS_HASH ? L->key_words : 0;
  t.desc = o->descending ? 1 : 0;
  t.key_base = o->key_base;
  if (o->source == PGPU_TOPK_AGG) {
    const int a = o->agg_index;
    if (a < 0 || a >= 16) return fail(PGPU_E_INVALID, "top-k aggregation index %d", a);
    const int sec = L->agg_section[a];
    t.sec = sec;
    const bool split = L->agg_sum_parts[a] > 1;
    const int op = L->section_op[sec];
    const int vt = L->agg_value_type[a];
    t.fxe = split && (vt == PGPU_FLOAT || vt == PGPU_DOUBLE) ? L->agg_sum_exp[a] : 0;
    t.parts = split ? L->agg_sum_parts[a] : 1;
    switch (o->agg_fn) {
      case PGPU_AGG_COUNT: t.mode = PGPU_TK_COUNT; break;
      case PGPU_AGG_SUM:
        t.mode = op == PGPU_RED_SUM_F64 ? PGPU_TK_SUM_F64 : (split ? PGPU_TK_SUM_SPLIT : PGPU_TK_SUM_I64);
        break;
      case PGPU_AGG_AVG:
        t.mode = op == PGPU_RED_SUM_F64 ? PGPU_TK_AVG_F64 : (split ? PGPU_TK_AVG_SPLIT : PGPU_TK_AVG_I64);
        break;
      case PGPU_AGG_MIN:
      case PGPU_AGG_MAX:
        t.mode = (vt == PGPU_INT || vt == PGPU_LONG) ? PGPU_TK_MINMAX_INT : PGPU_TK_MINMAX_FP;
        break;
      default: return fail(PGPU_E_INVALID, "top-k aggregation fn %d", o->agg_fn);
    }
    if (o->agg_fn != PGPU_AGG_COUNT && sec <= 0) return fail(PGPU_E_INVALID, "top-k aggregation %d has no section", a);
  } else if (o->source == PGPU_TOPK_GROUP) {
    const int g = o->group_index, n = o->num_group_columns;
    if (g < 0 || g >= n || !o->group_cardinalities) return fail(PGPU_E_INVALID, "top-k group column %d", g);
    const int split = t.kw == 2 ? L->key_split : n;
    t.word = g < split ? 0 : 1;
    uint64_t st = 1;
    for (int j = t.word == 0 ? 0 : split; j < g; ++j) st *= (uint64_t)std::max(1, o->group_cardinalities[j]);
    t.stride = st;
    t.card = (uint64_t)std::max(1, o->group_cardinalities[g]);
    t.mode = PGPU_TK_GROUP;
  } else {
    return fail(PGPU_E_INVALID, "top-k source %d", o->source);
  }
  *out = t;
  return PGPU_OK;
}

// Compact the non-empty rows of a device table into host buffers; with `order` (k > 0) only the best k by its key
// (ties with the k-th kept), selected on the device by radix select.
int compact_into(pgpu_context* ctx, Workspace* ws, const pgpu_table_layout* L, const void* dev_table,
                 hipStream_t st, int64_t* out_keys, int64_t* out_cells, uint64_t capacity,
                 uint64_t* out_num_groups, const pgpu_topk* order = nullptr) {
  const uint64_t G = L->num_keys;
  const int nsec = L->num_sections;
  const int kw = L->key_kind == PGPU_KEYS_HASH ? L->key_words : 0;  // 0: the cell index is the key
  const int okw = kw > 1 ? kw : 1;
  const uint64_t nb = (G + 4095) / 4096;
  HIP_TRY(ws->cmp_counts.ensure(4 * nb + 16, ctx->mpool, st));
  HIP_TRY(ws->cmp_total.ensure(16, ctx->mpool, st));
  HIP_TRY(ws->h_total.ensure(16));
  const uint64_t* okey = nullptr;
  const TopkState* tstate = nullptr;
  if (order && order->k > 0 && G > order->k) {  // a table of at most k cells has nothing to trim
    TopkDev spec;
    const int rc = topk_spec(L, order, &spec);
    if (rc) return rc;
    HIP_TRY(ws->tk_keys.ensure(8 * G + 16, ctx->mpool, st));
    HIP_TRY(ws->tk_state.ensure(sizeof(TopkState) + 4 * 256 + 16, ctx->mpool, st));
    TopkState* ts = (TopkState*)ws->tk_state.p;
    uint32_t* hist = (uint32_t*)((char*)ws->tk_state.p + sizeof(TopkState));
    HIP_TRY(pgpu_launch_topk((const int64_t*)dev_table, spec, order->k, (uint64_t*)ws->tk_keys.p, ts, hist, st));
    okey = (const uint64_t*)ws->tk_keys.p;
    tstate = ts;
  }
  HIP_TRY(pgpu_launch_compact((const int64_t*)dev_table, G, nsec, kw, (int32_t*)ws->cmp_counts.p,
                              (int64_t*)ws->cmp_total.p, nullptr, nullptr, true, st, okey, tstate));
  HIP_TRY(hipMemcpyAsync(ws->h_total.p, ws->cmp_total.p, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t n = (uint64_t)*(const int64_t*)ws->h_total.p;
  *out_num_groups = n;
  if (n > capacity)
    return fail(PGPU_E_INVALID, "%llu non-empty groups exceed capacity %llu", (unsigned long long)n,
                (unsigned long long)capacity);
  if (n == 0) return PGPU_OK;
  HIP_TRY(ws->cmp_keys.ensure(8 * n * okw, ctx->mpool, st));
  HIP_TRY(ws->cmp_cells.ensure(8 * n * nsec, ctx->mpool, st));
  HIP_TRY(pgpu_launch_compact((const int64_t*)dev_table, G, nsec, kw, (int32_t*)ws->cmp_counts.p, nullptr,
                              (int64_t*)ws->cmp_keys.p, (int64_t*)ws->cmp_cells.p, false, st, okey, tstate));
  HIP_TRY(hipMemcpyAsync(out_keys, ws->cmp_keys.p, 8 * n * okw, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(out_cells, ws->cmp_cells.p, 8 * n * nsec, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  (void)ctx;
  return PGPU_OK;
}

// The device half of compact_into, enqueued without any host synchronisation (pgpu_query_submit): capacity for
// every key, the row count copied into pinned memory.  pgpu_query_collect reads it and copies the rows out.
int enqueue_compact(pgpu_context* ctx, Workspace* ws, const pgpu_table_layout* L, const void* dev_table,
                    hipStream_t st, const pgpu_topk* order) {
  const uint64_t G = L->num_keys;
  const int nsec = L->num_sections;
  const int kw = L->key_kind == PGPU_KEYS_HASH ? L->key_words : 0;
  const int okw = kw > 1 ? kw : 1;
  const uint64_t nb = (G + 4095) / 4096;
  HIP_TRY(ws->cmp_counts.ensure(4 * nb + 16, ctx->mpool, st));
  HIP_TRY(ws->cmp_total.ensure(16, ctx->mpool, st));
  HIP_TRY(ws->h_total.ensure(16));
  HIP_TRY(ws->cmp_keys.ensure(8 * G * okw + 16, ctx->mpool, st));
  HIP_TRY(ws->cmp_cells.ensure(8 * G * nsec + 16, ctx->mpool, st));
  const uint64_t* okey = nullptr;
  const TopkState* tstate = nullptr;
  if (order && order->k > 0 && G > order->k) {
    TopkDev spec;
    const int rc = topk_spec(L, order, &spec);
    if (rc) return rc;
    HIP_TRY(ws->tk_keys.ensure(8 * G + 16, ctx->mpool, st));
    HIP_TRY(ws->tk_state.ensure(sizeof(TopkState) + 4 * 256 + 16, ctx->mpool, st));
    TopkState* ts = (TopkState*)ws->tk_state.p;
    uint32_t* hist = (uint32_t*)((char*)ws->tk_state.p + sizeof(TopkState));
    HIP_TRY(pgpu_launch_topk((const int64_t*)dev_table, spec, order->k, (uint64_t*)ws->tk_keys.p, ts, hist, st));
    okey = (const uint64_t*)ws->tk_keys.p;
    tstate = ts;
  }
  HIP_TRY(pgpu_launch_compact((const int64_t*)dev_table, G, nsec, kw, (int32_t*)ws->cmp_counts.p,
                              (int64_t*)ws->cmp_total.p, nullptr, nullptr, true, st, okey, tstate));
  HIP_TRY(pgpu_launch_compact((const int64_t*)dev_table, G, nsec, kw, (int32_t*)ws->cmp_counts.p, nullptr,
                              (int64_t*)ws->cmp_keys.p, (int64_t*)ws->cmp_cells.p, false, st, okey, tstate));
  HIP_TRY(hipMemcpyAsync(ws->h_total.p, ws->cmp_total.p, 8, hipMemcpyDeviceToHost, st));
  return PGPU_OK;
}

// compact_into's passes with the rows left in device buffers (keys [n][max(kw, 1)], cells [n][nsec])
int compact_device(pgpu_context* ctx, Workspace* ws, const pgpu_table_layout* L, const void* dev_table,
                   hipStream_t st, int64_t* dkeys, int64_t* dcells, uint64_t capacity, uint64_t* out_n) {
  const uint64_t G = L->num_keys;
  const int nsec = L->num_sections;
  const int kw = L->key_kind == PGPU_KEYS_HASH ? L->key_words : 0;
  const uint64_t nb = (G + 4095) / 4096;
  HIP_TRY(ws->cmp_counts.ensure(4 * nb + 16, ctx->mpool, st));
  HIP_TRY(ws->cmp_total.ensure(16, ctx->mpool, st));
  HIP_TRY(ws->h_total.ensure(16));
  HIP_TRY(pgpu_launch_compact((const int64_t*)dev_table, G, nsec, kw, (int32_t*)ws->cmp_counts.p,
                              (int64_t*)ws->cmp_total.p, nullptr, nullptr, true, st, nullptr, nullptr));
  HIP_TRY(hipMemcpyAsync(ws->h_total.p, ws->cmp_total.p, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  const uint64_t n = (uint64_t)*(const int64_t*)ws->h_total.p;
  *out_n = n;
  if (n > capacity) return fail(PGPU_E_INVALID, "%llu rows exceed the device buffer", (unsigned long long)n);
  if (n == 0) return PGPU_OK;
  HIP_TRY(pgpu_launch_compact((const int64_t*)dev_table, G, nsec, kw, (int32_t*)ws->cmp_counts.p, nullptr, dkeys,
                              dcells, false, st, nullptr, nullptr));
  HIP_TRY(hipStreamSynchronize(st));
  return PGPU_OK;
}

}  // namespace

// pgpu_node.cpp: the non-empty rows of a (hash) table compacted into device buffers that hold `capacity` rows.
int pgpu_compact_to_device(pgpu_context* ctx, const pgpu_table_layout* L, const void* dev_table, hipStream_t st,
                           int64_t* dkeys, int64_t* dcells, uint64_t capacity, uint64_t* out_n) {
  if (!ctx || !L || !dev_table || !out_n) return fail(PGPU_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(ctx->device));
  int rc = 0;
  Workspace* ws = acquire_ws(ctx, &rc);
  if (!ws) return rc;
  rc = compact_device(ctx, ws, L, dev_table, st ? st : ws->stream, dkeys, dcells, capacity, out_n);
  release_ws(ctx, ws);
  return rc;
}

extern "C" {

int pgpu_table_compact(pgpu_context* ctx, const pgpu_table_layout* layout, const void* dev_table, void* stream,
                       int64_t* out_keys, int64_t* out_cells, uint64_t capacity, uint64_t* out_num_groups) {
  if (!ctx || !layout || !dev_table || !out_num_groups) return fail(PGPU_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(ctx->device));
  int rc = 0;
  Workspace* ws = acquire_ws(ctx, &rc);
  if (!ws) return rc;
  rc = compact_into(ctx, ws, layout, dev_table, stream ? (hipStream_t)stream : ws->stream, out_keys, out_cells,
                    capacity, out_num_groups);
  release_ws(ctx, ws);
  return rc;
}

int pgpu_table_topk(pgpu_context* ctx, const pgpu_table_layout* layout, const void* dev_table, void* stream,
                    const pgpu_topk* order, int64_t* out_keys, int64_t* out_cells, uint64_t capacity,
                    uint64_t* out_num_groups) {
  if (!ctx || !layout || !dev_table || !out_num_groups) return fail(PGPU_E_INVALID, "null argument");
  HIP_TRY(hipSetDevice(ctx->device));
  int rc = 0;
  Workspace* ws = acquire_ws(ctx, &rc);
  if (!ws) return rc;
  rc = compact_into(ctx, ws, layout, dev_table, stream ? (hipStream_t)stream : ws->stream, out_keys, out_cells,
                    capacity, out_num_groups, order);
  release_ws(ctx, ws);
  return rc;
}

}  // extern "C"

// ---- per-segment filter planning from literal predicates (pgpu_query_*_expr) --------------------------------------
// The host-side work the reference does per segment before any doc is touched, restated in C++ for numeric
// columns (pinot_amd/plan.py + predicate.py are the same rules in Python, used for STRING columns):
//   dictionary predicate evaluators (core/operator/filter/predicate/<X>PredicateEvaluatorFactory.java; literal
//     lookups = BaseImmutableDictionary.insertionIndexOf, seglocal/.../BaseImmutableDictionary.java:125-270),
//   FilterPlanNode.constructPhysicalOperator (core/plan/FilterPlanNode.java:192-313) and FilterOperatorUtils
//     (EMPTY / MATCH_ALL folding, leaf choice sorted > inverted > scan, stable AND re-ordering by priority;
//     core/operator/filter/FilterOperatorUtils.java:42-221).
namespace {

struct Leaf {
  int kind;  // 0 EMPTY, 1 ALL, 2 SCAN, 3 INV, 4 SORTED
  bool exclusive = false;
  bool range = false;  // RANGE evaluator [start, end)
  int32_t start = 0, end = 0;
  std::vector<int32_t> ids;  // SET evaluator: matching ids, or non-matching ids for exclusive predicates
};

struct PlanNode {
  int kind;  // 0 EMPTY, 1 ALL, 2 SCAN, 3 INV, 4 SORTED, 5 AND, 6 OR, 7 NOT
  int column = -1;
  Leaf leaf;
  std::vector<PlanNode> kids;
  int priority() const {
    switch (kind) {
      case 4: return 0;
      case 3: return 1;
      case 5: return 3;
      case 6: return 4;
      case 7: return kids[0].priority();
      default: return 5;
    }
  }
};

// BaseImmutableDictionary.insertionIndexOf: >= 0 exact match index, else -(insertion point + 1)
int64_t insertion_index(const HostColumn& c, const pgpu_literal& lit) {
  const int32_t n = c.dict_card;
  const uint8_t* d = c.hdict.data();
  int64_t lo = 0, hi = n;
  if (c.dict_type == PGPU_INT || c.dict_type == PGPU_LONG) {
    auto at = [&](int64_t i) -> int64_t {
      if (c.dict_type == PGPU_INT) { int32_t v; memcpy(&v, d + 4 * i, 4); return v; }
      int64_t v; memcpy(&v, d + 8 * i, 8); return v;
    };
    if (lit.is_integral) {
      while (lo < hi) { const int64_t m = (lo + hi) / 2; if (at(m) < lit.i) lo = m + 1; else hi = m; }
      return lo < n && at(lo) == lit.i ? lo : -(lo + 1);
    }
    // a fractional literal on an integer dictionary is never equal; its insertion point compares as double
    while (lo < hi) { const int64_t m = (lo + hi) / 2; if ((double)at(m) < lit.d) lo = m + 1; else hi = m; }
    return -(lo + 1);
  }
  double key = lit.d;
  if (c.dict_type == PGPU_FLOAT) key = (double)(float)lit.d;
  auto at = [&](int64_t i) -> double {
    if (c.dict_type == PGPU_FLOAT) { float v; memcpy(&v, d + 4 * i, 4); return v; }
    double v; memcpy(&v, d + 8 * i, 8); return v;
  };
  while (lo < hi) { const int64_t m = (lo + hi) / 2; if (at(m) < key) lo = m + 1; else hi = m; }
  return lo < n && at(lo) == key ? lo : -(lo + 1);
}

// PredicateEvaluatorProvider.getPredicateEvaluator for dictionary-encoded columns
Leaf evaluate(const HostColumn& c, const pgpu_expr_node& x) {
  Leaf l;
  const int32_t card = c.dict_card;
  auto index_of = [&](const pgpu_literal& v) -> int32_t {
    const int64_t i = insertion_index(c, v);
    return i >= 0 ? (int32_t)i : -1;
  };
  auto id_set = [&]() {
    std::vector<int32_t> ids;
    for (int k = 0; k < x.num_values; ++k) {
      const int32_t i = index_of(x.values[k]);
      if (i >= 0) ids.push_back(i);
    }
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    return ids;
  };
  switch (x.pred) {
    case PGPU_P_EQ: {
      const int32_t i = x.num_values > 0 ? index_of(x.values[0]) : -1;
      if (i < 0) { l.kind = 0; return l; }
      l.kind = card == 1 ? 1 : 2;
      l.ids = {i};
      return l;
    }
    case PGPU_P_NOT_EQ: {
      const int32_t i = x.num_values > 0 ? index_of(x.values[0]) : -1;
      if (i < 0) { l.kind = 1; return l; }
      l.kind = card == 1 ? 0 : 2;
      l.exclusive = true;
      l.ids = {i};
      return l;
    }
    case PGPU_P_IN:
      l.ids = id_set();
      l.kind = l.ids.empty() ? 0 : ((int32_t)l.ids.size() == card ? 1 : 2);
      return l;
    case PGPU_P_NOT_IN:
      l.ids = id_set();
      l.exclusive = true;
      l.kind = l.ids.empty() ? 1 : ((int32_t)l.ids.size() == card ? 0 : 2);
      return l;
    default: {  // RANGE
      int64_t start = 0, end = card;
      if (!x.lower_unbounded) {
        const int64_t ins = insertion_index(c, x.values[0]);
        start = ins < 0 ? -(ins + 1) : (x.lower_inclusive ? ins : ins + 1);
      }
      if (!x.upper_unbounded) {
        const int64_t ins = insertion_index(c, x.values[x.num_values - 1]);
        end = ins < 0 ? -(ins + 1) : (x.upper_inclusive ? ins + 1 : ins);
      }
      l.range = true;
      l.start = (int32_t)start;
      l.end = (int32_t)end;
      const int64_t n = end - start;
      l.kind = n <= 0 ? 0 : (n == card ? 1 : 2);
      return l;
    }
  }
}

struct ExprPlanner {
  const pgpu_query_desc* q;
  const pgpu_segment_plan* sp;
  const pgpu_segment* seg;
  const pgpu_expr_node* x;
  int n;
  int err = PGPU_OK;

  const HostColumn* column(int qc) {
    if (qc < 0 || qc >= q->num_columns) { err = fail(PGPU_E_INVALID, "expression column %d", qc); return nullptr; }
    const int32_t slot = sp->column_map[qc];
    if (slot < 0 || slot >= (int32_t)seg->cols.size()) { err = fail(PGPU_E_INVALID, "expression column slot"); return nullptr; }
    const HostColumn& c = seg->cols[slot];
    if (c.dict_type < PGPU_INT || c.dict_type > PGPU_DOUBLE || c.hdict.empty()) {
      err = fail(PGPU_E_UNSUPPORTED, "expression on a non-numeric column (plan it on the host)");
      return nullptr;
    }
    return &c;
  }

  // FilterPlanNode.constructPhysicalOperator over the subtree starting at node i; *next = first node after it
  PlanNode build(int i, int* next) {
    PlanNode out;
    out.kind = 0;
    if (i >= n) { err = fail(PGPU_E_INVALID, "malformed filter expression"); *next = n; return out; }
    const pgpu_expr_node& e = x[i];
    if (e.op == PGPU_X_AND || e.op == PGPU_X_OR) {
      const bool is_and = e.op == PGPU_X_AND;
      int j = i + 1;
      std::vector<PlanNode> kids;
      bool empty = false, all = false;
      for (int k = 0; k < e.num_children && !err; ++k) {
        PlanNode ch = build(j, &j);
        if (is_and) {
          if (ch.kind == 0) empty = true;
          else if (ch.kind != 1) kids.push_back(std::move(ch));
        } else {
          if (ch.kind == 1) all = true;
          else if (ch.kind != 0) kids.push_back(std::move(ch));
        }
      }
      *next = j;
      if (is_and ? empty : all) { out.kind = is_and ? 0 : 1; return out; }
      if (kids.empty()) { out.kind = is_and ? 1 : 0; return out; }
      if (kids.size() == 1) return std::move(kids[0]);
      if (is_and)
        std::stable_sort(kids.begin(), kids.end(),
                         [](const PlanNode& a, const PlanNode& b) { return a.priority() < b.priority(); });
      out.kind = is_and ? 5 : 6;
      out.kids = std::move(kids);
      return out;
    }
    if (e.op == PGPU_X_NOT) {
      PlanNode ch = build(i + 1, next);
      if (ch.kind == 1) { out.kind = 0; return out; }
      if (ch.kind == 0) { out.kind = 1; return out; }
      out.kind = 7;
      out.kids.push_back(std::move(ch));
      return out;
    }
    *next = i + 1;
    const HostColumn* c = column(e.column);
    if (!c) return out;
    Leaf l = evaluate(*c, e);
    out.column = e.column;
    if (l.kind == 0 || l.kind == 1) { out.kind = l.kind; return out; }
    if (c->kind == PGPU_COL_SORTED) out.kind = 4;
    else if (e.pred != PGPU_P_RANGE && c->inv_card > 0) out.kind = 3;
    else out.kind = 2;
    out.leaf = std::move(l);
    return out;
  }

  // emit the prefix-order pgpu_filter_node program; id lists go to `pool` (offsets patched afterwards)
  void emit(const PlanNode& o, std::vector<pgpu_filter_node>& nodes, std::vector<int32_t>& pool,
            std::vector<std::pair<int, int>>& id_at) {
    pgpu_filter_node nd;
    memset(&nd, 0, sizeof(nd));
    auto with_ids = [&](const std::vector<int32_t>& v, int count) {
      id_at.emplace_back((int)nodes.size(), (int)pool.size());
      pool.insert(pool.end(), v.begin(), v.end());
      nd.num_ids = count;
    };
    switch (o.kind) {
      case 0: case 1:
        nd.op = o.kind == 0 ? PGPU_F_EMPTY : PGPU_F_MATCH_ALL;
        nodes.push_back(nd);
        return;
      case 2: {
        const Leaf& l = o.leaf;
        nd.op = PGPU_F_SCAN;
        nd.column = o.column;
        nd.negate = l.exclusive ? 1 : 0;
        if (l.range) {
          nd.pred = PGPU_PRED_RANGE; nd.lo = l.start; nd.hi = l.end;
        } else if (!l.ids.empty() && l.ids.back() - l.ids.front() + 1 == (int32_t)l.ids.size()) {
          nd.pred = PGPU_PRED_RANGE; nd.lo = l.ids.front(); nd.hi = l.ids.back() + 1;
        } else {
          nd.pred = PGPU_PRED_SET;
          with_ids(l.ids, (int)l.ids.size());
        }
        nodes.push_back(nd);
        return;
      }
      case 3: {  // INV: matching ids, or the non-matching ids of an exclusive predicate (flipped)
        const Leaf& l = o.leaf;
        nd.op = PGPU_F_INVERTED;
        nd.column = o.column;
        nd.negate = l.exclusive ? 1 : 0;
        with_ids(l.ids, (int)l.ids.size());
        nodes.push_back(nd);
        return;
      }
      case 4: {  // SORTED: doc ranges of the (non-)matching ids, adjacent ranges merged
        const Leaf& l = o.leaf;
        const HostColumn& c = seg->cols[sp->column_map[o.column]];
        std::vector<int32_t> flat;
        if (l.range) {
          flat = {c.sorted_pairs[2 * l.start], c.sorted_pairs[2 * (l.end - 1) + 1]};
        } else {
          for (int32_t id : l.ids) {
            const int32_t s0 = c.sorted_pairs[2 * id], e0 = c.sorted_pairs[2 * id + 1];
            if (!flat.empty() && s0 == flat.back() + 1) flat.back() = e0;
            else { flat.push_back(s0); flat.push_back(e0); }
          }
        }
        nd.op = PGPU_F_SORTED;
        nd.column = o.column;
        nd.negate = (l.exclusive && !l.range) ? 1 : 0;
        with_ids(flat, (int)flat.size() / 2);
        nodes.push_back(nd);
        return;
      }
      case 5: case 6: {
        const bool a = o.kind == 5;
        nd.op = a ? PGPU_F_AND_BEGIN : PGPU_F_OR_BEGIN;
        nodes.push_back(nd);
        for (const PlanNode& ch : o.kids) {
          emit(ch, nodes, pool, id_at);
          pgpu_filter_node ce;
          memset(&ce, 0, sizeof(ce));
          ce.op = a ? PGPU_F_AND_CHILD_END : PGPU_F_OR_CHILD_END;
          nodes.push_back(ce);
        }
        pgpu_filter_node en;
        memset(&en, 0, sizeof(en));
        en.op = a ? PGPU_F_AND_END : PGPU_F_OR_END;
        nodes.push_back(en);
        return;
      }
      default:
        nd.op = PGPU_F_NOT;
        nodes.push_back(nd);
        emit(o.kids[0], nodes, pool, id_at);
        return;
    }
  }
};

// Descriptor copy whose segment plans carry the filter programs planned from `expr`.
struct PlannedDesc {
  pgpu_query_desc q;
  std::vector<pgpu_segment_plan> plans;
  std::vector<std::vector<pgpu_filter_node>> nodes;
  std::vector<std::vector<int32_t>> pools;
};

int plan_expr(const pgpu_query_desc* q, const pgpu_expr_node* expr, int32_t num_nodes, PlannedDesc& out) {
  if (!q || (!expr && num_nodes > 0) || num_nodes < 0) return fail(PGPU_E_INVALID, "null argument");
  out.q = *q;
  out.plans.assign(q->segments, q->segments + q->num_segments);
  out.nodes.resize(q->num_segments);
  out.pools.resize(q->num_segments);
  for (int s = 0; s < q->num_segments; ++s) {
    pgpu_segment_plan& sp = out.plans[s];
    sp.filter = nullptr;
    sp.num_filter_nodes = 0;
    if (num_nodes == 0) continue;
    if (!sp.segment || !sp.column_map) return fail(PGPU_E_INVALID, "segment %d plan", s);
    ExprPlanner pl{q, &sp, sp.segment, expr, num_nodes};
    int next = 0;
    PlanNode root = pl.build(0, &next);
    if (pl.err) return pl.err;
    if (next != num_nodes) return fail(PGPU_E_INVALID, "filter expression has %d trailing nodes", num_nodes - next);
    if (root.kind == 1) continue;  // match all: no program
    std::vector<std::pair<int, int>> id_at;
    pl.emit(root, out.nodes[s], out.pools[s], id_at);
    for (const auto& ia : id_at) out.nodes[s][ia.first].ids = out.pools[s].data() + ia.second;
    sp.filter = out.nodes[s].data();
    sp.num_filter_nodes = (int32_t)out.nodes[s].size();
  }
  out.q.segments = out.plans.data();
  return PGPU_OK;
}

}  // namespace

extern "C" {

static int submit_impl(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_topk* order, pgpu_query** out_query) {
  if (!ctx || !q || !out_query) return fail(PGPU_E_INVALID, "null argument");
  const double t0 = HostTiming::us();
  pgpu_table_layout L;
  int rc = pgpu_table_layout_of(q, &L);
  if (rc) return rc;
  host_timing().add(1, t0, HostTiming::us());
  HIP_TRY(hipSetDevice(ctx->device));
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->qstream) HIP_TRY(hipStreamCreateWithFlags(&ctx->qstream, hipStreamNonBlocking));
  }
  int err = 0;
  Workspace* tws = acquire_ws(ctx, &err);  // owns the partial table until pgpu_query_collect
  if (!tws) return err;
  const uint64_t bytes = pgpu_table_bytes(&L);
  hipError_t e = tws->table.ensure(bytes, ctx->mpool, ctx->qstream);
  if (e != hipSuccess) {
    release_ws(ctx, tws);
    return fail(PGPU_E_HIP, "table allocation: %s", hipGetErrorString(e));
  }
  // small tables (aggregation only, or up to a few hundred thousand keys) are exported whole into pinned host
  // memory right behind the kernel and compacted on the host: pgpu_query_collect then synchronises once
  const bool small = bytes <= (8u << 20);
  void* h_table_dev = nullptr;
  if (small) {
    e = tws->h_table.ensure(bytes);
    if (e == hipSuccess) e = tws->h_table.device_ptr(&h_table_dev);
    if (e != hipSuccess) {
      release_ws(ctx, tws);
      return fail(PGPU_E_HIP, "host table buffer: %s", hipGetErrorString(e));
    }
  }
  pgpu_query* qq = nullptr;
  // big tables are compacted right behind the kernels on the query stream: the compaction of query i must not
  // wait in collect() behind query i+1's kernel, which holds every CU (the table stays intact, so a collect with
  // another order still selects from it)
  const bool ordered = order && order->k > 0 && L.num_keys > order->k;
  rc = launch_impl(ctx, q, ctx->qstream, tws->table.p, tws->table.n, (int64_t*)h_table_dev, &qq, !small,
                   ordered ? order : nullptr);
  if (rc) {
    release_ws(ctx, tws);
    return rc;
  }
  qq->tws = tws;
  qq->layout = L;
  qq->small = small;
  qq->eager_ordered = ordered;
  *out_query = qq;
  return PGPU_OK;
}

int pgpu_query_submit(pgpu_context* ctx, const pgpu_query_desc* q, pgpu_query** out_query) {
  return submit_impl(ctx, q, nullptr, out_query);
}

int pgpu_query_submit_ordered(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_expr_node* expr,
                              int32_t num_nodes, const pgpu_topk* order, pgpu_query** out_query) {
  if (!ctx || !q || !out_query) return fail(PGPU_E_INVALID, "null argument");
  if (!expr) return submit_impl(ctx, q, order, out_query);
  const double t0 = HostTiming::us();
  PlannedDesc pd;
  int rc = plan_expr(q, expr, num_nodes, pd);
  if (rc) return rc;
  host_timing().add(0, t0, HostTiming::us());
  rc = submit_impl(ctx, &pd.q, order, out_query);  // the descriptor is copied by the submit
  host_timing().add(5, t0, HostTiming::us());
  host_timing().done();
  return rc;
}

int pgpu_query_collect(pgpu_query* qq, int64_t* out_keys, int64_t* out_cells, uint64_t capacity,
                       uint64_t* out_num_groups, pgpu_query_stats* out_stats) {
  return pgpu_query_collect_topk(qq, nullptr, out_keys, out_cells, capacity, out_num_groups, out_stats);
}

int pgpu_query_collect_topk(pgpu_query* qq, const pgpu_topk* order, int64_t* out_keys, int64_t* out_cells,
                            uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats) {
  if (!qq || !qq->tws || !out_num_groups) return fail(PGPU_E_INVALID, "query was not submitted");
  int rc = pgpu_query_wait(qq, out_stats);
  const pgpu_table_layout& L = qq->layout;
  const bool trim = order && order->k > 0 && L.num_keys > order->k;
  if (rc == PGPU_OK && qq->eager && trim == qq->eager_ordered) {
    // compacted on the device behind the kernels (enqueue_compact): only the rows cross PCIe, on the copy engine
    const uint64_t n = (uint64_t)*(const int64_t*)qq->ws->h_total.p;
    *out_num_groups = n;
    if (n > capacity) {
      rc = fail(PGPU_E_INVALID, "%llu non-empty groups exceed capacity %llu", (unsigned long long)n,
                (unsigned long long)capacity);
    } else if (n > 0) {
      const int okw = L.key_kind == PGPU_KEYS_HASH && L.key_words == 2 ? 2 : 1;
      hipStream_t cs = qq->ws->stream;
      hipError_t e = hipMemcpyAsync(out_keys, qq->ws->cmp_keys.p, 8 * n * okw, hipMemcpyDeviceToHost, cs);
      if (e == hipSuccess)
        e = hipMemcpyAsync(out_cells, qq->ws->cmp_cells.p, 8 * n * L.num_sections, hipMemcpyDeviceToHost, cs);
      if (e == hipSuccess) e = hipStreamSynchronize(cs);
      if (e != hipSuccess) rc = fail(PGPU_E_HIP, "result copy: %s", hipGetErrorString(e));
    }
  } else if (rc == PGPU_OK && trim) {
    // the ORDER BY ... LIMIT trim runs on the device copy of the table (small tables too: the host copy is only
    // a shortcut for plain compaction)
    rc = compact_into(qq->ctx, qq->ws, &L, qq->tws->table.p, qq->ws->stream, out_keys, out_cells, capacity,
                      out_num_groups, order);
  } else if (rc == PGPU_OK && qq->small) {
    const int64_t* t = (const int64_t*)qq->tws->h_table.p;
    const uint64_t G = L.num_keys;
    const int nsec = L.num_sections;
    const bool hash = L.key_kind == PGPU_KEYS_HASH;
    const int okw = hash && L.key_words == 2 ? 2 : 1;
    const int64_t* w0 = t + (size_t)nsec * G;
    uint64_t n = 0;
    for (uint64_t k = 0; k < G; ++k) {
      if (t[k] <= 0) continue;
      if (n < capacity) {
        if (!hash) {
          out_keys[n] = (int64_t)k;
        } else if (okw == 1) {
          out_keys[n] = w0[k];
        } else {  // two-level key: (interned word-0 slot << 32 | word 1)
          const uint64_t c = (uint64_t)w0[k];
          out_keys[2 * n] = w0[G + (c >> 32)];
          out_keys[2 * n + 1] = (int64_t)(c & 0xFFFFFFFFull);
        }
        for (int sc = 0; sc < nsec; ++sc) out_cells[n * nsec + sc] = t[(size_t)sc * G + k];
      }
      ++n;
    }
    *out_num_groups = n;
    if (n > capacity)
      rc = fail(PGPU_E_INVALID, "%llu non-empty groups exceed capacity %llu", (unsigned long long)n,
                (unsigned long long)capacity);
  } else if (rc == PGPU_OK) {
    // the table is complete (waited above): compact it on the query's own workspace stream
    rc = compact_into(qq->ctx, qq->ws, &L, qq->tws->table.p, qq->ws->stream, out_keys, out_cells, capacity,
                      out_num_groups);
  }
  pgpu_query_release(qq);
  return rc;
}

int pgpu_query_submit_expr(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_expr_node* expr,
                           int32_t num_nodes, pgpu_query** out_query) {
  if (!ctx || !q || !out_query) return fail(PGPU_E_INVALID, "null argument");
  PlannedDesc pd;
  const int rc = plan_expr(q, expr, num_nodes, pd);
  if (rc) return rc;
  return pgpu_query_submit(ctx, &pd.q, out_query);  // the descriptor is copied by the submit
}

int pgpu_query_launch_expr(pgpu_context* ctx, const pgpu_query_desc* q, const pgpu_expr_node* expr,
                           int32_t num_nodes, void* stream, void* dev_table, uint64_t table_bytes,
                           pgpu_query** out_query) {
  if (!ctx || !q || !out_query) return fail(PGPU_E_INVALID, "null argument");
  PlannedDesc pd;
  const int rc = plan_expr(q, expr, num_nodes, pd);
  if (rc) return rc;
  return pgpu_query_launch(ctx, &pd.q, stream, dev_table, table_bytes, out_query);
}

int pgpu_query_execute(pgpu_context* ctx, const pgpu_query_desc* q, int64_t* out_keys, int64_t* out_cells,
                       uint64_t capacity, uint64_t* out_num_groups, pgpu_query_stats* out_stats) {
  if (!ctx || !q || !out_num_groups) return fail(PGPU_E_INVALID, "null argument");
  pgpu_query* qq = nullptr;
  int rc = pgpu_query_submit(ctx, q, &qq);
  if (rc) return rc;
  return pgpu_query_collect(qq, out_keys, out_cells, capacity, out_num_groups, out_stats);
}

}  // extern "C"
