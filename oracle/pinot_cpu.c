/*
 * pinot_cpu.c — C restatement of Pinot's CPU query operators for the bench workloads (TEST INFRASTRUCTURE:
 * the cpu_baseline leg of bench.py and oracle cross-checks; never linked by the product path).
 *
 * Per segment, exactly the reference's execution structure:
 *   - filter: AND of scan leaves -> AndDocIdIterator leap-frogging SVScanDocIdIterators
 *       (core/operator/docidsets/AndDocIdSet.java:60-146 with only scan children -> AndDocIdIterator,
 *        core/operator/dociditerators/AndDocIdIterator.java:40-73,
 *        core/operator/dociditerators/SVScanDocIdIterator.java:57-70: one getDictId + predicate per doc)
 *   - DocIdSetOperator: blocks of up to 10,000 matching doc ids (core/operator/DocIdSetOperator.java:58-83,
 *        core/plan/DocIdSetPlanNode.java:29)
 *   - projection: dict ids per block via FixedBitSVForwardIndexReaderV2.readDictIds (bulk when contiguous,
 *        seglocal/segment/index/readers/forward/FixedBitSVForwardIndexReaderV2.java:62-96), dictionary values
 *   - group key = mixed-radix dict ids (DictionaryBasedGroupKeyGenerator ArrayBased / IntMap raw key,
 *        core/query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:275-322) into a dense holder
 *   - SUM in double, COUNT, MIN/MAX in double (core/query/aggregation/function/{Sum,Count,Min,Max}AggregationFunction.java)
 *   - segment-level task parallelism: one task per segment, min(#segments, threads) workers
 *        (core/operator/combine/CombineOperatorUtils.java:37-50), per-segment results merged afterwards.
 * Predicates arrive as a truth bitset over the dictionary (the oracle evaluates the literal against every
 * dictionary value), which covers the RANGE / EQ / IN / NOT IN evaluators.
 *
 * Filter trees with index leaves (pc_query.num_nodes > 0) follow the doc-id set algebra of
 *   core/operator/docidsets/AndDocIdSet.java:60-146 (index-based children merged into one bitmap, scan children
 *   applied with ScanBasedDocIdIterator.applyAnd: one getDictId per doc of the merged bitmap),
 *   core/operator/docidsets/OrDocIdSet.java:58-120 (index-based children ORed), NotDocIdSet (complement),
 *   core/operator/filter/BitmapBasedFilterOperator.java:66-101 (OR of the matching ids' Roaring bitmaps, flipped
 *   over [0, numDocs) for exclusive predicates) and SortedIndexBasedFilterOperator (doc ranges of the matching ids),
 * with the Roaring bitmaps decoded from their portable serialization into flat 64-bit-word doc-id sets: the same
 * doc ids and scan counts as the reference, on a representation at least as fast as RoaringBitmap's for these
 * densities.  Matching docs then go through the same 10,000-doc blocks as the scan path.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PC_BLOCK 10000
#define PC_EOF (-1)

typedef struct {
  const uint8_t* fwd;      /* fixed-bit forward index, big-endian MSB-first (NULL for a sorted column) */
  int32_t bits;
  int32_t card;
  const double* dict;      /* dictionary values as double (getDoubleValuesSV) */
  const uint8_t* inv;      /* BitmapInvertedIndexWriter file: (card + 1) big-endian offsets, Roaring blobs; or NULL */
  const uint8_t* sorted;   /* sorted index: (start, end) inclusive big-endian int32 pairs per dict id; or NULL */
} pc_column;

enum { PC_SCAN = 0, PC_BITMAP = 1, PC_SORTED = 2, PC_AND = 3, PC_OR = 4, PC_NOT = 5, PC_EMPTY = 6 };

typedef struct {
  int32_t kind;
  int32_t col;
  const uint8_t* truth;     /* PC_SCAN: bitset over dict ids */
  const int32_t* ids;       /* PC_BITMAP: the ids whose bitmaps are ORed (the NON-matching ids when exclusive);
                               PC_SORTED: the matching ids */
  int32_t num_ids;
  int32_t exclusive;
  int32_t first_child;      /* children: child_idx[first_child .. first_child + num_children) */
  int32_t num_children;
} pc_node;

typedef struct {
  int32_t num_docs;
  int32_t num_columns;
  const pc_column* cols;
} pc_segment;

typedef struct {
  int32_t num_leaves;          /* AND of scan leaves, in evaluation order */
  const int32_t* leaf_col;
  const uint8_t* const* leaf_truth; /* per leaf: bitset over dict ids */
  int32_t num_aggs;
  const int32_t* agg_fn;       /* 0 COUNT 1 SUM 2 MIN 3 MAX */
  const int32_t* agg_col;
  int32_t num_group_cols;
  const int32_t* group_col;
  int64_t num_keys;            /* product of group column cardinalities (1 for aggregation only) */
  int32_t num_nodes;           /* > 0: filter tree (nodes[root]) instead of the AND-of-scan leaves */
  const pc_node* nodes;
  const int32_t* child_idx;
  int32_t root;
} pc_query;

/* FixedBitIntReader.readUnchecked: 8-byte big-endian window at the value's byte offset (buffers are padded). */
static inline uint32_t read_id(const uint8_t* buf, int32_t bits, int64_t doc) {
  const uint64_t bit = (uint64_t)doc * (uint64_t)bits;
  const uint8_t* p = buf + (bit >> 3);
  uint64_t w = ((uint64_t)p[0] << 56) | ((uint64_t)p[1] << 48) | ((uint64_t)p[2] << 40) | ((uint64_t)p[3] << 32) |
               ((uint64_t)p[4] << 24) | ((uint64_t)p[5] << 16) | ((uint64_t)p[6] << 8) | (uint64_t)p[7];
  const unsigned shift = 64u - (unsigned)(bit & 7) - (unsigned)bits;
  return (uint32_t)((w >> shift) & (bits == 32 ? 0xFFFFFFFFull : ((1ull << bits) - 1)));
}

typedef struct {
  const pc_column* col;
  const uint8_t* truth;
  int32_t next_doc;
  int32_t num_docs;
  int64_t scanned;
} scan_iter;

/* SVScanDocIdIterator.advance(target): scan forward from target until the predicate matches. */
static int32_t scan_advance(scan_iter* it, int32_t target) {
  it->next_doc = target;
  while (it->next_doc < it->num_docs) {
    const int32_t d = it->next_doc++;
    it->scanned++;
    const uint32_t id = read_id(it->col->fwd, it->col->bits, d);
    if ((it->truth[id >> 3] >> (id & 7)) & 1) return d;
  }
  return PC_EOF;
}

/* AndDocIdIterator.next(). */
static int32_t and_next(scan_iter* its, int n, int32_t* next_doc) {
  int32_t max_doc = *next_doc;
  int max_idx = -1;
  int i = 0;
  while (i < n) {
    if (i == max_idx) { ++i; continue; }
    const int32_t d = scan_advance(&its[i], max_doc);
    if (d == PC_EOF) return PC_EOF;
    if (d == max_doc) {
      ++i;
    } else {
      max_doc = d;
      max_idx = i;
      i = 0;
    }
  }
  *next_doc = max_doc + 1;
  return max_doc;
}

typedef struct {
  double* sums;     /* [num_aggs][num_keys] */
  int64_t* counts;  /* [num_keys] */
  int64_t matched;
  int64_t scanned;
  char pad[96];     /* one partial per 128-B line pair: workers update theirs per block */
} pc_partial;

typedef struct {
  int32_t* docs;
  int64_t* keys;
  uint32_t* ids;
} pc_block;

/* One DocIdSetOperator block through the projection and the aggregation / group-by. */
static void process_block(const pc_segment* seg, const pc_query* q, pc_block* b, int cnt, pc_partial* out) {
  const int32_t* docs = b->docs;
  int64_t* keys = b->keys;
  uint32_t* ids = b->ids;
  out->matched += cnt;
  for (int i = 0; i < cnt; ++i) keys[i] = 0;
  int64_t mult = 1;
  for (int g = 0; g < q->num_group_cols; ++g) {
    const pc_column* c = &seg->cols[q->group_col[g]];
    for (int i = 0; i < cnt; ++i) keys[i] += (int64_t)read_id(c->fwd, c->bits, docs[i]) * mult;
    mult *= c->card;
  }
  for (int i = 0; i < cnt; ++i) out->counts[keys[i]]++;
  /* aggregations (values fetched per block, as the projection does) */
  for (int a = 0; a < q->num_aggs; ++a) {
    if (q->agg_fn[a] == 0) continue;
    const pc_column* c = &seg->cols[q->agg_col[a]];
    for (int i = 0; i < cnt; ++i) ids[i] = read_id(c->fwd, c->bits, docs[i]);
    double* s = out->sums + (int64_t)a * q->num_keys;
    for (int i = 0; i < cnt; ++i) {
      const double v = c->dict[ids[i]];
      double* cell = &s[keys[i]];
      if (q->agg_fn[a] == 1) *cell += v;
      else if (q->agg_fn[a] == 2) { if (v < *cell) *cell = v; }
      else { if (v > *cell) *cell = v; }
    }
  }
}

/* ---- doc-id sets as flat bitmaps (the filter-tree path) ---------------------------------------------------- */
static inline uint32_t rd_le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static inline uint32_t rd_le32(const uint8_t* p) { return rd_le16(p) | (rd_le16(p + 2) << 16); }
static inline int32_t rd_be32(const uint8_t* p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
}

/* set docs [lo, hi] (inclusive), clipped to the set's nw words */
static void set_range(uint64_t* w, int64_t nw, int64_t lo, int64_t hi) {
  if (hi >= nw * 64) hi = nw * 64 - 1;
  if (lo > hi) return;
  const int64_t a = lo >> 6, b = hi >> 6;
  const uint64_t ma = ~0ull << (lo & 63), mb = ~0ull >> (63 - (hi & 63));
  if (a == b) { w[a] |= ma & mb; return; }
  w[a] |= ma;
  for (int64_t i = a + 1; i < b; ++i) w[i] = ~0ull;
  w[b] |= mb;
}

/* OR one portable-format Roaring bitmap (cookie 12346 / 12347; array, bitmap and run containers) into w. */
static int roaring_or(const uint8_t* b, uint64_t* w, int64_t nw) {
  const uint32_t cookie = rd_le32(b);
  const uint8_t* runflags = NULL;
  const uint8_t* p;
  int32_t size;
  if ((cookie & 0xFFFF) == 12347) {
    size = (int32_t)(cookie >> 16) + 1;
    runflags = b + 4;
    p = b + 4 + (size + 7) / 8;
  } else if (cookie == 12346) {
    size = (int32_t)rd_le32(b + 4);
    p = b + 8;
  } else {
    return -1;
  }
  const uint8_t* kc = p;
  p += 4 * size;
  if (!runflags || size >= 4) p += 4 * size; /* offset header */
  for (int32_t i = 0; i < size; ++i) {
    const int64_t base = (int64_t)rd_le16(kc + 4 * i) << 16;
    const int32_t card = (int32_t)rd_le16(kc + 4 * i + 2) + 1;
    if (runflags && ((runflags[i >> 3] >> (i & 7)) & 1)) {
      const int32_t nr = (int32_t)rd_le16(p);
      p += 2;
      for (int32_t r = 0; r < nr; ++r)
        set_range(w, nw, base + rd_le16(p + 4 * r), base + rd_le16(p + 4 * r) + rd_le16(p + 4 * r + 2));
      p += 4 * nr;
    } else if (card > 4096) {
      const int64_t w0 = base >> 6;
      for (int32_t j = 0; j < 1024 && w0 + j < nw; ++j) {
        uint64_t v = 0;
        for (int k = 7; k >= 0; --k) v = (v << 8) | p[8 * j + k];
        w[w0 + j] |= v;
      }
      p += 8192;
    } else {
      for (int32_t j = 0; j < card; ++j) {
        const int64_t d = base + rd_le16(p + 2 * j);
        if ((d >> 6) < nw) w[d >> 6] |= 1ull << (d & 63);
      }
      p += 2 * card;
    }
  }
  return 0;
}

static void complement(uint64_t* w, int64_t nw, int32_t n) {
  for (int64_t i = 0; i < nw; ++i) w[i] = ~w[i];
  if (n & 63) w[nw - 1] &= (1ull << (n & 63)) - 1;
}

static inline int is_index_kind(int k) { return k != PC_SCAN; }

/* Per-worker free list of doc-id sets, reused across segments and across pc_execute calls (fresh multi-MB
 * callocs per node are mmap / munmap pairs whose page faults and TLB shootdowns serialise the workers; a
 * long-running JVM allocates its Roaring containers from an already-faulted heap).  pc_release_pools frees them. */
typedef struct {
  uint64_t* bufs[64];
  int64_t cap[64];
  int n;
} set_pool;

static uint64_t* get_set(set_pool* pl, int64_t nw) {
  for (int i = pl->n - 1; i >= 0; --i) {
    if (pl->cap[i] >= nw) {
      uint64_t* b = pl->bufs[i];
      pl->bufs[i] = pl->bufs[pl->n - 1];
      pl->cap[i] = pl->cap[pl->n - 1];
      pl->n--;
      memset(b, 0, (size_t)(nw + 1) * 8);
      return b;
    }
  }
  return (uint64_t*)calloc((size_t)nw + 1, 8);
}

static void put_set(set_pool* pl, uint64_t* b, int64_t nw) {
  if (pl->n < 64) {
    pl->bufs[pl->n] = b;
    pl->cap[pl->n] = nw;
    pl->n++;
  } else {
    free(b);
  }
}

static void drain_pool(set_pool* pl) {
  for (int i = 0; i < pl->n; ++i) free(pl->bufs[i]);
  pl->n = 0;
}

/* Evaluate node `ni` into a fresh calloc'ed doc-id set; scan entries counted into *scanned. */
static uint64_t* eval_node(const pc_segment* seg, const pc_query* q, int32_t ni, int64_t* scanned, set_pool* pl) {
  const pc_node* nd = &q->nodes[ni];
  const int32_t n = seg->num_docs;
  const int64_t nw = ((int64_t)n + 63) >> 6;
  uint64_t* w = NULL;
  switch (nd->kind) {
    case PC_EMPTY:
      return get_set(pl, nw);
    case PC_SCAN: {
      /* SVScanDocIdIterator over every doc (an OR / NOT child, or an AND of scans only) */
      const pc_column* c = &seg->cols[nd->col];
      w = get_set(pl, nw);
      for (int32_t d = 0; d < n; ++d) {
        const uint32_t id = read_id(c->fwd, c->bits, d);
        if ((nd->truth[id >> 3] >> (id & 7)) & 1) w[d >> 6] |= 1ull << (d & 63);
      }
      *scanned += n;
      return w;
    }
    case PC_BITMAP: {
      const pc_column* c = &seg->cols[nd->col];
      w = get_set(pl, nw);
      const int32_t first = rd_be32(c->inv);
      const uint8_t* blobs = c->inv + 4 * ((int64_t)c->card + 1);  /* BitmapInvertedIndexReader: offsets - first */
      for (int32_t k = 0; k < nd->num_ids; ++k) roaring_or(blobs + (rd_be32(c->inv + 4 * (int64_t)nd->ids[k]) - first), w, nw);
      if (nd->exclusive) complement(w, nw, n);
      return w;
    }
    case PC_SORTED: {
      const pc_column* c = &seg->cols[nd->col];
      w = get_set(pl, nw);
      for (int32_t k = 0; k < nd->num_ids; ++k) {
        const uint8_t* pr = c->sorted + 8 * (int64_t)nd->ids[k];
        set_range(w, nw, rd_be32(pr), rd_be32(pr + 4));
      }
      return w;
    }
    case PC_NOT:
      w = eval_node(seg, q, q->child_idx[nd->first_child], scanned, pl);
      complement(w, nw, n);
      return w;
    case PC_OR:
      for (int32_t k = 0; k < nd->num_children; ++k) {
        uint64_t* x = eval_node(seg, q, q->child_idx[nd->first_child + k], scanned, pl);
        if (!w) { w = x; continue; }
        for (int64_t i = 0; i < nw; ++i) w[i] |= x[i];
        put_set(pl, x, nw);
      }
      return w;
    case PC_AND: {
      /* index-based (and compound) children merged first, in order; then every scan child applied to the
       * merged set (applyAnd: one dict-id read per doc still in the set) */
      for (int32_t k = 0; k < nd->num_children; ++k) {
        const int32_t ci = q->child_idx[nd->first_child + k];
        if (!is_index_kind(q->nodes[ci].kind)) continue;
        uint64_t* x = eval_node(seg, q, ci, scanned, pl);
        if (!w) { w = x; continue; }
        for (int64_t i = 0; i < nw; ++i) w[i] &= x[i];
        put_set(pl, x, nw);
      }
      for (int32_t k = 0; k < nd->num_children; ++k) {
        const int32_t ci = q->child_idx[nd->first_child + k];
        const pc_node* ch = &q->nodes[ci];
        if (is_index_kind(ch->kind)) continue;
        if (!w) { w = eval_node(seg, q, ci, scanned, pl); continue; }
        const pc_column* c = &seg->cols[ch->col];
        for (int64_t i = 0; i < nw; ++i) {
          uint64_t m = w[i], keep = m;
          while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t id = read_id(c->fwd, c->bits, i * 64 + b);
            ++*scanned;
            if (!((ch->truth[id >> 3] >> (id & 7)) & 1)) keep &= ~(1ull << b);
          }
          w[i] = keep;
        }
      }
      return w;
    }
    default:
      return get_set(pl, nw);
  }
}

static void execute_segment(const pc_segment* seg, const pc_query* q, pc_partial* out, set_pool* pl) {
  const int32_t n = seg->num_docs;
  pc_block blk;
  blk.docs = (int32_t*)malloc(sizeof(int32_t) * PC_BLOCK);
  blk.keys = (int64_t*)malloc(sizeof(int64_t) * PC_BLOCK);
  blk.ids = (uint32_t*)malloc(sizeof(uint32_t) * PC_BLOCK);
  if (q->num_nodes > 0) {
    const int64_t nw = ((int64_t)n + 63) >> 6;
    int64_t scanned = 0;
    uint64_t* w = eval_node(seg, q, q->root, &scanned, pl);
    out->scanned += scanned;
    int cnt = 0;
    for (int64_t i = 0; i < nw; ++i) {
      uint64_t m = w[i];
      while (m) {
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        blk.docs[cnt++] = (int32_t)(i * 64 + b);
        if (cnt == PC_BLOCK) {
          process_block(seg, q, &blk, cnt, out);
          cnt = 0;
        }
      }
    }
    if (cnt) process_block(seg, q, &blk, cnt, out);
    put_set(pl, w, nw);
  } else {
    scan_iter its[16];
    const int nl = q->num_leaves;
    for (int l = 0; l < nl; ++l) {
      its[l].col = &seg->cols[q->leaf_col[l]];
      its[l].truth = q->leaf_truth[l];
      its[l].next_doc = 0;
      its[l].num_docs = n;
      its[l].scanned = 0;
    }
    int32_t and_next_doc = 0, all_next = 0;
    int eof = 0;
    while (!eof) {
      /* DocIdSetOperator.getNextBlock: up to 10,000 doc ids; the iterator is not called again after EOF */
      int cnt = 0;
      while (cnt < PC_BLOCK) {
        int32_t d;
        if (nl == 0) d = all_next < n ? all_next++ : PC_EOF;
        else if (nl == 1) d = scan_advance(&its[0], its[0].next_doc);
        else d = and_next(its, nl, &and_next_doc);
        if (d == PC_EOF) {
          eof = 1;
          break;
        }
        blk.docs[cnt++] = d;
      }
      if (cnt == 0) break;
      process_block(seg, q, &blk, cnt, out);
    }
    for (int l = 0; l < nl; ++l) out->scanned += its[l].scanned;
  }
  free(blk.docs);
  free(blk.keys);
  free(blk.ids);
}

typedef struct {
  const pc_segment* segs;
  int num_segs;
  const pc_query* q;
  pc_partial* parts;
  int next;
} pool_t;

/* A persistent worker pool, as the server's query executor keeps one (freshly created threads per query start a
 * scheduler tick apart and share CPUs until the load balancer moves them, which serialises short segments).
 * Worker i keeps its own doc-id-set free list across queries; pc_release_pools frees the lists. */
#define PC_MAX_WORKERS 256
static set_pool g_pools[PC_MAX_WORKERS];
static pthread_t g_threads[PC_MAX_WORKERS];
static int g_num_threads = 0;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cv_work = PTHREAD_COND_INITIALIZER;
static pthread_cond_t g_cv_done = PTHREAD_COND_INITIALIZER;
static pool_t* g_job = NULL;
static uint64_t g_gen = 0;
static int g_job_threads = 0;
static int g_active = 0;

/* Pin worker `id` to the id-th CPU this process may use: without it, workers woken together can queue on the
 * waker's CPU for many scheduler ticks (seen on small VMs), which serialises segments of a few ms. */
static void pin_worker(int id) {
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  const int n = CPU_COUNT(&allowed);
  if (n <= 1) return;
  int want = id % n, seen = 0;
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &allowed)) continue;
    if (seen++ == want) {
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(c, &one);
      pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
      return;
    }
  }
}

static void* worker(void* arg) {
  const int id = (int)(intptr_t)arg;
  uint64_t seen = 0;
  pin_worker(id);
  for (;;) {
    pthread_mutex_lock(&g_mu);
    while (g_gen == seen || id >= g_job_threads) {
      if (g_gen != seen) seen = g_gen;  /* a job this worker sits out */
      pthread_cond_wait(&g_cv_work, &g_mu);
    }
    seen = g_gen;
    pool_t* job = g_job;
    pthread_mutex_unlock(&g_mu);
    for (;;) {
      const int s = __atomic_fetch_add(&job->next, 1, __ATOMIC_RELAXED);
      if (s >= job->num_segs) break;
      execute_segment(&job->segs[s], job->q, &job->parts[s], &g_pools[id]);
    }
    pthread_mutex_lock(&g_mu);
    if (--g_active == 0) pthread_cond_signal(&g_cv_done);
    pthread_mutex_unlock(&g_mu);
  }
  return NULL;
}

void pc_release_pools(void) {
  pthread_mutex_lock(&g_mu);
  for (int i = 0; i < PC_MAX_WORKERS; ++i) drain_pool(&g_pools[i]);
  pthread_mutex_unlock(&g_mu);
}

static void init_partial(const pc_query* q, pc_partial* p) {
  /* cache-line aligned and padded: the partials of segments run by different workers must not share lines */
  const size_t sb = (sizeof(double) * (size_t)q->num_aggs * (size_t)q->num_keys + 8 + 127) & ~(size_t)127;
  const size_t cb = (sizeof(int64_t) * ((size_t)q->num_keys + 1) + 127) & ~(size_t)127;
  p->sums = (double*)aligned_alloc(128, sb);
  p->counts = (int64_t*)aligned_alloc(128, cb);
  memset(p->counts, 0, cb);
  for (int a = 0; a < q->num_aggs; ++a) {
    const double init = q->agg_fn[a] == 2 ? __builtin_inf() : (q->agg_fn[a] == 3 ? -__builtin_inf() : 0.0);
    for (int64_t k = 0; k < q->num_keys; ++k) p->sums[(int64_t)a * q->num_keys + k] = init;
  }
  p->matched = 0;
  p->scanned = 0;
}

/* Run the query over all segments with `threads` workers; merge into out_sums[num_aggs][num_keys] and
 * out_counts[num_keys] (SUM: +, MIN/MAX: min/max).  Returns matched docs; *out_scanned = entries scanned. */
int64_t pc_execute(const pc_segment* segs, int32_t num_segs, const pc_query* q, int32_t threads, double* out_sums,
                   int64_t* out_counts, int64_t* out_scanned) {
  pool_t pool;
  pool.segs = segs;
  pool.num_segs = num_segs;
  pool.q = q;
  pool.next = 0;
  pool.parts = (pc_partial*)calloc((size_t)num_segs, sizeof(pc_partial));
  for (int s = 0; s < num_segs; ++s) init_partial(q, &pool.parts[s]);
  if (threads < 1) threads = 1;
  if (threads > num_segs) threads = num_segs;
  if (threads > PC_MAX_WORKERS) threads = PC_MAX_WORKERS;
  pthread_mutex_lock(&g_mu);
  while (g_num_threads < threads) {
    if (pthread_create(&g_threads[g_num_threads], NULL, worker, (void*)(intptr_t)g_num_threads) != 0) break;
    g_num_threads++;
  }
  if (threads > g_num_threads) threads = g_num_threads;
  if (threads == 0) { /* no worker could be started: run on the caller */
    pthread_mutex_unlock(&g_mu);
    for (int s = 0; s < num_segs; ++s) execute_segment(&segs[s], q, &pool.parts[s], &g_pools[0]);
    pthread_mutex_lock(&g_mu);
  }
  g_job = &pool;
  g_job_threads = threads;
  g_active = threads;
  g_gen++;
  pthread_cond_broadcast(&g_cv_work);
  while (g_active > 0) pthread_cond_wait(&g_cv_done, &g_mu);
  g_job = NULL;
  pthread_mutex_unlock(&g_mu);
  int64_t matched = 0, scanned = 0;
  pc_partial acc;
  init_partial(q, &acc);
  for (int s = 0; s < num_segs; ++s) {
    pc_partial* p = &pool.parts[s];
    matched += p->matched;
    scanned += p->scanned;
    for (int64_t k = 0; k < q->num_keys; ++k) acc.counts[k] += p->counts[k];
    for (int a = 0; a < q->num_aggs; ++a) {
      for (int64_t k = 0; k < q->num_keys; ++k) {
        double* d = &acc.sums[(int64_t)a * q->num_keys + k];
        const double v = p->sums[(int64_t)a * q->num_keys + k];
        if (q->agg_fn[a] == 2) { if (v < *d) *d = v; }
        else if (q->agg_fn[a] == 3) { if (v > *d) *d = v; }
        else *d += v;
      }
    }
    free(p->sums);
    free(p->counts);
  }
  memcpy(out_sums, acc.sums, sizeof(double) * (size_t)q->num_aggs * (size_t)q->num_keys);
  memcpy(out_counts, acc.counts, sizeof(int64_t) * (size_t)q->num_keys);
  free(acc.sums);
  free(acc.counts);
  free(pool.parts);
  if (out_scanned) *out_scanned = scanned;
  return matched;
}

/* ---- synthetic segment generator (restates pinot_amd/csrc/synth.hip's uniform synth_id) ---------------------- */
static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* FixedBitSVForwardIndexWriter layout of ids(doc) = ((splitmix64(seed ^ doc*K) >> 32) * card) >> 32, or with a
 * CDF table (Zipf keys, pinot_amd.synth.zipf_cdf) the first k with cdf[k] > u(doc), as synth.hip's synth_id. */
void pc_synth_fixed_bit(uint8_t* out, int64_t num_docs, int32_t bits, uint32_t card, uint64_t seed,
                        const uint32_t* cdf) {
  uint64_t acc = 0;  /* pending bits, MSB-aligned count `have` */
  int have = 0;
  int64_t pos = 0;
  for (int64_t d = 0; d < num_docs; ++d) {
    const uint32_t u = (uint32_t)(splitmix64(seed ^ ((uint64_t)d * 0xD1B54A32D192ED03ull)) >> 32);
    uint64_t v;
    if (!cdf) {
      v = ((uint64_t)u * card) >> 32;
    } else {
      uint32_t lo = 0, hi = card - 1;
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
      }
      v = lo;
    }
    acc = (acc << bits) | v;
    have += bits;
    while (have >= 8) {
      out[pos++] = (uint8_t)(acc >> (have - 8));
      have -= 8;
    }
    acc &= (have ? ((1ull << have) - 1) : 0);
  }
  if (have) out[pos++] = (uint8_t)(acc << (8 - have));
}
