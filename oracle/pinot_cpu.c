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
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PC_BLOCK 10000
#define PC_EOF (-1)

typedef struct {
  const uint8_t* fwd;      /* fixed-bit forward index, big-endian MSB-first */
  int32_t bits;
  int32_t card;
  const double* dict;      /* dictionary values as double (getDoubleValuesSV) */
} pc_column;

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
} pc_partial;

static void execute_segment(const pc_segment* seg, const pc_query* q, pc_partial* out) {
  const int32_t n = seg->num_docs;
  scan_iter its[16];
  const int nl = q->num_leaves;
  for (int l = 0; l < nl; ++l) {
    its[l].col = &seg->cols[q->leaf_col[l]];
    its[l].truth = q->leaf_truth[l];
    its[l].next_doc = 0;
    its[l].num_docs = n;
    its[l].scanned = 0;
  }
  int32_t* docs = (int32_t*)malloc(sizeof(int32_t) * PC_BLOCK);
  int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * PC_BLOCK);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * PC_BLOCK);
  int32_t and_next_doc = 0, all_next = 0;
  for (;;) {
    /* DocIdSetOperator.getNextBlock: up to 10,000 doc ids */
    int cnt = 0;
    while (cnt < PC_BLOCK) {
      int32_t d;
      if (nl == 0) d = all_next < n ? all_next++ : PC_EOF;
      else if (nl == 1) d = scan_advance(&its[0], its[0].next_doc);
      else d = and_next(its, nl, &and_next_doc);
      if (d == PC_EOF) break;
      docs[cnt++] = d;
    }
    if (cnt == 0) break;
    out->matched += cnt;
    /* group keys */
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
  for (int l = 0; l < nl; ++l) out->scanned += its[l].scanned;
  free(docs);
  free(keys);
  free(ids);
}

typedef struct {
  const pc_segment* segs;
  int num_segs;
  const pc_query* q;
  pc_partial* parts;
  int next;
  pthread_mutex_t mu;
} pool_t;

static void init_partial(const pc_query* q, pc_partial* p) {
  p->sums = (double*)malloc(sizeof(double) * (size_t)q->num_aggs * (size_t)q->num_keys + 8);
  p->counts = (int64_t*)calloc((size_t)q->num_keys + 1, sizeof(int64_t));
  for (int a = 0; a < q->num_aggs; ++a) {
    const double init = q->agg_fn[a] == 2 ? __builtin_inf() : (q->agg_fn[a] == 3 ? -__builtin_inf() : 0.0);
    for (int64_t k = 0; k < q->num_keys; ++k) p->sums[(int64_t)a * q->num_keys + k] = init;
  }
  p->matched = 0;
  p->scanned = 0;
}

static void* worker(void* arg) {
  pool_t* pool = (pool_t*)arg;
  for (;;) {
    pthread_mutex_lock(&pool->mu);
    const int s = pool->next++;
    pthread_mutex_unlock(&pool->mu);
    if (s >= pool->num_segs) break;
    execute_segment(&pool->segs[s], pool->q, &pool->parts[s]);
  }
  return NULL;
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
  pthread_mutex_init(&pool.mu, NULL);
  pool.parts = (pc_partial*)calloc((size_t)num_segs, sizeof(pc_partial));
  for (int s = 0; s < num_segs; ++s) init_partial(q, &pool.parts[s]);
  if (threads < 1) threads = 1;
  if (threads > num_segs) threads = num_segs;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)(threads > 0 ? threads : 1));
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker, &pool);
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  free(th);
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
  pthread_mutex_destroy(&pool.mu);
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

/* FixedBitSVForwardIndexWriter layout of ids(doc) = ((splitmix64(seed ^ doc*K) >> 32) * card) >> 32. */
void pc_synth_fixed_bit(uint8_t* out, int64_t num_docs, int32_t bits, uint32_t card, uint64_t seed) {
  uint64_t acc = 0;  /* pending bits, MSB-aligned count `have` */
  int have = 0;
  int64_t pos = 0;
  for (int64_t d = 0; d < num_docs; ++d) {
    const uint32_t u = (uint32_t)(splitmix64(seed ^ ((uint64_t)d * 0xD1B54A32D192ED03ull)) >> 32);
    const uint64_t v = ((uint64_t)u * card) >> 32;
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
