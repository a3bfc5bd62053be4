// The reference's numEntriesScannedInFilter, restated over per-leaf match bitmaps (PGPU_Q_EXACT_FILTER_STATS).
//
// The GPU evaluates whole tiles, so its own count of evaluated forward-index entries equals the reference's only
// where the reference's iterators touch every doc of a scanned column in order (a lone scan, scans under
// applyAnd, OR / NOT driven by next()).  Where the reference leap-frogs (AndDocIdIterator over scan iterators, an
// OR or NOT advanced by a parent AND), the count depends on where each SVScanDocIdIterator resumes.  This file
// drives the same iterator tree the reference builds, over the leaves' match bitmaps produced by
// leafbits_kernel, and counts the entries every scan iterator reads:
//   SVScanDocIdIterator.next / advance / applyAnd  core/operator/dociditerators/SVScanDocIdIterator.java:57-98
//   AndDocIdSet.iterator (index merge, applyAnd)   core/operator/docidsets/AndDocIdSet.java:60-146
//   OrDocIdSet.iterator                             core/operator/docidsets/OrDocIdSet.java:58-110
//   AndDocIdIterator / OrDocIdIterator / NotDocIdIterator   core/operator/dociditerators/*.java
// (oracle/engine.py holds the same model in Python; both are pinned by the InnerSegment KAT's 84,134.)
#include <cstdint>
#include <memory>
#include <vector>

#include "pgpu_host.h"

namespace {

constexpr int32_t kEOF = INT32_MIN;  // Constants.EOF

// A doc-id set as a bitmap over [0, n).
struct BitSet {
  std::vector<uint64_t> w;
  int32_t n = 0;
  explicit BitSet(int32_t docs = 0) : w(((size_t)docs + 63) / 64, 0), n(docs) {}
  static BitSet from_words32(const uint32_t* src, int32_t docs) {
    BitSet b(docs);
    for (size_t i = 0; i < b.w.size(); ++i) {
      const uint64_t lo = src[2 * i];
      const uint64_t hi = (2 * i + 1) * 32 < (size_t)docs ? src[2 * i + 1] : 0;
      b.w[i] = lo | (hi << 32);
    }
    b.trim();
    return b;
  }
  void trim() {
    if (n % 64 && !w.empty()) w.back() &= (1ull << (n % 64)) - 1;
  }
  bool test(int32_t d) const { return (w[d >> 6] >> (d & 63)) & 1; }
  int32_t next(int32_t from) const {  // first member >= from, or kEOF
    if (from < 0) from = 0;
    if (from >= n) return kEOF;
    size_t i = (size_t)from >> 6;
    uint64_t x = w[i] & (~0ull << (from & 63));
    while (!x) {
      if (++i >= w.size()) return kEOF;
      x = w[i];
    }
    const int32_t d = (int32_t)(i * 64 + __builtin_ctzll(x));
    return d < n ? d : kEOF;
  }
  int64_t count() const {
    int64_t c = 0;
    for (uint64_t x : w) c += __builtin_popcountll(x);
    return c;
  }
};

enum Kind { SCAN, BITMAP, SORTED, OTHER };

struct Iter {
  Kind kind = OTHER;
  virtual ~Iter() = default;
  virtual int32_t next() = 0;
  virtual int32_t advance(int32_t target) = 0;
};

// SVScanDocIdIterator: every doc from the resume position up to (and including) the next match is read.
// MVScanDocIdIterator (MVScanDocIdIterator.java:56-100) is the same walk reading each row's length in entries:
// `off` (row offsets) turns a doc range into its entry count.
struct ScanIter : Iter {
  const BitSet* bits;
  int32_t nxt = 0;
  int64_t* counter;
  const int32_t* off;
  ScanIter(const BitSet* b, int64_t* c, const int32_t* o = nullptr) : bits(b), counter(c), off(o) { kind = SCAN; }
  int64_t entries(int32_t a, int32_t b) const { return off ? (int64_t)off[b] - off[a] : (int64_t)b - a; }
  int32_t next() override {
    if (nxt >= bits->n) return kEOF;
    const int32_t d = bits->next(nxt);
    if (d != kEOF) {
      *counter += entries(nxt, d + 1);
      nxt = d + 1;
      return d;
    }
    *counter += entries(nxt, bits->n);
    nxt = bits->n;
    return kEOF;
  }
  int32_t advance(int32_t t) override {
    nxt = t;
    return next();
  }
  // applyAnd: reads one entry per candidate doc
  void apply_and(BitSet& docs) const {
    if (!off) {
      *counter += docs.count();
    } else {
      for (size_t i = 0; i < docs.w.size(); ++i)
        for (uint64_t m = docs.w[i]; m; m &= m - 1) {
          const int32_t d = (int32_t)(i * 64 + __builtin_ctzll(m));
          *counter += (int64_t)off[d + 1] - off[d];
        }
    }
    for (size_t i = 0; i < docs.w.size(); ++i) docs.w[i] &= bits->w[i];
  }
};

// Bitmap / sorted / match-all / empty / merged iterators: walk a doc-id set, read no forward index.
struct DocsIter : Iter {
  std::shared_ptr<BitSet> docs;
  int32_t pos = 0;
  DocsIter(std::shared_ptr<BitSet> d, Kind k) : docs(std::move(d)) { kind = k; }
  int32_t next() override {
    const int32_t d = docs->next(pos);
    pos = d == kEOF ? docs->n : d + 1;
    return d;
  }
  int32_t advance(int32_t t) override {
    if (t > pos) pos = t;
    return next();
  }
};

// AndDocIdIterator: leap-frog to the first doc every child agrees on.
struct AndIter : Iter {
  std::vector<std::unique_ptr<Iter>> its;
  int32_t nxt = 0;
  int32_t next() override {
    int32_t mx = nxt, mi = -1;
    size_t i = 0;
    while (i < its.size()) {
      if ((int32_t)i == mi) {
        ++i;
        continue;
      }
      const int32_t d = its[i]->advance(mx);
      if (d == kEOF) return kEOF;
      if (d == mx) {
        ++i;
      } else {
        mx = d;
        mi = (int32_t)i;
        i = 0;
      }
    }
    nxt = mx + 1;
    return mx;
  }
  int32_t advance(int32_t t) override {
    nxt = t;
    return next();
  }
};

// OrDocIdIterator: the smallest next doc of the children; exhausted children dropped.
struct OrIter : Iter {
  std::vector<std::unique_ptr<Iter>> its;
  std::vector<int32_t> nd;
  int32_t prev = -1;
  void drop() {
    size_t i = 0, k = its.size();
    while (i < k) {
      if (nd[i] == kEOF) {
        --k;
        std::swap(its[i], its[k]);
        std::swap(nd[i], nd[k]);
      } else {
        ++i;
      }
    }
    its.resize(k);
    nd.resize(k);
  }
  void init() { nd.assign(its.size(), -1); }
  int32_t next() override {
    bool have = false, ex = false;
    int32_t best = 0;
    for (size_t i = 0; i < its.size(); ++i) {
      int32_t d = nd[i];
      if (d == prev) {
        d = its[i]->next();
        nd[i] = d;
        if (d == kEOF) {
          ex = true;
          continue;
        }
      }
      if (!have || d < best) best = d;
      have = true;
    }
    if (ex) drop();
    if (!have) return kEOF;
    prev = best;
    return best;
  }
  int32_t advance(int32_t t) override {
    bool have = false, ex = false;
    int32_t best = 0;
    for (size_t i = 0; i < its.size(); ++i) {
      int32_t d = nd[i];
      if (d < t) {
        d = its[i]->advance(t);
        nd[i] = d;
        if (d == kEOF) {
          ex = true;
          continue;
        }
      }
      if (!have || d < best) best = d;
      have = true;
    }
    if (ex) drop();
    if (!have) return kEOF;
    prev = best;
    return best;
  }
};

// NotDocIdIterator: the docs the child does not yield.
struct NotIter : Iter {
  std::unique_ptr<Iter> child;
  int32_t n, nxt = 0, nnm;
  NotIter(std::unique_ptr<Iter> c, int32_t docs) : child(std::move(c)), n(docs) {
    const int32_t d = child->next();
    nnm = d == kEOF ? n : d;
  }
  int32_t next() override {
    while (nxt == nnm) {
      ++nxt;
      const int32_t d = child->next();
      nnm = d == kEOF ? n : d;
    }
    if (nxt >= n) return kEOF;
    return nxt++;
  }
  int32_t advance(int32_t t) override {
    nxt = t;
    if (t > nnm) {
      const int32_t d = child->advance(t);
      nnm = d == kEOF ? n : d;
    }
    return next();
  }
};

// Filter tree of one segment's prefix-order program.
struct Node {
  int op = PGPU_F_MATCH_ALL;
  int leaf = -1;
  std::vector<Node> kids;
};

constexpr int kMaxDepth = 256;  // nesting bound: a malformed program fails, it never exhausts the stack

int parse(const pgpu_filter_node* nd, int n, int i, int* leaf, Node* out, int depth = 0) {
  if (i < 0 || i >= n || depth > kMaxDepth) return -1;
  const int op = nd[i].op;
  out->op = op;
  switch (op) {
    case PGPU_F_MATCH_ALL:
    case PGPU_F_EMPTY:
    case PGPU_F_SCAN:
    case PGPU_F_INVERTED:
    case PGPU_F_SORTED:
    case PGPU_F_RAW_SCAN:
    case PGPU_F_RANGE_INDEX:
      if (op != PGPU_F_MATCH_ALL && op != PGPU_F_EMPTY) out->leaf = (*leaf)++;
      return i + 1;
    case PGPU_F_NOT: {
      out->kids.emplace_back();
      return parse(nd, n, i + 1, leaf, &out->kids.back(), depth + 1);
    }
    case PGPU_F_AND_BEGIN:
    case PGPU_F_OR_BEGIN: {
      const bool a = op == PGPU_F_AND_BEGIN;
      int j = i + 1;
      while (j < n && nd[j].op != (a ? PGPU_F_AND_END : PGPU_F_OR_END)) {
        out->kids.emplace_back();
        j = parse(nd, n, j, leaf, &out->kids.back(), depth + 1);
        if (j < 0 || j >= n || nd[j].op != (a ? PGPU_F_AND_CHILD_END : PGPU_F_OR_CHILD_END)) return -1;
        ++j;
      }
      return j < n ? j + 1 : -1;
    }
    default:
      return -1;
  }
}

struct Builder {
  const std::vector<BitSet>* leaves;
  int32_t n;
  int64_t* counter;
  const int32_t* const* leaf_off;  // per leaf: multi-value row offsets or null (may be null altogether)

  std::unique_ptr<Iter> make(const Node& x) {
    switch (x.op) {
      case PGPU_F_SCAN:
      case PGPU_F_RAW_SCAN:  // SVScanDocIdIterator over raw values counts like the dictionary scan
        return std::unique_ptr<Iter>(new ScanIter(&(*leaves)[x.leaf], counter, leaf_off ? leaf_off[x.leaf] : nullptr));
      case PGPU_F_RANGE_INDEX:  // RangeIndexBasedFilterOperator: a BitmapDocIdSet of the exact index's matches
      case PGPU_F_INVERTED:
        return std::unique_ptr<Iter>(new DocsIter(std::make_shared<BitSet>((*leaves)[x.leaf]), BITMAP));
      case PGPU_F_SORTED:
        return std::unique_ptr<Iter>(new DocsIter(std::make_shared<BitSet>((*leaves)[x.leaf]), SORTED));
      case PGPU_F_MATCH_ALL: {
        auto b = std::make_shared<BitSet>(n);
        for (auto& w : b->w) w = ~0ull;
        b->trim();
        return std::unique_ptr<Iter>(new DocsIter(b, OTHER));
      }
      case PGPU_F_EMPTY:
        return std::unique_ptr<Iter>(new DocsIter(std::make_shared<BitSet>(n), OTHER));
      case PGPU_F_NOT:
        return std::unique_ptr<Iter>(new NotIter(make(x.kids[0]), n));
      default:
        break;
    }
    const bool is_and = x.op == PGPU_F_AND_BEGIN;
    std::vector<std::unique_ptr<Iter>> its;
    for (const Node& k : x.kids) its.push_back(make(k));
    std::vector<Iter*> idx, scans;
    for (auto& it : its) {
      if (it->kind == SORTED || it->kind == BITMAP) idx.push_back(it.get());
      else if (it->kind == SCAN) scans.push_back(it.get());
    }
    auto rest_of = [&](bool keep_scans) {
      std::vector<std::unique_ptr<Iter>> rest;
      for (auto& it : its)
        if (it->kind == OTHER || (keep_scans && it->kind == SCAN)) rest.push_back(std::move(it));
      return rest;
    };
    if (is_and) {
      if ((!idx.empty() && !scans.empty()) || idx.size() > 1) {
        // index children intersected into one set, then each scan child's applyAnd over it
        auto docs = std::make_shared<BitSet>(*static_cast<DocsIter*>(idx[0])->docs);
        for (size_t k = 1; k < idx.size(); ++k) {
          const BitSet& o = *static_cast<DocsIter*>(idx[k])->docs;
          for (size_t i = 0; i < docs->w.size(); ++i) docs->w[i] &= o.w[i];
        }
        for (Iter* s : scans) static_cast<ScanIter*>(s)->apply_and(*docs);
        std::unique_ptr<Iter> merged(new DocsIter(docs, BITMAP));  // RangelessBitmapDocIdIterator
        auto rest = rest_of(false);
        if (rest.empty()) return merged;
        auto* a = new AndIter();
        a->its.push_back(std::move(merged));
        for (auto& r : rest) a->its.push_back(std::move(r));
        return std::unique_ptr<Iter>(a);
      }
      auto* a = new AndIter();
      a->its = std::move(its);
      return std::unique_ptr<Iter>(a);
    }
    if (idx.size() > 1) {
      auto docs = std::make_shared<BitSet>(n);
      for (Iter* it : idx) {
        const BitSet& o = *static_cast<DocsIter*>(it)->docs;
        for (size_t i = 0; i < docs->w.size(); ++i) docs->w[i] |= o.w[i];
      }
      std::unique_ptr<Iter> merged(new DocsIter(docs, BITMAP));  // BitmapDocIdIterator
      auto rest = rest_of(true);
      if (rest.empty()) return merged;
      auto* o = new OrIter();
      o->its.push_back(std::move(merged));
      for (auto& r : rest) o->its.push_back(std::move(r));
      o->init();
      return std::unique_ptr<Iter>(o);
    }
    auto* o = new OrIter();
    o->its = std::move(its);
    o->init();
    return std::unique_ptr<Iter>(o);
  }
};

}  // namespace

// numEntriesScannedInFilter of one segment: the program's iterator tree drained like DocIdSetOperator does.
// leaf_words[k] = match bits of leaf k (prefix order), doc d at bit d % 32 of word d / 32.  Returns -1 on a
// malformed program.
int64_t reference_entries_scanned(const pgpu_filter_node* nodes, int num_nodes, const uint32_t* const* leaf_words,
                                  int num_leaves, int32_t num_docs, const int32_t* const* leaf_offsets) {
  if (num_nodes <= 0) return 0;
  Node root;
  int leaf = 0;
  if (parse(nodes, num_nodes, 0, &leaf, &root) != num_nodes || leaf != num_leaves) return -1;
  std::vector<BitSet> leaves;
  leaves.reserve(num_leaves);
  for (int k = 0; k < num_leaves; ++k) leaves.push_back(BitSet::from_words32(leaf_words[k], num_docs));
  int64_t counter = 0;
  Builder b{&leaves, num_docs, &counter, leaf_offsets};
  std::unique_ptr<Iter> it = b.make(root);
  while (it->next() != kEOF) {
  }
  return counter;
}

namespace {

bool has_scan(const Node& x) {
  if (x.op == PGPU_F_SCAN || x.op == PGPU_F_RAW_SCAN) return true;
  for (const Node& k : x.kids)
    if (has_scan(k)) return true;
  return false;
}

// Does the GPU's own count (every scan leaf reads the docs that survive the AND children before it, OR / NOT
// children read their parent's docs) equal the reference's for this subtree driven by next() from its start?
bool gpu_count_matches(const Node& x) {
  switch (x.op) {
    case PGPU_F_NOT:
      return gpu_count_matches(x.kids[0]);
    case PGPU_F_OR_BEGIN:
      for (const Node& k : x.kids)  // OrDocIdIterator drives every child with next() (merged index sets too)
        if (!gpu_count_matches(k)) return false;
      return true;
    case PGPU_F_AND_BEGIN: {
      int idx = 0, scans = 0;
      bool rest = false, rest_scans = false;
      for (const Node& k : x.kids) {
        if (k.op == PGPU_F_SORTED || k.op == PGPU_F_INVERTED || k.op == PGPU_F_RANGE_INDEX) ++idx;
        else if (k.op == PGPU_F_SCAN || k.op == PGPU_F_RAW_SCAN) ++scans;
        else {
          rest = true;
          rest_scans |= has_scan(k);
        }
      }
      if ((idx > 0 && scans > 0) || idx > 1)  // index merge, then applyAnd per scan in order: the GPU's order
        return !rest || (scans == 0 && !rest_scans);
      return scans == 0 && !rest_scans;  // leap-frogging scan iterators resume at data-dependent docs
    }
    default:
      return true;
  }
}

}  // namespace

// Whether the GPU's filter count equals the reference's for this program (pgpu_runtime.cpp).
bool pgpu_filter_count_is_reference(const pgpu_filter_node* nodes, int num_nodes) {
  if (num_nodes <= 0) return true;
  Node root;
  int leaf = 0;
  if (parse(nodes, num_nodes, 0, &leaf, &root) != num_nodes) return false;
  return gpu_count_matches(root);
}

extern "C" int pgpu_filter_entries_scanned(const pgpu_filter_node* nodes, int32_t num_nodes,
                                           const uint32_t* const* leaf_bits, int32_t num_leaves, int32_t num_docs,
                                           int64_t* out) {
  if (!out || num_docs < 0 || num_leaves < 0 || (num_nodes > 0 && !nodes) || (num_leaves > 0 && !leaf_bits))
    return PGPU_E_INVALID;
  const int64_t c = reference_entries_scanned(nodes, num_nodes, leaf_bits, num_leaves, num_docs, nullptr);
  if (c < 0) return PGPU_E_INVALID;
  *out = c;
  return PGPU_OK;
}
