// nlp/ingest.hxx -- host-side input preparation of the reference's experiment
// (SURVEY.md §8(f) N1 and N2), bit-compatible with its graph library:
//
//   readMtx            MatrixMarket -> sorted, deduplicated adjacency rows
//                      (mtx.hxx:39-54, 119-135, 235-244; LazyBitset update with an
//                      empty row = sort + keep-last unique, _bitset.hxx:245-262,
//                      _algorithm.hxx:181)
//   symmetrize         reverse edges merged into every row with the reference's
//                      set_union_last_inplace, INCLUDING its duplicate quirk
//                      (symmetrize.hxx:72-82, _algorithm.hxx:176-214)
//   removeSelfLoops    one occurrence of (u, u) per vertex (selfLoop.hxx:120-126)
//   generateEdgeDeletions
//                      the reference's sampler, draw for draw: std::default_random_engine
//                      (minstd_rand0) + uniform_real_distribution<double>, u uniform in
//                      [i, i + n), then the floor(U * deg u)-th entry of N(u), both
//                      directions, up to 5 attempts per deletion (batch.hxx:29-58,
//                      99-112, _utility.hxx:199-203)
//   tidyDeletions      keep existing, sort by (u, v), unique (batch.hxx:152-208)
//   applyDeletions     remove ONE occurrence per deletion (set_difference_inplace,
//                      _algorithm.hxx:113-143, _bitset.hxx:227-239, batch.hxx:239-247)
//   ingestExperiment   main.cxx:241-245 + 164-169 in one call.
//
// Everything here is plain C++17 over CSR arrays (no reference types): the
// graph is a `HostCsr` with the graph concept the predict.hxx mirror accepts
// (key_type, span, hasVertex, forEachEdgeKey).  Rows are processed in parallel
// with OpenMP when compiled with -fopenmp; the results do not depend on it.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <random>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace nlp {

/** A directed multigraph as CSR with the reference's vertex ids (row 0 empty). */
struct HostCsr {
  using key_type = uint32_t;
  std::vector<uint64_t> off{0};  // span + 1
  std::vector<uint32_t> keys;
  size_t span() const { return off.size() - 1; }
  size_t size() const { return keys.size(); }                   // Graph::size(): entries, duplicates counted
  uint64_t degree(uint32_t u) const { return off[u + 1] - off[u]; }
  bool hasVertex(uint32_t u) const { return u >= 1 && u < span(); }  // ids 1..n exist (mtx.hxx:214)
  template <class F>
  void forEachEdgeKey(uint32_t u, F f) const {
    for (uint64_t i = off[u]; i < off[u + 1]; ++i) f(keys[i]);
  }
  /** Any occurrence of v in N(u) (LazyBitset::has). */
  bool hasEdge(uint32_t u, uint32_t v) const {
    if (u >= span()) return false;
    return std::binary_search(keys.begin() + off[u], keys.begin() + off[u + 1], v);
  }
};

namespace detail {

// Rows from per-row lists.
inline HostCsr fromRows(const std::vector<std::vector<uint32_t>>& rows) {
  HostCsr g;
  g.off.assign(rows.size() + 1, 0);
  for (size_t u = 0; u < rows.size(); ++u) g.off[u + 1] = g.off[u] + rows[u].size();
  g.keys.resize(g.off.back());
  for (size_t u = 0; u < rows.size(); ++u) std::copy(rows[u].begin(), rows[u].end(), g.keys.begin() + g.off[u]);
  return g;
}

/**
 * The reference's in-place union of a sorted row x with sorted pending keys y,
 * keeping the last of matching entries (_algorithm.hxx:176-214), restated on
 * keys.  Equal keys met while an x entry waits in the deque are not merged, so
 * the result can hold adjacent duplicates: that is the behaviour
 * the reference's graphs carry into prediction, and it is kept here on purpose.
 */
inline std::vector<uint32_t> unionLastQuirk(const std::vector<uint32_t>& x, const std::vector<uint32_t>& y) {
  if (y.empty()) return x;
  std::vector<uint32_t> out;
  out.reserve(x.size() + y.size());
  auto uniqueTail = [&](size_t j) {  // unique_last_copy of y[j..]
    for (; j < y.size(); ++j)
      if (j + 1 == y.size() || y[j + 1] != y[j]) out.push_back(y[j]);
  };
  if (x.empty()) { uniqueTail(0); return out; }
  size_t i = 0, j = 0;
  // deque-free phase: skip x entries below y[j], absorb equal keys
  for (;;) {
    while (x[i] < y[j]) {
      if (++i == x.size()) {
        out.assign(x.begin(), x.end());
        uniqueTail(j);
        return out;
      }
    }
    if (x[i] != y[j]) break;  // x[i] > y[j]
    if (++j == y.size()) return x;
  }
  out.assign(x.begin(), x.begin() + i);  // the untouched prefix
  std::deque<uint32_t> q;
  q.push_back(x[i++]);
  out.push_back(y[j++]);
  while (j < y.size()) {
    if (out.back() == y[j]) {  // equal to the last written entry: replaced
      ++j;
      continue;
    }
    if (i < x.size()) q.push_back(x[i++]);
    if (!q.empty() && q.front() < y[j]) {
      out.push_back(q.front());
      q.pop_front();
    } else {
      out.push_back(y[j++]);
    }
  }
  for (;;) {
    if (i < x.size()) q.push_back(x[i++]);
    if (q.empty()) break;
    out.push_back(q.front());
    q.pop_front();
  }
  return out;
}

/** Remove one occurrence of every key of the sorted list y from the sorted
 *  row x (set_difference_inplace, _algorithm.hxx:113-143). */
inline void differenceOnce(std::vector<uint32_t>& x, const std::vector<uint32_t>& y) {
  if (x.empty() || y.empty()) return;
  std::vector<uint32_t> out;
  out.reserve(x.size());
  size_t i = 0, j = 0;
  while (i < x.size()) {
    while (j < y.size() && y[j] < x[i]) ++j;
    if (j < y.size() && y[j] == x[i]) {
      ++i;
      ++j;  // this y key is used up
      continue;
    }
    out.push_back(x[i++]);
  }
  x.swap(out);
}

inline std::vector<std::vector<uint32_t>> toRows(const HostCsr& g) {
  std::vector<std::vector<uint32_t>> rows(g.span());
#pragma omp parallel for schedule(dynamic, 2048)
  for (int64_t u = 0; u < (int64_t)g.span(); ++u) rows[u].assign(g.keys.begin() + g.off[u], g.keys.begin() + g.off[u + 1]);
  return rows;
}

// fast unsigned parse; returns false at end of line / input
inline bool parseU64(const char*& p, const char* e, uint64_t& v) {
  while (p < e && (*p == ' ' || *p == '\t')) ++p;
  if (p >= e || *p < '0' || *p > '9') return false;
  uint64_t x = 0;
  while (p < e && *p >= '0' && *p <= '9') x = x * 10 + (uint64_t)(*p++ - '0');
  v = x;
  return true;
}

}  // namespace detail

/** The body of a MatrixMarket coordinate file: its order n = max(rows, cols),
 *  the header's symmetry, and the directed pairs the reference's reader hands
 *  to its graph (mtx.hxx:119-188: both directions for a symmetric header), in
 *  file order. */
struct MtxPairs {
  uint64_t n = 0;
  bool coordinate = false;
  bool symmetric = false;
  std::vector<uint32_t> src, dst;
};

/**
 * Parse a MatrixMarket file's pairs on all threads (the reference's
 * readMtxDoOmp parses 131072-line batches with `#pragma omp parallel for`,
 * mtx.hxx:152-188): the file is read once, the body cut into one byte range
 * per thread at line ends, every range parsed into its own pair list, the
 * lists concatenated in file order.  A line that does not start with two
 * integers ends the body (mtx.hxx:130); an id beyond n throws.
 */
inline MtxPairs readMtxPairs(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("nlp::readMtx: cannot open " + path);
  std::vector<char> text;
  {
    // a regular file is read in one piece; a stream that cannot seek (a pipe,
    // `nlp_main <(zcat g.mtx.gz)`) in chunks until its end, like the
    // reference's ifstream (mtx.hxx:138)
    const long sz = fseek(f, 0, SEEK_END) == 0 ? ftell(f) : -1L;
    if (sz > 0 && fseek(f, 0, SEEK_SET) == 0) {
      text.resize((size_t)sz);
      if (fread(text.data(), 1, text.size(), f) != text.size()) {
        fclose(f);
        throw std::runtime_error("nlp::readMtx: short read of " + path);
      }
    } else {
      clearerr(f);
      const size_t chunk = size_t(1) << 24;
      for (;;) {
        const size_t at = text.size();
        text.resize(at + chunk);
        const size_t got = fread(text.data() + at, 1, chunk, f);
        text.resize(at + got);
        if (got < chunk) break;
      }
      if (ferror(f)) {
        fclose(f);
        throw std::runtime_error("nlp::readMtx: read error on " + path);
      }
    }
    fclose(f);
  }
  if (text.empty()) throw std::runtime_error("nlp::readMtx: empty input " + path);
  const char* p = text.data();
  const char* e = p + text.size();
  MtxPairs out;
  std::string line;
  // comments and the banner (mtx.hxx:42-48)
  while (p < e) {
    const char* q = (const char*)memchr(p, '\n', e - p);
    if (!q) q = e;
    line.assign(p, q);
    p = q < e ? q + 1 : e;
    if (line.rfind("%", 0) != 0) break;
    if (line.rfind("%%", 0) != 0) continue;
    char h[5][64] = {};
    sscanf(line.c_str(), "%63s %63s %63s %63s %63s", h[0], h[1], h[2], h[3], h[4]);
    out.coordinate = strcmp(h[1], "matrix") == 0 && strcmp(h[2], "coordinate") == 0;
    out.symmetric = strcmp(h[4], "symmetric") == 0 || strcmp(h[4], "skew-symmetric") == 0;
  }
  if (!out.coordinate) return out;  // the reference reads nothing (mtx.hxx:49)
  unsigned long long rows = 0, cols = 0, size = 0;
  sscanf(line.c_str(), "%llu %llu %llu", &rows, &cols, &size);
  out.n = std::max(rows, cols);
  if (out.n == 0) return out;
  const uint64_t n = out.n;
  const bool sym = out.symmetric;
  // one byte range per thread, starting after a line end
  int T = 1;
#ifdef _OPENMP
  T = omp_get_max_threads();
#endif
  const size_t body = (size_t)(e - p);
  T = (int)std::max<size_t>(1, std::min<size_t>((size_t)T, body / 4096 + 1));
  std::vector<const char*> cut(T + 1);
  cut[0] = p;
  cut[T] = e;
  for (int t = 1; t < T; ++t) {
    const char* c = p + body * t / T;
    const char* nl = c > p ? (const char*)memchr(c - 1, '\n', e - (c - 1)) : c;
    cut[t] = nl ? std::max(cut[t - 1], nl + 1) : e;
  }
  std::vector<std::vector<uint32_t>> ps(T), pd(T);
  std::vector<char> bad(T, 0), oob(T, 0);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t < T; ++t) {
    const char* a = cut[t];
    const char* z = cut[t + 1];
    auto& su = ps[t];
    auto& sv = pd[t];
    su.reserve((size_t)(z - a) / 8 * (sym ? 2 : 1));
    sv.reserve(su.capacity());
    while (a < z) {
      uint64_t u, v;
      const char* q = a;
      if (!detail::parseU64(q, z, u) || !detail::parseU64(q, z, v)) {
        bad[t] = 1;  // the body ends here (mtx.hxx:130)
        break;
      }
      const char* nl = (const char*)memchr(q, '\n', z - q);
      a = nl ? nl + 1 : z;
      if (u > n || v > n) {
        oob[t] = 1;
        break;
      }
      su.push_back((uint32_t)u);
      sv.push_back((uint32_t)v);
      if (sym) {
        su.push_back((uint32_t)v);
        sv.push_back((uint32_t)u);
      }
    }
  }
  // file order: the ranges up to the first one that ended the body
  int last = T - 1;
  for (int t = 0; t < T; ++t)
    if (bad[t] || oob[t]) {
      last = t;
      break;
    }
  for (int t = 0; t <= last; ++t)
    if (oob[t]) throw std::runtime_error("nlp::readMtx: vertex id beyond the header's order");
  std::vector<size_t> at(last + 2, 0);
  for (int t = 0; t <= last; ++t) at[t + 1] = at[t] + ps[t].size();
  out.src.resize(at[last + 1]);
  out.dst.resize(at[last + 1]);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t <= last; ++t) {
    std::copy(ps[t].begin(), ps[t].end(), out.src.begin() + at[t]);
    std::copy(pd[t].begin(), pd[t].end(), out.dst.begin() + at[t]);
  }
  return out;
}

/**
 * Read a MatrixMarket coordinate file as the reference does (readMtxOmpW with
 * weighted = false): header "%%MatrixMarket matrix coordinate <field> <sym>",
 * span = max(rows, cols) + 1, 1-based ids, symmetric / skew-symmetric headers
 * add both directions; every row is sorted and deduplicated.  `symmetricHeader`
 * receives whether the header said symmetric.
 */
inline HostCsr readMtx(const std::string& path, bool* symmetricHeader = nullptr) {
  MtxPairs mp = readMtxPairs(path);
  if (symmetricHeader) *symmetricHeader = mp.symmetric;
  if (!mp.coordinate) return HostCsr();
  const uint64_t n = mp.n;
  HostCsr g;
  g.off.assign(n + 2, 0);
  if (n == 0) return g;
  const std::vector<uint32_t>& eu = mp.src;
  const std::vector<uint32_t>& ev = mp.dst;
  // counting sort by source, stable (file order inside a row)
  for (size_t i = 0; i < eu.size(); ++i) ++g.off[eu[i] + 1];
  for (size_t u = 1; u < g.off.size(); ++u) g.off[u] += g.off[u - 1];
  std::vector<uint32_t> keys(eu.size());
  {
    std::vector<uint64_t> cur(g.off.begin(), g.off.end() - 1);
    for (size_t i = 0; i < eu.size(); ++i) keys[cur[eu[i]]++] = ev[i];
  }
  // update of rows that were empty: sort + unique (_bitset.hxx:258-259, _algorithm.hxx:181)
  std::vector<uint64_t> deg(n + 1);
#pragma omp parallel for schedule(dynamic, 2048)
  for (int64_t u = 0; u <= (int64_t)n; ++u) {
    auto b = keys.begin() + g.off[u], en = keys.begin() + g.off[u + 1];
    std::sort(b, en);
    deg[u] = std::unique(b, en) - b;
  }
  HostCsr o;
  o.off.assign(n + 2, 0);
  for (uint64_t u = 0; u <= n; ++u) o.off[u + 1] = o.off[u] + deg[u];
  o.keys.resize(o.off.back());
#pragma omp parallel for schedule(dynamic, 2048)
  for (int64_t u = 0; u <= (int64_t)n; ++u)
    std::copy(keys.begin() + g.off[u], keys.begin() + g.off[u] + deg[u], o.keys.begin() + o.off[u]);
  return o;
}

/** symmetrizeOmp (symmetrize.hxx:72-82): every row v receives u for each u -> v,
 *  merged with the reference's union (duplicate quirk included). */
inline HostCsr symmetrize(const HostCsr& x) {
  const size_t S = x.span();
  // pending keys of row v: the sources u of u -> v in ascending u (the order
  // addEdge appends them; distinct, so the update's sort leaves them as is)
  std::vector<uint64_t> toff(S + 1, 0);
  for (uint32_t v : x.keys) ++toff[v + 1];
  for (size_t v = 1; v <= S; ++v) toff[v] += toff[v - 1];
  std::vector<uint32_t> tkeys(x.size());
  {
    std::vector<uint64_t> cur(toff.begin(), toff.end() - 1);
    for (size_t u = 0; u < S; ++u)
      for (uint64_t i = x.off[u]; i < x.off[u + 1]; ++i) tkeys[cur[x.keys[i]]++] = (uint32_t)u;
  }
  std::vector<std::vector<uint32_t>> rows(S);
#pragma omp parallel for schedule(dynamic, 2048)
  for (int64_t v = 0; v < (int64_t)S; ++v) {
    std::vector<uint32_t> xr(x.keys.begin() + x.off[v], x.keys.begin() + x.off[v + 1]);
    std::vector<uint32_t> yr(tkeys.begin() + toff[v], tkeys.begin() + toff[v + 1]);
    rows[v] = detail::unionLastQuirk(xr, yr);
  }
  return detail::fromRows(rows);
}

/** removeSelfLoopsOmpU (selfLoop.hxx:120-126): one occurrence of u leaves N(u). */
inline HostCsr removeSelfLoops(const HostCsr& x) {
  std::vector<std::vector<uint32_t>> rows = detail::toRows(x);
#pragma omp parallel for schedule(dynamic, 2048)
  for (int64_t u = 1; u < (int64_t)x.span(); ++u) detail::differenceOnce(rows[u], {(uint32_t)u});
  return detail::fromRows(rows);
}

/**
 * generateEdgeDeletions (batch.hxx:99-112) with the reference's random draws:
 * per deletion up to 5 attempts (retry, _utility.hxx:199-203); an attempt draws
 * u = i + floor(n U) and, when deg(u) > 0, the entry floor(U deg(u)) of N(u)
 * (duplicates counted).  Pushes (u, v) and, if undirected, (v, u).
 */
template <class R>
inline std::vector<std::pair<uint32_t, uint32_t>> generateEdgeDeletions(R& rnd, const HostCsr& x, size_t batchSize,
                                                                        size_t i, size_t n, bool undirected) {
  std::vector<std::pair<uint32_t, uint32_t>> del;
  for (size_t l = 0; l < batchSize; ++l) {
    for (int attempt = 0; attempt < 5; ++attempt) {
      std::uniform_real_distribution<> dis(0.0, 1.0);
      const uint32_t u = (uint32_t)(i + n * dis(rnd));
      if (u >= x.span() || x.degree(u) == 0) continue;
      std::uniform_real_distribution<> dis2(0.0, 1.0);
      const uint32_t vi = (uint32_t)(dis2(rnd) * x.degree(u));
      const uint32_t v = x.keys[x.off[u] + vi];
      del.emplace_back(u, v);
      if (undirected) del.emplace_back(v, u);
      break;
    }
  }
  return del;
}

/** tidyBatchUpdateU for deletions (batch.hxx:200-208): keep edges present in x,
 *  sort by (u, v), unique. */
inline void tidyDeletions(std::vector<std::pair<uint32_t, uint32_t>>& del, const HostCsr& x) {
  del.erase(std::remove_if(del.begin(), del.end(), [&](const auto& e) { return !x.hasEdge(e.first, e.second); }),
            del.end());
  std::sort(del.begin(), del.end());
  del.erase(std::unique(del.begin(), del.end()), del.end());
}

/** applyBatchUpdateOmpU with deletions only (batch.hxx:239-247): one occurrence
 *  of each (u, v) leaves N(u); `del` sorted and unique. */
inline HostCsr applyDeletions(const HostCsr& x, const std::vector<std::pair<uint32_t, uint32_t>>& del) {
  std::vector<std::vector<uint32_t>> rows = detail::toRows(x);
  std::vector<uint64_t> start(x.span() + 1, 0);
  for (const auto& e : del)
    if (e.first < x.span()) ++start[e.first + 1];
  for (size_t u = 1; u <= x.span(); ++u) start[u] += start[u - 1];
#pragma omp parallel for schedule(dynamic, 2048)
  for (int64_t u = 0; u < (int64_t)x.span(); ++u) {
    if (start[u] == start[u + 1]) continue;
    std::vector<uint32_t> y;
    for (uint64_t j = start[u]; j < start[u + 1]; ++j)
      if (x.hasVertex(del[j].second)) y.push_back(del[j].second);  // removeEdgeIf (Graph.hxx:343-346)
    detail::differenceOnce(rows[u], y);
  }
  return detail::fromRows(rows);
}

/** The experiment's input: main.cxx:241-245 (read, symmetrize unless the
 *  input is already symmetric, remove self-loops), then one deletion batch of
 *  fraction d of the entries (main.cxx:164-169) drawn from `rnd`. */
struct Experiment {
  HostCsr x;  // after ingest
  HostCsr y;  // after the deletions
  std::vector<std::pair<uint32_t, uint32_t>> deletions;  // directed, sorted, unique (main.cxx deletions0)
};

template <class R>
inline Experiment ingestExperiment(const std::string& mtx, bool symmetricInput, double d, R& rnd) {
  Experiment ex;
  ex.x = readMtx(mtx);
  if (!symmetricInput) ex.x = symmetrize(ex.x);
  ex.x = removeSelfLoops(ex.x);
  ex.deletions = generateEdgeDeletions(rnd, ex.x, (size_t)(d * ex.x.size() / 2), 1, ex.x.span() - 1, true);
  tidyDeletions(ex.deletions, ex.x);
  ex.y = applyDeletions(ex.x, ex.deletions);
  return ex;
}

}  // namespace nlp
