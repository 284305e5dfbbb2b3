// cgx_mm.cpp — Matrix-Market ingest and emit at scale.
//
// cgx_mm_read has the semantics of the reference loader's read_file
// (test/mm_reader.cpp:154-171), rebuilt as a parallel parser:
//   * line 1 is the banner and must hold 5 words (parse_header, :109-144);
//   * line 2 is always discarded (:163-164, quirk Q1): a file without a
//     comment line loses its size line there;
//   * then every line starting with '%' is skipped (skip_comments, :146-152);
//   * the next line is the size line. Its words 0 and 2 must be integers
//     (std::stoi, :49-50); their values are unused;
//   * the body is read as whitespace-separated triplets "i j v"
//     (`while (f >> n >> m >> value)`, :62-66), stopping at the first token
//     that does not parse;
//   * every off-diagonal entry is mirrored, whatever the banner says (:68-74,
//     Q2);
//   * entries are sorted by (row, col) (:76-86). The reference's comparator
//     leaves equal (row, col) pairs in unspecified order; here they keep
//     file order, originals before mirrors, as in the oracle;
//   * rowptr gets a new entry only when the row index increases (:88-104,
//     Q3): empty rows vanish and N counts the non-empty rows.
// Differences, on inputs the reference mishandles:
//   * 1-based indices < 1 are rejected (the reference would index
//     coordinates with negative rows);
//   * a token glued to garbage ("3.0abc") ends the body before its triplet
//     (istream would keep the "3.0" and stop after it).
//
// The body is split at line boundaries into one chunk per thread; chunks
// parse independently when every chunk holds whole triplets, and otherwise
// the body is parsed sequentially. The CSR is built by a stable counting
// sort on rows, then a per-row stable sort on columns (threads over rows).
//
// cgx_mm_write_lower emits the lower triangle as a `symmetric` file with a
// comment line (so Q1 and Q2 round-trip it), values printed "%.17g".
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cgx_objects.h"

namespace {

int pick_threads(int threads) {
  if (threads > 0) return std::min(threads, 256);
  if (const char *e = std::getenv("OMP_NUM_THREADS")) {
    const int t = std::atoi(e);
    if (t > 0) return std::min(t, 256);
  }
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
}

template <class F> void parallel_for(int nt, F &&f) {
  if (nt <= 1) {
    f(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve((size_t)nt);
  for (int t = 0; t < nt; ++t) th.emplace_back(f, t);
  for (auto &x : th) x.join();
}

inline bool is_ws(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

// The next whitespace-delimited token of [p, e): [*tb, *te); false at end.
inline bool next_token(const char *&p, const char *e, const char **tb, const char **te) {
  while (p < e && is_ws(*p)) ++p;
  if (p >= e) return false;
  *tb = p;
  while (p < e && !is_ws(*p)) ++p;
  *te = p;
  return true;
}

inline bool parse_int(const char *b, const char *e, int *out) {
  if (b < e && *b == '+') ++b;
  auto r = std::from_chars(b, e, *out);
  return r.ec == std::errc() && r.ptr == e;
}

inline bool parse_double(const char *b, const char *e, double *out) {
  if (b < e && *b == '+') ++b;
  auto r = std::from_chars(b, e, *out);
  return r.ec == std::errc() && r.ptr == e;
}

// Whitespace-separated words of one line [b, e).
std::vector<std::string> words_of(const char *b, const char *e) {
  std::vector<std::string> w;
  const char *tb, *te;
  while (next_token(b, e, &tb, &te)) w.emplace_back(tb, te);
  return w;
}

// One line starting at p: returns its end (the '\n' or e) and advances p past it.
inline const char *take_line(const char *&p, const char *e) {
  const char *nl = (const char *)std::memchr(p, '\n', (size_t)(e - p));
  const char *end = nl ? nl : e;
  p = nl ? nl + 1 : e;
  return end;
}

struct Chunk {
  std::vector<int> r, c;
  std::vector<double> v;
  int64_t tokens = 0;
  bool stopped = false;  // a token failed to parse: the body ends in this chunk
};

// Triplets of [p, e) into ch; stops at the first token that does not parse
// (the triplet it belongs to is dropped, later text ignored).
void parse_triplets(const char *p, const char *e, Chunk &ch) {
  const char *tb, *te;
  for (;;) {
    int i, j;
    double v;
    if (!next_token(p, e, &tb, &te)) return;
    if (!parse_int(tb, te, &i)) { ch.stopped = true; return; }
    if (!next_token(p, e, &tb, &te)) { ch.stopped = true; return; }
    if (!parse_int(tb, te, &j)) { ch.stopped = true; return; }
    if (!next_token(p, e, &tb, &te)) { ch.stopped = true; return; }
    if (!parse_double(tb, te, &v)) { ch.stopped = true; return; }
    ch.r.push_back(i - 1);
    ch.c.push_back(j - 1);
    ch.v.push_back(v);
  }
}

int64_t count_tokens(const char *p, const char *e) {
  int64_t n = 0;
  const char *tb, *te;
  while (next_token(p, e, &tb, &te)) ++n;
  return n;
}

}  // namespace

using namespace cgx;

extern "C" int cgx_mm_read(const char *path, int threads, int64_t *n_out, int64_t *nnz_out,
                           int **rowptr_out, int **col_out, double **val_out) {
  CGX_REQUIRE(path && n_out && nnz_out && rowptr_out && col_out && val_out, CGX_EINVAL,
              "NULL argument");
  *rowptr_out = *col_out = nullptr;
  *val_out = nullptr;
  FILE *f = std::fopen(path, "rb");
  CGX_REQUIRE(f, CGX_EINVAL, "cannot open %s", path);
  std::fseek(f, 0, SEEK_END);
  const long fsz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<char> buf((size_t)std::max(fsz, 0L));
  const size_t got = buf.empty() ? 0 : std::fread(buf.data(), 1, buf.size(), f);
  std::fclose(f);
  CGX_REQUIRE(got == buf.size(), CGX_EINVAL, "short read of %s", path);
  const char *p = buf.data(), *e = buf.data() + buf.size();
  // banner (parse_header): 5 words
  {
    const char *b = p, *le = take_line(p, e);
    CGX_REQUIRE(words_of(b, le).size() == 5, CGX_EINVAL,
                "%s: the banner line must have 5 words (mm_reader.cpp:118)", path);
  }
  // line 2: discarded unconditionally (Q1)
  CGX_REQUIRE(p < e, CGX_EINVAL, "%s: no line after the banner", path);
  take_line(p, e);
  // comments
  while (p < e && *p == '%') take_line(p, e);
  // size line: words 0 and 2 parse as integers (std::stoi)
  {
    const char *b = p, *le = take_line(p, e);
    auto w = words_of(b, le);
    CGX_REQUIRE(w.size() >= 3, CGX_EINVAL, "%s: size line has %zu words", path, w.size());
    // std::stoi: optional sign, then at least one digit (trailing text ignored)
    auto stoi_ok = [](const std::string &s) {
      size_t k = (!s.empty() && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
      return k < s.size() && s[k] >= '0' && s[k] <= '9';
    };
    CGX_REQUIRE(stoi_ok(w[0]) && stoi_ok(w[2]), CGX_EINVAL,
                "%s: size line words 0 and 2 must be integers", path);
  }
  // body: one chunk per thread, split at line starts
  const int nt = pick_threads(threads);
  const int64_t body = e - p;
  const int nch = (int)std::max<int64_t>(1, std::min<int64_t>(nt, body / (1 << 16)));
  std::vector<const char *> cut((size_t)nch + 1);
  cut[0] = p;
  cut[(size_t)nch] = e;
  for (int k = 1; k < nch; ++k) {
    const char *q = p + body * k / nch;
    q = std::max(q, cut[(size_t)k - 1]);
    const char *nl = (const char *)std::memchr(q, '\n', (size_t)(e - q));
    cut[(size_t)k] = nl ? nl + 1 : e;
  }
  std::vector<Chunk> ch((size_t)nch);
  bool aligned = true;
  if (nch > 1) {
    parallel_for(nch, [&](int k) { ch[(size_t)k].tokens = count_tokens(cut[(size_t)k], cut[(size_t)k + 1]); });
    for (auto &c : ch) aligned = aligned && (c.tokens % 3 == 0);
  }
  if (nch > 1 && aligned) {
    parallel_for(nch, [&](int k) { parse_triplets(cut[(size_t)k], cut[(size_t)k + 1], ch[(size_t)k]); });
  } else {
    ch.assign(1, Chunk{});
    parse_triplets(p, e, ch[0]);
  }
  // triplets in file order, up to the first failure
  std::vector<int> R, Cc;
  std::vector<double> V;
  {
    size_t tot = 0;
    for (auto &c : ch) {
      tot += c.r.size();
      if (c.stopped) break;
    }
    R.reserve(tot);
    Cc.reserve(tot);
    V.reserve(tot);
    for (auto &c : ch) {
      R.insert(R.end(), c.r.begin(), c.r.end());
      Cc.insert(Cc.end(), c.c.begin(), c.c.end());
      V.insert(V.end(), c.v.begin(), c.v.end());
      std::vector<int>().swap(c.r);
      std::vector<int>().swap(c.c);
      std::vector<double>().swap(c.v);
      if (c.stopped) break;
    }
  }
  const size_t h = R.size();
  CGX_REQUIRE(h > 0, CGX_EINVAL, "%s: no entries (the reference reads coordinates[0])", path);
  int maxr = 0;
  for (size_t k = 0; k < h; ++k) {
    CGX_REQUIRE(R[k] >= 0 && Cc[k] >= 0, CGX_EINVAL, "%s: entry %zu has an index < 1", path, k);
    maxr = std::max(maxr, std::max(R[k], Cc[k]));
  }
  // stable counting sort on rows: originals in file order, then mirrors (Q2)
  const size_t nrow = (size_t)maxr + 1;
  std::vector<int64_t> start(nrow + 1, 0);
  size_t cnt = h;
  for (size_t k = 0; k < h; ++k) {
    ++start[(size_t)R[k] + 1];
    if (R[k] != Cc[k]) {
      ++start[(size_t)Cc[k] + 1];
      ++cnt;
    }
  }
  CGX_REQUIRE(cnt < ((size_t)1 << 31), CGX_EINVAL, "%s: %zu entries exceed int32 CSR", path, cnt);
  for (size_t i = 0; i < nrow; ++i) start[i + 1] += start[i];
  std::vector<int64_t> fill(start.begin(), start.end() - 1);
  int *col = (int *)std::malloc(cnt * sizeof(int));
  double *val = (double *)std::malloc(cnt * sizeof(double));
  CGX_REQUIRE(col && val, CGX_ENOMEM, "host allocation of %zu entries failed", cnt);
  for (size_t k = 0; k < h; ++k) {
    const int64_t d = fill[(size_t)R[k]]++;
    col[d] = Cc[k];
    val[d] = V[k];
  }
  for (size_t k = 0; k < h; ++k) {
    if (R[k] == Cc[k]) continue;
    const int64_t d = fill[(size_t)Cc[k]]++;
    col[d] = R[k];
    val[d] = V[k];
  }
  std::vector<int>().swap(R);
  std::vector<int>().swap(Cc);
  std::vector<double>().swap(V);
  // per-row stable sort on columns (rows already grouped)
  std::atomic<size_t> next{0};
  parallel_for(nt, [&](int) {
    std::vector<std::pair<int, double>> tmp;
    for (;;) {
      const size_t i0 = next.fetch_add(4096);
      if (i0 >= nrow) return;
      const size_t i1 = std::min(nrow, i0 + 4096);
      for (size_t i = i0; i < i1; ++i) {
        const int64_t a = start[i], b = start[i + 1];
        bool sorted = true;
        for (int64_t k = a + 1; k < b && sorted; ++k) sorted = col[k - 1] <= col[k];
        if (sorted) continue;
        tmp.clear();
        for (int64_t k = a; k < b; ++k) tmp.emplace_back(col[k], val[k]);
        std::stable_sort(tmp.begin(), tmp.end(),
                         [](const auto &x, const auto &y) { return x.first < y.first; });
        for (int64_t k = a; k < b; ++k) {
          col[k] = tmp[(size_t)(k - a)].first;
          val[k] = tmp[(size_t)(k - a)].second;
        }
      }
    }
  });
  // rowptr over non-empty rows only (Q3)
  int64_t nne = 0;
  for (size_t i = 0; i < nrow; ++i) nne += start[i + 1] > start[i];
  int *rp = (int *)std::malloc(((size_t)nne + 1) * sizeof(int));
  if (!rp) {
    std::free(col);
    std::free(val);
    set_error("host allocation failed");
    return CGX_ENOMEM;
  }
  int64_t q = 0;
  for (size_t i = 0; i < nrow; ++i)
    if (start[i + 1] > start[i]) rp[q++] = (int)start[i];
  rp[q] = (int)cnt;
  *n_out = nne;
  *nnz_out = (int64_t)cnt;
  *rowptr_out = rp;
  *col_out = col;
  *val_out = val;
  return CGX_OK;
}

extern "C" int cgx_mm_write_lower(const char *path, int64_t n, const int *rowptr, const int *col,
                                  const double *val, int threads) {
  CGX_REQUIRE(path && rowptr && (n == 0 || (col && val)), CGX_EINVAL, "NULL argument");
  CGX_REQUIRE(n >= 0, CGX_EINVAL, "n=%lld", (long long)n);
  const int nt = pick_threads(threads);
  const int nparts = (int)std::max<int64_t>(1, std::min<int64_t>(nt * 4, n / 4096 + 1));
  std::vector<std::string> part((size_t)nparts);
  std::vector<int64_t> lower((size_t)nparts, 0);
  std::atomic<int> next{0};
  parallel_for(std::min(nt, nparts), [&](int) {
    char line[96];
    for (;;) {
      const int k = next.fetch_add(1);
      if (k >= nparts) return;
      const int64_t i0 = n * k / nparts, i1 = n * (k + 1) / nparts;
      std::string &s = part[(size_t)k];
      for (int64_t i = i0; i < i1; ++i)
        for (int j = rowptr[i]; j < rowptr[i + 1]; ++j)
          if (col[j] <= i) {
            // "%lld %d %.17g\n" (to_chars general, precision 17: same text)
            char *q = line, *qe = line + sizeof line;
            q = std::to_chars(q, qe, (long long)(i + 1)).ptr;
            *q++ = ' ';
            q = std::to_chars(q, qe, col[j] + 1).ptr;
            *q++ = ' ';
            q = std::to_chars(q, qe, val[j], std::chars_format::general, 17).ptr;
            *q++ = '\n';
            s.append(line, (size_t)(q - line));
            ++lower[(size_t)k];
          }
    }
  });
  int64_t tot = 0;
  for (int64_t l : lower) tot += l;
  FILE *f = std::fopen(path, "wb");
  CGX_REQUIRE(f, CGX_EINVAL, "cannot create %s", path);
  bool ok = std::fprintf(f,
                         "%%%%MatrixMarket matrix coordinate real symmetric\n"
                         "%% written by cgx_mm_write_lower (lower triangle)\n"
                         "%lld %lld %lld\n",
                         (long long)n, (long long)n, (long long)tot) > 0;
  for (auto &s : part)
    ok = ok && (s.empty() || std::fwrite(s.data(), 1, s.size(), f) == s.size());
  ok = (std::fclose(f) == 0) && ok;
  CGX_REQUIRE(ok, CGX_EINVAL, "write to %s failed", path);
  return CGX_OK;
}
