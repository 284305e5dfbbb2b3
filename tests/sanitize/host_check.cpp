// host_check.cpp — drives libcgx's host-only code under AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/sanitize/Makefile builds the host
// objects with -fsanitize=address,undefined; the device code is not
// instrumented). No GPU is touched. Covered:
//   * cgx_mm_read / cgx_mm_write_lower (cgx_mm.cpp) on every golden .mtx
//     (including the quirk files) at 1..8 threads, and a write/read round
//     trip;
//   * the SELL and SELL-P planners (cgx_sell_plan, cgx_sellp_plan) and the
//     row-block schedule (cgx_row_blocks) on Poisson, irregular, empty-row
//     and single-row matrices;
//   * the halo planners (cgx_plan_ghosts, cgx_plan_remap) on 1-D row
//     partitions of those matrices at 1..5 ranks.
// Any sanitizer report aborts with a non-zero exit; the test checks exit 0.
//   host_check <golden dir> <tmp dir>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "cgx.h"

#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAILED %s at %s:%d\n", #c, __FILE__, __LINE__); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

struct Csr {
  std::vector<int> rp, col;
  std::vector<double> val;
  int64_t n() const { return (int64_t)rp.size() - 1; }
};

static Csr poisson(int dim, int nx, int ny, int nz) {
  Csr m;
  m.rp.push_back(0);
  const long nxy = (long)nx * ny;
  for (long z = 0; z < (dim == 3 ? nz : 1); ++z)
    for (long y = 0; y < ny; ++y)
      for (long x = 0; x < nx; ++x) {
        const long r = x + nx * y + nxy * z;
        auto add = [&](long c, double v) { m.col.push_back((int)c); m.val.push_back(v); };
        if (dim == 3 && z > 0) add(r - nxy, -1);
        if (y > 0) add(r - nx, -1);
        if (x > 0) add(r - 1, -1);
        add(r, 2.0 * dim);
        if (x < nx - 1) add(r + 1, -1);
        if (y < ny - 1) add(r + nx, -1);
        if (dim == 3 && z < nz - 1) add(r + nxy, -1);
        m.rp.push_back((int)m.col.size());
      }
  return m;
}

// rows of 0..maxlen random distinct ascending columns (empty rows included)
static Csr irregular(int64_t n, int maxlen, uint64_t seed) {
  Csr m;
  m.rp.push_back(0);
  uint64_t s = seed;
  auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return s >> 33; };
  for (int64_t r = 0; r < n; ++r) {
    const int len = (int)(rnd() % (maxlen + 1));
    std::vector<int> cs;
    for (int k = 0; k < len; ++k) {
      int64_t c = r + (int64_t)(rnd() % 2001) - 1000;
      if (c < 0) c = 0;
      if (c >= n) c = n - 1;
      cs.push_back((int)c);
    }
    std::sort(cs.begin(), cs.end());
    cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
    for (int c : cs) { m.col.push_back(c); m.val.push_back(1.0 + (double)(rnd() % 7)); }
    m.rp.push_back((int)m.col.size());
  }
  return m;
}

static void plans(const Csr &m) {
  const int64_t n = m.n();
  int64_t nrb = 0;
  int *rb = nullptr;
  int mx = 0;
  EXPECT(cgx_row_blocks(m.rp.data(), n, &nrb, &rb, &mx) == CGX_OK);
  EXPECT(nrb >= 1 && rb[0] == 0 && rb[nrb] == n);
  cgx_free_host(rb);
  for (int R : {1, 2}) {
    int64_t nsl = 0, ndict = 0, nidx = 0, vs = 0;
    int64_t *sl = nullptr;
    int *dict = nullptr;
    unsigned long long *idx = nullptr;
    EXPECT(cgx_sell_plan(m.rp.data(), m.col.data(), n, R, &nsl, &sl, &ndict, &dict, &nidx, &idx,
                         &vs) == CGX_OK);
    cgx_free_host(sl);
    cgx_free_host(dict);
    cgx_free_host(idx);
  }
  int64_t nsl = 0, npat = 0, vs = 0;
  int64_t *sl = nullptr;
  int *pat = nullptr;
  int maxw = 0;
  EXPECT(cgx_sellp_plan(m.rp.data(), m.col.data(), n, &nsl, &sl, &npat, &pat, &vs, &maxw) ==
         CGX_OK);
  cgx_free_host(sl);
  cgx_free_host(pat);
  // halo plans of a 1-D row partition at 1..5 ranks
  for (int world = 1; world <= 5; ++world) {
    std::vector<int64_t> begins(world), counts(world);
    for (int r = 0; r < world; ++r) {
      begins[r] = n * r / world;
      counts[r] = n * (r + 1) / world - begins[r];
    }
    for (int r = 0; r < world; ++r) {
      const int64_t b = begins[r], c = counts[r];
      if (c == 0) continue;
      std::vector<int> cols(m.col.begin() + m.rp[b], m.col.begin() + m.rp[b + c]);
      int64_t ng = 0;
      int64_t *gh = nullptr;
      std::vector<int64_t> recv(world);
      EXPECT(cgx_plan_ghosts(c, b, (int64_t)cols.size(), cols.data(), world, begins.data(),
                             counts.data(), &ng, &gh, recv.data()) == CGX_OK);
      int64_t tot = 0;
      for (int64_t v : recv) tot += v;
      EXPECT(tot == ng);
      EXPECT(cgx_plan_remap(c, b, (int64_t)cols.size(), cols.data(), ng, gh) == CGX_OK);
      for (int v : cols) EXPECT(v >= 0 && v < c + ng);
      cgx_free_host(gh);
    }
  }
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  const std::string gold = argv[1], tmp = argv[2];
  const char *files[] = {"poisson2d_16.mtx", "poisson2d_128.mtx", "poisson3d_16.mtx",
                         "quirks_emptyrow.mtx", "quirks_general.mtx", "quirks_nocomment.mtx"};
  for (const char *f : files) {
    for (int threads : {1, 3, 8}) {
      int64_t n = 0, nnz = 0;
      int *rp = nullptr, *col = nullptr;
      double *val = nullptr;
      EXPECT(cgx_mm_read((gold + "/" + f).c_str(), threads, &n, &nnz, &rp, &col, &val) == CGX_OK);
      Csr m;
      m.rp.assign(rp, rp + n + 1);
      m.col.assign(col, col + nnz);
      m.val.assign(val, val + nnz);
      cgx_free_host(rp);
      cgx_free_host(col);
      cgx_free_host(val);
      // the quirk files keep the loader's Q3 behaviour (empty rows dropped, so
      // columns may point past N): no partition owns those columns
      if (threads == 1 && std::string(f).rfind("quirks", 0) != 0) plans(m);
    }
  }
  // write / read round trip of a symmetric matrix
  Csr p = poisson(3, 9, 7, 5);
  const std::string out = tmp + "/rt.mtx";
  EXPECT(cgx_mm_write_lower(out.c_str(), p.n(), p.rp.data(), p.col.data(), p.val.data(), 4) ==
         CGX_OK);
  int64_t n = 0, nnz = 0;
  int *rp = nullptr, *col = nullptr;
  double *val = nullptr;
  EXPECT(cgx_mm_read(out.c_str(), 4, &n, &nnz, &rp, &col, &val) == CGX_OK);
  EXPECT(n == p.n() && nnz == (int64_t)p.val.size());
  for (int64_t k = 0; k < nnz; ++k) EXPECT(col[k] == p.col[k] && val[k] == p.val[k]);
  cgx_free_host(rp);
  cgx_free_host(col);
  cgx_free_host(val);
  // a missing file is an error, not a crash
  EXPECT(cgx_mm_read((tmp + "/missing.mtx").c_str(), 2, &n, &nnz, &rp, &col, &val) != CGX_OK);
  plans(poisson(2, 130, 70, 1));
  plans(poisson(3, 33, 17, 9));
  plans(irregular(20000, 40, 1));
  plans(irregular(3000, 200, 2));
  plans(poisson(2, 1, 1, 1));
  std::printf("host_check ok\n");
  return 0;
}
