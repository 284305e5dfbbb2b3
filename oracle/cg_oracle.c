/*
 * cg_oracle.c — CPU restatement of the reference CG hot path (test
 * infrastructure only; see cg_oracle.h for who may call it and for the
 * parity-pinning status). Every function cites the reference lines it
 * restates. Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).
 */
#define _GNU_SOURCE
#include "cg_oracle.h"

#include <ctype.h>
#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------------ */
/* Matrix-Market loader: test/mm_reader.cpp                                  */
/* ------------------------------------------------------------------------ */

typedef struct {
  int r, c;
  double v;
  int64_t seq; /* insertion order; makes the sort total (see note below) */
} orc_coo;

/* mm_reader.cpp:133-143 sorts by (row, col) with a `<=` comparator. That is
 * not a strict weak ordering, so std::sort's behaviour on duplicate (row,
 * col) keys is undefined; for unique keys any correct sort gives the same
 * sequence. We break ties by insertion order. */
static int coo_cmp(const void *a, const void *b) {
  const orc_coo *x = (const orc_coo *)a, *y = (const orc_coo *)b;
  if (x->r != y->r) return x->r < y->r ? -1 : 1;
  if (x->c != y->c) return x->c < y->c ? -1 : 1;
  return (x->seq > y->seq) - (x->seq < y->seq);
}

static int count_words(const char *s) {
  int n = 0, in = 0;
  for (; *s; ++s) {
    if (isspace((unsigned char)*s)) in = 0;
    else if (!in) { in = 1; ++n; }
  }
  return n;
}

static int read_line(FILE *f, char **buf, size_t *cap) {
  return getline(buf, cap, f) >= 0;
}

int orc_read_mtx(const char *path, int64_t *n_out, int64_t *nnz_out,
                 int **rowptr_out, int **col_out, double **val_out) {
  FILE *f = fopen(path, "r");
  if (!f) return 1;
  char *line = NULL;
  size_t cap = 0;
  int rc = 0;
  orc_coo *co = NULL;
  /* parse_header (mm_reader.cpp:109-144): the banner must have 5 words
   * (assert at :118); the parsed qualifier is never used afterwards. */
  if (!read_line(f, &line, &cap) || count_words(line) != 5) { rc = 2; goto out; }
  /* read_file (mm_reader.cpp:163-164): line 2 is discarded unconditionally
   * (quirk Q1: a file without a comment line loses its size line here). */
  if (!read_line(f, &line, &cap)) { rc = 3; goto out; }
  /* skip_comments (mm_reader.cpp:146-152) */
  for (;;) {
    int ch = fgetc(f);
    if (ch == EOF) break;
    ungetc(ch, f);
    if (ch != '%') break;
    if (!read_line(f, &line, &cap)) break;
  }
  /* read_real_coordinate_matrix (mm_reader.cpp:45-52): one line is taken as
   * the size line; words[0] and words[2] are parsed and never used. */
  if (!read_line(f, &line, &cap) || count_words(line) < 3) { rc = 4; goto out; }

  /* mm_reader.cpp:62-66: `while (f >> i >> j >> v)` */
  size_t cnt = 0, ccap = 1 << 16;
  co = (orc_coo *)malloc(ccap * sizeof(orc_coo));
  int i, j;
  double v;
  while (fscanf(f, "%d %d %lf", &i, &j, &v) == 3) {
    if (cnt == ccap) { ccap *= 2; co = (orc_coo *)realloc(co, ccap * sizeof(orc_coo)); }
    co[cnt].r = i - 1; co[cnt].c = j - 1; co[cnt].v = v; co[cnt].seq = (int64_t)cnt;
    ++cnt;
  }
  if (cnt == 0) { rc = 5; goto out; } /* reference indexes coordinates[0] (:92) */
  /* mm_reader.cpp:68-74: every off-diagonal entry is mirrored, whatever the
   * banner's qualifier says (quirk Q2). */
  size_t h = cnt;
  for (size_t k = 0; k < h; ++k) {
    if (co[k].r != co[k].c) {
      if (cnt == ccap) { ccap *= 2; co = (orc_coo *)realloc(co, ccap * sizeof(orc_coo)); }
      co[cnt].r = co[k].c; co[cnt].c = co[k].r; co[cnt].v = co[k].v; co[cnt].seq = (int64_t)cnt;
      ++cnt;
    }
  }
  qsort(co, cnt, sizeof(orc_coo), coo_cmp); /* :76-86 */
  /* CSR build (mm_reader.cpp:88-104): rowptr grows only when the row index
   * increases, so empty rows vanish (quirk Q3). */
  int *rp = (int *)malloc((cnt + 2) * sizeof(int));
  int *cl = (int *)malloc(cnt * sizeof(int));
  double *vl = (double *)malloc(cnt * sizeof(double));
  int64_t nrp = 0;
  rp[nrp++] = 0;
  vl[0] = co[0].v; cl[0] = co[0].c;
  for (size_t k = 1; k < cnt; ++k) {
    vl[k] = co[k].v; cl[k] = co[k].c;
    if (co[k].r > co[k - 1].r) rp[nrp++] = (int)k;
  }
  rp[nrp++] = (int)cnt;
  *rowptr_out = rp; *col_out = cl; *val_out = vl;
  *n_out = nrp - 1; *nnz_out = (int64_t)cnt;
out:
  free(co);
  free(line);
  fclose(f);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Synthetic Poisson generator + lower-triangle writer        */
/* ------------------------------------------------------------------------ */

int64_t orc_poisson_nnz(int dim, int nx, int ny, int nz) {
  int64_t n = (int64_t)nx * ny * (dim == 3 ? nz : 1);
  int64_t e = 0; /* off-diagonal couplings in one direction, counted twice */
  e += (int64_t)(nx - 1) * ny * (dim == 3 ? nz : 1);
  e += (int64_t)nx * (ny - 1) * (dim == 3 ? nz : 1);
  if (dim == 3) e += (int64_t)nx * ny * (nz - 1);
  return n + 2 * e;
}

void orc_poisson(int dim, int nx, int ny, int nz, int *rowptr, int *col,
                 double *val) {
  const double diag = 2.0 * dim;
  int64_t k = 0, row = 0;
  const int64_t sxy = (int64_t)nx * ny;
  const int zmax = dim == 3 ? nz : 1;
  rowptr[0] = 0;
  for (int z = 0; z < zmax; ++z)
    for (int y = 0; y < ny; ++y)
      for (int x = 0; x < nx; ++x, ++row) {
        if (dim == 3 && z > 0) { col[k] = (int)(row - sxy); val[k++] = -1.0; }
        if (y > 0) { col[k] = (int)(row - nx); val[k++] = -1.0; }
        if (x > 0) { col[k] = (int)(row - 1); val[k++] = -1.0; }
        col[k] = (int)row; val[k++] = diag;
        if (x < nx - 1) { col[k] = (int)(row + 1); val[k++] = -1.0; }
        if (y < ny - 1) { col[k] = (int)(row + nx); val[k++] = -1.0; }
        if (dim == 3 && z < nz - 1) { col[k] = (int)(row + sxy); val[k++] = -1.0; }
        rowptr[row + 1] = (int)k;
      }
}

int orc_write_mtx_lower(const char *path, int64_t n, const int *rowptr,
                        const int *col, const double *val) {
  FILE *f = fopen(path, "w");
  if (!f) return 1;
  int64_t lower = 0;
  for (int64_t i = 0; i < n; ++i)
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j)
      if (col[j] <= i) ++lower;
  fprintf(f, "%%%%MatrixMarket matrix coordinate real symmetric\n");
  fprintf(f, "%% written by conjugategradient_amd oracle (lower triangle)\n");
  fprintf(f, "%lld %lld %lld\n", (long long)n, (long long)n, (long long)lower);
  for (int64_t i = 0; i < n; ++i)
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j)
      if (col[j] <= i)
        fprintf(f, "%lld %d %.17g\n", (long long)(i + 1), col[j] + 1, val[j]);
  return fclose(f) == 0 ? 0 : 2;
}

/* ------------------------------------------------------------------------ */
/* VectorOperations (src/VectorOperations.hpp)                               */
/* ------------------------------------------------------------------------ */

/* spmv, VectorOperations.hpp:455-462: one row at a time, ascending j,
 * single_result starts at 0 and adds the rounded product. */
void orc_spmv(int64_t n, const int *rowptr, const int *col, const double *val,
              const double *x, double *y) {
  for (int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
    y[i] = s;
  }
}

/* dot_product_trivial, VectorOperations.hpp:300-305: a sycl::reduction
 * without initialize_to_identity adds into the existing scalar (Q4). */
double orc_dot_acc(int64_t n, const double *x, const double *y, double init) {
  double s = init;
  for (int64_t i = 0; i < n; ++i) s += x[i] * y[i];
  return s;
}

/* norm, VectorOperations.hpp:323-327 (sum of squares, no sqrt) */
double orc_norm_acc(int64_t n, const double *x, double init) {
  double s = init;
  for (int64_t i = 0; i < n; ++i) s += x[i] * x[i];
  return s;
}

/* sapbx, VectorOperations.hpp:422-424: result = x + b*y */
void orc_sapbx(int64_t n, const double *x, const double *y, double b,
               double *res) {
  for (int64_t i = 0; i < n; ++i) res[i] = x[i] + b * y[i];
}

/* sambx, VectorOperations.hpp:391-393: result = x - b*y */
void orc_sambx(int64_t n, const double *x, const double *y, double b,
               double *res) {
  for (int64_t i = 0; i < n; ++i) res[i] = x[i] - b * y[i];
}

/* saxpby, VectorOperations.hpp:361-363: result = a*x + b*y */
void orc_saxpby(int64_t n, const double *x, const double *y, double a,
                double b, double *res) {
  for (int64_t i = 0; i < n; ++i) res[i] = a * x[i] + b * y[i];
}

/* ------------------------------------------------------------------------ */
/* CG::solve (src/CG.hpp:255-454), executed in submission order */
/* ------------------------------------------------------------------------ */

int orc_cg_solve(int64_t n, const int *rowptr, const int *col,
                 const double *val, const double *b, double *x, int has_x0,
                 double tol, int64_t max_iter, orc_cg_result *res) {
  if (!b) return 1;                       /* CG.hpp:266-268 */
  if (!rowptr || !col || !val) return 2;  /* CG.hpp:270-272 */
  if (!has_x0) memset(x, 0, (size_t)n * sizeof(double)); /* :291-297 */
  double *helper = (double *)calloc((size_t)n, sizeof(double));
  double *r = (double *)calloc((size_t)n, sizeof(double));
  double *rnext = (double *)calloc((size_t)n, sizeof(double));
  double *p = (double *)calloc((size_t)n, sizeof(double));
  double rxr = 0, value2, value3, alpha, beta, r0;
  const double acc = tol;

  /* InitializeVectors, CG.hpp:324-332 */
  for (int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
    r[i] = b[i] - s;
    p[i] = r[i];
    rnext[i] = p[i];
  }
  rxr = orc_dot_acc(n, r, r, rxr);        /* :341 */
  if (res) res->rxr0 = rxr;
  r0 = sqrt(rxr) * acc;                   /* :351-352 (dead) */
  (void)r0;

  int64_t counter = 0, bodies = 0;
  int done = 0;
  do {
    memset(helper, 0, (size_t)n * sizeof(double));       /* :362 */
    value2 = 0; value3 = 0; alpha = 0; beta = 0;         /* :364-371 */
    orc_spmv(n, rowptr, col, val, p, helper);            /* :374-375 */
    value2 = orc_dot_acc(n, helper, p, value2);          /* :378-379 */
    alpha = rxr / value2;                                /* :385-386 */
    orc_sapbx(n, x, p, alpha, x);                        /* :390 */
    orc_sambx(n, rnext, helper, alpha, rnext);           /* :392-393 */
    if (isnan(rxr) || sqrt(rxr) <= acc) done = 1;        /* :400-403 */
    value3 = orc_dot_acc(n, rnext, rnext, value3);       /* :406-407 */
    beta = value3 / rxr;                                 /* :414 */
    rxr = value3;                                        /* :415 */
    orc_sapbx(n, rnext, p, beta, p);                     /* :418 */
    memcpy(r, rnext, (size_t)n * sizeof(double));        /* :420-423 (dead) */
    ++bodies;
    if (max_iter >= 0 && bodies >= max_iter) break;      /* extension */
  } while ((uint64_t)(counter++) < (uint64_t)n && !done); /* :436 */
  (void)beta; (void)alpha;

  if (res) {
    res->iterations = bodies;
    res->rxr = rxr;
    res->stopped_by_tol = done;
  }
  free(helper); free(r); free(rnext); free(p);
  return 0;
}

/* CG::accuracy, CG.hpp:470-514 */
double orc_accuracy(int64_t n, const int *rowptr, const int *col,
                    const double *val, const double *b, const double *x) {
  double normres = 0, normx = 0;
  for (int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
    double a = b[i] - s;
    normres += a * a;
    normx += x[i] * x[i];
  }
  return fabs(normres / normx);
}

/* ------------------------------------------------------------------------ */
/* CPU baseline: the reference's command sequence on OpenMP threads          */
/* ------------------------------------------------------------------------ */

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

double orc_cg_timed_omp(int64_t n, const int *rowptr, const int *col, const double *val,
                        const double *b, double *x, int64_t warmup, int64_t iters,
                        int threads) {
  omp_set_num_threads(threads > 0 ? threads : 1);
  double *helper = (double *)malloc((size_t)n * sizeof(double));
  double *r = (double *)malloc((size_t)n * sizeof(double));
  double *rnext = (double *)malloc((size_t)n * sizeof(double));
  double *p = (double *)malloc((size_t)n * sizeof(double));
  double rxr = 0;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) x[i] = 0;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
    r[i] = b[i] - s; p[i] = r[i]; rnext[i] = p[i];
  }
#pragma omp parallel for schedule(static) reduction(+ : rxr)
  for (int64_t i = 0; i < n; ++i) rxr += r[i] * r[i];

  double t0 = now_s();
  for (int64_t it = 0; it < warmup + iters; ++it) {
    double value2 = 0, value3 = 0, alpha, beta;
    if (it == warmup) t0 = now_s(); /* the first `warmup` bodies run untimed */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) helper[i] = 0;               /* fill */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {                             /* spmv */
      double s = 0;
      for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * p[col[j]];
      helper[i] = s;
    }
#pragma omp parallel for schedule(static) reduction(+ : value2)
    for (int64_t i = 0; i < n; ++i) value2 += helper[i] * p[i];
    alpha = rxr / value2;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) x[i] = x[i] + alpha * p[i];
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) rnext[i] = rnext[i] - alpha * helper[i];
#pragma omp parallel for schedule(static) reduction(+ : value3)
    for (int64_t i = 0; i < n; ++i) value3 += rnext[i] * rnext[i];
    beta = value3 / rxr;
    rxr = value3;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) p[i] = rnext[i] + beta * p[i];
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) r[i] = rnext[i];              /* copy */
  }
  const double t1 = now_s();
  free(helper); free(r); free(rnext); free(p);
  return t1 - t0;
}

double orc_cg_fixed_iters_omp(int64_t n, const int *rowptr, const int *col,
                              const double *val, const double *b, double *x,
                              int64_t iters, int threads) {
  return orc_cg_timed_omp(n, rowptr, col, val, b, x, 0, iters, threads);
}

/* orc_cg_solve on OpenMP threads (full-size parity tests at 16.8 M rows):
 * the same statements as orc_cg_solve / CG.hpp:314-436 in submission order,
 * stop rule Q5 (old rxr tested after the x update, NaN stops, cap N+1 or
 * max_iter), with each parallel_for an OpenMP loop and each dot an OpenMP
 * reduction (its summation order differs from orc_cg_solve's index order;
 * every other value is rounded identically). x is in/out as in
 * orc_cg_solve (zero-filled first when has_x0 == 0). */
int orc_cg_solve_omp(int64_t n, const int *rowptr, const int *col,
                     const double *val, const double *b, double *x, int has_x0,
                     double tol, int64_t max_iter, int threads,
                     orc_cg_result *res) {
  omp_set_num_threads(threads > 0 ? threads : 1);
  double *helper = (double *)malloc((size_t)n * sizeof(double));
  double *rnext = (double *)malloc((size_t)n * sizeof(double));
  double *p = (double *)malloc((size_t)n * sizeof(double));
  if (!helper || !rnext || !p) { free(helper); free(rnext); free(p); return 3; }
  double rxr = 0;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {                               /* :324-332 */
    if (!has_x0) x[i] = 0;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
    rnext[i] = b[i] - s;
    p[i] = rnext[i];
  }
#pragma omp parallel for schedule(static) reduction(+ : rxr)
  for (int64_t i = 0; i < n; ++i) rxr += rnext[i] * rnext[i];
  if (res) res->rxr0 = rxr;
  int64_t counter = 0, bodies = 0;
  int done = 0;
  do {
    double value2 = 0, value3 = 0, alpha, beta;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {                             /* :374-375 */
      double s = 0;
      for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * p[col[j]];
      helper[i] = s;
    }
#pragma omp parallel for schedule(static) reduction(+ : value2)
    for (int64_t i = 0; i < n; ++i) value2 += helper[i] * p[i];   /* :378-379 */
    alpha = rxr / value2;                                         /* :385-386 */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      x[i] = x[i] + alpha * p[i];                                 /* :390 */
      rnext[i] = rnext[i] - alpha * helper[i];                    /* :392-393 */
    }
    if (isnan(rxr) || sqrt(rxr) <= tol) done = 1;                 /* :400-403 */
#pragma omp parallel for schedule(static) reduction(+ : value3)
    for (int64_t i = 0; i < n; ++i) value3 += rnext[i] * rnext[i];/* :406-407 */
    beta = value3 / rxr;                                          /* :414 */
    rxr = value3;                                                 /* :415 */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) p[i] = rnext[i] + beta * p[i];/* :418 */
    ++bodies;
    if (max_iter >= 0 && bodies >= max_iter) break;
  } while ((uint64_t)(counter++) < (uint64_t)n && !done);        /* :436 */
  if (res) {
    res->iterations = bodies;
    res->rxr = rxr;
    res->stopped_by_tol = done;
  }
  free(helper); free(rnext); free(p);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* The engine's dot model (round 6): the same iteration as                  */
/* orc_cg_solve_omp, every dot a double-length sum                          */
/* ------------------------------------------------------------------------ */

/* The reference's dots (VectorOperations.hpp:287-309, CG.hpp:378-379,
 * 406-407) are sycl::reduction sums in an order AdaptiveCpp chooses (parity
 * unpinned, cg_oracle.h). The GPU engine sums them as unevaluated pairs
 * hi + lo (TwoSum on every addition) and rounds once, so its value does not
 * depend on how rows are split. Here the same model on the CPU: each OpenMP
 * thread sums its static chunk as a pair, the pairs are combined in thread
 * order, one rounding. Both are the exact sum of the rounded products to
 * within ~n u^2 of the sum of their magnitudes, so their rounded values agree
 * except when the exact sum lies that close to a rounding boundary; every
 * other value of the iteration is rounded as in orc_cg_solve. This is a
 * checker for the engine's arithmetic (x bit for bit), not a claim about the
 * reference's summation order. */
typedef struct { double hi, lo; } orc_dd;
static inline void dd_add(orc_dd *s, double x) {
  const double t = s->hi + x;
  const double z = t - s->hi;
  s->lo += (s->hi - (t - z)) + (x - z);
  s->hi = t;
}
#define ORC_MAX_THREADS 256
static double dot_dd(int64_t n, const double *a, const double *b) {
  orc_dd part[ORC_MAX_THREADS];
  int nt = 1;
#pragma omp parallel
  {
    const int t = omp_get_thread_num();
#pragma omp single
    nt = omp_get_num_threads();
    orc_dd s = {0.0, 0.0};
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) dd_add(&s, a[i] * b[i]);
    if (t < ORC_MAX_THREADS) part[t] = s;
  }
  orc_dd s = part[0];
  for (int t = 1; t < nt && t < ORC_MAX_THREADS; ++t) {
    dd_add(&s, part[t].hi);
    s.lo += part[t].lo;
  }
  return s.hi + s.lo;
}

int orc_cg_solve_dd(int64_t n, const int *rowptr, const int *col, const double *val,
                    const double *b, double *x, int has_x0, double tol, int64_t max_iter,
                    int threads, orc_cg_result *res) {
  if (threads > ORC_MAX_THREADS) threads = ORC_MAX_THREADS;
  omp_set_num_threads(threads > 0 ? threads : 1);
  double *helper = (double *)malloc((size_t)n * sizeof(double));
  double *rnext = (double *)malloc((size_t)n * sizeof(double));
  double *p = (double *)malloc((size_t)n * sizeof(double));
  if (!helper || !rnext || !p) { free(helper); free(rnext); free(p); return 3; }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {                               /* :324-332 */
    if (!has_x0) x[i] = 0;
  }
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * x[col[j]];
    rnext[i] = b[i] - s;
    p[i] = rnext[i];
  }
  double rxr = dot_dd(n, rnext, rnext);                           /* :341 */
  if (res) res->rxr0 = rxr;
  int64_t counter = 0, bodies = 0;
  int done = 0;
  do {
    double alpha, beta;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {                             /* :374-375 */
      double s = 0;
      for (int j = rowptr[i]; j < rowptr[i + 1]; ++j) s += val[j] * p[col[j]];
      helper[i] = s;
    }
    const double value2 = dot_dd(n, helper, p);                   /* :378-379 */
    alpha = rxr / value2;                                         /* :385-386 */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      x[i] = x[i] + alpha * p[i];                                 /* :390 */
      rnext[i] = rnext[i] - alpha * helper[i];                    /* :392-393 */
    }
    if (isnan(rxr) || sqrt(rxr) <= tol) done = 1;                 /* :400-403 */
    const double value3 = dot_dd(n, rnext, rnext);                /* :406-407 */
    beta = value3 / rxr;                                          /* :414 */
    rxr = value3;                                                 /* :415 */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) p[i] = rnext[i] + beta * p[i];/* :418 */
    ++bodies;
    if (max_iter >= 0 && bodies >= max_iter) break;
  } while ((uint64_t)(counter++) < (uint64_t)n && !done);        /* :436 */
  if (res) {
    res->iterations = bodies;
    res->rxr = rxr;
    res->stopped_by_tol = done;
  }
  free(helper); free(rnext); free(p);
  return 0;
}
