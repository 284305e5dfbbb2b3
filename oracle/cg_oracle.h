/*
 * cg_oracle.h — CPU restatement of the reference CG hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker or the
 * reported CPU baseline. The product path (libcgx.so) never links or calls it.
 *
 * Parity status:
 *   - Matrix-Market loader: pinned bit-exact against oracle/_ref/libmmref.so,
 *     which is the reference's own test/mm_reader.cpp compiled unmodified
 *     from /root/reference (oracle/Makefile).
 *   - CG solve / accuracy(): the reference (src/CG.hpp) needs AdaptiveCpp,
 *     which is absent, so it cannot be built here. This restatement is pinned
 *     to the reference outputs recorded in SURVEY.md §6/§8(c) (iteration
 *     counts 103 / 972 / 479 / 152 / 76 / 686 and accuracy() 2.136e-29 on
 *     128^2) and to an independent direct solve (scipy). Beyond those
 *     recorded values, CG parity is "parity unpinned".
 *
 * Arithmetic follows the reference statement by statement: products are
 * rounded before they are added (no FMA contraction; build with
 * -ffp-contract=off), row sums run in ascending column order starting from 0
 * (VectorOperations.hpp:456-461, CG.hpp:325-329), reductions accumulate into
 * the existing value in index order (VectorOperations.hpp:300-305, Q4).
 */
#ifndef CG_ORACLE_H
#define CG_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Matrix-Market loader (test/mm_reader.cpp:45-171) ------------------ */
/* Returns 0 on success; arrays are malloc'ed and owned by the caller
 * (release with orc_free). n = rowptr length - 1, as Tester.cpp:27 derives it. */
int orc_read_mtx(const char *path, int64_t *n_out, int64_t *nnz_out,
                 int **rowptr, int **col, double **val);
void orc_free(void *p);

/* ---- synthetic Dirichlet Poisson CSR --------------------- */
/* dim = 2 (5-point, nz ignored) or 3 (7-point); lexicographic order, x fastest,
 * columns ascending per row. Caller allocates rowptr[n+1], col[nnz], val[nnz]. */
int64_t orc_poisson_nnz(int dim, int nx, int ny, int nz);
void orc_poisson(int dim, int nx, int ny, int nz, int *rowptr, int *col,
                 double *val);
/* Write the lower triangle as a `symmetric` .mtx with one comment line
 * (mm_reader quirks Q1/Q2). Returns 0 on success. */
int orc_write_mtx_lower(const char *path, int64_t n, const int *rowptr,
                        const int *col, const double *val);

/* ---- VectorOperations kernels (src/VectorOperations.hpp) ---------------- */
void orc_spmv(int64_t n, const int *rowptr, const int *col, const double *val,
              const double *x, double *y);                 /* :438-466 */
double orc_dot_acc(int64_t n, const double *x, const double *y,
                   double init);                           /* :287-309 */
double orc_norm_acc(int64_t n, const double *x, double init); /* :311-331 */
void orc_sapbx(int64_t n, const double *x, const double *y, double b,
               double *res);                               /* :410-428 */
void orc_sambx(int64_t n, const double *x, const double *y, double b,
               double *res);                               /* :380-397 */
void orc_saxpby(int64_t n, const double *x, const double *y, double a,
                double b, double *res);                    /* :349-367 */

/* ---- CG::solve (src/CG.hpp:255-454) ------------------------------------- */
typedef struct {
  int64_t iterations;  /* loop bodies executed (CG.hpp:359-436)            */
  double rxr;          /* final rxr scalar (CG.hpp:437-438)                */
  double rxr0;         /* r0.r0 after the init kernel (CG.hpp:341)         */
  int stopped_by_tol;  /* is_done was set (CG.hpp:401-402)                 */
} orc_cg_result;

/* x is in/out: when has_x0 == 0 it is zero-filled first (CG.hpp:291-297).
 * max_iter < 0 keeps the reference cap (counter++ < N, i.e. N+1 bodies);
 * max_iter >= 0 additionally caps the bodies (extension for benchmarking). */
int orc_cg_solve(int64_t n, const int *rowptr, const int *col,
                 const double *val, const double *b, double *x, int has_x0,
                 double tol, int64_t max_iter, orc_cg_result *res);

/* CG::accuracy (CG.hpp:463-515): |sum (b-Ax)^2 / sum x^2| */
double orc_accuracy(int64_t n, const int *rowptr, const int *col,
                    const double *val, const double *b, const double *x);

/* CPU baseline: the same per-iteration command sequence as CG.hpp:359-436,
 * with every parallel_for run as an OpenMP loop on `threads` threads (the
 * AdaptiveCpp OpenMP backend's execution model). Runs exactly `iters` loop
 * bodies, no stop test. Returns wall seconds of the iteration loop only.
 * orc_cg_timed_omp runs `warmup` untimed bodies before the `iters` timed
 * ones (the SURVEY 8(d) protocol: K = 500 after 20 warm-up). */
double orc_cg_timed_omp(int64_t n, const int *rowptr, const int *col, const double *val,
                        const double *b, double *x, int64_t warmup, int64_t iters,
                        int threads);
double orc_cg_fixed_iters_omp(int64_t n, const int *rowptr, const int *col,
                              const double *val, const double *b, double *x,
                              int64_t iters, int threads);

/* orc_cg_solve with OpenMP loops and OpenMP-reduction dots: the full-size
 * parity oracle (16.8 M rows). Only the dots' summation order differs from
 * orc_cg_solve. */
int orc_cg_solve_omp(int64_t n, const int *rowptr, const int *col,
                     const double *val, const double *b, double *x, int has_x0,
                     double tol, int64_t max_iter, int threads,
                     orc_cg_result *res);

/* orc_cg_solve_omp with every dot a double-length sum (per-thread TwoSum
 * pairs combined in thread order, one rounding): the GPU engine's dot model
 * since round 6, whose value does not depend on how rows are split. A
 * checker for the engine's arithmetic at full size (x bit for bit), not a
 * statement about the reference's (unpinned) summation order. */
int orc_cg_solve_dd(int64_t n, const int *rowptr, const int *col, const double *val,
                    const double *b, double *x, int has_x0, double tol, int64_t max_iter,
                    int threads, orc_cg_result *res);

#ifdef __cplusplus
}
#endif
#endif
