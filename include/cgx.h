/*
 * cgx.h — C ABI of libcgx.so, the MI355X (gfx950) conjugate-gradient engine.
 *
 * The reference (XeniaHerr/ConjugateGradient) has no FFI: its boundary is the
 * header-only C++ template API in src/CG.hpp, src/VectorOperations.hpp and
 * src/LinearAlgebraTypes.hpp. Our drop-in copies of those
 * headers (include/CG.hpp, include/VectorOperations.hpp,
 * include/LinearAlgebraTypes.hpp) are thin C++ over the entry points below;
 * each entry point names the reference interface it replaces.
 *
 * Conventions
 *   - Every function returns int: 0 = CGX_OK, otherwise an error code; the
 *     message is in cgx_last_error() (thread-local).
 *   - Pointers named d_* are device pointers (hipMalloc'ed, e.g. by cgx_alloc);
 *     h_* are host pointers. Sizes are element counts unless named *_bytes.
 *   - dtype: CGX_F64 or CGX_F32 (the reference's DT template parameter).
 *   - All kernels are asynchronous on the context's stream (the SYCL queue's
 *     role, CG.hpp:590); functions documented as "blocking" drain it, as the
 *     reference's executeQueue() does (CG.hpp:561-578).
 *   - Indices are int32 (Matrix<DT> stores int columns/rows,
 *     LinearAlgebraTypes.hpp:620-622).
 */
#ifndef CGX_H
#define CGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { CGX_OK = 0, CGX_EINVAL = 1, CGX_EHIP = 2, CGX_ENOMEM = 3, CGX_ESTATE = 4,
       CGX_ENCCL = 5, CGX_EUNSUPPORTED = 6 };
enum { CGX_F64 = 0, CGX_F32 = 1 };

typedef struct cgx_ctx cgx_ctx; /* device + stream (+ optional RCCL comm)      */
typedef struct cgx_csr cgx_csr; /* CSR matrix view + SpMV row-block schedule  */
typedef struct cgx_cg cgx_cg;   /* fused CG solver state                      */

/* ---- errors / version ---------------------------------------------------- */
const char *cgx_last_error(void);
const char *cgx_version(void);
/* Number of visible HIP devices (0 when none; never fails on a CPU host). */
int cgx_device_count(int *count);

/* ---- context: replaces the sycl::queue (CG.hpp:61,70-77,590) -------------- */
int cgx_create(int device, cgx_ctx **out);          /* CG::createCG :70-77   */
int cgx_destroy(cgx_ctx *ctx);
int cgx_sync(cgx_ctx *ctx);                          /* executeQueue :561-578 */
int cgx_get_stream(cgx_ctx *ctx, void **hip_stream);
int cgx_get_device(cgx_ctx *ctx, int *device);
/* the device's max_work_group_size (VectorOperations.hpp:478-487 queries it
 * through sycl::info::device::max_work_group_size) */
int cgx_max_work_group_size(cgx_ctx *ctx, int *size);

/* ---- memory: replaces sycl::malloc_device/free/copy/fill ------------------
 * (LinearAlgebraTypes.hpp:43-49 Asycl_deleter, :109-119 Matrix::init,
 *  :160-183 Vector::init_empty/init, :217-224 Scalar::init) */
int cgx_alloc(cgx_ctx *ctx, size_t bytes, void **d_out);
int cgx_free(cgx_ctx *ctx, void *d_ptr);
int cgx_h2d(cgx_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);     /* blocking */
int cgx_d2h(cgx_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);     /* blocking */
int cgx_d2d(cgx_ctx *ctx, void *d_dst, const void *d_src, size_t bytes);     /* async    */
int cgx_h2d_async(cgx_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
int cgx_fill(cgx_ctx *ctx, int dtype, void *d_ptr, double value, size_t n);  /* async    */

/* ---- CSR matrix (Matrix<DT>, LinearAlgebraTypes.hpp:57-132) ---------------
 * The device arrays stay owned by the caller (the Matrix object's
 * shared_ptrs); cgx_csr only adds the SpMV schedule. h_rowptr may be NULL (it
 * is then read back from the device). */
int cgx_csr_create(cgx_ctx *ctx, int64_t n, int64_t nnz, const int *d_rowptr,
                   const int *d_col, const void *d_val, int dtype,
                   const int *h_rowptr, cgx_csr **out);
int cgx_csr_destroy(cgx_csr *csr);
int cgx_csr_info(cgx_csr *csr, int64_t *n, int64_t *nnz, int64_t *row_blocks,
                 int *max_row_nnz);
/* Rebuild the SpMV schedule for row blocks of `tile` entries (2048, the
 * default, or 1024 with at most 128 rows). Blocking. */
int cgx_csr_set_tile(cgx_csr *csr, int tile);
/* CSR-stream's row-block visit order. A matrix from a 3-D grid gathers p one
 * plane (D rows) away from every row; walking chunks of `chunk_rows` rows of a
 * plane through the planes of each XCD's eighth keeps those p lines in the
 * XCD's L2. chunk_rows: 0 the natural order, -1 automatic (an order only
 * where a dominant offset D makes two planes of stream overflow half an L2),
 * > 0 that chunk (CGX_EINVAL without a dominant offset). The result is the
 * same for any order; only the p.Ap partials group differently. Blocking.
 * Replaces nothing in the reference: a schedule of VectorOperations.hpp:
 * 438-466's SpMV. */
int cgx_csr_set_block_order(cgx_csr *csr, int chunk_rows);
/* The order in use: the plane offset D and the chunk rows (0 / 0: natural). */
int cgx_csr_block_order_info(cgx_csr *csr, int *D, int *chunk_rows);
/* SpMV variant the matrix's launches use: the one cgx_csr_create picked by
 * timing the candidate kernels on the device ($CGX_SPMV_VARIANT or
 * cgx_csr_set_variant override), resolved against the matrix's layout
 * (e.g. 6146 = SELL, 2 rows per lane, non-temporal loads). */
int cgx_csr_variant(cgx_csr *csr, int *variant);
/* Force the SpMV variant of this matrix (0: size heuristic). Variants with
 * bit 2048 use the SELL-64 copy cgx_csr_create builds for matrices whose
 * slices of 64 rows have at most 64 distinct (col - row) offsets; they fail
 * with CGX_EUNSUPPORTED when the matrix has none (or it was freed because
 * the autotune chose a CSR-stream variant). */
int cgx_csr_set_variant(cgx_csr *csr, int variant);
/* Rebuild the SELL copy: 1 or 2 = dictionary SELL with 1 or 2 rows per
 * lane (slices of 64 or 128 rows), 3 = SELL-P (slices of 128 rows, one
 * offset pattern per slice, one slot mask per row), 0 = drop it. A matrix
 * that does not qualify ends without one. Blocking. */
int cgx_csr_set_sell(cgx_csr *csr, int rows_per_lane);
/* The matrix's SELL layout (0 none, 1 / 2 dictionary SELL with that many
 * rows per lane, 3 SELL-P) and its padded entry count. */
int cgx_csr_sell_info(cgx_csr *csr, int *has_sell, int64_t *padded_entries);
/* The SELL walk's slice visit order: 1 when the slices are walked in
 * XCD-local chunks of z-planes (automatic where planes span >= 1,024
 * slices), 2 when a partitioned matrix's interior slice
 * list is, 0 for the natural order. */
int cgx_csr_visit_order(cgx_csr *csr, int *ordered);
/* Distinct values of the matrix's SELL-P value codes (variant bit 32768:
 * one code byte per slot into a dictionary of at most 255 values, built by
 * cgx_csr_create when the SELL-P copy exists and the matrix has that few
 * distinct values; $CGX_VALUE_CODES=0 disables it), 0 when it has none. */
int cgx_csr_value_codes(cgx_csr *csr, int *n_values);
/* Value-code templates (variant bit 8388608): the number of distinct 4-bit
 * code chunks stored once and read from LDS, and the slices that use one
 * (0 / 0: none). */
int cgx_csr_templates(cgx_csr *csr, int *n_templates, int64_t *slices);
/* The lean stencil walk (variant bit 33554432, kept by the autotune where it
 * wins or requested with cgx_csr_set_variant): slices whose pattern is a
 * subset of one stencil's {-D, -a, -1, 0, +1, +a, +D} and whose template
 * chunk holds one value per slot, summed from per-class values with no
 * per-row stream. *classes: distinct (template, pattern) classes, *slices:
 * slices that run it, *grid: its launch's workgroups, *D / *a: the stencil's
 * offsets, *chunked: 1 when its waves walk chunks of a plane through the
 * planes (planes wider than a grid step; all 0 when the matrix has none
 * built). Replaces nothing in the reference: a format of
 * VectorOperations.hpp:438-466's SpMV. */
int cgx_csr_lean_info(cgx_csr *csr, int *classes, int64_t *slices, int *grid, int *D, int *a,
                      int *chunked);
/* The SpMV autotune's record of this matrix (cgx_csr_create /
 * cgx_csr_create_dist): every form it timed, how it was timed and its median
 * µs per launch over the interleaved rounds; *count = the record's length
 * (0 when a variant was forced or the matrix is small enough for the size
 * rule). Up to `cap` entries are written. A form displaces the preferred
 * (more specialised) one only when at least 3% faster. Replaces nothing in
 * the reference (its SpMV has one form, VectorOperations.hpp:438-466). */
#define CGX_TUNE_DOT 0          /* k_spmv_dot over the whole matrix */
#define CGX_TUNE_DOT_INTERIOR 1 /* k_spmv_dot over a split matrix's interior slices */
#define CGX_TUNE_FD 2           /* k_spmv_fd (mode 4's SpMV; 2-D plane march) */
#define CGX_TUNE_LEAN 3         /* the lean walk over the whole matrix */
#define CGX_TUNE_LEAN_INTERIOR 4 /* the lean walk over a split matrix's interior */
#define CGX_TUNE_LEAN_TEAM 5     /* mode 4's fused walk, team form (cgx_csr_set_lean_team) */
#define CGX_TUNE_INCUMBENT 6     /* the pick before the lean walk's rounds, re-timed in them */
#define CGX_TUNE_BOUNDARY 7      /* a split matrix's boundary rows (CSR-stream launch), added
                                    to its interior forms' times before the pick */
int cgx_csr_autotune_record(cgx_csr *csr, int *variants, int *kinds, float *us, int cap,
                            int *count);
/* The setup cost of cgx_csr_create / cgx_csr_create_dist by phase, wall
 * milliseconds (*count = 6; up to `cap` written): [0] row-block schedule (and
 * the halo plan of a partitioned matrix), [1] SELL plan and pack, [2] value
 * codes and templates, [3] interior / boundary split, [4] SpMV autotune
 * (lean layouts included), [5] the rest. Replaces nothing in the reference
 * (Matrix::init only uploads, LinearAlgebraTypes.hpp:101-121). */
int cgx_csr_setup_times(cgx_csr *csr, double *ms, int cap, int *count);
/* Mode 4's fused lean walk (k_spmv_fd_lean) in its team form: 1,024-thread
 * workgroups whose 16 waves share their slices' formed p_k neighbour pairs
 * through LDS instead of gathering r and p_{k-1} for them.
 * on = 1 selects it (grid / 4 workgroups), 0 the 4-wave form; the plain
 * SpMV always runs the 4-wave walk. CGX_EUNSUPPORTED without an f64
 * whole-matrix lean layout whose grid is a multiple of 32. The autotune
 * decides it at creation. Replaces nothing in the reference
 * (VectorOperations.hpp:438-466 has one SpMV form). */
int cgx_csr_set_lean_team(cgx_csr *csr, int on);
int cgx_csr_lean_team(cgx_csr *csr, int *on);
/* The plane-march plan of the matrix's SELL-P copy (variant bit 2097152):
 * *stride = slices (of 128 rows) between a slice and its +-D neighbour
 * (0: the dominant slice pattern is not a 7-point / 5-point stencil with D
 * a multiple of 128 rows, and the bit is ignored), *offset_a = the 3-D
 * form's +-a offset (0: 2-D form), *run_planes = planes per run (0: chosen
 * per launch to fill the grid). */
int cgx_csr_march_info(cgx_csr *csr, int *stride, int *offset_a, int *run_planes);
/* Bytes of the matrix stream one SpMV launch in the matrix's current
 * variant reads (values, indices / codes / masks, slice descriptors;
 * vectors excluded): the format's algorithmic bytes, next to CSR's
 * 12 nnz + 4 (n + 1) in fp64. */
int cgx_csr_stream_bytes(cgx_csr *csr, int64_t *bytes);

/* ---- VectorOperations<DT> (src/VectorOperations.hpp) ----------------------
 * Scalars are DEVICE pointers, as in the reference (Scalar<DT>::ptr()). */
/* y = A x over all rows; `count` must equal A.N() (spmv :438-466, assert :444) */
int cgx_spmv(cgx_ctx *ctx, cgx_csr *A, const void *d_x, void *d_y, int64_t count);
/* *d_res += x.y  (dot_product_trivial :287-309: accumulates, Q4) */
int cgx_dot_acc(cgx_ctx *ctx, int dtype, int64_t n, const void *d_x,
                const void *d_y, void *d_res);
/* *d_res += x.x  (norm :311-331; sum of squares, no sqrt) */
int cgx_norm_acc(cgx_ctx *ctx, int dtype, int64_t n, const void *d_x, void *d_res);
/* res = x + (*d_b) y (sapbx :410-428), res = x - (*d_b) y (sambx :380-397),
 * res = (*d_a) x + (*d_b) y (saxpby :349-367). res may alias x or y. */
int cgx_sapbx(cgx_ctx *ctx, int dtype, int64_t n, const void *d_x,
              const void *d_y, const void *d_b, void *d_res);
int cgx_sambx(cgx_ctx *ctx, int dtype, int64_t n, const void *d_x,
              const void *d_y, const void *d_b, void *d_res);
int cgx_saxpby(cgx_ctx *ctx, int dtype, int64_t n, const void *d_x,
               const void *d_y, const void *d_a, const void *d_b, void *d_res);
/* Device scalar helper: *d_out = *d_num / *d_den (CG.hpp:385-386, :414). */
int cgx_scalar_div(cgx_ctx *ctx, int dtype, const void *d_num, const void *d_den,
                   void *d_out);

/* ---- fused CG: CG<DT>::solve (CG.hpp:255-454) -----------------------------
 * Per iteration three kernels (SpMV+p.Ap, r-update+r.r, x/p-update), device-
 * resident scalars and stop flag; the host polls every few iterations instead
 * of draining the queue every iteration (CG.hpp:425). Iteration semantics are
 * the reference's (Q5): the stop test uses the r.r at the START of the body
 * after the body's x update, NaN stops, at most A.N()+1 bodies. */
int cgx_cg_create(cgx_ctx *ctx, cgx_csr *A, cgx_cg **out);
int cgx_cg_destroy(cgx_cg *cg);
/* Blocking. d_x holds the initial guess (zero it for the reference default)
 * and receives the result. max_bodies < 0 keeps the reference cap N+1;
 * otherwise the cap is min(N+1, max_bodies). */
int cgx_cg_solve(cgx_cg *cg, const void *d_b, void *d_x, double tol,
                 int64_t max_bodies, int64_t *bodies_out, double *rxr_out);
/* Split form used by benchmarks: init (r = b - A x, p = r, rxr = r.r) then
 * run up to `bodies` more loop bodies (stops early on the stop rule). */
int cgx_cg_begin(cgx_cg *cg, const void *d_b, void *d_x, double tol,
                 int64_t max_bodies);
int cgx_cg_run(cgx_cg *cg, int64_t bodies, int64_t *bodies_total, int *stopped);
/* Capture, ahead of time, the hipGraphs a following cgx_cg_run(cg, bodies)
 * replays (chunks of the poll interval from the current slot; a run builds
 * only full chunks itself and launches a shorter tail eagerly). Blocking
 * host work, no kernel runs. Benchmarks call it before a timed run. */
int cgx_cg_prepare(cgx_cg *cg, int64_t bodies);
/* r.r after the last body run so far (the value the reference reads back
 * after its loop, CG.hpp:437-440); blocking. */
int cgx_cg_rxr(cgx_cg *cg, double *rxr);
/* Per-kernel device time, accumulated with HIP events on the solver stream
 * while enabled: avg_ms[0..3] = init, spmv_dot, update_r, update_xp;
 * calls[0..3] = launches timed. */
int cgx_cg_set_kernel_timing(cgx_cg *cg, int enable);
int cgx_cg_kernel_times(cgx_cg *cg, double *avg_ms, int64_t *calls);
/* The same kernels' execution times: event pairs each kernel's dispatch
 * records itself (hipExtLaunchKernel), so without the dispatch latency the
 * pairs of cgx_cg_kernel_times include; the durations rocprofv3 reports.
 * calls[i] = 0 where a launch did not record them. */
int cgx_cg_kernel_exec_times(cgx_cg *cg, double *avg_ms, int64_t *calls);
/* Tuning knobs (0 = default): iterations per host poll; use hipGraph replay. */
int cgx_cg_config(cgx_cg *cg, int poll_every, int use_graph);
/* Iteration structure (before cgx_cg_begin): 0 auto (4 for the 2-D plane
 * march, cache-resident stencil matrices, lean walks of >= 32 M rows and
 * partitioned lean interiors of <= 4 M rows, else 3; the default), 1
 * three kernels
 * (SpMV+p.Ap, r-update+r.r, x/p-update), 2 fused (single device only): two
 * kernels, the x/p update folded into the next iteration's SpMV (p_j =
 * r_j + beta p_old_j computed in the gather), 8 bytes/row less traffic but
 * twice the gathers; 3 three kernels with the x update deferred: p cycles
 * through four buffers and x += a0 p0 + ... + a3 p3 (in order) runs once
 * per four bodies and at the end of each cgx_cg_run (34 N instead of 40 N
 * bytes per body for the x/p update); 4 fused with deferred x (f64,
 * production SpMV formats): two kernels per body, p_k = r +
 * beta p_{k-1} computed where the SpMV reads it and stored once into the
 * p ring, update_r with the stop rule, x from the four p buffers in slot 3
 * (72 N + matrix bytes per body against 78 N in mode 3); on a partitioned
 * matrix it needs the device peer transport and the lean interior walk
 * (three launches: interior walk with the push of the formed p_k, boundary
 * rows, update_r with both all-reduces; x bit-identical to mode 3; auto at
 * <= 4 M rows per rank); 5 persistent body
 * (single device, f64; register forms up to 1024 rows per CU, the streamed form
 * up to 8 x 1024 x min(256, CUs) rows): one launch runs a whole chunk of
 * bodies, each with two grid-wide exchanges of the dot partials instead of
 * three kernel boundaries; Ap bit-identical, the dots summed in another
 * order (x equal to rounding). $CGX_COOP_R picks its rows per thread,
 * $CGX_COOP_STREAM=1 / 0 always / never the streamed form.
 * Mode 6 (round 6; single device, the lean stencil walk): mode 3's body with
 * no Ap vector — kernel 1 walks A p keeping only p.Ap, kernel 2 walks A p
 * again and updates r in its epilogue (8 N bytes written and read less).
 * Mode 7 (single device, f64, a 3-D stencil whose lean layout takes the tile
 * walk): mode 4's body with no Ap vector — kernel 1 forms p_k into the p ring
 * and keeps p.Ap, kernel 2 walks A p_k again, updates r and runs the stop
 * rule, slot 3 adds the x flush launch (60 N + 2 x matrix bytes per body);
 * never auto (slower than mode 6 at 256^3).
 * The dots are double-length sums (round 6), so modes 1, 3, 4, 6 and 7 give
 * bit-identical x whatever their grids. */
int cgx_cg_set_mode(cgx_cg *cg, int mode);
/* mode 5's launch shape: rows per thread, threads per workgroup (1024),
 * workgroups, and the form: 0 the register form (drained write-through
 * stores), 2 the streamed form (the matrix read every body, entries staged
 * through LDS; $CGX_COOP_STREAM=1 forces it, $CGX_COOP_R its rows per
 * thread) */
int cgx_cg_coop_shape(cgx_cg *cg, int *rows_per_thread, int *threads, int *workgroups,
                      int *form);
/* diagnostics: with $CGX_COOP_TRACE=1 set before mode 5 is chosen, the
 * wall-clock stamps (100 MHz) of the last launch: [workgroup][body 8..15]
 * [phase 0..7] (0 body start, 1 SpMV done, 2 p.Ap partial ready, 3 p.Ap
 * exchanged, 4 r.r partial ready, 5 next gathers done, 6 r.r exchanged) */
int cgx_cg_coop_trace(cgx_cg *cg, uint64_t *host, int64_t words);
/* the iteration structure in effect (1-5; auto resolved) */
int cgx_cg_get_mode(cgx_cg *cg, int *mode);
/* mode 4's fused SpMV grid and the SpMV's: where they are equal mode 4 is
 * bit-identical to mode 1, else equal to rounding (one dot's sum order) */
int cgx_csr_fd_grid(cgx_csr *A, int *fd_grid, int *spmv_grid);

/* CG::accuracy (CG.hpp:463-515): blocking; |sum (b-Ax)^2 / sum x^2|. */
int cgx_accuracy(cgx_ctx *ctx, cgx_csr *A, const void *d_b, const void *d_x,
                 double *out);

/* ---- synthetic inputs ---------------------------------------
 * Dirichlet Poisson CSR generated on the device (dim 2: 5-point, dim 3:
 * 7-point; lexicographic, x fastest; columns ascending; diag 2*dim, off -1).
 * Rows [row_begin, row_end) of the global matrix; column indices global. */
int64_t cgx_poisson_nnz(int dim, int nx, int ny, int nz, int64_t row_begin,
                        int64_t row_end);
int cgx_poisson_fill(cgx_ctx *ctx, int dtype, int dim, int nx, int ny, int nz,
                     int64_t row_begin, int64_t row_end, int *d_rowptr,
                     int *d_col, void *d_val);
/* b_i = i + 1 + offset (Tester.cpp:29-30) */
int cgx_iota(cgx_ctx *ctx, int dtype, void *d_b, int64_t n, double offset);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI --------
 * Rows are partitioned in contiguous blocks; p's ghost entries are exchanged
 * each iteration with ncclSend/ncclRecv and the two dots are all-reduced. */
int cgx_nccl_unique_id(char *id_out, size_t len);            /* len >= 128 */
int cgx_dist_init(cgx_ctx *ctx, int rank, int world, const char *id, size_t len);
int cgx_dist_rank(cgx_ctx *ctx, int *rank, int *world);
/* Host-staged transport: the same partitioned solver with every collective
 * done by caller callbacks on HOST buffers (return 0 on success). Used to run
 * several ranks on one GPU (RCCL refuses that) in tests; slow by design.
 *   allgather: recv[world * bytes] <- every rank's `bytes` from send
 *   allreduce: vals[count] <- element-wise sum over ranks (in place)
 *   exchange : for i < n, send[i] (send_bytes[i]) to peers[i] and receive
 *              recv_bytes[i] from peers[i] into recv[i] */
typedef int (*cgx_allgather_fn)(void *user, const void *send, size_t bytes, void *recv);
typedef int (*cgx_allreduce_fn)(void *user, double *vals, int count);
typedef int (*cgx_exchange_fn)(void *user, int n, const int *peers, const void *const *send,
                               const size_t *send_bytes, void *const *recv,
                               const size_t *recv_bytes);
int cgx_dist_init_host(cgx_ctx *ctx, int rank, int world, cgx_allgather_fn allgather,
                       cgx_allreduce_fn allreduce, cgx_exchange_fn exchange, void *user);
/* Host transport, asynchronous halo: the per-iteration exchange runs on the
 * context's comm stream (D2H, `exchange` as a host function, H2D, an event the
 * solver stream waits on), so a split SpMV's interior slices overlap it — the
 * stream/event ordering of the RCCL exchange. The callback then runs on the
 * HIP runtime's callback thread. Call before cgx_csr_create_dist. */
int cgx_dist_host_async(cgx_ctx *ctx, int on);
/* exchanges a partitioned matrix has posted on the comm stream (host transport) */
int cgx_csr_halo_async_calls(cgx_csr *A, int64_t *calls);
/* Local block of a globally row-partitioned matrix: rows
 * [row_begin, row_begin + n_local) with GLOBAL column indices (device arrays,
 * caller-owned, d_col is rewritten in place to local/ghost numbering).
 * n_global is the global dimension. Collective over the communicator. */
int cgx_csr_create_dist(cgx_ctx *ctx, int64_t n_global, int64_t row_begin,
                        int64_t n_local, int64_t nnz_local, const int *d_rowptr,
                        int *d_col, const void *d_val, int dtype, cgx_csr **out);
/* ghost entries this rank receives per iteration */
int cgx_csr_halo_info(cgx_csr *csr, int64_t *ghosts, int *neighbours);
/* Reduce a host double over ranks (sum); utility for tests. */
/* Slices of a partitioned SELL matrix without / with ghost columns: the
 * SpMV runs the interior ones while the halo exchange is in flight. Both 0
 * when the matrix is not split (no SELL copy, or no ghosts). */
int cgx_csr_split_info(cgx_csr *csr, int *interior_slices, int *boundary_slices);
int cgx_dist_allreduce_sum(cgx_ctx *ctx, double *value);
/* Device peer transport over xGMI for a partitioned matrix (collective):
 * every rank maps the other ranks' mailboxes and its neighbours' halo
 * landing buffers (hipIpc, uncached device memory), and the solver's halo
 * exchange and dot all-reduces then run as kernels that store straight into
 * peer memory — no host-enqueued collective per iteration, so the
 * partitioned iteration is graph-captured like the single-GPU one. The
 * transport is checked against the setup transport (RCCL or host) before it
 * is used: *enabled = 1 when every rank passed, 0 when the solver keeps the
 * setup transport (not an error; cgx_last_error() says why). Call before
 * cgx_cg_create. $CGX_PEER=0 declines; $CGX_PEER_TIMEOUT_S bounds every
 * device-side wait (default 10 s; a timeout stops the solve with an error). */
int cgx_dist_peer_enable(cgx_csr *csr, int *enabled);
int cgx_dist_peer_info(cgx_csr *csr, int *enabled);
/* The peer transport's iteration form: *colocated = ranks whose device is
 * this rank's (0 when the transport is off), *one_waiter = 1 when at most one
 * workgroup per rank waits on another rank at any time (a one-workgroup wait
 * launch before the boundary rows, one-workgroup all-reduces before the
 * kernels that consume the dots). Taken on every rank when any two ranks
 * share a GPU, where whole waiting grids could hold the CUs a peer needs;
 * otherwise the fused form (the waits inside the consuming kernels, fewer
 * launches). Same values either way. $CGX_PEER_ONE_WAITER=0/1 forces it. */
int cgx_dist_peer_form(cgx_csr *csr, int *colocated, int *one_waiter);

/* ---- host-only helpers (no device needed; the CPU test-suite drives them) --
 * Halo plan of rows [row_begin, row_begin + n_local) whose global column
 * indices are `col`: sorted distinct off-block columns (*ghosts, malloc'ed,
 * release with cgx_free_host) and per-rank receive counts (recv_cnt[world]);
 * begins/counts give every rank's row range (contiguous, ordered by rank). */
int cgx_plan_ghosts(int64_t n_local, int64_t row_begin, int64_t nnz, const int *col,
                    int world, const int64_t *begins, const int64_t *counts,
                    int64_t *n_ghost, int64_t **ghosts, int64_t *recv_cnt);
/* Global -> local column numbering (own rows, then ghosts in list order). */
int cgx_plan_remap(int64_t n_local, int64_t row_begin, int64_t nnz, int *col,
                   int64_t n_ghost, const int64_t *ghosts);
/* The SpMV row-block schedule cgx_csr_create builds (for tests). */
int cgx_row_blocks(const int *h_rowptr, int64_t n, int64_t *nrb, int **rb,
                   int *max_row_nnz);
void cgx_free_host(void *p);
/* Host-only: the SELL layout (rows_per_lane 1 or 2) cgx_csr_create would
 * build for a host CSR (DESIGN.md §SpMV formats). *nsl = 0 when the matrix
 * does not qualify.
 * slices[4 q .. 4 q + 3] = {first value slot, first index word, first
 * dictionary entry, width} of slice q; dict[ndict] = the offset pool (col -
 * row), idx[nidx] = 8 one-byte dictionary indices per word (0xff: padding);
 * value_slots = length of the value array. Release with cgx_free_host. */
/* ---- Matrix-Market ingest / emit (test/mm_reader.cpp read_file) ---------
 * cgx_mm_read: the reference loader's semantics (banner of 5 words, line 2
 * always discarded, '%' lines skipped, a size line, "i j v" triplets until
 * the first token that does not parse, off-diagonals always mirrored,
 * entries sorted by (row, col), empty rows dropped from rowptr), parsed with
 * `threads` threads (0: $OMP_NUM_THREADS or min(cores, 16)). Arrays are
 * host memory; release with cgx_free_host. Replaces read_file
 * (mm_reader.cpp:154-171).
 * cgx_mm_write_lower: the lower triangle as a `symmetric` file with one
 * comment line, values "%.17g" (reads back bit-identically). */
int cgx_mm_read(const char *path, int threads, int64_t *n, int64_t *nnz, int **rowptr,
                int **col, double **val);
int cgx_mm_write_lower(const char *path, int64_t n, const int *rowptr, const int *col,
                       const double *val, int threads);

/* Host-only: the SELL-P layout (2 rows per lane, slices of 128 rows): per
 * slice {first value slot, first 16-byte value-code chunk, first pattern
 * entry, pattern width}; pat[npat]
 * the sorted (col - row) patterns. *nsl = 0 when the matrix does not
 * qualify (a pattern wider than 32, unsorted rows, too much padding). */
int cgx_sellp_plan(const int *h_rowptr, const int *h_col, int64_t n, int64_t *nsl,
                   int64_t **slices, int64_t *npat, int **pat, int64_t *value_slots,
                   int *max_width);
/* The same plan formed on the device (cgx_csr_create's own path since round
 * 6): k_sellp_plan builds each slice's pattern with one wave, so the column
 * array never crosses to the host; the pattern pool, offsets and padding
 * bound follow on the host as above. Outputs as cgx_sellp_plan (free with
 * cgx_free_host). Needs a device. */
int cgx_sellp_plan_device(cgx_ctx *ctx, const int *d_rowptr, const int *d_col, int64_t n,
                          int64_t nnz, int64_t *nsl, int64_t **slices, int64_t *npat, int **pat,
                          int64_t *value_slots, int *max_width);
int cgx_sell_plan(const int *h_rowptr, const int *h_col, int64_t n, int rows_per_lane,
                  int64_t *nsl,
                  int64_t **slices, int64_t *ndict, int **dict, int64_t *nidx,
                  unsigned long long **idx, int64_t *value_slots);

/* ---- diagnostics ------------------------------------------------------------
 * Average device time (ms) of `iters` launches of the SpMV + p.Ap kernel in
 * variant `variant` (bit 1: XCD-contiguous split, 2: non-temporal val/col
 * loads, 4: paired 16-B/8-B loads), y = A x. For A/B tuning on one device. */
int cgx_tune_spmv(cgx_ctx *ctx, cgx_csr *A, int variant, const void *d_x, void *d_y,
                  int iters, double *avg_ms);

#ifdef __cplusplus
}
#endif
#endif /* CGX_H */
