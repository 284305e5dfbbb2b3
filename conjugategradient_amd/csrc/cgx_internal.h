// cgx_internal.h — shared definitions between the HIP kernels
// (cgx_kernels.hip) and the C-ABI host code (cgx_abi.cpp, cgx_dist.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace cgx {

// ---- launch geometry --------------------------------------------------------
constexpr int kBlock = 256;        // threads per workgroup (4 waves of 64)
constexpr int kTile = 2048;        // CSR entries staged in LDS per row block
constexpr int kTileCap = kTile - 6; // entries a row block may hold (quad loads overrun)
constexpr int kRowsPerBlock = 256; // max rows per row block (one per thread)
constexpr int kMaxGrid = 2048;     // persistent grid cap: 256 CUs x 8 WGs
constexpr int kMaxRed = 2;         // values reduced together (accuracy: 2)

// ---- device-resident CG scalars (CG.hpp:280-289, made a ring) ----------------
// Iteration k of a solve uses slot s = k % 4. Kernels of iteration k read
// active[s] at entry and return at once when it is 0; the x/p-update kernel of
// iteration k writes active[(s+1)%4] and rxr[(s+1)%4] (nobody in iteration k
// reads those), which makes many iterations enqueue-able without a host sync
// and keeps the reference's stop rule exact (CG.hpp:396-404,436).
template <typename T> struct CgScalars {
  T rxr[4];   // r.r at the start of the iteration in slot s
  T pAp[4];   // value2 (CG.hpp:378)
  T rr[4];    // value3 (CG.hpp:406)
  T tol;      // acc (CG.hpp:286)
  T pad_t;
  int active[4];
  int xpend[4];      // fused iteration: body in slot s has its x update pending
  long long bodies;  // loop bodies executed (the reference's counter + 1)
  long long cap;     // max bodies: N+1 (CG.hpp:436) or a caller cap
  int stopped;       // 0 running, 1 stop rule (tol / NaN), 2 cap reached,
                     // 3 peer transport fault (a spin timed out), 4 a mode-5
                     // grid-wide exchange timed out
  // mode 4 on a partitioned matrix: the r.r all-reduce in kernel 3's last
  // workgroup timed out (written by that workgroup only: stopped and active
  // belong to workgroup 0 of the same launch); the host stops as on 3
  int tail_fault;
  // deferred x update (mode 3, cgx_abi.cpp enqueue_iter_defer): alpha of the
  // body in slot s, set by its update_r; ran[s]: the body ran and its x
  // update is not applied yet (set by its update_xp, cleared by the slot-3
  // flush); skip[s]: an end-of-run flush already applied it (cleared by the
  // body's update_r). Each is written and read by different launches.
  T alpha[4];
  int ran[4];
  int skip[4];
};

// Grid-reduction workspace. Arrivals are sharded over kRedGroups tickets
// (workgroup b arrives on ticket b % kRedGroups, i.e. on its own XCD), the
// last arrival of each group pre-sums that group's partials into gsum, and
// the last group to finish sums gsum in group order. Same-address atomics
// serialize (~12 ns each, MI355X guide §atomics); 2048 arrivals on one
// counter put ~25 us of that at the kernel's tail.
constexpr int kRedGroups = 8;
template <typename T> struct RedWs {
  unsigned int ticket[kRedGroups];
  unsigned int top;
  unsigned int pad[7];
  T gsum[kMaxRed * kRedGroups];
  T partials[kMaxRed * kMaxGrid];
  // per-workgroup partials of the iteration's two dots, summed by the NEXT
  // kernel (every workgroup, fixed order): no tail chain in the producer
  // (each partial a double-length pair hi, lo: cgx_kernels.hip Dd)
  T pap_part[4 * kMaxGrid];  // room for the interior + boundary launches of a split SpMV
  T rr_part[4 * kMaxGrid];
};

// SELL copy of a matrix (built by cgx_csr_create when the matrix qualifies,
// DESIGN.md §SpMV formats), R = 1 or 2 rows per lane: rows in slices of
// 64 R, one wave per slice, lane l owns rows 64 R s + R l + r (r < R).
// Entry j of that row sits at val[voff + (64 j + l) R + r]; its column is
// row + dict[dict + k] where k is byte j % 8 of the 64-bit word
// idx[ioff + (64 (j / 8) + l) R + r] (k = 0xff: padding). R = 2 makes every
// value and index access of a lane one 16-byte load.
constexpr int kSellRows = 64;
constexpr int kSellMaxDict = 64;    // distinct (col - row) per slice: one VGPR
constexpr int kSellMaxWidth = 64;   // longest row of a slice
constexpr unsigned kSellPad = 0xff;
constexpr int kSellPatMax = 32;   // SELL-P: offsets per slice pattern (u32 masks)
constexpr int kSellDefaultR = 2;    // rows per lane of the SELL copy cgx_csr_create builds
                                    // (2: 16-byte loads, profiles/r01_tune_sell2.log)
// SELL-P value codes ("value codes"): a matrix with at most
// kVcMax distinct values (bit patterns) gets, beside the SELL-P values, one
// code byte per slot: 16 bytes per lane per chunk of 8 slots (byte 2 j + r:
// slot j of the lane's row r), chunks of a slice consecutive from
// SellSlice.ioff (in 16-byte units); kVcAbsent marks an empty slot. The
// kernel reads the dictionary into LDS; the stream is 1 B per slot
// instead of 8 (+ the row mask, which the code replaces).
constexpr int kVcMax = 255;
constexpr int kVcDict = 256;  // dictionary slots (entries past nvdict: zero)
constexpr unsigned kVcAbsent = 0xff;
constexpr int kVc4Max = 15;  // 4-bit codes: 15 values, 0xf empty
// Value-code templates (variant bit kVT): the most frequent
// 64-lane chunks of 4-bit codes (a constant-coefficient stencil has a
// handful) are stored once, up to kVtMax of them, and copied into every
// workgroup's LDS; a slice whose chunk equals template t byte for byte has
// its code word read from LDS instead of HBM. Its descriptor in the
// template copy of the slice table (CsrDev::sl_t) carries t + 1 in the high
// half of its width (widths are at most 64).
constexpr int kVT = 8388608;
// CSR-stream with 16-bit column deltas (bit 128 on the paired loop: 133 =
// 5 | 128): 10 bytes per entry instead of 12
constexpr int kC16 = 128;
// CSR-stream on the interleaved copy of val / col (variant bit kIL on the
// pipelined paired loop: 15 | kIL, 13 | kIL; round 6): the value pairs and
// column pairs of each chunk of kIlCh consecutive pairs (2 kIlCh entries)
// side by side in one array, kIlCh x 16 B of values then kIlCh x 8 B of
// columns; the same 12 B per entry as the two CSR arrays, one stream instead
// of two independently placed ones
constexpr int kIL = 67108864;
constexpr int kIlLog = 8;
constexpr int kIlCh = 1 << kIlLog;          // pairs per chunk
constexpr int64_t kIlChBytes = kIlCh * 24;  // 6 KiB (f64)
constexpr int kVtMax = 8;
constexpr int kVtWidthMask = 0xffff;
// Lean stencil walk (variant bit kVL; DESIGN.md §4 "lean stencil walk"): a
// slice whose offset pattern is a subset of a stencil's {-D, -a, -1, 0, +1,
// +a, +D} (a = 0: the 2-D {-D, -1, 0, +1, +D}) and whose template chunk gives
// every row of a slot the same value (rows 0 and 1 of a lane alike) has no
// per-row data at all: its class (template, pattern) holds the seven values
// and which slots are present. The only entries a row of such a slice may
// lack are the x-line ends' -1 (lane 0, row 0) and +1 (lane 63, row 1); the
// kernel then multiplies v by z = -copysign(0, v), whose product -0.0 is the
// identity of +, so the row's sum is the one that skips the entry, bit for
// bit (v finite). Classes per slice: one byte, 0xff for the slices that run
// the per-slice value-code form, laid out wave-major for the launch's grid
// (row of wave w of XCD group g: (g step + w) * nst, step = grid / 2 waves).
constexpr int kVL = 33554432;
constexpr int kVlMaxCls = 32;
struct VlClass {
  double v[8];      // value of canonical slot j: -D, -a, -1, 0, +1, +a, +D
  double zlo, zhi;  // -copysign(0, v[2]), -copysign(0, v[4])
  int plo, phi;     // lane 0's row 0 has its -1 entry; lane 63's row 1 its +1
  int pres;         // bit 0 -D, 1 -a, 2 +a, 3 +D present (-1, 0, +1 always are)
  int pad;
};

struct SellSlice {
  int64_t voff;  // first value of the slice (entries)
  int64_t ioff;  // first index word of the slice (SELL-P: first 16-byte code chunk)
  int dict;      // first entry of the slice's offset dictionary
  int width;     // entries per row in this slice (longest row)
};

struct PeerDev;  // cgx_objects.h

// ---- launchers (cgx_kernels.hip) --------------------------------------------
struct CsrDev {
  int64_t n, nnz;
  const int *rowptr;
  const int *col;
  const void *val;
  const int *rb;   // row-block starts, nrb + 1 entries
  const int *rbk;  // rowptr[rb[i]], nrb + 1 entries
  int nrb;
  int tile = kTile; // entries per row block the schedule was built for (2048 | 1024 | 512)
  int variant = 0;  // SpMV variant picked for this matrix (0: size heuristic)
  // SELL-64 copy (null when the matrix does not qualify)
  const SellSlice *sl = nullptr;
  const int *sdict = nullptr;
  const unsigned long long *sidx = nullptr;
  const void *sval = nullptr;
  int64_t nsl = 0;
  int sell_maxw = 0;  // widest slice
  int sell_r = 1;     // rows per lane of the SELL copy
  const int *sorder = nullptr;  // visit order of the slices (null: index order)
  // SELL-P (pattern) copy: per-slice offset pattern (in sdict) and one slot
  // mask per row (u8 or u32); 0: dictionary SELL, 1: u8 masks, 2: u32 masks
  int sell_kind = 0;
  const void *smask = nullptr;
  int64_t nx = 0;  // length of the gathered vector (n, + ghosts when partitioned)
  // SELL-P value codes (variant bit 32768, null when the matrix has more
  // than kVcMax distinct values): one byte per slot, index into svdict
  // (kVcAbsent: the row has no entry in the slot); layout at SellSlice.ioff
  const void *svc = nullptr;
  const void *svdict = nullptr;  // kVcDict values of the matrix's type
  int nvdict = 0;                // distinct values (0: no codes)
  // 4-bit codes (variant bit 262144; at most kVc4Max values): 8 bytes per
  // lane per chunk, byte j = slot j, row 0 in the low nibble
  const void *svc4 = nullptr;
  // plane march (variant bit 2097152; cgx_abi.cpp plan_march): the dominant
  // SELL-P pattern is {-D, (-a,) -1, 0, 1, (a,) D} with D = 128 march_k rows
  // at pool base march_pat; march_len: planes per run (0: fill the grid)
  int march_k = 0, march_a = 0, march_pat = -1, march_len = 0;
  // value-code templates (kVT): the slice table with template ids, the
  // templates (nvt x 64 words of 4-bit codes)
  const SellSlice *sl_t = nullptr;
  const void *vct = nullptr;
  int nvt = 0;
  // CSR-stream with 16-bit column deltas (variant bit kC16): entry k of row
  // block b stores col[k] - rb[b] (every such delta fits int16; null when
  // one does not or the copy was not built)
  const short *col16 = nullptr;
  // the interleaved val / col copy of the CSR-stream forms (kIL; null when
  // not built): chunk c at c * kIlChBytes (f64; half the value bytes for f32)
  const char *il = nullptr;
  // lean stencil walk (kVL, cgx_abi.cpp build_lean): the class bytes in the
  // wave-major layout of a vl_grid-workgroup launch (vl_nst bytes per wave),
  // the class table, the stencil's D and a; `lean`: the loop's SpMV runs it
  const unsigned char *vl_cls = nullptr;
  const VlClass *vl_tab = nullptr;
  int vl_grid = 0, vl_nst = 0, vl_D = 0, vl_a = 0;
  int vl_P = 0, vl_K = 0;  // the chunked walk's planes per XCD group, slices per plane
  int vl_lds = 0;  // the per-slice form's dictionary and templates copied to LDS first
  // a partitioned matrix's layout: its boundary slices (the split's, run by
  // the boundary launch) are skipped, so the walk covers the interior only
  int vl_split = 0;
  // mode 4's fused walk (k_spmv_fd_lean) in its team form (1,024-thread
  // workgroups sharing their neighbours' formed p_k pairs through LDS;
  // cgx_kernels.hip spmv_lean_team): vl_grid / 4 workgroups; whole-matrix
  // walks only
  int vl_team = 0;
  bool lean = false;
  // a partitioned matrix's SELL copy holds its boundary slices only as
  // placeholders (their rows may be unsorted in local numbering: ghosts from
  // lower ranks come after the own rows); whole-matrix SpMVs take CSR-stream
  int sell_partial = 0;
  // CSR-stream block visit order (cgx_abi.cpp build_block_order; null:
  // natural): walk position -> row block, a permutation within each XCD
  // eighth that walks chunks of ob_W rows through planes ob_D rows apart
  const int *rbo = nullptr;
  int ob_D = 0, ob_W = 0;
};

// The templates apply to the pipelined 4-bit value-code walks (bits 524288,
// 262144; the consecutive walk and the plane march) of a matrix that has
// them, when the requested variant asks for them: spmv_variant keeps kVT and
// the kernel arguments take the template slice table under exactly this
// condition.
__host__ __device__ inline bool vt_active(const CsrDev &A) {
  return (A.variant & kVT) && A.sl_t && A.vct && A.nvt > 0 && A.svc4 && A.svc && A.sl &&
         A.sell_kind && A.sell_maxw <= 8 && (A.variant & 524288) && (A.variant & 262144);
}
// the loop's k_spmv_dot is the lean walk (its generic slices run the
// template value-code form, so vt_active holds too)
__host__ __device__ inline bool vl_active(const CsrDev &A) {
  return A.lean && A.vl_cls && A.vl_tab && A.vl_grid > 0 && vt_active(A);
}
// the lean walk covers the whole matrix (not a partitioned matrix's interior)
__host__ __device__ inline bool vl_whole(const CsrDev &A) {
  return vl_active(A) && !A.vl_split && !A.sell_partial;
}
// the tile form of the lean walk (cgx_kernels.hip spmv_lean_tile) applies,
// and the partial count of its launches (modes 6 and 7's kernel 1)
bool lean_tile_ok(const CsrDev &A);
int lean_dot_parts(const CsrDev &A);
int fd_dot_parts(const CsrDev &A);  // mode 7's kernel 1 (lean_tile_ok)
int lean_updr_parts(const CsrDev &A);  // mode 6's kernel 2
bool lean_updr_tile(const CsrDev &A);

// Kernel-execution timing (cgx_abi.cpp timed(), kernel timing on): the next
// launch takes these start / stop events, recorded by its dispatch itself
// (hipExtLaunchKernel: the kernel's own duration, as rocprofv3 reports it,
// without the dispatch latency an event pair around the launch includes).
// One launch consumes them; `used` tells the caller it happened.
struct ExecTiming {
  hipEvent_t start = nullptr, stop = nullptr;
  bool used = false;
};
extern thread_local ExecTiming g_exec;

template <typename T> struct Launch {
  static int grid_rows(int nrb);
  static int grid_elems(int64_t n, int cap);
  // y = A x by k_spmv_dot in A's variant (st: slot 0 active; its p.Ap
  // partials land in ws, unread): the standalone SpMV runs the loop's kernel
  static hipError_t spmv(const CsrDev &A, const T *x, T *y, CgScalars<T> *st, RedWs<T> *ws,
                         hipStream_t s);
  static hipError_t cg_init(const CsrDev &A, const T *x, const T *b, T *r, T *p,
                            CgScalars<T> *st, RedWs<T> *ws, T tol, long long cap,
                            hipStream_t s);
  // rev: sweep the rows high to low (alternating sweep directions, cgx_abi.cpp)
  static hipError_t spmv_dot(const CsrDev &A, const T *p, T *Ap, CgScalars<T> *st,
                             int slot, RedWs<T> *ws, hipStream_t s, int rev = 0);
  static hipError_t spmv_dot_variant(int v, const CsrDev &A, const T *p, T *Ap,
                                     CgScalars<T> *st, RedWs<T> *ws, hipStream_t s);
  // the lean stencil walk's resident workgroups (its grid's upper bound)
  static int lean_resident();
  // np_pap > 0: p.Ap from the spmv_dot partials; 0: from st->pAp[slot]
  static hipError_t update_r(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                             RedWs<T> *ws, hipStream_t s, bool fused = false, int np_pap = 0,
                             int rev = 0, const T *rin = nullptr,  // rin: r_old (null: r)
                             int rule = 0,   // mode 4: the stop rule runs here
                             const PeerDev *peer = nullptr);  // p.Ap all-reduced here
  // mode 4 (fused deferred-x iteration, cgx_abi.cpp enqueue_iter_fdefer):
  // kernel 1 computes p_k = r + beta p_{k-1} into pc where the SpMV reads it
  static bool fd_supported(const CsrDev &A);
  static int fd_parts(const CsrDev &A);  // kernel 1's grid (its p.Ap partials)
  static hipError_t spmv_fd(const CsrDev &A, const T *r, const T *pold, T *pc, T *Ap,
                            CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr,
                            hipStream_t s, int rev = 0);
  static hipError_t flush_group(int64_t n, T *x, T *const P[4], CgScalars<T> *st,
                                hipStream_t s, int rev = 0);
  // a partitioned matrix's boundary rows: CSR-stream over the row blocks
  // `blocks` (count), partials at [part_off, part_off + grid); with P the
  // ghosts come from the peer landing buffer after the neighbours' pushes
  static hipError_t spmv_dot_rows(const CsrDev &A, const int *blocks, int count, int part_off,
                                  const T *p, T *Ap, CgScalars<T> *st, int slot, RedWs<T> *ws,
                                  hipStream_t s, const PeerDev *P);
  static int rows_grid(const CsrDev &A, int count);
  // mode 6 (recomputed Ap; the whole-matrix lean walk only): kernel 1, the
  // walk's p.Ap partials [0, vl_grid) with no Ap stored; kernel 2, alpha, the
  // walk again with r -= alpha (A p) in its epilogue, r.r partials [0, vl_grid)
  static hipError_t lean_dot(const CsrDev &A, const T *p, CgScalars<T> *st, int slot,
                             RedWs<T> *ws, hipStream_t s, int rev);
  // mode 7 (lean_tile_ok): the fused walk forming p_k with p.Ap only, then
  // the recomputing r update with the stop rule
  static hipError_t fd_dot_tile(const CsrDev &A, const T *r, const T *pold, T *pc,
                                CgScalars<T> *st, int slot, RedWs<T> *ws, int np_rr,
                                hipStream_t s, int rev);
  static hipError_t lean_updr_rule(const CsrDev &A, const T *p, T *r, CgScalars<T> *st, int slot,
                                   RedWs<T> *ws, hipStream_t s, int rev);
  static hipError_t lean_updr(const CsrDev &A, const T *p, T *r, CgScalars<T> *st, int slot,
                              RedWs<T> *ws, hipStream_t s, int rev);
  // a partitioned matrix's interior slices by the lean walk (A.vl_split), the
  // halo push in the first wg0 workgroups when P is given; partials [0, vl_grid)
  static hipError_t spmv_lean_interior(const CsrDev &A, const T *p, T *Ap, CgScalars<T> *st,
                                       int slot, RedWs<T> *ws, hipStream_t s, int rev,
                                       const PeerDev *P, int wg0);
  // mode 4, slot 3: update_r (stop rule) and the group flush in one launch
  static hipError_t update_r_flush(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                                   RedWs<T> *ws, int np_pap, int rev, T *x, T *const P[4],
                                   hipStream_t s);
  static hipError_t rr_settle(CgScalars<T> *st, RedWs<T> *ws, int np_rr, hipStream_t s);
  // mode 4 on a partitioned matrix (device peer transport, the lean interior
  // with CSR-stream boundary rows), f64: kernel 1 (interior walk forming p_k,
  // the formed p_k pushed by the first wg0 workgroups; partials [0, vl_grid)),
  // kernel 2 (boundary row blocks, partials from part_off), kernel 3
  // (update_r with the stop rule and the world r.r; P4 non-null in slot 3:
  // the group flush)
  static hipError_t spmv_fd_lean_push(const CsrDev &A, const T *r, const T *pold, T *pc, T *Ap,
                                      CgScalars<T> *st, int slot, RedWs<T> *ws, hipStream_t s,
                                      int rev, const PeerDev &P, int wg0);
  static hipError_t spmv_fd_rows_bnd(const CsrDev &A, const int *blocks, int count, int part_off,
                                     const T *r, const T *pold, T *pc, T *Ap, CgScalars<T> *st,
                                     int slot, RedWs<T> *ws, hipStream_t s, const PeerDev &P);
  static hipError_t update_r_peer_rule(int64_t n, T *r, const T *Ap, CgScalars<T> *st, int slot,
                                       RedWs<T> *ws, int np_pap, int rev, T *x,
                                       T *const *P4, hipStream_t s, const PeerDev &P);
  // partial counts the consumers pass (the producers' grid sizes)
  static int spmv_parts(const CsrDev &A);
  // SpMV + p.Ap over `count` SELL slices listed at `list` (device), partials
  // at [part_off, part_off + slice_grid(count)); SELL matrices only
  static hipError_t spmv_dot_slices(const CsrDev &A, const int *list, int count, int part_off,
                                    const T *p, T *Ap, CgScalars<T> *st, int slot, RedWs<T> *ws,
                                    hipStream_t s, int rev = 0);
  static int slice_grid(const CsrDev &A, int count);
  // the same interior launch with the peer transport's halo push in its first
  // wg0 workgroups (k_spmv_dot_push); slice_grid_push: its SpMV workgroups
  static bool push_supported(const CsrDev &A);
  static int slice_grid_push(const CsrDev &A, int count, int wg0);
  static hipError_t spmv_dot_slices_push(const CsrDev &A, const int *list, int count,
                                         int part_off, const T *p, T *Ap, CgScalars<T> *st,
                                         int slot, RedWs<T> *ws, hipStream_t s, int rev,
                                         const PeerDev &P, int wg0);
  // the boundary launch with the peer transport's halo wait folded in: ghost
  // values read from the landing buffer (k_spmv_dot_bnd)
  static bool bnd_supported(const CsrDev &A);
  static hipError_t spmv_dot_slices_bnd(const CsrDev &A, const int *list, int count,
                                        int part_off, const T *p, T *Ap, CgScalars<T> *st,
                                        int slot, RedWs<T> *ws, hipStream_t s, int rev,
                                        const PeerDev &P);
  static int update_parts(int64_t n);
  // *dst = sum of part[0..np) (one workgroup; partitioned runs, before RCCL)
  static hipError_t finalize(const T *part, int np, T *dst, hipStream_t s);
  static bool fused_supported(const CsrDev &A);  // mode 2 (production forms)
  static hipError_t spmv_fused(const CsrDev &A, const T *r, const T *pp, T *pc, T *x, T *Ap,
                               CgScalars<T> *st, int slot, RedWs<T> *ws, hipStream_t s);
  static hipError_t flush_x(int64_t n, T *x, const T *p, CgScalars<T> *st, int slot,
                            RedWs<T> *ws, hipStream_t s);
  // np_rr > 0: r.r from the update_r partials; 0: from st->rr[slot]
  // peer: a partitioned run's r.r all-reduced in the kernel (device peer
  // transport; np_rr the local partials)
  static hipError_t update_xp(int64_t n, T *x, T *p, const T *r, CgScalars<T> *st,
                              int slot, RedWs<T> *ws, int np_rr, hipStream_t s, int rev = 0,
                              const PeerDev *peer = nullptr);
  static hipError_t update_p_defer(int64_t n, T *x, const T *p, T *pn, T *const P[4],
                                   const T *r, CgScalars<T> *st, int slot, RedWs<T> *ws,
                                   int np_rr, hipStream_t s, int rev = 0,
                                   const PeerDev *peer = nullptr);
  static hipError_t flush_defer(int64_t n, T *x, T *const P[4], CgScalars<T> *st,
                                hipStream_t s);
  static hipError_t dot_acc(int64_t n, const T *x, const T *y, T *res, RedWs<T> *ws,
                            hipStream_t s);
  static hipError_t axpby(int mode, int64_t n, const T *x, const T *y, const T *a,
                          const T *b, T *res, hipStream_t s);
  static hipError_t scalar_div(const T *num, const T *den, T *out, hipStream_t s);
  static hipError_t fill(T *d, T v, int64_t n, hipStream_t s);
  static hipError_t iota(T *d, int64_t n, double offset, hipStream_t s);
  static hipError_t accuracy(const CsrDev &A, const T *b, const T *x, T *out2,
                             RedWs<T> *ws, hipStream_t s);
  static hipError_t poisson(int dim, int nx, int ny, int nz, int64_t row_begin,
                            int64_t row_end, int *rowptr, int *col, T *val,
                            hipStream_t s);
  static hipError_t gather(const T *src, const int *idx, int64_t n, T *dst,
                           hipStream_t s);
  static hipError_t sell_pack(const CsrDev &A, const T *val, T *sval, hipStream_t s);
  static hipError_t sellp_pack(const CsrDev &A, const T *val, T *sval, void *mask,
                               hipStream_t s);
  // value codes of the SELL-P layout (dict: nd sorted bit patterns); *miss
  // counts the values not in the dictionary, the first kVcDict of them
  // stored at missv
  static hipError_t sellpv_pack(const CsrDev &A, const T *val, const T *dict, int nd,
                                unsigned char *codes, int *miss, T *missv, hipStream_t s);
  // 8-bit codes (chunks x 16 B) -> 4-bit codes (chunks x 8 B)
  static hipError_t vc_narrow(const void *codes8, void *codes4, int64_t chunks, hipStream_t s);
};

// axpby modes
enum { AX_SAPBX = 0, AX_SAMBX = 1, AX_SAXPBY = 2 };

// ---- persistent CG body (mode 5, cgx_coop.hip) -------------------------------
constexpr int kCoopK = 8;       // entries per row held in registers (7 in the 1,024-thread form)
constexpr int kCoopMaxG = 256;  // workgroups: at most one per CU (exchange granules)
// exchange granules ({tag, half of a double}: two per workgroup and exchange),
// zeroed before every launch
struct CoopWs {
  unsigned long long ga[2 * kCoopMaxG];  // p.Ap partials
  unsigned long long gb[2 * kCoopMaxG];  // r.r partials
  unsigned int tmo;                      // a workgroup's spin gave up
  unsigned int pad[3];
};
// the register form: 1 (one row per thread of 1,024) when n rows fit
// min(max_g, kCoopMaxG) workgroups; 0: none
int coop_rows_per_thread(int64_t n, int max_g);
// the streamed form: the least R <= kCoopStreamMaxR for which n rows fit
// min(max_g, kCoopMaxG) workgroups of 1,024 threads; 0: none
constexpr int kCoopStreamMaxR = 8;
int coop_stream_rows(int64_t n, int want, int max_g);
// up to m bodies from slot0 in one launch (f64, single device): x, r, p0 in
// and out in the standard layout, p1 scratch (n entries); stops as the
// three-kernel body does, or sets st->stopped = 4 when a spin gave up.
// Register form (R = 1) or, `streamed`, the form that reads the matrix every
// body (R rows per thread of 1,024). hipErrorCooperativeLaunchTooLarge: the
// occupancy API does not place every workgroup at once.
hipError_t cg_coop(int64_t n, int R, bool streamed, const int *rowptr, const int *col,
                   const double *val, double *x, double *r, double *p0, double *p1,
                   CgScalars<double> *st, int slot0, int m, CoopWs *cw, long long ticks,
                   unsigned long long *trace, int stall, hipStream_t s);
constexpr int kCoopTraceWords = kCoopMaxG * 8 * 8;  // workgroups x bodies 8-15 x phases

// value-code templates (cgx_abi.cpp build_value_templates): per slice the
// hash of its 4-bit code chunk (0: wider than one chunk); the template slice
// table of nt templates, exact byte matches only (*count: matched slices)
hipError_t vc_hash(const CsrDev &A, unsigned long long *hash, hipStream_t s);
hipError_t vc_match(const CsrDev &A, const unsigned long long *tmpl, int nt, SellSlice *sl_t,
                    unsigned *count, hipStream_t s);
// the 16-bit column deltas of A's row blocks into col16 (nnz + 2 entries);
// *bad counts the entries whose delta does not fit
hipError_t col16_build(const CsrDev &A, short *col16, unsigned *bad, hipStream_t s);
// the interleaved val / col copy (kIL) of A's CSR arrays into il
// ((nnz + 1) / 2 pairs, padded to whole chunks); element size es (4 / 8)
hipError_t il_build(const CsrDev &A, int es, char *il, hipStream_t s);
inline int64_t il_bytes(int64_t nnz, int es) {
  const int64_t pairs = (nnz + 1) / 2, chunks = (pairs + kIlCh - 1) / kIlCh;
  return chunks * kIlCh * (2 * es + 8);
}

// the SpMV variant a launch on A uses (dtype: CGX_F64 / CGX_F32)
int launch_variant(const CsrDev &A, int dtype);
// true when the variant A resolves to (launch_variant) has a k_spmv_dot
// instantiation: a request that resolves to anything else would only fail
// at its first launch
bool launch_variant_ok(const CsrDev &A, int dtype);
// v is a form k_spmv_dot is instantiated for (CGX_SPMV_LIST)
bool spmv_listed(int v);

// host-side row-block schedule (cgx_abi.cpp)
// cuts: sorted rows no block may straddle (a block ends before each)
std::vector<int> build_row_blocks(const int *rowptr, int64_t n, int *max_row_nnz,
                                  int tile = kTile, const std::vector<int64_t> *cuts = nullptr);

__host__ __device__ int64_t poisson_row_offset(int dim, int nx, int ny, int nz, int64_t row);

// the SELL-P plan's per-slice patterns on the device (k_sellp_plan): w[q]
// width (kSellPatMax + 1: too many offsets, -1: an unsorted row outside
// skip), pat[q * kSellPatMax ...] the ascending offsets
hipError_t sellp_plan_dev(int64_t n, int64_t nsl, const int *rowptr, const int *col,
                          const char *skip, int *pat, int *w, hipStream_t s);

}  // namespace cgx
