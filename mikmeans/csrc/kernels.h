// mikmeans — host-side launcher declarations for the gfx950 kernels.
//
// Every launcher is stream-ordered (takes the hipStream_t it must launch on),
// allocates nothing and never synchronises, so a caller may capture a whole
// Lloyd iteration into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mk {

enum DType : int { DT_F32 = 0, DT_BF16 = 1 };

// Number of f64 accumulation slots the assign kernel spreads its per-workgroup
// inertia / changed-label partials over (slot = blockIdx % NSLOT, 8 doubles each).
constexpr int NSLOT = 256;
constexpr int SLOT_STRIDE = 8;

// ---- centroid packing -------------------------------------------------------
// The assign kernel reads centroids from a "fragment-packed" array: for tile t (16
// centroids) and 16-byte piece q, the 64 lanes' MFMA A-operand fragments are stored
// contiguously (1 KiB), so one LDS-DMA wave-instruction stages a piece and one
// ds_read_b128 per lane fetches it conflict-free.
//   element (k, d): t = k/16, r = k%16, q = d / (4V), g = (d / V) % 4
//   offset = ((t*NQ + q)*64 + r + 16*g)*V + d%V,  V = 16/sizeof(T), NQ = DPAD/(4V)
// (piece q of lane group g holds features [(4q+g)V, +V): the four lane groups of a
// point read 64 contiguous bytes of its row per fragment load, see assign16.hip)
// The stored value is -2*c (exact in bf16/f32) and cn[k] = |c_q|^2 of the quantised
// centroid, so the MFMA chain seeded with cn directly yields
// score = |c|^2 - 2 x.c  (= |x-c|^2 - |x|^2).
// A/B experiment switches (scripts/ab_ext.py, A/B harnesses, tests).  No launcher reads the
// environment: the values are taken from MIKMEANS_<NAME> once when the extension loads and
// changed only through set_variant (mikmeans.ops.native.variant); -1 = the built-in rule.
// A captured hipGraph keeps the geometry that was in force when it was recorded.
// (Round 6 removed the measured losers: the persistent grid, the centre-stationary kernel, the
// first-wave stagger and the prologue priority; their results stay in profiles/.)
enum Variant { V_ASSIGN_VARG = 0, V_ASSIGN_PMAJ, V_ASSIGN_GEOM, V_UPDATE_KS, V_UPDATE_KS_GM, V_BLOBS_TPR,
               V_ASSIGN_TOP2_GEOM, V_ASSIGN_EPI, V_ASSIGN_EARLY, V_COLSTAT_BLOCKS, V_COUNT };
int variant(Variant v);
void set_variant(Variant v, int value);

int assign16_chunk_tiles(int dtype, int dpad);  // centroid tiles per LDS chunk (0 = unsupported)
int assign_kpad(int dtype, int dpad, int K);     // K rounded to a chunk multiple
int assign_cn_len(int kpad);                     // cn array length (multiple of 256 floats)

struct AssignArgs {
  const void* X; int64_t N; int D; int64_t ldx;
  const void* Cpack; const float* cn; int Kpad;
  const float* xn;      // optional: |x|^2 per row, needed for mind/inertia
  int32_t* labels;      // in/out (old labels read when track_changed)
  float* mind;          // optional: squared distance to the chosen centroid
  double* slots;        // optional: [NSLOT][SLOT_STRIDE] order-free digit slots (common.h slot_add)
  int track_changed;
  // optional u64 [N] all-ones scratch; small N then splits the centre range over
  // grid.y (split_finish_kernel writes labels and restores the all-ones)
  unsigned long long* split_keys = nullptr;
  // optional gathered batch: logical row i is X row rows[i] (labels / mind / xn stay
  // logical; without xn the inertia uses |x|^2 of the gathered fragments)
  const int64_t* rows = nullptr;
  // bounded E-step (models/lloyd.py, Hamerly bounds): with ub/lb the kernel also tracks each
  // point's second-smallest score and writes ub = distance to the chosen centre, lb = distance
  // to the second nearest (one-pass grid, no value-only argmin); scatter: a gathered batch's
  // outputs (labels, mind, ub, lb) and inputs (old labels, xn) live at row rows[i], not at i
  float* ub = nullptr;
  float* lb = nullptr;
  int scatter = 0;
  // optional device row count (int64): the launch covers N rows, the kernel assigns the first
  // min(N, *n_dev) -- a compacted batch whose size only the device knows (no host sync, so
  // the bounded E-step captures into a graph); workgroups past it exit at once
  const int64_t* n_dev = nullptr;
  // optional per-row seed offsets (bf16, indexed by X row): every row's scores are seeded with
  // oseed[row] -- the offset the full (ungathered) pass gives it, from launch_seed_offsets -- so a
  // gathered batch ranks each row bitwise as the full pass does (the bounded E-step)
  const float* oseed = nullptr;
  // optional timeline (profiling, launcher-set from set_assign_timeline): per workgroup 8 u64 --
  // real-time ticks (10 ns) at entry, chunk-loop start, epilogue start and exit, then HW_ID
  // and XCC_ID (which CU ran it), then the tick wave 0's prologue loads had all landed
  unsigned long long* timeline = nullptr;
  // launcher-set (A/B switch V_ASSIGN_EPI, default on): the epilogue's old labels and caller
  // norms are fetched with the prologue's fragments instead of in the epilogue
  int epi_prefetch = 1;
  // launcher-set (A/B switch V_ASSIGN_EARLY): norms first, fragments in flight across the
  // seed-offset barrier (plain full bf16 rows with caller norms)
  int early_prologue = 1;
};
// Profiling hook: every assign16 launch writes its workgroups' timelines to buf (nullptr: off;
// the caller sizes it for the grid, 8 u64 per workgroup, capacity in workgroups)
void set_assign_timeline(unsigned long long* buf, int64_t capacity);
hipError_t launch_assign16(int dtype, int dpad, const AssignArgs& a, hipStream_t s);
// Rows per workgroup of the full (ungathered, unbounded) assign for this shape: the block its
// bf16 seed offset is taken over (mirrors launch16_d / launch16_w)
int assign16_block_rows(int dtype, int dpad, int kpad);
// oseed[i] = the full pass's seed offset of row i (block_rows from assign16_block_rows; bf16)
hipError_t launch_seed_offsets(const float* xn, int64_t n, int block_rows, float* oseed, hipStream_t s);

// ---- transform: every row's distance to every centre (csrc/transform.hip) --------------
struct TransformArgs {
  const void* X; int64_t N; int D; int64_t ldx;
  const void* pack; const float* cn; int K; int Kpad;   // the assign kernel's packed centres
  const float* xn;      // |x|^2 per row
  float* out; int64_t ldo;
  int squared;          // 1: squared distances, 0: distances
};
hipError_t launch_transform(int dtype, int dpad, const TransformArgs& a, hipStream_t s);

// ---- Hamerly bounds (csrc/rows.hip) ----------------------------------------------------
// Moves every point's bounds by the last M-step's centre shifts (ub += |dc_label|,
// lb -= the largest |dc_k| over k != label) and flags the points whose bounds no longer prove
// their label (cand[i] = 1): shift2 = squared shifts [K] of the centres the assign ranks
// (finalize qshift); cn = |c|^2 of the packed centres, xn = |x|^2, oseed (bf16: the rows'
// full-pass seed offsets, else null) and nterms (the features) size the rounding slack of the
// kernel's scores; work: 4 floats scratch.  A row stays unflagged only where the full
// assign's keys provably keep its label (the slack counted on both sides of the test), so
// skipping it changes nothing.
hipError_t launch_bounds_update(const int32_t* labels, float* ub, float* lb, const float* shift2, const float* cn,
                                int K, const float* xn, int64_t n, uint8_t* cand, float* work, const float* oseed,
                                int nterms, hipStream_t s);
// rows[0..*count) = indices of the nonzero flags, ascending (deterministic, no host sync);
// bscratch: int64 [compact_blocks(n)]
int64_t compact_blocks(int64_t n);
// Hamerly's tightening over the compacted candidates rows[0..*count): ub = |x - c_label| (f32
// centres C [K][ldc], bf16-rounded for bf16 points: the centres the assign ranks); cand = 0 where the bounds test of launch_bounds_update passes with it
// (xn, work, oseed as there, nterms = D: work holds that step's slack terms).  n_max bounds *count
hipError_t launch_tighten(int dtype, const void* X, int64_t ldx, int D, const int32_t* labels, const float* C,
                          int64_t ldc, const int64_t* rows, const int64_t* count, int64_t n_max, float* ub,
                          const float* lb, uint8_t* cand, const float* xn, const float* work, const float* oseed,
                          hipStream_t s);
// k-means|| round: cand[i] = u(start + i) < ell * d2[i] / psi[0] (philox uniform keyed by the global row)
hipError_t launch_kpar_select(const float* d2, int64_t n, int64_t start, const double* psi, double ell,
                              uint64_t seed, uint32_t round, uint8_t* cand, hipStream_t s);
hipError_t launch_compact(const uint8_t* cand, int64_t n, int64_t* rows, int64_t* count, int64_t* bscratch,
                          hipStream_t s);

// ---- update (LDS-privatised scatter-add) -------------------------------------
// Sums are accumulated in FIXED POINT: every contribution x*w is rounded to a
// 32-bit integer at scale 2^sum_exp (|x*w| * 2^sum_exp <= 2^30) and added with
// 64-bit integer LDS atomics (ds_add_u64, ~8 cycles per wave-instruction on
// gfx950, against ~170 for ds_add_f32).  Integer addition is associative, so
// the M-step is bitwise reproducible whatever the atomic order.
struct UpdateArgs {
  const void* X; int64_t N; int D; int64_t ldx;
  const int32_t* labels; int K;
  int n_chunks;          // multiple of 8
  long long* slab;       // [n_chunks][K][D] fixed-point partial sums
  long long* cnt_slab;   // [n_chunks][K] fixed-point partial counts
  const float* weights;  // optional per-row weights (sample_weight)
  const int* col_exp;    // [D] column d's contributions are rne(x * w * 2^col_exp[d]), |.| <= 2^20
  int cnt_exp;           // counts scale 2^cnt_exp (0 when unweighted)
  int clamp;             // saturate contributions outside +-2^20 (streamed data) ...
  int* clamp_count = nullptr;  // ... and count the workgroups that did (optional)
  // Residual (lo) pass of wide-range columns (optional): contributions are
  // rne((x*w*2^col_exp - rne(x*w*2^col_exp)) * 2^(col_exp2 - col_exp)) on columns with
  // col_exp2 > -200, nothing elsewhere; slices without such a column are skipped.
  const int* col_exp2 = nullptr;
  // Incremental M-step (optional): rows whose label changed since the last M-step, as
  // (row, previous label) pairs from launch_label_delta.  Each is added to its new
  // label and subtracted from its old one; when *dcount > dcap the list overflowed
  // and the kernel accumulates all N rows instead (the reduce then restarts totals).
  const int2* dlist = nullptr;
  const int* dcount = nullptr;
  int dcap = 0;
  // Gathered batch (optional, plain passes only): logical row i is X row rows[i], so a
  // mini-batch drawn from an HBM-resident shard is never copied (labels / weights logical).
  const int64_t* rows = nullptr;
};
int update_slice_width(int dtype, int K, int D, bool weighted = false);  // 0 = global fallback
int update_n_chunks(int dtype, int K, int D, int64_t N, bool weighted = false);
int fixed_exp(double maxabs);                     // largest e with maxabs * 2^e <= 2^20
void set_update_max_sw(int sw);                   // cap the slice width (0 = none)
hipError_t launch_update(int dtype, const UpdateArgs& a, hipStream_t s);
// Changed rows: for every i with labels[i] != prev[i], append (i, prev[i]) to list
// (first `cap` entries kept, *count counts all) and set prev[i] = labels[i].
// Zeroes *count first (stream-ordered).
hipError_t launch_label_delta(const int32_t* labels, int32_t* prev, int64_t N, int2* list, int cap,
                              int* count, hipStream_t s);
// The same over the candidate rows rows[0..*rcount) only (bounded E-step; n_max >= *rcount)
hipError_t launch_label_delta_rows(const int32_t* labels, int32_t* prev, const int64_t* rows, const int64_t* rcount,
                                   int64_t n_max, int2* list, int cap, int* count, hipStream_t s);

// Reduce slabs (+ assign slots) into the packed f64 message
// [K*D sums | K counts | inertia | n_changed] (length K*D + K + 2).
hipError_t launch_reduce(const long long* slab, const long long* cnt_slab, int n_chunks, int K,
                         int D, const int* col_exp, int cnt_exp, double* slots, double* packed,
                         hipStream_t s, long long* tot = nullptr, const int* dcount = nullptr,
                         int dcap = 0);
// With `tot` ([K*D + K] int64, persistent across iterations): tot += slab sums (or
// tot = slab sums when *dcount > dcap), and the message is built from tot.
// out[k*nw + j] = 2^-exps[j] * sum_c slab[c][k][cols[j]]  (wide-column lo sums)
hipError_t launch_reduce_cols(const long long* slab, int n_chunks, int K, int D, const int* cols,
                              const int* exps, int nw, double* out, hipStream_t s);

// ---- finalize (new centroids + shift + re-pack) -------------------------------
enum FinalizeMode : int { FIN_PACK_ONLY = 0, FIN_LLOYD = 1, FIN_MINIBATCH = 2 };
struct FinalizeArgs {
  const double* packed;   // may be null for FIN_PACK_ONLY
  const float* Cold; float* Cnew; int K; int D;
  const uint8_t* frozen;  // optional
  double* mb_counts;      // FIN_MINIBATCH running per-centre counts
  int dtype; int dpad; int Kpad;
  void* pack; float* cn;
  float* shift;           // optional [K]
  float* counts_out;      // optional [K]
  int mode;
  // optional [K]: |q(C_new) - q(C_old)|^2, the move of the quantised centres the assign ranks
  // (q = bf16 rounding; the f32 shift for f32 points) -- the bounded E-step's shifts
  float* qshift = nullptr;
};
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s);

// ---- row squared norms -------------------------------------------------------
// Per-column max |x| (as f32 bit patterns, atomicMax into a zeroed out[D]); optionally, all
// together, fstats = [sum |x| | sum x | sum x^2] (f64 [3][D], zeroed), the nonzero count
// (u64 [D], zeroed) and the lowest set bit's exponent over nonzero finite values (int [D],
// initialised to INT_MAX by the caller).
// The f64 sums are bitwise reproducible: each block writes its partials to its row of fpart
// (f64 [colstat_rows(dtype, N, D)][3][D], zeroed by the caller) and one fixed-order pass sums them.
// xn (optional, D <= 64 pieces): every row's |x|^2 from the same pass, bitwise row_sqnorm's.
int colstat_blocks();
int colstat_rows(int dtype, int64_t N, int D);   // fpart rows one launch_col_absmax call writes
hipError_t launch_col_absmax(int dtype, const void* X, int64_t N, int D, int64_t ldx, uint32_t* out,
                             hipStream_t s, double* fstats = nullptr, unsigned long long* nnz = nullptr,
                             int* lowbit = nullptr, double* fpart = nullptr, float* xn = nullptr);
hipError_t launch_row_sqnorm(int dtype, const void* X, int64_t N, int D, int64_t ldx, float* out,
                             hipStream_t s);

// ---- rows (csrc/rows.hip) ----------------------------------------------------------
// Mini-batch sampler: out[j] = X[idx_j] for j < b, idx_j = floor(u * n) from Philox keyed by
// (seed; j, step, rank) (NumPy mirror: mikmeans/data/sampler.py); xn / idx_out optional.
hipError_t launch_sample_rows(int dtype, const void* X, int64_t n, int64_t ldx, int D, void* out,
                              int64_t ldo, int64_t b, uint64_t seed, uint32_t rank, uint32_t step,
                              float* xn, int64_t* idx_out, hipStream_t s);
// idx[j] = the sampler's source row of batch row j (the same draws as launch_sample_rows).
hipError_t launch_sample_index(int64_t n, int64_t b, uint64_t seed, uint32_t rank, uint32_t step, int64_t* idx,
                               hipStream_t s);
// In place x <- x / max(|x|, 1e-30) per row (cosine metric); xn (optional) = |x_rounded|^2.
hipError_t launch_row_normalize(int dtype, void* X, int64_t N, int D, int64_t ldx, float* xn, hipStream_t s);
// out[0] += sum a[i] * b[i] (f64 accumulation, deterministic order; scratch: wdot_scratch_len() f64).
int wdot_scratch_len();
hipError_t launch_wdot(const float* a, const float* b, int64_t n, double* out, double* scratch, hipStream_t s);

// ---- k-means++ ---------------------------------------------------------------
// With owner[N] (int32: centre each d2 was measured against) and cc[k] (|c - c_j|^2, from
// launch_kpp_cc) rows the triangle inequality rules out are not read (bit-identical
// result); knew >= 0 records the new centre as the owner of rows whose d2 drops.
hipError_t launch_kpp_d2(int dtype, const void* X, int64_t N, int D, int64_t ldx, const float* c,
                         int first, float* d2, double* block_sums, int64_t rows_per_block,
                         int nblocks, hipStream_t s, int32_t* owner = nullptr,
                         const float* cc = nullptr, int kcc = 0, int knew = -1);
hipError_t launch_kpp_cc(const float* C, int64_t ldc, int k, int D, const float* cnew, float* cc,
                         hipStream_t s);
// mode 0: target = device double (rank-local; < 0 writes zeros to crow); mode 1: target
// holds u, scaled by this rank's total; mode 2: target holds u, totals_all[world] decide
// the owner rank and its local target on device.
hipError_t launch_kpp_sample(int dtype, const double* block_sums, int nblocks, const float* d2,
                             int64_t N, int64_t rows_per_block, const double* target, const void* X,
                             int D, int64_t ldx, float* crow, int64_t* idx_out, int mode,
                             const double* totals_all, int world, int rank, hipStream_t s);

// Weighted k-means++ over M candidates (the k-means|| recluster): Ct f32 [D][M] (column-major),
// w f64 [M], u f64 [K]; d2 f64 [M] (= +inf before the first step), cum f64 [M] and part f64
// [ceil(M/256)] scratch, state int64 {previous pick (-1 first), next k}.  Enqueues `steps`
// draws, each writing out[k][0..D) (row stride ldo); no host read.
hipError_t launch_wkpp(const float* Ct, int64_t M, int D, const double* w, double* d2, double* cum, double* part,
                       const double* u, int64_t* state, float* out, int64_t ldo, int steps, hipStream_t s);

// ---- synthetic Gaussian blobs (counter-based Philox, deterministic by index) --
hipError_t launch_blob_centers(float* centers, int n_centers, int D, float box, uint64_t seed,
                               hipStream_t s);
hipError_t launch_blobs(int dtype, void* X, int64_t i0, int64_t n, int D, int64_t ldx,
                        const float* centers, int n_centers, float stddev, uint64_t seed,
                        int32_t* y, float* xn, hipStream_t s);

}  // namespace mk
