// mikmeans — torch extension binding for the gfx950 kernels (+ native host helpers).
//
// Thin, allocation-free wrappers: every op takes pre-allocated tensors, checks
// shapes/dtypes/devices on the host (a hand-written kernel must never see a
// shape it does not assume), and launches on the current HIP stream.  Built by
// hipcc directly (mikmeans/_build.py) -- no hipify, no CUDA compatibility layer.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "jsnum.h"
#include "kernels.h"

namespace {

using at::Tensor;

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "mikmeans: ", what, " failed: ", hipGetErrorString(e));
}
hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dtype_of(const Tensor& X) {
  if (X.scalar_type() == at::kBFloat16) return mk::DT_BF16;
  TORCH_CHECK(X.scalar_type() == at::kFloat, "mikmeans: points must be bfloat16 or float32");
  return mk::DT_F32;
}
int vec_of(int dt) { return dt == mk::DT_BF16 ? 8 : 4; }

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "mikmeans: ", name, " must be a GPU tensor");
}
void check_f32(const Tensor& t, const char* name, int64_t numel_min = 0) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous(), "mikmeans: ", name,
              " must be contiguous float32");
  TORCH_CHECK(t.numel() >= numel_min, "mikmeans: ", name, " too small (", t.numel(), " < ",
              numel_min, ")");
}
void check_i32(const Tensor& t, const char* name, int64_t numel_min) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kInt && t.is_contiguous(), "mikmeans: ", name,
              " must be contiguous int32");
  TORCH_CHECK(t.numel() >= numel_min, "mikmeans: ", name, " too small");
}
void check_f64(const Tensor& t, const char* name, int64_t numel_min) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kDouble && t.is_contiguous(), "mikmeans: ", name,
              " must be contiguous float64");
  TORCH_CHECK(t.numel() >= numel_min, "mikmeans: ", name, " too small");
}
// Points: 2-D, unit column stride, 16-B aligned rows whose length is a multiple of 16 B.
int64_t check_points(const Tensor& X, int dt) {
  check_cuda(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "mikmeans: X must be 2-D with unit column stride");
  const int v = vec_of(dt);
  TORCH_CHECK(X.size(1) % v == 0, "mikmeans: D must be a multiple of ", v,
              " for the vector path (pad the columns)");
  TORCH_CHECK(X.size(0) <= 1 || X.stride(0) % v == 0, "mikmeans: row stride must be 16-B aligned");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0, "mikmeans: X must be 16-B aligned");
  return X.size(0) <= 1 ? X.size(1) : X.stride(0);
}
template <typename T>
T* opt_ptr(const c10::optional<Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// ----------------------------------------------------------------------------
void check_i64(const Tensor& t, const char* name, int64_t numel_min);

void assign(const Tensor& X, const Tensor& pack, const Tensor& cn, const c10::optional<Tensor>& xn,
            const Tensor& labels, const c10::optional<Tensor>& mind,
            const c10::optional<Tensor>& slots, int64_t Kpad, int64_t dpad, bool track_changed,
            const c10::optional<Tensor>& keys, const c10::optional<Tensor>& rows,
            const c10::optional<Tensor>& ub, const c10::optional<Tensor>& lb, bool scatter,
            const c10::optional<Tensor>& count, const c10::optional<Tensor>& oseed) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  // gathered batch: N logical rows, row i = X[rows[i]] (indices from sample_index: in range
  // by construction -- the binding cannot check them without a device sync)
  const bool gathered = rows.has_value() && rows->defined();
  if (gathered) {
    check_i64(*rows, "rows", 0);
    TORCH_CHECK(X.size(0) > 0 || rows->numel() == 0, "mikmeans: gathered rows from an empty X");
    TORCH_CHECK(!(keys.has_value() && keys->defined()), "mikmeans: gathered rows take the one-pass grid");
  }
  const int64_t N = gathered ? rows->numel() : X.size(0);
  TORCH_CHECK(!scatter || gathered, "mikmeans: scatter needs rows");
  const int64_t NO = scatter ? X.size(0) : N;   // per-row outputs / inputs: at rows[i] when scattering
  const int D = (int)X.size(1);
  TORCH_CHECK(D <= dpad, "mikmeans: D exceeds dpad");
  TORCH_CHECK(mk::assign_kpad(dt, (int)dpad, (int)Kpad) == Kpad, "mikmeans: bad Kpad ", Kpad, " for dpad ",
              dpad);
  const bool bounds = ub.has_value() && ub->defined();
  TORCH_CHECK(bounds == (lb.has_value() && lb->defined()), "mikmeans: ub and lb come together");
  if (bounds) {
    check_f32(*ub, "ub", NO);
    check_f32(*lb, "lb", NO);
    TORCH_CHECK(xn.has_value() && !(keys.has_value() && keys->defined()),
                "mikmeans: bounds need xn and the one-pass grid");
  }
  check_cuda(pack, "pack");
  TORCH_CHECK(pack.is_contiguous() && pack.scalar_type() == X.scalar_type(),
              "mikmeans: pack dtype must match X");
  TORCH_CHECK(pack.numel() >= Kpad * dpad, "mikmeans: pack too small");
  check_f32(cn, "cn", mk::assign_cn_len((int)Kpad));
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kInt && labels.is_contiguous() &&
                  labels.numel() >= NO,
              "mikmeans: labels must be contiguous int32 [N]");
  if (xn.has_value()) check_f32(*xn, "xn", NO);
  if (mind.has_value()) check_f32(*mind, "mind", NO);
  if (slots.has_value()) check_f64(*slots, "slots", mk::NSLOT * mk::SLOT_STRIDE);
  TORCH_CHECK(!mind.has_value() || xn.has_value(), "mikmeans: mind needs xn");
  mk::AssignArgs a;
  a.X = X.data_ptr(); a.N = N; a.D = D; a.ldx = ldx;
  a.Cpack = pack.data_ptr(); a.cn = cn.data_ptr<float>(); a.Kpad = (int)Kpad;
  a.xn = opt_ptr<const float>(xn);
  a.labels = labels.data_ptr<int32_t>();
  a.mind = opt_ptr<float>(mind);
  a.slots = opt_ptr<double>(slots);
  a.track_changed = track_changed ? 1 : 0;
  if (keys.has_value()) {  // all-ones u64 scratch: lets small N split the centre range
    check_i64(*keys, "keys", N);
    TORCH_CHECK(!xn.has_value() || mind.has_value(), "mikmeans: split assign with xn needs mind");
    a.split_keys = (unsigned long long*)keys->data_ptr<int64_t>();
  }
  if (gathered) a.rows = rows->data_ptr<int64_t>();
  if (bounds) {
    a.ub = ub->data_ptr<float>();
    a.lb = lb->data_ptr<float>();
  }
  a.scatter = scatter ? 1 : 0;
  if (count.has_value() && count->defined()) {   // device row count: assign rows[:min(N, count)]
    check_i64(*count, "count", 1);
    TORCH_CHECK(gathered && !(keys.has_value() && keys->defined()),
                "mikmeans: a device row count takes a gathered batch on the one-pass grid");
    a.n_dev = count->data_ptr<int64_t>();
  }
  if (oseed.has_value() && oseed->defined()) {   // per-row seed offsets at the X rows (bf16 keys)
    TORCH_CHECK(dt == mk::DT_BF16, "mikmeans: seed offsets are the bf16 keys'");
    check_f32(*oseed, "oseed", X.size(0));
    a.oseed = oseed->data_ptr<float>();
  }
  hip_check(mk::launch_assign16(dt, (int)dpad, a, stream()), "assign");
}

void transform(const Tensor& X, const Tensor& pack, const Tensor& cn, int64_t K, int64_t Kpad, int64_t dpad,
               const Tensor& xn, const Tensor& out, bool squared) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const int64_t N = X.size(0);
  TORCH_CHECK(X.size(1) <= dpad, "mikmeans: D exceeds dpad");
  TORCH_CHECK(mk::assign_kpad(dt, (int)dpad, (int)K) == Kpad, "mikmeans: bad Kpad ", Kpad);
  check_cuda(pack, "pack");
  TORCH_CHECK(pack.is_contiguous() && pack.scalar_type() == X.scalar_type() && pack.numel() >= Kpad * dpad,
              "mikmeans: pack must be the points' dtype, [Kpad * dpad]");
  check_f32(cn, "cn", Kpad);
  check_f32(xn, "xn", N);
  check_cuda(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.dim() == 2 && out.size(0) == N && out.size(1) == K &&
                  out.stride(1) == 1 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "mikmeans: out must be float32 [N, K] with unit column stride, 16-B aligned");
  mk::TransformArgs a;
  a.X = X.data_ptr(); a.N = N; a.D = (int)X.size(1); a.ldx = ldx;
  a.pack = pack.data_ptr(); a.cn = cn.data_ptr<float>(); a.K = (int)K; a.Kpad = (int)Kpad;
  a.xn = xn.data_ptr<float>();
  a.out = out.data_ptr<float>(); a.ldo = N > 1 ? out.stride(0) : K;
  a.squared = squared ? 1 : 0;
  hip_check(mk::launch_transform(dt, (int)dpad, a, stream()), "transform");
}

void check_i64(const Tensor& t, const char* name, int64_t numel_min) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == at::kLong && t.is_contiguous(), "mikmeans: ", name,
              " must be contiguous int64");
  TORCH_CHECK(t.numel() >= numel_min, "mikmeans: ", name, " too small");
}

void update(const Tensor& X, const Tensor& labels, int64_t K, const Tensor& slab,
            const Tensor& cnt_slab, int64_t n_chunks, const c10::optional<Tensor>& weights,
            const Tensor& col_exp, int64_t cnt_exp, bool clamp,
            const c10::optional<Tensor>& clamp_count, const c10::optional<Tensor>& col_exp2,
            const c10::optional<Tensor>& rows) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const bool gathered = rows.has_value() && rows->defined();
  if (gathered) {
    check_i64(*rows, "rows", 0);
    TORCH_CHECK(!clamp && !(col_exp2.has_value() && col_exp2->defined()),
                "mikmeans: gathered rows take plain (bounded) M-step passes");
    TORCH_CHECK(X.size(0) > 0 || rows->numel() == 0, "mikmeans: gathered rows from an empty X");
  }
  const int64_t N = gathered ? rows->numel() : X.size(0);
  const int D = (int)X.size(1);
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kInt && labels.numel() >= N,
              "mikmeans: labels must be int32 [N]");
  const int sw = mk::update_slice_width(dt, (int)K, D, weights.has_value());
  TORCH_CHECK(sw == 0 ? n_chunks == 1 : n_chunks % 8 == 0, "mikmeans: bad n_chunks");
  check_i64(slab, "slab", n_chunks * K * D);
  check_i64(cnt_slab, "cnt_slab", n_chunks * K);
  if (weights.has_value()) check_f32(*weights, "weights", N);
  check_i32(col_exp, "col_exp", D);
  if (sw == 0) {  // global-atomic fallback accumulates into zeroed buffers
    hip_check(hipMemsetAsync(slab.data_ptr(), 0, K * D * 8, stream()), "memset");
    hip_check(hipMemsetAsync(cnt_slab.data_ptr(), 0, K * 8, stream()), "memset");
  }
  mk::UpdateArgs a;
  a.X = X.data_ptr(); a.N = N; a.D = D; a.ldx = ldx;
  a.labels = labels.data_ptr<int32_t>(); a.K = (int)K; a.n_chunks = (int)n_chunks;
  a.slab = (long long*)slab.data_ptr<int64_t>(); a.cnt_slab = (long long*)cnt_slab.data_ptr<int64_t>();
  a.weights = opt_ptr<const float>(weights);
  a.col_exp = col_exp.data_ptr<int32_t>(); a.cnt_exp = (int)cnt_exp; a.clamp = clamp ? 1 : 0;
  if (clamp_count.has_value()) {
    check_i32(*clamp_count, "clamp_count", 1);
    a.clamp_count = clamp_count->data_ptr<int32_t>();
  }
  if (col_exp2.has_value()) {
    TORCH_CHECK(sw > 0 && !clamp, "mikmeans: the residual pass needs the LDS path and no clamp");
    check_i32(*col_exp2, "col_exp2", D);
    a.col_exp2 = col_exp2->data_ptr<int32_t>();
  }
  if (gathered) a.rows = rows->data_ptr<int64_t>();
  hip_check(mk::launch_update(dt, a, stream()), "update");
}

// Incremental M-step (LloydEngine(incremental=True)): the changed-row list ...
void label_delta_rows(const Tensor& labels, const Tensor& prev, const Tensor& rows, const Tensor& rcount,
                      const Tensor& list, const Tensor& count) {
  const int64_t N = labels.numel();
  check_i32(labels, "labels", N);
  check_i32(prev, "prev", N);
  check_i32(count, "count", 1);
  check_i64(rows, "rows", 0);
  check_i64(rcount, "rcount", 1);
  TORCH_CHECK(rows.numel() <= N, "mikmeans: more candidate rows than labels");
  check_cuda(list, "list");
  TORCH_CHECK(list.scalar_type() == at::kInt && list.dim() == 2 && list.size(1) == 2 && list.is_contiguous(),
              "mikmeans: list must be contiguous int32 [cap, 2]");
  TORCH_CHECK(N < ((int64_t)1 << 31) && list.size(0) < ((int64_t)1 << 31), "mikmeans: shard too large");
  hip_check(mk::launch_label_delta_rows(labels.data_ptr<int32_t>(), prev.data_ptr<int32_t>(),
                                        rows.data_ptr<int64_t>(), rcount.data_ptr<int64_t>(), rows.numel(),
                                        (int2*)list.data_ptr<int32_t>(), (int)list.size(0),
                                        count.data_ptr<int32_t>(), stream()),
            "label_delta_rows");
}

void label_delta(const Tensor& labels, const Tensor& prev, const Tensor& list, const Tensor& count) {
  const int64_t N = labels.numel();
  check_i32(labels, "labels", N);
  check_i32(prev, "prev", N);
  check_i32(count, "count", 1);
  check_cuda(list, "list");
  TORCH_CHECK(list.scalar_type() == at::kInt && list.dim() == 2 && list.size(1) == 2 && list.is_contiguous(),
              "mikmeans: list must be contiguous int32 [cap, 2]");
  TORCH_CHECK(N < ((int64_t)1 << 31) && list.size(0) < ((int64_t)1 << 31), "mikmeans: shard too large");
  hip_check(mk::launch_label_delta(labels.data_ptr<int32_t>(), prev.data_ptr<int32_t>(), N,
                                   (int2*)list.data_ptr<int32_t>(), (int)list.size(0),
                                   count.data_ptr<int32_t>(), stream()),
            "label_delta");
}

// ... its scatter-add: +x to the new label, -x to the old one (all rows on overflow)
void update_delta(const Tensor& X, const Tensor& labels, int64_t K, const Tensor& slab,
                  const Tensor& cnt_slab, int64_t n_chunks, const c10::optional<Tensor>& weights,
                  const Tensor& col_exp, int64_t cnt_exp, const Tensor& list, const Tensor& count) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const int64_t N = X.size(0);
  const int D = (int)X.size(1);
  check_i32(labels, "labels", N);
  check_i32(count, "count", 1);
  check_cuda(list, "list");
  TORCH_CHECK(list.scalar_type() == at::kInt && list.dim() == 2 && list.size(1) == 2 && list.is_contiguous(),
              "mikmeans: list must be contiguous int32 [cap, 2]");
  const int sw = mk::update_slice_width(dt, (int)K, D, true);
  TORCH_CHECK(sw > 0, "mikmeans: incremental M-step needs an LDS slice (K too large)");
  TORCH_CHECK(n_chunks % 8 == 0, "mikmeans: bad n_chunks");
  check_i64(slab, "slab", n_chunks * K * D);
  check_i64(cnt_slab, "cnt_slab", n_chunks * K);
  if (weights.has_value()) check_f32(*weights, "weights", N);
  check_i32(col_exp, "col_exp", D);
  mk::UpdateArgs a;
  a.X = X.data_ptr(); a.N = N; a.D = D; a.ldx = ldx;
  a.labels = labels.data_ptr<int32_t>(); a.K = (int)K; a.n_chunks = (int)n_chunks;
  a.slab = (long long*)slab.data_ptr<int64_t>(); a.cnt_slab = (long long*)cnt_slab.data_ptr<int64_t>();
  a.weights = opt_ptr<const float>(weights);
  a.col_exp = col_exp.data_ptr<int32_t>(); a.cnt_exp = (int)cnt_exp; a.clamp = 0;
  a.dlist = (const int2*)list.data_ptr<int32_t>(); a.dcount = count.data_ptr<int32_t>();
  a.dcap = (int)list.size(0);
  hip_check(mk::launch_update(dt, a, stream()), "update_delta");
}

// ... and the running totals it feeds (tot = [K*D sums | K counts] int64)
void reduce_delta(const Tensor& slab, const Tensor& cnt_slab, int64_t n_chunks, int64_t K, int64_t D,
                  const c10::optional<Tensor>& slots, const Tensor& packed, const Tensor& col_exp,
                  int64_t cnt_exp, const Tensor& tot, const Tensor& count, int64_t cap) {
  check_i64(slab, "slab", n_chunks * K * D);
  check_i64(cnt_slab, "cnt_slab", n_chunks * K);
  check_f64(packed, "packed", K * D + K + 2);
  if (slots.has_value()) check_f64(*slots, "slots", mk::NSLOT * mk::SLOT_STRIDE);
  check_i32(col_exp, "col_exp", D);
  check_i64(tot, "tot", K * D + K);
  check_i32(count, "count", 1);
  hip_check(mk::launch_reduce((const long long*)slab.data_ptr<int64_t>(),
                              (const long long*)cnt_slab.data_ptr<int64_t>(), (int)n_chunks, (int)K,
                              (int)D, col_exp.data_ptr<int32_t>(), (int)cnt_exp, opt_ptr<double>(slots),
                              packed.data_ptr<double>(), stream(), (long long*)tot.data_ptr<int64_t>(),
                              count.data_ptr<int32_t>(), (int)cap),
            "reduce_delta");
}

void reduce(const Tensor& slab, const Tensor& cnt_slab, int64_t n_chunks, int64_t K, int64_t D,
            const c10::optional<Tensor>& slots, const Tensor& packed, const Tensor& col_exp,
            int64_t cnt_exp) {
  check_i64(slab, "slab", n_chunks * K * D);
  check_i64(cnt_slab, "cnt_slab", n_chunks * K);
  check_f64(packed, "packed", K * D + K + 2);
  if (slots.has_value()) check_f64(*slots, "slots", mk::NSLOT * mk::SLOT_STRIDE);
  check_i32(col_exp, "col_exp", D);
  hip_check(mk::launch_reduce((const long long*)slab.data_ptr<int64_t>(),
                              (const long long*)cnt_slab.data_ptr<int64_t>(), (int)n_chunks, (int)K,
                              (int)D, col_exp.data_ptr<int32_t>(), (int)cnt_exp, opt_ptr<double>(slots),
                              packed.data_ptr<double>(), stream()),
            "reduce");
}

// Wide-range column lo sums: out[k*nw + j] = 2^-exps[j] * sum_c slab[c][k][cols[j]].
void reduce_cols(const Tensor& slab, int64_t n_chunks, int64_t K, int64_t D, const Tensor& cols,
                 const Tensor& exps, const Tensor& out) {
  check_i64(slab, "slab", n_chunks * K * D);
  const int64_t nw = cols.numel();
  check_i32(cols, "cols", nw);
  check_i32(exps, "exps", nw);
  check_f64(out, "out", K * nw);
  // (column indices are validated once by the engine: no host read here, the call is graph-captured)
  hip_check(mk::launch_reduce_cols((const long long*)slab.data_ptr<int64_t>(), (int)n_chunks, (int)K, (int)D,
                                   cols.data_ptr<int32_t>(), exps.data_ptr<int32_t>(), (int)nw,
                                   out.data_ptr<double>(), stream()),
            "reduce_cols");
}

void finalize(int64_t mode, const c10::optional<Tensor>& packed, const Tensor& Cold,
              const c10::optional<Tensor>& Cnew, const c10::optional<Tensor>& frozen,
              const c10::optional<Tensor>& mb_counts, const Tensor& pack, const Tensor& cn,
              const c10::optional<Tensor>& shift, const c10::optional<Tensor>& counts,
              int64_t dpad, int64_t Kpad, const c10::optional<Tensor>& qshift) {
  check_f32(Cold, "C");
  TORCH_CHECK(Cold.dim() == 2, "mikmeans: C must be [K, D]");
  const int K = (int)Cold.size(0), D = (int)Cold.size(1);
  const int dt = pack.scalar_type() == at::kBFloat16 ? mk::DT_BF16 : mk::DT_F32;
  TORCH_CHECK(mk::assign_kpad(dt, (int)dpad, K) == Kpad, "mikmeans: bad Kpad");
  TORCH_CHECK(D <= dpad, "mikmeans: D > dpad");
  check_cuda(pack, "pack");
  TORCH_CHECK(pack.is_contiguous() && pack.numel() >= Kpad * dpad, "mikmeans: pack too small");
  check_f32(cn, "cn", mk::assign_cn_len((int)Kpad));
  if (mode != mk::FIN_PACK_ONLY) {
    TORCH_CHECK(packed.has_value(), "mikmeans: finalize needs the packed message");
    check_f64(*packed, "packed", (int64_t)K * D + K + 2);
  }
  if (mode == mk::FIN_MINIBATCH) {
    TORCH_CHECK(mb_counts.has_value(), "mikmeans: minibatch finalize needs counts");
    check_f64(*mb_counts, "mb_counts", K);
  }
  if (Cnew.has_value()) check_f32(*Cnew, "Cnew", (int64_t)K * D);
  if (shift.has_value()) check_f32(*shift, "shift", K);
  if (counts.has_value()) check_f32(*counts, "counts", K);
  if (qshift.has_value()) check_f32(*qshift, "qshift", K);
  if (frozen.has_value())
    TORCH_CHECK(frozen->is_cuda() && frozen->scalar_type() == at::kByte && frozen->numel() >= K,
                "mikmeans: frozen must be uint8 [K]");
  mk::FinalizeArgs a;
  a.packed = opt_ptr<const double>(packed);
  a.Cold = Cold.data_ptr<float>(); a.Cnew = opt_ptr<float>(Cnew); a.K = K; a.D = D;
  a.frozen = opt_ptr<const uint8_t>(frozen);
  a.mb_counts = opt_ptr<double>(mb_counts);
  a.dtype = dt; a.dpad = (int)dpad; a.Kpad = (int)Kpad;
  a.pack = pack.data_ptr(); a.cn = cn.data_ptr<float>();
  a.shift = opt_ptr<float>(shift); a.counts_out = opt_ptr<float>(counts);
  a.qshift = opt_ptr<float>(qshift);
  a.mode = (int)mode;
  hip_check(mk::launch_finalize(a, stream()), "finalize");
}

void row_sqnorm(const Tensor& X, const Tensor& out) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  check_f32(out, "out", X.size(0));
  hip_check(mk::launch_row_sqnorm(dt, X.data_ptr(), X.size(0), (int)X.size(1), ldx,
                                  out.data_ptr<float>(), stream()),
            "row_sqnorm");
}

// out: int32 [D] zero-filled by the caller; receives max |x[:, d]| as float bit patterns.
// Optional column statistics (all three or none): fstats f64 [3, D] (sum |x|, sum x,
// sum x^2) and nnz int64 [D] zero-filled, lowbit int32 [D] filled with INT_MAX.
void col_absmax(const Tensor& X, const Tensor& out, const c10::optional<Tensor>& fstats,
                const c10::optional<Tensor>& nnz, const c10::optional<Tensor>& lowbit,
                const c10::optional<Tensor>& xn) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  check_cuda(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kInt && out.is_contiguous() && out.numel() == X.size(1),
              "mikmeans: col_absmax out must be int32 [D]");
  TORCH_CHECK(fstats.has_value() == nnz.has_value() && fstats.has_value() == lowbit.has_value(),
              "mikmeans: col_absmax statistics come together (fstats, nnz, lowbit)");
  if (fstats.has_value()) {
    check_f64(*fstats, "fstats", 3 * X.size(1));
    check_i64(*nnz, "nnz", X.size(1));
    check_i32(*lowbit, "lowbit", X.size(1));
  }
  if (xn.has_value()) {
    check_f32(*xn, "xn", X.size(0));
    TORCH_CHECK(X.size(1) <= 64 * (dt == mk::DT_BF16 ? 8 : 4), "mikmeans: fused row norms up to 64 pieces per row");
  }
  // per-block partial sums, summed in a fixed order by the launcher (bitwise reproducible)
  Tensor fpart;
  if (fstats.has_value())
    fpart = at::zeros({(int64_t)mk::colstat_rows(dt, X.size(0), (int)X.size(1)) * 3 * X.size(1)},
                      X.options().dtype(at::kDouble));
  hip_check(mk::launch_col_absmax(dt, X.data_ptr(), X.size(0), (int)X.size(1), ldx,
                                  reinterpret_cast<uint32_t*>(out.data_ptr<int32_t>()), stream(),
                                  opt_ptr<double>(fstats), opt_ptr<unsigned long long>(nnz),
                                  opt_ptr<int>(lowbit), fstats.has_value() ? fpart.data_ptr<double>() : nullptr,
                                  opt_ptr<float>(xn)),
            "col_absmax");
}

// Mini-batch sampler (csrc/rows.hip): out[:b] = X[philox indices of (seed, rank, step)].
void sample_rows(const Tensor& X, const Tensor& out, int64_t b, int64_t seed, int64_t rank, int64_t step,
                 const c10::optional<Tensor>& xn, const c10::optional<Tensor>& idx_out) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const int64_t ldo = check_points(out, dt);
  TORCH_CHECK(out.scalar_type() == X.scalar_type() && out.size(1) == X.size(1), "mikmeans: sample_rows out must match X");
  TORCH_CHECK(b >= 0 && b <= out.size(0) && b < ((int64_t)1 << 32), "mikmeans: sample_rows batch out of range");
  TORCH_CHECK(b == 0 || X.size(0) > 0, "mikmeans: sample_rows from an empty shard");
  TORCH_CHECK(rank >= 0 && step >= 0 && step < ((int64_t)1 << 32), "mikmeans: sample_rows rank/step range");
  if (xn.has_value()) check_f32(*xn, "xn", b);
  if (idx_out.has_value()) check_i64(*idx_out, "idx_out", b);
  hip_check(mk::launch_sample_rows(dt, X.data_ptr(), X.size(0), ldx, (int)X.size(1), out.data_ptr(), ldo, b,
                                   (uint64_t)seed, (uint32_t)rank, (uint32_t)step, opt_ptr<float>(xn),
                                   opt_ptr<int64_t>(idx_out), stream()),
            "sample_rows");
}

void sample_index(int64_t n, int64_t b, int64_t seed, int64_t rank, int64_t step, const Tensor& idx) {
  check_i64(idx, "idx", b);
  TORCH_CHECK(b >= 0 && b < ((int64_t)1 << 32) && rank >= 0 && step >= 0 && step < ((int64_t)1 << 32),
              "mikmeans: sample_index range");
  TORCH_CHECK(b == 0 || n > 0, "mikmeans: sample_index from an empty shard");
  hip_check(mk::launch_sample_index(n, b, (uint64_t)seed, (uint32_t)rank, (uint32_t)step,
                                    idx.data_ptr<int64_t>(), stream()),
            "sample_index");
}

void row_normalize(const Tensor& X, const c10::optional<Tensor>& xn) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  if (xn.has_value()) check_f32(*xn, "xn", X.size(0));
  hip_check(mk::launch_row_normalize(dt, X.data_ptr(), X.size(0), (int)X.size(1), ldx, opt_ptr<float>(xn), stream()),
            "row_normalize");
}

void wdot(const Tensor& a, const Tensor& b, const Tensor& out, const Tensor& scratch) {
  check_f32(a, "a");
  check_f32(b, "b", a.numel());
  check_f64(out, "out", 1);
  check_f64(scratch, "scratch", mk::wdot_scratch_len());
  hip_check(mk::launch_wdot(a.data_ptr<float>(), b.data_ptr<float>(), a.numel(), out.data_ptr<double>(),
                            scratch.data_ptr<double>(), stream()),
            "wdot");
}

void kpp_d2(const Tensor& X, const Tensor& c, bool first, const Tensor& d2, const Tensor& block_sums,
            int64_t rows_per_block, const c10::optional<Tensor>& owner, const c10::optional<Tensor>& cc,
            int64_t kcc, int64_t knew) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const int64_t N = X.size(0);
  check_f32(c, "c", X.size(1));
  check_f32(d2, "d2", N);
  const int64_t nb = (N + rows_per_block - 1) / rows_per_block;
  check_f64(block_sums, "block_sums", nb);
  int32_t* own = nullptr;
  const float* ccp = nullptr;
  if (owner.has_value() && owner->defined()) {
    // pruned pass: owner values are centre indices < cc.numel() (the kernel gathers cc[owner[i]])
    TORCH_CHECK(!first, "mikmeans: the first k-means++ pass cannot be pruned");
    check_i32(*owner, "owner", N);
    TORCH_CHECK(cc.has_value() && cc->defined(), "mikmeans: a pruned kpp_d2 needs cc");
    check_f32(*cc, "cc", 1);
    TORCH_CHECK(knew < cc->numel() && kcc >= 1 && kcc <= cc->numel(), "mikmeans: bad k for cc");
    own = owner->data_ptr<int32_t>();
    ccp = cc->data_ptr<float>();
  }
  hip_check(mk::launch_kpp_d2(dt, X.data_ptr(), N, (int)X.size(1), ldx, c.data_ptr<float>(),
                              first ? 1 : 0, d2.data_ptr<float>(), block_sums.data_ptr<double>(),
                              rows_per_block, (int)nb, stream(), own, ccp, (int)kcc, (int)knew),
            "kpp_d2");
}

void kpp_cc(const Tensor& centers, int64_t k, const Tensor& cnew, const Tensor& cc) {
  check_f32(centers, "centers");
  TORCH_CHECK(centers.dim() == 2 && k >= 0 && k <= centers.size(0), "mikmeans: kpp_cc needs k <= K");
  check_f32(cnew, "cnew", centers.size(1));
  check_f32(cc, "cc", k);
  hip_check(mk::launch_kpp_cc(centers.data_ptr<float>(), centers.size(1), (int)k, (int)centers.size(1),
                              cnew.data_ptr<float>(), cc.data_ptr<float>(), stream()),
            "kpp_cc");
}

// Weighted k-means++ draws over a candidate set (csrc/kpp.hip wkpp): `steps` draws into out
void wkpp(const Tensor& Ct, const Tensor& w, const Tensor& d2, const Tensor& cum, const Tensor& part,
          const Tensor& u, const Tensor& state, const Tensor& out, int64_t steps) {
  check_cuda(Ct, "Ct");
  TORCH_CHECK(Ct.scalar_type() == at::kFloat && Ct.dim() == 2 && Ct.is_contiguous(),
              "mikmeans: Ct must be contiguous f32 [D, M]");
  const int64_t D = Ct.size(0), M = Ct.size(1);
  TORCH_CHECK(M >= 1 && D >= 1 && D <= 8192, "mikmeans: bad candidate set [", D, ", ", M, "]");
  check_f64(w, "w", M);
  check_f64(d2, "d2", M);
  check_f64(cum, "cum", M);
  check_f64(part, "part", (M + 255) / 256);
  check_f64(u, "u", 1);
  check_i64(state, "state", 2);
  check_f32(out, "out", 1);
  TORCH_CHECK(out.dim() == 2 && out.size(1) >= D && out.stride(1) == 1, "mikmeans: out must be f32 [K, >=D]");
  TORCH_CHECK(steps >= 0 && steps <= out.size(0) && steps <= u.numel(), "mikmeans: more steps than draws");
  hip_check(mk::launch_wkpp(Ct.data_ptr<float>(), M, (int)D, w.data_ptr<double>(), d2.data_ptr<double>(),
                            cum.data_ptr<double>(), part.data_ptr<double>(), u.data_ptr<double>(),
                            state.data_ptr<int64_t>(), out.data_ptr<float>(), out.stride(0), (int)steps, stream()),
            "wkpp");
}

void kpp_sample(const Tensor& block_sums, const Tensor& d2, int64_t rows_per_block,
                const Tensor& target, const Tensor& X, const Tensor& crow,
                const c10::optional<Tensor>& idx_out, int64_t mode,
                const c10::optional<Tensor>& totals_all, int64_t rank) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const int64_t N = X.size(0);
  const int64_t nb = (N + rows_per_block - 1) / rows_per_block;
  check_f64(block_sums, "block_sums", nb);
  check_f32(d2, "d2", N);
  check_f64(target, "target", 1);
  check_f32(crow, "crow", X.size(1));
  if (idx_out.has_value())
    TORCH_CHECK(idx_out->is_cuda() && idx_out->scalar_type() == at::kLong, "idx_out must be int64");
  TORCH_CHECK(N > 0, "mikmeans: kpp_sample on an empty shard");
  TORCH_CHECK(mode >= 0 && mode <= 2, "mikmeans: kpp_sample mode");
  int world = 1;
  if (mode == 2) {
    TORCH_CHECK(totals_all.has_value(), "mikmeans: mode 2 needs totals_all");
    check_f64(*totals_all, "totals_all", 1);
    world = (int)totals_all->numel();
    TORCH_CHECK(rank >= 0 && rank < world, "mikmeans: bad rank");
  }
  hip_check(mk::launch_kpp_sample(dt, block_sums.data_ptr<double>(), (int)nb, d2.data_ptr<float>(),
                                  N, rows_per_block, target.data_ptr<double>(), X.data_ptr(),
                                  (int)X.size(1), ldx, crow.data_ptr<float>(),
                                  opt_ptr<int64_t>(idx_out), (int)mode, opt_ptr<double>(totals_all),
                                  world, (int)rank, stream()),
            "kpp_sample");
}

void blob_centers(const Tensor& centers, double box, int64_t seed) {
  check_f32(centers, "centers");
  TORCH_CHECK(centers.dim() == 2, "centers must be [C, D]");
  hip_check(mk::launch_blob_centers(centers.data_ptr<float>(), (int)centers.size(0),
                                    (int)centers.size(1), (float)box, (uint64_t)seed, stream()),
            "blob_centers");
}

void blobs(const Tensor& X, int64_t i0, const Tensor& centers, double stddev, int64_t seed,
           const c10::optional<Tensor>& y, const c10::optional<Tensor>& xn) {
  const int dt = dtype_of(X);
  check_cuda(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "X must be 2-D with unit column stride");
  check_f32(centers, "centers");
  TORCH_CHECK(centers.dim() == 2 && centers.size(1) == X.size(1), "centers must be [C, D]");
  if (y.has_value())
    TORCH_CHECK(y->is_cuda() && y->scalar_type() == at::kInt && y->numel() >= X.size(0),
                "y must be int32 [n]");
  if (xn.has_value()) check_f32(*xn, "xn", X.size(0));
  const int64_t ldx = X.size(0) <= 1 ? X.size(1) : X.stride(0);
  hip_check(mk::launch_blobs(dt, X.data_ptr(), i0, X.size(0), (int)X.size(1), ldx,
                             centers.data_ptr<float>(), (int)centers.size(0), (float)stddev,
                             (uint64_t)seed, opt_ptr<int32_t>(y), opt_ptr<float>(xn), stream()),
            "blobs");
}

// Page-lock a host tensor in place (out-of-core streaming: async H2D DMA straight from the
// caller's rows, no pinned copy of a shard that may be hundreds of GB).  False when the
// range was already registered / pinned.
bool host_register(const Tensor& t) {
  TORCH_CHECK(!t.is_cuda() && t.is_contiguous(), "mikmeans: host_register needs a contiguous CPU tensor");
  if (t.nbytes() == 0) return false;
  const hipError_t e = hipHostRegister(t.data_ptr(), t.nbytes(), hipHostRegisterDefault);
  if (e == hipErrorHostMemoryAlreadyRegistered) { (void)hipGetLastError(); return false; }
  hip_check(e, "hipHostRegister");
  return true;
}
void host_unregister(const Tensor& t) {
  hip_check(hipHostUnregister(t.data_ptr()), "hipHostUnregister");
}

}  // namespace

namespace mk {
// The A/B switch registry (kernels.h): environment read once at load, then set_variant only.
static const char* const kVariantEnv[V_COUNT] = {"MIKMEANS_ASSIGN_VARG", "MIKMEANS_ASSIGN_PMAJ",
                                                 "MIKMEANS_ASSIGN_GEOM", "MIKMEANS_UPDATE_KS",
                                                 "MIKMEANS_UPDATE_KS_GM", "MIKMEANS_BLOBS_TPR",
                                                 "MIKMEANS_ASSIGN_TOP2_GEOM", "MIKMEANS_ASSIGN_EPI",
                                                 "MIKMEANS_ASSIGN_EARLY", "MIKMEANS_COLSTAT_BLOCKS"};
static int* variant_table() {
  static int t[V_COUNT] = {};
  static const bool init = [] {
    for (int i = 0; i < V_COUNT; ++i) {
      const char* e = getenv(kVariantEnv[i]);
      t[i] = (e && *e) ? atoi(e) : -1;
    }
    return true;
  }();
  (void)init;
  return t;
}
int variant(Variant v) { return variant_table()[v]; }
void set_variant(Variant v, int value) { variant_table()[v] = value; }
}  // namespace mk

namespace {

// Hamerly bounds step (csrc/rows.hip): work = 4 floats of device scratch (top-2 shifts, the
// largest's centre, max |c|^2).
void compact(const Tensor& cand, const Tensor& rows, const Tensor& count, const Tensor& scratch) {
  check_cuda(cand, "cand");
  TORCH_CHECK(cand.scalar_type() == at::kByte && cand.is_contiguous(), "mikmeans: cand must be contiguous uint8");
  const int64_t n = cand.numel();
  check_i64(rows, "rows", n);
  check_i64(count, "count", 1);
  check_i64(scratch, "scratch", mk::compact_blocks(n));
  hip_check(mk::launch_compact(cand.data_ptr<uint8_t>(), n, rows.data_ptr<int64_t>(), count.data_ptr<int64_t>(),
                               scratch.data_ptr<int64_t>(), stream()),
            "compact");
}

void kpar_select(const Tensor& d2, int64_t start, const Tensor& psi, double ell, int64_t seed, int64_t round,
                 const Tensor& cand) {
  const int64_t n = d2.numel();
  check_f32(d2, "d2", n);
  check_f64(psi, "psi", 1);
  check_cuda(cand, "cand");
  TORCH_CHECK(cand.scalar_type() == at::kByte && cand.is_contiguous() && cand.numel() >= n,
              "mikmeans: cand must be contiguous uint8 [n]");
  hip_check(mk::launch_kpar_select(d2.data_ptr<float>(), n, start, psi.data_ptr<double>(), ell, (uint64_t)seed,
                                   (uint32_t)round, cand.data_ptr<uint8_t>(), stream()),
            "kpar_select");
}

void tighten(const Tensor& X, int64_t D, const Tensor& labels, const Tensor& C, const Tensor& rows,
             const Tensor& count, const Tensor& ub, const Tensor& lb, const Tensor& cand, const Tensor& xn,
             const Tensor& work, const c10::optional<Tensor>& oseed) {
  const int dt = dtype_of(X);
  const int64_t ldx = check_points(X, dt);
  const int64_t n = X.size(0);
  TORCH_CHECK(D >= 1 && D <= X.size(1), "mikmeans: bad D");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= n,
              "mikmeans: labels must be contiguous int32 [n]");
  check_cuda(C, "C");
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.dim() == 2 && C.stride(1) == 1 && C.size(1) >= D,
              "mikmeans: C must be f32 [K, >=D] with unit column stride");
  check_i64(rows, "rows", 0);
  TORCH_CHECK(rows.numel() <= n, "mikmeans: more candidate rows than X rows");
  check_i64(count, "count", 1);
  check_f32(ub, "ub", n);
  check_f32(lb, "lb", n);
  check_cuda(cand, "cand");
  TORCH_CHECK(cand.scalar_type() == at::kByte && cand.is_contiguous() && cand.numel() >= n,
              "mikmeans: cand must be contiguous uint8 [n]");
  check_f32(xn, "xn", n);
  check_f32(work, "work", 4);
  if (oseed.has_value()) check_f32(*oseed, "oseed", n);
  hip_check(mk::launch_tighten(dt, X.data_ptr(), ldx, (int)D, labels.data_ptr<int32_t>(), C.data_ptr<float>(),
                               C.stride(0), rows.data_ptr<int64_t>(), count.data_ptr<int64_t>(), rows.numel(),
                               ub.data_ptr<float>(), lb.data_ptr<float>(), cand.data_ptr<uint8_t>(),
                               xn.data_ptr<float>(), work.data_ptr<float>(), opt_ptr<const float>(oseed), stream()),
            "tighten");
}

// oseed = the full assign's per-row seed offsets (bf16 keys) for rows with norms xn
void seed_offsets(const Tensor& xn, const Tensor& oseed, int64_t block_rows) {
  const int64_t n = xn.numel();
  check_f32(xn, "xn", n);
  check_f32(oseed, "oseed", n);
  TORCH_CHECK(block_rows > 0 && block_rows <= 4096, "mikmeans: bad block_rows ", block_rows);
  hip_check(mk::launch_seed_offsets(xn.data_ptr<float>(), n, (int)block_rows, oseed.data_ptr<float>(), stream()),
            "seed_offsets");
}

void bounds_update(const Tensor& labels, const Tensor& ub, const Tensor& lb, const Tensor& shift2, const Tensor& cn,
                   const Tensor& xn, const Tensor& cand, const Tensor& work, const c10::optional<Tensor>& oseed,
                   int64_t nterms) {
  const int64_t n = labels.numel();
  const int K = (int)shift2.numel();
  check_i32(labels, "labels", n);
  check_f32(ub, "ub", n);
  check_f32(lb, "lb", n);
  check_f32(xn, "xn", n);
  check_f32(shift2, "shift2", 1);
  check_f32(cn, "cn", K);
  check_f32(work, "work", 4);
  if (oseed.has_value()) check_f32(*oseed, "oseed", n);
  TORCH_CHECK(nterms >= 1 && nterms <= 1 << 20, "mikmeans: bad nterms");
  check_cuda(cand, "cand");
  TORCH_CHECK(cand.scalar_type() == at::kByte && cand.is_contiguous() && cand.numel() >= n,
              "mikmeans: cand must be contiguous uint8 [n]");
  hip_check(mk::launch_bounds_update(labels.data_ptr<int32_t>(), ub.data_ptr<float>(), lb.data_ptr<float>(),
                                     shift2.data_ptr<float>(), cn.data_ptr<float>(), K, xn.data_ptr<float>(), n,
                                     cand.data_ptr<uint8_t>(), work.data_ptr<float>(), opt_ptr<const float>(oseed),
                                     (int)nterms, stream()),
            "bounds_update");
}

// Tear down a stream capture that an error left open.  When a capture is invalidated,
// hipStreamEndCapture inside torch's capture_end can fail and leave the stream in the
// capturing state; every later launch on the legacy stream then fails with "operation
// failed due to a previous error during capture".  Ends it (discarding any partial graph)
// and clears the error state.  Returns the capture status found (0 = none).
int capture_teardown(int64_t stream_ptr) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream_ptr);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) { (void)hipGetLastError(); return -1; }
  if (st != hipStreamCaptureStatusNone) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(s, &g);
    if (g) (void)hipGraphDestroy(g);
  }
  (void)hipGetLastError();
  return (int)st;
}

std::string js_format(double v) {
  std::string s;
  mk::js_number(v, s);
  return s;
}

// Flat JSON array of a CPU float32/float64 tensor, each value widened to f64
// (what JSON.stringify(Array.from(Float32Array)) prints), no spaces.
std::string js_array(const Tensor& t) {
  TORCH_CHECK(!t.is_cuda(), "js_array expects a CPU tensor");
  Tensor c = t.contiguous().view(-1);
  std::string s;
  s.reserve((size_t)c.numel() * 12 + 2);
  s += '[';
  const int64_t n = c.numel();
  if (c.scalar_type() == at::kFloat) {
    const float* p = c.data_ptr<float>();
    for (int64_t i = 0; i < n; ++i) { if (i) s += ','; mk::js_number((double)p[i], s); }
  } else {
    TORCH_CHECK(c.scalar_type() == at::kDouble, "js_array: float32 or float64 only");
    const double* p = c.data_ptr<double>();
    for (int64_t i = 0; i < n; ++i) { if (i) s += ','; mk::js_number(p[i], s); }
  }
  s += ']';
  return s;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "mikmeans native ops (gfx950 HIP kernels + host helpers)";
  m.def("kpar_select", &kpar_select, "k-means|| oversampling flags (philox keyed by the global row)");
  m.def("tighten", &tighten, "Hamerly tightening: exact distance to the label's centre for the candidates");
  m.def("compact", &compact, "rows of the nonzero flags, ascending; count on the device");
  m.def("compact_blocks", &mk::compact_blocks);
  m.def("assign", &assign, "fused MFMA distance + argmin (K2)", py::arg("X"), py::arg("pack"), py::arg("cn"),
        py::arg("xn"), py::arg("labels"), py::arg("mind"), py::arg("slots"), py::arg("Kpad"), py::arg("dpad"),
        py::arg("track_changed"), py::arg("keys") = py::none(), py::arg("rows") = py::none(),
        py::arg("ub") = py::none(), py::arg("lb") = py::none(), py::arg("scatter") = false,
        py::arg("count") = py::none(), py::arg("oseed") = py::none());
  m.def("seed_offsets", &seed_offsets, "the full assign's per-row bf16 seed offsets (bounded E-step)");
  m.def("assign_block_rows", [](int64_t dt, int64_t dpad, int64_t kpad) {
    return mk::assign16_block_rows((int)dt, (int)dpad, (int)kpad);
  }, "rows per workgroup of the full assign (its seed-offset block)");
  m.def("update", &update, "LDS-privatised per-cluster sums/counts (K3)", py::arg("X"), py::arg("labels"),
        py::arg("K"), py::arg("slab"), py::arg("cnt_slab"), py::arg("n_chunks"), py::arg("weights"),
        py::arg("col_exp"), py::arg("cnt_exp"), py::arg("clamp"), py::arg("clamp_count") = py::none(),
        py::arg("col_exp2") = py::none(), py::arg("rows") = py::none());
  m.def("transform", &transform, "distances of every row to every centre on the MFMA tiles", py::arg("X"),
        py::arg("pack"), py::arg("cn"), py::arg("K"), py::arg("Kpad"), py::arg("dpad"), py::arg("xn"), py::arg("out"),
        py::arg("squared") = false);
  m.def("reduce_cols", &reduce_cols, "lo sums of the wide-range columns (residual pass)");
  m.def("reduce", &reduce, "slab reduction into the packed f64 all-reduce message");
  m.def("label_delta", &label_delta, "changed-row list for the incremental M-step");
  m.def("label_delta_rows", &label_delta_rows, "changed-row list over a candidate list (bounded E-step)");
  m.def("update_delta", &update_delta, "incremental M-step scatter-add (+new / -old label)");
  m.def("reduce_delta", &reduce_delta, "slab reduction into running totals + packed message");
  m.def("finalize", &finalize, "new centroids, shift, fragment re-pack (K4)", py::arg("mode"), py::arg("packed"),
        py::arg("Cold"), py::arg("Cnew"), py::arg("frozen"), py::arg("mb_counts"), py::arg("pack"), py::arg("cn"),
        py::arg("shift"), py::arg("counts"), py::arg("dpad"), py::arg("Kpad"), py::arg("qshift") = py::none());
  m.def("row_sqnorm", &row_sqnorm, "row squared norms (K1)");
  m.def("col_absmax", &col_absmax,
        "per-column max |x| as f32 bit patterns (+ optional sum |x|, nonzero count, lowest-bit exponent)",
        py::arg("X"), py::arg("out"), py::arg("fstats") = py::none(), py::arg("nnz") = py::none(),
        py::arg("lowbit") = py::none(), py::arg("xn") = py::none());
  m.attr("COLSTAT_FUSED_PIECES") = 64;
  m.def("sample_rows", &sample_rows, "mini-batch rows X[philox(seed; j, step, rank) * n] (+ norms, indices)",
        py::arg("X"), py::arg("out"), py::arg("b"), py::arg("seed"), py::arg("rank"), py::arg("step"),
        py::arg("xn") = py::none(), py::arg("idx_out") = py::none());
  m.def("sample_index", &sample_index, "the mini-batch sampler's source rows of one step (int64 [b])");
  m.def("row_normalize", &row_normalize, "in-place unit rows (cosine metric)", py::arg("X"), py::arg("xn") = py::none());
  m.def("wdot", &wdot, "out[0] += sum a*b in f64, fixed order (weighted inertia)");
  m.attr("WDOT_SCRATCH") = mk::wdot_scratch_len();
  m.def("kpp_d2", &kpp_d2, "k-means++ D^2 update (K5; triangle-inequality pruned with owner/cc)",
        py::arg("X"), py::arg("c"), py::arg("first"), py::arg("d2"), py::arg("block_sums"),
        py::arg("rows_per_block"), py::arg("owner") = py::none(), py::arg("cc") = py::none(),
        py::arg("kcc") = 0, py::arg("knew") = -1);
  m.def("wkpp", &wkpp, "weighted k-means++ draws over a candidate set (k-means|| recluster)");
  m.def("kpp_cc", &kpp_cc, "centre-centre squared distances for the pruned K5 pass");
  m.def("kpp_sample", &kpp_sample, "k-means++ D^2 sampling (K6)");
  m.def("blob_centers", &blob_centers, "Philox blob centres");
  m.def("blobs", &blobs, "Philox Gaussian blobs (K8)");
  m.def("assign_kpad", [](int64_t dt, int64_t dpad, int64_t K) { return mk::assign_kpad((int)dt, (int)dpad, (int)K); });
  m.def("assign16_supported", [](int64_t dt, int64_t dpad) { return mk::assign16_chunk_tiles((int)dt, (int)dpad) > 0; });
  m.def("set_update_max_sw", [](int64_t sw) { mk::set_update_max_sw((int)sw); },
        "cap the M-step slice width (smaller LDS footprint for overlap with assign)");
  m.def("assign_cn_len", [](int64_t kpad) { return mk::assign_cn_len((int)kpad); });
  m.def("update_slice_width", [](int64_t dt, int64_t K, int64_t D, bool w) { return mk::update_slice_width((int)dt, (int)K, (int)D, w); },
        py::arg("dtype"), py::arg("K"), py::arg("D"), py::arg("weighted") = false);
  m.def("update_n_chunks", [](int64_t dt, int64_t K, int64_t D, int64_t N, bool w) { return mk::update_n_chunks((int)dt, (int)K, (int)D, N, w); },
        py::arg("dtype"), py::arg("K"), py::arg("D"), py::arg("N"), py::arg("weighted") = false);
  m.def("fixed_exp", [](double maxabs) { return mk::fixed_exp(maxabs); },
        "fixed-point exponent e with maxabs * 2^e <= 2^30 (M-step accumulators)");
  m.def("host_register", &host_register, "page-lock a CPU tensor in place (hipHostRegister)");
  m.def("host_unregister", &host_unregister, "undo host_register");
  m.def("variant_names", []() {
    std::vector<std::string> n;
    for (int i = 0; i < mk::V_COUNT; ++i) n.emplace_back(mk::kVariantEnv[i] + 9);   // strip "MIKMEANS_"
    return n;
  }, "A/B switch names (lower-cased by mikmeans.ops.native)");
  m.def("set_assign_timeline", [](c10::optional<torch::Tensor> buf) {
    // the binding holds a reference while the hook is armed: a caller that drops its buffer
    // cannot leave later launches writing into memory the caching allocator handed on
    static torch::Tensor held;
    if (!buf.has_value()) { mk::set_assign_timeline(nullptr, 0); held = torch::Tensor(); return; }
    TORCH_CHECK(buf->is_cuda() && buf->scalar_type() == torch::kInt64 && buf->is_contiguous(),
                "mikmeans: timeline buffer must be a contiguous int64 CUDA tensor");
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    TORCH_CHECK(buf->get_device() == dev, "mikmeans: timeline buffer on device ", buf->get_device(),
                ", launches run on device ", dev);
    held = *buf;
    mk::set_assign_timeline((unsigned long long*)held.data_ptr<int64_t>(), held.numel() / 8);
  }, py::arg("buf"));
  m.def("get_variant", [](int64_t i) {
    TORCH_CHECK(i >= 0 && i < mk::V_COUNT, "mikmeans: no A/B switch ", i);
    return mk::variant((mk::Variant)i);
  });
  m.def("set_variant", [](int64_t i, int64_t v) {
    TORCH_CHECK(i >= 0 && i < mk::V_COUNT, "mikmeans: no A/B switch ", i);
    mk::set_variant((mk::Variant)i, (int)v);
  },
        "set an A/B switch (-1 = built-in rule); launchers never read the environment");
  (void)mk::variant(mk::V_ASSIGN_VARG);   // snapshot the environment now, at load
  m.def("bounds_update", &bounds_update, "Hamerly bounds moved by the centre shifts; flags the rows to re-assign");
  m.def("capture_teardown", &capture_teardown, "end a stream capture an error left open (status found)");
  m.def("js_format", &js_format, "ECMAScript Number::toString of a double");
  m.def("js_array", &js_array, "JSON array of a CPU float tensor with JS number formatting");
  m.def("colstat_rows", &mk::colstat_rows, "f64 partial rows one column-statistics pass of N rows writes");
  m.attr("NSLOT") = mk::NSLOT;
  m.attr("SLOT_STRIDE") = mk::SLOT_STRIDE;
}
