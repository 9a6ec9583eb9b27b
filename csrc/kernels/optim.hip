// Flat-buffer optimizer kernels for the ZeRO engine (gfx950).
//
// The ZeRO engine keeps every rank's optimizer partition (fp32 master, exp_avg,
// exp_avg_sq, fp32 grad) as ONE contiguous buffer each, so the whole update is
// a single launch instead of DeepSpeed's multi_tensor_apply chunk lists
// (§2.6 K1, K2, K8):
//   * grad_stats   : sum(g^2) and count(!isfinite(g)) in one pass (two tiny
//                    deterministic launches: per-block partials, then a final sum).
//                    Feeds gradient clipping, the fp16 loss scaler and the NaN trap.
//   * adamw_step   : decoupled-weight-decay Adam; reads the clip coefficient and
//                    the overflow flag from the device stats buffer, so a step has
//                    NO host synchronisation; writes the bf16 compute copy of the
//                    parameter in the same pass (the all-gather source under ZeRO-3).
//   * accumulate   : dst(fp32) = beta*dst + alpha*src(bf16|fp32) -- gradient
//                    accumulation of a bf16 micro-batch grad into the fp32 shard.
//   * cast_f32_bf16: master -> compute copy (after load / init).
// All are HBM-streaming: float4 / bf16x4 per lane; AdamW launches one vector per lane (no grid-stride reuse).
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

constexpr int kThreads = 256;

// Streaming launches give every lane one 16-byte vector per operand (the kernels keep a grid-stride loop, so
// the clamp only bounds the block index): AdamW 6.04 TB/s this way vs 5.51 TB/s with 8 workgroups per CU
// looping, same arithmetic and bit-identical results (profiles/adamw_stats_grid_ab_r04.jsonl)
// HIP on AMD needs gridDim.x * blockDim.x <= UINT32_MAX: cap the grid there (2^24 blocks of 256 lanes; the loop covers
// the rest of a flat buffer over 2^34 elements)
int64_t stream_grid(int64_t n_vec) {
  const int64_t b = (n_vec + kThreads - 1) / kThreads;
  return std::max<int64_t>(1, std::min<int64_t>(b, (int64_t)(UINT32_MAX / kThreads)));
}

// grad_stats: 8 vectors in flight per lane, up to 16 workgroups per CU and per tensor (pure-read sweep of 4 GiB of
// fp32: 6.43 TB/s vs 5.17 TB/s at 4 vectors, 4 workgroups per CU and ordinary loads,
// profiles/adamw_stats_grid_ab_r04.jsonl)
constexpr int kStatsUnroll = 8;
constexpr int64_t kStatsMaxGrid = 256 * 16;

// NT: non-temporal load (a buffer streamed once per step, far larger than L2 + MALL)
template <bool NT, typename V>
__device__ __forceinline__ V ld_vec(const V* a) {
  if constexpr (NT) return __builtin_nontemporal_load(a);
  return *a;
}

template <typename T, bool NT = false>
__device__ __forceinline__ void load4(const T* p, float (&o)[4]) {
  const auto v = ld_vec<NT>(reinterpret_cast<const vec4_t<T>*>(p));
  o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
}

template <typename T>
__global__ __launch_bounds__(kThreads) void grad_stats_partial_kernel(const T* __restrict__ g, int64_t n,
                                                                      float2* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  float ss = 0.f, bad = 0.f;
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  // kStatsUnroll independent non-temporal loads in flight per lane before any of them is consumed
  for (; i + (kStatsUnroll - 1) * stride < nv; i += kStatsUnroll * stride) {
    float v[kStatsUnroll][4];
#pragma unroll
    for (int u = 0; u < kStatsUnroll; ++u) load4<T, true>(g + (i + u * stride) * 4, v[u]);
#pragma unroll
    for (int u = 0; u < kStatsUnroll; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool fin = __builtin_isfinite(v[u][j]);
        bad += fin ? 0.f : 1.f;
        ss += fin ? v[u][j] * v[u][j] : 0.f;
      }
  }
  for (; i < nv; i += stride) {
    float v[4];
    load4<T>(g + i * 4, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool fin = __builtin_isfinite(v[j]);
      bad += fin ? 0.f : 1.f;
      ss += fin ? v[j] * v[j] : 0.f;
    }
  }
  if (blockIdx.x == 0)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += kThreads) {
      const float v = (float)g[i];
      const bool fin = __builtin_isfinite(v);
      bad += fin ? 0.f : 1.f;
      ss += fin ? v * v : 0.f;
    }
  ss = block_sum<kThreads / 64>(ss, red);
  bad = block_sum<kThreads / 64>(bad, red);
  if (threadIdx.x == 0) part[blockIdx.x] = make_float2(ss, bad);
}

__global__ __launch_bounds__(kThreads) void grad_stats_final_kernel(const float2* __restrict__ part, int n,
                                                                    float* __restrict__ out, bool accumulate) {
  __shared__ float red[kThreads / 64];
  float ss = 0.f, bad = 0.f;
  for (int i = threadIdx.x; i < n; i += kThreads) {
    ss += part[i].x;
    bad += part[i].y;
  }
  ss = block_sum<kThreads / 64>(ss, red);
  bad = block_sum<kThreads / 64>(bad, red);
  if (threadIdx.x == 0) {
    if (accumulate) {
      out[0] += ss;
      out[1] += bad;
    } else {
      out[0] = ss;
      out[1] = bad;
    }
  }
}

struct AdamHyper {
  float lr, b1, b2, eps, wd, bc1, bc2, grad_scale, max_norm;
};

// inv_scale: optional device word, 1 / (dynamic loss scale) of the fp16 path
__device__ __forceinline__ float clip_coef(const float* stats, const float* inv_scale, const AdamHyper& h,
                                           bool& skip) {
  const float gsc = h.grad_scale * (inv_scale ? *inv_scale : 1.f);
  if (!stats) {
    skip = false;
    return gsc;
  }
  skip = stats[1] > 0.f;
  float coef = gsc;
  if (h.max_norm > 0.f) {
    const float norm = sqrtf(stats[0]) * gsc;
    coef *= fminf(1.f, h.max_norm / (norm + 1e-6f));
  }
  return coef;
}

template <bool NT, typename V>
__device__ __forceinline__ void st_stream(V* a, V v) {
  if constexpr (NT) __builtin_nontemporal_store(v, a);
  else *a = v;
}

// One float4 of the update (shared by the flat and the tiled-transposing kernels: the same instructions, so the
// same bits).
__device__ __forceinline__ void adam4(f32x4& pp, f32x4& mm, f32x4& vv, const float (&gg)[4], float gc, float decay,
                                      float step_size, float inv_sqrt_bc2, const AdamHyper& h) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gj = gg[j] * gc;
    mm[j] = h.b1 * mm[j] + (1.f - h.b1) * gj;
    vv[j] = h.b2 * vv[j] + (1.f - h.b2) * gj * gj;
    const float denom = sqrtf(vv[j]) * inv_sqrt_bc2 + h.eps;
    pp[j] = pp[j] * decay - step_size * mm[j] / denom;
  }
}

// NT: the optimizer state and the compute copy are streamed once per step -- non-temporal loads / stores keep
// them from displacing anything in L2 / MALL (5.51 TB/s vs ordinary accesses, profiles/adamw_nt_ab_r03.json)
template <typename GT, typename PT, bool NT>
__global__ __launch_bounds__(kThreads) void adamw_kernel(float* __restrict__ p, float* __restrict__ m,
                                                         float* __restrict__ v, const GT* __restrict__ g,
                                                         PT* __restrict__ p16, const float* __restrict__ stats,
                                                         const float* __restrict__ inv_scale, int64_t n,
                                                         AdamHyper h) {
  bool skip;
  const float gc = clip_coef(stats, inv_scale, h, skip);
  if (skip) return;  // overflow / NaN: the whole step is dropped (fp16 loss-scaler semantics)
  const float decay = 1.f - h.lr * h.wd;
  const float step_size = h.lr / h.bc1;
  const float inv_sqrt_bc2 = rsqrtf(h.bc2);
  const int64_t nv = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kThreads) {
    f32x4 pp = ld_vec<NT>(reinterpret_cast<const f32x4*>(p + i * 4));
    f32x4 mm = ld_vec<NT>(reinterpret_cast<const f32x4*>(m + i * 4));
    f32x4 vv = ld_vec<NT>(reinterpret_cast<const f32x4*>(v + i * 4));
    float gg[4];
    load4<GT, NT>(g + i * 4, gg);
    adam4(pp, mm, vv, gg, gc, decay, step_size, inv_sqrt_bc2, h);
    st_stream<NT>(reinterpret_cast<f32x4*>(p + i * 4), pp);
    st_stream<NT>(reinterpret_cast<f32x4*>(m + i * 4), mm);
    st_stream<NT>(reinterpret_cast<f32x4*>(v + i * 4), vv);
    if (p16) st_stream<NT>(reinterpret_cast<vec4_t<PT>*>(p16 + i * 4), __builtin_convertvector(pp, vec4_t<PT>));
  }
  if (blockIdx.x == 0)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += kThreads) {
      const float gj = (float)g[i] * gc;
      m[i] = h.b1 * m[i] + (1.f - h.b1) * gj;
      v[i] = h.b2 * v[i] + (1.f - h.b2) * gj * gj;
      p[i] = p[i] * decay - step_size * m[i] / (sqrtf(v[i]) * inv_sqrt_bc2 + h.eps);
      if (p16) p16[i] = (PT)p[i];
    }
}

template <typename ST>
__global__ __launch_bounds__(kThreads) void accumulate_kernel(float* __restrict__ dst, const ST* __restrict__ src,
                                                              int64_t n, float alpha, float beta) {
  const int64_t nv = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kThreads) {
    float s[4];
    load4<ST>(src + i * 4, s);
    f32x4 d = beta == 0.f ? (f32x4)(0.f) : *reinterpret_cast<f32x4*>(dst + i * 4) * beta;
    d += (f32x4){s[0], s[1], s[2], s[3]} * alpha;
    *reinterpret_cast<f32x4*>(dst + i * 4) = d;
  }
  if (blockIdx.x == 0)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += kThreads)
      dst[i] = (beta == 0.f ? 0.f : dst[i] * beta) + alpha * (float)src[i];
}

template <typename PT>
__global__ __launch_bounds__(kThreads) void cast_kernel(const float* __restrict__ src, PT* __restrict__ dst,
                                                        int64_t n) {
  const int64_t nv = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kThreads)
    *reinterpret_cast<vec4_t<PT>*>(dst + i * 4) =
        __builtin_convertvector(*reinterpret_cast<const f32x4*>(src + i * 4), vec4_t<PT>);
  if (blockIdx.x == 0)
    for (int64_t i = nv * 4 + threadIdx.x; i < n; i += kThreads) dst[i] = (PT)src[i];
}

// DeepSpeed dynamic loss scaler, one thread, on the device: state = [scale, 1/scale, good steps, hysteresis
// left]; stats[1] = non-finite gradient count of the step just taken (reference fp16 block,
// deepspeed_launcher.py:175-183: initial_scale_power, loss_scale_window, hysteresis, min_loss_scale).
__global__ void loss_scale_update_kernel(float* __restrict__ st, const float* __restrict__ stats, float window,
                                         float hysteresis, float min_scale) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float scale = st[0], good = st[2], hyst = st[3];
  if (stats[1] > 0.f) {
    hyst -= 1.f;
    if (hyst <= 0.f) {
      scale = fmaxf(scale * 0.5f, min_scale);
      hyst = hysteresis;
    }
    good = 0.f;
  } else {
    good += 1.f;
    if (fmodf(good, window) == 0.f) scale *= 2.f;
  }
  st[0] = scale;
  st[1] = 1.f / scale;
  st[2] = good;
  st[3] = hyst;
}

void check_flat(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), name, " must be a contiguous GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

}  // namespace

// stats[0] = sum g^2 over all finite elements, stats[1] = count of non-finite elements.
void dlgm_grad_stats(at::TensorList grads, at::Tensor out, bool accumulate) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.numel() >= 2, "grad_stats: bad out");
  auto stream = c10::hip::getCurrentHIPStream();
  std::vector<int64_t> grids;
  int64_t total = 0;
  for (const auto& g : grads) {
    check_flat(g, "grad");
    const int64_t gr = std::max<int64_t>(1, std::min<int64_t>((g.numel() / 4 + kThreads - 1) / kThreads, kStatsMaxGrid));
    grids.push_back(gr);
    total += gr;
  }
  if (total == 0) {
    if (!accumulate) out.zero_();
    return;
  }
  auto part = at::empty({total * 2}, out.options());
  auto pp = reinterpret_cast<float2*>(part.data_ptr<float>());
  int64_t off = 0;
  for (size_t i = 0; i < grads.size(); ++i) {
    const auto& g = grads[i];
    if (g.scalar_type() == at::kFloat)
      grad_stats_partial_kernel<float><<<grids[i], kThreads, 0, stream>>>(g.data_ptr<float>(), g.numel(), pp + off);
    else
      DLGM_DISPATCH_16(g.scalar_type(), E, grad_stats_partial_kernel<E><<<grids[i], kThreads, 0, stream>>>(
                                               reinterpret_cast<const E*>(g.data_ptr()), g.numel(), pp + off));
    off += grids[i];
  }
  grad_stats_final_kernel<<<1, kThreads, 0, stream>>>(pp, (int)total, out.data_ptr<float>(), accumulate);
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_adamw_step_(at::Tensor p, at::Tensor m, at::Tensor v, const at::Tensor& g,
                      const c10::optional<at::Tensor>& p16, const c10::optional<at::Tensor>& stats, double lr,
                      double beta1, double beta2, double eps, double weight_decay, double bc1, double bc2,
                      double grad_scale, double max_norm, const c10::optional<at::Tensor>& scale_state) {
  check_flat(p, "param");
  check_flat(m, "exp_avg");
  check_flat(v, "exp_avg_sq");
  check_flat(g, "grad");
  const int64_t n = p.numel();
  TORCH_CHECK(p.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat,
              "adamw: master/state must be fp32");
  TORCH_CHECK(m.numel() == n && v.numel() == n && g.numel() == n, "adamw: size mismatch");
  const bool has16 = p16.has_value() && p16->defined();
  if (has16) {
    check_flat(*p16, "param_16");
    TORCH_CHECK(DLGM_IS16(*p16) && p16->numel() == n, "adamw: bad bf16/fp16 compute copy");
  }
  const float* sp = nullptr;
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->scalar_type() == at::kFloat && stats->numel() >= 2 && stats->is_cuda(), "adamw: bad stats");
    sp = stats->data_ptr<float>();
  }
  const float* inv = nullptr;
  if (scale_state.has_value() && scale_state->defined()) {
    TORCH_CHECK(scale_state->is_cuda() && scale_state->scalar_type() == at::kFloat && scale_state->numel() >= 2,
                "adamw: bad loss-scale state");
    inv = scale_state->data_ptr<float>() + 1;
  }
  if (n == 0) return;
  AdamHyper h{(float)lr, (float)beta1, (float)beta2, (float)eps, (float)weight_decay, (float)bc1, (float)bc2,
              (float)grad_scale, (float)max_norm};
  auto stream = c10::hip::getCurrentHIPStream();
  const int64_t grid = stream_grid(n / 4);
  // the compute copy's dtype selects the instantiation (bf16 unless the engine runs the fp16 path)
  DLGM_DISPATCH_16(has16 ? p16->scalar_type() : at::kBFloat16, PT, {
    PT* p16p = has16 ? reinterpret_cast<PT*>(p16->data_ptr()) : nullptr;
    if (g.scalar_type() == at::kFloat) {
      adamw_kernel<float, PT, true><<<grid, kThreads, 0, stream>>>(p.data_ptr<float>(), m.data_ptr<float>(),
                                                                   v.data_ptr<float>(), g.data_ptr<float>(), p16p,
                                                                   sp, inv, n, h);
    } else {
      DLGM_DISPATCH_16(g.scalar_type(), GT, adamw_kernel<GT, PT, false><<<grid, kThreads, 0, stream>>>(
                                                p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                                                reinterpret_cast<const GT*>(g.data_ptr()), p16p, sp, inv, n, h));
    }
  });
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_accumulate_(at::Tensor dst, const at::Tensor& src, double alpha, double beta) {
  check_flat(dst, "dst");
  check_flat(src, "src");
  TORCH_CHECK(dst.scalar_type() == at::kFloat, "accumulate: dst must be fp32");
  TORCH_CHECK(dst.numel() == src.numel(), "accumulate: size mismatch");
  const int64_t n = dst.numel();
  if (n == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  const int64_t grid = stream_grid(n / 4);
  if (src.scalar_type() == at::kFloat)
    accumulate_kernel<float><<<grid, kThreads, 0, stream>>>(dst.data_ptr<float>(), src.data_ptr<float>(), n,
                                                            (float)alpha, (float)beta);
  else
    DLGM_DISPATCH_16(src.scalar_type(), E, accumulate_kernel<E><<<grid, kThreads, 0, stream>>>(
                                             dst.data_ptr<float>(), reinterpret_cast<const E*>(src.data_ptr()), n,
                                             (float)alpha, (float)beta));
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_cast_f32_bf16_(at::Tensor dst, const at::Tensor& src) {
  check_flat(dst, "dst");
  check_flat(src, "src");
  TORCH_CHECK(src.scalar_type() == at::kFloat && DLGM_IS16(dst) && src.numel() == dst.numel(),
              "cast: expects fp32 -> bf16/fp16 of equal size");
  const int64_t n = src.numel();
  if (n == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  DLGM_DISPATCH_16(dst.scalar_type(), PT, cast_kernel<PT><<<stream_grid(n / 4), kThreads, 0, stream>>>(
                                             src.data_ptr<float>(), reinterpret_cast<PT*>(dst.data_ptr()), n));
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_loss_scale_update_(at::Tensor state, const at::Tensor& stats, int64_t window, int64_t hysteresis,
                             double min_scale) {
  TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kFloat && state.numel() >= 4 && state.is_contiguous(),
              "loss_scale_update: state must be a contiguous device fp32 [4]");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.numel() >= 2, "loss_scale_update: stats");
  loss_scale_update_kernel<<<1, 64, 0, c10::hip::getCurrentHIPStream()>>>(
      state.data_ptr<float>(), stats.data_ptr<float>(), (float)std::max<int64_t>(1, window), (float)hysteresis,
      (float)min_scale);
  DLGM_CHECK_HIP(hipGetLastError());
}
