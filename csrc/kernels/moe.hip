// Mixture-of-experts token combine (gfx950), SURVEY.md §2.6 K9.
//
// After the router picks top-K experts per token, tokens are permuted into expert
// order (one gather), run through the experts as dense GEMMs, and must then be
// combined back:  out[t] = sum_k gate[t,k] * y[pos[t,k]].
// Written as a GATHER (each output row reads its K expert rows) so it needs no
// atomics and is deterministic. The backward is its exact adjoint:
//   dy[pos[t,k]] = gate[t,k] * dout[t]     (pos is a permutation: each slot written once)
//   dgate[t,k]   = <dout[t], y[pos[t,k]]>   (wave64 reduction)
// The same forward kernel with gate = 1 sums the K per-slot input gradients back
// onto the token (the adjoint of the dispatch gather) -- again without atomics.
// One wave per token row, 16 B per lane per access.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

template <int K>
__global__ __launch_bounds__(256) void moe_combine_fwd_kernel(const bf16* __restrict__ y, const int64_t* __restrict__ pos,
                                                              const float* __restrict__ gates, bf16* __restrict__ out,
                                                              int64_t T, int64_t D) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  int64_t rows[K];
  float g[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    rows[k] = pos[t * K + k];
    g[k] = gates ? gates[t * K + k] : 1.f;
  }
  for (int64_t c = lane * 8; c < D; c += 512) {
    f32x8 acc = (f32x8)(0.f);
#pragma unroll
    for (int k = 0; k < K; ++k) acc += load8f(y + rows[k] * D + c) * g[k];
    store8f(out + t * D + c, acc);
  }
}

template <int K>
__global__ __launch_bounds__(256) void moe_combine_bwd_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ y,
                                                              const int64_t* __restrict__ pos,
                                                              const float* __restrict__ gates, bf16* __restrict__ dy,
                                                              float* __restrict__ dgates, int64_t T, int64_t D) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  int64_t rows[K];
  float g[K], dot[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    rows[k] = pos[t * K + k];
    g[k] = gates[t * K + k];
    dot[k] = 0.f;
  }
  for (int64_t c = lane * 8; c < D; c += 512) {
    f32x8 d = load8f(dout + t * D + c);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      f32x8 yy = load8f(y + rows[k] * D + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) dot[k] += d[j] * yy[j];
      store8f(dy + rows[k] * D + c, d * g[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const float s = wave_sum(dot[k]);
    if (lane == 0) dgates[t * K + k] = s;
  }
}

void check(const at::Tensor& y, const at::Tensor& pos, int64_t D) {
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.dim() == 2,
              "moe: rows must be a contiguous [N, D] bf16 GPU tensor");
  TORCH_CHECK(D % 8 == 0, "moe: D must be a multiple of 8");
  TORCH_CHECK(pos.scalar_type() == at::kLong && pos.is_contiguous() && pos.dim() == 2, "moe: pos must be int64 [T, K]");
}

}  // namespace

at::Tensor dlgm_moe_combine_fwd(const at::Tensor& y, const at::Tensor& pos, const c10::optional<at::Tensor>& gates) {
  const int64_t D = y.size(1);
  check(y, pos, D);
  const int64_t T = pos.size(0), K = pos.size(1);
  const bool has_g = gates.has_value() && gates->defined();
  if (has_g)
    TORCH_CHECK(gates->scalar_type() == at::kFloat && gates->is_contiguous() && gates->numel() == T * K,
                "moe: gates must be fp32 [T, K]");
  auto out = at::empty({T, D}, y.options());
  if (T == 0) return out;
  auto stream = c10::hip::getCurrentHIPStream();
  const dim3 grid((T + 3) / 4);
  auto yp = reinterpret_cast<const bf16*>(y.data_ptr());
  auto gp = has_g ? gates->data_ptr<float>() : nullptr;
  auto op = reinterpret_cast<bf16*>(out.data_ptr());
  switch (K) {
    case 1: moe_combine_fwd_kernel<1><<<grid, 256, 0, stream>>>(yp, pos.data_ptr<int64_t>(), gp, op, T, D); break;
    case 2: moe_combine_fwd_kernel<2><<<grid, 256, 0, stream>>>(yp, pos.data_ptr<int64_t>(), gp, op, T, D); break;
    case 4: moe_combine_fwd_kernel<4><<<grid, 256, 0, stream>>>(yp, pos.data_ptr<int64_t>(), gp, op, T, D); break;
    default: TORCH_CHECK(false, "moe: top-k must be 1, 2 or 4");
  }
  DLGM_CHECK_HIP(hipGetLastError());
  return out;
}

std::tuple<at::Tensor, at::Tensor> dlgm_moe_combine_bwd(const at::Tensor& dout, const at::Tensor& y,
                                                        const at::Tensor& pos, const at::Tensor& gates) {
  const int64_t D = y.size(1);
  check(y, pos, D);
  const int64_t T = pos.size(0), K = pos.size(1);
  TORCH_CHECK(dout.is_contiguous() && dout.scalar_type() == at::kBFloat16 && dout.numel() == T * D, "moe: bad dout");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.is_contiguous() && gates.numel() == T * K, "moe: bad gates");
  auto dy = at::zeros_like(y);  // slots not referenced by any token (none in practice) stay zero
  auto dg = at::empty({T, K}, gates.options());
  if (T == 0) return {dy, dg};
  auto stream = c10::hip::getCurrentHIPStream();
  const dim3 grid((T + 3) / 4);
  auto dp = reinterpret_cast<const bf16*>(dout.data_ptr());
  auto yp = reinterpret_cast<const bf16*>(y.data_ptr());
  auto dyp = reinterpret_cast<bf16*>(dy.data_ptr());
  switch (K) {
    case 1: moe_combine_bwd_kernel<1><<<grid, 256, 0, stream>>>(dp, yp, pos.data_ptr<int64_t>(), gates.data_ptr<float>(), dyp, dg.data_ptr<float>(), T, D); break;
    case 2: moe_combine_bwd_kernel<2><<<grid, 256, 0, stream>>>(dp, yp, pos.data_ptr<int64_t>(), gates.data_ptr<float>(), dyp, dg.data_ptr<float>(), T, D); break;
    case 4: moe_combine_bwd_kernel<4><<<grid, 256, 0, stream>>>(dp, yp, pos.data_ptr<int64_t>(), gates.data_ptr<float>(), dyp, dg.data_ptr<float>(), T, D); break;
    default: TORCH_CHECK(false, "moe: top-k must be 1, 2 or 4");
  }
  DLGM_CHECK_HIP(hipGetLastError());
  return {dy, dg};
}
