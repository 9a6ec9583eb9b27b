// SwiGLU activation  y = silu(gate) * up  (SURVEY.md §2.6 K5), gfx950.
//
// The gate and up projections are ONE GEMM producing gu = [T, 2F]
// (gate = gu[:, :F], up = gu[:, F:]), so the activation reads one buffer.
// Forward writes y [T, F]; backward reads dy and gu and writes dgu [T, 2F]
// -- the gradient of the fused GEMM output -- in a single pass.
// Pure HBM streaming: one 16-B vector per lane and operand, fp32 math; bf16 or fp16 storage.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

// One 8-element vector per lane, no grid-stride loop: block b covers row b / bpr, vectors (b % bpr) * 256 + lane
// (bpr = blocks per row; the row split is wave-uniform scalar math, no per-lane 64-bit division). Rows at or past
// nrows exit at once.
template <typename T>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const T* __restrict__ gu, T* __restrict__ y, int F,
                                                         int64_t gu_stride, uint32_t bpr,
                                                         const int* __restrict__ nrows) {
  const uint32_t t = blockIdx.x / bpr;
  if (nrows != nullptr && (int64_t)t >= (int64_t)nrows[0]) return;
  const int c = ((blockIdx.x - t * bpr) * 256 + threadIdx.x) * 8;
  if (c >= F) return;
  const T* row = gu + (int64_t)t * gu_stride;
  f32x8 g = load8f(row + c), u = load8f(row + F + c);
  f32x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = silu(g[j]) * u[j];
  store8f(y + (int64_t)t * F + c, o);
}

template <typename T>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ gu,
                                                         T* __restrict__ dgu, int F, int64_t gu_stride, uint32_t bpr,
                                                         const int* __restrict__ nrows) {
  const uint32_t t = blockIdx.x / bpr;
  if (nrows != nullptr && (int64_t)t >= (int64_t)nrows[0]) return;
  const int c = ((blockIdx.x - t * bpr) * 256 + threadIdx.x) * 8;
  if (c >= F) return;
  const T* row = gu + (int64_t)t * gu_stride;
  f32x8 g = load8f(row + c), u = load8f(row + F + c), d = load8f(dy + (int64_t)t * F + c);
  f32x8 dg, du;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float s = 1.f / (1.f + __expf(-g[j]));
    const float sg = g[j] * s;
    du[j] = d[j] * sg;
    dg[j] = d[j] * u[j] * (s + sg * (1.f - s));
  }
  T* out = dgu + (int64_t)t * 2 * F;
  store8f(out + c, dg);
  store8f(out + F + c, du);
}

// blocks per row and the grid for T rows (host-checked to stay within a 32-bit block index)
uint32_t blocks_per_row(int64_t F) { return (uint32_t)((F / 8 + 255) / 256); }

int64_t grid_for(int64_t T, int64_t F) {
  const int64_t g = T * blocks_per_row(F);
  TORCH_CHECK(g < (int64_t(1) << 31) && F < (int64_t(1) << 30), "swiglu: too many rows for one launch");
  return g;
}

}  // namespace

static const int* rows_ptr(const c10::optional<at::Tensor>& nrows) {
  if (!nrows.has_value() || !nrows->defined()) return nullptr;
  TORCH_CHECK(nrows->is_cuda() && nrows->scalar_type() == at::kInt && nrows->numel() == 1, "swiglu: nrows int32 [1]");
  return nrows->data_ptr<int>();
}

// nrows (optional, int32 [1] on the device): only rows [0, nrows) are computed; the rest of the output is left
// uninitialised (the MoE capacity layout's unused overflow rows, whose count is known only on the device)
at::Tensor dlgm_swiglu_fwd(const at::Tensor& gu, const c10::optional<at::Tensor>& nrows) {
  TORCH_CHECK(gu.is_cuda() && DLGM_IS16(gu) && gu.dim() == 2 && gu.stride(1) == 1,
              "swiglu: gu must be a [T, 2F] bf16/fp16 GPU tensor");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.size(1) % 2 == 0 && F % 8 == 0 && gu.stride(0) % 8 == 0, "swiglu: F must be a multiple of 8");
  auto y = at::empty({T, F}, gu.options());
  if (T == 0) return y;
  auto stream = c10::hip::getCurrentHIPStream();
  DLGM_DISPATCH_16(gu.scalar_type(), E, swiglu_fwd_kernel<E><<<grid_for(T, F), 256, 0, stream>>>(
      reinterpret_cast<const E*>(gu.data_ptr()), reinterpret_cast<E*>(y.data_ptr()), (int)F, gu.stride(0),
      blocks_per_row(F), rows_ptr(nrows)));
  DLGM_CHECK_HIP(hipGetLastError());
  return y;
}

at::Tensor dlgm_swiglu_bwd(const at::Tensor& dy, const at::Tensor& gu, const c10::optional<at::Tensor>& nrows) {
  TORCH_CHECK(gu.is_cuda() && DLGM_IS16(gu) && gu.dim() == 2 && gu.stride(1) == 1,
              "swiglu_bwd: gu must be a [T, 2F] bf16/fp16 GPU tensor");
  const int64_t T = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(dy.is_contiguous() && dy.scalar_type() == gu.scalar_type() && dy.numel() == T * F,
              "swiglu_bwd: dy must be a contiguous [T, F] tensor of gu's dtype");
  auto dgu = at::empty({T, 2 * F}, gu.options());
  if (T == 0) return dgu;
  auto stream = c10::hip::getCurrentHIPStream();
  DLGM_DISPATCH_16(gu.scalar_type(), E, swiglu_bwd_kernel<E><<<grid_for(T, F), 256, 0, stream>>>(
      reinterpret_cast<const E*>(dy.data_ptr()), reinterpret_cast<const E*>(gu.data_ptr()),
      reinterpret_cast<E*>(dgu.data_ptr()), (int)F, gu.stride(0), blocks_per_row(F), rows_ptr(nrows)));
  DLGM_CHECK_HIP(hipGetLastError());
  return dgu;
}
