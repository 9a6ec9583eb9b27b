// Fused softmax-cross-entropy forward + backward over a large vocabulary (gfx950).
//
// the LM-head output for Llama-3 (V = 128256) at T = 8192 is a
// 2.1 GB bf16 tensor. Materialising fp32 logits / probabilities would triple that,
// so one kernel does everything in place:
//   pass 1: per-row online (max, sum-exp) in fp32, 16 B bf16 loads per lane;
//   pass 2: d logits = (softmax - onehot(label)) * grad_scale, written back over
//           the logits (bf16) -- the row is 256 KB, so the re-read is an L2/MALL hit.
// The per-row loss (lse - logit[label]) is returned in fp32. Because the engine
// knows the loss gradient up front (1 / tokens, times the loss scale) the backward
// needs no second sweep over the logits.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;

template <typename E>
__global__ __launch_bounds__(kThreads) void ce_kernel(E* __restrict__ logits, const int64_t* __restrict__ labels,
                                                      float* __restrict__ loss, float* __restrict__ lse_out,
                                                      int64_t V, int64_t row_stride, int64_t ignore_index,
                                                      float grad_scale, const float* __restrict__ scale,
                                                      bool compute_grad) {
  __shared__ float red[kWaves];
  const int64_t row = blockIdx.x;
  E* x = logits + row * row_stride;
  const int64_t label = labels[row];
  const int64_t nvec = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (int64_t c = threadIdx.x; c < nvec; c += kThreads) {
    f32x8 v = load8f(x + c * 8);
    float cm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) cm = fmaxf(cm, v[j]);
    if (cm > m) {
      s *= __expf(m - cm);
      m = cm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
  }
  for (int64_t j = nvec * 8 + threadIdx.x; j < V; j += kThreads) {
    const float v = (float)x[j];
    if (v > m) {
      s *= __expf(m - v);
      m = v;
    }
    s += __expf(v - m);
  }
  const float M = block_max<kWaves>(m, red);
  const float S = block_sum<kWaves>(m == -INFINITY ? 0.f : s * __expf(m - M), red);
  const float lse = M + __logf(S);
  const bool valid = label != ignore_index && label >= 0 && label < V;
  if (threadIdx.x == 0) {
    loss[row] = valid ? lse - (float)x[label] : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!compute_grad) return;
  __syncthreads();  // the label logit is read above before being overwritten below
  // fp16 path: the dynamic loss scale lives on the device (no host read per step)
  const float gs = valid ? grad_scale * (scale ? scale[0] : 1.f) : 0.f;
  for (int64_t c = threadIdx.x; c < nvec; c += kThreads) {
    f32x8 v = load8f(x + c * 8);
    f32x8 g;
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = __expf(v[j] - lse) * gs;
    if (label >= c * 8 && label < c * 8 + 8) g[label - c * 8] -= gs;
    store8f(x + c * 8, g);
  }
  for (int64_t j = nvec * 8 + threadIdx.x; j < V; j += kThreads) {
    float g = __expf((float)x[j] - lse) * gs;
    if (j == label) g -= gs;
    x[j] = (E)g;
  }
}

}  // namespace

// Returns (loss_per_row fp32 [T], lse fp32 [T]). When compute_grad, logits is overwritten
// with d(loss_sum * grad_scale * scale[0])/d logits (scale: optional device fp32, the loss scale).
std::tuple<at::Tensor, at::Tensor> dlgm_cross_entropy_(at::Tensor logits, const at::Tensor& labels,
                                                       int64_t ignore_index, double grad_scale,
                                                       bool compute_grad, const c10::optional<at::Tensor>& scale) {
  TORCH_CHECK(logits.is_cuda() && DLGM_IS16(logits) && logits.dim() == 2 && logits.stride(1) == 1,
              "cross_entropy: logits must be a [T, V] bf16/fp16 GPU tensor with unit inner stride");
  TORCH_CHECK(logits.stride(0) % 8 == 0, "cross_entropy: row stride must be a multiple of 8");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0) && labels.is_contiguous(),
              "cross_entropy: labels must be contiguous int64 [T]");
  const float* sp = nullptr;
  if (scale.has_value() && scale->defined()) {
    TORCH_CHECK(scale->is_cuda() && scale->scalar_type() == at::kFloat && scale->numel() >= 1,
                "cross_entropy: scale must be a device fp32 tensor");
    sp = scale->data_ptr<float>();
  }
  const int64_t T = logits.size(0), V = logits.size(1);
  auto loss = at::empty({T}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({T}, logits.options().dtype(at::kFloat));
  if (T == 0) return {loss, lse};
  auto stream = c10::hip::getCurrentHIPStream();
  DLGM_DISPATCH_16(logits.scalar_type(), E,
                   ce_kernel<E><<<T, kThreads, 0, stream>>>(reinterpret_cast<E*>(logits.data_ptr()),
                                                            labels.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                                            lse.data_ptr<float>(), V, logits.stride(0), ignore_index,
                                                            (float)grad_scale, sp, compute_grad));
  DLGM_CHECK_HIP(hipGetLastError());
  return {loss, lse};
}
