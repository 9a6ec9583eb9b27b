// Rotary position embedding (rotate-half / Llama convention), in place, gfx950.
//
// Applied directly on the fused QKV projection output [T, (Hq + 2*Hkv) * hd]
// (SURVEY.md §2.6 K4): the first `n_rope_heads` (= Hq + Hkv) heads of each row are
// rotated, V is left alone, so no split / transpose copy is ever made -- the
// attention kernel consumes the strided q/k/v views of the same buffer.
//
// Each lane rotates 8 (x_i, x_{i+hd/2}) pairs: two 16-byte bf16/fp16 loads of the
// row, two float4-pair loads of the cos/sin table (fp32, [max_pos, hd/2],
// precomputed on the host -- no on-device trig, Appendix B "Element-wise").
// Backward is the same kernel with the rotation inverted.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

template <typename E, bool INVERSE>
__global__ __launch_bounds__(256) void rope_kernel(E* __restrict__ qkv, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t,
                                                   const int64_t* __restrict__ pos_ids, int64_t T,
                                                   int64_t row_stride, int n_heads, int hd, int seq_len) {
  const int lanes_per_head = hd >> 4;  // 8 pairs per lane
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t head_row = g / lanes_per_head;
  const int sub = (int)(g - head_row * lanes_per_head);
  if (head_row >= T * n_heads) return;
  const int64_t t = head_row / n_heads;
  const int head = (int)(head_row - t * n_heads);
  const int64_t pos = pos_ids ? pos_ids[t] : (t % seq_len);
  const int half = hd >> 1;
  const int i0 = sub * 8;
  E* p = qkv + t * row_stride + (int64_t)head * hd;
  const float* cp = cos_t + pos * half + i0;
  const float* sp = sin_t + pos * half + i0;
  f32x8 a = load8f(p + i0);
  f32x8 b = load8f(p + i0 + half);
  f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
  f32x4 s0 = *reinterpret_cast<const f32x4*>(sp), s1 = *reinterpret_cast<const f32x4*>(sp + 4);
  f32x8 c = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
  f32x8 s = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
  if constexpr (INVERSE) s = -s;
  store8f(p + i0, a * c - b * s);
  store8f(p + i0 + half, b * c + a * s);
}

}  // namespace

void dlgm_rope_(at::Tensor qkv, const at::Tensor& cos_t, const at::Tensor& sin_t,
                const c10::optional<at::Tensor>& pos_ids, int64_t n_rope_heads, int64_t head_dim,
                int64_t seq_len, bool inverse) {
  TORCH_CHECK(qkv.is_cuda() && DLGM_IS16(qkv), "rope: qkv must be a bf16/fp16 GPU tensor");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "rope: qkv must be [T, C] with unit inner stride");
  TORCH_CHECK(head_dim % 16 == 0, "rope: head_dim must be a multiple of 16");
  TORCH_CHECK(n_rope_heads * head_dim <= qkv.size(1), "rope: heads exceed row width");
  TORCH_CHECK(qkv.stride(0) % 8 == 0, "rope: row stride must keep 16-byte alignment");
  TORCH_CHECK(cos_t.scalar_type() == at::kFloat && sin_t.scalar_type() == at::kFloat &&
                  cos_t.is_contiguous() && sin_t.is_contiguous(),
              "rope: tables must be contiguous fp32");
  TORCH_CHECK(cos_t.size(-1) == head_dim / 2, "rope: table width must be head_dim/2");
  const int64_t T = qkv.size(0);
  const bool has_pos = pos_ids.has_value() && pos_ids->defined();
  if (has_pos) {
    TORCH_CHECK(pos_ids->scalar_type() == at::kLong && pos_ids->numel() == T, "rope: bad pos_ids");
  } else {
    TORCH_CHECK(seq_len > 0 && seq_len <= cos_t.size(0), "rope: seq_len exceeds table");
  }
  if (T == 0) return;
  const int64_t threads = T * n_rope_heads * (head_dim / 16);
  const int64_t blocks = (threads + 255) / 256;
  auto stream = c10::hip::getCurrentHIPStream();
  const int64_t* pp = has_pos ? pos_ids->data_ptr<int64_t>() : nullptr;
  DLGM_DISPATCH_16(qkv.scalar_type(), E, {
    auto p = reinterpret_cast<E*>(qkv.data_ptr());
    if (inverse)
      rope_kernel<E, true><<<blocks, 256, 0, stream>>>(p, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), pp, T,
                                                       qkv.stride(0), n_rope_heads, head_dim, seq_len);
    else
      rope_kernel<E, false><<<blocks, 256, 0, stream>>>(p, cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), pp, T,
                                                        qkv.stride(0), n_rope_heads, head_dim, seq_len);
  });
  DLGM_CHECK_HIP(hipGetLastError());
}
