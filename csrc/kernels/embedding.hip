// Token embedding forward / backward and the MoE router top-k (gfx950), SURVEY.md §2.6 K9/K10.
//
// Embedding forward is a row gather: one wave per token, 16 B per lane, the table row read
// straight into the output row (Llama-3: 8 KiB rows of a 1 GB table).
//
// Embedding backward adds dY rows into an fp32 gradient table WITHOUT atomics and
// deterministically: the caller hands over the token positions sorted by id (stable), and
// one wave per sorted position checks whether it starts a run of equal ids; the run's
// first wave sums the run's dY rows in sorted order and adds the sum into the table row.
// Every table row therefore has exactly one writer, there is no host sync (runs are found
// on the device) and the result does not depend on scheduling.
//
// Router top-k (Mixtral, E <= 64 experts, K <= 4): one thread per token reads its E fp32
// logits, forms the full softmax (for the load-balancing loss), selects the K largest
// logits (ties -> lower expert id, as torch.topk) and the renormalised gates = softmax over
// the selected logits -- the whole routing decision in one pass over [T, E].
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

__global__ __launch_bounds__(256) void embedding_fwd_kernel(const bf16* __restrict__ table,
                                                            const int64_t* __restrict__ ids, bf16* __restrict__ out,
                                                            int64_t T, int64_t D, int64_t V) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  int64_t id = ids[t];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);  // ids are validated on the host; never read out of bounds
  const bf16* src = table + id * D;
  bf16* dst = out + t * D;
  for (int64_t c = lane * 8; c < D; c += 512)
    *reinterpret_cast<bf16x8*>(dst + c) = *reinterpret_cast<const bf16x8*>(src + c);
}

// sorted_ids / order: ids sorted ascending (stable) and the token index of each sorted slot.
template <typename E, bool F32G>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ order,
                                                            const E* __restrict__ dy, void* __restrict__ grad,
                                                            int64_t T, int64_t D, int64_t V) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= T) return;
  const int64_t id = sorted_ids[i];
  if ((i > 0 && sorted_ids[i - 1] == id) || id < 0 || id >= V) return;  // not the start of a run
  int64_t end = i + 1;
  while (end < T && sorted_ids[end] == id) ++end;
  for (int64_t c = lane * 8; c < D; c += 512) {
    f32x8 s = (f32x8)(0.f);
    for (int64_t j = i; j < end; ++j) s += load8f(dy + order[j] * D + c);
    if constexpr (F32G) {
      float* g = reinterpret_cast<float*>(grad) + id * D + c;
      f32x4 a = *reinterpret_cast<f32x4*>(g), b = *reinterpret_cast<f32x4*>(g + 4);
      *reinterpret_cast<f32x4*>(g) = (f32x4){a[0] + s[0], a[1] + s[1], a[2] + s[2], a[3] + s[3]};
      *reinterpret_cast<f32x4*>(g + 4) = (f32x4){b[0] + s[4], b[1] + s[5], b[2] + s[6], b[3] + s[7]};
    } else {
      E* g = reinterpret_cast<E*>(grad) + id * D + c;
      store8f(g, load8f(g) + s);
    }
  }
}

template <int E, int K>
__global__ __launch_bounds__(256) void router_topk_kernel(const float* __restrict__ logits, float* __restrict__ probs,
                                                          int64_t* __restrict__ topi, float* __restrict__ gates,
                                                          int64_t T) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  float l[E];
#pragma unroll
  for (int e = 0; e < E; ++e) l[e] = logits[t * E + e];
  float mx = l[0];
#pragma unroll
  for (int e = 1; e < E; ++e) mx = fmaxf(mx, l[e]);
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) sum += __expf(l[e] - mx);
  const float inv = 1.f / sum;
#pragma unroll
  for (int e = 0; e < E; ++e) probs[t * E + e] = __expf(l[e] - mx) * inv;
  // top-K by repeated selection (E small): strictly greater wins, so ties keep the lower id
  int sel[K];
  float val[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    int best = -1;
    float bv = -INFINITY;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      bool taken = false;
#pragma unroll
      for (int j = 0; j < k; ++j) taken |= sel[j] == e;
      if (!taken && (best < 0 || l[e] > bv)) {
        best = e;
        bv = l[e];
      }
    }
    sel[k] = best;
    val[k] = bv;
  }
  float gs = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) gs += __expf(val[k] - val[0]);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    topi[t * K + k] = sel[k];
    gates[t * K + k] = __expf(val[k] - val[0]) / gs;
  }
}

}  // namespace

at::Tensor dlgm_embedding_fwd(const at::Tensor& table, const at::Tensor& ids) {
  // a row copy: the 16-bit payload moves bit-exactly whether it is bf16 or fp16
  TORCH_CHECK(table.is_cuda() && DLGM_IS16(table) && table.is_contiguous() && table.dim() == 2,
              "embedding: table must be a contiguous [V, D] bf16/fp16 GPU tensor");
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "embedding: ids must be int64");
  const int64_t V = table.size(0), D = table.size(1), T = ids.numel();
  TORCH_CHECK(D % 8 == 0, "embedding: D must be a multiple of 8");
  auto out = at::empty({T, D}, table.options());
  if (T == 0) return out;
  auto stream = c10::hip::getCurrentHIPStream();
  embedding_fwd_kernel<<<(T + 3) / 4, 256, 0, stream>>>(reinterpret_cast<const bf16*>(table.data_ptr()),
                                                        ids.data_ptr<int64_t>(), reinterpret_cast<bf16*>(out.data_ptr()),
                                                        T, D, V);
  DLGM_CHECK_HIP(hipGetLastError());
  return out;
}

// grad (fp32 or bf16 [V, D], may be a view of the flat gradient partition) += scatter of dy rows.
void dlgm_embedding_bwd_(at::Tensor grad, const at::Tensor& dy, const at::Tensor& sorted_ids, const at::Tensor& order) {
  TORCH_CHECK(grad.is_cuda() && grad.is_contiguous() && grad.dim() == 2, "embedding_bwd: grad must be contiguous [V, D]");
  TORCH_CHECK(DLGM_IS16(dy) && dy.is_contiguous() && dy.numel() == sorted_ids.numel() * grad.size(1),
              "embedding_bwd: dy must be contiguous bf16/fp16 [T, D]");
  TORCH_CHECK(sorted_ids.scalar_type() == at::kLong && order.scalar_type() == at::kLong && sorted_ids.is_contiguous() &&
                  order.is_contiguous() && order.numel() == sorted_ids.numel(),
              "embedding_bwd: sorted ids / order must be int64 [T]");
  const int64_t V = grad.size(0), D = grad.size(1), T = sorted_ids.numel();
  TORCH_CHECK(D % 8 == 0, "embedding_bwd: D must be a multiple of 8");
  if (T == 0) return;
  auto stream = c10::hip::getCurrentHIPStream();
  DLGM_DISPATCH_16(dy.scalar_type(), E, {
    auto dyp = reinterpret_cast<const E*>(dy.data_ptr());
    if (grad.scalar_type() == at::kFloat) {
      embedding_bwd_kernel<E, true><<<(T + 3) / 4, 256, 0, stream>>>(
          sorted_ids.data_ptr<int64_t>(), order.data_ptr<int64_t>(), dyp, grad.data_ptr(), T, D, V);
    } else {
      TORCH_CHECK(grad.scalar_type() == dy.scalar_type(), "embedding_bwd: grad must be fp32 or dy's dtype");
      embedding_bwd_kernel<E, false><<<(T + 3) / 4, 256, 0, stream>>>(
          sorted_ids.data_ptr<int64_t>(), order.data_ptr<int64_t>(), dyp, grad.data_ptr(), T, D, V);
    }
  });
  DLGM_CHECK_HIP(hipGetLastError());
}

// logits fp32 [T, E] -> (probs [T, E], topi int64 [T, K], gates fp32 [T, K])
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_router_topk(const at::Tensor& logits, int64_t k) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kFloat && logits.is_contiguous() && logits.dim() == 2,
              "router_topk: logits must be a contiguous fp32 [T, E] GPU tensor");
  const int64_t T = logits.size(0), E = logits.size(1);
  auto probs = at::empty_like(logits);
  auto topi = at::empty({T, k}, logits.options().dtype(at::kLong));
  auto gates = at::empty({T, k}, logits.options());
  if (T == 0) return {probs, topi, gates};
  auto stream = c10::hip::getCurrentHIPStream();
  const dim3 grid((T + 255) / 256);
  auto lp = logits.data_ptr<float>();
#define ROUTER(EE, KK)                                                                                     \
  if (E == EE && k == KK) {                                                                                \
    router_topk_kernel<EE, KK><<<grid, 256, 0, stream>>>(lp, probs.data_ptr<float>(), topi.data_ptr<int64_t>(), \
                                                         gates.data_ptr<float>(), T);                      \
    DLGM_CHECK_HIP(hipGetLastError());                                                                     \
    return {probs, topi, gates};                                                                           \
  }
  ROUTER(4, 1) ROUTER(4, 2) ROUTER(8, 1) ROUTER(8, 2) ROUTER(8, 4) ROUTER(16, 2) ROUTER(16, 4) ROUTER(32, 2)
  ROUTER(64, 2)
#undef ROUTER
  TORCH_CHECK(false, "router_topk: unsupported (experts, top-k) = (", E, ", ", k, ")");
}
