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
//
// moe_permute: the expert-sort of the (token, k) slots ON THE DEVICE, in one single-workgroup launch
// (E <= 32): per-thread expert histograms of a contiguous slot range -> one block-wide exclusive scan
// over the [expert][thread] counts (which is exactly each thread's first position per expert, since
// the sorted order is expert-major and slot-ordered within an expert, i.e. a stable argsort) ->
// positions. Outputs: offsets [E + 1] (int32: the grouped-GEMM segment bounds), pos [T, K] (slot ->
// sorted row), src [T*K] (sorted row -> token). Nothing is read back to the host.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

template <typename E, int K>
__global__ __launch_bounds__(256) void moe_combine_fwd_kernel(const E* __restrict__ y, const int64_t* __restrict__ pos,
                                                              const float* __restrict__ gates, E* __restrict__ out,
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

template <typename E, int K>
__global__ __launch_bounds__(256) void moe_combine_bwd_kernel(const E* __restrict__ dout, const E* __restrict__ y,
                                                              const int64_t* __restrict__ pos,
                                                              const float* __restrict__ gates, E* __restrict__ dy,
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

constexpr int kPermThreads = 1024;
constexpr int kPermRegs = 16;

__global__ __launch_bounds__(kPermThreads) void moe_permute_kernel(const int64_t* __restrict__ topi, int64_t n, int K,
                                                                   int E, int* __restrict__ offsets,
                                                                   int64_t* __restrict__ pos,
                                                                   int64_t* __restrict__ src) {
  extern __shared__ int cnt[];  // [E][kPermThreads], then the per-wave scan totals
  int* wsum = cnt + E * kPermThreads;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t per = (n + kPermThreads - 1) / kPermThreads;
  const int64_t lo = min<int64_t>(n, t * per), hi = min<int64_t>(n, lo + per);
  for (int e = 0; e < E; ++e) cnt[e * kPermThreads + t] = 0;
  // one workgroup walks the whole routing: its latency is the kernel's time, so a thread's expert ids (up to
  // kPermRegs of them, n <= 16k slots) are loaded at once into registers and reused by the placement pass
  // (a load-then-count loop per slot measured ~105 us for Mixtral's 8192 slots)
  const bool in_regs = per <= kPermRegs;
  int ev[kPermRegs];
  if (in_regs) {
#pragma unroll
    for (int i = 0; i < kPermRegs; ++i) ev[i] = lo + i < hi ? (int)topi[lo + i] : -1;
#pragma unroll
    for (int i = 0; i < kPermRegs; ++i)
      if (ev[i] >= 0) cnt[ev[i] * kPermThreads + t] += 1;
  } else {
    for (int64_t s = lo; s < hi; ++s) cnt[(int)topi[s] * kPermThreads + t] += 1;
  }
  __syncthreads();
  // exclusive scan of the E*1024 counts in [expert][thread] order: thread t owns entries E*t .. E*t+E-1
  int local[32];
  int run = 0;
  for (int j = 0; j < E; ++j) {
    local[j] = run;
    run += cnt[t * E + j];  // flat index f = t*E + j over the [E][1024] array
  }
  int incl = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int wbase = 0;
  for (int i = 0; i < wv; ++i) wbase += wsum[i];
  const int excl = wbase + incl - run;
  __syncthreads();
  for (int j = 0; j < E; ++j) cnt[t * E + j] = excl + local[j];  // now the first position of (e, thread)
  __syncthreads();
  if (t < E) offsets[t] = cnt[t * kPermThreads];  // expert t's first row = position of (t, thread 0)
  if (t == 0) offsets[E] = (int)n;
  if (in_regs) {
#pragma unroll
    for (int i = 0; i < kPermRegs; ++i) {
      if (ev[i] < 0) continue;
      const int s = (int)lo + i;  // (n < 2^31: checked on the host)
      const int p = cnt[ev[i] * kPermThreads + t]++;
      pos[s] = p;
      src[p] = s / K;
    }
    return;
  }
  for (int64_t s = lo; s < hi; ++s) {
    const int e = (int)topi[s];
    const int p = cnt[e * kPermThreads + t]++;
    pos[s] = p;
    src[p] = s / K;
  }
}

constexpr int kMaxGroups = 64;

// Aligned re-layout of expert-sorted rows: expert e's rows start at padded row poff[e] (a multiple of `align`,
// poff[e+1] - poff[e] = count rounded up to align). rows[p] = the sorted row at padded row p, or -1 (padding; also
// every p past poff[G]). With it a transposed [D, P] image has every expert's reduction range on whole K tiles.
__global__ __launch_bounds__(256) void moe_pad_plan_kernel(const int* __restrict__ offsets, int G, int64_t P,
                                                           int align, int* __restrict__ rows, int* __restrict__ poff) {
  __shared__ int s_off[kMaxGroups + 1], s_pad[kMaxGroups + 1];
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < G; ++e) {
      s_off[e] = offsets[e];
      s_pad[e] = acc;
      acc += (offsets[e + 1] - offsets[e] + align - 1) / align * align;
    }
    s_off[G] = offsets[G];
    s_pad[G] = acc;
  }
  __syncthreads();
  if (blockIdx.x == 0 && (int)threadIdx.x <= G) poff[threadIdx.x] = s_pad[threadIdx.x];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (int64_t)gridDim.x * blockDim.x) {
    int src = -1;
    if (p < s_pad[G]) {
      int e = 0;
      while (s_pad[e + 1] <= p) ++e;
      const int r = (int)p - s_pad[e];
      if (r < s_off[e + 1] - s_off[e]) src = s_off[e] + r;
    }
    rows[p] = src;
  }
}

// The same re-layout over S row sets (micro-batches) at once: expert e's rows of set 0, then of set 1, ... are
// contiguous from padded row poff[e] (a multiple of align). rows[p] = (set << 24) | row within the set, or -1.
// offsets [S, G + 1]: set s's expert split. One grouped-K launch then reduces each expert over all its rows with
// contiguous, tile-aligned K ranges (no per-segment selection inside the GEMM's pipelined loop).
constexpr int kMaxSets = 8;

__global__ __launch_bounds__(256) void moe_pad_plan_multi_kernel(const int* __restrict__ offsets, int S, int G,
                                                                 int64_t P, int align, int* __restrict__ rows,
                                                                 int* __restrict__ poff) {
  __shared__ int s_off[kMaxSets][kMaxGroups + 1], s_cum[kMaxSets + 1][kMaxGroups], s_pad[kMaxGroups + 1];
  for (int i = threadIdx.x; i < S * (G + 1); i += blockDim.x) s_off[i / (G + 1)][i % (G + 1)] = offsets[i];
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < G; ++e) {
      int c = 0;
      for (int t = 0; t < S; ++t) {
        s_cum[t][e] = c;
        c += s_off[t][e + 1] - s_off[t][e];
      }
      s_cum[S][e] = c;
      s_pad[e] = acc;
      acc += (c + align - 1) / align * align;
    }
    s_pad[G] = acc;
  }
  __syncthreads();
  if (blockIdx.x == 0 && (int)threadIdx.x <= G) poff[threadIdx.x] = s_pad[threadIdx.x];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (int64_t)gridDim.x * blockDim.x) {
    int src = -1;
    if (p < s_pad[G]) {
      int e = 0;
      while (s_pad[e + 1] <= p) ++e;
      const int r = (int)p - s_pad[e];
      if (r < s_cum[S][e]) {
        int t = 0;
        while (s_cum[t + 1][e] <= r) ++t;
        src = (t << 24) | (s_off[t][e] + r - s_cum[t][e]);
      }
    }
    rows[p] = src;
  }
}

void check(const at::Tensor& y, const at::Tensor& pos, int64_t D) {
  TORCH_CHECK(y.is_cuda() && DLGM_IS16(y) && y.is_contiguous() && y.dim() == 2,
              "moe: rows must be a contiguous [N, D] bf16/fp16 GPU tensor");
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
  auto gp = has_g ? gates->data_ptr<float>() : nullptr;
  DLGM_DISPATCH_16(y.scalar_type(), E, {
    auto yp = reinterpret_cast<const E*>(y.data_ptr());
    auto op = reinterpret_cast<E*>(out.data_ptr());
    switch (K) {
      case 1: moe_combine_fwd_kernel<E, 1><<<grid, 256, 0, stream>>>(yp, pos.data_ptr<int64_t>(), gp, op, T, D); break;
      case 2: moe_combine_fwd_kernel<E, 2><<<grid, 256, 0, stream>>>(yp, pos.data_ptr<int64_t>(), gp, op, T, D); break;
      case 4: moe_combine_fwd_kernel<E, 4><<<grid, 256, 0, stream>>>(yp, pos.data_ptr<int64_t>(), gp, op, T, D); break;
      default: TORCH_CHECK(false, "moe: top-k must be 1, 2 or 4");
    }
  });
  DLGM_CHECK_HIP(hipGetLastError());
  return out;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_moe_permute(const at::Tensor& topi, int64_t n_experts) {
  TORCH_CHECK(topi.is_cuda() && topi.scalar_type() == at::kLong && topi.is_contiguous() && topi.dim() == 2,
              "moe_permute: topi must be a contiguous int64 [T, K] GPU tensor");
  TORCH_CHECK(n_experts >= 1 && n_experts <= 32, "moe_permute: 1..32 experts");
  const int64_t T = topi.size(0), K = topi.size(1), n = T * K;
  TORCH_CHECK(n < (1ll << 31), "moe_permute: too many slots");
  auto offsets = at::empty({n_experts + 1}, topi.options().dtype(at::kInt));
  auto pos = at::empty({T, K}, topi.options());
  auto src = at::empty({n}, topi.options());
  const size_t lds = (size_t)(n_experts * kPermThreads + kPermThreads / 64) * sizeof(int);
  auto stream = c10::hip::getCurrentHIPStream();
  if (lds > 64 * 1024)  // > 64 KiB of dynamic LDS (up to 160 KiB on gfx950) has to be opted into
    DLGM_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(moe_permute_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  moe_permute_kernel<<<1, kPermThreads, lds, stream>>>(topi.data_ptr<int64_t>(), n, (int)K, (int)n_experts,
                                                      offsets.data_ptr<int>(), pos.data_ptr<int64_t>(),
                                                      src.data_ptr<int64_t>());
  DLGM_CHECK_HIP(hipGetLastError());
  return {offsets, pos, src};
}

std::tuple<at::Tensor, at::Tensor> dlgm_moe_pad_plan(const at::Tensor& offsets, int64_t padded_rows, int64_t align) {
  TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.is_contiguous() && offsets.dim() == 1,
              "moe_pad_plan: offsets must be a contiguous int32 [G + 1] GPU tensor");
  const int64_t G = offsets.numel() - 1;
  TORCH_CHECK(G >= 1 && G <= kMaxGroups && align >= 1 && padded_rows >= 0 && padded_rows < (1ll << 31),
              "moe_pad_plan: 1..64 groups, align >= 1");
  auto rows = at::empty({padded_rows}, offsets.options());
  auto poff = at::empty({G + 1}, offsets.options());
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((padded_rows + 255) / 256, 2048));
  moe_pad_plan_kernel<<<(unsigned)blocks, 256, 0, c10::hip::getCurrentHIPStream()>>>(
      offsets.data_ptr<int>(), (int)G, padded_rows, (int)align, rows.data_ptr<int>(), poff.data_ptr<int>());
  DLGM_CHECK_HIP(hipGetLastError());
  return {rows, poff};
}

std::tuple<at::Tensor, at::Tensor> dlgm_moe_pad_plan_multi(const at::Tensor& offsets, int64_t padded_rows,
                                                            int64_t align) {
  TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.is_contiguous() && offsets.dim() == 2,
              "moe_pad_plan_multi: offsets must be a contiguous int32 [S, G + 1] GPU tensor");
  const int64_t S = offsets.size(0), G = offsets.size(1) - 1;
  TORCH_CHECK(S >= 1 && S <= kMaxSets && G >= 1 && G <= kMaxGroups && align >= 1 && padded_rows >= 0 &&
                  padded_rows < (1ll << 31), "moe_pad_plan_multi: 1..8 sets, 1..64 groups, align >= 1");
  auto rows = at::empty({padded_rows}, offsets.options());
  auto poff = at::empty({G + 1}, offsets.options());
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((padded_rows + 255) / 256, 2048));
  moe_pad_plan_multi_kernel<<<(unsigned)blocks, 256, 0, c10::hip::getCurrentHIPStream()>>>(
      offsets.data_ptr<int>(), (int)S, (int)G, padded_rows, (int)align, rows.data_ptr<int>(), poff.data_ptr<int>());
  DLGM_CHECK_HIP(hipGetLastError());
  return {rows, poff};
}

std::tuple<at::Tensor, at::Tensor> dlgm_moe_combine_bwd(const at::Tensor& dout, const at::Tensor& y,
                                                        const at::Tensor& pos, const at::Tensor& gates) {
  const int64_t D = y.size(1);
  check(y, pos, D);
  const int64_t T = pos.size(0), K = pos.size(1);
  TORCH_CHECK(dout.is_contiguous() && dout.scalar_type() == y.scalar_type() && dout.numel() == T * D, "moe: bad dout");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.is_contiguous() && gates.numel() == T * K, "moe: bad gates");
  auto dy = at::zeros_like(y);  // slots not referenced by any token (none in practice) stay zero
  auto dg = at::empty({T, K}, gates.options());
  if (T == 0) return {dy, dg};
  auto stream = c10::hip::getCurrentHIPStream();
  const dim3 grid((T + 3) / 4);
  DLGM_DISPATCH_16(y.scalar_type(), E, {
    auto dp = reinterpret_cast<const E*>(dout.data_ptr());
    auto yp = reinterpret_cast<const E*>(y.data_ptr());
    auto dyp = reinterpret_cast<E*>(dy.data_ptr());
    auto pp = pos.data_ptr<int64_t>();
    auto gp = gates.data_ptr<float>();
    auto dgp = dg.data_ptr<float>();
    switch (K) {
      case 1: moe_combine_bwd_kernel<E, 1><<<grid, 256, 0, stream>>>(dp, yp, pp, gp, dyp, dgp, T, D); break;
      case 2: moe_combine_bwd_kernel<E, 2><<<grid, 256, 0, stream>>>(dp, yp, pp, gp, dyp, dgp, T, D); break;
      case 4: moe_combine_bwd_kernel<E, 4><<<grid, 256, 0, stream>>>(dp, yp, pp, gp, dyp, dgp, T, D); break;
      default: TORCH_CHECK(false, "moe: top-k must be 1, 2 or 4");
    }
  });
  DLGM_CHECK_HIP(hipGetLastError());
  return {dy, dg};
}
