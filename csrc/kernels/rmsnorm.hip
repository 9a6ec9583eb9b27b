// RMSNorm forward / backward (optionally fused with the residual add) for gfx950.
//
// Llama-style RMSNorm  y = x * rsqrt(mean(x^2) + eps) * w  sits twice in every
// transformer block.  Both directions are HBM-bound, so the
// kernels are built around 16-byte-per-lane accesses:
//   * one row per wave64: lane l owns 8-element chunks l, l+64, l+128, ... of the
//     row and keeps them in registers (no LDS round trip for the row data);
//   * the residual add of the block (h = x + r) is fused into the forward norm,
//     and the residual-gradient add (dx += dres) into the backward norm, so the
//     residual stream is read once per direction;
//   * dw (a column reduction over T rows) is reduced wave -> block in registers
//     and LDS, written as one fp32 partial row per block, and summed by a tiny
//     column-reduce kernel (deterministic, no float atomics).
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

constexpr int kThreads = 256;  // 4 waves -> 4 rows in flight per block
constexpr int kWaves = kThreads / 64;

template <typename E, int MAXC, bool RESID>
__global__ __launch_bounds__(kThreads) void rmsnorm_fwd_kernel(
    const E* __restrict__ x, const E* __restrict__ r, const E* __restrict__ w,
    E* __restrict__ y, E* __restrict__ h, float* __restrict__ rstd_out, int T, int D,
    float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= T) return;
  const int nch = D >> 3;
  const size_t base = (size_t)row * D;
  // the row is held as raw 16-bit values (4 VGPRs per 8 elements, widened on use): half the registers of an fp32
  // copy, so a whole T = 8192 launch is resident at once (same arithmetic, bit-identical outputs)
  vec8_t<E> v[MAXC];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      if constexpr (RESID) {
        // the normalised value is computed from the rounded residual stream, so forward and backward see the same h
        v[c] = __builtin_convertvector(load8f(x + base + ch * 8) + load8f(r + base + ch * 8), vec8_t<E>);
        *reinterpret_cast<vec8_t<E>*>(h + base + ch * 8) = v[c];
      } else {
        v[c] = *reinterpret_cast<const vec8_t<E>*>(x + base + ch * 8);
      }
      const f32x8 f = __builtin_convertvector(v[c], f32x8);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)D + eps);
  if (lane == 0) rstd_out[row] = rs;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      f32x8 wv = load8f(w + ch * 8);
      store8f(y + base + ch * 8, __builtin_convertvector(v[c], f32x8) * rs * wv);
    }
  }
}

// Backward. Grid-strided over rows: wave `gw` handles rows gw, gw+NW, ...
// dx = rstd * (dy*w - xhat * mean(dy*w*xhat)) (+ dres);   dw_partial[block] = sum dy*xhat
// Register budget is what sets this kernel's speed (HBM-bound, one memory round trip per row):
// the row is held as raw bf16 (4 VGPRs per 8 elements, widened on use), w is re-read from L1
// instead of pinned in 64 VGPRs, and the residual-gradient row is loaded together with dy and h,
// so a row costs ONE dependent HBM latency and 3 waves fit per SIMD (was 1-2, ~2.2 TB/s).
template <typename E, int MAXC, bool DRES>
__global__ __launch_bounds__(kThreads) void rmsnorm_bwd_kernel(
    const E* __restrict__ dy, const E* __restrict__ hin, const E* __restrict__ w,
    const float* __restrict__ rstd, const E* __restrict__ dres, E* __restrict__ dx,
    float* __restrict__ dw_part, int T, int D) {
  __shared__ __attribute__((aligned(16))) f32x8 red[kWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = D >> 3;
  const int nw = gridDim.x * kWaves;
  f32x8 acc[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) acc[c] = (f32x8)(0.f);
  for (int row = blockIdx.x * kWaves + wid; row < T; row += nw) {
    const size_t base = (size_t)row * D;
    const float rs = rstd[row];
    vec8_t<E> gr[MAXC], hr[MAXC], rr[DRES ? MAXC : 1];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        gr[c] = *reinterpret_cast<const vec8_t<E>*>(dy + base + ch * 8);
        hr[c] = *reinterpret_cast<const vec8_t<E>*>(hin + base + ch * 8);
        if constexpr (DRES) rr[c] = *reinterpret_cast<const vec8_t<E>*>(dres + base + ch * 8);
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        const f32x8 g = __builtin_convertvector(gr[c], f32x8);
        const f32x8 xh = __builtin_convertvector(hr[c], f32x8) * rs;
        acc[c] += g * xh;
        const f32x8 gw = g * load8f(w + ch * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) dot += gw[j] * xh[j];
      }
    }
    dot = wave_sum(dot) / (float)D;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        const f32x8 gw = __builtin_convertvector(gr[c], f32x8) * load8f(w + ch * 8);
        const f32x8 xh = __builtin_convertvector(hr[c], f32x8) * rs;
        f32x8 o = (gw - xh * dot) * rs;
        if constexpr (DRES) o += __builtin_convertvector(rr[c], f32x8);
        store8f(dx + base + ch * 8, o);
      }
    }
  }
  // block-level reduction of the dw accumulators, one 512-column chunk at a time
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (c * 64 >= nch) break;  // uniform across the block
    red[wid][lane] = acc[c];
    __syncthreads();
    if (wid == (c & (kWaves - 1))) {
      f32x8 s = red[0][lane];
#pragma unroll
      for (int k = 1; k < kWaves; ++k) s += red[k][lane];
      const int ch = lane + c * 64;
      if (ch < nch) {
        float* dst = dw_part + (size_t)blockIdx.x * D + ch * 8;
        *reinterpret_cast<f32x4*>(dst) = (f32x4){s[0], s[1], s[2], s[3]};
        *reinterpret_cast<f32x4*>(dst + 4) = (f32x4){s[4], s[5], s[6], s[7]};
      }
    }
    __syncthreads();
  }
}

// Backward for wide rows (D a multiple of 2048: Llama-3 8B/70B, Mixtral): one ROW per block
// iteration, thread t of the 256 owns the 8-element chunks t, t+256, ... (CPL of them). Each
// thread keeps its own dw columns for every row the block visits, so the block's dw partial needs
// no LDS reduction, and the per-thread state is tiny (~80 VGPRs -> 5-6 waves per SIMD): the row is
// loaded once (dy, h, dres together), reduced across the block through a 2-slot LDS array (one
// barrier per row; slot parity keeps a fast wave from overwriting a value a slow wave still reads).
// GUARD: rows whose chunk count is not a multiple of 256 (D = 5120, 6144, 7168, ...; without it those widths took
// the wave-per-row kernel at 16 chunks per lane, which spills 217-253 VGPRs): a thread's chunks past the row end
// hold zeros and store nothing.
template <typename E, int CPL, bool DRES, bool GUARD = false>
__global__ __launch_bounds__(kThreads) void rmsnorm_bwd_rowblock_kernel(
    const E* __restrict__ dy, const E* __restrict__ hin, const E* __restrict__ w,
    const float* __restrict__ rstd, const E* __restrict__ dres, E* __restrict__ dx,
    float* __restrict__ dw_part, int T, int D) {
  __shared__ float red[2][kWaves];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nch = D >> 3;
  auto live = [&](int c) { return !GUARD || tid + c * kThreads < nch; };
  f32x8 acc[CPL], wv[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    acc[c] = (f32x8)(0.f);
    wv[c] = live(c) ? load8f(w + (tid + c * kThreads) * 8) : (f32x8)(0.f);
  }
  const float inv_d = 1.f / (float)D;
  int it = 0;
  for (int row = blockIdx.x; row < T; row += gridDim.x, ++it) {
    const size_t base = (size_t)row * D;
    const float rs = rstd[row];
    vec8_t<E> gr[CPL], hr[CPL], rr[DRES ? CPL : 1];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const size_t off = base + (size_t)(tid + c * kThreads) * 8;
      if (live(c)) {
        gr[c] = *reinterpret_cast<const vec8_t<E>*>(dy + off);
        hr[c] = *reinterpret_cast<const vec8_t<E>*>(hin + off);
        if constexpr (DRES) rr[c] = *reinterpret_cast<const vec8_t<E>*>(dres + off);
      } else {
        gr[c] = hr[c] = (vec8_t<E>)((E)0.f);
        if constexpr (DRES) rr[c] = (vec8_t<E>)((E)0.f);
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const f32x8 g = __builtin_convertvector(gr[c], f32x8);
      const f32x8 xh = __builtin_convertvector(hr[c], f32x8) * rs;
      acc[c] += g * xh;
      const f32x8 gw = g * wv[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) dot += gw[j] * xh[j];
    }
    dot = wave_sum(dot);
    if (lane == 0) red[it & 1][wid] = dot;
    __syncthreads();
    dot = (red[it & 1][0] + red[it & 1][1] + red[it & 1][2] + red[it & 1][3]) * inv_d;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const f32x8 gw = __builtin_convertvector(gr[c], f32x8) * wv[c];
      const f32x8 xh = __builtin_convertvector(hr[c], f32x8) * rs;
      f32x8 o = (gw - xh * dot) * rs;
      if constexpr (DRES) o += __builtin_convertvector(rr[c], f32x8);
      if (live(c)) store8f(dx + base + (size_t)(tid + c * kThreads) * 8, o);
    }
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    if (!live(c)) continue;
    float* dst = dw_part + (size_t)blockIdx.x * D + (size_t)(tid + c * kThreads) * 8;
    *reinterpret_cast<f32x4*>(dst) = (f32x4){acc[c][0], acc[c][1], acc[c][2], acc[c][3]};
    *reinterpret_cast<f32x4*>(dst + 4) = (f32x4){acc[c][4], acc[c][5], acc[c][6], acc[c][7]};
  }
}

// dw[d] = (accumulate ? dw[d] : 0) + sum_b part[b][d]; each block owns 64 columns,
// its 4 waves split the partial rows, LDS combines them.
template <typename OutT>
__global__ __launch_bounds__(kThreads) void column_reduce_kernel(const float* __restrict__ part,
                                                                 OutT* __restrict__ out, int R,
                                                                 int D, bool accumulate) {
  __shared__ float red[kWaves][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < D) {
#pragma unroll 8
    for (int r = wid; r < R; r += kWaves) s += part[(size_t)r * D + col];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && col < D) {
    float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (accumulate) t += (float)out[col];
    out[col] = (OutT)t;
  }
}

// First pass of the dw reduction when the partial has many rows: part [R, D] -> part2 [gridDim.y, D].
// 256 consecutive columns per block (1 KiB per row read), blockIdx.y selects a slice of rows, so a
// [1024 x 4096] partial is read by 1024 blocks with 8 loads in flight per thread instead of 64
// blocks walking 1024 rows each.
__global__ __launch_bounds__(kThreads) void column_partial_kernel(const float* __restrict__ part,
                                                                  float* __restrict__ part2, int R, int D,
                                                                  int rows_per_slice) {
  const int col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= D) return;
  const int r0 = blockIdx.y * rows_per_slice;
  const int r1 = min(R, r0 + rows_per_slice);
  float s = 0.f;
#pragma unroll 8
  for (int r = r0; r < r1; ++r) s += part[(size_t)r * D + col];
  part2[(size_t)blockIdx.y * D + col] = s;
}

int max_chunks_for(int64_t D) {
  const int64_t per_lane = (D / 8 + 63) / 64;
  if (per_lane <= 2) return 2;
  if (per_lane <= 4) return 4;
  if (per_lane <= 8) return 8;
  if (per_lane <= 16) return 16;
  return -1;
}

void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(DLGM_IS16(t), name, " must be bf16 or fp16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

}  // namespace

std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_rmsnorm_fwd(const at::Tensor& x,
                                                                const c10::optional<at::Tensor>& residual,
                                                                const at::Tensor& w, double eps) {
  check_rows(x, "x");
  check_rows(w, "w");
  const int64_t D = x.size(-1);
  const int64_t T = x.numel() / D;
  TORCH_CHECK(D % 8 == 0, "rmsnorm: hidden size must be a multiple of 8");
  TORCH_CHECK(w.numel() == D, "rmsnorm: weight size mismatch");
  const int MAXC = max_chunks_for(D);
  TORCH_CHECK(MAXC > 0, "rmsnorm: hidden size too large (max 8192)");
  auto y = at::empty_like(x);
  auto rstd = at::empty({T}, x.options().dtype(at::kFloat));
  at::Tensor h;
  const bool resid = residual.has_value() && residual->defined();
  if (resid) {
    check_rows(*residual, "residual");
    TORCH_CHECK(residual->numel() == x.numel(), "rmsnorm: residual shape mismatch");
    h = at::empty_like(x);
  }
  if (T == 0) return {y, resid ? h : x, rstd};
  auto stream = c10::hip::getCurrentHIPStream();
  const dim3 grid((T + kWaves - 1) / kWaves);
  TORCH_CHECK(w.scalar_type() == x.scalar_type() && (!resid || residual->scalar_type() == x.scalar_type()),
              "rmsnorm: x, residual and w must share one dtype");
#define LAUNCH_FWD(C)                                                                        \
  if (resid)                                                                                 \
    rmsnorm_fwd_kernel<E, C, true><<<grid, kThreads, 0, stream>>>(xp, rp, wp, yp, hp,        \
                                                               rstd.data_ptr<float>(), T, D, \
                                                               (float)eps);                  \
  else                                                                                       \
    rmsnorm_fwd_kernel<E, C, false><<<grid, kThreads, 0, stream>>>(xp, rp, wp, yp, hp,       \
                                                                rstd.data_ptr<float>(), T, D, \
                                                                (float)eps);
  DLGM_DISPATCH_16(x.scalar_type(), E, {
  auto xp = reinterpret_cast<const E*>(x.data_ptr());
  auto rp = resid ? reinterpret_cast<const E*>(residual->data_ptr()) : nullptr;
  auto wp = reinterpret_cast<const E*>(w.data_ptr());
  auto yp = reinterpret_cast<E*>(y.data_ptr());
  auto hp = resid ? reinterpret_cast<E*>(h.data_ptr()) : nullptr;
  switch (MAXC) {
    case 2: LAUNCH_FWD(2); break;
    case 4: LAUNCH_FWD(4); break;
    case 8: LAUNCH_FWD(8); break;
    default: LAUNCH_FWD(16); break;
  }
  });
#undef LAUNCH_FWD
  DLGM_CHECK_HIP(hipGetLastError());
  return {y, resid ? h : x, rstd};
}

// Returns dx. dw (bf16 or fp32, D elements, may be a view into a flat grad buffer)
// receives sum_t dy*xhat (added to its old value when accumulate_dw).
at::Tensor dlgm_rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w,
                            const at::Tensor& rstd, const c10::optional<at::Tensor>& dres,
                            at::Tensor dw, bool accumulate_dw) {
  check_rows(dy, "dy");
  check_rows(h, "h");
  check_rows(w, "w");
  const int64_t D = dy.size(-1);
  const int64_t T = dy.numel() / D;
  TORCH_CHECK(h.numel() == dy.numel(), "rmsnorm_bwd: shape mismatch");
  TORCH_CHECK(rstd.numel() == T && rstd.scalar_type() == at::kFloat, "rmsnorm_bwd: bad rstd");
  TORCH_CHECK(dw.numel() == D && dw.is_contiguous(), "rmsnorm_bwd: bad dw");
  const int MAXC = max_chunks_for(D);
  TORCH_CHECK(MAXC > 0 && D % 8 == 0, "rmsnorm_bwd: unsupported hidden size");
  const bool has_dres = dres.has_value() && dres->defined();
  if (has_dres) check_rows(*dres, "dres");
  auto dx = at::empty_like(dy);
  auto stream = c10::hip::getCurrentHIPStream();
  int64_t nblk = 0;
  at::Tensor part;
  TORCH_CHECK(h.scalar_type() == dy.scalar_type() && w.scalar_type() == dy.scalar_type() &&
                  (!has_dres || dres->scalar_type() == dy.scalar_type()), "rmsnorm_bwd: mixed dtypes");
  const int cpl = (D % (8 * kThreads) == 0) ? (int)(D / (8 * kThreads)) : 0;
  const bool guarded = cpl == 0 && D > 4096;  // 4096 < D <= 8192, not a multiple of 2048: guarded 4-chunk row block
#define LAUNCH_ROWBLOCK(C)                                                                                  \
    if (has_dres)                                                                                           \
      rmsnorm_bwd_rowblock_kernel<E, C, true><<<nblk, kThreads, 0, stream>>>(dyp, hp, wp, rstd.data_ptr<float>(), \
                                                                        drp, dxp, part.data_ptr<float>(), T, D); \
    else                                                                                                    \
      rmsnorm_bwd_rowblock_kernel<E, C, false><<<nblk, kThreads, 0, stream>>>(dyp, hp, wp, rstd.data_ptr<float>(), \
                                                                         drp, dxp, part.data_ptr<float>(), T, D);
#define LAUNCH_ROWBLOCK_GUARD                                                                              \
    if (has_dres)                                                                                           \
      rmsnorm_bwd_rowblock_kernel<E, 4, true, true><<<nblk, kThreads, 0, stream>>>(                         \
          dyp, hp, wp, rstd.data_ptr<float>(), drp, dxp, part.data_ptr<float>(), T, D);                     \
    else                                                                                                    \
      rmsnorm_bwd_rowblock_kernel<E, 4, false, true><<<nblk, kThreads, 0, stream>>>(                        \
          dyp, hp, wp, rstd.data_ptr<float>(), drp, dxp, part.data_ptr<float>(), T, D);
#define LAUNCH_BWD(C)                                                                                \
    if (has_dres)                                                                                    \
      rmsnorm_bwd_kernel<E, C, true><<<nblk, kThreads, 0, stream>>>(dyp, hp, wp, rstd.data_ptr<float>(),  \
                                                                 drp, dxp, part.data_ptr<float>(), T, D); \
    else                                                                                             \
      rmsnorm_bwd_kernel<E, C, false><<<nblk, kThreads, 0, stream>>>(dyp, hp, wp, rstd.data_ptr<float>(), \
                                                                  drp, dxp, part.data_ptr<float>(), T, D);
  DLGM_DISPATCH_16(dy.scalar_type(), E, {
  auto dyp = reinterpret_cast<const E*>(dy.data_ptr());
  auto hp = reinterpret_cast<const E*>(h.data_ptr());
  auto wp = reinterpret_cast<const E*>(w.data_ptr());
  auto drp = has_dres ? reinterpret_cast<const E*>(dres->data_ptr()) : nullptr;
  auto dxp = reinterpret_cast<E*>(dx.data_ptr());
  if (cpl == 1 || cpl == 2 || cpl == 4 || guarded) {
    // block-per-row kernel: 1024 blocks (~5 resident per CU), 8 rows each at T = 8192
    nblk = std::max<int64_t>(1, std::min<int64_t>(T, 1024));
    part = at::empty({nblk, D}, dy.options().dtype(at::kFloat));
    if (T > 0) {
      if (guarded) {
        LAUNCH_ROWBLOCK_GUARD;
      } else {
        switch (cpl) {
          case 1: LAUNCH_ROWBLOCK(1); break;
          case 2: LAUNCH_ROWBLOCK(2); break;
          default: LAUNCH_ROWBLOCK(4); break;
        }
      }
    } else {
      part.zero_();
    }
  } else {
    // wave-per-row kernel for narrow rows: 3 waves / SIMD over 256 CUs = 768 blocks of 4 waves
    nblk = std::max<int64_t>(1, std::min<int64_t>((T + kWaves - 1) / kWaves, 768));
    part = at::empty({nblk, D}, dy.options().dtype(at::kFloat));
    switch (MAXC) {
      case 2: LAUNCH_BWD(2); break;
      case 4: LAUNCH_BWD(4); break;
      case 8: LAUNCH_BWD(8); break;
      default: LAUNCH_BWD(16); break;
    }
  }
  });
#undef LAUNCH_ROWBLOCK
#undef LAUNCH_ROWBLOCK_GUARD
#undef LAUNCH_BWD
  DLGM_CHECK_HIP(hipGetLastError());
  // many partial rows: fold them 16 at a time in a wide first pass (fixed order: deterministic)
  constexpr int kSlice = 16;
  int64_t rows = nblk;
  if (nblk > 4 * kSlice) {
    const int64_t slices = (nblk + kSlice - 1) / kSlice;
    auto part2 = at::empty({slices, D}, part.options());
    const dim3 pgrid((D + kThreads - 1) / kThreads, slices);
    column_partial_kernel<<<pgrid, kThreads, 0, stream>>>(part.data_ptr<float>(), part2.data_ptr<float>(), nblk,
                                                          D, kSlice);
    DLGM_CHECK_HIP(hipGetLastError());
    part = part2;
    rows = slices;
  }
  const dim3 rgrid((D + 63) / 64);
  if (dw.scalar_type() == at::kFloat)
    column_reduce_kernel<float><<<rgrid, kThreads, 0, stream>>>(part.data_ptr<float>(),
                                                                dw.data_ptr<float>(), rows, D,
                                                                accumulate_dw);
  else {
    DLGM_DISPATCH_16(dw.scalar_type(), E, column_reduce_kernel<E><<<rgrid, kThreads, 0, stream>>>(
        part.data_ptr<float>(), reinterpret_cast<E*>(dw.data_ptr()), rows, D, accumulate_dw));
  }
  DLGM_CHECK_HIP(hipGetLastError());
  return dx;
}
