// bf16 matrix transpose y[C, R] = x[R, C]^T (gfx950), used to hand hipBLASLt the
// K-contiguous operand layout for weight-gradient GEMMs (dW = dy^T x reads both operands
// with the token dimension -- the GEMM's K -- strided, a layout hipBLASLt runs ~25% slower).
//
// No LDS: each lane moves one 8x8 bf16 block through registers -- 8 row loads of 16 B,
// an in-register 8x8 transpose, 8 column-row stores of 16 B. A wave covers a 64x64 tile
// with lanes laid out 8 (row chunks) x 8 (column chunks), so each load instruction reads
// 8 full 128-B segments (8 rows) and each store instruction writes 8 full 128-B segments.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

// rows (optional): output column r of y takes source row rows[r] of x, or zeros when rows[r] < 0 (R = len(rows))
struct Sources {  // up to 8 row-major sources of one row stride, passed by value (no host-to-device copy)
  const bf16* p[8];
  int n;
};

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                             int64_t R, int64_t C, int64_t ldx, int64_t ldy,
                                                             const int* __restrict__ rows, Sources srcs) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // tile bookkeeping in 32 bits (a 64-bit divide is a long software sequence; tiles, R < 2^30 are checked on the host)
  const int tiles_c = (int)((C + 63) >> 6), tiles_r = (int)((R + 63) >> 6), tiles = tiles_r * tiles_c;
  const int kr = lane >> 3, kc = lane & 7;  // row chunk, column chunk inside the 64x64 tile
  // tiles walk super-columns of kSuper column tiles, row tiles within: the ~16k waves in flight cover
  // ~256 row tiles x 64 column tiles, so every output row is written in ~32 KB runs and every input row read
  // in 8 KB runs
  constexpr int kSuper = 64;
  const int wv = (int)wave, nw = (int)nwaves;
  auto tile_of = [&](int t, int& rt, int& ct) {
    const int sc = t / (tiles_r * kSuper), tt = t - sc * tiles_r * kSuper;
    const int w = min(kSuper, tiles_c - sc * kSuper);
    rt = tt / w;
    ct = sc * kSuper + (tt - rt * w);
  };
  auto store = [&](const short8 (&v)[8], int64_t r0, int64_t c0) {
    short8 o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[i][j] = v[j][i];
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<short8*>(y + (c0 + i) * ldy + r0) = o[i];
  };
  if (rows == nullptr) {
    for (int t = wv; t < tiles; t += nw) {
      int rt, ct;
      tile_of(t, rt, ct);
      const int64_t r0 = (int64_t)rt * 64 + kr * 8, c0 = (int64_t)ct * 64 + kc * 8;
      if (r0 >= R || c0 >= C) continue;  // R, C are multiples of 8: a chunk is wholly in or out
      short8 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const short8*>(x + (r0 + j) * ldx + c0);
      store(v, r0, c0);
    }
    return;
  }
  // remapped rows: lane l resolves the source row pointer of the tile's row l once (rows[] = (source << 24) | row,
  // or -1 for a zero row), a tile ahead so the data loads do not wait behind the index load; the 8 rows a lane
  // reads are then fetched from their owners by two lane shuffles each
  auto row_ptr = [&](int t) -> uint64_t {
    if (t >= tiles) return 0;
    int rt, ct;
    tile_of(t, rt, ct);
    const int64_t r = (int64_t)rt * 64 + lane;
    const int src = r < R ? rows[r] : -1;
    if (src < 0) return 0;
    const bf16* xs = x;
    int64_t row = src;
    if (srcs.n > 0) {
      const int si = src >> 24;
      xs = srcs.p[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) xs = si == q ? srcs.p[q] : xs;
      row = src & 0xFFFFFF;
    }
    return reinterpret_cast<uint64_t>(xs + row * ldx);
  };
  uint64_t next = row_ptr(wv);
  for (int t = wv; t < tiles; t += nw) {
    const uint64_t mine = next;
    next = row_ptr(t + nw);
    int rt, ct;
    tile_of(t, rt, ct);
    const int64_t r0 = (int64_t)rt * 64 + kr * 8, c0 = (int64_t)ct * 64 + kc * 8;
    uint64_t pj[8];  // (shuffled while every lane is active: a lane past the edge still serves its row)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int srcl = kr * 8 + j;
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)mine, srcl), hi = (uint32_t)__shfl((int)(mine >> 32), srcl);
      pj[j] = ((uint64_t)hi << 32) | lo;
    }
    if (r0 >= R || c0 >= C) continue;
    short8 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = pj[j] ? *reinterpret_cast<const short8*>(reinterpret_cast<const bf16*>(pj[j]) + c0) : (short8)(0);
    store(v, r0, c0);
  }
}

}  // namespace

// out[C, R] = x[R, C]^T (a remapped out allocated here has its rows padded to 64 elements: a [C, R] view); x may be a row-strided view (stride(1) == 1). With `rows` (int32 [R'],
// R' % 8 == 0) the transpose runs over a remapped row space: out[C, R'] with column r = x[rows[r]] (zeros for
// rows[r] < 0) -- e.g. expert-sorted rows re-laid with every expert starting on an aligned column.
at::Tensor dlgm_transpose(const at::Tensor& x, const c10::optional<at::Tensor>& out_opt,
                          const c10::optional<at::Tensor>& rows_opt) {
  // 16-bit payload moved bit-exactly: serves bf16 and fp16
  TORCH_CHECK(x.is_cuda() && DLGM_IS16(x) && x.dim() == 2, "transpose: bf16/fp16 2-D GPU tensor");
  TORCH_CHECK(x.stride(1) == 1, "transpose: rows must be contiguous");
  const bool remap = rows_opt.has_value() && rows_opt->defined();
  if (remap)
    TORCH_CHECK(rows_opt->is_cuda() && rows_opt->scalar_type() == at::kInt && rows_opt->is_contiguous() &&
                    rows_opt->dim() == 1, "transpose: rows must be a contiguous int32 GPU vector");
  const int64_t R = remap ? rows_opt->numel() : x.size(0), C = x.size(1);
  TORCH_CHECK(R % 8 == 0 && C % 8 == 0 && x.stride(0) % 8 == 0, "transpose: dims and row stride must be multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "transpose: input must be 16-byte aligned");
  // a remapped (padded-layout) out that is allocated here gets its rows padded to whole 128-B lines: with
  // R % 64 != 0 every 128-B chunk of a row would straddle two lines (a [28672, 33272] transpose ran at 3.1 TB/s
  // against 4.7 TB/s at R = 32768). The plain transpose keeps a contiguous out (its R is a token count).
  const int64_t ldy = out_opt.has_value() || !remap ? R : (R + 63) / 64 * 64;
  at::Tensor y = out_opt.has_value() ? *out_opt : at::empty({C, ldy}, x.options()).narrow(1, 0, R);
  TORCH_CHECK(y.sizes() == at::IntArrayRef({C, R}) && y.stride(0) == ldy && y.stride(1) == 1 &&
                  y.scalar_type() == x.scalar_type(), "transpose: out must be a contiguous [C, R] tensor of x's dtype");
  if (R == 0 || C == 0) return y;
  const int64_t tiles = ((R + 63) / 64) * ((C + 63) / 64);
  TORCH_CHECK(tiles < (int64_t(1) << 30) && R < (int64_t(1) << 30), "transpose: too many 64x64 tiles");
  // remapped: one 64x64 tile per wave (the MoE dW re-layout 6 % faster); plain: at most 16 workgroups per CU
  // walking tiles (the activation transposes of the Llama step ran 13 % slower with one tile per wave;
  // profiles/transpose_grid_ab_r04.json)
  const int64_t grid = remap ? (tiles + 3) / 4 : std::min<int64_t>((tiles + 3) / 4, 256 * 16);
  transpose_bf16_kernel<<<grid, 256, 0, c10::hip::getCurrentHIPStream()>>>(
      reinterpret_cast<const bf16*>(x.data_ptr()), reinterpret_cast<bf16*>(y.data_ptr()), R, C, x.stride(0), ldy,
      remap ? rows_opt->data_ptr<int>() : nullptr, Sources{{}, 0});
  DLGM_CHECK_HIP(hipGetLastError());
  return y;
}

// out[C, P] = the columns of several row-major sources x_s [R_s, C] (one row stride), laid out by `rows` (int32 [P],
// P % 8 == 0: (s << 24) | row, or -1 for a zero column): the deferred expert dW's K-contiguous operand with every
// expert's rows of all micro-batches contiguous (ops.moe.pad_plan_multi).
at::Tensor dlgm_transpose_multi(const std::vector<at::Tensor>& xs, const at::Tensor& rows) {
  TORCH_CHECK(!xs.empty() && xs.size() <= 8, "transpose_multi: 1..8 sources");
  const at::Tensor& x0 = xs[0];
  TORCH_CHECK(rows.is_cuda() && rows.scalar_type() == at::kInt && rows.is_contiguous() && rows.dim() == 1,
              "transpose_multi: rows must be a contiguous int32 GPU vector");
  const int64_t P = rows.numel(), C = x0.size(1);
  Sources srcs{{}, (int)xs.size()};
  for (const at::Tensor& x : xs) {
    TORCH_CHECK(x.is_cuda() && DLGM_IS16(x) && x.dim() == 2 && x.stride(1) == 1 && x.size(1) == C &&
                    x.stride(0) == x0.stride(0) && x.scalar_type() == x0.scalar_type() && x.size(0) < (1 << 24),
                "transpose_multi: sources [R_s, C] of one dtype and row stride, R_s < 2^24");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "transpose_multi: 16-byte aligned sources");
    srcs.p[&x - &xs[0]] = reinterpret_cast<const bf16*>(x.data_ptr());
  }
  TORCH_CHECK(P % 8 == 0 && C % 8 == 0 && x0.stride(0) % 8 == 0, "transpose_multi: P, C and the row stride % 8");
  const int64_t ldy = (P + 63) / 64 * 64;  // rows padded to whole 128-B lines (see dlgm_transpose)
  at::Tensor y = at::empty({C, ldy}, x0.options()).narrow(1, 0, P);
  if (P == 0 || C == 0) return y;
  const int64_t tiles = ((P + 63) / 64) * ((C + 63) / 64);
  TORCH_CHECK(tiles < (int64_t(1) << 30) && P < (int64_t(1) << 30), "transpose_multi: too many 64x64 tiles");
  const int64_t grid = (tiles + 3) / 4;  // one 64x64 tile per wave (see dlgm_transpose)
  transpose_bf16_kernel<<<grid, 256, 0, c10::hip::getCurrentHIPStream()>>>(
      reinterpret_cast<const bf16*>(x0.data_ptr()), reinterpret_cast<bf16*>(y.data_ptr()), P, C, x0.stride(0), ldy,
      rows.data_ptr<int>(), srcs);
  DLGM_CHECK_HIP(hipGetLastError());
  return y;
}
