// Hand-written MFMA GEMM for gfx950 (CDNA4): dense and expert-grouped, any operand layout.
//
// C[M, N] (=|+=) A[M, K] . B[K, N], bf16 operands, fp32 accumulation, written for the two GEMM
// families the engine runs outside hipBLASLt's sweet spot:
//
//  * weight gradients  dW = dY^T X: both operands arrive with the reduction (token) dimension as
//    the ROW index -- A = dY [T, out] and B = X [T, in] are "MN-contiguous". They are staged as
//    row-major [64 k][256] LDS images and read back K-contiguous with ds_read_b64_tr_b16 (the
//    hardware transpose read), so no HBM transpose pass is needed, and the fp32 gradient is
//    accumulated in the epilogue (beta = 1) straight into the optimizer's gradient partition;
//  * Mixtral experts (grouped): one launch covers every expert. Group sizes live on the DEVICE
//    (exclusive offsets over the expert-sorted rows), so the dispatch needs no host sync:
//      grouped-M  rows [off_e, off_e+1) of A and C use expert e's weight (forward / input grads);
//      grouped-K  the reduction runs over rows [off_e, off_e+1) and writes expert e's C (weight
//                 grads); an expert with no tokens gets zeros (store) or is left as is (accumulate).
//
// Structure (cdna_hip_programming.md §5): 256x256 block tile, BK = 64, 8 waves (2 along M x 4
// along N, 128x64 outputs per wave), v_mfma_f32_16x16x32_bf16 (the bf16 shape the chip clocks
// higher under DVFS, MI355X_MICROARCH.md 'DVFS give-back' (7)). Operand tiles move HBM -> LDS by
// LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction) through buffer descriptors
// whose record count bounds the valid rows (rows past a group's end read as zero), double
// buffered: tile t+1 is in flight while tile t's MFMAs run. LDS images:
//    K-contiguous operand: [256 rows][64 k], 128-B rows, 16-B chunk c stored at c ^ ((row>>1)&7);
//                          fragments by ds_read_b128 (conflict-free for the 16x16x32 lane map);
//    MN-contiguous operand: [64 k][256 cols], 512-B rows, chunk c at c ^ 2*((k&3) | ((k>>3)&1)<<2);
//                          fragments by two ds_read_b64_tr_b16 (conflict-free, T10).
// The XOR swizzles are applied to the DMA's per-lane SOURCE address (the DMA writes lane-linearly)
// and to the reads. The MFMA computes D^T = B^T A^T so each lane ends up holding 4 consecutive
// columns of one row of C: the epilogue moves 16-byte float4 (fp32) / 8-byte bf16x4 vectors.
// Work order: blocks are remapped so consecutive tiles (sharing an A row panel) land on one XCD.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int TILE_BYTES = 256 * BK * 2;  // one operand tile: 32 KiB

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) void* lptr_t;

enum Epi { kStoreBf16 = 0, kStoreF32 = 1, kAccF32 = 2 };
enum Mode { kDense = 0, kGroupM = 1, kGroupK = 2 };

struct GemmArgs {
  const bf16* a;
  const bf16* b;
  void* c;
  int64_t lda, ldb, ldc;           // leading (non-unit) strides in elements
  int64_t a_gstride, b_gstride, c_gstride;  // per-group pointer steps (elements) for grouped modes
  const int* offsets;              // [G + 1] exclusive prefix over the grouped dimension (device)
  int M, N, K;                     // K: dense / grouped-M reduction length; M: rows for dense/grouped-K
  int G, mode;
  int tiles_n, tiles_m;
};

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat4(bf16x4 a, bf16x4 b) {
  return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ int swz_k(int row) { return (row >> 1) & 7; }                          // K-contig image
__device__ __forceinline__ int swz_mn(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }  // MN-contig image

// One LDS-DMA piece through a buffer descriptor: 64 lanes x 16 B land lane-linearly at `lds`.
__device__ __forceinline__ void dma16(const void* base, uint32_t nbytes, uint32_t voff, uint32_t soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes,
                                                                             0x00020000),
                                           (lptr_t)lds, 16, voff, soff, 0, 0);
}

// Staging plan of one operand tile (256 rows/cols x 64 k): the per-lane byte offset is loop-invariant,
// each wave issues 4 pieces that differ by a scalar step (the swizzle period divides the piece step).
template <bool KMAJ>
struct Stager {
  uint32_t voff;
  uint32_t step;
  int wave;
  __device__ __forceinline__ Stager(int64_t ld, int wave_, int lane) : wave(wave_) {
    if constexpr (KMAJ) {  // piece j = rows 8j .. 8j+7 (128 B each); this wave: j = wave + 8 i
      const int row = 8 * wave + (lane >> 3), phys = lane & 7;
      const int c = phys ^ swz_k(row);
      voff = (uint32_t)((row * ld + c * 8) * 2);
      step = (uint32_t)(64 * ld * 2);
    } else {  // piece j = k rows 2j, 2j+1 (512 B each); this wave: j = wave + 8 i
      const int row = 2 * wave + (lane >> 5), phys = lane & 31;
      const int c = phys ^ swz_mn(row);
      voff = (uint32_t)((row * ld + c * 8) * 2);
      step = (uint32_t)(16 * ld * 2);
    }
  }
  // `base` = first element of the tile (row 0 / k row 0), `nbytes` bounds the valid region from base.
  // The piece step goes into the VGPR offset (a raw buffer's range check covers voffset only), and on
  // a partial tile (`nvalid` < rows of the image) rows past the end are clamped onto the last valid row,
  // so no lane ever addresses memory outside the operand whatever the range check does; the duplicated
  // rows are finite and are either masked out of the reduction (k rows, read_frag) or feed output
  // rows that are never stored (m / n rows).
  __device__ __forceinline__ void issue(char* img, const bf16* base, uint32_t nbytes, int64_t ld, int nvalid) const {
    constexpr int ROWS = KMAJ ? 256 : 64;
    // last line of defence: a lane whose 16 B would end past `nbytes` reads the tile's first chunk instead
    auto guard = [nbytes](uint32_t vo) { return vo + 16 <= nbytes ? vo : 0u; };
    if (__builtin_amdgcn_readfirstlane(nvalid) >= ROWS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dma16(base, nbytes, guard(voff + i * step), 0, img + (wave + 8 * i) * 1024);
      return;
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row, c;
      if constexpr (KMAJ) {
        row = 8 * wave + 64 * i + (lane >> 3);
        c = (lane & 7) ^ swz_k(row);
      } else {
        row = 2 * wave + 16 * i + (lane >> 5);
        c = (lane & 31) ^ swz_mn(row);
      }
      const int src = row < nvalid ? row : nvalid - 1;
      dma16(base, nbytes, guard((uint32_t)((src * ld + c * 8) * 2)), 0, img + (wave + 8 * i) * 1024);
    }
  }
};

// 16x16x32 fragment (lane: row/col l&15, k = 8(l>>4) + j) of the operand image, k-substep s.
// `kv` < BK: a partial K tile of an MN image -- elements with k >= kv are zeroed (their LDS rows
// hold a clamped copy of the last valid row).
template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag(const char* img, int r0, int s, int lane, int kv) {
  const int i = lane & 15, g = lane >> 4;
  if constexpr (KMAJ) {
    const int r = r0 + i, c = 4 * s + g;
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + ((c ^ swz_k(r)) << 4));
  } else {
    const int q = i >> 2, p = i & 3;
    const int ch = (r0 >> 3) + (p >> 1);
    const int k1 = 32 * s + 8 * g + q;
    const int x = swz_mn(k1);  // k1 and k1 + 4 share it
    const char* a = img + k1 * 512 + ((ch ^ x) << 4) + (p & 1) * 8;
    bf16x8 v = cat4(lds_tr(a), lds_tr(a + 4 * 512));
    if (__builtin_amdgcn_readfirstlane(kv) < BK) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (32 * s + 8 * g + j >= kv) v[j] = (bf16)0.f;
    }
    return v;
  }
}

__device__ __forceinline__ int xcd_remap(int id, int total) {
  const int q = total / 8, r = total % 8, x = id % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
}

template <int MODE, bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(NTHR, 1) void gemm_mfma_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * TILE_BYTES];  // [buf][A | B]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- which tile (and group) this block computes. The mode is a template parameter: each
  // instantiation has straight-line pointer setup (no mode-dependent phis for the operand bases).
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  int tm = 0, tn, grp = 0;
  int m_lo = 0, m_hi = p.M;  // valid rows of A / C for this block
  int k_lo = 0, k_hi = p.K;  // reduction range
  constexpr int CES = EPI == kStoreBf16 ? 2 : 4;
  if constexpr (MODE == kDense) {
    tm = id / p.tiles_n;
    tn = id - tm * p.tiles_n;
  } else if constexpr (MODE == kGroupM) {
    tn = id % p.tiles_n;
    int j = id / p.tiles_n;
    grp = -1;
    for (int e = 0; e < p.G; ++e) {
      const int lo = p.offsets[e], hi = p.offsets[e + 1];
      const int te = (hi - lo + BM - 1) / BM;
      if (j < te) {
        grp = e;
        m_lo = lo + j * BM;  // this block's first row (absolute)
        m_hi = hi;
        break;
      }
      j -= te;
    }
    if (grp < 0) return;  // spare block: the grid is sized for the worst case
  } else {  // grouped-K
    const int per = p.tiles_m * p.tiles_n;
    grp = id / per;
    const int rem = id - grp * per;
    tm = rem / p.tiles_n;
    tn = rem - tm * p.tiles_n;
    k_lo = p.offsets[grp];
    k_hi = p.offsets[grp + 1];
  }
  const bf16* A = p.a;
  const bf16* B = p.b + (MODE == kGroupM ? (int64_t)grp * p.b_gstride : 0);
  char* C = (char*)p.c + (MODE == kGroupK ? (int64_t)grp * p.c_gstride * CES : 0);
  const int m0 = MODE == kGroupM ? m_lo : tm * BM;
  const int n0 = tn * BN;
  const int rows_valid = min(BM, m_hi - m0);
  if (rows_valid <= 0) return;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)(0.f);

  const int nk = (k_hi - k_lo + BK - 1) / BK;
  if (nk > 0) {
    const Stager<AK> sa(p.lda, w, lane);
    const Stager<BKM> sb(p.ldb, w, lane);
    // A tile t: AK -> rows m0.., k from k_lo + 64t ; !AK -> k rows, columns m0..
    auto stage = [&](int buf, int t) {
      const int k0 = k_lo + t * BK;
      char* img = smem + buf * 2 * TILE_BYTES;
      const int kv = min(BK, k_hi - k0);
      if constexpr (AK) {
        const bf16* base = A + (int64_t)m0 * p.lda + k0;
        sa.issue(img, base, (uint32_t)(((int64_t)(rows_valid - 1) * p.lda + BK) * 2), p.lda, rows_valid);
      } else {
        const bf16* base = A + (int64_t)k0 * p.lda + m0;
        sa.issue(img, base, (uint32_t)(((int64_t)(kv - 1) * p.lda + BM) * 2), p.lda, kv);
      }
      if constexpr (BKM) {
        const bf16* base = B + (int64_t)n0 * p.ldb + k0;
        sb.issue(img + TILE_BYTES, base, (uint32_t)(((int64_t)(BN - 1) * p.ldb + BK) * 2), p.ldb, BN);
      } else {
        const bf16* base = B + (int64_t)k0 * p.ldb + n0;
        sb.issue(img + TILE_BYTES, base, (uint32_t)(((int64_t)(kv - 1) * p.ldb + BN) * 2), p.ldb, kv);
      }
    };
    auto tile = [&](auto bufc, int t) {
      constexpr int buf = decltype(bufc)::value;
      const char* aimg = smem + buf * 2 * TILE_BYTES;
      const char* bimg = aimg + TILE_BYTES;
      const int kv = min(BK, k_hi - (k_lo + t * BK));
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 bfr[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) bfr[ni] = read_frag<BKM>(bimg, wc * 64 + 16 * ni, s, lane, kv);
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) {
          const bf16x8 afr = read_frag<AK>(aimg, wr * 128 + 16 * mi, s, lane, kv);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(bfr[ni], afr, acc[mi][ni]);
        }
      }
    };
    stage(0, 0);
    for (int t = 0; t < nk; t += 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < nk) stage(1, t + 1);
      tile(std::integral_constant<int, 0>{}, t);
      if (t + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t + 2 < nk) stage(0, t + 2);
        tile(std::integral_constant<int, 1>{}, t + 1);
      }
    }
  }

  // ---- epilogue: lane holds C[m][n .. n+3] (m = column of D^T, n = 4 rows of D^T)
  const int i = lane & 15, g = lane >> 4;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int mrow = wr * 128 + 16 * mi + i;  // row within the block tile
    if (mrow >= rows_valid) continue;
    const int64_t m = m0 + mrow;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = n0 + wc * 64 + 16 * ni + 4 * g;
      if constexpr (EPI == kStoreBf16) {
        bf16x4 v = {(bf16)acc[mi][ni][0], (bf16)acc[mi][ni][1], (bf16)acc[mi][ni][2], (bf16)acc[mi][ni][3]};
        *reinterpret_cast<bf16x4*>(C + (m * p.ldc + n) * 2) = v;
      } else if constexpr (EPI == kStoreF32) {
        *reinterpret_cast<f32x4*>(C + (m * p.ldc + n) * 4) = acc[mi][ni];
      } else {
        f32x4* dst = reinterpret_cast<f32x4*>(C + (m * p.ldc + n) * 4);
        *dst = *dst + acc[mi][ni];
      }
    }
  }
}

template <int MODE, bool AK, bool BKM>
void launch_epi(int epi, dim3 grid, hipStream_t st, const GemmArgs& a) {
  if (epi == kStoreBf16)
    gemm_mfma_kernel<MODE, AK, BKM, kStoreBf16><<<grid, NTHR, 0, st>>>(a);
  else if (epi == kStoreF32)
    gemm_mfma_kernel<MODE, AK, BKM, kStoreF32><<<grid, NTHR, 0, st>>>(a);
  else
    gemm_mfma_kernel<MODE, AK, BKM, kAccF32><<<grid, NTHR, 0, st>>>(a);
}

}  // namespace

// out = a @ b (accumulate: out += a @ b), a logically [M, K], b logically [K, N], both bf16 with ONE unit
// stride each (any of the four layouts); out [M, N] bf16 (store) or fp32 (store / accumulate).
// mode 0 dense; mode 1 grouped-M: `offsets` [G+1] (int32, device) splits the M rows, b is [G, ...] with
// b_gstride elements per group; mode 2 grouped-K: offsets split the K rows, out is [G, M, N].
void dlgm_gemm_mfma(at::Tensor out, const at::Tensor& a, const at::Tensor& b, bool accumulate,
                    const c10::optional<at::Tensor>& offsets, int64_t mode, int64_t M, int64_t N, int64_t K,
                    int64_t G, int64_t b_gstride) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm_mfma: GPU tensors");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "gemm_mfma: bf16 operands");
  TORCH_CHECK(a.dim() == 2 && b.dim() >= 2 && out.dim() >= 2, "gemm_mfma: 2-D operand views");
  const bool out32 = out.scalar_type() == at::kFloat;
  TORCH_CHECK(out32 || (out.scalar_type() == at::kBFloat16 && !accumulate), "gemm_mfma: bf16 out only stores");
  TORCH_CHECK(out.stride(-1) == 1, "gemm_mfma: out must be row-major");
  // operand layouts: a as [M, K] (stride(1) == 1 -> K-contiguous) or M-contiguous (stride(0) == 1)
  const bool ak = a.stride(1) == 1;
  TORCH_CHECK(ak || a.stride(0) == 1, "gemm_mfma: a needs a unit stride");
  const int64_t lda = ak ? a.stride(0) : a.stride(1);
  const at::Tensor b2 = b.dim() == 3 ? b.select(0, 0) : b;  // grouped weights: one group's [K, N] view
  const bool bk = b2.stride(0) == 1 && b2.stride(1) != 1;     // element (k, n) at b[n * ldb + k]
  TORCH_CHECK(bk || b2.stride(1) == 1, "gemm_mfma: b needs a unit stride");
  const int64_t ldb = bk ? b2.stride(1) : b2.stride(0);
  const int64_t ldc = out.stride(-2);
  TORCH_CHECK(N % BN == 0, "gemm_mfma: N must be a multiple of 256");
  TORCH_CHECK(mode == kGroupM || M % BM == 0 || ak, "gemm_mfma: M-contiguous a needs M % 256 == 0");
  TORCH_CHECK(mode == kGroupK || K % BK == 0, "gemm_mfma: K must be a multiple of 64");
  // a group's reduction range ends anywhere: only the MN-contiguous images mask partial k tiles
  TORCH_CHECK(mode != kGroupK || (!ak && !bk), "gemm_mfma: grouped-K needs token-major (row = k) operands");
  TORCH_CHECK(mode != kGroupM || ak, "gemm_mfma: grouped-M needs row-major (K-contiguous) rows");
  TORCH_CHECK(mode == kDense || mode == kGroupM || mode == kGroupK, "gemm_mfma: bad mode");
  for (const at::Tensor* t : {&a, &b2}) {
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_mfma: operands 16-byte aligned");
  }
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "gemm_mfma: leading strides must keep 16-B rows");
  GemmArgs p{};
  p.a = reinterpret_cast<const bf16*>(a.data_ptr());
  p.b = reinterpret_cast<const bf16*>(b.data_ptr());
  p.c = out.data_ptr();
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.G = (int)G;
  p.mode = (int)mode;
  p.b_gstride = b_gstride;
  p.c_gstride = mode == kGroupK ? out.stride(0) : 0;
  p.tiles_n = (int)(N / BN);
  p.tiles_m = (int)((M + BM - 1) / BM);
  int64_t nblk;
  if (mode == kDense) {
    nblk = (int64_t)p.tiles_m * p.tiles_n;
  } else {
    TORCH_CHECK(offsets.has_value() && offsets->is_cuda() && offsets->scalar_type() == at::kInt &&
                    offsets->numel() == G + 1, "gemm_mfma: grouped modes need int32 offsets[G+1] on the GPU");
    p.offsets = offsets->data_ptr<int>();
    if (mode == kGroupM)
      nblk = ((M + BM - 1) / BM + G) * p.tiles_n;  // M = total rows: worst-case tiles over all groups
    else
      nblk = G * (int64_t)p.tiles_m * p.tiles_n;
  }
  if (nblk == 0) return;
  const int epi = !out32 ? kStoreBf16 : accumulate ? kAccF32 : kStoreF32;
  auto st = c10::hip::getCurrentHIPStream();
  dim3 grid((unsigned)nblk);
  if (mode == kDense) {
    if (ak && bk)
      launch_epi<kDense, true, true>(epi, grid, st, p);
    else if (ak)
      launch_epi<kDense, true, false>(epi, grid, st, p);
    else if (bk)
      launch_epi<kDense, false, true>(epi, grid, st, p);
    else
      launch_epi<kDense, false, false>(epi, grid, st, p);
  } else if (mode == kGroupM) {  // token rows x expert weights ([G, N, K] or [G, K, N])
    if (bk)
      launch_epi<kGroupM, true, true>(epi, grid, st, p);
    else
      launch_epi<kGroupM, true, false>(epi, grid, st, p);
  } else {  // token-major operands (checked above)
    launch_epi<kGroupK, false, false>(epi, grid, st, p);
  }
  DLGM_CHECK_HIP(hipGetLastError());
}
