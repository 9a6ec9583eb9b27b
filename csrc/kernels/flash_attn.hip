// Causal GQA flash attention, forward + backward, hand-written for gfx950 (CDNA4).
//
// SURVEY.md §2.6 K6 -- the largest non-GEMM compute kernel of Llama-3 / Mixtral
// training. Designed for the CDNA4 execution model, not translated from a
// warp-32 CUDA kernel:
//
//  * MFMA v_mfma_f32_32x32x16_bf16 everywhere, wave64 fragment maps
//    (lane l: r = l&31, h = l>>5; A[r][8h+j], B[8h+j][r];
//     C/D col = l&31, row = (reg&3) + 8*(reg>>2) + 4h).
//  * Forward uses the *swapped* product S^T = K * Q^T: every lane holds one query
//    column, so the softmax row reductions are lane-local plus ONE cross-half
//    shuffle, and the S^T accumulator is directly the B operand of O^T += V^T P^T
//    (no LDS round trip for P).
//  * V^T operands come from the row-major V tile through ds_read_b64_tr_b16
//    (hardware transpose read); K is read with ds_read_b128. Both LDS images are
//    XOR-swizzled on 16-byte chunks so every read is bank-conflict free.
//  * K/V (forward, dQ) and Q/dO (dK/dV) tiles arrive by LDS-DMA (buffer_load ... lds,
//    TileDma): 16 B per lane landing lane-linearly, the swizzle applied to the source
//    offset, the tile advance a scalar soffset; tile t+1 is in flight while tile t's
//    MFMAs run (one barrier per tile).
//  * Work ordering: causal blocks are launched heaviest-first, and blocks that
//    share one (batch, kv-head) -- i.e. the same K/V stream -- are grouped on one
//    XCD (blockIdx % 8 labels an XCD) so the K/V re-reads of the GQA group hit L2.
//  * Backward = two deterministic passes, no atomics (an atomic-dQ single pass would move
//    2.15 GB of fp32 adds per Llama-3-8B layer at S = 8192, >= 1.65 ms at the chip-wide
//    float-atomic rate):
//      dQ (first): one workgroup per (b, q head, 128 queries), the forward's structure; it also computes
//        delta = rowsum(dO * O) for its rows (it holds dO in registers) and writes the [-delta, -lse/scale]
//        rows dK/dV starts its accumulators from; dS^T is used in place as the B operand of dQ^T += K^T dS^T;
//      dK/dV: one workgroup per (b, q head, 128 keys), the wave's 32 keys on the MFMA lanes,
//        K in registers, V in LDS, S^T / dP^T computed with the key on the lane so they feed
//        dV^T / dK^T as accumulator operands; fp32 per-q-head partials, summed over the GQA
//        group by gqa_reduce into the packed dqkv.
//    Measured and removed (round 3): a separate delta launch (the fused one saves it), dQ on a side stream beside
//    dK/dV (2.20 vs 1.92 ms: both fill the chip), dQ from a dS^T stored by dK/dV (dQ 750 -> 519 us but dK/dV
//    1116 -> 1307 us for 2.15 GB of dS^T writes at the board's power limit: +0.1-0.2 % end to end for +2.3 GiB).
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __fp16 hf16x4 __attribute__((ext_vector_type(4)));  // the transpose-read builtin's f16 vector type
typedef __attribute__((address_space(3))) hf16x4 lds_f16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
// Deferred rescale (forward): the running max used for exponentiation is only raised when a
// row's new max exceeds it by more than 2^kRescaleLog2 -- P stays <= 256, exact in fp32 sums.
constexpr float kRescaleLog2 = 8.f;

// v_exp_f32 as is: exp2f() adds a denormal range fix-up (cmp + cndmask + ldexp per element) that
// softmax does not need (arguments are <= 0 up to the deferred-rescale slack; underflow -> 0).
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Packed fp32 pairs: v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 do two lanes' worth of softmax arithmetic per
// issue slot. The attention loops are bound by vector-instruction issue next to the MFMAs (PMC: 5-8 VALU per
// MFMA), so the elementwise work runs on pairs of accumulator registers.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// A condition the caller knows is wave-uniform, made provably so (scalar branch, no exec masking).
__device__ __forceinline__ bool uniform(bool c) { return __builtin_amdgcn_readfirstlane((int)c) != 0; }

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// fp16 compute path (DeepSpeed "fp16" block): the same fragment maps on the f16 MFMA
__device__ __forceinline__ f32x16 mfma32(const f16x8& a, const f16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// 16-byte-chunk XOR swizzles (see header). D = head dim, rows of D bf16.
template <int D>
__device__ __forceinline__ int swz_row(int row, int ch) {  // image read by ds_read_b128 rows
  if constexpr (D == 128) return ch ^ (row & 15);
  else return ch ^ ((row >> 1) & 7);
}
template <int D>
__device__ __forceinline__ int swz_tr(int row, int ch) {  // image read by ds_read_b64_tr_b16
  if constexpr (D == 128) return ch ^ ((row & 3) << 2);
  else return ch ^ (((row >> 1) & 1) << 2);
}
// One image good for both kinds of read (used by the backward's Q / dO / K tiles):
// plain 256-B rows, chunk ^ (((row&3)<<2) | ((row>>2)&3)); the 128-B-row variant
// for D = 64 folds the row parity in instead.
template <int D>
__device__ __forceinline__ int swz_dual(int row, int ch) {
  if constexpr (D == 128) return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  else return ch ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
}

// Makes x opaque to the optimiser: a per-lane LDS offset computed once before a loop then stays in its
// register instead of being rebuilt from its row and swizzle parts inside the loop (hipcc re-added
// them before every read: one v_add_u32 per ds_read in the backward's tile loops).
__device__ __forceinline__ void pin(int& x) { asm volatile("" : "+v"(x)); }

template <typename E>
__device__ __forceinline__ vec8_t<E> lds_read_b128(const E* base) {
  return *reinterpret_cast<const vec8_t<E>*>(base);
}

// x of lane i ^ 32 (the other half-wave): one v_permlane32_swap instead of an LDS bpermute round trip
__device__ __forceinline__ float swap_halves(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(__lane_id() < 32 ? r[1] : r[0]);
}

// Store one 32-row x D accumulator row block (lane (r, h) holds columns 8k + 4h .. +3 of row r for
// each 8-column group k) as bf16, scaled. One half-exchange (v_permlane32_swap) per dword of a group
// pair (k, k+1) leaves lanes h = 0 with columns 8k .. 8k+7 and lanes h = 1 with 8k+8 .. 8k+15: one
// 16-byte store per pair instead of two 8-byte stores (the tail is store-issue bound). Both lanes of
// a pair share the row, so the swap runs on all lanes and only the store is guarded by `valid`.
template <int DT, typename E>
__device__ __forceinline__ void store_rows_bf16(E* row, const f32x16 (&acc)[DT], float scale, int h, bool valid) {
#pragma unroll
  for (int k = 0; k < 4 * DT; k += 2) {
    const f32x16& oa = acc[k >> 2];
    const f32x16& ob = acc[(k + 1) >> 2];
    const int ja = 4 * (k & 3), jb = 4 * ((k + 1) & 3);
    vec4_t<E> va = {(E)(oa[ja] * scale), (E)(oa[ja + 1] * scale), (E)(oa[ja + 2] * scale),
                    (E)(oa[ja + 3] * scale)};
    vec4_t<E> vb = {(E)(ob[jb] * scale), (E)(ob[jb + 1] * scale), (E)(ob[jb + 2] * scale),
                    (E)(ob[jb + 3] * scale)};
    uint2 a = __builtin_bit_cast(uint2, va), c = __builtin_bit_cast(uint2, vb);
    const auto sx = __builtin_amdgcn_permlane32_swap(a.x, c.x, false, false);
    const auto sy = __builtin_amdgcn_permlane32_swap(a.y, c.y, false, false);
    if (valid) *reinterpret_cast<uint4*>(row + 8 * k + 8 * h) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
  }
}

__device__ __forceinline__ bf16x4 lds_read_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
__device__ __forceinline__ f16x4 lds_read_tr(const f16* p) {
  return __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_f16x4*)(p)));
}

__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ f16x8 cat(f16x4 a, f16x4 b) {
  return (f16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// One LDS-DMA piece: 64 lanes x 16 B = 1 KiB landing lane-linearly at `lds` (wave-uniform).
__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)lds, 4, 0, 0);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One LDS-DMA piece through a buffer descriptor (buffer_load_dwordx4 ... lds): `base` and `nbytes`
// are wave-uniform (the descriptor lives in SGPRs, reads at or past nbytes return zero), `voff`
// is the per-lane byte offset, `soff` a wave-uniform byte offset (the tile advance).
__device__ __forceinline__ void dma16(const void* base, int nbytes, uint32_t voff, uint32_t soff, lptr_t lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes,
                                                                             0x00020000),
                                           lds, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ void dma16(const void* base, int nbytes, uint32_t voff, uint32_t soff, void* lds) {
  dma16(base, nbytes, voff, soff, (lptr_t)lds);
}

// Loop-invariant LDS-DMA plan for a tile of ROWS x D bf16 rows that is re-staged every iteration
// (the forward's recipe): the per-lane byte offsets of this wave's pieces are computed once, a
// tile is then PPW buffer_load...lds per wave with a scalar row advance and no VALU. On the tail
// tile rows at or past S re-read row S-1 (so no address leaves the tensor). SWZ: 0 = row image, 1 = dual image, 2 = tr image.
// A wave's pieces sit NW*PR rows apart (16 at D = 128, 32 at D = 64), a multiple of every swizzle's
// row period, so they share ONE per-lane offset (1 VGPR) and differ only by a scalar soffset step.
template <typename E, int D, int ROWS, int SWZ, bool TAIL, int NW = 4>
struct TileDma {
  static constexpr int CH = D / 8, PR = 64 / CH, NP = ROWS / PR, PPW = NP / NW;
  static_assert(NP % NW == 0, "pieces must split evenly over the waves");
  static_assert((NW * PR) % 16 == 0, "piece row step must be a multiple of the swizzle period");
  uint32_t off0;
  int wave, nbytes, nrows;
  int64_t stride;
  const E* base;
  __device__ __forceinline__ TileDma(const E* base_, int64_t row_stride, int nrows_, int wave_, int lane)
      : wave(wave_), nbytes((int)(((int64_t)(nrows_ - 1) * row_stride + D) * 2)), nrows(nrows_), stride(row_stride),
        base(base_) {
    const int rin = lane / CH, phys = lane % CH;
    const int row = wave * PR + rin;
    const int logical = SWZ == 2 ? swz_tr<D>(row, phys) : SWZ == 1 ? swz_dual<D>(row, phys) : swz_row<D>(row, phys);
    off0 = (uint32_t)((row * row_stride + logical * 8) * 2);
  }
  // extra_soff: a wave-uniform byte offset added to every piece (the second head of a dK/dV workgroup),
  // covered by extend()
  __device__ __forceinline__ void extend(int64_t bytes) { nbytes += (int)bytes; }
  __device__ __forceinline__ void issue(E* img, int row0, uint32_t extra_soff = 0) const {
    if (!TAIL || row0 + ROWS <= nrows) {  // whole tile in range: scalar row advance
      const uint32_t step = (uint32_t)(NW * PR * stride * 2);
      uint32_t soff = (uint32_t)(row0 * stride * 2) + extra_soff;
      uint32_t lds = (uint32_t)(uintptr_t)(lptr_t)(img + wave * 512);  // LDS byte offset
      // both offsets advance piece by piece in scalar registers, made opaque to the optimiser: hoisted out of the
      // tile loop as PPW precomputed values per tile image they outgrew the SGPR file and came back through
      // v_readlane -- two vector instructions per LDS-DMA piece in the forward / dQ loops
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        dma16(base, nbytes, off0, soff, (lptr_t)(uintptr_t)lds);
        soff += step;
        lds += NW * 512 * (uint32_t)sizeof(E);
        asm volatile("" : "+s"(soff), "+s"(lds));
      }
      return;
    }
    if constexpr (TAIL) {
      // tail tile (S % tile != 0 -- a separate instantiation, so the full-tile kernels keep their
      // registers): every address stays inside the tensor -- rows at or past nrows re-read row
      // nrows-1 (finite; masked to zero weight by the kernels), the whole offset goes through voffset
      const int rin = wave * PR + (int)(threadIdx.x & 63) / CH;
#pragma unroll
      for (int j = 0; j < PPW; ++j) {
        const int r = min(row0 + NW * PR * j + rin, nrows - 1);
        dma16(base, nbytes, off0 + (uint32_t)((int64_t)(r - rin) * stride * 2), extra_soff, img + (wave + NW * j) * 512);
      }
    }
  }
};

// bijective remap of the block id so that consecutive work items land on one XCD
__device__ __forceinline__ int xcd_remap(int id, int total) {
  if (total % 8 != 0) return id;
  return (id % 8) * (total / 8) + id / 8;
}

template <typename E>
struct FwdParams {
  const E* q;
  const E* k;
  const E* v;
  E* o;
  float* lse;
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int B, S, Hq, Hkv;
  float scale_log2;  // softmax_scale * log2(e)
  bool causal;
};

constexpr int kFwdThreads = 256;
constexpr int kFwdBQ = 128;  // 4 waves x 32 query rows
constexpr int kFwdBKV = 64;

template <typename E, int D, bool TAIL>
__global__ __launch_bounds__(kFwdThreads, 2) void flash_fwd_kernel(FwdParams<E> p) {
  constexpr int CH = D / 8;   // 16-byte chunks per row
  constexpr int KK = D / 16;  // MFMA k-steps over the head dim
  constexpr int DT = D / 32;  // 32-wide output tiles over the head dim
  constexpr int TILE = kFwdBKV * D;
  __shared__ __attribute__((aligned(16))) E smem[4 * TILE];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, i16 = lane & 15, g = lane >> 4;

  const int nqt = (p.S + kFwdBQ - 1) / kFwdBQ;
  const int group = p.Hq / p.Hkv;
  const int total = gridDim.x;
  const int work = xcd_remap(blockIdx.x, total);
  const int per_kv = group * nqt;  // blocks sharing one (b, kv head)
  const int bk = work / per_kv;
  const int rem = work - bk * per_kv;
  const int qt = nqt - 1 - rem / group;  // heaviest (last) query tile first
  const int hq = (bk % p.Hkv) * group + rem % group;
  const int b = bk / p.Hkv;
  const int hk = hq / group;

  const int q0 = qt * kFwdBQ;
  const int q0w = q0 + 32 * w;
  const E* qb = p.q + b * p.q_sb + hq * p.q_sh;
  const E* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const E* vb = p.v + b * p.v_sb + hk * p.v_sh;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q0w + r][16kk + 8h .. +7]
  vec8_t<E> qf[KK];
  {
    const int qrow = q0w + r;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      qf[kk] = qrow < p.S ? *reinterpret_cast<const vec8_t<E>*>(qb + (int64_t)qrow * p.q_ss + 16 * kk + 8 * h)
                          : (vec8_t<E>)((E)0.f);
  }

  const int kv_end = p.causal ? min(p.S, q0 + kFwdBQ) : p.S;
  const int nt = (kv_end + kFwdBKV - 1) / kFwdBKV;

  // K/V tiles arrive by LDS-DMA (buffer_load ... lds, TileDma): 16 B per lane landing
  // lane-linearly, the XOR swizzle applied to the SOURCE offset, the tile advance a scalar soffset
  // -- staging costs no VALU and no VGPR round trip; rows past S read as zero.
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const TileDma<E, D, kFwdBKV, 0, TAIL> kdma(kb, p.k_ss, p.S, wu, lane);
  const TileDma<E, D, kFwdBKV, 2, TAIL> vdma(vb, p.v_ss, p.S, wu, lane);
  auto stage = [&](int buf, int t) {
    kdma.issue(smem + buf * TILE, t * kFwdBKV);
    vdma.issue(smem + (2 + buf) * TILE, t * kFwdBKV);
  };

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x16)(0.f);
  float m_run = -INFINITY, l_run = 0.f;
  const int qcol = q0w + r;

  // One KV tile. The loop below is unrolled by two so that the LDS buffer is a compile-time
  // constant in each copy: every ds_read then addresses (per-lane offset VGPR + immediate), with no
  // per-read address add in the loop.
  auto tile = [&](auto bufc, int t) {
    constexpr int buf = decltype(bufc)::value;
    vm_drain();  // this tile's DMA has landed (this wave's pieces) ...
    __syncthreads();  // ... and every wave's; the other buffer's readers are done
    if (t + 1 < nt) stage(buf ^ 1, t + 1);
    const int kv0 = t * kFwdBKV;
    if (p.causal && kv0 > q0w + 31) return;  // whole tile above this wave's diagonal
    const E* kt = smem + buf * TILE;
    const E* vt = smem + (2 + buf) * TILE;

    // ---- S^T = K Q^T for two 32-key subtiles
    f32x16 s[2] = {(f32x16)(0.f), (f32x16)(0.f)};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int row = 32 * u + r;
        vec8_t<E> a = lds_read_b128(kt + row * D + swz_row<D>(row, 2 * kk + h) * 8);
        s[u] = mfma32(a, qf[kk], s[u]);
      }
    }

    // ---- masking (only on diagonal / tail tiles)
    const bool need_mask = uniform((p.causal && kv0 + kFwdBKV - 1 > q0w) || (kv0 + kFwdBKV > p.S));
    if (need_mask) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kv = kv0 + 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (kv >= p.S || (p.causal && kv > qcol)) s[u][i] = -INFINITY;
        }
    }

    // ---- online softmax (log2 domain), row = this lane's query
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[u][i]);
    mx = fmaxf(mx, swap_halves(mx)) * p.scale_log2;
    // raise the reference max only when some row of the wave outgrew it by > 2^kRescaleLog2
    // (wave-uniform branch: the common case skips the O / l rescale entirely)
    if (__any(mx > m_run + kRescaleLog2)) {
      const float m_new = fmaxf(m_run, mx);
      const float alpha = m_new == -INFINITY ? 1.f : fast_exp2(m_run - m_new);
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    }
    const float m_use = m_run == -INFINITY ? 0.f : m_run;
    vec8_t<E> pf[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = fast_exp2(s[u][i] * p.scale_log2 - m_use);
        s[u][i] = e;
        l_run += e;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        pf[u][s2] = (vec8_t<E>){(E)s[u][8 * s2 + 0], (E)s[u][8 * s2 + 1], (E)s[u][8 * s2 + 2],
                             (E)s[u][8 * s2 + 3], (E)s[u][8 * s2 + 4], (E)s[u][8 * s2 + 5],
                             (E)s[u][8 * s2 + 6], (E)s[u][8 * s2 + 7]};
    }

    // ---- O^T += V^T P^T  (P^T accumulator used in place as the B operand)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = dt * 32 + 16 * (g & 1) + 4 * (i16 & 3);
      const int ch = col >> 3, within = col & 7;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r1 = 32 * u + 16 * s2 + 4 * h + (i16 >> 2);
          const int r2 = r1 + 8;
          vec4_t<E> a1 = lds_read_tr(vt + r1 * D + swz_tr<D>(r1, ch) * 8 + within);
          vec4_t<E> a2 = lds_read_tr(vt + r2 * D + swz_tr<D>(r2, ch) * 8 + within);
          o[dt] = mfma32(cat(a1, a2), pf[u][s2], o[dt]);
        }
    }
  };
  stage(0, 0);
  for (int t = 0; t < nt; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < nt) tile(std::integral_constant<int, 1>{}, t + 1);
  }

  // ---- epilogue: normalise, store O [b, q, hq, d] and LSE [b, hq, q]
  const float l_tot = l_run + swap_halves(l_run);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  store_rows_bf16<DT>(p.o + (((int64_t)b * p.S + qcol) * p.Hq + hq) * D, o, inv, h, qcol < p.S);
  if (qcol < p.S && h == 0) p.lse[((int64_t)b * p.Hq + hq) * p.S + qcol] = (m_run + log2f(l_tot)) * kLn2;
}

// ----------------------------------------------------------------------------------
// Backward
// ----------------------------------------------------------------------------------

template <typename E>
struct BwdParams {
  const E* q;
  const E* k;
  const E* v;
  const E* dout;
  const float* lse;    // [B, Hq, S], natural log of sum exp(scale * s)
  const float* delta;  // [2, B, Hq, S]: -delta, then -lse / scale (written by the dQ pass, read by dK/dV)
  const E* o;          // forward output [B, S, Hq, D] contiguous (read by the dQ pass that computes delta)
  E* dq;            // [B, S, Hq, D]
  float* dk_part;      // [group, B, S, Hkv, D] fp32 partials (one per q head of the GQA group)
  float* dv_part;
  E* dk;            // [B, S, Hkv, D] (written directly when group == 1)
  E* dv;
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t do_sb, do_ss, do_sh;
  int64_t dq_ss, dkv_ss;  // token (row) strides of the dq and dk/dv outputs: Hq*D / Hkv*D, or the fused
                          // [T, (Hq + 2 Hkv) D] dQKV row when the caller hands over one buffer
  E* ds;                  // dS in MFMA-fragment order, one 2 KiB block per (b, q head, 32 queries, 32 keys)
  int64_t ds_nblk;        // blocks per (b, q head): the causal triangle or the full square of 32-blocks
  int B, S, Hq, Hkv;
  float scale;          // softmax scale
  float scale_log2;     // scale * log2(e)
  float neg_inv_scale;  // -1 / scale (kernel argument: a scalar register, not a VGPR)
  bool causal;
};



// Stage ROWS x D bf16 rows (row r at base + r*row_stride, r clamped to < nrows_valid) into an
// LDS image swizzled by SWZ, using LDS-DMA pieces issued by `wave` of `nwaves`. The image is
// lane-linear per piece; the swizzle is applied to the global SOURCE address (involution).
template <typename E, int D, int ROWS, int SWZ, int NW = 4>  // SWZ: 0 = row image, 1 = dual image; NW waves share it
__device__ __forceinline__ void stage_rows(E* img, const E* base, int64_t row_stride, int row0, int nvalid,
                                           int wave, int lane) {
  constexpr int CH = D / 8;
  constexpr int PR = 64 / CH;               // rows per 1 KiB piece
  constexpr int NP = ROWS / PR;             // pieces
  const int rin = lane / CH, phys = lane % CH;
  for (int pc = wave; pc < NP; pc += NW) {
    const int row = pc * PR + rin;
    const int logical = SWZ ? swz_dual<D>(row, phys) : swz_row<D>(row, phys);
    int grow = row0 + row;
    grow = grow < nvalid ? grow : nvalid - 1;
    glds16(base + (int64_t)grow * row_stride + logical * 8, img + pc * 512);
  }
}

// ---- stored dS (the single-recompute backward, DLGM_ATTN_BWD=ds): dK/dV computes dS = P (dP - delta) once per (query, key)
// and writes it out in the exact register order in which the dQ pass consumes it as the B operand of
// dQ^T += K^T dS^T: block (query block qb, key block kb) of 32 x 32 is 2 x 1 KiB, k-step s2 at +512 elements,
// lane l's 8 keys at +8 l -- each wave stores and loads it as one fully coalesced 16 B per lane access.
// The dQ pass then recomputes neither S = QK^T nor dP = dO V^T: 2.5 forward-equivalents of MFMA work instead of 3.5
// (VERDICT r05 item 2), for 2 B per causal (query, key) pair written once and read once. Measured at the Llama-3-8B
// shape it is 5 % SLOWER than the recompute backward (the default): the dS write costs dK/dV more than the recompute
// it saves the dQ pass (profiles/attn_bwd_stored_ds_ab_r06.json).
__device__ __forceinline__ int64_t ds_block(int qb, int kb, int nkb, bool causal) {
  return causal ? (int64_t)qb * (qb + 1) / 2 + kb : (int64_t)qb * nkb + kb;
}
constexpr int kTsRow = 36;             // LDS row of the per-wave dS transpose tile: 32 queries + 4 pad (72 B rows)
constexpr int kTsWave = 32 * kTsRow;   // one wave's [32 keys][36] tile

// ---- dK / dV: one workgroup per (b, q head, 128 keys); 4 waves x 32 keys on the MFMA lanes.
constexpr int kKvThreads = 256;
constexpr int kKvBKV = 128;
constexpr int kKvBQ = 32;

// HP: q heads per workgroup (2 when the GQA group is even): the heads of a pair share this block's K / V, so
// the workgroup walks both heads' query tiles into one dK/dV accumulator -- half the fp32 partials written
// and summed by gqa_reduce, half the K / V block loads.
template <typename E, int D, bool TAIL, int HP = 1, bool STORE_DS = false>
__global__ __launch_bounds__(kKvThreads, 2) void flash_bwd_dkdv_kernel(BwdParams<E> p) {
  constexpr int KK = D / 16;
  constexpr int DT = D / 32;
  constexpr int QT = kKvBQ * D;
  __shared__ __attribute__((aligned(16))) E smem[2 * 2 * QT + kKvBKV * D];  // [buf][Q | dO], then V rows
  __shared__ __attribute__((aligned(16))) float rc[2][64];        // [buf][-lse/scale 0..31 | -delta 32..63]
  // STORE_DS: each wave's dS tile goes through LDS once ([key][query] rows written from the accumulator layout,
  // read back transposed with ds_read_b64_tr_b16 into the dQ pass's B-operand order)
  __shared__ __attribute__((aligned(16))) E ts[STORE_DS ? 4 * kTsWave : 1];
  E* vimg = smem + 2 * 2 * QT;  // this block's 128 V rows (row image): B operand of dP, re-read per tile

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5, i16 = lane & 15, g = lane >> 4;
  const int nkt = (p.S + kKvBKV - 1) / kKvBKV;
  const int group = p.Hq / p.Hkv;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = work / nkt;                 // blocks of one (b, head pair) share the Q / dO stream -> one XCD
  const int kt = work - bh * nkt;            // ascending = most queries first under the causal mask
  const int b = bh / (p.Hq / HP), hq = (bh % (p.Hq / HP)) * HP;  // first head of the workgroup
  const int hk = hq / group, hh = hq % group;
  const int k0 = kt * kKvBKV;
  const int kw0 = k0 + 32 * w;
  const int key = kw0 + r;
  const E* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const E* vb = p.v + b * p.v_sb + hk * p.v_sh;
  const E* qb = p.q + b * p.q_sb + hq * p.q_sh;
  const E* dob = p.dout + b * p.do_sb + hq * p.do_sh;
  const float* dlb = p.delta + ((int64_t)b * p.Hq + hq) * p.S;        // -delta
  const float* lseb = dlb + (int64_t)p.B * p.Hq * p.S;                  // -lse / scale

  // K^T B-operand fragments of this wave's 32 keys stay in registers for the whole block; the V
  // rows go to LDS once (registers are the binding constraint at 2 waves / SIMD)
  vec8_t<E> kf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const bool ok = key < p.S;
    kf[kk] = ok ? *reinterpret_cast<const vec8_t<E>*>(kb + (int64_t)key * p.k_ss + 16 * kk + 8 * h) : (vec8_t<E>)((E)0.f);
  }
  stage_rows<E, D, kKvBKV, 0>(vimg, vb, p.v_ss, k0, p.S, w, lane);
  f32x16 dkt[DT], dvt[DT];  // dK^T, dV^T : [d][key]
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dkt[dt] = (f32x16)(0.f);
    dvt[dt] = (f32x16)(0.f);
  }
  const int nqt = (p.S + kKvBQ - 1) / kKvBQ;
  const int t0 = p.causal ? k0 / kKvBQ : 0;
  const int vrow = 32 * w + r;
  int qoff[KK], voff[KK];  // element offsets of this lane's Q / dO (dual image) and V (row image) fragments
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    qoff[kk] = r * D + swz_dual<D>(r, 2 * kk + h) * 8;
    voff[kk] = vrow * D + swz_row<D>(vrow, 2 * kk + h) * 8;
    pin(qoff[kk]);
    pin(voff[kk]);
  }

  TileDma<E, D, kKvBQ, 1, TAIL> qdma(qb, p.q_ss, p.S, w, lane), dodma(dob, p.do_ss, p.S, w, lane);
  if constexpr (HP > 1) {
    qdma.extend((int64_t)(HP - 1) * p.q_sh * 2);
    dodma.extend((int64_t)(HP - 1) * p.do_sh * 2);
  }
  // tile index j over (head of the pair, query tile): head j / nt_h, query tile t0 + j % nt_h
  const int nt_h = nqt - t0 > 0 ? nqt - t0 : 0;
  const int ntot = HP * nt_h;
  auto stage = [&](int buf, int j) {
    const int hp = HP > 1 ? j / nt_h : 0;
    const int q0 = (t0 + j - hp * nt_h) * kKvBQ;
    E* img = smem + buf * 2 * QT;
    qdma.issue(img, q0, (uint32_t)(hp * p.q_sh * 2));
    dodma.issue(img + QT, q0, (uint32_t)(hp * p.do_sh * 2));
    if (w == 0) {
      int q = q0 + (lane & 31);
      q = q < p.S ? q : p.S - 1;
      glds4((lane < 32 ? lseb : dlb) + (int64_t)hp * p.S + q, &rc[buf][0]);
    }
  };

  // STORE_DS: the previous tile's two dS stores are this wave's youngest vector-memory operations; CDNA4's vmcnt
  // counts stores too, so a full drain would wait for their write-back every tile -- wait for the DMA only
  bool stored = false;
  // unrolled by two: the LDS buffer is a compile-time constant in each copy (immediate ds_read offsets)
  auto tile = [&](auto bufc, int j) {
    constexpr int buf = decltype(bufc)::value;
    if (STORE_DS && stored) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else vm_drain();  // this tile's LDS-DMA has landed ...
    stored = false;
    __syncthreads();  // ... for every wave, and the other buffer's readers are done
    if (j + 1 < ntot) stage(buf ^ 1, j + 1);
    const int t = t0 + (HP > 1 ? j % nt_h : j);
    const int q0 = t * kKvBQ;
    const int hp_cur = HP > 1 ? j / nt_h : 0;
    const bool active = uniform(!(p.causal && q0 + kKvBQ - 1 < kw0));
    if (active) {
      const E* qi = smem + buf * 2 * QT;
      const E* di = qi + QT;
      f32x16 sacc, dpacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = (i & 3) + 8 * (i >> 2) + 4 * h;
        sacc[i] = rc[buf][qr];        // S' = S - lse/scale  ->  p = exp2(S' * scale * log2e)
        dpacc[i] = rc[buf][32 + qr];  // dP - delta
      }
      // S^T and dP^T as two interleaved accumulation chains: each MFMA's operand reads are covered by the
      // other chain's MFMA instead of stalling a single chain on LDS latency
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        vec8_t<E> a = lds_read_b128(qi + qoff[kk]);
        vec8_t<E> d = lds_read_b128(di + qoff[kk]);
        vec8_t<E> vv = lds_read_b128(vimg + voff[kk]);
        sacc = mfma32(a, kf[kk], sacc);
        dpacc = mfma32(d, vv, dpacc);
      }
      // dS = P (dP - delta); the softmax scale is applied once to dK at the end. Masked scores go to
      // -inf BEFORE the exponentials (exp2 -> 0), in a block of its own: a mask test inside the
      // exponential loop became one scalar branch per element, which kept the exps out of the MFMA
      // schedule (the forward's structure)
      const bool need_mask = uniform((p.causal && q0 < kw0 + 31) || q0 + kKvBQ > p.S || kw0 + 32 > p.S);
      if (need_mask) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int q = q0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (key >= p.S || q >= p.S || (p.causal && key > q)) sacc[i] = -INFINITY;
        }
      }
      const f32x2 sl2 = {p.scale_log2, p.scale_log2};
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 x = (f32x2){sacc[i], sacc[i + 1]} * sl2;
        const f32x2 pv = {fast_exp2(x.x), fast_exp2(x.y)};
        const f32x2 ds = (f32x2){dpacc[i], dpacc[i + 1]} * pv;
        sacc[i] = pv.x;
        sacc[i + 1] = pv.y;
        dpacc[i] = ds.x;
        dpacc[i + 1] = ds.y;
      }
      vec8_t<E> pfr[2], dsf[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        pfr[s2] = (vec8_t<E>){(E)sacc[8 * s2 + 0], (E)sacc[8 * s2 + 1], (E)sacc[8 * s2 + 2],
                           (E)sacc[8 * s2 + 3], (E)sacc[8 * s2 + 4], (E)sacc[8 * s2 + 5],
                           (E)sacc[8 * s2 + 6], (E)sacc[8 * s2 + 7]};
        dsf[s2] = (vec8_t<E>){(E)dpacc[8 * s2 + 0], (E)dpacc[8 * s2 + 1], (E)dpacc[8 * s2 + 2],
                           (E)dpacc[8 * s2 + 3], (E)dpacc[8 * s2 + 4], (E)dpacc[8 * s2 + 5],
                           (E)dpacc[8 * s2 + 6], (E)dpacc[8 * s2 + 7]};
      }
      // STORE_DS (DLGM_ATTN_BWD=ds): lane (key r, half h) holds dS for queries 8m + 4h + 0..3 in registers 4m..4m+3 --
      // four 8-byte row pieces of the wave's [key][query] LDS tile; the transposed reads give lane (query l&31, half
      // l>>5) its 8 keys {16 s2 + 8 (j >> 2) + 4 h + (j & 3)} -- the key order of the dQ pass's K^T reads -- stored as
      // 16 B per lane. (Measured placing the read-back after the dV / dK MFMAs instead: 7 % slower.)
      if (STORE_DS && uniform(kw0 < p.S)) {  // a wave whose keys all lie past S owns no dS block
        E* tw = ts + w * kTsWave;
#pragma unroll
        for (int m = 0; m < 4; ++m)
          *reinterpret_cast<vec4_t<E>*>(tw + r * kTsRow + 8 * m + 4 * h) =
              (vec4_t<E>){(E)dpacc[4 * m], (E)dpacc[4 * m + 1], (E)dpacc[4 * m + 2], (E)dpacc[4 * m + 3]};
        __builtin_amdgcn_wave_barrier();
        const int colq = 16 * (g & 1) + 4 * (i16 & 3);
        E* dst = p.ds + ((int64_t)(b * p.Hq + hq + hp_cur) * p.ds_nblk +
                         ds_block(t, kw0 / 32, (p.S + 31) / 32, p.causal)) * 1024 + lane * 8;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r1 = 16 * s2 + 4 * h + (i16 >> 2);
          *reinterpret_cast<vec8_t<E>*>(dst + 512 * s2) =
              cat(lds_read_tr(tw + r1 * kTsRow + colq), lds_read_tr(tw + (r1 + 8) * kTsRow + colq));
        }
        stored = true;
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int col = dt * 32 + 16 * (g & 1) + 4 * (i16 & 3);
        const int ch = col >> 3, within = col & 7;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r1 = 16 * s2 + 4 * h + (i16 >> 2);
          const int r2 = r1 + 8;
          vec8_t<E> a_do = cat(lds_read_tr(di + r1 * D + swz_dual<D>(r1, ch) * 8 + within),
                            lds_read_tr(di + r2 * D + swz_dual<D>(r2, ch) * 8 + within));
          dvt[dt] = mfma32(a_do, pfr[s2], dvt[dt]);
          vec8_t<E> a_q = cat(lds_read_tr(qi + r1 * D + swz_dual<D>(r1, ch) * 8 + within),
                           lds_read_tr(qi + r2 * D + swz_dual<D>(r2, ch) * 8 + within));
          dkt[dt] = mfma32(a_q, dsf[s2], dkt[dt]);
        }
      }
    }
  };
  if (ntot > 0) stage(0, 0);
  for (int j = 0; j < ntot; j += 2) {
    tile(std::integral_constant<int, 0>{}, j);
    if (j + 1 < ntot) tile(std::integral_constant<int, 1>{}, j + 1);
  }
  if (group == HP) {  // one partial per kv head: written directly (the lane-pair swaps of the widened store
                      // need every lane, in or out of range)
    store_rows_bf16<DT>(p.dk + ((int64_t)b * p.S + key) * p.dkv_ss + hk * D, dkt, p.scale, h, key < p.S);
    store_rows_bf16<DT>(p.dv + ((int64_t)b * p.S + key) * p.dkv_ss + hk * D, dvt, 1.f, h, key < p.S);
    return;
  }
  if (key >= p.S) return;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dkt[dt] *= p.scale;
  {
    const int64_t off = ((((int64_t)(hh / HP) * p.B + b) * p.S + key) * p.Hkv + hk) * D;
    float* dkr = p.dk_part + off;
    float* dvr = p.dv_part + off;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * h;
        *reinterpret_cast<f32x4*>(dkr + d) = (f32x4){dkt[dt][4 * g4 + 0], dkt[dt][4 * g4 + 1], dkt[dt][4 * g4 + 2],
                                                     dkt[dt][4 * g4 + 3]};
        *reinterpret_cast<f32x4*>(dvr + d) = (f32x4){dvt[dt][4 * g4 + 0], dvt[dt][4 * g4 + 1], dvt[dt][4 * g4 + 2],
                                                     dvt[dt][4 * g4 + 3]};
      }
  }
}

// Sum the per-q-head fp32 partials of the GQA group (fixed order: deterministic) -> bf16.
template <typename E>
__global__ __launch_bounds__(256) void gqa_reduce_kernel(const float* __restrict__ part, E* __restrict__ out,
                                                         int group, int64_t n, int row_len, int64_t out_stride) {
  const int64_t nv = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = (i * 8) / row_len, col = (i * 8) - row * row_len;
    f32x8 s = (f32x8)(0.f);
    for (int gq = 0; gq < group; ++gq) {
      const float* src = part + gq * n + i * 8;
      f32x4 a = *reinterpret_cast<const f32x4*>(src);
      f32x4 c = *reinterpret_cast<const f32x4*>(src + 4);
      s += (f32x8){a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]};
    }
    store8f(out + row * out_stride + col, s);
  }
}

// ---- dQ: one workgroup per (b, q head, 128 queries) -- the forward's structure (query on the
// lane, S^T = K Q^T, dP^T = V dO^T); dQ^T += K^T dS^T takes the dS^T accumulator in place as the
// B operand, so dQ needs no atomics and no LDS round trip.
constexpr int kDqThreads = 256;
constexpr int kDqBQ = 128;
constexpr int kDqBKV = 64;

// The pass also computes delta = rowsum(dO * O) for its query rows (it holds dO in registers already) and
// writes the [-delta, -lse/scale] rows the dK/dV pass reads -- no separate delta launch; dQ runs first.
template <typename E, int D, bool TAIL>
__global__ __launch_bounds__(kDqThreads, 2) void flash_bwd_dq_kernel(BwdParams<E> p) {
  constexpr int KK = D / 16;
  constexpr int DT = D / 32;
  constexpr int TILE = kDqBKV * D;
  constexpr int SLOT = 2 * TILE;
  __shared__ __attribute__((aligned(16))) E smem[2 * SLOT];  // [buf][K | V]

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5, i16 = lane & 15, g = lane >> 4;
  const int nqt = (p.S + kDqBQ - 1) / kDqBQ;
  const int group = p.Hq / p.Hkv;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int per_kv = group * nqt;
  const int bk = work / per_kv;
  const int rem = work - bk * per_kv;
  const int qt = nqt - 1 - rem / group;
  const int hq = (bk % p.Hkv) * group + rem % group;
  const int b = bk / p.Hkv;
  const int hk = hq / group;
  const int q0 = qt * kDqBQ;
  const int q0w = q0 + 32 * w;
  const int qcol = q0w + r;
  const E* qb = p.q + b * p.q_sb + hq * p.q_sh;
  const E* dob = p.dout + b * p.do_sb + hq * p.do_sh;
  const E* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const E* vb = p.v + b * p.v_sb + hk * p.v_sh;

  vec8_t<E> qf[KK], dof[KK];
  float lse2 = 0.f, nd = 0.f;
  {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const bool ok = qcol < p.S;
      qf[kk] = ok ? *reinterpret_cast<const vec8_t<E>*>(qb + (int64_t)qcol * p.q_ss + 16 * kk + 8 * h) : (vec8_t<E>)((E)0.f);
      dof[kk] = ok ? *reinterpret_cast<const vec8_t<E>*>(dob + (int64_t)qcol * p.do_ss + 16 * kk + 8 * h) : (vec8_t<E>)((E)0.f);
    }
    const int64_t rowc = ((int64_t)b * p.Hq + hq) * p.S;
    lse2 = qcol < p.S ? p.lse[rowc + qcol] * kLog2e : INFINITY;
    {
      // this lane holds dO[qcol][16kk + 8h .. +7]: the matching O chunks, a 64-term dot, the other half-wave's 64
      float acc = 0.f;
      if (qcol < p.S) {
        const E* orow = p.o + (((int64_t)b * p.S + qcol) * p.Hq + hq) * D + 8 * h;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          const vec8_t<E> ov = *reinterpret_cast<const vec8_t<E>*>(orow + 16 * kk);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += (float)dof[kk][j] * (float)ov[j];
        }
      }
      nd = -(acc + swap_halves(acc));
      if (qcol < p.S && h == 0) {
        float* dl = const_cast<float*>(p.delta);
        dl[rowc + qcol] = nd;
        dl[(int64_t)p.B * p.Hq * p.S + rowc + qcol] = p.lse[rowc + qcol] * p.neg_inv_scale;
      }
    }
  }

  f32x16 dqt[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dqt[dt] = (f32x16)(0.f);

  const int kv_end = p.causal ? min(p.S, q0 + kDqBQ) : p.S;
  const int nt = (kv_end + kDqBKV - 1) / kDqBKV;
  // element offsets of this lane's K (dual image) and V (row image) fragments; row 32 + r has the same
  // swizzle as row r, so the second 32-key subtile is an immediate offset away
  int koff[KK], voff[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    koff[kk] = r * D + swz_dual<D>(r, 2 * kk + h) * 8;
    voff[kk] = r * D + swz_row<D>(r, 2 * kk + h) * 8;
    pin(koff[kk]);
    pin(voff[kk]);
  }
  const TileDma<E, D, kDqBKV, 1, TAIL> kdma(kb, p.k_ss, p.S, w, lane);
  const TileDma<E, D, kDqBKV, 0, TAIL> vdma(vb, p.v_ss, p.S, w, lane);
  auto stage = [&](int buf, int t) {
    E* img = smem + buf * SLOT;
    kdma.issue(img, t * kDqBKV);
    vdma.issue(img + TILE, t * kDqBKV);
  };
  // unrolled by two: the LDS buffer is a compile-time constant in each copy (immediate ds_read offsets)
  auto tile = [&](auto bufc, int t) {
    constexpr int buf = decltype(bufc)::value;
    vm_drain();
    __syncthreads();
    if (t + 1 < nt) stage(buf ^ 1, t + 1);
    const int kv0 = t * kDqBKV;
    if (!(p.causal && kv0 > q0w + 31)) {
      const E* kt = smem + buf * SLOT;
      const E* vt = kt + TILE;
      vec8_t<E> dsf[2][2];
      f32x16 s[2] = {(f32x16)(0.f), (f32x16)(0.f)};
      f32x16 dp[2] = {(f32x16)(0.f), (f32x16)(0.f)};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          vec8_t<E> a = lds_read_b128(kt + 32 * u * D + koff[kk]);
          s[u] = mfma32(a, qf[kk], s[u]);
          vec8_t<E> c = lds_read_b128(vt + 32 * u * D + voff[kk]);
          dp[u] = mfma32(c, dof[kk], dp[u]);
        }
      }
      // masked scores -> -inf before the exponentials, in a block of their own (see dK/dV)
      const bool need_mask = uniform((p.causal && kv0 + kDqBKV - 1 > q0w) || kv0 + kDqBKV > p.S);
      if (need_mask) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kv = kv0 + 32 * u + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (kv >= p.S || (p.causal && kv > qcol)) s[u][i] = -INFINITY;
          }
      }
      const f32x2 sl2 = {p.scale_log2, p.scale_log2}, nl2 = {-lse2, -lse2}, nd2 = {nd, nd};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 x = pk_fma((f32x2){s[u][i], s[u][i + 1]}, sl2, nl2);
          const f32x2 pv = {fast_exp2(x.x), fast_exp2(x.y)};
          const f32x2 ds = ((f32x2){dp[u][i], dp[u][i + 1]} + nd2) * pv;  // dS = P (dP - delta)
          s[u][i] = ds.x;
          s[u][i + 1] = ds.y;
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          dsf[u][s2] = (vec8_t<E>){(E)s[u][8 * s2 + 0], (E)s[u][8 * s2 + 1], (E)s[u][8 * s2 + 2],
                                (E)s[u][8 * s2 + 3], (E)s[u][8 * s2 + 4], (E)s[u][8 * s2 + 5],
                                (E)s[u][8 * s2 + 6], (E)s[u][8 * s2 + 7]};
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int col = dt * 32 + 16 * (g & 1) + 4 * (i16 & 3);
        const int ch = col >> 3, within = col & 7;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int r1 = 32 * u + 16 * s2 + 4 * h + (i16 >> 2);
            const int r2 = r1 + 8;
            vec8_t<E> a = cat(lds_read_tr(kt + r1 * D + swz_dual<D>(r1, ch) * 8 + within),
                           lds_read_tr(kt + r2 * D + swz_dual<D>(r2, ch) * 8 + within));
            dqt[dt] = mfma32(a, dsf[u][s2], dqt[dt]);
          }
      }
    }
  };
  stage(0, 0);
  for (int t = 0; t < nt; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < nt) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  store_rows_bf16<DT>(p.dq + ((int64_t)b * p.S + qcol) * p.dq_ss + hq * D, dqt, p.scale, h, qcol < p.S);
}

// ---- dQ from the stored dS (DLGM_ATTN_BWD=ds): one workgroup per (b, q head, 128 queries), the dQ pass's structure
// with the recompute gone -- per 64-key tile a wave loads its 2 x 2 dS fragments (16 B per lane, coalesced; issued
// one tile ahead, beside the K tile's LDS-DMA) and runs the 16 MFMAs of dQ^T += K^T dS^T. Bound by the dS read.
template <typename E, int D, bool TAIL>
__global__ __launch_bounds__(kDqThreads, 2) void flash_bwd_dq_ds_kernel(BwdParams<E> p) {
  constexpr int DT = D / 32;
  constexpr int TILE = kDqBKV * D;
  __shared__ __attribute__((aligned(16))) E smem[2 * TILE];  // [buf] K tile (dual image)

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, i16 = lane & 15, g = lane >> 4;
  const int nqt = (p.S + kDqBQ - 1) / kDqBQ;
  const int group = p.Hq / p.Hkv;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int per_kv = group * nqt;
  const int bk = work / per_kv;
  const int rem = work - bk * per_kv;
  const int qt = nqt - 1 - rem / group;
  const int hq = (bk % p.Hkv) * group + rem % group;
  const int b = bk / p.Hkv;
  const int hk = hq / group;
  const int q0 = qt * kDqBQ;
  const int q0w = q0 + 32 * w;
  const int qcol = q0w + (lane & 31);
  const int nkb = (p.S + 31) / 32;
  const int qb = q0w / 32;
  const E* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const E* dsb = p.ds + (int64_t)(b * p.Hq + hq) * p.ds_nblk * 1024 + lane * 8;

  f32x16 dqt[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dqt[dt] = (f32x16)(0.f);
  const int kv_end = p.causal ? min(p.S, q0 + kDqBQ) : p.S;
  const int nt = (kv_end + kDqBKV - 1) / kDqBKV;
  const TileDma<E, D, kDqBKV, 1, TAIL> kdma(kb, p.k_ss, p.S, w, lane);
  // a dS block of this wave exists when its queries and the block's keys lie inside the sequence and the block is on
  // or below the diagonal (a wave whose 32 queries all lie past S -- the tail of the last 128-query tile -- has none)
  auto have = [&](int kbk) { return uniform(qb < nkb && kbk < nkb && !(p.causal && kbk > qb)); };
  auto load = [&](vec8_t<E> (&f)[2][2], int t) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kbk = 2 * t + u;
      if (have(kbk)) {
        const E* src = dsb + ds_block(qb, kbk, nkb, p.causal) * 1024;
        f[u][0] = __builtin_nontemporal_load(reinterpret_cast<const vec8_t<E>*>(src));
        f[u][1] = __builtin_nontemporal_load(reinterpret_cast<const vec8_t<E>*>(src + 512));
      }
    }
  };
  auto tile = [&](auto bufc, int t, vec8_t<E> (&cur)[2][2], vec8_t<E> (&nxt)[2][2]) {
    constexpr int buf = decltype(bufc)::value;
    vm_drain();  // this tile's K (LDS-DMA) and dS fragments (registers) have landed ...
    __syncthreads();  // ... for every wave, and the other buffer's readers are done
    if (t + 1 < nt) {
      kdma.issue(smem + (buf ^ 1) * TILE, (t + 1) * kDqBKV);
      load(nxt, t + 1);
    }
    const E* kt = smem + buf * TILE;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!have(2 * t + u)) continue;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int col = dt * 32 + 16 * (g & 1) + 4 * (i16 & 3);
        const int ch = col >> 3, within = col & 7;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int r1 = 32 * u + 16 * s2 + 4 * h + (i16 >> 2);
          const int r2 = r1 + 8;
          vec8_t<E> a = cat(lds_read_tr(kt + r1 * D + swz_dual<D>(r1, ch) * 8 + within),
                            lds_read_tr(kt + r2 * D + swz_dual<D>(r2, ch) * 8 + within));
          dqt[dt] = mfma32(a, cur[u][s2], dqt[dt]);
        }
      }
    }
  };
  vec8_t<E> fa[2][2], fb[2][2];
  kdma.issue(smem, 0);
  load(fa, 0);
  for (int t = 0; t < nt; t += 2) {
    tile(std::integral_constant<int, 0>{}, t, fa, fb);
    if (t + 1 < nt) tile(std::integral_constant<int, 1>{}, t + 1, fb, fa);
  }
  store_rows_bf16<DT>(p.dq + ((int64_t)b * p.S + qcol) * p.dq_ss + hq * D, dqt, p.scale, h, qcol < p.S);
}

// delta = rowsum(dO * O) per (b, s, q head), written as the [-delta, -lse / scale] rows the dK/dV pass starts its
// accumulators from (the recompute backward folds this into its dQ pass, which runs first; here dK/dV runs first).
// D / 8 lanes per row, 16 B per lane of each operand, a shuffle reduction inside the row's lane group.
template <typename E, int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(BwdParams<E> p) {
  constexpr int L = D / 8;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / L;  // (b, s, hq) in [B, S, Hq] order
  const int c = (int)(gid % L);
  const int64_t R = (int64_t)p.B * p.S * p.Hq;
  float acc = 0.f;
  int b = 0, sq = 0, hq = 0;
  if (row < R) {
    hq = (int)(row % p.Hq);
    const int64_t bs = row / p.Hq;
    sq = (int)(bs % p.S);
    b = (int)(bs / p.S);
    const f32x8 d = load8f(p.dout + b * p.do_sb + (int64_t)sq * p.do_ss + hq * p.do_sh + 8 * c);
    const f32x8 o = load8f(p.o + row * D + 8 * c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += d[j] * o[j];
  }
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < R && c == 0) {
    const int64_t rc = ((int64_t)b * p.Hq + hq) * p.S + sq;
    float* dl = const_cast<float*>(p.delta);
    dl[rc] = -acc;
    dl[R + rc] = p.lse[rc] * p.neg_inv_scale;
  }
}

void check_qkv(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && DLGM_IS16(t), name, " must be a bf16/fp16 GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, name, " must be [B, S, H, D] with unit stride on D");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              name, " strides must keep 16-byte alignment");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

bool attn_bwd_store_ds() {  // read per call (a getenv): A/B runs switch it inside one process
  const char* e = std::getenv("DLGM_ATTN_BWD");
  return e != nullptr && std::strcmp(e, "ds") == 0;
}

}  // namespace

// q [B,S,Hq,D], k/v [B,S,Hkv,D] (strided views allowed) -> out [B,S,Hq,D] contiguous, lse [B,Hq,S] fp32
std::tuple<at::Tensor, at::Tensor> dlgm_flash_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                       double softmax_scale, bool causal) {
  check_qkv(q, "q");
  check_qkv(k, "k");
  check_qkv(v, "v");
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && k.size(1) == S && k.size(3) == D && v.sizes() == k.sizes(),
              "flash_attn: k/v shape mismatch");
  TORCH_CHECK(Hq % Hkv == 0, "flash_attn: Hq must be a multiple of Hkv");
  TORCH_CHECK(D == 128 || D == 64, "flash_attn: head dim must be 64 or 128");
  auto out = at::empty({B, S, Hq, D}, q.options());
  auto lse = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  if (B == 0 || S == 0) return {out, lse};
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type(), "flash_attn: mixed dtypes");
  const int nqt = (S + kFwdBQ - 1) / kFwdBQ;
  const int64_t blocks = (int64_t)nqt * B * Hq;
  auto stream = c10::hip::getCurrentHIPStream();
  DLGM_DISPATCH_16(q.scalar_type(), E, {
    FwdParams<E> p{reinterpret_cast<const E*>(q.data_ptr()), reinterpret_cast<const E*>(k.data_ptr()),
                   reinterpret_cast<const E*>(v.data_ptr()), reinterpret_cast<E*>(out.data_ptr()),
                   lse.data_ptr<float>(), q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                   v.stride(0), v.stride(1), v.stride(2), B, S, Hq, Hkv, (float)(softmax_scale * kLog2e), causal};
    const bool tail = S % 128 != 0;  // a partial K/V tile exists: the clamped-staging instantiation
    if (D == 128) {
      if (tail) flash_fwd_kernel<E, 128, true><<<blocks, kFwdThreads, 0, stream>>>(p);
      else flash_fwd_kernel<E, 128, false><<<blocks, kFwdThreads, 0, stream>>>(p);
    } else {
      if (tail) flash_fwd_kernel<E, 64, true><<<blocks, kFwdThreads, 0, stream>>>(p);
      else flash_fwd_kernel<E, 64, false><<<blocks, kFwdThreads, 0, stream>>>(p);
    }
  });
  DLGM_CHECK_HIP(hipGetLastError());
  return {out, lse};
}

// Returns (dq, dk, dv) with the shapes of q, k, v (contiguous).
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_flash_attn_bwd(const at::Tensor& dout, const at::Tensor& q,
                                                                   const at::Tensor& k, const at::Tensor& v,
                                                                   const at::Tensor& out, const at::Tensor& lse,
                                                                   double softmax_scale, bool causal,
                                                                   const c10::optional<at::Tensor>& dqkv) {
  check_qkv(q, "q");
  check_qkv(k, "k");
  check_qkv(v, "v");
  check_qkv(dout, "dout");
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = k.size(2);
  const int group = Hq / Hkv;
  TORCH_CHECK(D == 128 || D == 64, "flash_attn_bwd: head dim must be 64 or 128");
  TORCH_CHECK(out.is_contiguous() && out.sizes() == q.sizes(), "flash_attn_bwd: out must be contiguous [B,S,Hq,D]");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)B * Hq * S, "flash_attn_bwd: bad lse");
  TORCH_CHECK(dout.sizes() == q.sizes(), "flash_attn_bwd: dout shape mismatch");
  at::Tensor dq, dk, dv;
  int64_t dq_ss = (int64_t)Hq * D, dkv_ss = (int64_t)Hkv * D;
  if (dqkv.has_value()) {
    // one fused [B*S, (Hq + 2 Hkv) D] gradient: the layout of the QKV projection output, so the
    // caller's inverse RoPE and dW/dX GEMMs read it without a concatenation pass
    const int64_t C = (int64_t)(Hq + 2 * Hkv) * D;
    const at::Tensor& f = *dqkv;
    TORCH_CHECK(f.is_cuda() && f.scalar_type() == q.scalar_type() && f.is_contiguous() &&
                    f.numel() == (int64_t)B * S * C,
                "flash_attn_bwd: dqkv must be a contiguous [B*S, (Hq+2Hkv)*D] tensor of q's dtype");
    auto f3 = f.view({B, S, C});
    dq = f3.narrow(2, 0, (int64_t)Hq * D).unflatten(2, {Hq, D});
    dk = f3.narrow(2, (int64_t)Hq * D, (int64_t)Hkv * D).unflatten(2, {Hkv, D});
    dv = f3.narrow(2, (int64_t)(Hq + Hkv) * D, (int64_t)Hkv * D).unflatten(2, {Hkv, D});
    dq_ss = dkv_ss = C;
  } else {
    dk = at::empty({B, S, Hkv, D}, q.options());
    dv = at::empty({B, S, Hkv, D}, q.options());
    dq = at::empty({B, S, Hq, D}, q.options());
  }
  if (B == 0 || S == 0) return {dq.zero_(), dk.zero_(), dv.zero_()};
  auto delta = at::empty({2, B, Hq, S}, q.options().dtype(at::kFloat));  // -delta, -lse/scale
  const bool tail = S % 128 != 0;
  // two q heads per dK/dV workgroup when the GQA group is even
  const int hp = group % 2 == 0 ? 2 : 1;
  const int nparts = group / hp;  // fp32 dK/dV partials summed by gqa_reduce
  at::Tensor dk_part, dv_part;
  if (nparts > 1) {
    dk_part = at::empty({nparts, B, S, Hkv, D}, q.options().dtype(at::kFloat));
    dv_part = at::empty({nparts, B, S, Hkv, D}, q.options().dtype(at::kFloat));
  }
  // default: the two-recompute backward (dQ pass first, computing delta itself). DLGM_ATTN_BWD=ds: dK/dV stores dS once
  // and dQ reads it -- 29 % fewer MFMAs, but measured slower on MI355X (profiles/attn_bwd_stored_ds_ab_r06.json: dQ
  // 718 -> 508 us, dK/dV 1013 -> 1288 us for the 2.15 GB dS write at the board's power limit, + a 32 us delta launch)
  const bool store_ds = attn_bwd_store_ds();
  const int64_t nkb = (S + 31) / 32;
  const int64_t ds_nblk = causal ? nkb * (nkb + 1) / 2 : nkb * nkb;
  at::Tensor ds;
  if (store_ds) ds = at::empty({(int64_t)B * Hq * ds_nblk * 1024}, q.options());
  auto stream = c10::hip::getCurrentHIPStream();
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type() &&
                  dout.scalar_type() == q.scalar_type() && out.scalar_type() == q.scalar_type(),
              "flash_attn_bwd: mixed dtypes");
  const int64_t kv_blocks = (int64_t)B * (Hq / hp) * ((S + kKvBKV - 1) / kKvBKV);
  const int64_t dq_blocks = (int64_t)B * Hq * ((S + kDqBQ - 1) / kDqBQ);
  DLGM_DISPATCH_16(q.scalar_type(), E, {
    auto dop = reinterpret_cast<const E*>(dout.data_ptr());
    auto outp = reinterpret_cast<const E*>(out.data_ptr());
    BwdParams<E> p{reinterpret_cast<const E*>(q.data_ptr()), reinterpret_cast<const E*>(k.data_ptr()),
                   reinterpret_cast<const E*>(v.data_ptr()), dop, lse.data_ptr<float>(), delta.data_ptr<float>(),
                   outp, reinterpret_cast<E*>(dq.data_ptr()), nparts > 1 ? dk_part.data_ptr<float>() : nullptr,
                   nparts > 1 ? dv_part.data_ptr<float>() : nullptr, reinterpret_cast<E*>(dk.data_ptr()),
                   reinterpret_cast<E*>(dv.data_ptr()), q.stride(0), q.stride(1), q.stride(2), k.stride(0),
                   k.stride(1), k.stride(2), v.stride(0), v.stride(1), v.stride(2), dout.stride(0), dout.stride(1),
                   dout.stride(2), dq_ss, dkv_ss, store_ds ? reinterpret_cast<E*>(ds.data_ptr()) : nullptr,
                   ds_nblk, B, S, Hq, Hkv, (float)softmax_scale, (float)(softmax_scale * kLog2e),
                   (float)(-1.0 / softmax_scale), causal};
    // one backward per head dim / tail instantiation
    auto run = [&](auto dc, auto tc) {
      constexpr int DD = decltype(dc)::value;
      constexpr bool TT = decltype(tc)::value;
      if (store_ds) {
        const int64_t rows = (int64_t)B * S * Hq * (DD / 8);
        attn_delta_kernel<E, DD><<<(rows + 255) / 256, 256, 0, stream>>>(p);
        if (hp == 2) flash_bwd_dkdv_kernel<E, DD, TT, 2, true><<<kv_blocks, kKvThreads, 0, stream>>>(p);
        else flash_bwd_dkdv_kernel<E, DD, TT, 1, true><<<kv_blocks, kKvThreads, 0, stream>>>(p);
        flash_bwd_dq_ds_kernel<E, DD, TT><<<dq_blocks, kDqThreads, 0, stream>>>(p);
      } else {
        flash_bwd_dq_kernel<E, DD, TT><<<dq_blocks, kDqThreads, 0, stream>>>(p);
        if (hp == 2) flash_bwd_dkdv_kernel<E, DD, TT, 2><<<kv_blocks, kKvThreads, 0, stream>>>(p);
        else flash_bwd_dkdv_kernel<E, DD, TT><<<kv_blocks, kKvThreads, 0, stream>>>(p);
      }
    };
    if (D == 128) {
      if (tail) run(std::integral_constant<int, 128>{}, std::true_type{});
      else run(std::integral_constant<int, 128>{}, std::false_type{});
    } else {
      if (tail) run(std::integral_constant<int, 64>{}, std::true_type{});
      else run(std::integral_constant<int, 64>{}, std::false_type{});
    }
    DLGM_CHECK_HIP(hipGetLastError());
    if (nparts > 1) {
      const int64_t n = (int64_t)B * S * Hkv * D;
      const int64_t grid = std::min<int64_t>((n / 8 + 255) / 256, 4096);
      gqa_reduce_kernel<E><<<grid, 256, 0, stream>>>(dk_part.data_ptr<float>(), reinterpret_cast<E*>(dk.data_ptr()),
                                                     nparts, n, Hkv * D, dkv_ss);
      gqa_reduce_kernel<E><<<grid, 256, 0, stream>>>(dv_part.data_ptr<float>(), reinterpret_cast<E*>(dv.data_ptr()),
                                                     nparts, n, Hkv * D, dkv_ss);
      DLGM_CHECK_HIP(hipGetLastError());
    }
  });
  return {dq, dk, dv};
}
