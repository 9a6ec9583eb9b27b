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
//  * K/V tiles are register-staged with the async-STAGE split: global loads for
//    tile t+1 are issued before the MFMAs of tile t and written to the other LDS
//    buffer after the next barrier (one barrier per KV tile).
//  * Work ordering: causal blocks are launched heaviest-first, and blocks that
//    share one (batch, kv-head) -- i.e. the same K/V stream -- are grouped on one
//    XCD (blockIdx % 8 labels an XCD) so the K/V re-reads of the GQA group hit L2.
//  * Backward (FA2 structure, one workgroup per 128 keys of one (batch, kv head),
//    looping over the q heads of the GQA group and the query tiles): K and V of the
//    wave's 32 keys live in registers, dK^T/dV^T accumulate in registers (no
//    cross-workgroup sum), S and dP are computed with the key on the lane so they
//    feed dV^T / dK^T directly as accumulator-operands, -LSE and -delta are loaded
//    as the initial accumulators, and dQ is summed across key blocks with fp32
//    atomics shaped as 128-byte row segments.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
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

__device__ __forceinline__ bf16x8 lds_read_b128(const bf16* base) {
  return *reinterpret_cast<const bf16x8*>(base);
}

__device__ __forceinline__ bf16x4 lds_read_tr(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return (bf16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// bijective remap of the block id so that consecutive work items land on one XCD
__device__ __forceinline__ int xcd_remap(int id, int total) {
  if (total % 8 != 0) return id;
  return (id % 8) * (total / 8) + id / 8;
}

struct FwdParams {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  bf16* o;
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

template <int D>
__global__ __launch_bounds__(kFwdThreads, 2) void flash_fwd_kernel(FwdParams p) {
  constexpr int CH = D / 8;   // 16-byte chunks per row
  constexpr int KK = D / 16;  // MFMA k-steps over the head dim
  constexpr int DT = D / 32;  // 32-wide output tiles over the head dim
  constexpr int TILE = kFwdBKV * D;
  constexpr int LOADS = kFwdBKV * CH / kFwdThreads;  // 16B chunks per thread per tensor
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * TILE];

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
  const bf16* qb = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16* vb = p.v + b * p.v_sb + hk * p.v_sh;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q0w + r][16kk + 8h .. +7]
  bf16x8 qf[KK];
  {
    const int qrow = q0w + r;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      qf[kk] = qrow < p.S ? *reinterpret_cast<const bf16x8*>(qb + (int64_t)qrow * p.q_ss + 16 * kk + 8 * h)
                          : (bf16x8)((bf16)0.f);
  }

  const int kv_end = p.causal ? min(p.S, q0 + kFwdBQ) : p.S;
  const int nt = (kv_end + kFwdBKV - 1) / kFwdBKV;

  uint4 kreg[LOADS], vreg[LOADS];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int c = threadIdx.x + i * kFwdThreads;
      const int row = c / CH, ch = c % CH;
      const int kv = t * kFwdBKV + row;
      if (kv < p.S) {
        kreg[i] = *reinterpret_cast<const uint4*>(kb + (int64_t)kv * p.k_ss + ch * 8);
        vreg[i] = *reinterpret_cast<const uint4*>(vb + (int64_t)kv * p.v_ss + ch * 8);
      } else {
        kreg[i] = make_uint4(0, 0, 0, 0);
        vreg[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int c = threadIdx.x + i * kFwdThreads;
      const int row = c / CH, ch = c % CH;
      *reinterpret_cast<uint4*>(smem + buf * TILE + row * D + swz_row<D>(row, ch) * 8) = kreg[i];
      *reinterpret_cast<uint4*>(smem + (2 + buf) * TILE + row * D + swz_tr<D>(row, ch) * 8) = vreg[i];
    }
  };

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x16)(0.f);
  float m_run = -INFINITY, l_run = 0.f;
  const int qcol = q0w + r;

  gload(0);
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    lstore(buf);
    __syncthreads();
    if (t + 1 < nt) gload(t + 1);
    const int kv0 = t * kFwdBKV;
    if (p.causal && kv0 > q0w + 31) continue;  // whole tile above this wave's diagonal
    const bf16* kt = smem + buf * TILE;
    const bf16* vt = smem + (2 + buf) * TILE;

    // ---- S^T = K Q^T for two 32-key subtiles
    f32x16 s[2] = {(f32x16)(0.f), (f32x16)(0.f)};
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int row = 32 * u + r;
        bf16x8 a = lds_read_b128(kt + row * D + swz_row<D>(row, 2 * kk + h) * 8);
        s[u] = mfma32(a, qf[kk], s[u]);
      }
    }

    // ---- masking (only on diagonal / tail tiles)
    const bool need_mask = (p.causal && kv0 + kFwdBKV - 1 > q0w) || (kv0 + kFwdBKV > p.S);
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
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx * p.scale_log2);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    l_run *= alpha;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    bf16x8 pf[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = exp2f(s[u][i] * p.scale_log2 - m_use);
        s[u][i] = e;
        l_run += e;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        pf[u][s2] = (bf16x8){(bf16)s[u][8 * s2 + 0], (bf16)s[u][8 * s2 + 1], (bf16)s[u][8 * s2 + 2],
                             (bf16)s[u][8 * s2 + 3], (bf16)s[u][8 * s2 + 4], (bf16)s[u][8 * s2 + 5],
                             (bf16)s[u][8 * s2 + 6], (bf16)s[u][8 * s2 + 7]};
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
          bf16x4 a1 = lds_read_tr(vt + r1 * D + swz_tr<D>(r1, ch) * 8 + within);
          bf16x4 a2 = lds_read_tr(vt + r2 * D + swz_tr<D>(r2, ch) * 8 + within);
          o[dt] = mfma32(cat(a1, a2), pf[u][s2], o[dt]);
        }
    }
  }

  // ---- epilogue: normalise, store O [b, q, hq, d] and LSE [b, hq, q]
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qcol < p.S) {
    bf16* orow = p.o + (((int64_t)b * p.S + qcol) * p.Hq + hq) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * h;
        bf16x4 v = {(bf16)(o[dt][4 * g4 + 0] * inv), (bf16)(o[dt][4 * g4 + 1] * inv),
                    (bf16)(o[dt][4 * g4 + 2] * inv), (bf16)(o[dt][4 * g4 + 3] * inv)};
        *reinterpret_cast<bf16x4*>(orow + d) = v;
      }
    if (h == 0) p.lse[((int64_t)b * p.Hq + hq) * p.S + qcol] = (m_run + log2f(l_tot)) * kLn2;
  }
}

// ----------------------------------------------------------------------------------
// Backward
// ----------------------------------------------------------------------------------

// delta[b, hq, q] = sum_d dO[b,q,hq,d] * O[b,q,hq,d]   (one wave per row)
template <int D>
__global__ __launch_bounds__(256) void flash_bwd_delta_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ out,
                                                              float* __restrict__ delta, int B, int S, int Hq,
                                                              int64_t do_ss, int64_t do_sh, int64_t do_sb) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // row over (b, q, hq)
  if (row >= (int64_t)B * S * Hq) return;
  const int hq = row % Hq;
  const int64_t bq = row / Hq;
  const int q = bq % S, b = bq / S;
  float acc = 0.f;
  for (int d = lane * 8; d < D; d += 512) {
    f32x8 a = load8f(dout + b * do_sb + (int64_t)q * do_ss + hq * do_sh + d);
    f32x8 c = load8f(out + row * D + d);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * c[j];
  }
  acc = wave_sum(acc);
  if (lane == 0) delta[((int64_t)b * Hq + hq) * S + q] = acc;
}

struct BwdParams {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  const bf16* dout;
  const float* lse;    // [B, Hq, S], natural log of sum exp(scale * s)
  const float* delta;  // [B, Hq, S]
  float* dq;           // fp32 [B, S, Hq, D] accumulator
  bf16* dk;            // [B, S, Hkv, D]
  bf16* dv;            // [B, S, Hkv, D]
  int64_t q_sb, q_ss, q_sh;
  int64_t k_sb, k_ss, k_sh;
  int64_t v_sb, v_ss, v_sh;
  int64_t do_sb, do_ss, do_sh;
  int B, S, Hq, Hkv;
  float scale;       // softmax scale
  float scale_log2;  // scale * log2(e)
  bool causal;
};

constexpr int kBwdThreads = 256;  // 4 waves x 32 keys
constexpr int kBwdBKV = 128;
constexpr int kBwdBQ = 32;

template <int D>
__global__ __launch_bounds__(kBwdThreads, 1) void flash_bwd_kernel(BwdParams p) {
  constexpr int CH = D / 8;
  constexpr int KK = D / 16;
  constexpr int DT = D / 32;
  // LDS: K image [128][D] (dual swizzle, tr-read for dQ), Q and dO tiles [32][D] (dual),
  // dS^T image [128 keys][32 q] (64-B rows), lse/delta for the q tile.
  __shared__ __attribute__((aligned(16))) bf16 k_lds[kBwdBKV * D];
  __shared__ __attribute__((aligned(16))) bf16 q_lds[kBwdBQ * D];
  __shared__ __attribute__((aligned(16))) bf16 do_lds[kBwdBQ * D];
  __shared__ __attribute__((aligned(16))) bf16 ds_lds[kBwdBKV * kBwdBQ];
  __shared__ float lse_lds[kBwdBQ];
  __shared__ float dl_lds[kBwdBQ];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5, i16 = lane & 15, g = lane >> 4;
  const int nkt = (p.S + kBwdBKV - 1) / kBwdBKV;
  const int work = xcd_remap(blockIdx.x, gridDim.x);
  const int bk = work / nkt;
  const int kt = nkt - 1 - (work - bk * nkt);  // under the causal mask the first key blocks see the most queries
  const int b = bk / p.Hkv, hk = bk % p.Hkv;
  const int group = p.Hq / p.Hkv;
  const int k0 = kt * kBwdBKV;
  const int kw0 = k0 + 32 * w;  // this wave's 32 keys
  const bf16* kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16* vb = p.v + b * p.v_sb + hk * p.v_sh;

  // stage K block into LDS (dual image) and this wave's K / V rows into registers
  for (int c = threadIdx.x; c < kBwdBKV * CH; c += kBwdThreads) {
    const int row = c / CH, ch = c % CH;
    const int kv = k0 + row;
    uint4 val = kv < p.S ? *reinterpret_cast<const uint4*>(kb + (int64_t)kv * p.k_ss + ch * 8) : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(k_lds + row * D + swz_dual<D>(row, ch) * 8) = val;
  }
  bf16x8 kf[KK], vf[KK];  // B operands: K^T / V^T, lane holds row (kw0 + r), d = 16kk + 8h ..
  {
    const int kv = kw0 + r;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      kf[kk] = kv < p.S ? *reinterpret_cast<const bf16x8*>(kb + (int64_t)kv * p.k_ss + 16 * kk + 8 * h) : (bf16x8)((bf16)0.f);
      vf[kk] = kv < p.S ? *reinterpret_cast<const bf16x8*>(vb + (int64_t)kv * p.v_ss + 16 * kk + 8 * h) : (bf16x8)((bf16)0.f);
    }
  }
  f32x16 dkt[DT], dvt[DT];  // dK^T, dV^T : [d][key], col = key = kw0 + r
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dkt[dt] = (f32x16)(0.f);
    dvt[dt] = (f32x16)(0.f);
  }
  const int nqt = (p.S + kBwdBQ - 1) / kBwdBQ;
  const int qt_begin = p.causal ? k0 / kBwdBQ : 0;
  const int key = kw0 + r;

  for (int hh = 0; hh < group; ++hh) {
    const int hq = hk * group + hh;
    const bf16* qb = p.q + b * p.q_sb + hq * p.q_sh;
    const bf16* dob = p.dout + b * p.do_sb + hq * p.do_sh;
    const float* lseb = p.lse + ((int64_t)b * p.Hq + hq) * p.S;
    const float* dlb = p.delta + ((int64_t)b * p.Hq + hq) * p.S;
    float* dqb = p.dq + ((int64_t)b * p.S * p.Hq + hq) * D;
    for (int qt = qt_begin; qt < nqt; ++qt) {
      const int q0 = qt * kBwdBQ;
      __syncthreads();  // previous tile's LDS reads are done
      for (int c = threadIdx.x; c < kBwdBQ * CH; c += kBwdThreads) {
        const int row = c / CH, ch = c % CH;
        const int q = q0 + row;
        uint4 qv = make_uint4(0, 0, 0, 0), dv = make_uint4(0, 0, 0, 0);
        if (q < p.S) {
          qv = *reinterpret_cast<const uint4*>(qb + (int64_t)q * p.q_ss + ch * 8);
          dv = *reinterpret_cast<const uint4*>(dob + (int64_t)q * p.do_ss + ch * 8);
        }
        *reinterpret_cast<uint4*>(q_lds + row * D + swz_dual<D>(row, ch) * 8) = qv;
        *reinterpret_cast<uint4*>(do_lds + row * D + swz_dual<D>(row, ch) * 8) = dv;
      }
      if (threadIdx.x < kBwdBQ) {
        const int q = q0 + threadIdx.x;
        lse_lds[threadIdx.x] = q < p.S ? lseb[q] * kLog2e : INFINITY;  // log2 domain; +inf -> p = 0
        dl_lds[threadIdx.x] = q < p.S ? dlb[q] : 0.f;
      }
      __syncthreads();
      const bool wave_active = !(p.causal && q0 + kBwdBQ - 1 < kw0);  // some query sees some key
      f32x16 sacc, dpacc;
      if (wave_active) {
        // init accumulators with the row constants: S' = S*scale*log2e - lse2, dP' = dP - delta
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = (i & 3) + 8 * (i >> 2) + 4 * h;
          sacc[i] = -lse_lds[qr] / p.scale_log2;
          dpacc[i] = -dl_lds[qr];
        }
        // S = Q K^T (key on lane): A = Q rows, B = K^T frags
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          bf16x8 a = lds_read_b128(q_lds + r * D + swz_dual<D>(r, 2 * kk + h) * 8);
          sacc = mfma32(a, kf[kk], sacc);
        }
        // dP = dO V^T
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          bf16x8 a = lds_read_b128(do_lds + r * D + swz_dual<D>(r, 2 * kk + h) * 8);
          dpacc = mfma32(a, vf[kk], dpacc);
        }
        // P and dS (row = query, col = key)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int q = q0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          float pv = exp2f(sacc[i] * p.scale_log2);
          if (key >= p.S || q >= p.S || (p.causal && key > q)) pv = 0.f;
          sacc[i] = pv;
          dpacc[i] = pv * dpacc[i] * p.scale;  // dS (includes the softmax scale for dQ / dK)
        }
        bf16x8 pfr[2], dsf[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          pfr[s2] = (bf16x8){(bf16)sacc[8 * s2 + 0], (bf16)sacc[8 * s2 + 1], (bf16)sacc[8 * s2 + 2],
                             (bf16)sacc[8 * s2 + 3], (bf16)sacc[8 * s2 + 4], (bf16)sacc[8 * s2 + 5],
                             (bf16)sacc[8 * s2 + 6], (bf16)sacc[8 * s2 + 7]};
          dsf[s2] = (bf16x8){(bf16)dpacc[8 * s2 + 0], (bf16)dpacc[8 * s2 + 1], (bf16)dpacc[8 * s2 + 2],
                             (bf16)dpacc[8 * s2 + 3], (bf16)dpacc[8 * s2 + 4], (bf16)dpacc[8 * s2 + 5],
                             (bf16)dpacc[8 * s2 + 6], (bf16)dpacc[8 * s2 + 7]};
        }
        // dV^T += dO^T P ; dK^T += Q^T dS   (A operands by transposed reads of the q-tile images)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int col = dt * 32 + 16 * (g & 1) + 4 * (i16 & 3);
          const int ch = col >> 3, within = col & 7;
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const int r1 = 16 * s2 + 4 * h + (i16 >> 2);
            const int r2 = r1 + 8;
            bf16x8 a_do = cat(lds_read_tr(do_lds + r1 * D + swz_dual<D>(r1, ch) * 8 + within),
                              lds_read_tr(do_lds + r2 * D + swz_dual<D>(r2, ch) * 8 + within));
            dvt[dt] = mfma32(a_do, pfr[s2], dvt[dt]);
            bf16x8 a_q = cat(lds_read_tr(q_lds + r1 * D + swz_dual<D>(r1, ch) * 8 + within),
                             lds_read_tr(q_lds + r2 * D + swz_dual<D>(r2, ch) * 8 + within));
            dkt[dt] = mfma32(a_q, dsf[s2], dkt[dt]);
          }
        }
        // dS^T image [key 0..127][q 0..31]: 64-B rows, 8-B pieces; swizzle 16-B chunks by key
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int krow = 32 * w + r;
          const int qc = 8 * g4 + 4 * h;  // 4 consecutive queries
          const int ch = qc >> 3, within = qc & 7;
          bf16x4 v = {(bf16)dpacc[4 * g4 + 0], (bf16)dpacc[4 * g4 + 1], (bf16)dpacc[4 * g4 + 2],
                      (bf16)dpacc[4 * g4 + 3]};
          *reinterpret_cast<bf16x4*>(ds_lds + krow * kBwdBQ + ((ch ^ ((krow >> 1) & 3)) * 8) + within) = v;
        }
      } else {
        // keys of this wave all lie after the tile's queries: dS = 0
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int krow = 32 * w + r;
          const int qc = 8 * g4 + 4 * h;
          const int ch = qc >> 3, within = qc & 7;
          *reinterpret_cast<bf16x4*>(ds_lds + krow * kBwdBQ + ((ch ^ ((krow >> 1) & 3)) * 8) + within) =
              (bf16x4)((bf16)0.f);
        }
      }
      __syncthreads();
      // dQ[q][d] += dS[q][key] K[key][d] over the block's 128 keys; wave w owns d-tile w (D=128)
      // A = dS (q on rows, natural k order) via transposed reads of the dS^T image,
      // B = K (key = k, d on lane) via transposed reads of the K image.
      for (int dt = w; dt < DT; dt += 4) {
        f32x16 dqacc = (f32x16)(0.f);
        const int kmax = p.causal ? min(kBwdBKV, q0 + kBwdBQ - k0) : kBwdBKV;  // keys beyond the last query give dS = 0
#pragma unroll 2
        for (int ks = 0; ks < kBwdBKV / 16; ++ks) {
          if (ks * 16 >= kmax) break;
          // A: lane (r = q, h) elements j = dS[q = r][key = 16ks + 8h + j]; rows of the dS^T image are keys
          const int qcol = 16 * (g & 1) + 4 * (i16 & 3);  // column block of the dS^T image (queries)
          const int kr1 = 16 * ks + 8 * h + (i16 >> 2);
          const int kr2 = kr1 + 4;
          const int ach = qcol >> 3, aw = qcol & 7;
          bf16x8 a = cat(lds_read_tr(ds_lds + kr1 * kBwdBQ + ((ach ^ ((kr1 >> 1) & 3)) * 8) + aw),
                         lds_read_tr(ds_lds + kr2 * kBwdBQ + ((ach ^ ((kr2 >> 1) & 3)) * 8) + aw));
          // B: lane (r = d, h) elements j = K[key = 16ks + 8h + j][d = 32dt + r]
          const int dcol = dt * 32 + 16 * (g & 1) + 4 * (i16 & 3);
          const int bch = dcol >> 3, bw = dcol & 7;
          bf16x8 bb = cat(lds_read_tr(k_lds + kr1 * D + swz_dual<D>(kr1, bch) * 8 + bw),
                          lds_read_tr(k_lds + kr2 * D + swz_dual<D>(kr2, bch) * 8 + bw));
          dqacc = mfma32(a, bb, dqacc);
        }
        // rows = queries, col = d: each atomic instruction covers two 128-B row segments
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int q = q0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (q < p.S) atomicAdd(dqb + (int64_t)q * p.Hq * D + dt * 32 + r, dqacc[i]);
        }
      }
    }
  }
  // write dK, dV (scale already folded into dS)
  if (key < p.S) {
    bf16* dkr = p.dk + (((int64_t)b * p.S + key) * p.Hkv + hk) * D;
    bf16* dvr = p.dv + (((int64_t)b * p.S + key) * p.Hkv + hk) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * h;
        *reinterpret_cast<bf16x4*>(dkr + d) = (bf16x4){(bf16)dkt[dt][4 * g4 + 0], (bf16)dkt[dt][4 * g4 + 1],
                                                       (bf16)dkt[dt][4 * g4 + 2], (bf16)dkt[dt][4 * g4 + 3]};
        *reinterpret_cast<bf16x4*>(dvr + d) = (bf16x4){(bf16)dvt[dt][4 * g4 + 0], (bf16)dvt[dt][4 * g4 + 1],
                                                       (bf16)dvt[dt][4 * g4 + 2], (bf16)dvt[dt][4 * g4 + 3]};
      }
  }
}

__global__ void f32_to_bf16_rows_kernel(const float* __restrict__ src, bf16* __restrict__ dst, int64_t n) {
  const int64_t nv = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 a = *reinterpret_cast<const f32x4*>(src + i * 8);
    f32x4 c = *reinterpret_cast<const f32x4*>(src + i * 8 + 4);
    store8f(dst + i * 8, (f32x8){a[0], a[1], a[2], a[3], c[0], c[1], c[2], c[3]});
  }
}

void check_qkv(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, name, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, name, " must be [B, S, H, D] with unit stride on D");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              name, " strides must keep 16-byte alignment");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
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
  FwdParams p{reinterpret_cast<const bf16*>(q.data_ptr()), reinterpret_cast<const bf16*>(k.data_ptr()),
              reinterpret_cast<const bf16*>(v.data_ptr()), reinterpret_cast<bf16*>(out.data_ptr()),
              lse.data_ptr<float>(), q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
              v.stride(0), v.stride(1), v.stride(2), B, S, Hq, Hkv, (float)(softmax_scale * kLog2e), causal};
  const int nqt = (S + kFwdBQ - 1) / kFwdBQ;
  const int64_t blocks = (int64_t)nqt * B * Hq;
  auto stream = c10::hip::getCurrentHIPStream();
  if (D == 128)
    flash_fwd_kernel<128><<<blocks, kFwdThreads, 0, stream>>>(p);
  else
    flash_fwd_kernel<64><<<blocks, kFwdThreads, 0, stream>>>(p);
  DLGM_CHECK_HIP(hipGetLastError());
  return {out, lse};
}

// Returns (dq, dk, dv) with the shapes of q, k, v (contiguous).
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_flash_attn_bwd(const at::Tensor& dout, const at::Tensor& q,
                                                                   const at::Tensor& k, const at::Tensor& v,
                                                                   const at::Tensor& out, const at::Tensor& lse,
                                                                   double softmax_scale, bool causal) {
  check_qkv(q, "q");
  check_qkv(k, "k");
  check_qkv(v, "v");
  check_qkv(dout, "dout");
  const int B = q.size(0), S = q.size(1), Hq = q.size(2), D = q.size(3);
  const int Hkv = k.size(2);
  TORCH_CHECK(D == 128 || D == 64, "flash_attn_bwd: head dim must be 64 or 128");
  TORCH_CHECK(out.is_contiguous() && out.sizes() == q.sizes(), "flash_attn_bwd: out must be contiguous [B,S,Hq,D]");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)B * Hq * S, "flash_attn_bwd: bad lse");
  TORCH_CHECK(dout.sizes() == q.sizes(), "flash_attn_bwd: dout shape mismatch");
  auto dq32 = at::zeros({B, S, Hq, D}, q.options().dtype(at::kFloat));
  auto dk = at::empty({B, S, Hkv, D}, q.options());
  auto dv = at::empty({B, S, Hkv, D}, q.options());
  auto dq = at::empty({B, S, Hq, D}, q.options());
  if (B == 0 || S == 0) return {dq.zero_(), dk.zero_(), dv.zero_()};
  auto delta = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  auto stream = c10::hip::getCurrentHIPStream();
  const int64_t rows = (int64_t)B * S * Hq;
  auto dop = reinterpret_cast<const bf16*>(dout.data_ptr());
  if (D == 128)
    flash_bwd_delta_kernel<128><<<(rows + 3) / 4, 256, 0, stream>>>(dop, reinterpret_cast<const bf16*>(out.data_ptr()),
                                                                     delta.data_ptr<float>(), B, S, Hq, dout.stride(1),
                                                                     dout.stride(2), dout.stride(0));
  else
    flash_bwd_delta_kernel<64><<<(rows + 3) / 4, 256, 0, stream>>>(dop, reinterpret_cast<const bf16*>(out.data_ptr()),
                                                                    delta.data_ptr<float>(), B, S, Hq, dout.stride(1),
                                                                    dout.stride(2), dout.stride(0));
  DLGM_CHECK_HIP(hipGetLastError());
  BwdParams p{reinterpret_cast<const bf16*>(q.data_ptr()), reinterpret_cast<const bf16*>(k.data_ptr()),
              reinterpret_cast<const bf16*>(v.data_ptr()), dop, lse.data_ptr<float>(), delta.data_ptr<float>(),
              dq32.data_ptr<float>(), reinterpret_cast<bf16*>(dk.data_ptr()), reinterpret_cast<bf16*>(dv.data_ptr()),
              q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2), v.stride(0), v.stride(1),
              v.stride(2), dout.stride(0), dout.stride(1), dout.stride(2), B, S, Hq, Hkv, (float)softmax_scale,
              (float)(softmax_scale * kLog2e), causal};
  const int nkt = (S + kBwdBKV - 1) / kBwdBKV;
  const int64_t blocks = (int64_t)nkt * B * Hkv;
  if (D == 128)
    flash_bwd_kernel<128><<<blocks, kBwdThreads, 0, stream>>>(p);
  else
    flash_bwd_kernel<64><<<blocks, kBwdThreads, 0, stream>>>(p);
  DLGM_CHECK_HIP(hipGetLastError());
  const int64_t n = dq32.numel();
  f32_to_bf16_rows_kernel<<<std::min<int64_t>((n / 8 + 255) / 256, 4096), 256, 0, stream>>>(
      dq32.data_ptr<float>(), reinterpret_cast<bf16*>(dq.data_ptr()), n);
  DLGM_CHECK_HIP(hipGetLastError());
  return {dq, dk, dv};
}
