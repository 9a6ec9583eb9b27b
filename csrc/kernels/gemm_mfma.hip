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
// Work order: blocks are remapped so consecutive tiles (sharing an A row panel) land on one XCD. Grouped-M launches
// with K >= 4096 run each XCD's whole rounds of tiles as usual and its short last round as 2-4 K parts per tile
// (fp32 partials + tail_reduce_kernel), so the last round is not left mostly idle (tail_plan).
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include <cstdlib>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int TILE_BYTES = 256 * BK * 2;  // one operand tile: 32 KiB

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) void* lptr_t;

enum Epi { kStoreBf16 = 0, kStoreF32 = 1, kAccF32 = 2 };
enum Mode { kDense = 0, kGroupM = 1, kGroupK = 2, kGroupKSeg = 3 };
constexpr int kMaxSeg = 8;  // grouped-K over segments: at most this many (micro-batch) row sets per launch

struct GemmArgs {
  const bf16* a;
  const bf16* b;
  void* c;
  // kGroupKSeg: segment s has its own token-major operands (a_seg[s] [R_s, M], b_seg[s] [R_s, N]) and
  // offsets[s * (G + 1) ..] split its rows by group; group g reduces over its rows of every segment
  const bf16* a_seg[kMaxSeg];
  const bf16* b_seg[kMaxSeg];
  int nseg;
  int64_t lda, ldb, ldc;           // leading (non-unit) strides in elements
  int64_t a_gstride, b_gstride, c_gstride;  // per-group pointer steps (elements) for grouped modes
  const int* offsets;              // [G + 1] exclusive prefix over the grouped dimension (device)
  int M, N, K;                     // K: dense / grouped-M reduction length; M: rows for dense/grouped-K
  int G, mode;
  int tiles_n, tiles_m;
  int qskip;  // skip the MFMAs of row quadrants wholly past the valid rows (+0.5 % Mixtral, round 3)
  int chunk;  // grouped-M: balanced remap over the real tiles (+0.7 % vs contiguous over the grid, round 3)
  int splitk;          // grouped-M split-K: each tile's K range in this many parts, fp32 partials
  int64_t c_sstride;   // elements between the partial slices of C (split-K)
  int nreal;           // grouped-K with the chunk remap: real blocks (the grid is rounded up to 8 * kChunk)
  float* stats_part;   // grouped-K fp32 epilogues: per-tile (sum of squares of the finite, #non-finite) of the
                       // FINAL C values, at [2 * tile] (deterministic: reduced later in a fixed order)
  // bf16 epilogue fused with the SwiGLU backward (the MoE down projection's input gradient): the tile's values are
  // dA = dY @ W_down; instead of storing dA, read gate / up of the same rows and columns from glu ([rows, 2 glu_f],
  // row stride ldc) and store dgate at column c and dup at column glu_f + c of C ([rows, 2 glu_f])
  const bf16* glu;
  int glu_f;
  // grouped-M tail split (bf16 out): per XCD, the whole rounds of tiles run unsplit and the short last round's
  // tiles run with their K range in s parts (s = 2..4 blocks a tile, chosen to fill the CUs best); those blocks
  // store fp32 partials at tpart [8 XCDs][kMaxSplit * xcu slices][BM][BN] that tail_reduce_kernel sums into C.
  // xcu = CUs per XCD (one block per CU: the kernel's LDS and registers admit one)
  int tsplit, xcu, tmax;  // tmax: most K parts per tail tile (2..kMaxSplit)
  int tbands;             // tail_reduce_kernel blocks per tile (row bands of BM / tbands rows)
  float* tpart;
};

constexpr int kMaxSplit = 4;

// Per-XCD plan of the tail split: the XCD runs tiles [x q, x q + qx); the first `full` of them unsplit, then (s > 1)
// the remaining `tail` tiles as s K parts each. s minimises the last round's length ceil(tail s / xcu) / s tile
// times (ties: the fewer parts), e.g. with 32 CUs: tail 8 -> 4 parts (1/4), 10 -> 3, 16 -> 2, 20 -> 3 (2/3),
// 24 -> 4 (3/4), 25.. -> none.
struct TailPlan {
  int qx, full, tail, s;
};

__device__ __forceinline__ TailPlan tail_plan(int real, int q, int x, int xcu, int tmax) {
  TailPlan t;
  t.qx = max(0, min(q, real - x * q));
  const int whole = t.qx / xcu * xcu;
  t.tail = t.qx - whole;
  t.s = 1;
  if (t.tail > 0) {
    int best_num = 1, best_den = 1;  // last-round length as a fraction of a tile time: rounds / s
    for (int s = 2; s <= tmax; ++s) {
      const int rounds = (t.tail * s + xcu - 1) / xcu;
      if (rounds * best_den < best_num * s) {
        best_num = rounds;
        best_den = s;
        t.s = s;
      }
    }
  }
  t.full = t.s > 1 ? whole : t.qx;
  return t;
}

// grouped-M: the tiles of a group are its row tiles x all column tiles, group after group, row tiles fastest
// (see the kernel). Tile j -> group, column tile, first row and row end; false past the last group's tiles.
__device__ __forceinline__ bool group_tile(const GemmArgs& p, int j, int& grp, int& tn, int& m_lo, int& m_hi) {
  for (int e = 0; e < p.G; ++e) {
    const int lo = p.offsets[e], hi = p.offsets[e + 1];
    const int te = (hi - lo + BM - 1) / BM;
    if (j < te * p.tiles_n) {
      grp = e;
      tn = j / te;
      m_lo = lo + (j - tn * te) * BM;
      m_hi = hi;
      return true;
    }
    j -= te * p.tiles_n;
  }
  return false;
}

__device__ __forceinline__ int grouped_real_tiles(const GemmArgs& p) {
  int real = 0;
  for (int e = 0; e < p.G; ++e) real += (p.offsets[e + 1] - p.offsets[e] + BM - 1) / BM;
  return real * p.tiles_n;
}


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

// 16 zero bytes in global memory: the source of the k rows past a partial K tile (grouped-K group ends)
__device__ __attribute__((aligned(16))) bf16 g_zero16[8];

// Half-tile staging plan of one operand. OP 0 = A (halves split the M rows by quadrant: half h holds rows
// wr*128 + h*64 + [0, 64) of both wave rows), OP 1 = B (half h holds columns wc*64 + h*32 + [0, 32) of all four
// wave columns), so a wave's quadrant (mq, nq) reads exactly A half mq and B half nq. Half images:
//   K-contiguous: [128 rows][64 k], 128-B rows, chunk c at c ^ ((row>>1)&7)       (ds_read_b128 fragments)
//   MN-contiguous: [64 k][128 cols], 256-B rows, chunk c at c ^ swz_mn(k)          (ds_read_b64_tr_b16 pairs)
// 16 pieces of 1 KiB per half; wave w moves pieces w and w+8, whose source offsets differ by a constant
// (the swizzle period divides the piece step), as do the two halves: one VGPR offset per operand.
template <bool KMAJ, int OP>
struct HalfStager {
  uint32_t voff, piece2, hstep;
  int wave;
  __device__ __forceinline__ HalfStager(int64_t ld, int wave_, int lane) : wave(wave_) {
    if constexpr (KMAJ) {
      const int hr = 8 * wave + (lane >> 3), c = (lane & 7) ^ swz_k(hr);
      const int grow = OP == 0 ? (hr >> 6) * 128 + (hr & 63) : (hr >> 5) * 64 + (hr & 31);
      voff = (uint32_t)((grow * ld + c * 8) * 2);
      piece2 = (uint32_t)(128 * ld * 2);  // half-row + 64 -> tile row + 128 (both operands)
      hstep = (uint32_t)((OP == 0 ? 64 : 32) * ld * 2);
    } else {
      const int k = 4 * wave + (lane >> 4), c = (lane & 15) ^ swz_mn(k);
      const int lc = c * 8;
      const int gcol = OP == 0 ? (lc >> 6) * 128 + (lc & 63) : (lc >> 5) * 64 + (lc & 31);
      voff = (uint32_t)((k * ld + gcol) * 2);
      piece2 = (uint32_t)(32 * ld * 2);  // k + 32
      hstep = (uint32_t)((OP == 0 ? 64 : 32) * 2);
    }
  }
  // Stage half `h` of the tile at `base` (row / k-row 0 of the tile; `nbytes` bounds the valid region from
  // base) into `img`. `nvalid` < the image's rows (256 tile rows K-contiguous, 64 k-rows MN-contiguous): a
  // partial tile, whose rows past the end are clamped onto the last valid one (no address leaves the
  // operand; the copies are masked out of the reduction or feed output rows that are never stored).
  template <bool PART>  // PART: partial tiles can occur in this instantiation
  __device__ __forceinline__ void issue(char* img, const bf16* base, uint32_t nbytes, int64_t ld, int h,
                                        int nvalid) const {
    auto guard = [nbytes](uint32_t vo) { return vo + 16 <= nbytes ? vo : 0u; };
    constexpr int ROWS = KMAJ ? 256 : 64;
    const uint32_t v0 = voff + h * hstep;
    if (!PART || __builtin_amdgcn_readfirstlane(nvalid) >= ROWS) {
      dma16(base, nbytes, guard(v0), 0, img + wave * 1024);
      dma16(base, nbytes, guard(v0 + piece2), 0, img + (wave + 8) * 1024);
      return;
    }
    if constexpr (!PART) return;
    // partial tile: the same offsets, each lane's row moved onto the last valid one (negative deltas wrap)
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int row;  // the tile row (K-contiguous) or k-row (MN-contiguous) this lane's 16 B come from
      if constexpr (KMAJ) {
        const int hr = 8 * (wave + 8 * j) + (lane >> 3);
        row = OP == 0 ? (hr >> 6) * 128 + h * 64 + (hr & 63) : (hr >> 5) * 64 + h * 32 + (hr & 31);
      } else {
        row = 4 * (wave + 8 * j) + (lane >> 4);
      }
      if constexpr (KMAJ) {  // rows past the end feed output rows that are never stored: clamp them
        const int src = row < nvalid ? row : nvalid - 1;
        dma16(base, nbytes, guard(v0 + j * piece2 + (uint32_t)((int64_t)(src - row) * ld * 2)), 0,
              img + (wave + 8 * j) * 1024);
      } else {  // k rows past the end must contribute zero: those lanes copy from a zero chunk instead
        if (row < nvalid)
          dma16(base, nbytes, guard(v0 + j * piece2), 0, img + (wave + 8 * j) * 1024);
        else
          dma16(g_zero16, 16, 0, 0, img + (wave + 8 * j) * 1024);
      }
    }
  }
};

// 16x16x32 fragment (lane: row l&15, k = 8(l>>4) + j) of a HALF image, k-substep s, rows r0.. of the half.
// (MASK: zero the elements with k >= kv in registers -- unused: partial K tiles are zero-filled in LDS by
// the staging, which keeps the grouped-K kernel free of spills.)
template <bool KMAJ, bool MASK>
__device__ __forceinline__ bf16x8 frag(const char* img, int r0, int s, int lane, int kv) {
  const int i = lane & 15, g = lane >> 4;
  if constexpr (KMAJ) {
    const int r = r0 + i, c = 4 * s + g;
    return *reinterpret_cast<const bf16x8*>(img + r * 128 + ((c ^ swz_k(r)) << 4));
  } else {
    const int q = i >> 2, p = i & 3;
    const int ch = (r0 >> 3) + (p >> 1);
    const int k1 = 32 * s + 8 * g + q;
    const int x = swz_mn(k1);  // k1 and k1 + 4 share it
    const char* a = img + k1 * 256 + ((ch ^ x) << 4) + (p & 1) * 8;
    bf16x8 v = cat4(lds_tr(a), lds_tr(a + 4 * 256));
    if (MASK && __builtin_amdgcn_readfirstlane(kv) < BK) {
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

constexpr int kChunk = 32;  // consecutive ids kept on one XCD (a 4-row x 8-column patch of one group's tiles)

// block b runs on XCD b % 8 as its (b / 8)-th block; chunk c of kChunk consecutive ids goes to XCD c % 8
__device__ __forceinline__ int chunk_remap(int b) {
  const int x = b & 7, k = b >> 3;
  return (k / kChunk) * (8 * kChunk) + x * kChunk + (k % kChunk);
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// One K-tile of the main loop = 4 phases; each phase: this phase's LDS fragment reads, one half-tile of
// LDS-DMA for a later K-tile, a counted vmcnt, barrier, 16 MFMAs (one 64x32 output quadrant x K=64),
// barrier. The two wave rows run one barrier apart (wave row 1 takes an extra barrier up front), so on
// every SIMD one wave issues its reads / DMA while the other runs MFMAs. Read / restage rules
// (cdna_hip_programming.md §5 '8-phase template'): a half-tile is read one phase after the wait that retires
// it, and restaged at least two phases after its last read:
//   phase 1 reads A half 0 + B half 0 (K-tile k) and stages B half 1 of k+1 (other buffer),
//   phase 2 reads B half 1 and stages A half 1 of k+1,
//   phase 3 reads A half 1 and stages A half 0 of k+2 (this buffer: last read in phase 1),
//   phase 4 reads nothing (every fragment is in registers) and stages B half 0 of k+2.
// With that order four half-tiles are always in flight: vmcnt(8) (2 DMA instructions per half-tile) before
// each phase's first barrier retires exactly what the next phase reads, until the stages run out (then 0).
template <int N>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N == 6)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int MODE, bool AK, bool BKM, int EPI>
__global__ __launch_bounds__(NTHR, 1) void gemm_mfma_kernel(GemmArgs p) {
  // DMA placement (tools/gemm_sched_ab.py, profiles/gemm_sched_ab_r04*.jsonl, random operands, bit-identical output):
  //   SC 1: two half-tiles in phases 2 and 4 only (B1 A1 of t+1 | B0 A0 of t+2), none beside phase 1's 12 reads --
  //         dense and grouped-M 2-4 % faster than SC 0, grouped-K (dW) 1.5 % faster once its operand rows are whole
  //         128-B lines (profiles/transpose_row_pad_r04.jsonl; with misaligned rows SC 0 had measured 4-6 % faster);
  //   SC 0: one half-tile per phase (B1 | A1 | A0 | B0), phase reads 12 / 4 / 8 / 0 -- kept for the segmented
  //         grouped-K over token-major or per-segment operands. (Reading B half 0 of the next tile a phase early into
  //         a second register set, phase reads 8 / 4 / 8 / 4, was slower than SC 1 on every shape.)
  constexpr int SC = MODE == kGroupKSeg ? 0 : 1;
  __shared__ __attribute__((aligned(1024))) char smem[4 * TILE_BYTES];  // [buf][A | B][half][16 KiB]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- which tile (and group) this block computes. The mode is a template parameter: each
  // instantiation has straight-line pointer setup (no mode-dependent phis for the operand bases).
  // grouped-M grids are sized for the worst case and their tail is spare blocks: the XCD-contiguous remap over the
  // whole grid hands every spare id to the last XCD(s) and leaves them idle (the real tiles are the low ids)
  int id;
  int tslice = -1, tpi = 0, tparts = 1;  // tail split: partial slice, K part and parts of this block's tile
  if constexpr (MODE == kGroupM) {
    if (p.chunk) {
      // balanced XCD-contiguous order over the REAL tiles (counted from the device offsets): XCD x runs ids
      // [x*q, (x+1)*q) first and its spare blocks last, so every XCD gets 1/8 of the work and each keeps the
      // contiguous, L2-sharing run of an expert's tiles
      const int real = grouped_real_tiles(p) * p.splitk;
      const int q = (real + 7) / 8, x = blockIdx.x & 7, k = blockIdx.x >> 3;
      if (p.tsplit) {  // the XCD's whole rounds unsplit, then its short last round as K parts (s blocks a tile)
        const TailPlan tp = tail_plan(real, q, x, p.xcu, p.tmax);
        if (k < tp.full) {
          id = x * q + k;
        } else if (tp.s > 1 && k - tp.full < tp.s * tp.tail) {
          const int kk = k - tp.full;
          id = x * q + tp.full + kk / tp.s;
          tslice = x * kMaxSplit * p.xcu + kk;  // = the tile's first slice + its part
          tpi = kk % tp.s;
          tparts = tp.s;
        } else {
          return;  // spare block
        }
      } else {
        id = x * q + k;
        if (k >= q || id >= real) return;  // spare block (grid sized for the worst case)
      }
    } else {
      id = xcd_remap(blockIdx.x, gridDim.x);
    }
  } else if constexpr (MODE == kGroupK || MODE == kGroupKSeg) {
    // grouped-K: a group's tiles are contiguous ids and their work scales with the group's rows, so the XCD-
    // contiguous remap gave each XCD about one expert and the launch waited for the busiest expert's XCD (+29 %
    // at Mixtral routing); chunks of kChunk consecutive ids dealt round-robin give every XCD the same mix of
    // experts and keep each chunk's A / B panels inside one L2. The grid is a multiple of 8 * kChunk.
    if (p.chunk) {
      id = chunk_remap(blockIdx.x);
      if (id >= p.nreal) return;
    } else {
      id = xcd_remap(blockIdx.x, gridDim.x);
    }
  } else {
    id = xcd_remap(blockIdx.x, gridDim.x);
  }
  int tm = 0, tn, grp = 0;
  int m_lo = 0, m_hi = p.M;  // valid rows of A / C for this block
  int k_lo = 0, k_hi = p.K;  // reduction range
  int64_t split_off = 0;     // grouped-M split-K: this block's partial slice of C (elements)
  constexpr int CES = EPI == kStoreBf16 ? 2 : 4;
  // tile order: GM output rows x all columns per group, walked down the GM rows first, so the ~32 blocks
  // resident on one XCD (consecutive ids after the XCD remap) cover a GM x (32/GM) patch: per K-step they
  // read GM A tiles + 32/GM B tiles instead of 1-2 A + ~30 B tiles (half the L2 misses, measured)
  constexpr int GM = 4;
  auto grouped_tile = [&](int lin, int tiles_m, int& om, int& on) {
    const int per = GM * p.tiles_n;
    const int g = lin / per, rem = lin - g * per;
    const int gm = min(GM, tiles_m - g * GM);
    on = rem / gm;
    om = g * GM + (rem - on * gm);
  };
  if constexpr (MODE == kDense) {
    grouped_tile(id, p.tiles_m, tm, tn);
  } else if constexpr (MODE == kGroupM) {
    // expert by expert; within an expert the row tiles run fastest, so the ~32 blocks resident on one XCD
    // (consecutive ids after the remap) share each weight column panel across all the expert's row tiles
    // (one HBM read of the panel, the rest L2 hits) instead of streaming every panel once per row tile
    int j = id;
    if (p.splitk > 1) {  // adjacent ids = the K parts of one tile (same XCD: their A / B panels share L2 lines)
      const int part = j % p.splitk;
      j /= p.splitk;
      const int ks = ((p.K + p.splitk - 1) / p.splitk + BK - 1) / BK * BK;
      k_lo = part * ks;
      k_hi = min(p.K, k_lo + ks);
      split_off = (int64_t)part * p.c_sstride;
    }
    if (tslice >= 0) {
      const int ks = ((p.K + tparts - 1) / tparts + BK - 1) / BK * BK;
      k_lo = min(p.K, tpi * ks);
      k_hi = min(p.K, k_lo + ks);
    }
    // expert by expert, row tiles fastest (group_tile); m_lo = this block's first row (absolute)
    if (!group_tile(p, j, grp, tn, m_lo, m_hi)) return;  // spare block: the grid is sized for the worst case
  } else {  // grouped-K (one segment, or kGroupKSeg: the group's rows of every segment)
    const int per = p.tiles_m * p.tiles_n;
    grp = id / per;
    grouped_tile(id - grp * per, p.tiles_m, tm, tn);
    if constexpr (MODE == kGroupK) {
      k_lo = p.offsets[grp];
      k_hi = p.offsets[grp + 1];
    }
  }
  // kGroupKSeg: this group's row range in every segment and the cumulative K-tile counts (seg_cum[s] = first
  // K-tile of segment s), loaded once: the stage calls inside the pipelined loop then select among registers
  // (a scalar load there would add an lgkmcnt wait, which also drains the in-flight LDS fragment reads)
  int seg_cum[kMaxSeg + 1], seg_lo[kMaxSeg], seg_hi[kMaxSeg];
  seg_cum[0] = 0;
  if constexpr (MODE == kGroupKSeg) {
#pragma unroll
    for (int sg = 0; sg < kMaxSeg; ++sg) {
      int lo = 0, hi = 0;
      if (sg < p.nseg) {
        lo = p.offsets[sg * (p.G + 1) + grp];
        hi = p.offsets[sg * (p.G + 1) + grp + 1];
      }
      seg_lo[sg] = __builtin_amdgcn_readfirstlane(lo);
      seg_hi[sg] = __builtin_amdgcn_readfirstlane(hi);
      seg_cum[sg + 1] = seg_cum[sg] + (seg_hi[sg] - seg_lo[sg] + BK - 1) / BK;
    }
  }
  const bf16* A0 = p.a;
  const bf16* B0 = p.b + (MODE == kGroupM ? (int64_t)grp * p.b_gstride : 0);
  char* C = (char*)p.c + (MODE == kGroupK || MODE == kGroupKSeg ? (int64_t)grp * p.c_gstride * CES : 0) +
            split_off * CES;
  const int m0 = MODE == kGroupM ? m_lo : tm * BM;
  const int n0 = tn * BN;
  const int rows_valid = min(BM, m_hi - m0);
  if (rows_valid <= 0) return;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4)(0.f);

  const int nk = MODE == kGroupKSeg ? seg_cum[kMaxSeg] : (k_hi - k_lo + BK - 1) / BK;
  // an empty reduction that accumulates leaves C as it is: skip the read-modify-write of the tile (the MoE
  // capacity layout's overflow dW launches cover every expert and usually find no rows at all)
  if (EPI == kAccF32 && nk <= 0 && p.stats_part == nullptr) return;  // (with stats: count the old values)
  // partial tiles: K (grouped-K group ends), M rows (K-contiguous A: grouped-M group ends / M % 256 != 0)
  constexpr bool PK = MODE == kGroupK || MODE == kGroupKSeg, PM = AK;
  if (nk > 0) {
    const HalfStager<AK, 0> sa(p.lda, w, lane);
    const HalfStager<BKM, 1> sb(p.ldb, w, lane);
    auto region = [&](int buf, int op, int h) { return smem + buf * 2 * TILE_BYTES + op * TILE_BYTES + h * (TILE_BYTES / 2); };
    // stage half h of operand op for K-tile t (skipped past the end); returns whether anything was issued
    auto stage = [&](int op, int h, int t) -> bool {
      if (t >= nk) return false;
      int k0, kv;
      const bf16* A = A0;
      const bf16* B = B0;
      if constexpr (MODE == kGroupKSeg) {
        // the segment holding K-tile t (empty segments are stepped over), selected among registers
        int cum = 0, lo = 0, hi = 0;
#pragma unroll
        for (int q = 0; q < kMaxSeg; ++q) {
          const bool in = t >= seg_cum[q];
          cum = in ? seg_cum[q] : cum;
          lo = in ? seg_lo[q] : lo;
          hi = in ? seg_hi[q] : hi;
          A = in ? p.a_seg[q] : A;
          B = in ? p.b_seg[q] : B;
        }
        k0 = lo + (t - cum) * BK;
        kv = min(BK, hi - k0);
      } else {
        k0 = k_lo + t * BK;
        kv = min(BK, k_hi - k0);
      }
      char* img = region(t & 1, op, h);
      if (op == 0) {
        if constexpr (AK)
          sa.template issue<PM>(img, A + (int64_t)m0 * p.lda + k0, (uint32_t)(((int64_t)(rows_valid - 1) * p.lda + BK) * 2), p.lda,
                   h, rows_valid);
        else
          sa.template issue<PK>(img, A + (int64_t)k0 * p.lda + m0, (uint32_t)(((int64_t)(kv - 1) * p.lda + BM) * 2), p.lda, h, kv);
      } else {
        if constexpr (BKM)
          sb.template issue<false>(img, B + (int64_t)n0 * p.ldb + k0, (uint32_t)(((int64_t)(BN - 1) * p.ldb + BK) * 2), p.ldb, h, BN);
        else
          sb.template issue<PK>(img, B + (int64_t)k0 * p.ldb + n0, (uint32_t)(((int64_t)(kv - 1) * p.ldb + BN) * 2), p.ldb, h, kv);
      }
      return true;
    };
    auto wait = [](bool all_issued) {
      if (all_issued)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    bf16x8 af[4][2], bq0[2][2], bq1[2][2];
    auto mma = [&](int mq, int nq) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * mq + i][2 * nq + j] = mfma16(nq ? bq1[j][s2] : bq0[j][s2], af[i][s2], acc[4 * mq + i][2 * nq + j]);
      __builtin_amdgcn_s_setprio(0);
    };
    // a partial M tile (a group's last row tile, or M % 256): a wave skips the MFMAs of its 64-row quadrants that
    // lie wholly past the valid rows (their outputs are never stored) -- the SIMD's MFMA pipe then serves the
    // partner wave alone. Barriers and DMA are unchanged, so the phase structure holds for every wave.
    const int rv = p.qskip ? __builtin_amdgcn_readfirstlane(rows_valid) : BM;
    auto phase_end = [&](bool issued, int mq, int nq) {
      wait(issued);
      raw_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (wr * 128 + mq * 64 < rv) mma(mq, nq);
      raw_barrier();
    };
    // SC 1: the wait keeps the N youngest DMA instructions in flight when the newest stage call issued (N 99: none)
    auto phase_end_n = [&](auto nc, bool issued, int mq, int nq) {
      constexpr int N = decltype(nc)::value;
      if constexpr (N != 99) {
        if (issued)
          vm_wait<N>();
        else
          vm_wait<0>();
      }
      raw_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (wr * 128 + mq * 64 < rv) mma(mq, nq);
      raw_barrier();
    };
    auto ktile = [&](auto bufc, int t) {
      constexpr int buf = decltype(bufc)::value;
      const int kv = min(BK, k_hi - (k_lo + t * BK));
      const char* a0 = region(buf, 0, 0);
      const char* a1 = region(buf, 0, 1);
      const char* b0 = region(buf, 1, 0);
      const char* b1 = region(buf, 1, 1);
      if constexpr (SC == 0) {
        // phase 1: A half 0 + B half 0 -> quadrant (0, 0)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int j = 0; j < 2; ++j) bq0[j][s2] = frag<BKM, false>(b0, wc * 32 + 16 * j, s2, lane, kv);
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i][s2] = frag<AK, false>(a0, wr * 64 + 16 * i, s2, lane, kv);
        }
        phase_end(stage(1, 1, t + 1), 0, 0);
        // phase 2: B half 1 -> quadrant (0, 1)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 2; ++j) bq1[j][s2] = frag<BKM, false>(b1, wc * 32 + 16 * j, s2, lane, kv);
        phase_end(stage(0, 1, t + 1), 0, 1);
        // phase 3: A half 1 -> quadrant (1, 1)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i][s2] = frag<AK, false>(a1, wr * 64 + 16 * i, s2, lane, kv);
        phase_end(stage(0, 0, t + 2), 1, 1);
        // phase 4: registers only -> quadrant (1, 0)
        phase_end(stage(1, 0, t + 2), 1, 0);
      } else {
        // SC 1: DMA only in phases 2 (B1, A1 of t+1) and 4 (B0, A0 of t+2). Waits: phase p's retires what
        // phase p+1 reads, counted in DMA instructions issued after it (6 / 8 / none / 8)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
          for (int j = 0; j < 2; ++j) bq0[j][s2] = frag<BKM, false>(b0, wc * 32 + 16 * j, s2, lane, kv);
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i][s2] = frag<AK, false>(a0, wr * 64 + 16 * i, s2, lane, kv);
        }
        phase_end_n(std::integral_constant<int, 6>{}, t + 1 < nk, 0, 0);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 2; ++j) bq1[j][s2] = frag<BKM, false>(b1, wc * 32 + 16 * j, s2, lane, kv);
        stage(1, 1, t + 1);
        phase_end_n(std::integral_constant<int, 8>{}, stage(0, 1, t + 1), 0, 1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i][s2] = frag<AK, false>(a1, wr * 64 + 16 * i, s2, lane, kv);
        phase_end_n(std::integral_constant<int, 99>{}, true, 1, 1);
        stage(1, 0, t + 2);
        phase_end_n(std::integral_constant<int, 8>{}, stage(0, 0, t + 2), 1, 0);
      }
    };
    if constexpr (SC == 0) {
      // prologue: the six half-tiles the loop expects in flight (in the loop's stage order)
      stage(0, 0, 0);
      stage(1, 0, 0);
      stage(1, 1, 0);
      stage(0, 1, 0);
      stage(0, 0, 1);
      wait(stage(1, 0, 1));
      raw_barrier();
    } else {
      // prologue: the queue of the steady state before tile 0 (B0 A0 | B1 A1 of 0 | B0 A0 of 1)
      stage(1, 0, 0);
      stage(0, 0, 0);
      stage(1, 1, 0);
      stage(0, 1, 0);
      stage(1, 0, 1);
      if (stage(0, 0, 1))
        vm_wait<8>();
      else
        vm_wait<0>();
      raw_barrier();
    }
    if (wr == 1) raw_barrier();  // wave row 1 runs one barrier behind
    for (int t = 0; t < nk; t += 2) {
      ktile(std::integral_constant<int, 0>{}, t);
      if (t + 1 < nk) ktile(std::integral_constant<int, 1>{}, t + 1);
    }
    if (wr == 0) raw_barrier();  // equal barrier counts for both wave rows
  }

  // ---- epilogue: lane holds C[m][n .. n+3] (m = column of D^T, n = 4 rows of D^T)
  const int i = lane & 15, g = lane >> 4;
  float st_ss = 0.f, st_bad = 0.f;  // gradient statistics of the stored values (grouped-K, p.stats_part)
  auto tally = [&](const f32x4& v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool fin = __builtin_isfinite(v[j]);
      st_bad += fin ? 0.f : 1.f;
      st_ss += fin ? v[j] * v[j] : 0.f;
    }
  };
  constexpr bool KSTATS = (MODE == kGroupK || MODE == kGroupKSeg) && EPI != kStoreBf16;
  if constexpr (MODE == kGroupM && EPI == kStoreBf16) {
    if (tslice >= 0) {  // a split tail tile: this K part's fp32 partial, summed into C by tail_reduce_kernel
      float* T = p.tpart + (int64_t)tslice * BM * BN;
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        const int mrow = wr * 128 + 16 * mi + i;
        if (mrow >= rows_valid) continue;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          *reinterpret_cast<f32x4*>(T + mrow * BN + wc * 64 + 16 * ni + 4 * g) = acc[mi][ni];
      }
      return;
    }
  }
  if constexpr (EPI == kStoreBf16) {
    // bf16 tile through LDS: the accumulators' native layout gives 8-byte stores of 16 rows x 32 B each; staged as
    // a row-major [256][512 B] image (16-B chunk c of row r at c ^ (r & 31): conflict-free 8-byte writes and
    // 16-byte reads), every wave then stores two whole 512-B rows per instruction
    __syncthreads();  // every wave is done with the operand images (the last DMA was drained by vmcnt(0))
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int mrow = wr * 128 + 16 * mi + i;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int byte = (wc * 64 + 16 * ni + 4 * g) * 2;  // within the 512-B row
        const int ch = (byte >> 4) ^ (mrow & 31);
        bf16x4 v = {(bf16)acc[mi][ni][0], (bf16)acc[mi][ni][1], (bf16)acc[mi][ni][2], (bf16)acc[mi][ni][3]};
        *reinterpret_cast<bf16x4*>(smem + mrow * 512 + ch * 16 + (byte & 8)) = v;
      }
    }
    __syncthreads();
    const int half = lane >> 5, c = lane & 31;
    if (p.glu != nullptr) {
      // SwiGLU backward on the rounded bf16 dA (the same values and the same fp32 math as swiglu_bwd_kernel)
#pragma unroll 2
      for (int it = 0; it < 16; ++it) {
        const int r = 32 * w + 2 * it + half;
        if (r >= rows_valid) break;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + r * 512 + ((c ^ (r & 31)) << 4));
        const int64_t row = (int64_t)(m0 + r) * p.ldc;
        const int col = n0 + c * 8;
        const f32x8 g = load8f(p.glu + row + col), u = load8f(p.glu + row + p.glu_f + col);
        const f32x8 d = __builtin_convertvector(v, f32x8);
        f32x8 dg, du;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float sg_ = 1.f / (1.f + __expf(-g[j]));
          const float gs = g[j] * sg_;
          du[j] = d[j] * gs;
          dg[j] = d[j] * u[j] * (sg_ + gs * (1.f - sg_));
        }
        bf16* out = reinterpret_cast<bf16*>(C) + row + col;
        store8f(out, dg);
        store8f(out + p.glu_f, du);
      }
      return;
    }
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int r = 32 * w + 2 * it + half;
      if (r >= rows_valid) break;  // (rows are ascending in it: the rest of this wave's rows are past the end)
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + r * 512 + ((c ^ (r & 31)) << 4));
      *reinterpret_cast<bf16x8*>(C + ((int64_t)(m0 + r) * p.ldc + n0 + c * 8) * 2) = v;
    }
    return;
  }
  // fp32 tiles store from the accumulators' layout (16-B stores of 16 rows x 64 B; an LDS-staged whole-row form
  // measured neutral here, unlike the bf16 one)
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int mrow = wr * 128 + 16 * mi + i;  // row within the block tile
    if (mrow >= rows_valid) continue;
    const int64_t m = m0 + mrow;
    if constexpr (EPI == kAccF32) {  // the row group's four reads in flight before the adds
      f32x4 old[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        old[ni] = *reinterpret_cast<const f32x4*>(C + (m * p.ldc + n0 + wc * 64 + 16 * ni + 4 * g) * 4);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const f32x4 nv = old[ni] + acc[mi][ni];
        *reinterpret_cast<f32x4*>(C + (m * p.ldc + n0 + wc * 64 + 16 * ni + 4 * g) * 4) = nv;
        if (KSTATS) tally(nv);
      }
      continue;
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      *reinterpret_cast<f32x4*>(C + (m * p.ldc + n0 + wc * 64 + 16 * ni + 4 * g) * 4) = acc[mi][ni];
      if (KSTATS) tally(acc[mi][ni]);
    }
  }
  if constexpr (KSTATS) {
    if (p.stats_part != nullptr) {  // block reduce in LDS (the main loop is over), one float2 per tile
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);
      const float a = wave_sum(st_ss), b = wave_sum(st_bad);
      if (lane == 0) {
        red[2 * w] = a;
        red[2 * w + 1] = b;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        float sa = 0.f, sb = 0.f;
        for (int q = 0; q < NTHR / 64; ++q) {
          sa += red[2 * q];
          sb += red[2 * q + 1];
        }
        p.stats_part[2 * id] = sa;
        p.stats_part[2 * id + 1] = sb;
      }
    }
  }
}

// out[i] = sum over the split-K partial slices (fp32, `parts` x n) -> bf16; 8 elements per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, bf16* __restrict__ out,
                                                            int parts, int64_t n) {
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 a0 = *reinterpret_cast<const f32x4*>(part + i * 8), a1 = *reinterpret_cast<const f32x4*>(part + i * 8 + 4);
    for (int s2 = 1; s2 < parts; ++s2) {
      a0 += *reinterpret_cast<const f32x4*>(part + s2 * n + i * 8);
      a1 += *reinterpret_cast<const f32x4*>(part + s2 * n + i * 8 + 4);
    }
    const f32x8 acc = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    store8f(out + i * 8, acc);
  }
}


// C rows / columns of the split tail tiles = the sum of their s partial slices -> bf16. tbands blocks (row bands) per
// possible split tile (8 XCDs x xcu), each recomputing the kernel's plan from the device offsets; idle when unused.
__global__ __launch_bounds__(256) void tail_reduce_kernel(GemmArgs p) {
  const int band = blockIdx.x % p.tbands, slot = blockIdx.x / p.tbands;  // a row band of one tile
  const int x = slot / p.xcu, s = slot - x * p.xcu;
  const int real = grouped_real_tiles(p);
  const int q = (real + 7) / 8;
  const TailPlan tp = tail_plan(real, q, x, p.xcu, p.tmax);
  if (tp.s < 2 || s >= tp.tail) return;
  int grp, tn, m_lo, m_hi;
  if (!group_tile(p, x * q + tp.full + s, grp, tn, m_lo, m_hi)) return;
  const int rows = min(BM, m_hi - m_lo);
  const float* T = p.tpart + ((int64_t)x * kMaxSplit * p.xcu + (int64_t)s * tp.s) * BM * BN;  // the tile's slices
  const int c = (threadIdx.x & 31) * 8;
  bf16* C = reinterpret_cast<bf16*>(p.c);
  const int rb = BM / p.tbands, r_end = min(rows, (band + 1) * rb);
  for (int r = band * rb + (threadIdx.x >> 5); r < r_end; r += 8) {
    const int o = r * BN + c;
    f32x4 a0 = *reinterpret_cast<const f32x4*>(T + o), a1 = *reinterpret_cast<const f32x4*>(T + o + 4);
    for (int pt = 1; pt < tp.s; ++pt) {  // fixed order: deterministic
      a0 += *reinterpret_cast<const f32x4*>(T + (int64_t)pt * BM * BN + o);
      a1 += *reinterpret_cast<const f32x4*>(T + (int64_t)pt * BM * BN + o + 4);
    }
    const f32x8 v = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    store8f(C + (int64_t)(m_lo + r) * p.ldc + tn * BN + c, v);
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
                    int64_t G, int64_t b_gstride, const c10::optional<at::Tensor>& stats_part,
                    const c10::optional<at::Tensor>& glu) {
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
  // grouped-K: token-major operands (row = k; partial K tiles at group ends are zero-filled in LDS), or both
  // K-contiguous with every group's K range on whole 64-wide tiles (the aligned re-layout, ops.moe.pad_plan_multi)
  TORCH_CHECK(mode != kGroupK || (!ak && !bk) || (ak && bk), "gemm_mfma: grouped-K operands both token-major or both K-major");
  TORCH_CHECK(mode != kGroupM || ak, "gemm_mfma: grouped-M needs row-major (K-contiguous) rows");
  TORCH_CHECK(mode == kDense || mode == kGroupM || mode == kGroupK, "gemm_mfma: bad mode");
  for (const at::Tensor* t : {&a, &b2}) {
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "gemm_mfma: operands 16-byte aligned");
  }
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "gemm_mfma: leading strides must keep 16-B rows");
  TORCH_CHECK(out32 || (ldc % 8 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0),
              "gemm_mfma: a bf16 out needs 16-byte rows (the epilogue stores 16-B row chunks)");
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
  p.qskip = 1;
  p.chunk = 1;
  p.splitk = 1;
  const bool fused_glu = glu.has_value() && glu->defined();
  if (fused_glu) {  // out = dgu [rows, 2N] (dgate | dup), glu = gu [rows, 2N]: the SwiGLU backward in the epilogue
    TORCH_CHECK(mode == kGroupM && !out32 && !accumulate, "gemm_mfma(glu): a grouped-M bf16 store");
    TORCH_CHECK(glu->is_cuda() && glu->scalar_type() == at::kBFloat16 && glu->is_contiguous() && glu->dim() == 2 &&
                    glu->size(1) == 2 * N && out.is_contiguous() && out.sizes() == glu->sizes() && glu->size(0) >= M,
                "gemm_mfma(glu): gu and out must be contiguous bf16 [rows, 2N]");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(glu->data_ptr()) % 16 == 0, "gemm_mfma(glu): 16-byte aligned gu");
    p.glu = reinterpret_cast<const bf16*>(glu->data_ptr());
    p.glu_f = (int)N;
  }
  // narrow grouped-M problems (<= 16 column tiles: the expert down projection and input gradients) fill only ~2.2
  // rounds of 256 CUs, so a third round runs ~20 % full: split the long K in two (fp32 partials + one reduce)
  at::Tensor part;
  at::Tensor out_final = out;
  // (round 4: splitting K >= 8192 in two and K >= 24576 in three measured 3-7 % slower on the Mixtral shapes than
  // this rule: the fp32 partial traffic outweighs the fuller last round; profiles/gemm_splitk_policy_ab_r04.jsonl)
  // round 6, every grouped-M bf16 launch with K >= 4096: the tail split instead -- each XCD runs its whole rounds of
  // tiles unsplit and only its short last round's tiles as K parts (fp32 partials for those tiles alone, summed
  // by tail_reduce_kernel): +1.7 % on the Mixtral step with halves for the narrow launches alone
  // (profiles/gemm_tail_split_ab_r06.json). DLGM_GEMM_TSPLIT=0 restores the rule below
  static const int tsplit_mode = [] {  // 0 off, 1 every width, 2 narrow launches (<= 16 column tiles) only
    const char* e = std::getenv("DLGM_GEMM_TSPLIT");
    return e == nullptr ? 1 : std::atoi(e);
  }();
  at::Tensor tpart;
  // (not on the fused SwiGLU-backward launch: with the SwiGLU backward in tail_reduce_kernel that launch measured
  // 1.3 % slower on the Mixtral step, profiles/gemm_tail_split_ab_r06.json glu_tail_split)
  if (mode == kGroupM && !out32 && !fused_glu && K >= 4096 && tsplit_mode != 0 &&
      (tsplit_mode == 1 || p.tiles_n <= 16)) {
    static int cu_count[64] = {};  // per device, queried once
    int dev = 0;
    DLGM_CHECK_HIP(hipGetDevice(&dev));
    int& cus = cu_count[dev & 63];
    if (cus == 0) DLGM_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    static const int tmax = [] {  // DLGM_GEMM_TSPLIT_PARTS: most K parts per tail tile (default and cap 4)
      const char* e = std::getenv("DLGM_GEMM_TSPLIT_PARTS");
      return std::min(kMaxSplit, std::max(2, e == nullptr ? kMaxSplit : std::atoi(e)));
    }();
    static const int tbands = [] {  // DLGM_GEMM_TRED_BANDS: reduce blocks per tile (1..32, a divisor of 256)
      const char* e = std::getenv("DLGM_GEMM_TRED_BANDS");
      const int v = e == nullptr ? 8 : std::atoi(e);
      return (v >= 1 && v <= 32 && 256 % v == 0) ? v : 8;
    }();
    p.tsplit = 1;
    p.tmax = tmax;
    p.tbands = tbands;
    p.xcu = std::max(2, cus / 8);
    tpart = at::empty({8 * kMaxSplit * p.xcu, BM, BN}, out.options().dtype(at::kFloat));
    p.tpart = tpart.data_ptr<float>();
  }
  if (mode == kGroupM && !out32 && !fused_glu && !p.tsplit && out.is_contiguous() && ldc == N && p.tiles_n <= 16 &&
      K >= 16384) {
    p.splitk = 2;
    part = at::empty({p.splitk, M, N}, out.options().dtype(at::kFloat));
    p.c = part.data_ptr();
    p.ldc = N;
    p.c_sstride = M * N;
  }
  TORCH_CHECK(!(stats_part.has_value() && stats_part->defined()) || mode == kGroupK,
              "gemm_mfma: stats_part is a grouped-K epilogue");
  int64_t nblk;
  if (mode == kDense) {
    nblk = (int64_t)p.tiles_m * p.tiles_n;
  } else {
    TORCH_CHECK(offsets.has_value() && offsets->is_cuda() && offsets->scalar_type() == at::kInt &&
                    offsets->numel() == G + 1, "gemm_mfma: grouped modes need int32 offsets[G+1] on the GPU");
    p.offsets = offsets->data_ptr<int>();
    if (mode == kGroupM) {
      nblk = ((M + BM - 1) / BM + G) * p.tiles_n * p.splitk;  // M = total rows: worst-case tiles over all groups
      if (p.tsplit) nblk += 8 * (kMaxSplit - 1) * p.xcu;  // an XCD's split tail: up to (s - 1) tail more blocks
      nblk = (nblk + 7) / 8 * 8;  // whole rounds of the 8 XCDs (the balanced remap's block -> XCD mapping)
    } else {
      nblk = G * (int64_t)p.tiles_m * p.tiles_n;
      p.nreal = (int)nblk;
      if (stats_part.has_value() && stats_part->defined()) {
        TORCH_CHECK(mode == kGroupK && out32 && stats_part->is_cuda() && stats_part->scalar_type() == at::kFloat &&
                        stats_part->is_contiguous() && stats_part->numel() == 2 * nblk,
                    "gemm_mfma: stats_part must be fp32 [2 * G * tiles] for a grouped-K fp32 launch");
        p.stats_part = stats_part->data_ptr<float>();
      }
      if (p.chunk) nblk = (nblk + 8 * kChunk - 1) / (8 * kChunk) * (8 * kChunk);
    }
  }
  if (nblk == 0) return;
  const int epi = p.splitk > 1 ? kStoreF32 : !out32 ? kStoreBf16 : accumulate ? kAccF32 : kStoreF32;
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
  } else if (ak && bk) {  // K-major, tile-aligned group ranges
    launch_epi<kGroupK, true, true>(epi, grid, st, p);
  } else {  // token-major operands (checked above)
    launch_epi<kGroupK, false, false>(epi, grid, st, p);
  }
  DLGM_CHECK_HIP(hipGetLastError());
  if (p.tsplit) {
    tail_reduce_kernel<<<8 * p.xcu * p.tbands, 256, 0, st>>>(p);
    DLGM_CHECK_HIP(hipGetLastError());
  }
  if (p.splitk > 1) {
    TORCH_CHECK(out_final.is_contiguous() && out_final.size(-1) == N && (N % 8) == 0, "gemm_mfma: split-K out layout");
    const int64_t n = M * N;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n / 8 + 255) / 256, 4096));
    splitk_reduce_kernel<<<(unsigned)blocks, 256, 0, st>>>(part.data_ptr<float>(),
                                                           reinterpret_cast<bf16*>(out_final.data_ptr()),
                                                           p.splitk, n);
    DLGM_CHECK_HIP(hipGetLastError());
  }
}

// Grouped-K over segments: out[g] (+)= sum over s of a[s][rows of g in s]^T @ b[s][rows of g in s], with
// a[s] [R_s, M] and b[s] [R_s, N] token-major (row-major) bf16 and offsets [nseg, G + 1] int32 on the device
// (offsets[s] splits segment s's rows by group). One launch reduces each group over all its rows of every
// segment -- e.g. an expert's weight gradient over the step's micro-batches -- without concatenating them.
//
// kmajor: the operands are given transposed, a[s] [M, P] and b[s] [N, P] row-major (the reduction dim contiguous,
// one P for all segments), with every group's range [offsets[s][g], offsets[s][g + 1]) a whole number of 64-wide
// K tiles (zero padded: ops.moe.pad_plan + the row-remapped transpose). Both images are then K-contiguous --
// the layout the kernel runs fastest (ds_read_b128 fragments, no transposed LDS reads).
void dlgm_gemm_mfma_seg(at::Tensor out, const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b,
                        const at::Tensor& offsets, bool accumulate, bool kmajor) {
  const int nseg = (int)a.size();
  TORCH_CHECK(nseg >= 1 && nseg <= kMaxSeg && (int)b.size() == nseg, "gemm_mfma_seg: 1..8 segments, a/b paired");
  TORCH_CHECK(out.is_cuda() && out.dim() == 3 && out.is_contiguous() && out.scalar_type() == at::kFloat,
              "gemm_mfma_seg: out [G, M, N] contiguous fp32");
  const int64_t G = out.size(0), M = out.size(1), N = out.size(2);
  TORCH_CHECK(M % BM == 0 && N % BN == 0, "gemm_mfma_seg: M and N must be multiples of 256");
  TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.is_contiguous() &&
                  offsets.dim() == 2 && offsets.size(0) == nseg && offsets.size(1) == G + 1,
              "gemm_mfma_seg: offsets [nseg, G + 1] int32 on the GPU");
  GemmArgs p{};
  for (int s = 0; s < nseg; ++s) {
    const at::Tensor& x = a[s];
    const at::Tensor& y = b[s];
    TORCH_CHECK(x.is_cuda() && y.is_cuda() && x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16,
                "gemm_mfma_seg: bf16 GPU operands");
    if (kmajor) {
      TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && x.size(0) == M && y.size(0) == N && x.size(1) == y.size(1) &&
                      x.stride(1) == 1 && y.stride(1) == 1,
                  "gemm_mfma_seg(kmajor): a[s] [M, P] and b[s] [N, P] row-major");
    } else {
      TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && x.size(1) == M && y.size(1) == N && x.size(0) == y.size(0) &&
                      x.stride(1) == 1 && y.stride(1) == 1,
                  "gemm_mfma_seg: a[s] [R_s, M] and b[s] [R_s, N] row-major");
    }
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0,
                "gemm_mfma_seg: operands 16-byte aligned");
    if (s == 0) {
      p.lda = x.stride(0);
      p.ldb = y.stride(0);
    }
    TORCH_CHECK(x.stride(0) == p.lda && y.stride(0) == p.ldb && p.lda % 8 == 0 && p.ldb % 8 == 0,
                "gemm_mfma_seg: one row stride per operand across segments, 16-byte rows");
    p.a_seg[s] = reinterpret_cast<const bf16*>(x.data_ptr());
    p.b_seg[s] = reinterpret_cast<const bf16*>(y.data_ptr());
  }
  p.a = p.a_seg[0];
  p.b = p.b_seg[0];
  p.c = out.data_ptr();
  p.ldc = N;
  p.nseg = nseg;
  p.offsets = offsets.data_ptr<int>();
  p.M = (int)M;
  p.N = (int)N;
  p.K = 0;
  p.G = (int)G;
  p.mode = kGroupKSeg;
  p.c_gstride = out.stride(0);
  p.tiles_n = (int)(N / BN);
  p.tiles_m = (int)(M / BM);
  int64_t nblk = G * (int64_t)p.tiles_m * p.tiles_n;
  if (nblk == 0) return;
  p.nreal = (int)nblk;
  p.chunk = 1;
  if (p.chunk) nblk = (nblk + 8 * kChunk - 1) / (8 * kChunk) * (8 * kChunk);
  if (kmajor)
    launch_epi<kGroupKSeg, true, true>(accumulate ? kAccF32 : kStoreF32, dim3((unsigned)nblk),
                                       c10::hip::getCurrentHIPStream(), p);
  else
    launch_epi<kGroupKSeg, false, false>(accumulate ? kAccF32 : kStoreF32, dim3((unsigned)nblk),
                                         c10::hip::getCurrentHIPStream(), p);
  DLGM_CHECK_HIP(hipGetLastError());
}
