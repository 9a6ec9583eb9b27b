// Device-driven xGMI mesh transport (SURVEY.md §5.8 plan item 3, §2.7 C1/C3/C6): a symmetric heap per rank,
// exported with HIP IPC and mapped by every peer, plus the kernels that move data through it and the flags that
// order it -- no host synchronisation, no library, capturable in a HIP graph.
//
// Shadow mode (state word kStShadow = 1; one rank of a world-W job alone on one GPU, every peer address = this
// rank's heap): a producer writes "peer" t's flag / slot as if it were rank t (so every wait completes and every
// slot is written once), the EP tables describe this rank receiving its own rows from every source -- true-size,
// deterministic traffic for the per-rank timing and stream-ordering rehearsals of the shadow rank.
//
// Heap (one allocation per rank, the same layout on every rank; offsets chosen by parallel/xgmi_mesh.py):
//   [0, kFlagBytes)      u64 flags[kind][channel][source rank], written by the SOURCE rank into this rank's heap
//   regions              ZeRO bf16 parameter shard (pulled by peers), reduce-scatter slots, EP dispatch / combine
//                        slots; a channel's region holds S slots, used round-robin by epoch (slot = epoch % S)
// State (ordinary device memory, int64 words, never shared): channel epochs, the parameter version, the
// last-block counters of the multi-block kernels, a sticky error word and the EP overflow word.
//
// Flag kinds:
//   CNT   EP routing counts of epoch e are in this rank's slot header (from rank src)
//   DATA  all of rank src's rows / chunks of epoch e are in this rank's slot
//   ACK   rank src has consumed epoch e of the channel: its slot e % S may be rewritten by this rank
//   VER   rank src's parameter shard is at version v (published after the optimizer wrote it)
//   RDONE rank src finished every read of version v of the peers' shards (the optimizer may overwrite them)
//
// Memory model (MI355X, gfx950; why a flag makes the data it guards visible):
// * The heap is allocated uncached (hipExtMallocWithFlags(hipDeviceMallocUncached); parallel/xgmi_mesh.py falls
//   back to fine-grained, then plain, memory if the driver refuses IPC export, and records which). Uncached
//   device memory is mapped MTYPE UC on the owner and on every peer that imports it, so neither the writer's nor
//   the owner's L2 ever holds a line of it: the owner cannot read a stale line of its own buffer, the question the
//   plain coarse-grained buffer of round 3 left open.
// * A producer makes its data visible at SYSTEM scope before it signals: every storing wave waits for its
//   stores (s_waitcnt vmcnt(0)), the workgroup joins a barrier, one lane executes a system-scope release fence
//   (it also writes back any dirty L2 lines, covering the fallback heaps) followed by an explicit vmcnt(0) wait
//   (the compiler drops the one after the write-back when the scoreboard looks empty: MI355X_MICROARCH.md,
//   "Compiler hazard") and then an agent-scope atomic add on a per-launch counter; the LAST workgroup to arrive
//   (it saw count == grid - 1) executes a system-scope acquire + release and stores the flag with a
//   system-scope atomic store (global_store ... sc0 sc1: write-through to the owner's memory over xGMI).
// * A consumer polls its OWN flags with system-scope relaxed atomic loads (they bypass L1 and L2), then executes a
//   system-scope acquire fence; the kernels that read the data are later launches on the same stream.
// * Every wait is bounded: past `timeout` ticks of the 100 MHz wall clock the waiting kernel records an error in
//   the state word and returns, so a dead peer ends in an error the host reads (XgmiMesh.check), never a hang.
// * Waiters are single-workgroup kernels and the multi-block kernels never wait, so ranks that share one GPU
//   (the tests) cannot starve each other's producers of compute units.
//
// All stores are vector-memory stores (flags: 8-byte atomic stores; data: 16-byte vectors).
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

constexpr int kMaxRanks = 64;
constexpr int kMaxCh = 8;
enum Kind { kCnt = 0, kData = 1, kAck = 2, kVer = 3, kRdone = 4, kKinds = 5 };
constexpr int64_t kFlagBytes = (int64_t)kKinds * kMaxCh * kMaxRanks * 8;
// state words
constexpr int kStEpoch = 0;    // [kMaxCh] transfers started per channel
constexpr int kStVer = 16;     // parameter version
constexpr int kStErr = 17;     // sticky: 1 = a wait timed out
constexpr int kStOvf = 18;     // sticky: 1 = an EP dispatch overflowed the receive capacity
constexpr int kStShadow = 19;  // 1 = shadow rank (parallel/comm.py ShadowComm): every "peer" is this rank's heap
constexpr int kStPushCtr = 32; // [kMaxCh] last-block counters of the push kernels
constexpr int kStCopyCtr = 48; // [kMaxCh] last-block counters of the consuming kernels
constexpr int kStateWords = 64;
constexpr int kThreads = 256;

__device__ __forceinline__ uint64_t* flag_at(int64_t heap, int kind, int ch, int src) {
  return reinterpret_cast<uint64_t*>(heap) + ((int64_t)(kind * kMaxCh + ch) * kMaxRanks + src);
}

__device__ __forceinline__ void release_system() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void acquire_system() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

__device__ __forceinline__ void store_flag(uint64_t* f, uint64_t v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t load_flag(uint64_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void set_word(int64_t* st, int idx, int64_t v) {
  __hip_atomic_store(st + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int64_t get_word(const int64_t* st, int idx) {
  return __hip_atomic_load(const_cast<int64_t*>(st) + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Poll until *f >= target (as signed: targets <= 0 pass at once); false after `timeout` wall-clock ticks, and at
// once when this rank already recorded a timeout (the sticky error word): after one dead-peer timeout every later
// wait of the step returns immediately and the host raises at the step boundary (XgmiMesh.check) instead of
// spinning `timeout` once per collective.
__device__ bool wait_ge(uint64_t* f, int64_t target, int64_t timeout, const int64_t* st) {
  if (target <= 0) return true;
  const uint64_t t0 = wall_clock64();
  while ((int64_t)load_flag(f) < target) {
    if (get_word(st, kStErr)) return false;
    __builtin_amdgcn_s_sleep(2);
    if ((int64_t)(wall_clock64() - t0) > timeout) return false;
  }
  return true;
}

// End of a multi-block producer / consumer: every wave drains its stores, the last workgroup to arrive stores
// flags[kind][ch][me] = value into every rank's heap. The counter resets itself for the next launch.
__device__ void last_block_signal(int64_t* st, int ctr, const int64_t* peers, int W, int me, int kind, int ch,
                                  int64_t value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    release_system();
    const unsigned nb = gridDim.x * gridDim.y;
    const int64_t old = __hip_atomic_fetch_add(st + ctr, (int64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (old == (int64_t)nb - 1);
    if (last) {
      acquire_system();
      set_word(st, ctr, 0);
      release_system();
    }
  }
  __syncthreads();
  const int who = get_word(st, kStShadow) ? (int)threadIdx.x : me;
  if (last && (int)threadIdx.x < W) store_flag(flag_at(peers[threadIdx.x], kind, ch, who), (uint64_t)value);
}

// ------------------------------------------------------------------------------------------------ sync
// One workgroup of 64 lanes (lane t <-> rank t):
//   inc >= 0        state[inc] += 1 first
//   store_kind >= 0 flags[store_kind][ch][me] = state[val] in every rank's heap (after a system release)
//   wait_kind >= 0  wait until own flags[wait_kind][ch][t] >= state[val] - lag for every rank t, then acquire
__global__ __launch_bounds__(64) void mesh_sync_kernel(int64_t* st, const int64_t* peers, int W, int me, int ch,
                                                       int inc, int val, int store_kind, int wait_kind, int64_t lag,
                                                       int64_t timeout) {
  const int t = threadIdx.x;
  if (inc >= 0 && t == 0) set_word(st, inc, get_word(st, inc) + 1);
  __syncthreads();
  const int64_t v = get_word(st, val);
  if (store_kind >= 0) {
    release_system();
    if (t < W) store_flag(flag_at(peers[t], store_kind, ch, get_word(st, kStShadow) ? t : me), (uint64_t)v);
  }
  if (wait_kind >= 0) {
    bool ok = true;
    if (t < W) ok = wait_ge(flag_at(peers[me], wait_kind, ch, t), v - lag, timeout, st);
    if (!ok) set_word(st, kStErr, 1);
    __syncthreads();
    acquire_system();
  }
}

// ------------------------------------------------------------------------------------------------ ZeRO
// all-gather as a PULL: rank r's shard is read from rank r's heap (src_off) into out[r * nbytes ...]
// (blockIdx.y = r, its own shard included). Version flags order it against the optimizer (mesh_sync).
__global__ __launch_bounds__(kThreads) void mesh_pull_kernel(const int64_t* peers, int64_t src_off, int64_t n16,
                                                             uint4* __restrict__ out) {
  const uint4* src = reinterpret_cast<const uint4*>(peers[blockIdx.y] + src_off);
  uint4* dst = out + (int64_t)blockIdx.y * n16;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  // four 16-byte reads in flight per lane: remote reads are latency-bound
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

__device__ __forceinline__ bf16x8 to_bf16x8(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  const f32x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_convertvector(v, bf16x8);
}

__device__ __forceinline__ bf16x8 to_bf16x8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// reduce-scatter, push half: chunk p of x ([W * n], fp32 or bf16) -> slot `me` of rank p's RS region as TS (bf16: the
// per-micro-batch scratch path; fp32: the once-per-step reduce of the fp32 local accumulator, no rounding before the
// sum) (blockIdx.y = p). n % 8 == 0.
__device__ __forceinline__ void store8(bf16* dst, const float* src) {
  *reinterpret_cast<bf16x8*>(dst) = to_bf16x8(src);
}
__device__ __forceinline__ void store8(bf16* dst, const bf16* src) {
  *reinterpret_cast<bf16x8*>(dst) = *reinterpret_cast<const bf16x8*>(src);
}
__device__ __forceinline__ void store8(float* dst, const float* src) {
  *reinterpret_cast<f32x4*>(dst) = *reinterpret_cast<const f32x4*>(src);
  *reinterpret_cast<f32x4*>(dst + 4) = *reinterpret_cast<const f32x4*>(src + 4);
}
__device__ __forceinline__ f32x8 load8f(const bf16* p) {
  return __builtin_convertvector(*reinterpret_cast<const bf16x8*>(p), f32x8);
}
__device__ __forceinline__ f32x8 load8f(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
  return f32x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <typename TI, typename TS>
__global__ __launch_bounds__(kThreads) void mesh_rs_push_kernel(const TI* __restrict__ x, int64_t n,
                                                                const int64_t* peers, int64_t region_off,
                                                                int64_t slot_bytes, int64_t rank_stride, int S,
                                                                int64_t* st, int ch, int me, int W) {
  const int p = blockIdx.y;
  const int64_t e = get_word(st, kStEpoch + ch);
  const int row = get_word(st, kStShadow) ? p : me;
  TS* dst = reinterpret_cast<TS*>(peers[p] + region_off + (e % S) * slot_bytes + row * rank_stride);
  const TI* src = x + (int64_t)p * n;
  const int64_t n8 = n / 8, stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n8; i += stride) store8(dst + i * 8, src + i * 8);
  last_block_signal(st, kStPushCtr + ch, peers, W, me, kData, ch, e);
}

// reduce-scatter, reduce half: out = [out +] (sum over ranks s = 0..W-1, in rank order, in fp32, of slot s) * scale
// (unfused multiply and add: bit-reproducible against the same expression in PyTorch). Then ACK every rank.
// TS: the slot element type the push wrote.
template <typename TO, typename TS>
__global__ __launch_bounds__(kThreads) void mesh_rs_reduce_kernel(TO* __restrict__ out, int64_t n, float scale,
                                                                  int accumulate, const int64_t* peers,
                                                                  int64_t region_off, int64_t slot_bytes,
                                                                  int64_t rank_stride, int S, int64_t* st, int ch,
                                                                  int me, int W) {
  const int64_t e = get_word(st, kStEpoch + ch);
  const char* base = reinterpret_cast<const char*>(peers[me] + region_off + (e % S) * slot_bytes);
  const int64_t n8 = n / 8, stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n8; i += stride) {
    constexpr int64_t B8 = 8 * sizeof(TS);  // bytes of 8 slot elements
    f32x8 acc = load8f(reinterpret_cast<const TS*>(base + i * B8));
    for (int s = 1; s < W; ++s) {
      const f32x8 v = load8f(reinterpret_cast<const TS*>(base + s * rank_stride + i * B8));
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __fadd_rn(acc[k], v[k]);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __fmul_rn(acc[k], scale);
    if constexpr (sizeof(TO) == 4) {
      float* o = reinterpret_cast<float*>(out) + i * 8;
      if (accumulate) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(o), b = *reinterpret_cast<const f32x4*>(o + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[k] = __fadd_rn(a[k], acc[k]);
          acc[k + 4] = __fadd_rn(b[k], acc[k + 4]);
        }
      }
      *reinterpret_cast<f32x4*>(o) = f32x4{acc[0], acc[1], acc[2], acc[3]};
      *reinterpret_cast<f32x4*>(o + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
    } else {
      bf16* o = reinterpret_cast<bf16*>(out) + i * 8;
      if (accumulate) {
        const f32x8 a = __builtin_convertvector(*reinterpret_cast<const bf16x8*>(o), f32x8);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = __fadd_rn(a[k], acc[k]);
      }
      *reinterpret_cast<bf16x8*>(o) = __builtin_convertvector(acc, bf16x8);
    }
  }
  last_block_signal(st, kStCopyCtr + ch, peers, W, me, kAck, ch, e);
}

// ------------------------------------------------------------------------------------------------ EP
// Segment table of a row transfer (int32, built on the device by mesh_ep_plan_kernel): the virtual row space
// [0, vstart[nseg]) is split into segments; virtual row v of segment k goes to row dst_row[k] + (v - vstart[k])
// of rank dst_rank[k]'s slot and comes from source row src[k] + (v - vstart[k]) when v - vstart[k] < valid[k],
// else it is a zero row (an overflow row the expert owner never received).
struct SegTab {
  const int* vstart;
  const int* src;
  const int* valid;
  const int* dst_rank;
  const int* dst_row;
  int nseg;
};

__device__ __forceinline__ int find_seg(const int* vstart, int nseg, int v) {
  int lo = 0, hi = nseg;  // largest k with vstart[k] <= v
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (vstart[mid] <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// One wave per virtual row, 16-byte vectors (row_vecs per row). hdr_bytes: the slot's header before its rows.
__global__ __launch_bounds__(kThreads) void mesh_push_rows_kernel(const uint4* __restrict__ x, int64_t row_vecs,
                                                                  SegTab tab, const int64_t* peers,
                                                                  int64_t region_off, int64_t slot_bytes,
                                                                  int64_t hdr_bytes, int S, int64_t* st, int ch,
                                                                  int me, int W) {
  const int64_t e = get_word(st, kStEpoch + ch);
  const int total = tab.vstart[tab.nseg];
  const int lane = threadIdx.x & 63;
  const int waves = gridDim.x * (kThreads / 64);
  for (int v = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); v < total; v += waves) {
    const int k = find_seg(tab.vstart, tab.nseg, v);
    const int r = v - tab.vstart[k];
    uint4* dst = reinterpret_cast<uint4*>(peers[tab.dst_rank[k]] + region_off + (e % S) * slot_bytes + hdr_bytes) +
                 (int64_t)(tab.dst_row[k] + r) * row_vecs;
    if (r < tab.valid[k]) {
      const uint4* src = x + (int64_t)(tab.src[k] + r) * row_vecs;
      for (int64_t c = lane; c < row_vecs; c += 64) dst[c] = src[c];
    } else {
      for (int64_t c = lane; c < row_vecs; c += 64) dst[c] = make_uint4(0u, 0u, 0u, 0u);
    }
  }
  last_block_signal(st, kStPushCtr + ch, peers, W, me, kData, ch, e);
}

// Copy rows [0, min(max_rows, *nrows)) of this rank's slot into out (nrows == nullptr: max_rows), then ACK.
__global__ __launch_bounds__(kThreads) void mesh_copy_rows_kernel(uint4* __restrict__ out, int64_t row_vecs,
                                                                  int64_t max_rows, const int* nrows,
                                                                  const int64_t* peers, int64_t region_off,
                                                                  int64_t slot_bytes, int64_t hdr_bytes, int S,
                                                                  int64_t* st, int ch, int me, int W) {
  const int64_t e = get_word(st, kStEpoch + ch);
  const uint4* src = reinterpret_cast<const uint4*>(peers[me] + region_off + (e % S) * slot_bytes + hdr_bytes);
  const int64_t rows = nrows != nullptr ? min(max_rows, (int64_t)nrows[0]) : max_rows;
  const int64_t n16 = rows * row_vecs, stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  for (; i + stride < n16; i += 2 * stride) {
    const uint4 a = src[i], b = src[i + stride];
    out[i] = a;
    out[i + stride] = b;
  }
  if (i < n16) out[i] = src[i];
  last_block_signal(st, kStCopyCtr + ch, peers, W, me, kAck, ch, e);
}

// Table layout (int32 offsets into the plan tensor), shared by host and device.
struct PlanLayout {
  int total, ovf, total_full;  // [0], [1], [2]
  int loff;                    // local expert offsets [El + 1]
  int d_vs, d_src, d_val, d_rank, d_row;  // dispatch segments (one per global expert, E)
  int c_vs, c_src, c_val, c_rank, c_row;  // combine segments (local expert j major, source rank s minor: El * W)
  int words;
};

PlanLayout plan_layout(int W, int E) {
  const int El = E / W, nc = El * W;
  PlanLayout L{};
  L.total = 0;
  L.ovf = 1;
  L.total_full = 2;
  int o = 4;
  L.loff = o;
  o += El + 1;
  L.d_vs = o; o += E + 1;
  L.d_src = o; o += E;
  L.d_val = o; o += E;
  L.d_rank = o; o += E;
  L.d_row = o; o += E;
  L.c_vs = o; o += nc + 1;
  L.c_src = o; o += nc;
  L.c_val = o; o += nc;
  L.c_rank = o; o += nc;
  L.c_row = o; o += nc;
  L.words = o;
  return L;
}

constexpr int kMaxPlan = 4096;  // W * E

// Routing exchange + transfer tables of one EP dispatch (single workgroup): opens epoch e of channel ch (waits
// until every rank released slot e % S), writes this rank's per-expert counts into every rank's slot header,
// signals CNT, waits for every rank's counts, and builds from the [W, E] count matrix (identical on every rank)
// the dispatch / combine segment tables, the local expert offsets and the overflow flag. Receive capacity: C rows.
__global__ __launch_bounds__(kThreads) void mesh_ep_plan_kernel(const int* __restrict__ offsets, int* __restrict__ plan,
                                                                PlanLayout L, int W, int E, int C,
                                                                const int64_t* peers, int64_t region_off,
                                                                int64_t slot_bytes, int S, int64_t* st, int ch,
                                                                int me, int64_t timeout) {
  __shared__ int M[kMaxPlan];
  __shared__ int64_t e_sh;
  const int t = threadIdx.x;
  const int El = E / W;
  const bool shadow = get_word(st, kStShadow) != 0;
  if (t == 0) {
    const int64_t e = get_word(st, kStEpoch + ch) + 1;
    set_word(st, kStEpoch + ch, e);
    e_sh = e;
  }
  __syncthreads();
  const int64_t e = e_sh;
  bool ok = true;
  if (t < W) ok = wait_ge(flag_at(peers[me], kAck, ch, t), e - S, timeout, st);
  if (!ok) set_word(st, kStErr, 1);
  __syncthreads();
  for (int i = t; i < W * E; i += kThreads) {
    const int p = i / E, x = i - p * E;
    int* hdr = reinterpret_cast<int*>(peers[p] + region_off + (e % S) * slot_bytes);
    hdr[(shadow ? p : me) * E + x] = offsets[x + 1] - offsets[x];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  release_system();
  if (t < W) store_flag(flag_at(peers[t], kCnt, ch, shadow ? t : me), (uint64_t)e);
  ok = true;
  if (t < W) ok = wait_ge(flag_at(peers[me], kCnt, ch, t), e, timeout, st);
  if (!ok) set_word(st, kStErr, 1);
  __syncthreads();
  acquire_system();
  const int* own = reinterpret_cast<const int*>(peers[me] + region_off + (e % S) * slot_bytes);
  for (int i = t; i < W * E; i += kThreads) M[i] = own[i];
  __syncthreads();
  if (t != 0) return;
  // position of block (source s, local expert j) in owner p's receive buffer: experts major, sources minor
  auto pos = [&](int p, int s, int j) {
    int v = 0;
    for (int jj = 0; jj < j; ++jj)
      for (int ss = 0; ss < W; ++ss) v += M[ss * E + p * El + jj];
    for (int ss = 0; ss < s; ++ss) v += M[ss * E + p * El + j];
    return v;
  };
  auto clampv = [&](int at, int n) { return max(0, min(n, C - at)); };
  int any_ovf = 0, total_me = 0;
  for (int p = 0; p < W; ++p) {
    int tot = 0;
    for (int s = 0; s < W; ++s)
      for (int j = 0; j < El; ++j) tot += M[s * E + p * El + j];
    if (tot > C) any_ovf = 1;
    if (p == me) total_me = tot;
  }
  plan[L.total] = min(total_me, C);
  plan[L.ovf] = any_ovf;
  plan[L.total_full] = total_me;
  if (any_ovf) set_word(st, kStOvf, 1);
  for (int j = 0; j <= El; ++j) plan[L.loff + j] = min(j < El ? pos(me, 0, j) : total_me, C);
  int vs = 0, srow = 0;
  if (shadow) {
    // this rank receives its own rows of each local expert j from every source s (W x El = E segments), and the
    // combine sends back only its own block: every written row has one writer, the traffic is true size
    auto own = [&](int x) { int o = 0; for (int xx = 0; xx < x; ++xx) o += M[me * E + xx]; return o; };
    for (int j = 0; j < El; ++j)
      for (int s2 = 0; s2 < W; ++s2) {
        const int k = j * W + s2, x = me * El + j, n = M[me * E + x], at = pos(me, s2, j), val = clampv(at, n);
        plan[L.d_vs + k] = vs;
        plan[L.d_src + k] = own(x);
        plan[L.d_val + k] = val;
        plan[L.d_rank + k] = me;
        plan[L.d_row + k] = at;
        vs += val;
      }
    plan[L.d_vs + E] = vs;
    vs = 0;
    for (int j = 0; j < El; ++j)
      for (int s2 = 0; s2 < W; ++s2) {
        const int k = j * W + s2, x = me * El + j, n = s2 == me ? M[me * E + x] : 0, at = pos(me, s2, j);
        plan[L.c_vs + k] = vs;
        plan[L.c_src + k] = at;
        plan[L.c_val + k] = clampv(at, n);
        plan[L.c_rank + k] = me;
        plan[L.c_row + k] = own(x);
        vs += n;
      }
    plan[L.c_vs + El * W] = vs;
    return;
  }
  // dispatch: one segment per global expert x, this rank's rows offsets[x] .. to owner x / El
  for (int x = 0; x < E; ++x) {
    const int p = x / El, j = x - p * El, n = M[me * E + x];
    const int at = pos(p, me, j), val = clampv(at, n);
    plan[L.d_vs + x] = vs;
    plan[L.d_src + x] = srow;
    plan[L.d_val + x] = val;
    plan[L.d_rank + x] = p;
    plan[L.d_row + x] = at;
    vs += val;
    srow += n;
  }
  plan[L.d_vs + E] = vs;
  // combine: segment (j, s): the rows source s sent for local expert j go back to s's expert-sorted order; rows
  // dropped by the capacity come back as zeros
  vs = 0;
  for (int j = 0; j < El; ++j) {
    const int x = me * El + j;
    for (int s = 0; s < W; ++s) {
      const int k = j * W + s, n = M[s * E + x];
      const int at = pos(me, s, j);
      int drow = 0;
      for (int xx = 0; xx < x; ++xx) drow += M[s * E + xx];
      plan[L.c_vs + k] = vs;
      plan[L.c_src + k] = at;
      plan[L.c_val + k] = clampv(at, n);
      plan[L.c_rank + k] = s;
      plan[L.c_row + k] = drow;
      vs += n;
    }
  }
  plan[L.c_vs + El * W] = vs;
}

void ipc_free(void* p) { (void)hipFree(p); }

const int64_t* peers_ptr(const at::Tensor& peers, int W) {
  TORCH_CHECK(peers.is_cuda() && peers.scalar_type() == at::kLong && peers.dim() == 1 && peers.numel() == W &&
                  peers.is_contiguous(),
              "mesh: peers must be an int64 GPU vector of the W heap addresses");
  return peers.data_ptr<int64_t>();
}

int64_t* state_ptr(const at::Tensor& st) {
  TORCH_CHECK(st.is_cuda() && st.scalar_type() == at::kLong && st.numel() >= kStateWords && st.is_contiguous(),
              "mesh: bad state tensor");
  return st.data_ptr<int64_t>();
}

void check_geom(int W, int me, int ch) {
  TORCH_CHECK(W >= 1 && W <= kMaxRanks && me >= 0 && me < W, "mesh: 1..64 ranks");
  TORCH_CHECK(ch >= 0 && ch < kMaxCh, "mesh: channel out of range");
}

unsigned grid_for(int64_t n16, int64_t cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n16 + kThreads - 1) / kThreads, cap));
}

}  // namespace

// ---------------------------------------------------------------------------------------------------- host API
// uint8 tensor of `nbytes` device memory in its own allocation. mode 0: uncached, 1: fine-grained, 2: hipMalloc.
at::Tensor dlgm_ipc_alloc(int64_t nbytes, int64_t mode) {
  TORCH_CHECK(nbytes > 0 && nbytes % 16 == 0, "ipc_alloc: a positive multiple of 16 bytes");
  void* p = nullptr;
  if (mode == 0) DLGM_CHECK_HIP(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocUncached));
  else if (mode == 1) DLGM_CHECK_HIP(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocFinegrained));
  else DLGM_CHECK_HIP(hipMalloc(&p, (size_t)nbytes));
  DLGM_CHECK_HIP(hipMemset(p, 0, (size_t)nbytes));
  DLGM_CHECK_HIP(hipDeviceSynchronize());
  const int dev = c10::hip::current_device();
  return torch::from_blob(p, {nbytes}, ipc_free,
                          torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, dev));
}

at::Tensor dlgm_ipc_handle(const at::Tensor& buf) {
  TORCH_CHECK(buf.is_cuda() && buf.scalar_type() == at::kByte && buf.is_contiguous(), "ipc_handle: uint8 GPU buffer");
  hipIpcMemHandle_t h;
  DLGM_CHECK_HIP(hipIpcGetMemHandle(&h, buf.data_ptr()));
  auto out = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, sizeof(h));
  return out;
}

int64_t dlgm_ipc_open(const at::Tensor& handle) {
  TORCH_CHECK(!handle.is_cuda() && handle.scalar_type() == at::kByte && handle.numel() == (int64_t)sizeof(hipIpcMemHandle_t),
              "ipc_open: a 64-byte CPU handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  void* p = nullptr;
  DLGM_CHECK_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<int64_t>(p);
}

void dlgm_ipc_close(int64_t ptr) { DLGM_CHECK_HIP(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr))); }

int64_t dlgm_mesh_flag_bytes() { return kFlagBytes; }

int64_t dlgm_mesh_state_words() { return kStateWords; }

void dlgm_mesh_sync(at::Tensor state, const at::Tensor& peers, int64_t me, int64_t ch, int64_t inc, int64_t val,
                    int64_t store_kind, int64_t wait_kind, int64_t lag, int64_t timeout) {
  const int W = (int)peers.numel();
  check_geom(W, (int)me, (int)ch);
  TORCH_CHECK(val >= 0 && val < kStateWords && inc < kStateWords, "mesh_sync: bad state index");
  TORCH_CHECK(store_kind < kKinds && wait_kind < kKinds, "mesh_sync: bad flag kind");
  mesh_sync_kernel<<<1, 64, 0, c10::hip::getCurrentHIPStream()>>>(state_ptr(state), peers_ptr(peers, W), W, (int)me,
                                                                 (int)ch, (int)inc, (int)val, (int)store_kind,
                                                                 (int)wait_kind, lag, timeout);
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_mesh_pull(at::Tensor out, const at::Tensor& peers, int64_t src_off, int64_t heap_bytes) {
  const int W = (int)peers.numel();
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "mesh_pull: contiguous 16-byte aligned GPU output");
  const int64_t nbytes = out.numel() * out.element_size();
  TORCH_CHECK(nbytes % (16 * W) == 0, "mesh_pull: output bytes must be a multiple of 16 * W");
  const int64_t per = nbytes / W;
  TORCH_CHECK(src_off >= 0 && src_off % 16 == 0 && src_off + per <= heap_bytes, "mesh_pull: read past the heap");
  if (per == 0) return;
  const unsigned gx = grid_for(per / 16, std::max(1, 1024 / W));
  mesh_pull_kernel<<<dim3(gx, W), kThreads, 0, c10::hip::getCurrentHIPStream()>>>(
      peers_ptr(peers, W), src_off, per / 16, reinterpret_cast<uint4*>(out.data_ptr()));
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_mesh_rs_push(const at::Tensor& x, const at::Tensor& peers, at::Tensor state, int64_t me, int64_t ch,
                       int64_t region_off, int64_t slot_bytes, int64_t rank_stride, int64_t slots,
                       int64_t heap_bytes, bool fp32_slots) {
  const int W = (int)peers.numel();
  check_geom(W, (int)me, (int)ch);
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && (x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16),
              "mesh_rs_push: contiguous fp32 / bf16 GPU input");
  TORCH_CHECK(x.numel() % (8 * W) == 0, "mesh_rs_push: numel must be a multiple of 8 * W");
  const int64_t n = x.numel() / W;
  TORCH_CHECK(!fp32_slots || x.scalar_type() == at::kFloat, "mesh_rs_push: fp32 slots take an fp32 input");
  TORCH_CHECK(n * (fp32_slots ? 4 : 2) <= rank_stride && rank_stride % 16 == 0 && (int64_t)W * rank_stride <= slot_bytes &&
                  region_off % 16 == 0 && region_off + slots * slot_bytes <= heap_bytes && slots >= 1,
              "mesh_rs_push: chunk does not fit the reduce-scatter slot");
  const unsigned gx = grid_for(n / 8, std::max(1, 1024 / W));
  dim3 grid(gx, W);
  auto s = c10::hip::getCurrentHIPStream();
  if (fp32_slots)
    mesh_rs_push_kernel<float, float><<<grid, kThreads, 0, s>>>(x.data_ptr<float>(), n, peers_ptr(peers, W),
                                                                region_off, slot_bytes, rank_stride, (int)slots,
                                                                state_ptr(state), (int)ch, (int)me, W);
  else if (x.scalar_type() == at::kFloat)
    mesh_rs_push_kernel<float, bf16><<<grid, kThreads, 0, s>>>(x.data_ptr<float>(), n, peers_ptr(peers, W), region_off,
                                                               slot_bytes, rank_stride, (int)slots, state_ptr(state),
                                                               (int)ch, (int)me, W);
  else
    mesh_rs_push_kernel<bf16, bf16><<<grid, kThreads, 0, s>>>(reinterpret_cast<const bf16*>(x.data_ptr()), n,
                                                        peers_ptr(peers, W), region_off, slot_bytes, rank_stride,
                                                        (int)slots, state_ptr(state), (int)ch, (int)me, W);
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_mesh_rs_reduce(at::Tensor out, double scale, bool accumulate, const at::Tensor& peers, at::Tensor state,
                         int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes, int64_t rank_stride,
                         int64_t slots, int64_t heap_bytes, bool fp32_slots) {
  const int W = (int)peers.numel();
  check_geom(W, (int)me, (int)ch);
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() &&
                  (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16) &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 32 == 0,
              "mesh_rs_reduce: contiguous 32-byte aligned fp32 / bf16 GPU output");
  const int64_t n = out.numel();
  TORCH_CHECK(n % 8 == 0 && n * (fp32_slots ? 4 : 2) <= rank_stride && (int64_t)W * rank_stride <= slot_bytes &&
                  region_off + slots * slot_bytes <= heap_bytes && slots >= 1,
              "mesh_rs_reduce: shard does not fit the reduce-scatter slot");
  const unsigned gx = grid_for(n / 8, 1024);
  auto s = c10::hip::getCurrentHIPStream();
  auto go = [&](auto to, auto ts) {
    using TO = decltype(to);
    using TS = decltype(ts);
    mesh_rs_reduce_kernel<TO, TS><<<gx, kThreads, 0, s>>>(reinterpret_cast<TO*>(out.data_ptr()), n, (float)scale,
                                                          accumulate ? 1 : 0, peers_ptr(peers, W), region_off,
                                                          slot_bytes, rank_stride, (int)slots, state_ptr(state),
                                                          (int)ch, (int)me, W);
  };
  if (out.scalar_type() == at::kFloat) {
    if (fp32_slots) go(float{}, float{});
    else go(float{}, bf16{});
  } else {
    TORCH_CHECK(!fp32_slots, "mesh_rs_reduce: fp32 slots reduce into an fp32 output");
    go(bf16{}, bf16{});
  }
  DLGM_CHECK_HIP(hipGetLastError());
}

std::vector<int64_t> dlgm_mesh_plan_layout(int64_t W, int64_t E) {
  TORCH_CHECK(W >= 1 && W <= kMaxRanks && E % W == 0 && W * E <= kMaxPlan, "mesh: bad EP geometry");
  const PlanLayout L = plan_layout((int)W, (int)E);
  return {L.total, L.ovf, L.total_full, L.loff, L.d_vs, L.d_src, L.d_val, L.d_rank, L.d_row,
          L.c_vs, L.c_src, L.c_val, L.c_rank, L.c_row, L.words};
}

void dlgm_mesh_ep_plan(const at::Tensor& offsets, at::Tensor plan, int64_t capacity, const at::Tensor& peers,
                       at::Tensor state, int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes,
                       int64_t slots, int64_t heap_bytes, int64_t timeout) {
  const int W = (int)peers.numel();
  check_geom(W, (int)me, (int)ch);
  const int E = (int)offsets.numel() - 1;
  TORCH_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kInt && offsets.is_contiguous() && E >= W &&
                  E % W == 0 && W * E <= kMaxPlan,
              "mesh_ep_plan: offsets must be a contiguous int32 [E + 1] GPU tensor, E a multiple of W");
  const PlanLayout L = plan_layout(W, E);
  TORCH_CHECK(plan.is_cuda() && plan.scalar_type() == at::kInt && plan.is_contiguous() && plan.numel() >= L.words,
              "mesh_ep_plan: plan tensor too small");
  TORCH_CHECK((int64_t)W * E * 4 <= slot_bytes && region_off + slots * slot_bytes <= heap_bytes && slots >= 1 &&
                  capacity >= 0 && capacity < (1ll << 30),
              "mesh_ep_plan: slot geometry");
  mesh_ep_plan_kernel<<<1, kThreads, 0, c10::hip::getCurrentHIPStream()>>>(
      offsets.data_ptr<int>(), plan.data_ptr<int>(), L, W, E, (int)capacity, peers_ptr(peers, W), region_off,
      slot_bytes, (int)slots, state_ptr(state), (int)ch, (int)me, timeout);
  DLGM_CHECK_HIP(hipGetLastError());
}

// rows of x (contiguous [R, D], 16-bit) through the segment table of `plan` (dispatch: combine = false)
void dlgm_mesh_push_rows(const at::Tensor& x, const at::Tensor& plan, bool combine, const at::Tensor& peers,
                         at::Tensor state, int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes,
                         int64_t hdr_bytes, int64_t slots, int64_t slot_rows, int64_t heap_bytes, int64_t n_experts) {
  const int W = (int)peers.numel();
  check_geom(W, (int)me, (int)ch);
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 2 && DLGM_IS16(x) &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "mesh_push_rows: contiguous [R, D] 16-bit GPU rows");
  const int64_t row_bytes = x.size(1) * x.element_size();
  TORCH_CHECK(row_bytes % 16 == 0, "mesh_push_rows: rows must be 16-byte multiples");
  TORCH_CHECK(hdr_bytes % 16 == 0 && hdr_bytes + slot_rows * row_bytes <= slot_bytes &&
                  region_off + slots * slot_bytes <= heap_bytes,
              "mesh_push_rows: slot geometry");
  const int E = (int)n_experts;
  const PlanLayout L = plan_layout(W, E);
  TORCH_CHECK(plan.scalar_type() == at::kInt && plan.numel() >= L.words, "mesh_push_rows: bad plan");
  const int* pl = plan.data_ptr<int>();
  SegTab tab = combine ? SegTab{pl + L.c_vs, pl + L.c_src, pl + L.c_val, pl + L.c_rank, pl + L.c_row, (E / W) * W}
                       : SegTab{pl + L.d_vs, pl + L.d_src, pl + L.d_val, pl + L.d_rank, pl + L.d_row, E};
  // the bounds the device tables can reach: every destination row < slot_rows (dispatch: the capacity C by the
  // clamp; combine: the source's own row count), every source row < x rows -- guaranteed by construction in
  // mesh_ep_plan_kernel, whose inputs are this rank's routing and the same capacity
  mesh_push_rows_kernel<<<1024, kThreads, 0, c10::hip::getCurrentHIPStream()>>>(
      reinterpret_cast<const uint4*>(x.data_ptr()), row_bytes / 16, tab, peers_ptr(peers, W), region_off,
      slot_bytes, hdr_bytes, (int)slots, state_ptr(state), (int)ch, (int)me, W);
  DLGM_CHECK_HIP(hipGetLastError());
}

void dlgm_mesh_copy_rows(at::Tensor out, const c10::optional<at::Tensor>& nrows, const at::Tensor& peers,
                         at::Tensor state, int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes,
                         int64_t hdr_bytes, int64_t slots, int64_t heap_bytes) {
  const int W = (int)peers.numel();
  check_geom(W, (int)me, (int)ch);
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.dim() == 2 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "mesh_copy_rows: contiguous [R, D] GPU output");
  const int64_t row_bytes = out.size(1) * out.element_size();
  TORCH_CHECK(row_bytes % 16 == 0 && hdr_bytes + out.size(0) * row_bytes <= slot_bytes &&
                  region_off + slots * slot_bytes <= heap_bytes,
              "mesh_copy_rows: slot geometry");
  const int* nr = nullptr;
  if (nrows.has_value()) {
    TORCH_CHECK(nrows->is_cuda() && nrows->scalar_type() == at::kInt && nrows->numel() >= 1, "mesh_copy_rows: nrows");
    nr = nrows->data_ptr<int>();
  }
  const unsigned gx = grid_for(out.size(0) * row_bytes / 16 / 2, 1024);
  mesh_copy_rows_kernel<<<gx, kThreads, 0, c10::hip::getCurrentHIPStream()>>>(
      reinterpret_cast<uint4*>(out.data_ptr()), row_bytes / 16, out.size(0), nr, peers_ptr(peers, W), region_off,
      slot_bytes, hdr_bytes, (int)slots, state_ptr(state), (int)ch, (int)me, W);
  DLGM_CHECK_HIP(hipGetLastError());
}
