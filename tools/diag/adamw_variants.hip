// A/B of the flat AdamW and grad-stats streaming schedules (standalone, no torch).
// Same per-element arithmetic as csrc/kernels/optim.hip; what varies is the grid size (waves per CU) and how many
// 16-byte vectors per array a lane has in flight per iteration. Prints one JSON line per variant and checks the
// variants' outputs are bit-identical to the baseline's on a small odd-sized buffer.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/diag/adamw_variants.hip -o gpurun_out/adamw_variants
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;

struct H {
  float lr, b1, b2, eps, wd, bc1, bc2, gc;
};

template <int U>
__global__ __launch_bounds__(kThreads) void adamw_v(float* __restrict__ p, float* __restrict__ m,
                                                     float* __restrict__ v, const float* __restrict__ g,
                                                     __bf16* __restrict__ p16, int64_t n, H h) {
  const float decay = 1.f - h.lr * h.wd;
  const float step_size = h.lr / h.bc1;
  const float inv_sqrt_bc2 = rsqrtf(h.bc2);
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  auto body = [&](f32x4& pp, f32x4& mm, f32x4& vv, const f32x4& gg) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = gg[j] * h.gc;
      mm[j] = h.b1 * mm[j] + (1.f - h.b1) * gj;
      vv[j] = h.b2 * vv[j] + (1.f - h.b2) * gj * gj;
      const float denom = sqrtf(vv[j]) * inv_sqrt_bc2 + h.eps;
      pp[j] = pp[j] * decay - step_size * mm[j] / denom;
    }
  };
  for (; i + (U - 1) * stride < nv; i += U * stride) {
    f32x4 pp[U], mm[U], vv[U], gg[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = (i + u * stride) * 4;
      pp[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + k));
      mm[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m + k));
      vv[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v + k));
      gg[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + k));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = (i + u * stride) * 4;
      body(pp[u], mm[u], vv[u], gg[u]);
      __builtin_nontemporal_store(pp[u], reinterpret_cast<f32x4*>(p + k));
      __builtin_nontemporal_store(mm[u], reinterpret_cast<f32x4*>(m + k));
      __builtin_nontemporal_store(vv[u], reinterpret_cast<f32x4*>(v + k));
      __builtin_nontemporal_store(__builtin_convertvector(pp[u], bf16x4), reinterpret_cast<bf16x4*>(p16 + k));
    }
  }
  for (; i < nv; i += stride) {
    f32x4 pp = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + i * 4));
    f32x4 mm = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(m + i * 4));
    f32x4 vv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v + i * 4));
    f32x4 gg = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g + i * 4));
    body(pp, mm, vv, gg);
    __builtin_nontemporal_store(pp, reinterpret_cast<f32x4*>(p + i * 4));
    __builtin_nontemporal_store(mm, reinterpret_cast<f32x4*>(m + i * 4));
    __builtin_nontemporal_store(vv, reinterpret_cast<f32x4*>(v + i * 4));
    __builtin_nontemporal_store(__builtin_convertvector(pp, bf16x4), reinterpret_cast<bf16x4*>(p16 + i * 4));
  }
  if (blockIdx.x == 0)
    for (int64_t t = nv * 4 + threadIdx.x; t < n; t += kThreads) {
      const float gj = g[t] * h.gc;
      m[t] = h.b1 * m[t] + (1.f - h.b1) * gj;
      v[t] = h.b2 * v[t] + (1.f - h.b2) * gj * gj;
      p[t] = p[t] * (1.f - h.lr * h.wd) - (h.lr / h.bc1) * m[t] / (sqrtf(v[t]) * rsqrtf(h.bc2) + h.eps);
      p16[t] = (__bf16)p[t];
    }
}

// pure read: sum of squares, U vectors in flight per lane, NT selects non-temporal loads
template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void sumsq_v(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  float ss = 0.f;
  const int64_t nv = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  for (; i + (U - 1) * stride < nv; i += U * stride) {
    f32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f32x4* a = reinterpret_cast<const f32x4*>(g + (i + u * stride) * 4);
      if constexpr (NT) x[u] = __builtin_nontemporal_load(a);
      else x[u] = *a;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) ss += __builtin_isfinite(x[u][j]) ? x[u][j] * x[u][j] : 0.f;
  }
  for (; i < nv; i += stride) {
    f32x4 x = *reinterpret_cast<const f32x4*>(g + i * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) ss += x[j] * x[j];
  }
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void fill_rand(float* x, int64_t n, uint32_t seed, float lo, float hi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t s = (uint32_t)i * 2654435761u ^ seed;
    s ^= s >> 13; s *= 0x5bd1e995u; s ^= s >> 15;
    x[i] = lo + (hi - lo) * (s & 0xffffff) / 16777216.f;
  }
}

typedef void (*AdamFn)(float*, float*, float*, const float*, __bf16*, int64_t, H);

struct AVariant {
  const char* name;
  AdamFn fn;
  int grid;
};

int main() {
  const int64_t n = 1ll << 30;
  float *p, *m, *v, *g, *part;
  __bf16* p16;
  CK(hipMalloc(&p, n * 4)); CK(hipMalloc(&m, n * 4)); CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&g, n * 4));
  CK(hipMalloc(&p16, n * 2)); CK(hipMalloc(&part, (1 << 20) * 4));
  fill_rand<<<4096, 256>>>(p, n, 1, -1.f, 1.f);
  fill_rand<<<4096, 256>>>(m, n, 2, -1e-3f, 1e-3f);
  fill_rand<<<4096, 256>>>(v, n, 3, 0.f, 1e-6f);
  fill_rand<<<4096, 256>>>(g, n, 4, -1e-3f, 1e-3f);
  CK(hipDeviceSynchronize());
  H h{1e-4f, 0.9f, 0.999f, 1e-8f, 0.01f, 0.19f, 0.001999f, 0.5f};
  std::vector<AVariant> av = {
      {"adamw_u1_g2048", adamw_v<1>, 2048}, {"adamw_u2_g2048", adamw_v<2>, 2048},
      {"adamw_u1_g4096", adamw_v<1>, 4096}, {"adamw_u2_g4096", adamw_v<2>, 4096},
      {"adamw_u2_g1024", adamw_v<2>, 1024}, {"adamw_u4_g1024", adamw_v<4>, 1024},
      {"adamw_u1_g8192", adamw_v<1>, 8192}, {"adamw_u1_g16384", adamw_v<1>, 16384},
      {"adamw_u2_g8192", adamw_v<2>, 8192}, {"adamw_u1_gfull", adamw_v<1>, 1 << 20},
  };
  // bit-identity on a small odd-sized buffer (tail path included)
  {
    const int64_t ns = (1 << 20) + 7;
    std::vector<float> ref;
    std::vector<uint16_t> ref16;
    float *sp, *sm, *sv, *sg;
    __bf16* s16;
    CK(hipMalloc(&sp, ns * 4)); CK(hipMalloc(&sm, ns * 4)); CK(hipMalloc(&sv, ns * 4)); CK(hipMalloc(&sg, ns * 4));
    CK(hipMalloc(&s16, ns * 2));
    for (size_t k = 0; k < av.size(); ++k) {
      fill_rand<<<256, 256>>>(sp, ns, 11, -1.f, 1.f);
      fill_rand<<<256, 256>>>(sm, ns, 12, -1e-3f, 1e-3f);
      fill_rand<<<256, 256>>>(sv, ns, 13, 0.f, 1e-6f);
      fill_rand<<<256, 256>>>(sg, ns, 14, -1e-3f, 1e-3f);
      av[k].fn<<<std::min<int64_t>(av[k].grid, (ns / 4 + 255) / 256), kThreads>>>(sp, sm, sv, sg, s16, ns, h);
      CK(hipDeviceSynchronize());
      std::vector<float> out(ns * 3);
      std::vector<uint16_t> o16(ns);
      CK(hipMemcpy(out.data(), sp, ns * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(out.data() + ns, sm, ns * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(out.data() + 2 * ns, sv, ns * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(o16.data(), s16, ns * 2, hipMemcpyDeviceToHost));
      if (k == 0) {
        ref = out;
        ref16 = o16;
      } else {
        const bool same = !memcmp(ref.data(), out.data(), ns * 12) && !memcmp(ref16.data(), o16.data(), ns * 2);
        printf("{\"check\": \"%s\", \"bit_identical\": %s}\n", av[k].name, same ? "true" : "false");
      }
    }
    hipFree(sp); hipFree(sm); hipFree(sv); hipFree(sg); hipFree(s16);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 8;
  for (int rep = 0; rep < 3; ++rep) {
    for (auto& a : av) {
      a.fn<<<a.grid, kThreads>>>(p, m, v, g, p16, n, h);
      CK(hipEventRecord(e0));
      for (int it = 0; it < iters; ++it) a.fn<<<a.grid, kThreads>>>(p, m, v, g, p16, n, h);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      printf("{\"rep\": %d, \"variant\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f}\n", rep, a.name, ms,
             n * 30.0 / ms / 1e6);
      fflush(stdout);
    }
    struct SV {
      const char* name;
      void (*fn)(const float*, int64_t, float*);
      int grid;
    } sv[] = {{"sumsq_u4_g1024", sumsq_v<4, false>, 1024}, {"sumsq_u4_g2048", sumsq_v<4, false>, 2048},
              {"sumsq_u8_g1024", sumsq_v<8, false>, 1024}, {"sumsq_u4_g1024_nt", sumsq_v<4, true>, 1024},
              {"sumsq_u8_g2048_nt", sumsq_v<8, true>, 2048}, {"sumsq_u4_g4096", sumsq_v<4, false>, 4096},
              {"sumsq_u8_g4096_nt", sumsq_v<8, true>, 4096}, {"sumsq_u4_g2048_nt", sumsq_v<4, true>, 2048},
              {"sumsq_u16_g1024_nt", sumsq_v<16, true>, 1024}, {"sumsq_u8_g1024_nt", sumsq_v<8, true>, 1024}};
    for (auto& s : sv) {
      s.fn<<<s.grid, kThreads>>>(g, n, part);
      CK(hipEventRecord(e0));
      for (int it = 0; it < iters; ++it) s.fn<<<s.grid, kThreads>>>(g, n, part);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      printf("{\"rep\": %d, \"variant\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f}\n", rep, s.name, ms, n * 4.0 / ms / 1e6);
      fflush(stdout);
    }
  }
  CK(hipGetLastError());
  return 0;
}
