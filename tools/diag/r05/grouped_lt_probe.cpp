// Round 5 probe: can hipBLASLt's grouped GEMM run the MoE expert GEMMs with the per-expert row counts read from
// DEVICE memory (hipblaslt_ext::GroupedGemm::run(deviceUserArgs)), i.e. without a host read of the routing?
// The problem is set on the host once with worst-case sizes; the per-group n (rows routed to the expert) is then
// rewritten in the device argument array. Checks sampled outputs against a host fp32 dot product and times the
// device-args run against a run initialised with the exact sizes.
//
// Expert forward, row-major: out_e [R_e, F] = x_e [R_e, D] @ W_e^T, W_e [F, D]. Column-major for hipBLASLt:
// D_e [F, R_e] = op_T(W_e as [D, F], ld D) x op_N(x_e as [D, R_e], ld D): m = F, n = R_e, k = D.
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 grouped_lt_probe.cpp -lhipblaslt -o grouped_lt_probe
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    auto e_ = (x);                                                               \
    if ((int)e_ != 0) {                                                          \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, (int)e_); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__global__ void fill(__hip_bfloat16* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = __float2bfloat16(((int)(h & 0xffff) - 32768) / 32768.0f);
  }
}

static float bf(const __hip_bfloat16& v) {
  uint16_t u;
  std::memcpy(&u, &v, 2);
  uint32_t w = (uint32_t)u << 16;
  float f;
  std::memcpy(&f, &w, 4);
  return f;
}

int main(int argc, char** argv) {
  const int E = 8, D = argc > 1 ? atoi(argv[1]) : 4096, F = argc > 2 ? atoi(argv[2]) : 28672;
  const int R = argc > 3 ? atoi(argv[3]) : 8192;  // rows routed in total (tokens x top-k)
  const int NMAX = argc > 4 ? atoi(argv[4]) : R;  // host-side per-group n at initialisation
  std::mt19937 rng(7);
  std::vector<int64_t> cnt(E);
  {
    std::vector<double> w(E);
    double s = 0;
    for (auto& x : w) s += (x = getenv("GLP_UNIFORM") ? 1.0 : 0.6 + (rng() % 1000) / 1000.0);
    int64_t used = 0;
    for (int e = 0; e < E; ++e) used += (cnt[e] = (int64_t)(R * w[e] / s));
    cnt[E - 1] += R - used;
  }
  std::vector<int64_t> off(E + 1, 0);
  for (int e = 0; e < E; ++e) off[e + 1] = off[e] + cnt[e];

  __hip_bfloat16 *x, *w, *out, *out_ref;
  CK(hipMalloc(&x, (size_t)R * D * 2));
  CK(hipMalloc(&w, (size_t)E * F * D * 2));
  CK(hipMalloc(&out, (size_t)R * F * 2));
  CK(hipMalloc(&out_ref, (size_t)R * F * 2));
  fill<<<4096, 256>>>(x, (size_t)R * D, 1);
  fill<<<4096, 256>>>(w, (size_t)E * F * D, 2);
  CK(hipMemset(out, 0, (size_t)R * F * 2));
  CK(hipDeviceSynchronize());

  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  for (auto oa : {HIPBLAS_OP_N, HIPBLAS_OP_T})
    for (auto ob : {HIPBLAS_OP_N, HIPBLAS_OP_T}) {
      std::vector<hipblasLtMatmulHeuristicResult_t> all;
      hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GROUPED_GEMM, oa, ob, HIP_R_16BF, HIP_R_16BF,
                                 HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all);
      std::vector<hipblasLtMatmulHeuristicResult_t> f32;
      hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GROUPED_GEMM, oa, ob, HIP_R_16BF, HIP_R_16BF,
                                 HIP_R_32F, HIP_R_32F, HIPBLAS_COMPUTE_32F, f32);
      std::printf("grouped solutions op%c%c: bf16-out %zu, f32-out %zu\n", oa == HIPBLAS_OP_N ? 'N' : 'T',
                  ob == HIPBLAS_OP_N ? 'N' : 'T', all.size(), f32.size());
    }
  size_t ws_bytes = 256u << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  float alpha = 1.f, beta = 0.f;

  auto build = [&](hipblaslt_ext::GroupedGemm& gg, const std::vector<int64_t>& n_host, hipblasLtMatmulAlgo_t* pick,
                   bool print) {
    std::vector<int64_t> m(E, F), n(n_host), k(E, D), b(E, 1);
    std::vector<hipblaslt_ext::GemmEpilogue> ep(E);
    std::vector<hipblaslt_ext::GemmInputs> in(E);
    for (int e = 0; e < E; ++e) {
      in[e].setA(w + (size_t)e * F * D);
      in[e].setB(x + (size_t)off[e] * D);
      in[e].setC(out + (size_t)off[e] * F);
      in[e].setD(out + (size_t)off[e] * F);
      in[e].setAlpha(&alpha);
      in[e].setBeta(&beta);
    }
    if (getenv("GLP_DESC")) {  // the hipblasLt-structure form: one matmul descriptor + layouts per group
      std::vector<hipblasLtMatmulDesc_t> md(E);
      std::vector<hipblasLtMatrixLayout_t> la(E), lb(E), lc(E);
      std::vector<void*> al(E, &alpha), be(E, &beta), A(E), B(E), C(E);
      for (int e = 0; e < E; ++e) {
        CK(hipblasLtMatmulDescCreate(&md[e], HIPBLAS_COMPUTE_32F, HIP_R_32F));
        int32_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
        CK(hipblasLtMatmulDescSetAttribute(md[e], HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
        CK(hipblasLtMatmulDescSetAttribute(md[e], HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
        CK(hipblasLtMatrixLayoutCreate(&la[e], HIP_R_16BF, D, F, D));
        CK(hipblasLtMatrixLayoutCreate(&lb[e], HIP_R_16BF, D, n[e], D));
        CK(hipblasLtMatrixLayoutCreate(&lc[e], HIP_R_16BF, F, n[e], F));
        A[e] = w + (size_t)e * F * D;
        B[e] = x + (size_t)off[e] * D;
        C[e] = out + (size_t)off[e] * F;
      }
      std::vector<void*> Dp(C);
      CK(gg.setProblem(md, al, A, la, B, lb, be, C, lc, Dp, lc));
    } else if (getenv("GLP_LD")) {
      std::vector<int64_t> lda(E, D), ldb(E, D), ldc(E, F), ldd(E, F), sa(E, (int64_t)F * D), sb(E, 0), sc(E, 0),
          sd(E, 0);
      for (int e = 0; e < E; ++e) sb[e] = sc[e] = sd[e] = 0;
      hipblaslt_ext::GemmProblemType pt(HIPBLAS_OP_T, HIPBLAS_OP_N, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF,
                                        HIPBLAS_COMPUTE_32F);
      CK(gg.setProblem(m, n, k, b, lda, ldb, ldc, ldd, sa, sb, sc, sd, ep, in, pt));
    } else {
      CK(gg.setProblem(m, n, k, b, ep, in));
    }
    hipblaslt_ext::GemmPreference pref;
    pref.setMaxWorkspaceBytes(ws_bytes);
    std::vector<hipblasLtMatmulHeuristicResult_t> res;
    gg.algoGetHeuristic(16, pref, res);
    if (print) std::printf("heuristic candidates: %zu\n", res.size());
    if (res.empty()) {  // fall back to every grouped solution of this type combination that accepts the problem
      std::vector<hipblasLtMatmulHeuristicResult_t> all, ok;
      hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GROUPED_GEMM, HIPBLAS_OP_T, HIPBLAS_OP_N,
                                 HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all);
      size_t n_ok_any = 0, min_ws = (size_t)-1;
      std::map<int, int> codes;
      for (auto& r : all) {
        size_t wsz = 0;
        const auto st = gg.isAlgoSupported(r.algo, wsz);
        codes[(int)st]++;
        if (st == HIPBLAS_STATUS_SUCCESS) {
          ++n_ok_any;
          min_ws = std::min(min_ws, wsz);
          if (wsz <= ws_bytes) ok.push_back(r);
        }
      }
      if (print) {
        std::printf("getAllAlgos grouped: %zu, supporting this problem: %zu (any workspace %zu, min ws %zu)\n",
                    all.size(), ok.size(), n_ok_any, min_ws);
        for (auto& c : codes) std::printf("  status %d: %d\n", c.first, c.second);
      }
      res = ok;
    }
    if (res.empty()) std::exit(2);
    *pick = res[0].algo;
    CK(gg.initialize(res[0].algo, ws));
    if (print) std::printf("kernel: %s\n", gg.getKernelName().c_str());
    return res;
  };

  // (1) exact sizes on the host
  hipblaslt_ext::GroupedGemm exact(h, HIPBLAS_OP_T, HIPBLAS_OP_N, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF,
                                   HIPBLAS_COMPUTE_32F);
  hipblasLtMatmulAlgo_t a_exact;
  build(exact, cnt, &a_exact, true);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(exact.run(0));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) CK(exact.run(0));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms_exact;
  CK(hipEventElapsedTime(&ms_exact, e0, e1));
  ms_exact /= reps;
  CK(hipMemcpy(out_ref, out, (size_t)R * F * 2, hipMemcpyDeviceToDevice));
  CK(hipMemset(out, 0, (size_t)R * F * 2));

  // (2) worst-case sizes on the host, true sizes in the device argument array
  hipblaslt_ext::GroupedGemm dyn(h, HIPBLAS_OP_T, HIPBLAS_OP_N, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF,
                                 HIPBLAS_COMPUTE_32F);
  hipblasLtMatmulAlgo_t a_dyn;
  build(dyn, std::vector<int64_t>(E, NMAX), &a_dyn, true);
  std::vector<hipblaslt_ext::UserArguments> ua(E);
  CK(dyn.getDefaultValueForDeviceUserArguments(ua.data()));
  for (int e = 0; e < E; ++e) ua[e].n = (uint32_t)cnt[e];
  std::printf("user args: m %u n %u k %u batch %u strideA1 %u strideB1 %u strideD1 %u\n", ua[0].m, ua[0].n, ua[0].k,
              ua[0].batch, ua[0].strideA1, ua[0].strideB1, ua[0].strideD1);
  void* dua;
  CK(hipMalloc(&dua, sizeof(hipblaslt_ext::UserArguments) * E));
  CK(hipMemcpy(dua, ua.data(), sizeof(hipblaslt_ext::UserArguments) * E, hipMemcpyHostToDevice));
  CK(dyn.run(dua, 0));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) CK(dyn.run(dua, 0));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms_dyn;
  CK(hipEventElapsedTime(&ms_dyn, e0, e1));
  ms_dyn /= reps;

  // correctness: sampled outputs vs a host dot product, and dyn == exact bitwise
  std::vector<__hip_bfloat16> ho((size_t)R * F), hr((size_t)R * F), hx((size_t)R * D), hw((size_t)F * D);
  CK(hipMemcpy(ho.data(), out, ho.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), out_ref, hr.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hx.data(), x, hx.size() * 2, hipMemcpyDeviceToHost));
  size_t diff = 0;
  for (size_t i = 0; i < ho.size(); ++i) diff += std::memcmp(&ho[i], &hr[i], 2) != 0;
  double max_rel = 0;
  for (int e = 0; e < E; ++e) {
    CK(hipMemcpy(hw.data(), w + (size_t)e * F * D, hw.size() * 2, hipMemcpyDeviceToHost));
    for (int s = 0; s < 24; ++s) {
      const int64_t r = off[e] + rng() % cnt[e];
      const int f = rng() % F;
      double acc = 0, mag = 0;
      for (int d = 0; d < D; ++d) {
        const double p = (double)bf(hx[(size_t)r * D + d]) * bf(hw[(size_t)f * D + d]);
        acc += p;
        mag += std::fabs(p);
      }
      max_rel = std::max(max_rel, std::fabs(bf(ho[(size_t)r * F + f]) - acc) / (mag + 1e-6));
    }
  }
  const double tf = 2.0 * R * (double)F * D / 1e12;
  std::printf("counts:");
  for (auto c : cnt) std::printf(" %ld", (long)c);
  std::printf("\nexact-host: %.3f ms (%.0f TF/s)  device-args(nmax %d): %.3f ms (%.0f TF/s)  dyn!=exact elems: %zu  "
              "max |err|/sum|p|: %.2e\n",
              ms_exact, tf / ms_exact * 1e3, NMAX, ms_dyn, tf / ms_dyn * 1e3, diff, max_rel);
  return (diff == 0 && max_rel < 1e-2) ? 0 : 3;
}
