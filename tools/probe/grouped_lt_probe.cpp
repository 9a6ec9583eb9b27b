// Round 6 probe: hipBLASLt's grouped GEMM (hipblaslt_ext::GroupedGemm) on the Mixtral expert shapes of one
// micro-batch (8 experts, ~1024 routed rows each, bf16 in / bf16 out, fp32 accumulate), against the engine's own
// grouped MFMA kernel's measured times (profiles/rocprof_kernel_stats_mixtral_2l_r05.csv: gate_up fwd 1.65 ms,
// down fwd 0.94 ms per launch). Host-side group sizes; the top heuristic candidates are each timed.
//   hipcc --offload-arch=gfx950 -O2 tools/probe/grouped_lt_probe.cpp -lhipblaslt -o /tmp/grouped_lt_probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <hipblaslt/hipblaslt-ext.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    auto _s = (x);                                                              \
    if ((int)_s != 0) {                                                         \
      std::fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, (int)_s); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

static void bench(hipblasLtHandle_t h, int G, const std::vector<int64_t>& rows, int64_t N, int64_t K, void* ws,
                  size_t wsb, hipStream_t st, const char* name) {
  int64_t T = 0;
  for (auto r : rows) T += r;
  void *x, *w, *o;
  CK(hipMalloc(&x, T * K * 2));
  CK(hipMalloc(&w, (int64_t)G * N * K * 2));
  CK(hipMalloc(&o, T * N * 2));
  CK(hipMemset(x, 0x3c, T * K * 2));
  CK(hipMemset(w, 0x3c, (int64_t)G * N * K * 2));
  // row-major out[T_g, N] = x[T_g, K] @ W_g^T (W_g [N, K] row-major) == column-major D[N, T_g] = op(A)[N,K] B[K,T_g]
  // with A = W_g (K x N column-major, transposed), B = x_g (K x T_g column-major)
  hipblaslt_ext::GroupedGemm gg(h, HIPBLAS_OP_T, HIPBLAS_OP_N, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF,
                                HIPBLAS_COMPUTE_32F);
  std::vector<int64_t> m(G, N), n(rows), k(G, K), b(G, 1);
  std::vector<hipblaslt_ext::GemmEpilogue> ep(G);
  std::vector<hipblaslt_ext::GemmInputs> in(G);
  static float alpha = 1.f, beta = 0.f;
  int64_t off = 0;
  for (int g = 0; g < G; ++g) {
    in[g].setA((char*)w + (int64_t)g * N * K * 2);
    in[g].setB((char*)x + off * K * 2);
    in[g].setC((char*)o + off * N * 2);
    in[g].setD((char*)o + off * N * 2);
    in[g].setAlpha(&alpha);
    in[g].setBeta(&beta);
    off += rows[g];
  }
  std::vector<int64_t> lda(G, K), ldb(G, K), ldc(G, N), ldd(G, N), sa(G, N * K), sb(G), sc(G), sd(G);
  for (int g = 0; g < G; ++g) sb[g] = K * rows[g], sc[g] = sd[g] = N * rows[g];
  hipblaslt_ext::GemmProblemType pt(HIPBLAS_OP_T, HIPBLAS_OP_N, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF,
                                    HIPBLAS_COMPUTE_32F);
  const int sp = (int)gg.setProblem(m, n, k, b, lda, ldb, ldc, ldd, sa, sb, sc, sd, ep, in, pt);
  std::printf("  setProblem status %d\n", sp);
  hipblaslt_ext::GemmPreference pref;
  pref.setMaxWorkspaceBytes(wsb);
  std::vector<hipblasLtMatmulHeuristicResult_t> res;
  CK(gg.algoGetHeuristic(16, pref, res));
  if (res.empty()) {  // no heuristic for grouped problems here: every grouped solution of the type combination
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    CK(hipblaslt_ext::getAllAlgos(h, hipblaslt_ext::GemmType::HIPBLASLT_GROUPED_GEMM, HIPBLAS_OP_T, HIPBLAS_OP_N,
                                  HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIP_R_16BF, HIPBLAS_COMPUTE_32F, all));
    std::printf("  heuristic empty; %zu grouped solutions in the library\n", all.size());
    int hist[16] = {0};
    for (auto& r : all) {
      size_t need = 0;
      const int stt = (int)gg.isAlgoSupported(r.algo, need);
      hist[stt < 16 ? stt : 15]++;
      if (stt == 0 && need <= wsb) res.push_back(r);
      if (res.size() >= 48) break;
    }
    std::printf("  isAlgoSupported status histogram:");
    for (int i = 0; i < 16; ++i)
      if (hist[i]) std::printf(" [%d]=%d", i, hist[i]);
    std::printf("\n");
  }
  const double flops = 2.0 * T * N * K;
  std::printf("%s: T=%lld N=%lld K=%lld, %zu candidates\n", name, (long long)T, (long long)N, (long long)K, res.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double best = 1e30;
  for (size_t i = 0; i < res.size(); ++i) {
    size_t need = 0;
    if (gg.isAlgoSupported(res[i].algo, need) != HIPBLAS_STATUS_SUCCESS || need > wsb) continue;
    if (gg.initialize(res[i].algo, ws) != HIPBLAS_STATUS_SUCCESS) continue;
    for (int r = 0; r < 3; ++r) CK(gg.run(st));
    CK(hipEventRecord(e0, st));
    const int it = 20;
    for (int r = 0; r < it; ++r) CK(gg.run(st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / it;
    best = us < best ? us : best;
    std::printf("  cand %2zu idx %d: %8.1f us  %6.3f PF/s\n", i, hipblaslt_ext::getIndexFromAlgo(res[i].algo), us,
                flops / us * 1e-9);
  }
  std::printf("%s best %.1f us (%.3f PF/s)\n", name, best, flops / best * 1e-9);
  CK(hipFree(x));
  CK(hipFree(w));
  CK(hipFree(o));
}

int main() {
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t wsb = 128ull << 20;
  void* ws;
  CK(hipMalloc(&ws, wsb));
  // a realistic top-2 routing of 4096 tokens over 8 experts (8192 rows)
  std::vector<int64_t> rows = {1012, 1047, 998, 1031, 1025, 979, 1066, 1034};
  bench(h, 8, rows, 28672, 4096, ws, wsb, st, "gate_up fwd");
  bench(h, 8, rows, 4096, 14336, ws, wsb, st, "down fwd");
  bench(h, 8, rows, 4096, 28672, ws, wsb, st, "gate_up dX");
  bench(h, 8, rows, 14336, 4096, ws, wsb, st, "down dX");
  std::vector<int64_t> one = {8192};
  bench(h, 1, one, 28672, 4096, ws, wsb, st, "dense gate_up (one weight, reference)");
  return 0;
}
