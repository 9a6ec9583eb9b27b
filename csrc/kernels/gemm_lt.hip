// hipBLASLt GEMM with per-shape solution selection, for the weight-gradient GEMMs.
//
// dW = dY^T X runs bf16 x bf16 -> fp32 and accumulates into the fp32 gradient partition
// (beta = 1, ops/gemm.py grad_mm). Through aten (`addmm(..., out_dtype=float32)`) that GEMM
// gets hipBLASLt's first heuristic pick, which on gfx950 was measured at 0.8-1.3 PF/s for the
// Llama-3-8B dW shapes while the bf16-output GEMMs of the same size reach 1.5 PF/s
// (profiles/rocprof_kernel_stats_r01_v8_ga8.csv). This op calls hipBLASLt directly and
// lets the caller pick the solution:
//
//   gemm_lt(out, a, b, beta, algo)          out[M,N] = a[M,K] @ b[K,N] (+ beta * out)
//   gemm_lt_tune(out, a, b, beta, n, reps)  time up to n candidate solutions on a scratch output
//                                            and return [(solution index, us)] fastest first
//
// Solution indices are hipBLASLt's own (hipblaslt_ext::getIndexFromAlgo) and are valid for one
// library build; ops/gemm.py keys its table by (shape, layouts, dtypes, beta) and records the
// library version beside it. Operands may be row-major or transposed views (one unit stride);
// the descriptors, layouts and resolved algorithm of each problem are cached, so a steady-state
// call is one hipblasLtMatmul on the current HIP stream, with that stream's own workspace.
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>
#include <torch/all.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

#define LT_CHECK(x)                                                                          \
  do {                                                                                       \
    hipblasStatus_t st_ = (x);                                                               \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #x, " failed with status ", (int)st_); \
  } while (0)

constexpr size_t kWorkspace = 128ull << 20;  // stream-K / split-K solutions need scratch

// problem key: shape, operand layouts (op + leading dim), output dtype, beta != 0, operand dtype (bf16 / fp16)
using Key = std::tuple<int64_t, int64_t, int64_t, int, int64_t, int, int64_t, int64_t, int, bool, int>;

struct Problem {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  std::map<int, hipblasLtMatmulAlgo_t> algos;  // solution index -> algo bound to this problem
  int default_index = -1;
};

struct State {
  hipblasLtHandle_t handle = nullptr;
  // One scratch per (device, HIP stream), as torch keys its own hipBLASLt workspaces: stream-K / split-K solutions
  // keep partial tiles and fix-up flags there, so two GEMMs on different streams must never share one. Each is
  // allocated from the caching allocator while its stream is current and is never freed.
  std::map<std::pair<int, hipStream_t>, at::Tensor> workspaces;
  std::map<Key, Problem> problems;
  std::mutex mu;
};

State& state() {
  static State s;
  return s;
}

// Column-major mapping of the row-major product out[M,N] = a[M,K] @ b[K,N]:
// out^T[N,M] = b^T[N,K] @ a^T[K,M], i.e. hipBLASLt's A := b, B := a.
struct Operand {
  hipblasOperation_t op;
  int64_t rows, cols, ld;
};

Operand as_lt(const at::Tensor& t) {  // t [R, C] row-major or a transposed view -> column-major operand of t^T
  if (t.stride(1) == 1) return {HIPBLAS_OP_N, t.size(1), t.size(0), std::max<int64_t>(t.stride(0), t.size(1))};
  TORCH_CHECK(t.stride(0) == 1, "gemm_lt: operands need one unit stride");
  return {HIPBLAS_OP_T, t.size(0), t.size(1), std::max<int64_t>(t.stride(1), t.size(0))};
}

hipDataType dt(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return HIP_R_32F;
  if (t.scalar_type() == at::kBFloat16) return HIP_R_16BF;
  if (t.scalar_type() == at::kHalf) return HIP_R_16F;
  TORCH_CHECK(false, "gemm_lt: unsupported dtype ", t.scalar_type());
}

Problem& problem(State& S, const at::Tensor& out, const at::Tensor& a, const at::Tensor& b, bool beta_nz) {
  const Operand A = as_lt(b), B = as_lt(a);  // hipBLASLt A = b, B = a
  const int64_t M = out.size(1), N = out.size(0), K = a.size(1);
  Key key{M, N, K, (int)A.op, A.ld, (int)B.op, B.ld, out.stride(0), (int)dt(out), beta_nz, (int)dt(a)};
  auto it = S.problems.find(key);
  if (it != S.problems.end()) return it->second;
  Problem p;
  LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  int32_t opa = A.op, opb = B.op;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.la, dt(b), A.rows, A.cols, A.ld));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lb, dt(a), B.rows, B.cols, B.ld));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.lc, dt(out), M, N, out.stride(0)));
  return S.problems.emplace(key, p).first->second;
}

void init(State& S) {
  if (S.handle == nullptr) LT_CHECK(hipblasLtCreate(&S.handle));
}

// the workspace of the current (device, stream)
void* workspace(State& S, hipStream_t stream) {
  const int dev = c10::hip::current_device();
  auto& w = S.workspaces[{dev, stream}];
  if (!w.defined())
    w = at::empty({(int64_t)kWorkspace}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
  return w.data_ptr();
}

void check_args(const at::Tensor& out, const at::Tensor& a, const at::Tensor& b) {
  TORCH_CHECK(out.is_cuda() && a.is_cuda() && b.is_cuda(), "gemm_lt: CUDA tensors expected");
  TORCH_CHECK(out.dim() == 2 && a.dim() == 2 && b.dim() == 2, "gemm_lt: 2-D operands");
  TORCH_CHECK(a.size(1) == b.size(0) && out.size(0) == a.size(0) && out.size(1) == b.size(1), "gemm_lt: shape mismatch");
  TORCH_CHECK((a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf) && b.scalar_type() == a.scalar_type(),
              "gemm_lt: bf16 or fp16 operands of one dtype");
  TORCH_CHECK(out.stride(1) == 1, "gemm_lt: row-major output");
}

// the algo for solution `index` bound to problem p (nullptr when the solution does not support it)
const hipblasLtMatmulAlgo_t* resolve(State& S, Problem& p, int index, const void* alpha, const void* beta) {
  auto it = p.algos.find(index);
  if (it != p.algos.end()) return &it->second;
  std::vector<int> idx{index};
  std::vector<hipblasLtMatmulHeuristicResult_t> res;
  if (hipblaslt_ext::getAlgosFromIndex(S.handle, idx, res) != HIPBLAS_STATUS_SUCCESS || res.empty()) return nullptr;
  size_t ws = 0;
  if (hipblaslt_ext::matmulIsAlgoSupported(S.handle, p.desc, alpha, p.la, p.lb, beta, p.lc, p.lc, res[0].algo, ws) !=
          HIPBLAS_STATUS_SUCCESS ||
      ws > kWorkspace)
    return nullptr;
  return &p.algos.emplace(index, res[0].algo).first->second;
}

std::vector<hipblasLtMatmulHeuristicResult_t> heuristic(State& S, Problem& p, int n) {
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t ws = kWorkspace;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(std::max(1, n));
  int got = 0;
  hipblasStatus_t st =
      hipblasLtMatmulAlgoGetHeuristic(S.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, (int)res.size(), res.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  res.resize(st == HIPBLAS_STATUS_SUCCESS ? got : 0);
  return res;
}

void run(State& S, Problem& p, const hipblasLtMatmulAlgo_t* algo, const void* alpha, const void* beta,
         const at::Tensor& out, const at::Tensor& a, const at::Tensor& b, hipStream_t stream) {
  LT_CHECK(hipblasLtMatmul(S.handle, p.desc, alpha, b.data_ptr(), p.la, a.data_ptr(), p.lb, beta, out.data_ptr(),
                           p.lc, out.data_ptr(), p.lc, algo, workspace(S, stream), kWorkspace, stream));
}

}  // namespace

int64_t dlgm_gemm_lt(at::Tensor out, const at::Tensor& a, const at::Tensor& b, double beta_d, int64_t algo_index) {
  check_args(out, a, b);
  State& S = state();
  std::lock_guard<std::mutex> g(S.mu);
  init(S);
  const float alpha = 1.f, beta = (float)beta_d;
  Problem& p = problem(S, out, a, b, beta != 0.f);
  int index = (int)algo_index;
  const hipblasLtMatmulAlgo_t* algo = index >= 0 ? resolve(S, p, index, &alpha, &beta) : nullptr;
  if (algo == nullptr) {  // no (valid) choice: hipBLASLt's first heuristic pick, remembered per problem
    if (p.default_index < 0) {
      auto res = heuristic(S, p, 1);
      TORCH_CHECK(!res.empty(), "gemm_lt: no hipBLASLt solution for this problem");
      p.default_index = hipblaslt_ext::getIndexFromAlgo(res[0].algo);
      p.algos.emplace(p.default_index, res[0].algo);
    }
    index = p.default_index;
    algo = &p.algos.at(index);
  }
  run(S, p, algo, &alpha, &beta, out, a, b, c10::hip::getCurrentHIPStream());
  return index;
}

// Candidates: hipBLASLt's heuristic list (n_heuristic) plus, if all_algos, every solution of the type
// combination the library reports as supporting this problem. Timed on a scratch output with the
// same strides, so `out` is untouched.
at::Tensor dlgm_gemm_lt_tune(const at::Tensor& out, const at::Tensor& a, const at::Tensor& b, double beta_d,
                             int64_t n_heuristic, bool all_algos, int64_t reps) {
  check_args(out, a, b);
  State& S = state();
  std::lock_guard<std::mutex> g(S.mu);
  init(S);
  const float alpha = 1.f, beta = (float)beta_d;
  Problem& p = problem(S, out, a, b, beta != 0.f);
  std::vector<hipblasLtMatmulAlgo_t> cands;
  std::vector<int> seen;
  auto add = [&](hipblasLtMatmulAlgo_t algo) {
    const int idx = hipblaslt_ext::getIndexFromAlgo(algo);
    if (idx < 0 || std::find(seen.begin(), seen.end(), idx) != seen.end()) return;
    size_t ws = 0;
    if (hipblaslt_ext::matmulIsAlgoSupported(S.handle, p.desc, &alpha, p.la, p.lb, &beta, p.lc, p.lc, algo, ws) !=
            HIPBLAS_STATUS_SUCCESS ||
        ws > kWorkspace)
      return;
    seen.push_back(idx);
    cands.push_back(algo);
  };
  for (auto& r : heuristic(S, p, (int)n_heuristic)) add(r.algo);
  if (all_algos) {
    std::vector<hipblasLtMatmulHeuristicResult_t> all;
    int32_t va = 0, vb = 0;
    size_t sz = 0;
    LT_CHECK(hipblasLtMatmulDescGetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &va, sizeof(va), &sz));
    LT_CHECK(hipblasLtMatmulDescGetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &vb, sizeof(vb), &sz));
    if (hipblaslt_ext::getAllAlgos(S.handle, hipblaslt_ext::GemmType::HIPBLASLT_GEMM, (hipblasOperation_t)va,
                                   (hipblasOperation_t)vb, dt(b), dt(a), dt(out), dt(out),
                                   HIPBLAS_COMPUTE_32F, all) == HIPBLAS_STATUS_SUCCESS)
      for (auto& r : all) add(r.algo);
  }
  TORCH_CHECK(!cands.empty(), "gemm_lt_tune: no hipBLASLt solution for this problem");
  at::Tensor scratch = at::zeros_like(out);
  hipStream_t stream = c10::hip::getCurrentHIPStream();
  hipEvent_t e0, e1;
  TORCH_CHECK(hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess, "hipEventCreate");
  std::vector<std::pair<float, int>> timed;
  for (size_t i = 0; i < cands.size(); ++i) {
    if (hipblasLtMatmul(S.handle, p.desc, &alpha, b.data_ptr(), p.la, a.data_ptr(), p.lb, &beta, scratch.data_ptr(),
                        p.lc, scratch.data_ptr(), p.lc, &cands[i], workspace(S, stream), kWorkspace,
                        stream) != HIPBLAS_STATUS_SUCCESS)
      continue;  // warm-up launch; a solution that fails to launch is skipped
    hipEventRecord(e0, stream);
    for (int r = 0; r < std::max<int64_t>(1, reps); ++r)
      run(S, p, &cands[i], &alpha, &beta, scratch, a, b, stream);
    hipEventRecord(e1, stream);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    timed.emplace_back(ms * 1000.f / std::max<int64_t>(1, reps), seen[i]);
    p.algos.emplace(seen[i], cands[i]);
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  std::sort(timed.begin(), timed.end());
  at::Tensor res = at::empty({(int64_t)timed.size(), 2}, at::kDouble);
  auto acc = res.accessor<double, 2>();
  for (size_t i = 0; i < timed.size(); ++i) {
    acc[i][0] = (double)timed[i].second;
    acc[i][1] = (double)timed[i].first;
  }
  return res;
}

int64_t dlgm_gemm_lt_version() {
  State& S = state();
  std::lock_guard<std::mutex> g(S.mu);
  if (S.handle == nullptr) LT_CHECK(hipblasLtCreate(&S.handle));
  int v = 0;
  LT_CHECK(hipblasLtGetVersion(S.handle, &v));
  return v;
}
