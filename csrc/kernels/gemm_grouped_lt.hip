// Expert-grouped GEMMs through hipBLASLt's grouped GEMM with DEVICE-side user arguments (gfx950).
//
// A Mixtral MoE layer runs one GEMM per local expert over that expert's token rows. The row ranges are
// only known on the device (ops.moe_permute's int32 offsets), so a per-expert launch loop has to read them
// on the host -- a synchronisation per layer and micro-batch that stalls the launch pipeline (VERDICT r2
// item 5). hipBLASLt's grouped GEMM takes its per-group problem (m, n, k, pointers, leading dimensions,
// alpha/beta) from an argument array in device memory (hipblaslt_ext::UserArguments), so:
//
//   fill_user_args<<<1, G>>>   one lane per expert reads offsets[e], offsets[e+1] and writes that group's
//                              sizes and pointers into the cached argument array (on the current stream);
//   GroupedGemm::run(args)     one launch for every expert, hipBLASLt's kernel for the shape.
//
// Nothing is read on the host. The solution is chosen once per (mode, shape, total rows) from host
// problem sizes in which EVERY group holds all rows (`rows_total`): the launch grid is sized from those, so
// it covers any split of the rows over the experts; work-groups past a group's real extent exit.
//
// Modes (row-major views; ops/gemm_grouped.py):
//   0 grouped-M  out[rows_e, N] = x[rows_e, K] @ (w[e]^T if trans_w else w[e])  -- expert forward / dX
//                (w [G, N, K] with trans_w, else [G, K, N]);
//   1 grouped-K  out[e] (+)= dy[rows_e]^T @ x[rows_e]  (out [G, N, K] fp32 / bf16)   -- expert dW: the
//                reduction length of group e is its row count (0 rows: beta * C, i.e. zeros or untouched).
// hipBLASLt is column-major: row-major out[M, N] = a @ b is out^T = b^T a^T, so hipBLASLt's A is `b`.
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>
#include <hipblaslt/hipblaslt-ext.hpp>
#include <hipblaslt/hipblaslt.h>
#include <torch/all.h>

#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

#define GLT_CHECK(x)                                                                                   \
  do {                                                                                                 \
    hipblasStatus_t st_ = (x);                                                                         \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt grouped: ", #x, " failed with status ", (int)st_); \
  } while (0)

using UA = hipblaslt_ext::UserArguments;
constexpr size_t kWorkspace = 128ull << 20;

// (mode, G, N, K, rows_total, out dtype, operand dtype, trans_w, beta != 0, algo index)
using Key = std::tuple<int, int, int64_t, int64_t, int64_t, int, int, bool, bool, int>;

struct Plan {
  std::unique_ptr<hipblaslt_ext::GroupedGemm> gg;
  at::Tensor args;  // device UserArguments[G]
  std::string kernel;
  int index = -1;
};

struct State {
  hipblasLtHandle_t handle = nullptr;
  at::Tensor workspace;
  std::map<Key, Plan> plans;
  std::mutex mu;
};

State& state() {
  static State s;
  return s;
}

hipDataType hdt(at::ScalarType t) {
  if (t == at::kFloat) return HIP_R_32F;
  if (t == at::kBFloat16) return HIP_R_16BF;
  if (t == at::kHalf) return HIP_R_16F;
  TORCH_CHECK(false, "grouped_lt: unsupported dtype");
}

// Per-group problem, written by one lane per expert. Offsets are element offsets of the operand bases.
struct FillArgs {
  UA* ua;
  const int* offsets;
  const char* a;  // hipBLASLt A (row-major `b` of the product): weights (mode 0) or x rows (mode 1)
  const char* b;  // hipBLASLt B: x rows (mode 0) or dy rows (mode 1)
  char* c;
  int G, mode, esz, osz;
  int64_t a_gstride, b_row, c_row, c_gstride;  // elements: weight step per group; row pitch of B / out
};

__global__ void fill_user_args(FillArgs f) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= f.G) return;
  const int lo = f.offsets[e], rows = f.offsets[e + 1] - lo;
  UA& u = f.ua[e];
  if (f.mode == 0) {  // D^T[N, rows_e] = W'[N, K] x^T[K, rows_e]: n = this expert's rows
    u.n = (uint32_t)rows;
    u.a = (void*)(f.a + (int64_t)e * f.a_gstride * f.esz);
    u.b = (void*)(f.b + (int64_t)lo * f.b_row * f.esz);
    u.c = (void*)(f.c + (int64_t)lo * f.c_row * f.osz);
  } else {  // dW^T[K_in, N_out] = x_e^T[K_in, rows_e] dy_e[rows_e, N_out]: k = this expert's rows
    u.k = (uint32_t)rows;
    u.a = (void*)(f.a + (int64_t)lo * f.c_row * f.esz);  // x rows: pitch = K_in = out row length
    u.b = (void*)(f.b + (int64_t)lo * f.b_row * f.esz);  // dy rows: pitch = N_out
    u.c = (void*)(f.c + (int64_t)e * f.c_gstride * f.osz);
  }
  u.d = u.c;
}

Plan& plan_for(State& S, const Key& key, int mode, int G, int64_t N, int64_t K, int64_t rows, at::ScalarType odt,
               at::ScalarType edt, bool trans_w, float beta, int algo_index, const at::Tensor& like) {
  auto it = S.plans.find(key);
  if (it != S.plans.end()) return it->second;
  Plan p;
  // hipBLASLt view: D[m_lt, n_lt] = op(A)[m_lt, k] op(B)[k, n_lt]
  hipblasOperation_t opA, opB;
  int64_t m_lt, n_lt, k_lt, lda, ldb, ldc;
  if (mode == 0) {
    m_lt = N;
    n_lt = rows;
    k_lt = K;
    opA = trans_w ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // w[e] [N, K] row-major == col-major [K, N]
    lda = trans_w ? K : N;
    opB = HIPBLAS_OP_N;  // x rows [rows, K] row-major == col-major [K, rows]
    ldb = K;
    ldc = N;
  } else {
    m_lt = K;  // out[e] is [N_out = N, K_in = K] row-major == col-major [K, N]
    n_lt = N;
    k_lt = rows;
    opA = HIPBLAS_OP_N;  // x rows [rows, K] == col-major [K, rows]
    lda = K;
    opB = HIPBLAS_OP_T;  // dy rows [rows, N] == col-major [N, rows], transposed -> [rows, N]
    ldb = N;
    ldc = K;
  }
  p.gg = std::make_unique<hipblaslt_ext::GroupedGemm>(S.handle, opA, opB, hdt(edt), hdt(edt), hdt(odt), hdt(odt),
                                                      HIPBLAS_COMPUTE_32F);
  std::vector<int64_t> vm(G, m_lt), vn(G, n_lt), vk(G, k_lt), vb(G, 1), vlda(G, lda), vldb(G, ldb), vldc(G, ldc),
      vldd(G, ldc), vsa(G, lda * (opA == HIPBLAS_OP_N ? k_lt : m_lt)), vsb(G, ldb * (opB == HIPBLAS_OP_N ? n_lt : k_lt)),
      vsc(G, ldc * n_lt), vsd(G, ldc * n_lt);
  std::vector<hipblaslt_ext::GemmEpilogue> epi(G);
  std::vector<hipblaslt_ext::GemmInputs> inputs(G);
  static const float one = 1.f, zero = 0.f;
  // placeholder pointers (the device argument array replaces them): any valid device address
  void* dummy = like.data_ptr();
  for (int e = 0; e < G; ++e) {
    inputs[e].setA(dummy);
    inputs[e].setB(dummy);
    inputs[e].setC(dummy);
    inputs[e].setD(dummy);
    inputs[e].setAlpha(&one);
    inputs[e].setBeta(beta != 0.f ? &one : &zero);
  }
  hipblaslt_ext::GemmProblemType pt(opA, opB, hdt(edt), hdt(edt), hdt(odt), hdt(odt), HIPBLAS_COMPUTE_32F);
  GLT_CHECK(p.gg->setProblem(vm, vn, vk, vb, vlda, vldb, vldc, vldd, vsa, vsb, vsc, vsd, epi, inputs, pt));
  hipblaslt_ext::GemmPreference pref;
  pref.setMaxWorkspaceBytes(kWorkspace);
  std::vector<hipblasLtMatmulHeuristicResult_t> heur;
  GLT_CHECK(p.gg->algoGetHeuristic(algo_index >= 0 ? std::max(algo_index + 1, 16) : 1, pref, heur));
  TORCH_CHECK(!heur.empty(), "hipBLASLt grouped: no solution");
  size_t pick = 0;
  if (algo_index >= 0) {
    pick = (size_t)algo_index < heur.size() ? (size_t)algo_index : heur.size() - 1;
  }
  hipblasLtMatmulAlgo_t algo = heur[pick].algo;
  size_t ws = 0;
  GLT_CHECK(p.gg->isAlgoSupported(algo, ws));
  TORCH_CHECK(ws <= kWorkspace, "hipBLASLt grouped: workspace too large");
  GLT_CHECK(p.gg->initialize(algo, S.workspace.data_ptr(), true, c10::hip::getCurrentHIPStream()));
  p.index = (int)pick;
  p.kernel = p.gg->getKernelName();
  // default arguments for every group (alpha / beta / leading dimensions / epilogue); the fill kernel then
  // patches sizes and pointers per call
  std::vector<UA> host(G);
  GLT_CHECK(p.gg->getDefaultValueForDeviceUserArguments(host.data()));
  p.args = at::empty({(int64_t)(G * sizeof(UA))}, like.options().dtype(at::kByte));
  TORCH_CHECK(reinterpret_cast<uintptr_t>(p.args.data_ptr()) % 16 == 0, "grouped_lt: args alignment");
  C10_HIP_CHECK(hipMemcpyAsync(p.args.data_ptr(), host.data(), G * sizeof(UA), hipMemcpyHostToDevice,
                               c10::hip::getCurrentHIPStream()));
  return S.plans.emplace(key, std::move(p)).first->second;
}

}  // namespace

// out / a / w / offsets as described in the header; returns the index of the heuristic solution used.
// mode 0: out [R, N] (x dtype), a = x [R, K], w [G, N, K] (trans_w) or [G, K, N]
// mode 1: out [G, N, K] fp32 or x dtype, a = dy [R, N], w = x [R, K]; beta 1 accumulates
int64_t dlgm_grouped_lt(at::Tensor out, const at::Tensor& a, const at::Tensor& w, const at::Tensor& offsets,
                        int64_t mode, bool trans_w, double beta, int64_t algo_index) {
  TORCH_CHECK(out.is_cuda() && a.is_cuda() && w.is_cuda() && offsets.is_cuda(), "grouped_lt: GPU tensors");
  TORCH_CHECK(offsets.scalar_type() == at::kInt && offsets.is_contiguous(), "grouped_lt: int32 offsets");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous() && out.is_contiguous(), "grouped_lt: contiguous operands");
  TORCH_CHECK(a.scalar_type() == w.scalar_type() && (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf),
              "grouped_lt: bf16/fp16 operands");
  const int G = (int)offsets.numel() - 1;
  TORCH_CHECK(G >= 1, "grouped_lt: need at least one group");
  int64_t N, K, R = a.size(0);
  FillArgs f{};
  if (mode == 0) {
    TORCH_CHECK(w.dim() == 3 && w.size(0) == G && a.dim() == 2, "grouped_lt: w [G, ., .], x [R, K]");
    N = trans_w ? w.size(1) : w.size(2);
    K = a.size(1);
    TORCH_CHECK((trans_w ? w.size(2) : w.size(1)) == K, "grouped_lt: K mismatch");
    TORCH_CHECK(out.dim() == 2 && out.size(0) == R && out.size(1) == N && out.scalar_type() == a.scalar_type(),
                "grouped_lt: out [R, N]");
    TORCH_CHECK(beta == 0.0, "grouped_lt: the forward mode stores");
    f.a = (const char*)w.data_ptr();
    f.b = (const char*)a.data_ptr();
    f.a_gstride = w.stride(0);
    f.b_row = K;
    f.c_row = N;
  } else {
    TORCH_CHECK(mode == 1 && w.dim() == 2 && w.size(0) == R && out.dim() == 3 && out.size(0) == G,
                "grouped_lt: wgrad out [G, N, K], dy [R, N], x [R, K]");
    N = a.size(1);
    K = w.size(1);
    TORCH_CHECK(out.size(1) == N && out.size(2) == K, "grouped_lt: out [G, N, K]");
    TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == a.scalar_type(), "grouped_lt: out dtype");
    f.a = (const char*)w.data_ptr();  // x rows
    f.b = (const char*)a.data_ptr();  // dy rows
    f.b_row = N;
    f.c_row = K;
    f.c_gstride = out.stride(0);
  }
  if (R == 0 && mode == 0) return -1;
  State& S = state();
  std::lock_guard<std::mutex> lk(S.mu);
  if (S.handle == nullptr) {
    GLT_CHECK(hipblasLtCreate(&S.handle));
    S.workspace = at::empty({(int64_t)kWorkspace}, a.options().dtype(at::kByte));
  }
  const Key key{(int)mode, G, N, K, R, (int)out.scalar_type(), (int)a.scalar_type(), trans_w, beta != 0.0,
                (int)algo_index};
  Plan& p = plan_for(S, key, (int)mode, G, N, K, std::max<int64_t>(R, 1), out.scalar_type(), a.scalar_type(),
                     trans_w, (float)beta, (int)algo_index, a);
  auto st = c10::hip::getCurrentHIPStream();
  f.ua = reinterpret_cast<UA*>(p.args.data_ptr());
  f.offsets = offsets.data_ptr<int>();
  f.c = (char*)out.data_ptr();
  f.G = G;
  f.mode = (int)mode;
  f.esz = (int)a.element_size();
  f.osz = (int)out.element_size();
  fill_user_args<<<(G + 63) / 64, 64, 0, st>>>(f);
  C10_HIP_CHECK(hipGetLastError());
  GLT_CHECK(p.gg->run(p.args.data_ptr(), st));
  return p.index;
}

// The hipBLASLt kernel a cached plan runs (profiling / records); empty if no such plan.
std::string dlgm_grouped_lt_kernel(int64_t mode, int64_t G, int64_t N, int64_t K, int64_t R) {
  State& S = state();
  std::lock_guard<std::mutex> lk(S.mu);
  for (auto& kv : S.plans) {
    const Key& k = kv.first;
    if (std::get<0>(k) == mode && std::get<1>(k) == G && std::get<2>(k) == N && std::get<3>(k) == K &&
        std::get<4>(k) == R)
      return kv.second.kernel;
  }
  return "";
}
