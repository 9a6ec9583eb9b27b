// Operator registry for the MI355X-native kernels: torch.ops.dlgm.*
//
// Registered with TORCH_LIBRARY so the ops are dispatcher-visible (usable
// from Python, capturable in HIP graphs, and loaded by torch.ops.load_library
// from the in-tree shared object -- never a pip-installed extension).
// Only the CUDA (= HIP on ROCm) dispatch key is implemented: CPU tensors take the
// plain PyTorch reference path in the Python wrappers, GPU tensors must hit
// these kernels.
#include <torch/library.h>
#include <torch/all.h>

// rmsnorm.hip
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_rmsnorm_fwd(const at::Tensor& x,
                                                                const c10::optional<at::Tensor>& residual,
                                                                const at::Tensor& w, double eps);
at::Tensor dlgm_rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w, const at::Tensor& rstd,
                            const c10::optional<at::Tensor>& dres, at::Tensor dw, bool accumulate_dw);
// rope.hip
void dlgm_rope_(at::Tensor qkv, const at::Tensor& cos_t, const at::Tensor& sin_t,
                const c10::optional<at::Tensor>& pos_ids, int64_t n_rope_heads, int64_t head_dim, int64_t seq_len,
                bool inverse);
// swiglu.hip
at::Tensor dlgm_swiglu_fwd(const at::Tensor& gu, const c10::optional<at::Tensor>& nrows);
at::Tensor dlgm_swiglu_bwd(const at::Tensor& dy, const at::Tensor& gu, const c10::optional<at::Tensor>& nrows);
// cross_entropy.hip
std::tuple<at::Tensor, at::Tensor> dlgm_cross_entropy_(at::Tensor logits, const at::Tensor& labels,
                                                       int64_t ignore_index, double grad_scale, bool compute_grad,
                                                       const c10::optional<at::Tensor>& scale);
// optim.hip
void dlgm_grad_stats(at::TensorList grads, at::Tensor out, bool accumulate);
void dlgm_adamw_step_(at::Tensor p, at::Tensor m, at::Tensor v, const at::Tensor& g,
                      const c10::optional<at::Tensor>& p16, const c10::optional<at::Tensor>& stats, double lr,
                      double beta1, double beta2, double eps, double weight_decay, double bc1, double bc2,
                      double grad_scale, double max_norm, const c10::optional<at::Tensor>& scale_state);
void dlgm_loss_scale_update_(at::Tensor state, const at::Tensor& stats, int64_t window, int64_t hysteresis,
                             double min_scale);
void dlgm_accumulate_(at::Tensor dst, const at::Tensor& src, double alpha, double beta);
void dlgm_cast_f32_bf16_(at::Tensor dst, const at::Tensor& src);
// flash_attn.hip
std::tuple<at::Tensor, at::Tensor> dlgm_flash_attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                       double softmax_scale, bool causal);
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_flash_attn_bwd(const at::Tensor& dout, const at::Tensor& q,
                                                                   const at::Tensor& k, const at::Tensor& v,
                                                                   const at::Tensor& out, const at::Tensor& lse,
                                                                   double softmax_scale, bool causal,
                                                                   const c10::optional<at::Tensor>& dqkv);

// moe.hip
at::Tensor dlgm_moe_combine_fwd(const at::Tensor& y, const at::Tensor& pos, const c10::optional<at::Tensor>& gates);
std::tuple<at::Tensor, at::Tensor> dlgm_moe_combine_bwd(const at::Tensor& dout, const at::Tensor& y,
                                                        const at::Tensor& pos, const at::Tensor& gates);
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_moe_permute(const at::Tensor& topi, int64_t n_experts);
std::tuple<at::Tensor, at::Tensor> dlgm_moe_pad_plan(const at::Tensor& offsets, int64_t padded_rows, int64_t align);
std::tuple<at::Tensor, at::Tensor> dlgm_moe_pad_plan_multi(const at::Tensor& offsets, int64_t padded_rows,
                                                            int64_t align);
// transpose.hip
at::Tensor dlgm_transpose(const at::Tensor& x, const c10::optional<at::Tensor>& out,
                          const c10::optional<at::Tensor>& rows);
at::Tensor dlgm_transpose_multi(const std::vector<at::Tensor>& xs, const at::Tensor& rows);
// embedding.hip
at::Tensor dlgm_embedding_fwd(const at::Tensor& table, const at::Tensor& ids);
void dlgm_embedding_bwd_(at::Tensor grad, const at::Tensor& dy, const at::Tensor& sorted_ids, const at::Tensor& order);
std::tuple<at::Tensor, at::Tensor, at::Tensor> dlgm_router_topk(const at::Tensor& logits, int64_t k);
// gemm_lt.hip
int64_t dlgm_gemm_lt(at::Tensor out, const at::Tensor& a, const at::Tensor& b, double beta, int64_t algo_index);
at::Tensor dlgm_gemm_lt_tune(const at::Tensor& out, const at::Tensor& a, const at::Tensor& b, double beta,
                             int64_t n_heuristic, bool all_algos, int64_t reps);
int64_t dlgm_gemm_lt_version();
// gemm_mfma.hip
void dlgm_gemm_mfma(at::Tensor out, const at::Tensor& a, const at::Tensor& b, bool accumulate,
                    const c10::optional<at::Tensor>& offsets, int64_t mode, int64_t M, int64_t N, int64_t K,
                    int64_t G, int64_t b_gstride, const c10::optional<at::Tensor>& stats_part,
                    const c10::optional<at::Tensor>& glu);
void dlgm_gemm_mfma_seg(at::Tensor out, const std::vector<at::Tensor>& a, const std::vector<at::Tensor>& b,
                        const at::Tensor& offsets, bool accumulate, bool kmajor);

// xgmi_mesh.hip
at::Tensor dlgm_ipc_alloc(int64_t nbytes, int64_t mode);
at::Tensor dlgm_ipc_handle(const at::Tensor& buf);
int64_t dlgm_ipc_open(const at::Tensor& handle);
void dlgm_ipc_close(int64_t ptr);
int64_t dlgm_mesh_flag_bytes();
int64_t dlgm_mesh_state_words();
void dlgm_mesh_sync(at::Tensor state, const at::Tensor& peers, int64_t me, int64_t ch, int64_t inc, int64_t val,
                    int64_t store_kind, int64_t wait_kind, int64_t lag, int64_t timeout);
void dlgm_mesh_pull(at::Tensor out, const at::Tensor& peers, int64_t src_off, int64_t heap_bytes);
void dlgm_mesh_rs_push(const at::Tensor& x, const at::Tensor& peers, at::Tensor state, int64_t me, int64_t ch,
                       int64_t region_off, int64_t slot_bytes, int64_t rank_stride, int64_t slots,
                       int64_t heap_bytes, bool fp32_slots);
void dlgm_mesh_rs_reduce(at::Tensor out, double scale, bool accumulate, const at::Tensor& peers, at::Tensor state,
                         int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes, int64_t rank_stride,
                         int64_t slots, int64_t heap_bytes, bool fp32_slots);
std::vector<int64_t> dlgm_mesh_plan_layout(int64_t W, int64_t E);
void dlgm_stream_delay_ns(int64_t ns);
void dlgm_mesh_ep_plan(const at::Tensor& offsets, at::Tensor plan, int64_t capacity, const at::Tensor& peers,
                       at::Tensor state, int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes,
                       int64_t slots, int64_t heap_bytes, int64_t timeout);
void dlgm_mesh_push_rows(const at::Tensor& x, const at::Tensor& plan, bool combine, const at::Tensor& peers,
                         at::Tensor state, int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes,
                         int64_t hdr_bytes, int64_t slots, int64_t slot_rows, int64_t heap_bytes, int64_t n_experts);
void dlgm_mesh_copy_rows(at::Tensor out, const c10::optional<at::Tensor>& nrows, const at::Tensor& peers,
                         at::Tensor state, int64_t me, int64_t ch, int64_t region_off, int64_t slot_bytes,
                         int64_t hdr_bytes, int64_t slots, int64_t heap_bytes);

TORCH_LIBRARY(dlgm, m) {
  m.def("rmsnorm_fwd(Tensor x, Tensor? residual, Tensor w, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor h, Tensor w, Tensor rstd, Tensor? dres, Tensor(a!) dw, bool accumulate_dw) -> Tensor");
  m.def("rope_(Tensor(a!) qkv, Tensor cos, Tensor sin, Tensor? pos_ids, int n_rope_heads, int head_dim, int seq_len, bool inverse) -> ()");
  m.def("swiglu_fwd(Tensor gu, Tensor? nrows=None) -> Tensor");
  m.def("swiglu_bwd(Tensor dy, Tensor gu, Tensor? nrows=None) -> Tensor");
  m.def("cross_entropy_(Tensor(a!) logits, Tensor labels, int ignore_index, float grad_scale, bool compute_grad, Tensor? scale=None) -> (Tensor, Tensor)");
  m.def("grad_stats(Tensor[] grads, Tensor(a!) out, bool accumulate) -> ()");
  m.def("adamw_step_(Tensor(a!) p, Tensor(b!) m, Tensor(c!) v, Tensor g, Tensor(d!)? p16, Tensor? stats, float lr, float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2, float grad_scale, float max_norm, Tensor? scale_state=None) -> ()");
  m.def("loss_scale_update_(Tensor(a!) state, Tensor stats, int window, int hysteresis, float min_scale) -> ()");
  m.def("accumulate_(Tensor(a!) dst, Tensor src, float alpha, float beta) -> ()");
  m.def("cast_f32_bf16_(Tensor(a!) dst, Tensor src) -> ()");
  m.def("flash_attn_fwd(Tensor q, Tensor k, Tensor v, float softmax_scale, bool causal) -> (Tensor, Tensor)");
  m.def("moe_combine_fwd(Tensor y, Tensor pos, Tensor? gates) -> Tensor");
  m.def("moe_combine_bwd(Tensor dout, Tensor y, Tensor pos, Tensor gates) -> (Tensor, Tensor)");
  m.def("moe_permute(Tensor topi, int n_experts) -> (Tensor, Tensor, Tensor)");
  m.def("moe_pad_plan(Tensor offsets, int padded_rows, int align) -> (Tensor, Tensor)");
  m.def("moe_pad_plan_multi(Tensor offsets, int padded_rows, int align) -> (Tensor, Tensor)");
  m.def("transpose_multi(Tensor[] xs, Tensor rows) -> Tensor");
  m.def("transpose(Tensor x, Tensor(a!)? out=None, Tensor? rows=None) -> Tensor");
  m.def("flash_attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor out, Tensor lse, float softmax_scale, bool causal, Tensor(a!)? dqkv=None) -> (Tensor, Tensor, Tensor)");
  m.def("embedding_fwd(Tensor table, Tensor ids) -> Tensor");
  m.def("embedding_bwd_(Tensor(a!) grad, Tensor dy, Tensor sorted_ids, Tensor order) -> ()");
  m.def("router_topk(Tensor logits, int k) -> (Tensor, Tensor, Tensor)");
  m.def("gemm_lt(Tensor(a!) out, Tensor a, Tensor b, float beta, int algo) -> int");
  m.def("gemm_lt_tune(Tensor out, Tensor a, Tensor b, float beta, int n_heuristic, bool all_algos, int reps) -> Tensor");
  m.def("gemm_lt_version() -> int", &dlgm_gemm_lt_version);
  m.def("stream_delay_ns(int ns) -> ()", &dlgm_stream_delay_ns);
  m.def("ipc_alloc(int nbytes, int mode=0) -> Tensor", &dlgm_ipc_alloc);
  m.def("ipc_handle(Tensor buf) -> Tensor", &dlgm_ipc_handle);
  m.def("ipc_open(Tensor handle) -> int", &dlgm_ipc_open);
  m.def("ipc_close(int ptr) -> ()", &dlgm_ipc_close);
  m.def("mesh_flag_bytes() -> int", &dlgm_mesh_flag_bytes);
  m.def("mesh_state_words() -> int", &dlgm_mesh_state_words);
  m.def("mesh_plan_layout(int W, int E) -> int[]", &dlgm_mesh_plan_layout);
  m.def("mesh_sync(Tensor(a!) state, Tensor peers, int me, int ch, int inc, int val, int store_kind, int wait_kind, int lag, int timeout) -> ()");
  m.def("mesh_pull(Tensor(a!) out, Tensor peers, int src_off, int heap_bytes) -> ()");
  m.def("mesh_rs_push(Tensor x, Tensor peers, Tensor(a!) state, int me, int ch, int region_off, int slot_bytes, int rank_stride, int slots, int heap_bytes, bool fp32_slots=False) -> ()");
  m.def("mesh_rs_reduce(Tensor(a!) out, float scale, bool accumulate, Tensor peers, Tensor(b!) state, int me, int ch, int region_off, int slot_bytes, int rank_stride, int slots, int heap_bytes, bool fp32_slots=False) -> ()");
  m.def("mesh_ep_plan(Tensor offsets, Tensor(a!) plan, int capacity, Tensor peers, Tensor(b!) state, int me, int ch, int region_off, int slot_bytes, int slots, int heap_bytes, int timeout) -> ()");
  m.def("mesh_push_rows(Tensor x, Tensor plan, bool combine, Tensor peers, Tensor(a!) state, int me, int ch, int region_off, int slot_bytes, int hdr_bytes, int slots, int slot_rows, int heap_bytes, int n_experts) -> ()");
  m.def("mesh_copy_rows(Tensor(a!) out, Tensor? nrows, Tensor peers, Tensor(b!) state, int me, int ch, int region_off, int slot_bytes, int hdr_bytes, int slots, int heap_bytes) -> ()");
  m.def("gemm_mfma(Tensor(a!) out, Tensor a, Tensor b, bool accumulate, Tensor? offsets, int mode, int M, int N, int K, int G, int b_gstride, Tensor(b!)? stats_part=None, Tensor? glu=None) -> ()");
  m.def("gemm_mfma_seg(Tensor(a!) out, Tensor[] a, Tensor[] b, Tensor offsets, bool accumulate, bool kmajor=False) -> ()");
}

TORCH_LIBRARY_IMPL(dlgm, CUDA, m) {
  m.impl("rmsnorm_fwd", &dlgm_rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &dlgm_rmsnorm_bwd);
  m.impl("rope_", &dlgm_rope_);
  m.impl("swiglu_fwd", &dlgm_swiglu_fwd);
  m.impl("swiglu_bwd", &dlgm_swiglu_bwd);
  m.impl("cross_entropy_", &dlgm_cross_entropy_);
  m.impl("grad_stats", &dlgm_grad_stats);
  m.impl("adamw_step_", &dlgm_adamw_step_);
  m.impl("loss_scale_update_", &dlgm_loss_scale_update_);
  m.impl("accumulate_", &dlgm_accumulate_);
  m.impl("cast_f32_bf16_", &dlgm_cast_f32_bf16_);
  m.impl("flash_attn_fwd", &dlgm_flash_attn_fwd);
  m.impl("flash_attn_bwd", &dlgm_flash_attn_bwd);
  m.impl("moe_combine_fwd", &dlgm_moe_combine_fwd);
  m.impl("moe_combine_bwd", &dlgm_moe_combine_bwd);
  m.impl("moe_permute", &dlgm_moe_permute);
  m.impl("moe_pad_plan", &dlgm_moe_pad_plan);
  m.impl("moe_pad_plan_multi", &dlgm_moe_pad_plan_multi);
  m.impl("transpose_multi", &dlgm_transpose_multi);
  m.impl("transpose", &dlgm_transpose);
  m.impl("embedding_fwd", &dlgm_embedding_fwd);
  m.impl("embedding_bwd_", &dlgm_embedding_bwd_);
  m.impl("router_topk", &dlgm_router_topk);
  m.impl("gemm_lt", &dlgm_gemm_lt);
  m.impl("gemm_lt_tune", &dlgm_gemm_lt_tune);
  m.impl("gemm_mfma", &dlgm_gemm_mfma);
  m.impl("gemm_mfma_seg", &dlgm_gemm_mfma_seg);
  m.impl("mesh_sync", &dlgm_mesh_sync);
  m.impl("mesh_pull", &dlgm_mesh_pull);
  m.impl("mesh_rs_push", &dlgm_mesh_rs_push);
  m.impl("mesh_rs_reduce", &dlgm_mesh_rs_reduce);
  m.impl("mesh_ep_plan", &dlgm_mesh_ep_plan);
  m.impl("mesh_push_rows", &dlgm_mesh_push_rows);
  m.impl("mesh_copy_rows", &dlgm_mesh_copy_rows);
}
