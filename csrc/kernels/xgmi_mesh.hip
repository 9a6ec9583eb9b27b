// Peer-write xGMI mesh all-gather: one symmetric buffer per rank, exported with HIP IPC and
// mapped into every peer; each rank's kernel writes its shard straight into all W-1 peers' buffers (one xGMI
// link per peer on an 8-GPU MI355X node, all links at once) and into its own. No ring steps, no staging, no
// library: completion is the stream order of the push kernel before a device-side barrier (parallel/xgmi_mesh.py).
//
//   ipc_alloc(nbytes)        uint8 tensor on the current device from hipMalloc (its own allocation, so its IPC
//                            handle names exactly this buffer, offset 0)
//   ipc_handle(buf)          the 64-byte hipIpcMemHandle of that buffer (CPU uint8 tensor)
//   ipc_open(handle)         map a peer's buffer into this process (hipIpcOpenMemHandle, lazy peer access);
//                            returns the device address as an int64
//   ipc_close(ptr)           unmap it
//   mesh_push(src, peers, dst_off, cap)  write src's bytes at dst_off into every peer address (int64 device tensor)
//
// Bounds: dst_off + src bytes <= cap (the symmetric buffer size every rank allocated) is checked on the host before
// the launch; the kernel moves 16-byte vectors only (src bytes and dst_off multiples of 16).
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

using namespace dlgm;

namespace {

// blockIdx.y = peer; blocks of a peer stride over the 16-byte vectors. Plain vector stores to the peer's memory
// over xGMI (no scalar stores, no atomics).
__global__ __launch_bounds__(256) void mesh_push_kernel(const uint4* __restrict__ src, int64_t n16,
                                                        const int64_t* __restrict__ peers, int64_t dst_off16) {
  uint4* dst = reinterpret_cast<uint4*>(peers[blockIdx.y]) + dst_off16;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // two vectors in flight per thread
  for (; i + stride < n16; i += 2 * stride) {
    const uint4 a = src[i], b = src[i + stride];
    dst[i] = a;
    dst[i + stride] = b;
  }
  if (i < n16) dst[i] = src[i];
}

void ipc_free(void* p) { (void)hipFree(p); }

}  // namespace

at::Tensor dlgm_ipc_alloc(int64_t nbytes) {
  TORCH_CHECK(nbytes > 0 && nbytes % 16 == 0, "ipc_alloc: a positive multiple of 16 bytes");
  void* p = nullptr;
  DLGM_CHECK_HIP(hipMalloc(&p, (size_t)nbytes));
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

void dlgm_mesh_push(const at::Tensor& src, const at::Tensor& peers, int64_t dst_off, int64_t cap) {
  TORCH_CHECK(src.is_cuda() && src.is_contiguous(), "mesh_push: contiguous GPU source");
  TORCH_CHECK(peers.is_cuda() && peers.scalar_type() == at::kLong && peers.dim() == 1 && peers.is_contiguous(),
              "mesh_push: peers must be an int64 GPU vector of device addresses");
  const int64_t nbytes = src.numel() * src.element_size();
  TORCH_CHECK(nbytes % 16 == 0 && dst_off % 16 == 0 && reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "mesh_push: 16-byte aligned source, size and offset");
  TORCH_CHECK(dst_off >= 0 && dst_off + nbytes <= cap, "mesh_push: write past the symmetric buffer");
  const int64_t np = peers.numel();
  if (np == 0 || nbytes == 0) return;
  TORCH_CHECK(np <= 64, "mesh_push: at most 64 peers");
  const int64_t n16 = nbytes / 16;
  const int64_t bx = std::max<int64_t>(1, std::min<int64_t>((n16 + 511) / 512, 1024 / np * 4));
  mesh_push_kernel<<<dim3((unsigned)bx, (unsigned)np), 256, 0, c10::hip::getCurrentHIPStream()>>>(
      reinterpret_cast<const uint4*>(src.data_ptr()), n16, peers.data_ptr<int64_t>(), dst_off / 16);
  DLGM_CHECK_HIP(hipGetLastError());
}
