// spin_ns: hold one wave on the current HIP stream for a wall-clock duration (the s_memrealtime 100 MHz counter,
// independent of the shader clock's DVFS). ShadowComm's link model (parallel/comm.py) queues it in front of each
// stand-in collective so the comm stream is busy for bytes / modelled xGMI bus bandwidth, as RCCL's would be:
// whether the engine hides that time behind compute is then measured on ONE MI355X.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>
#include "dlgm_common.h"

namespace {

__global__ __launch_bounds__(64) void spin_kernel(int64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

}  // namespace

void dlgm_spin_ns(int64_t ns) {
  TORCH_CHECK(ns >= 0 && ns < 60'000'000'000LL, "spin_ns: 0 <= ns < 60 s");
  if (ns == 0) return;
  spin_kernel<<<1, 64, 0, c10::hip::getCurrentHIPStream()>>>((ns + 9) / 10);  // 100 MHz: 10 ns per tick
  DLGM_CHECK_HIP(hipGetLastError());
}
