// stream_delay_ns: make the current HIP stream wait for a wall-clock duration WITHOUT occupying a compute unit.
// ShadowComm's link model (parallel/comm.py) queues it in front of each stand-in collective so that the comm stream is
// busy for bytes / modelled xGMI bus bandwidth, as RCCL's would be: whether the engine hides that time behind compute
// is then measured on ONE MI355X.
//
// First version: a one-wave kernel spinning on s_memrealtime. It held a wave slot -- and with it the whole CU for a
// kernel that runs one 256-VGPR workgroup per CU -- so the compute kernels ran 8 % longer beside it and the model
// blamed the link for it (profiles/zero3_overlap_model_r06.json, "spin_artifact"). This one is a host function on the
// stream (hipLaunchHostFunc): the command processor holds the stream until the host thread returns, and no CU, LDS
// or VGPR is taken.
#include <torch/all.h>
#include <c10/hip/HIPStream.h>

#include <chrono>
#include <thread>

#include "dlgm_common.h"

namespace {

void sleep_cb(void* arg) {
  std::this_thread::sleep_for(std::chrono::nanoseconds(reinterpret_cast<intptr_t>(arg)));
}

}  // namespace

void dlgm_stream_delay_ns(int64_t ns) {
  TORCH_CHECK(ns >= 0 && ns < 60'000'000'000LL, "stream_delay_ns: 0 <= ns < 60 s");
  if (ns == 0) return;
  DLGM_CHECK_HIP(hipLaunchHostFunc(c10::hip::getCurrentHIPStream(), sleep_cb, reinterpret_cast<void*>(ns)));
}
