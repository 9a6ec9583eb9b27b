"""Round-5 flake probe, stage 3: do torch's hipBLASLt GEMMs of the Mixtral-tiny shapes return different bits when
another stream keeps compute units busy (the async shadow comm's torch.cuda._sleep spin kernels)? Each shape runs
`reps` times alone and `reps` times beside a spinning kernel on a second stream; every result is compared bit for
bit with the first alone-result. Also lists the GEMM kernels each shape launched (torch.profiler names)."""
import json
import os
import sys

import torch

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
T = 128
SHAPES = {  # (M, K, N, out dtype, accumulate): mixtral-tiny d=256, ffn=256, E=4, vocab 512, qkv 512
    "router_fwd": (T, 256, 4, torch.bfloat16, False),
    "router_dw": (4, T, 256, torch.bfloat16, True),
    "router_dx": (T, 4, 256, torch.bfloat16, False),
    "wqkv_fwd": (T, 256, 512, torch.bfloat16, False),
    "wqkv_dw": (512, T, 256, torch.bfloat16, True),
    "wo_dw": (256, T, 256, torch.bfloat16, True),
    "head_fwd": (T, 256, 512, torch.bfloat16, False),
}
reps = int(os.environ.get("REPS", "200"))
side = torch.cuda.Stream(dev)
out = {}
for name, (M, K, N, odt, acc) in SHAPES.items():
    a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    b = torch.randn(K, N, device=dev, generator=g).to(torch.bfloat16)
    c0 = torch.randn(M, N, device=dev, generator=g).to(odt)

    def run():
        c = c0.clone()
        if acc:
            torch.addmm(c, a, b, beta=1.0, out=c)
        else:
            torch.mm(a, b, out=c)
        return c
    ref = run()
    torch.cuda.synchronize()
    bad_alone = sum(int(not torch.equal(run(), ref)) for _ in range(reps))
    bad_busy = 0
    for i in range(reps):
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000 + 1000 * (i % 50))
        r = run()
        torch.cuda.synchronize()
        bad_busy += int(not torch.equal(r, ref))
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        run()
        torch.cuda.synchronize()
    kern = sorted({e.name[:90] for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA})
    out[name] = {"bad_alone": bad_alone, "bad_busy": bad_busy, "reps": reps, "kernels": kern}
    print(name, out[name], flush=True)
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/sk_race.json", "w") as f:
    json.dump(out, f, indent=1)
sys.exit(0)
