"""Round-5 flake probe, stage 4: do torch's BLAS calls of the Mixtral router (N or K = n_experts = 4: 8-byte rows)
write outside their output, or read their inputs differently depending on what lies next to them? Every output is
placed inside a larger buffer filled with a canary; the canary must survive and the result must not depend on the
neighbouring bytes of the inputs (inputs placed before a region of NaN / of zeros). hipBLASLt and rocBLAS both."""
import json
import os

import torch

dev = torch.device("cuda", 0)
T, D, E = 128, 256, 4
res = {}


def place(shape, dtype, fill, pad=4096, stride=None):
    """A tensor of `shape` inside a flat buffer whose remaining elements hold `fill`."""
    n = 1
    for s in shape:
        n *= s
    buf = torch.full((pad + n + pad,), fill, dtype=dtype, device=dev)
    t = buf[pad:pad + n].view(shape)
    return buf, t


def case(name, fn, out_shape, out_dtype, inputs):
    out = {}
    for lib in ("hipblaslt", "rocblas"):
        torch.backends.cuda.preferred_blas_library("cublaslt" if lib == "hipblaslt" else "cublas")
        results = []
        canary_ok = True
        for fill in (float("nan"), 0.0, 1e30):
            ins = []
            for shp, transpose in inputs:
                src = torch.randn(shp, generator=torch.Generator().manual_seed(len(ins) + 7)).to(torch.bfloat16)
                _, t = place(shp, torch.bfloat16, fill)
                t.copy_(src.to(dev))
                ins.append(t.t() if transpose else t)
            obuf, o = place(out_shape, out_dtype, 1234.5)
            o.zero_()
            fn(o, *ins)
            torch.cuda.synchronize()
            pad = 4096
            canary_ok &= bool((obuf[:pad] == 1234.5).all() and (obuf[pad + o.numel():] == 1234.5).all())
            results.append(o.float().cpu())
        same = all(torch.equal(results[0], r) for r in results[1:])
        out[lib] = {"canary_intact": canary_ok, "same_for_any_neighbour": same,
                    "finite": bool(torch.isfinite(results[0]).all())}
    res[name] = out
    print(name, out, flush=True)


# router logits: hn2 [T, D] @ router[E, D].t() -> [T, E] (8-byte output rows)
case("router_fwd", lambda o, a, b: torch.mm(a, b, out=o), (T, E), torch.bfloat16, [((T, D), False), ((E, D), True)])
# router weight gradient: dl.t() [E, T] (a transposed view, lda = E) @ hn2 [T, D] accumulated into [E, D]
case("router_dw", lambda o, a, b: torch.addmm(o, a, b, beta=1.0, out=o), (E, D), torch.bfloat16,
     [((T, E), True), ((T, D), False)])
# router input gradient: dl [T, E] @ router [E, D] (K = 4)
case("router_dx", lambda o, a, b: o.copy_(torch.mm(a, b)), (T, D), torch.bfloat16, [((T, E), False), ((E, D), False)])
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/gemm_canary.json", "w") as f:
    json.dump(res, f, indent=1)
