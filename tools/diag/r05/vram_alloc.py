"""Round 5: time one process's allocation of N GiB of device memory (1 GiB tensors) and a fill of it. Run twice in a
row: does a process pay for VRAM another process has just freed (the 4.6-5.7 s engine construction of every
process after the first on a box)?"""
import json
import os
import sys
import time

import torch

n = int(float(os.environ.get("VRAM", "160")))
t0 = time.time()
torch.cuda.init()
torch.empty(1, device="cuda")
torch.cuda.synchronize()
init_s = time.time() - t0
t0 = time.time()
bufs = [torch.empty(1 << 30, dtype=torch.uint8, device="cuda") for _ in range(n)]
torch.cuda.synchronize()
alloc_s = time.time() - t0
t0 = time.time()
for b in bufs:
    b.fill_(7)
torch.cuda.synchronize()
fill_s = time.time() - t0
print(json.dumps({"tag": sys.argv[1] if len(sys.argv) > 1 else "", "GiB": n, "init_s": round(init_s, 2),
                  "alloc_s": round(alloc_s, 2), "fill_s": round(fill_s, 2)}), flush=True)
