"""Weight-gradient GEMM variants at B rows: dW = dz^T h as split-K bmm (S chunks), fp32 out."""
import json
import sys

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
dev = "cuda:0"
dz = torch.randn(B, 256, device=dev).to(torch.bfloat16)
res = {}


def t(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1000, 1)


for w in (256, 264, 320):
    h = torch.randn(B, w, device=dev).to(torch.bfloat16)
    for S in (4, 8, 16, 32, 64, 128):
        res[f"w{w}_S{S}"] = t(lambda: torch.bmm(dz.view(S, B // S, 256).transpose(1, 2), h.view(S, B // S, w),
                                                 out_dtype=torch.float32))
    hT = h.t().contiguous()
    for S in (16, 32, 64):
        # K-major activations (feature-major storage)
        res[f"w{w}_S{S}_kmajor"] = t(lambda: torch.bmm(dz.view(S, B // S, 256).transpose(1, 2),
                                                        hT.view(w, S, B // S).permute(1, 2, 0), out_dtype=torch.float32))
print(json.dumps(res))
