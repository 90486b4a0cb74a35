"""Time the trunk weight-gradient step at B rows, S splits: ppo_weight_grads (one MFMA launch for all
five layers) vs the five split-K torch.bmm calls it replaced (hipBLASLt), same (S, 256, w) partials."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allsteps_isaaclab_amd.learning import fused as FU  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
S = int(sys.argv[2]) if len(sys.argv) > 2 else FU._split(B)
dev = "cuda:0"
L = FU.load()
widths = [72] + [264] * 4
dz = [torch.randn(B, 256, device=dev).to(torch.bfloat16) for _ in range(5)]
hin = [torch.randn(B, w, device=dev).to(torch.bfloat16) for w in widths]
part = [torch.empty(S, 256, w, device=dev) for w in widths]
a = FU.PpoWgrad()
for k in range(5):
    a.dz[k], a.hin[k], a.part[k] = dz[k].data_ptr(), hin[k].data_ptr(), part[k].data_ptr()
    a.kin[k], a.hin_stride[k] = 64 if k == 0 else 256, widths[k]
a.rows, a.splits, a.layers, a.dtype = B, S, 5, 1  # bf16 (PPO_DT_BF16)


def kernel():
    FU._check(L.ppo_weight_grads(C.byref(a), torch.cuda.current_stream().cuda_stream), "wgrad")


def library():
    for k in range(5):
        torch.bmm(dz[k].view(S, B // S, 256).transpose(1, 2), hin[k].view(S, B // S, widths[k]), out_dtype=torch.float32)


def t(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


jobs, keep = [], []
for k in range(5):
    w, kin = widths[k], 64 if k == 0 else 256
    n_s = 256 * w
    gw = torch.empty(256, kin, device=dev)
    gb = torch.empty(256, device=dev)
    jobs += [FU.PpoReduceJob(part[k].data_ptr(), gw.data_ptr(), S, 256, w, kin, kin, n_s),
             FU.PpoReduceJob(part[k].data_ptr() + 4 * kin, gb.data_ptr(), S, 256, w, 1, 1, n_s)]
    keep += [gw, gb]
arr = (FU.PpoReduceJob * len(jobs))(*jobs)


def reduce():
    FU._check(L.ppo_reduce_rows(arr, len(jobs), torch.cuda.current_stream().cuda_stream), "reduce")


tk, tl, tr = t(kernel), (t(library) if B % S == 0 else float('nan')), t(reduce)
flops = 2 * B * 256 * (65 + 4 * 257)
in_bytes = sum(d.numel() * 2 for d in dz) + B * 2 * (64 + 4 * 256)
out_bytes = S * 256 * 4 * (65 + 4 * 257)
print(json.dumps({"rows": B, "splits": S, "kernel_us": round(tk, 1), "bmm_us": round(tl, 1), "reduce_us": round(tr, 1),
                  "kernel_tflops": round(flops / tk / 1e6, 1), "kernel_gbs": round((in_bytes + out_bytes) / tk / 1e3, 1)}))
