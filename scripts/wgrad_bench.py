"""Time the weight-gradient step at B rows: ppo_weight_grads (one MFMA launch: five trunk layers + the head
weights, fused.wgrad_splits) and the ppo_reduce_rows launch that sums its partials; prints HIP-event
microseconds per launch and the algorithmic bytes / FLOP rates.
    python scripts/wgrad_bench.py [rows] [dtype: f16 | bf16]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allsteps_isaaclab_amd.learning import fused as FU  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
dt = torch.float16 if (sys.argv[2] if len(sys.argv) > 2 else "f16") == "f16" else torch.bfloat16
dev = "cuda:0"
L = FU.load()
S = FU.wgrad_splits(B)
widths = [72] + [264] * 5
nout = [256] * 5 + [32]
dz = [torch.randn(B, nout[k], device=dev).to(dt) for k in range(6)]
hin = [torch.randn(B, w, device=dev).to(dt) for w in widths]
part = [torch.empty(S[k], nout[k], widths[k], device=dev) for k in range(6)]
a = FU.PpoWgrad()
for k in range(6):
    a.dz[k], a.hin[k], a.part[k] = dz[k].data_ptr(), hin[k].data_ptr(), part[k].data_ptr()
    a.kin[k], a.hin_stride[k], a.splits[k] = 64 if k == 0 else 256, widths[k], S[k]
a.rows, a.layers, a.dtype = B, 6, FU.PPO_DT[dt]


def kernel():
    FU._check(L.ppo_weight_grads(C.byref(a), torch.cuda.current_stream().cuda_stream), "wgrad")


jobs, keep = [], []
for k in range(6):
    w, kin = widths[k], 64 if k == 0 else 256
    n_s = nout[k] * w
    gw = torch.empty(nout[k], kin, device=dev)
    gb = torch.empty(nout[k], device=dev)
    jobs.append(FU.PpoReduceJob(part[k].data_ptr(), gw.data_ptr(), S[k], 22 if k == 5 else 256, w, kin, kin, n_s))
    if k < 5:
        jobs.append(FU.PpoReduceJob(part[k].data_ptr() + 4 * kin, gb.data_ptr(), S[k], 256, w, 1, 1, n_s))
    keep += [gw, gb]
arr = (FU.PpoReduceJob * len(jobs))(*jobs)


def reduce():
    FU._check(L.ppo_reduce_rows(arr, len(jobs), torch.cuda.current_stream().cuda_stream), "reduce")


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


tk, tr = t(kernel), t(reduce)
flops = 2 * B * (256 * (65 + 4 * 257) + 32 * 256)
in_bytes = sum(d.numel() * 2 for d in dz) + B * 2 * (64 + 5 * 256)
out_bytes = sum(p.numel() * 4 for p in part)
print(json.dumps({"rows": B, "splits": S, "kernel_us": round(tk, 1), "reduce_us": round(tr, 1),
                  "kernel_tflops": round(flops / tk / 1e6, 1), "kernel_in_MB": round(in_bytes / 1e6, 1),
                  "partials_MB": round(out_bytes / 1e6, 1),
                  "kernel_gbs": round((in_bytes + out_bytes) / tk / 1e3, 1)}), flush=True)
