"""Micro-benchmark of the PPO trunk (59 -> 256 x 5, ELU) forward + backward at minibatch B on cuda:0:
library Linear under bf16 autocast vs the split-K weight-gradient formulation (learning/fused_mlp.py)."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch import nn

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
dev = "cuda:0"
torch.manual_seed(0)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def mk():
    layers = []
    n = 59
    for _ in range(5):
        layers += [nn.Linear(n, 256), nn.ELU()]
        n = 256
    return nn.Sequential(*layers).to(dev)


x = torch.randn(B, 59, device=dev)
g = torch.randn(B, 256, device=dev)
res = {}
m = mk()
def base():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = m(x)
    y.float().backward(g)
res["library_bf16"] = timeit(base)
def base32():
    y = m(x)
    y.backward(g)
res["library_fp32"] = timeit(base32)

# split-K weight gradients
Wt = [l.weight.detach().to(torch.bfloat16) for l in m if isinstance(l, nn.Linear)]
for S in (16, 32, 64, 128):
    def wg(S=S):
        a = torch.randn(B, 256, device=dev, dtype=torch.bfloat16)
        return a
    A = torch.randn(B, 256, device=dev, dtype=torch.bfloat16)
    D = torch.randn(B, 256, device=dev, dtype=torch.bfloat16)
    def f(S=S):
        p = torch.bmm(D.view(S, B // S, 256).transpose(1, 2), A.view(S, B // S, 256), out_dtype=torch.float32)
        return p.sum(0)
    res[f"dW_splitK_S{S}"] = timeit(f)
def f_lib():
    return D.t().mm(A)
res["dW_library_mm"] = timeit(f_lib)
def f_db():
    return D.sum(0)
res["db_sum"] = timeit(f_db)
def f_db2():
    return D.view(64, B // 64, 256).float().sum(1).sum(0)
res["db_sum_2stage"] = timeit(f_db2)
def f_dx():
    return D.mm(Wt[1])
res["dX_mm"] = timeit(f_dx)
def f_fw():
    return torch.addmm(Wt[1][0], A, Wt[1].t())
res["fwd_addmm"] = timeit(f_fw)
print(json.dumps({k: round(v * 1000, 1) for k, v in res.items()}, indent=0))
