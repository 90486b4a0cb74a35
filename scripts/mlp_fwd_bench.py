"""Time ppo_mlp_forward (fused MFMA trunk) vs the hipBLASLt addmm + ELU chain at B rows."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from allsteps_isaaclab_amd.learning import fused as FU  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
dev = "cuda:0"
L = FU.load()
x = torch.randn(B, 64, device=dev).to(torch.bfloat16)
ws = [(torch.randn(256, 64 if i == 0 else 256, device=dev) / 16).to(torch.bfloat16) for i in range(5)]
bs = [torch.zeros(256, device=dev) for _ in range(5)]
bsb = [b.to(torch.bfloat16) for b in bs]
wh, bh = torch.randn(22, 256, device=dev) / 16, torch.zeros(22, device=dev)
hs = [torch.empty(B, 256, device=dev, dtype=torch.bfloat16) for _ in range(5)]
head = torch.empty(B, 22, device=dev)
a = FU.PpoMlpFwd()
a.x = x.data_ptr()
for i in range(5):
    a.w[i], a.b[i], a.h[i] = ws[i].data_ptr(), bs[i].data_ptr(), hs[i].data_ptr()
a.wh, a.bh, a.head, a.rows, a.nh = wh.data_ptr(), bh.data_ptr(), head.data_ptr(), B, 22
a.x_stride, a.h_stride, a.dtype = 64, 256, 1  # bf16 (PPO_DT_BF16)


def fused(store=True):
    if not store:
        b = FU.PpoMlpFwd.from_buffer_copy(a)
        for i in range(5):
            b.h[i] = None
        FU._check(L.ppo_mlp_forward(C.byref(b), torch.cuda.current_stream().cuda_stream), "fwd")
        return
    FU._check(L.ppo_mlp_forward(C.byref(a), torch.cuda.current_stream().cuda_stream), "fwd")


def lib():
    h = x
    for i in range(5):
        torch.addmm(bsb[i], h, ws[i].t(), out=hs[i])
        F.elu(hs[i], inplace=True)
        h = hs[i]
    torch.addmm(bh, hs[4].float(), wh.t(), out=head)


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
    return round(e0.elapsed_time(e1) / n * 1000, 1)


print(json.dumps({"rows": B, "fused_us": t(fused), "fused_nostore_us": t(lambda: fused(False)), "library_us": t(lib)}))
