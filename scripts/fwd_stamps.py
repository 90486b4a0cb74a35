"""Per-phase cycles of the fused forward from a PPO_FWD_DBG=8 build (stamps written over h5):
    python scripts/fwd_stamps.py LIB [rows]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from allsteps_isaaclab_amd.learning import fused as FU  # noqa: E402

L = C.CDLL(sys.argv[1])
L.ppo_mlp_forward.argtypes = [C.POINTER(FU.PpoMlpFwd), C.c_void_p]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
dev, dt = "cuda:0", torch.float16
x = (torch.randn(rows, 72, device=dev) * 0.5).to(dt)
ws = [(torch.randn(256, 64 if i == 0 else 256, device=dev) / 16).to(dt) for i in range(5)]
bs = [torch.zeros(256, device=dev) for _ in range(5)]
wh, bh = torch.randn(22, 256, device=dev) / 16, torch.zeros(22, device=dev)
hs = [torch.zeros(rows, 264, device=dev, dtype=dt) for _ in range(4)]
h5 = torch.zeros(rows, 256, device=dev)
head = torch.zeros(rows, 22, device=dev)
a = FU.PpoMlpFwd()
a.x = x.data_ptr()
for i in range(5):
    a.w[i], a.b[i] = ws[i].data_ptr(), bs[i].data_ptr()
for i in range(4):
    a.h[i] = hs[i].data_ptr()
a.wh, a.bh, a.h5, a.head, a.rows, a.nh = wh.data_ptr(), bh.data_ptr(), h5.data_ptr(), head.data_ptr(), rows, 22
a.x_stride, a.h_stride, a.dtype = 72, 264, FU.PPO_DT[dt]
for _ in range(3):
    assert L.ppo_mlp_forward(C.byref(a), torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
nb = (rows + 127) // 128
st = h5.view(torch.int64).reshape(-1)[: nb * 8 * 16].view(nb, 8, 16).cpu().numpy()[:, :, :14].astype(np.float64)
d = np.diff(st, axis=2)
names = ["stage x+w0", "bar0", "L0", "bar1", "L1", "bar2", "L2", "bar3", "L3", "bar4", "L4", "bar5", "heads"]
print(f"rows {rows}: mean cycles per wave (s_memtime), total {np.mean(st[:,:,13]-st[:,:,0]):.0f}, "
      f"max {np.max(st[:,:,13]-st[:,:,0]):.0f}")
print("  ".join(f"{n} {np.mean(d[:, :, k]):.0f}" for k, n in enumerate(names)))
