"""A/B of the fused trunk kernels between two builds of libppo_hip.so of one ABI, each library
timed in its own processes (round 5: two libraries loaded into ONE process timed the same kernels): the same random
16-bit inputs through ppo_mlp_forward (and ppo_mlp_backward) of library A and library B; prints the
largest differences of every output and each library's HIP-event time per launch.

    python scripts/mlp_ab.py LIB_A LIB_B [rows] [dtype: f16 | bf16] [obs]

With `obs` the forward forms its input from fp32 observations (the trainer's fused RunningMeanStd path).
"""

from __future__ import annotations

import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allsteps_isaaclab_amd.learning import fused as FU  # noqa: E402


def open_lib(path):
    L = C.CDLL(path)
    L.ppo_mlp_forward.argtypes = [C.POINTER(FU.PpoMlpFwd), C.c_void_p]
    L.ppo_mlp_backward.argtypes = [C.POINTER(FU.PpoMlpBwd), C.c_void_p]
    return L


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1000, 2)


def main():
    if sys.argv[1] == "--one":  # one library in this process: time it, save its outputs
        return one(sys.argv[2], sys.argv[3], sys.argv[4:])
    la, lb = sys.argv[1], sys.argv[2]
    rest = sys.argv[3:]
    import subprocess
    import tempfile
    tmp = tempfile.mkdtemp(prefix="mlp_ab_")
    best = {"A": [1e9, 1e9], "B": [1e9, 1e9]}
    # each library in its own processes (two libraries in one process can share kernel registrations by
    # name), alternated over rounds, each one's best kept
    for rnd in range(3):
        for tag, path in (("A", la), ("B", lb)):
            out = subprocess.run([sys.executable, __file__, "--one", path, os.path.join(tmp, tag + ".pt")] + rest,
                                 capture_output=True, text=True, check=True).stdout
            t = json.loads(out.strip().splitlines()[-1])
            best[tag] = [min(best[tag][0], t["fwd_us"]), min(best[tag][1], t["bwd_us"])]
    A = torch.load(os.path.join(tmp, "A.pt"), weights_only=True)
    B = torch.load(os.path.join(tmp, "B.pt"), weights_only=True)
    rows = int(rest[0]) if rest else 32768
    rep = {"rows": rows, "args": rest, "fwd_us": [best["A"][0], best["B"][0]], "bwd_us": [best["A"][1], best["B"][1]],
           "method": "separate processes per library, 3 alternating rounds, best per library"}
    for k in ("h", "dz"):
        rep[k + "_maxdiff"] = [round(float((p - q).abs().max()), 6) for p, q in zip(A[k], B[k])]
    rep["head_maxdiff"] = float((A["head"] - B["head"]).abs().max())
    print(json.dumps(rep), flush=True)


def one(path, save, rest):
    sys.argv = [sys.argv[0], path, path] + list(rest)
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 32768
    dt = torch.float16 if (sys.argv[4] if len(sys.argv) > 4 else "f16") == "f16" else torch.bfloat16
    use_obs = len(sys.argv) > 5 and sys.argv[5] == "obs"
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.zeros(rows, 72, device=dev)
    x[:, :59] = torch.randn(rows, 59, device=dev, generator=g).clamp(-5, 5)
    x = x.to(dt)
    ws = [(torch.randn(256, 64 if i == 0 else 256, device=dev, generator=g) / (8 if i == 0 else 16)).to(dt)
          for i in range(5)]
    ws[0][:, 59:] = 0
    wts = [w.t().contiguous() for w in ws[1:]]
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(5)]
    wh = torch.randn(22, 256, device=dev, generator=g) / 16
    bh = torch.randn(22, device=dev, generator=g) * 0.1
    dhead = torch.randn(rows, 22, device=dev, generator=g) * 0.01
    out = {}
    obs = torch.randn(2 * rows, 59, device=dev, generator=g) * 2
    midx = torch.tensor([1], device=dev, dtype=torch.int32)
    mean = torch.randn(59, device=dev, generator=g, dtype=torch.float64) * 0.1
    var = torch.rand(59, device=dev, generator=g, dtype=torch.float64) + 0.5
    dh16 = torch.zeros(rows, 32, device=dev, dtype=dt)
    dh16[:, :22] = dhead.to(dt)
    for tag, path in (("A", path),):
        L = open_lib(path)
        hs = [torch.zeros(rows, 264, device=dev, dtype=dt) for _ in range(5)]
        head = torch.zeros(rows, 22, device=dev)
        dzs = [torch.zeros(rows, 256, device=dev, dtype=dt) for _ in range(5)]
        a = FU.PpoMlpFwd()
        a.x = x.data_ptr()
        for i in range(5):
            a.w[i], a.b[i], a.h[i] = ws[i].data_ptr(), bs[i].data_ptr(), hs[i].data_ptr()
        a.wh, a.bh, a.head, a.rows, a.nh = wh.data_ptr(), bh.data_ptr(), head.data_ptr(), rows, 22
        a.x_stride, a.h_stride, a.dtype = 72, 264, FU.PPO_DT[dt]
        if use_obs:
            xo = torch.zeros(rows, 72, device=dev, dtype=dt)
            a.obs, a.mb_idx, a.mean, a.var, a.eps, a.obs_dim = (obs.data_ptr(), midx.data_ptr(), mean.data_ptr(),
                                                                var.data_ptr(), 1e-5, 59)
            a.x_out = xo.data_ptr()
        b = FU.PpoMlpBwd()
        b.dhead, b.wh, b.nh, b.rows, b.h_stride, b.dtype = dh16.data_ptr(), wh.data_ptr(), 22, rows, 264, FU.PPO_DT[dt]
        for k in range(4):
            b.wt[k] = wts[k].data_ptr()
        for k in range(5):
            b.h[k], b.dz[k] = hs[k].data_ptr(), dzs[k].data_ptr()
        s = torch.cuda.current_stream().cuda_stream
        fwd = lambda: L.ppo_mlp_forward(C.byref(a), s)  # noqa: E731
        bwd = lambda: L.ppo_mlp_backward(C.byref(b), s)  # noqa: E731
        assert fwd() == 0 and bwd() == 0
        torch.cuda.synchronize()
        out[tag] = {"h": [t[:, :256].float().clone() for t in hs], "head": head.clone(),
                    "dz": [t.float().clone() for t in dzs], "fn": (fwd, bwd), "keep": (a, b, hs, head, dzs),
                    "fwd_us": 1e9, "bwd_us": 1e9}
    fwd, bwd = out["A"]["fn"]
    for _ in range(3):
        out["A"]["fwd_us"] = min(out["A"]["fwd_us"], timed(fwd))
        out["A"]["bwd_us"] = min(out["A"]["bwd_us"], timed(bwd))
    A = out["A"]
    torch.save({"h": A["h"], "dz": A["dz"], "head": A["head"]}, save)
    print(json.dumps({"fwd_us": A["fwd_us"], "bwd_us": A["bwd_us"]}), flush=True)


if __name__ == "__main__":
    main()
