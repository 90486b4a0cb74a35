"""HIP-event time per launch of the PPO loss kernel at a minibatch of `rows` (A = 21): ppo_loss_grad alone and
ppo_loss_grad + ppo_loss_finalize; and of the optimizer step ppo_sqnorm + ppo_adam + ppo_tail on a
333k-element flat buffer with a row-major and a transposed fp16 mirror segment.
    python scripts/loss_bench.py [rows]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from allsteps_isaaclab_amd.learning import fused as FU  # noqa: E402


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
    return round(e0.elapsed_time(e1) / n * 1000, 2)


def main():
    L = FU.load()
    dev, A = "cuda:0", 21
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    g = torch.Generator(device=dev).manual_seed(4)
    r = lambda *sh: torch.randn(*sh, device=dev, generator=g)  # noqa: E731
    head, logstd = r(B, A + 1) * 0.5, r(A) * 0.1
    idx = torch.tensor([1], device=dev, dtype=torch.int32)
    ds = [r(2 * B, A), r(2 * B, A) * 0.3, torch.exp(r(2 * B, A) * 0.1), r(2 * B).abs() * 5 + 20, r(2 * B), r(2 * B),
          r(2 * B)]
    cfg = FU.PpoLossCfg(0.2, 4.0, 0.0, 1e-4, 1.1, 1, 1, 1)
    scale = torch.tensor([1024.0], device=dev)
    s = torch.cuda.current_stream().cuda_stream
    nblk = L.ppo_loss_blocks(B)
    dlp = torch.zeros(B, 32, device=dev, dtype=torch.float16)
    part = torch.zeros(nblk, 2 * A + 1 + 5, device=dev)
    ghb, gls, stats = torch.zeros(A + 1, device=dev), torch.zeros(A, device=dev), torch.zeros(2000, 5, device=dev)
    sidx, kl = torch.zeros(1, device=dev, dtype=torch.int32), torch.zeros(1, device=dev)
    args = (head.data_ptr(), logstd.data_ptr(), A, B, idx.data_ptr(), *[x.data_ptr() for x in ds], cfg, scale.data_ptr(),
            None, part.data_ptr(), dlp.data_ptr(), FU.PPO_DT[torch.float16])
    out = {"rows": B,
           "loss_grad_us": t(lambda: L.ppo_loss_grad(*args, s)),
           "loss_grad_then_finalize_us": t(lambda: (L.ppo_loss_grad(*args, s), L.ppo_loss_finalize(
               part.data_ptr(), nblk, A, B, 0.01, scale.data_ptr(), ghb.data_ptr(), gls.data_ptr(), stats.data_ptr(),
               sidx.data_ptr(), kl.data_ptr(), s)))}
    n = 333_333
    grads = r(n)
    p, m, v = r(n), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    nb = L.ppo_sqnorm_blocks()
    partials = torch.zeros(2 * nb, device=dev)
    mirror = torch.zeros(n, device=dev, dtype=torch.float16)
    segs = (FU.PpoSeg * 2)(FU.PpoSeg(0, 65536, 0, 256, 256, 0), FU.PpoSeg(65536, 65536, 65536, 256, 256, 1))
    lr = torch.tensor([3e-4], device=dev, dtype=torch.float64)
    step = torch.tensor([7.0], device=dev, dtype=torch.float64)
    scaler = torch.tensor([65536.0, 0.0], device=dev)
    mb, st = torch.zeros(1, device=dev, dtype=torch.int32), torch.zeros(1, device=dev, dtype=torch.int32)

    snap = torch.zeros(4, device=dev, dtype=torch.float64)

    def three():
        L.ppo_sqnorm(grads.data_ptr(), n, scaler.data_ptr(), partials.data_ptr(), None, None, None, s)
        L.ppo_adam(p.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), n, partials.data_ptr(), nb, 1.0,
                   lr.data_ptr(), step.data_ptr(), 0.9, 0.999, 1e-8, segs, 2, mirror.data_ptr(), 2, scaler.data_ptr(), s)
        L.ppo_tail(lr.data_ptr(), kl.data_ptr(), 0.008, 1e-6, 1e-2, step.data_ptr(), mb.data_ptr(), 4, st.data_ptr(),
                   scaler.data_ptr(), partials.data_ptr(), nb, 1 << 30, s)

    out["sqnorm_adam_tail_us"] = t(three)

    def two():  # the norm launch taking the snapshot, then Adam + tail in one launch (ppo_adam_step)
        L.ppo_sqnorm(grads.data_ptr(), n, scaler.data_ptr(), partials.data_ptr(), lr.data_ptr(), step.data_ptr(),
                     snap.data_ptr(), s)
        a = FU.PpoAdamStep(p.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), n, partials.data_ptr(), nb,
                           1.0, 0.9, 0.999, 1e-8, segs, 2, mirror.data_ptr(), 2, snap.data_ptr(), lr.data_ptr(),
                           kl.data_ptr(), 0.008, 1e-6, 1e-2, step.data_ptr(), mb.data_ptr(), 4, st.data_ptr(),
                           scaler.data_ptr(), 1 << 30)
        L.ppo_adam_step(C.byref(a), s)

    out["sqnorm_adam_step_us"] = t(two)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
