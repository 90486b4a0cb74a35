"""The PPO minibatch step as two HIP graphs (MI355X-first replacement of rl_games' autograd step).

rl_games 1.6.1 (``a2c_continuous.py::calc_gradients`` + ``trancate_gradients_and_step`` +
``a2c_common.py::train_epoch``) runs, per minibatch, an autograd forward/backward of
``ModelA2CContinuousLogStd`` under autocast, the PPO losses, ``clip_grad_norm_``, Adam, then the
adaptive LR from the KL -- ~300 kernel launches and several host round trips per minibatch.  Here
the same maths is an explicit forward / backward:

* trunk (59 -> 256 x 5, ELU) in fp16 (rl_games' autocast type; bf16 selectable) on the fused MFMA
  kernels, or on hipBLASLt: ``addmm`` forward, ``dz @ W`` for the input
  gradients, and the weight gradients as a **split-K** batched GEMM (``bmm`` over S row chunks,
  fp32 out, summed) -- the library's single ``dz^T h`` with K = 32768 and a 256 x 256 output runs on 16
  workgroups (measured 113 us vs 29 us split, scripts/mlp_microbench.py);
* heads (mu | value, 22 x 256) on the 16-bit layer-5 activations with fp32 accumulation and a 16-bit
  output, as autocast runs them (MFMA trunk); the losses and everything after them in fp32;
* ``libppo_hip.so`` (include/ppo.h) for the rest: obs normaliser update + normalise, the fused
  loss / KL / head-gradient kernel, ELU backward with bias-gradient partials, clip + Adam over the flat
  buffer (writing the fp16 / bf16 trunk mirror), adaptive LR and the device minibatch counter;
* ``mixed_precision``'s ``torch.cuda.amp.GradScaler`` on the device: the loss scale (2^16, x2 after
  2000 good steps, x0.5 and the step skipped on a non-finite gradient) enters the head gradients and
  leaves in the Adam kernel -- the fp16 input gradients of the trunk do not underflow;
* graph A = forward + losses + backward (gradients and the KL land in the flat [grads | kl] bucket),
  graph B = clip + Adam + LR; in multi-GPU ``allreduce`` mode the RCCL all-reduce of the bucket runs
  between them.  Minibatch rows are addressed through a device counter, so one graph serves every
  minibatch; two variants of A exist (obs normaliser updating: first mini-epoch; frozen: the rest).
  With nothing between A and B (one GPU, or the rollout all-gather mode) a whole mini-epoch's A, B,
  A, B, ... is captured as ONE graph (``run_minibatches``), one launch per mini-epoch.

``compute_dtype=torch.float32`` runs the same schedule in fp32 (tests compare it with autograd).
"""

from __future__ import annotations

import ctypes as C
import os

import torch
import torch.nn.functional as F

from .._native import PPO_LIB_PATH, NativeError, check_build_id

_LIB = None
PPO_ABI_VERSION = 5
PPO_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
SCALER_GROWTH_INTERVAL = 2000  # torch.cuda.amp.GradScaler defaults (rl_games builds it with defaults)
SCALER_INIT = 2.0 ** 16
PPO_LOSS_NSTAT = 5


class PpoLossCfg(C.Structure):
    _fields_ = [("e_clip", C.c_float), ("critic_coef", C.c_float), ("entropy_coef", C.c_float),
                ("bounds_coef", C.c_float), ("soft_bound", C.c_float), ("ppo", C.c_int32),
                ("clip_value", C.c_int32), ("bound_loss", C.c_int32)]


class PpoReduceJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("S", C.c_int32), ("out_rows", C.c_int32),
                ("src_cols", C.c_int32), ("dst_cols", C.c_int32), ("dst_stride", C.c_int32), ("src_n", C.c_int64)]


class PpoFwdLoss(C.Structure):
    _fields_ = [("A", C.c_int32), ("logstd", C.c_void_p), ("actions", C.c_void_p), ("ds_mu", C.c_void_p),
                ("ds_sigma", C.c_void_p), ("old_neglogp", C.c_void_p), ("advantages", C.c_void_p),
                ("old_values", C.c_void_p), ("returns", C.c_void_p), ("cfg", PpoLossCfg), ("grad_scale", C.c_void_p),
                ("dhead_lp", C.c_void_p), ("partials", C.c_void_p)]


class PpoMlpFwd(C.Structure):
    _fields_ = [("x", C.c_void_p), ("w", C.c_void_p * 5), ("b", C.c_void_p * 5), ("wh", C.c_void_p),
                ("bh", C.c_void_p), ("h", C.c_void_p * 5), ("head", C.c_void_p),
                ("rows", C.c_int32), ("nh", C.c_int32), ("x_stride", C.c_int32), ("h_stride", C.c_int32),
                ("dtype", C.c_int32), ("obs", C.c_void_p), ("mb_idx", C.c_void_p), ("mean", C.c_void_p),
                ("var", C.c_void_p), ("x_out", C.c_void_p), ("eps", C.c_float), ("obs_dim", C.c_int32),
                ("loss", PpoFwdLoss)]


class PpoMlpBwd(C.Structure):
    _fields_ = [("dhead", C.c_void_p), ("wh", C.c_void_p), ("wt", C.c_void_p * 4),
                ("h", C.c_void_p * 5), ("dz", C.c_void_p * 5), ("rows", C.c_int32), ("nh", C.c_int32),
                ("h_stride", C.c_int32), ("dtype", C.c_int32)]


class PpoLossSide(C.Structure):
    _fields_ = [("partials", C.c_void_p), ("nblk", C.c_int32), ("A", C.c_int32), ("mb_rows", C.c_int32),
                ("entropy_coef", C.c_float), ("grad_scale", C.c_void_p), ("grad_head_bias", C.c_void_p),
                ("grad_logstd", C.c_void_p), ("stats", C.c_void_p), ("stat_idx", C.c_void_p), ("kl_out", C.c_void_p)]


class PpoWgrad(C.Structure):
    _fields_ = [("dz", C.c_void_p * 6), ("hin", C.c_void_p * 6), ("part", C.c_void_p * 6), ("kin", C.c_int32 * 6),
                ("hin_stride", C.c_int32 * 6), ("splits", C.c_int32 * 6), ("rows", C.c_int32), ("layers", C.c_int32),
                ("dtype", C.c_int32), ("loss", PpoLossSide)]


class PpoSeg(C.Structure):
    _fields_ = [("off", C.c_int64), ("len", C.c_int64), ("moff", C.c_int64), ("cols", C.c_int32),
                ("mstride", C.c_int32), ("trans", C.c_int32)]


class PpoAdamStep(C.Structure):
    _fields_ = [("p", C.c_void_p), ("g", C.c_void_p), ("m", C.c_void_p), ("v", C.c_void_p), ("n", C.c_int64),
                ("norm_partials", C.c_void_p), ("nblk_norm", C.c_int32), ("max_norm", C.c_float),
                ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float), ("segs_host", C.POINTER(PpoSeg)),
                ("nseg", C.c_int32), ("mirror", C.c_void_p), ("mirror_dtype", C.c_int32), ("snap", C.c_void_p),
                ("lr", C.c_void_p), ("kl", C.c_void_p), ("kl_threshold", C.c_float), ("min_lr", C.c_double),
                ("max_lr", C.c_double), ("step", C.c_void_p), ("mb_idx", C.c_void_p), ("n_minibatches", C.c_int32),
                ("stat_idx", C.c_void_p), ("scaler", C.c_void_p), ("growth_interval", C.c_int32)]


EXPORTED_SYMBOLS = ["ppo_abi_version", "ppo_last_error", "ppo_obs_stats_blocks", "ppo_obs_stats",
                    "ppo_obs_stats_update", "ppo_obs_normalize", "ppo_loss_blocks", "ppo_loss_grad",
                    "ppo_loss_finalize", "ppo_elu_bwd_blocks", "ppo_elu_bwd", "ppo_sqnorm_blocks", "ppo_sqnorm",
                    "ppo_adam", "ppo_tail", "ppo_reduce_rows", "ppo_policy_sample", "ppo_counter_add",
                    "ppo_mlp_forward", "ppo_rollout_post_blocks", "ppo_rollout_post", "ppo_meter_update",
                    "ppo_mlp_backward", "ppo_weight_grads", "ppo_build_id", "ppo_reduce_rows_norm", "ppo_adam_step"]


def load() -> C.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.environ.get("PPO_HIP_LIB", PPO_LIB_PATH)
    if not os.path.exists(path):
        raise NativeError(f"{path} not found: the PPO HIP kernels are not built "
                          f"(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = C.CDLL(path)
    V, I32, I64, F32, F64 = C.c_void_p, C.c_int32, C.c_int64, C.c_float, C.c_double
    L.ppo_obs_stats.argtypes = [V, V, I32, I32, V, V]
    L.ppo_obs_stats_update.argtypes = [V, I32, I32, I32, V, V, V, V]
    L.ppo_obs_normalize.argtypes = [V, V, I32, I32, V, V, F32, V, I32, I32, I32, V]
    L.ppo_loss_grad.argtypes = [V, V, I32, I32, V, V, V, V, V, V, V, V, PpoLossCfg, V, V, V, V, I32, V]
    L.ppo_loss_finalize.argtypes = [V, I32, I32, I32, F32, V, V, V, V, V, V, V]
    L.ppo_elu_bwd.argtypes = [V, I32, V, I32, V, I32, I32, I32, V, V]
    L.ppo_sqnorm.argtypes = [V, I64, V, V, V, V, V, V]
    L.ppo_adam.argtypes = [V, V, V, V, I64, V, I32, F32, V, V, F32, F32, F32, C.POINTER(PpoSeg), I32, V, I32, V, V]
    L.ppo_tail.argtypes = [V, V, F32, F64, F64, V, V, I32, V, V, V, I32, I32, V]
    L.ppo_reduce_rows.argtypes = [C.POINTER(PpoReduceJob), I32, V]
    L.ppo_reduce_rows_norm.argtypes = [C.POINTER(PpoReduceJob), I32, V, V, I32, V, I32, V, I32, C.POINTER(I32), V, V,
                                       V, V]
    L.ppo_adam_step.argtypes = [C.POINTER(PpoAdamStep), V]
    L.ppo_policy_sample.argtypes = [V, V, I32, I32, C.c_uint64, V, V, V, F32, V, V, V, V, V, V]
    L.ppo_counter_add.argtypes = [V, I64, V]
    L.ppo_mlp_forward.argtypes = [C.POINTER(PpoMlpFwd), V]
    L.ppo_mlp_backward.argtypes = [C.POINTER(PpoMlpBwd), V]
    L.ppo_weight_grads.argtypes = [C.POINTER(PpoWgrad), V]
    L.ppo_rollout_post_blocks.argtypes = [I32]
    L.ppo_rollout_post.argtypes = [V, V, V, V, I32, F32, F32, F32, I32, V, V, V, V, V, V]
    L.ppo_meter_update.argtypes = [V, I32, F32, V, V, V]
    for f in ("ppo_obs_stats_blocks", "ppo_loss_blocks", "ppo_elu_bwd_blocks"):
        getattr(L, f).argtypes = [I32]
    L.ppo_last_error.restype = C.c_char_p
    L.ppo_build_id.restype = C.c_char_p
    if L.ppo_abi_version() != PPO_ABI_VERSION:
        raise NativeError(f"libppo_hip ABI {L.ppo_abi_version()} != {PPO_ABI_VERSION}")
    check_build_id(L.ppo_build_id(), path, "PPO_HIP_LIB")
    _LIB = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise NativeError(f"{what} failed ({rc}): {load().ppo_last_error().decode(errors='replace')}")


def _p(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _split(rows: int) -> int:
    """Split-K factor of the hipBLASLt weight-gradient bmm (the non-MFMA path): row chunks of >= 512, at
    most 32 chunks."""
    s = 1
    while s < 32 and rows % (2 * s) == 0 and rows // (2 * s) >= 512:
        s *= 2
    return s


def wgrad_splits(rows: int) -> list[int]:
    """Row splits of the six ppo_weight_grads jobs (trunk layers 0..4, the heads) for one chip of 256 CUs:
    a trunk split is two workgroups (output halves), a head split one.  At 32768 rows: layer 0 16 splits
    (its workgroups stream 384 B per row), layers 1..4 24 (768 B per row), the heads 32 (576 B per row)
    -> 2 x (16 + 4 x 24) + 32 = 256 workgroups of about equal bytes; the trunk pair count (112) is a
    multiple of 8, so every pair shares an XCD.  Small minibatches keep >= 128 rows per split."""
    t = 24 if rows >= 24 * 1024 else max(1, min(24, rows // 128))
    s0 = max(1, 2 * t // 3)
    sh = max(1, 4 * t // 3)
    return [s0, t, t, t, t, sh]


class FusedPPOUpdate:
    """Owns the static buffers and the two graphs of one agent's minibatch step."""

    def __init__(self, agent, compute_dtype: torch.dtype = torch.float16, use_graphs: bool = True,
                 scaler: torch.Tensor | None = None):
        self.L = load()
        self.agent = agent
        self.dev = agent.device
        if self.dev.type != "cuda":
            raise NativeError("the fused PPO update runs on the HIP device only")
        model = agent.model
        net = model.a2c_network
        self.linears = [m for m in net.actor_mlp if isinstance(m, torch.nn.Linear)]
        if not all(isinstance(m, (torch.nn.Linear, torch.nn.ELU)) for m in net.actor_mlp):
            raise NotImplementedError("the fused update implements the ELU trunk of the Allsteps agent")
        self.net, self.model = net, model
        self.A = agent.actions_num
        self.obs_dim = agent.obs_shape[0]
        self.mb = agent.dataset.minibatch_size
        self.n_mb = len(agent.dataset)
        if compute_dtype not in PPO_DT:
            raise ValueError(f"compute_dtype must be float32, bfloat16 or float16, got {compute_dtype}")
        self.dt = compute_dtype
        self.lp = compute_dtype != torch.float32   # 16-bit trunk (mixed_precision)
        self.dt_code = PPO_DT[compute_dtype]
        # the loss scaler state [scale, growth tracker] (device fp32; GradScaler), shared with the agent
        self.scaler = scaler
        self.k0 = (self.obs_dim + 7) // 8 * 8 if self.lp else self.obs_dim  # 16-B aligned 16-bit rows
        self.use_graphs = use_graphs
        flat = agent.flat
        self.flat = flat
        B, dev, dt = self.mb, self.dev, self.dt
        widths = [self.k0] + [m.out_features for m in self.linears]
        wmax = max(widths[1:])
        if any(w != wmax for w in widths[1:]):
            raise NotImplementedError("the fused update expects equal hidden widths (the agent's [256] x 5)")
        # fused MFMA trunk (csrc/ppo_mlp.hip): 16-bit mirror, 59 -> 256 x 5 ELU, heads <= 32
        self.mfma_trunk = bool(self.lp and len(self.linears) == 5 and widths[1:] == [256] * 5 and self.k0 == 64
                               and self.A + 1 <= 32 and getattr(agent, "config", {}).get("mfma_trunk", True))
        L = self.L
        if self.mfma_trunk:
            # layer inputs carry a constant ones column (x: col 64 of 72, hidden: col 256 of 264), so the
            # split-K weight-gradient GEMM also yields the bias gradient (its column `in`)
            # h[0] the normalised input, h[1..5] the five layers (16-bit, as autocast keeps them)
            self.h = [torch.zeros(B, 72, device=dev, dtype=dt)] + [torch.zeros(B, 264, device=dev, dtype=dt)
                                                                     for _ in range(5)]
            self.h[0][:, 64] = 1.0
            for t in self.h[1:]:
                t[:, 256] = 1.0
            self.h_last_f = None
            self.dzs = [torch.empty(B, 256, device=dev, dtype=dt) for _ in range(5)]
            self.dhead_lp = torch.zeros(B, 32, device=dev, dtype=dt)  # d loss / d [mu | value], 16-bit
        else:
            self.h = [torch.zeros(B, w, device=dev, dtype=dt) for w in widths]
            self.h_last_f = torch.empty(B, widths[-1], device=dev) if self.lp else self.h[-1]
            self.dz = torch.empty(B, wmax, device=dev, dtype=dt)
            self.dh = torch.empty(B, wmax, device=dev, dtype=dt)
            self.dh_last = torch.empty(B, widths[-1], device=dev)  # fp32 from the heads
            self.elu_partials = torch.empty(len(self.linears), L.ppo_elu_bwd_blocks(B), wmax, device=dev)
        self.head = torch.empty(B, self.A + 1, device=dev)
        self.dhead = torch.empty(B, self.A + 1, device=dev)
        self.S = _split(B)
        self.loss_partials = torch.empty(L.ppo_loss_blocks(B), 2 * self.A + 1 + PPO_LOSS_NSTAT, device=dev)
        self.stat_partials = torch.empty(L.ppo_obs_stats_blocks(B) * 2 * 64, device=dev, dtype=torch.float64)
        self.norm_partials = torch.empty(2 * L.ppo_sqnorm_blocks(), device=dev)  # norm sums | non-finite counts
        # the gradient norm's partials left by the reduce launch itself (no all-reduce between the two graphs:
        # one gradient pass, k_sqnorm, fewer per minibatch); `fuse_norm` False keeps the separate pass
        self.fuse_norm = bool(getattr(agent, "config", {}).get("fuse_norm", True)) and not (
            getattr(agent, "multi_gpu", False) and getattr(agent, "multi_gpu_mode", "") == "allreduce"
            and getattr(agent, "world_size", 1) > 1) and not bool(getattr(agent, "config", {}).get(
                "exchange_schedule", False))
        self.red_norm = torch.empty(2 * 4096, device=dev)
        self._red_nblk = C.c_int32(0)
        # ppo_opt_snap_t (lr, step, scale): taken by the norm launch, read by ppo_adam_step, whose first
        # block runs the tail on the originals
        self.opt_snap = torch.zeros(4, dtype=torch.float64, device=dev)
        # A/B knob: PPO_SEPARATE_TAIL=1 runs ppo_adam + ppo_tail as two launches (the round-5 form)
        self.fuse_tail = os.environ.get("PPO_SEPARATE_TAIL", "0") != "1"
        self.mb_idx = torch.zeros(1, device=dev, dtype=torch.int32)
        self.stat_idx = torch.zeros(1, device=dev, dtype=torch.int32)
        self.stats = torch.zeros(agent.mini_epochs_num * self.n_mb + 1, PPO_LOSS_NSTAT, device=dev)
        # grads of the trunk / heads as views of the flat bucket
        g = flat.grads
        self.gW, self.gb = [], []
        for m in self.linears:
            o = flat.offset(m.weight)
            self.gW.append(g[o:o + m.weight.numel()].view_as(m.weight))
            o = flat.offset(m.bias)
            self.gb.append(g[o:o + m.bias.numel()])
        o = flat.offset(net.mu.weight)
        self.Wh = flat.params[o:o + (self.A + 1) * widths[-1]].view(self.A + 1, widths[-1])  # [mu.w | value.w]
        self.gWh = g[o:o + (self.A + 1) * widths[-1]].view(self.A + 1, widths[-1])
        o = flat.offset(net.mu.bias)
        self.bh = flat.params[o:o + self.A + 1]
        self.gbh = g[o:o + self.A + 1]
        o = flat.offset(net.sigma)
        self.logstd = flat.params[o:o + self.A]
        self.gls = g[o:o + self.A]
        if net.value.weight.data_ptr() != self.Wh[self.A].data_ptr() or \
                net.value.bias.data_ptr() != self.bh[self.A:].data_ptr():
            raise RuntimeError("flat layout: value head must follow the mu head (fused_param_order)")
        # 16-bit trunk mirror (row-padded first layer), written by the Adam kernel
        segs, moff = [], 0
        self.W_lp, self.b_lp = [], []
        if self.lp:
            sizes = [m.out_features * (self.k0 if i == 0 else m.in_features) + m.out_features
                     for i, m in enumerate(self.linears)]
            if self.mfma_trunk:  # + W^T of layers 1..4 for the backward chain
                sizes += [m.weight.numel() for m in self.linears[1:]]
            self.mirror = torch.zeros(sum(sizes), device=dev, dtype=dt)
            for i, m in enumerate(self.linears):
                kin = self.k0 if i == 0 else m.in_features
                segs.append(PpoSeg(flat.offset(m.weight), m.weight.numel(), moff, m.in_features, kin, 0))
                self.W_lp.append(self.mirror[moff:moff + m.out_features * kin].view(m.out_features, kin))
                moff += m.out_features * kin
                segs.append(PpoSeg(flat.offset(m.bias), m.out_features, moff, m.out_features, m.out_features, 0))
                self.b_lp.append(self.mirror[moff:moff + m.out_features])
                moff += m.out_features
            self.WT_lp = []
            if self.mfma_trunk:
                for m in self.linears[1:]:
                    segs.append(PpoSeg(flat.offset(m.weight), m.weight.numel(), moff, m.in_features, m.out_features, 1))
                    self.WT_lp.append(self.mirror[moff:moff + m.weight.numel()].view(m.in_features, m.out_features))
                    moff += m.weight.numel()
            self.refresh_mirror()
        else:
            self.mirror = None
            self.W_lp = [m.weight.detach() for m in self.linears]
            self.b_lp = [m.bias.detach() for m in self.linears]
        if self.mfma_trunk:
            a = PpoMlpFwd()
            for i in range(5):
                a.w[i] = self.W_lp[i].data_ptr()
                o = flat.offset(self.linears[i].bias)
                a.b[i] = flat.params[o:o + 256].data_ptr()
            a.wh, a.bh, a.nh = self.Wh.data_ptr(), self.bh.data_ptr(), self.A + 1
            a.dtype = self.dt_code
            self._mlp_args = a
            bw = PpoMlpBwd()
            bw.dhead, bw.wh, bw.nh = self.dhead_lp.data_ptr(), self.Wh.data_ptr(), self.A + 1
            for k in range(4):
                bw.wt[k] = self.WT_lp[k].data_ptr()
            for k in range(5):
                bw.h[k] = self.h[k + 1].data_ptr()
                bw.dz[k] = self.dzs[k].data_ptr()
            bw.rows, bw.h_stride = B, self.h[1].stride(0)
            bw.dtype = self.dt_code
            self._mlp_bwd_args = bw
            # split-K partials of the weight / bias gradients: (S_l, 256, 72 | 264) fp32 per trunk layer and
            # (S_h, 32, 264) for the heads (dhead^T h5)
            self.wg_splits = wgrad_splits(B)
            self.wg_part = [torch.empty(self.wg_splits[k], 256 if k < 5 else 32, self.h[k].shape[1], device=dev)
                            for k in range(6)]
            wg = PpoWgrad()
            for k in range(6):
                dz = self.dzs[k] if k < 5 else self.dhead_lp
                wg.dz[k], wg.hin[k], wg.part[k] = dz.data_ptr(), self.h[k].data_ptr(), self.wg_part[k].data_ptr()
                wg.kin[k], wg.hin_stride[k], wg.splits[k] = 64 if k == 0 else 256, self.h[k].shape[1], self.wg_splits[k]
            wg.rows, wg.layers, wg.dtype = B, 6, self.dt_code
            self._wgrad_args = wg
        self.segs = (PpoSeg * max(len(segs), 1))(*segs)
        self.nseg = len(segs)
        c = agent.config
        blt = agent.bound_loss_type if agent.bounds_loss_coef is not None else None
        self.loss_cfg = PpoLossCfg(agent.e_clip, agent.critic_coef, agent.entropy_coef,
                                   float(agent.bounds_loss_coef or 0.0), 1.1, int(agent.ppo), int(agent.clip_value),
                                   {"bound": 1, "regularisation": 2}.get(blt, 0))
        sch = agent.scheduler
        self.kl_thr = float(getattr(sch, "kl_threshold", 0.0))
        self.min_lr, self.max_lr = float(getattr(sch, "min_lr", 1e-6)), float(getattr(sch, "max_lr", 1e-2))
        self.legacy = agent.schedule_type == "legacy"
        self.rms = model.running_mean_std
        if self.rms is None:
            raise NotImplementedError("the fused update expects normalize_input")
        self.graphs: dict = {}
        self.ds: dict | None = None
        del c

    # ------------------------------------------------------------------ helpers
    def refresh_mirror(self) -> None:
        """Rewrite the 16-bit trunk mirror from the fp32 parameters (after restore / broadcast)."""
        if self.mirror is None:
            return
        with torch.no_grad():
            for i, m in enumerate(self.linears):
                self.W_lp[i][:, :m.in_features].copy_(m.weight)
                self.b_lp[i].copy_(m.bias)
            for k, m in enumerate(self.linears[1:len(self.WT_lp) + 1]):
                self.WT_lp[k].copy_(m.weight.t())

    def set_dataset(self, ds: dict) -> None:
        """Bind the (static) dataset tensors; graphs are (re)captured when the pointers change."""
        need = ("obs", "actions", "mu", "sigma", "old_logp_actions", "advantages", "old_values", "returns")
        for k in need:
            if not ds[k].is_contiguous():
                raise ValueError(f"dataset tensor {k} must be contiguous")
        key = tuple(ds[k].data_ptr() for k in need)
        if self.ds is None or key != self._ds_key:
            self.graphs.clear()
        self.ds, self._ds_key = ds, key

    def _reduce(self, jobs, s) -> None:
        arr = (PpoReduceJob * len(jobs))(*jobs)
        if not self.fuse_norm:
            _check(self.L.ppo_reduce_rows(arr, len(jobs), s), "ppo_reduce_rows")
            return
        _check(self.L.ppo_reduce_rows_norm(arr, len(jobs), _p(self.scaler), _p(self.gbh), self.gbh.numel(),
                                           _p(self.gls), self.gls.numel(), _p(self.red_norm),
                                           self.red_norm.numel() // 2, C.byref(self._red_nblk), _p(self.agent.lr),
                                           _p(self.agent.optimizer.step_t), _p(self.opt_snap), s),
               "ppo_reduce_rows_norm")

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream

    # ------------------------------------------------------------------ the two halves
    def _trunk(self, x, idx, rows, h, h_last_f, head, fused_loss: bool = False) -> None:
        """Normalise rows [idx*rows, (idx+1)*rows) of x, run the trunk (16-bit mirror or fp32 weights) and
        the heads into head = [mu | value] (fp32 storage; with the MFMA trunk the heads run as rl_games'
        autocast runs them: 16-bit inputs / weights / bias, fp32 accumulation, a 16-bit-rounded output)."""
        L, s, rms = self.L, self._stream(), self.rms
        if self.mfma_trunk:
            # one launch: the input normalisation (RunningMeanStd), 5 x (MFMA + bias + ELU) with
            # weight-stationary waves and the activations through LDS, 16-bit heads; stores the normalised
            # input and layers 1..5 (16-bit) only when h has room for them (training)
            a = self._mlp_args
            a.obs, a.mb_idx, a.obs_dim = x.data_ptr(), idx.data_ptr(), self.obs_dim
            a.mean, a.var, a.eps = rms.running_mean.data_ptr(), rms.running_var.data_ptr(), rms.epsilon
            a.x_out = h[0].data_ptr() if len(h) > 1 else None
            a.x, a.x_stride = h[0].data_ptr(), h[0].stride(0)
            a.h_stride = h[1].stride(0) if len(h) > 1 else 256
            for i in range(5):
                a.h[i] = h[i + 1].data_ptr() if len(h) > 1 else None
            a.head, a.rows = head.data_ptr(), rows
            a.loss.A = 0
            if fused_loss:  # the losses in the forward's epilogue (ppo_mlp_fwd_t.loss)
                ds, fl = self.ds, a.loss
                fl.A, fl.logstd, fl.actions = self.A, _p(self.logstd), _p(ds["actions"])
                fl.ds_mu, fl.ds_sigma, fl.old_neglogp = _p(ds["mu"]), _p(ds["sigma"]), _p(ds["old_logp_actions"])
                fl.advantages, fl.old_values, fl.returns = _p(ds["advantages"]), _p(ds["old_values"]), _p(ds["returns"])
                fl.cfg, fl.grad_scale = self.loss_cfg, _p(self.scaler)
                fl.dhead_lp, fl.partials = _p(self.dhead_lp), _p(self.loss_partials)
            _check(L.ppo_mlp_forward(C.byref(a), s), "ppo_mlp_forward")
            return
        _check(L.ppo_obs_normalize(_p(x), _p(idx), rows, self.obs_dim, _p(rms.running_mean), _p(rms.running_var),
                                   rms.epsilon, _p(h[0]), self.k0, h[0].stride(0), self.dt_code, s),
               "ppo_obs_normalize")
        for i in range(len(self.linears)):  # z = h W^T + b ; h' = elu(z)
            out = h[i + 1]
            torch.addmm(self.b_lp[i], h[i], self.W_lp[i].t(), out=out)
            F.elu(out, inplace=True)
        if h_last_f is not h[-1]:
            h_last_f.copy_(h[-1])
        torch.addmm(self.bh, h_last_f, self.Wh.t(), out=head)

    # ------------------------------------------------------------------ rollout policy (graph-safe)
    def init_rollout(self, n_envs: int, seed: int) -> None:
        dev, dt = self.dev, self.dt
        widths = [self.k0] + [m.out_features for m in self.linears]
        self.N = n_envs
        if self.mfma_trunk:  # activations stay in registers: only the input row block is materialised
            self.hr = [torch.zeros(n_envs, widths[0], device=dev, dtype=dt)]
            self.hr_last_f = None
        else:
            self.hr = [torch.zeros(n_envs, w, device=dev, dtype=dt) for w in widths]
            self.hr_last_f = torch.empty(n_envs, widths[-1], device=dev) if self.lp else self.hr[-1]
        self.head_r = torch.empty(n_envs, self.A + 1, device=dev)
        self.zero_idx = torch.zeros(1, device=dev, dtype=torch.int32)
        self.step_ctr = torch.zeros(1, device=dev, dtype=torch.int64)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF

    @torch.no_grad()
    def policy_act(self, obs: torch.Tensor, out: dict) -> None:
        """ModelA2CContinuousLogStd eval forward + sample for the rollout, written into
        out['actions' | 'neglogpacs' | 'values' | 'mus' | 'sigmas'] (contiguous, rows = n_envs).
        Same trunk precision as the training forward (16-bit mirror when mixed_precision)."""
        if not obs.is_contiguous() or obs.shape[0] != self.N:
            raise ValueError("policy_act: obs must be contiguous (n_envs, obs_dim)")
        self._trunk(obs, self.zero_idx, self.N, self.hr, self.hr_last_f, self.head_r)
        vms = self.model.value_mean_std
        s = self._stream()
        _check(self.L.ppo_policy_sample(_p(self.head_r), _p(self.logstd), self.A, self.N, self.seed,
                                        _p(self.step_ctr), _p(vms.running_mean) if vms is not None else None,
                                        _p(vms.running_var) if vms is not None else None,
                                        vms.epsilon if vms is not None else 0.0, _p(out["actions"]),
                                        _p(out["neglogpacs"]), _p(out["values"]), _p(out["mus"]), _p(out["sigmas"]),
                                        s), "ppo_policy_sample")
        _check(self.L.ppo_counter_add(_p(self.step_ctr), 1, s), "ppo_counter_add")

    def init_bookkeeping(self, agent) -> None:
        """Bind the rollout bookkeeping kernel to the agent's episode buffers; the three AverageMeters
        are re-homed into one (2, 3) device block [means | sizes] the meter kernel updates."""
        n = agent.num_actors * agent.num_agents
        blk = torch.zeros(2, 3, device=self.dev)
        for k, m in enumerate((agent.game_rewards, agent.game_shaped_rewards, agent.game_lengths)):
            blk[0, k] = m.mean.reshape(-1)[0]
            blk[1, k] = m.current_size
            m.mean = blk[0, k:k + 1]
            m.current_size = blk[1, k]
        self.meters = blk
        self.post_partials = torch.zeros(self.L.ppo_rollout_post_blocks(n), 4, device=self.dev)
        self.max_games = float(agent.games_to_track)

    def rollout_post(self, agent, rewards, dones, time_outs, values, shaped_out) -> None:
        """play_steps' per-step bookkeeping in two launches (shaping, bootstrap, episode sums, meters)."""
        L, s = self.L, self._stream()
        sh = agent.rewards_shaper
        if sh.min_val != -float("inf") or sh.max_val != float("inf"):
            raise NotImplementedError("reward clipping in the fused rollout bookkeeping")
        n = rewards.shape[0]
        boot = int(agent.value_bootstrap and time_outs is not None)
        d = dones if dones.dtype == torch.uint8 else dones.view(torch.uint8)
        t = None if time_outs is None else (time_outs if time_outs.dtype == torch.uint8 else time_outs.view(torch.uint8))
        _check(L.ppo_rollout_post(_p(rewards), _p(d), _p(t), _p(values), n, float(sh.scale_value),
                                  float(sh.shift_value), float(agent.gamma), boot, _p(shaped_out),
                                  _p(agent.current_rewards), _p(agent.current_shaped_rewards),
                                  _p(agent.current_lengths), _p(self.post_partials), s), "ppo_rollout_post")
        _check(L.ppo_meter_update(_p(self.post_partials), self.post_partials.shape[0], self.max_games,
                                  _p(self.meters[0]), _p(self.meters[1]), s), "ppo_meter_update")

    @torch.no_grad()
    def policy_values(self, obs: torch.Tensor) -> torch.Tensor:
        """Denormalised values (n_envs, 1) of the rollout policy (get_values)."""
        self._trunk(obs.contiguous(), self.zero_idx, self.N, self.hr, self.hr_last_f, self.head_r)
        v = self.head_r[:, self.A:].clone()
        return self.model.denorm_value(v)

    @torch.no_grad()
    def _forward_backward(self, rms_train: bool) -> None:
        L, s, ds, B, A = self.L, self._stream(), self.ds, self.mb, self.A
        rms = self.rms
        if rms_train:
            _check(L.ppo_obs_stats(_p(ds["obs"]), _p(self.mb_idx), B, self.obs_dim, _p(self.stat_partials), s),
                   "ppo_obs_stats")
            _check(L.ppo_obs_stats_update(_p(self.stat_partials), L.ppo_obs_stats_blocks(B), self.obs_dim, B,
                                          _p(rms.running_mean), _p(rms.running_var), _p(rms.count), s),
                   "ppo_obs_stats_update")
        fused_loss = self.mfma_trunk and A in (12, 21)  # the forward runs ppo_loss_grad's work too
        self._trunk(ds["obs"], self.mb_idx, B, self.h, self.h_last_f, self.head, fused_loss)
        nl = len(self.linears)
        # no zero_grad: every entry of the [grads | kl] bucket is written below (loss finalize: head
        # biases, log-sigma, kl; the reduce jobs: every weight and bias gradient)
        if not fused_loss:
            _check(L.ppo_loss_grad(_p(self.head), _p(self.logstd), A, B, _p(self.mb_idx), _p(ds["actions"]),
                                   _p(ds["mu"]), _p(ds["sigma"]), _p(ds["old_logp_actions"]), _p(ds["advantages"]),
                                   _p(ds["old_values"]), _p(ds["returns"]), self.loss_cfg, _p(self.scaler),
                                   None if self.mfma_trunk else _p(self.dhead), _p(self.loss_partials),
                                   _p(self.dhead_lp) if self.mfma_trunk else None, self.dt_code, s), "ppo_loss_grad")
        if not self.mfma_trunk:  # (the MFMA path runs the finalize as a side job of ppo_weight_grads)
            _check(L.ppo_loss_finalize(_p(self.loss_partials), self.loss_partials.shape[0], A, B,
                                       self.loss_cfg.entropy_coef, _p(self.scaler), _p(self.gbh), _p(self.gls),
                                       _p(self.stats), _p(self.stat_idx), _p(self.flat.extra), s), "ppo_loss_finalize")
        S = self.S
        hl = self.h_last_f
        jobs, keep = [], []
        if self.mfma_trunk:
            self._backward_mfma()
            return

        def job(src: torch.Tensor, dst: torch.Tensor, n_s: int, out_rows: int, src_cols: int, dst_cols: int,
                dst_stride: int) -> None:
            keep.append(src)
            jobs.append(PpoReduceJob(src.data_ptr(), dst.data_ptr(), n_s, out_rows, src_cols, dst_cols, dst_stride,
                                     src.numel() // n_s))

        # heads: dWh = dhead^T h (split-K partials), dh_last = dhead Wh
        pw = torch.bmm(self.dhead.view(S, B // S, A + 1).transpose(1, 2), hl.view(S, B // S, hl.shape[1]))
        job(pw, self.gWh, S, A + 1, hl.shape[1], hl.shape[1], hl.shape[1])
        torch.mm(self.dhead, self.Wh, out=self.dh_last)
        dh, dh_t = self.dh_last, 0
        dt_code = self.dt_code
        nblk = self.elu_partials.shape[1]
        for i in reversed(range(nl)):
            m = self.linears[i]
            n_out = m.out_features
            dz = self.dz[:, :n_out]
            # dz_i = elu'(h_{i+1}) * dh_{i+1}; bias grad from the per-block column sums
            last = i == nl - 1 and self.mfma_trunk  # layer 5 is kept in fp32 by the MFMA trunk
            h_act, h_t = (self.h_last_f, 0) if last else (self.h[i + 1], dt_code)
            _check(L.ppo_elu_bwd(_p(dh), dh_t, _p(h_act), h_t, _p(dz), dt_code, B, n_out,
                                 _p(self.elu_partials[i]), s),
                   "ppo_elu_bwd")
            job(self.elu_partials[i], self.gb[i], nblk, 1, n_out, n_out, n_out)
            hin = self.h[i]
            kin = hin.shape[1]
            gw = torch.bmm(dz.view(S, B // S, n_out).transpose(1, 2), hin.view(S, B // S, kin),
                           out_dtype=torch.float32) if self.lp else \
                torch.bmm(dz.view(S, B // S, n_out).transpose(1, 2), hin.view(S, B // S, kin))
            job(gw, self.gW[i], S, n_out, kin, m.in_features, m.in_features)
            if i > 0:
                dhi = self.dh[:, :kin]
                torch.mm(dz, self.W_lp[i], out=dhi)
                dh, dh_t = dhi, dt_code
        self._reduce(jobs, s)
        del keep

    def _backward_mfma(self) -> None:
        """dz of all five layers from one MFMA launch (ppo_mlp_backward), then the trunk weight and bias
        gradients and the head weight gradient as split-K partials of ONE launch (ppo_weight_grads),
        summed by ONE reduce launch (the head bias and log-sigma gradients come from ppo_loss_finalize)."""
        L, s, A = self.L, self._stream(), self.A
        jobs = []
        _check(L.ppo_mlp_backward(C.byref(self._mlp_bwd_args), s), "ppo_mlp_backward")
        # + ppo_loss_finalize's work as the launch's side job (the head-bias / log-sigma gradients, the
        # statistics, the KL)
        f = self._wgrad_args.loss
        f.partials, f.nblk, f.A, f.mb_rows = _p(self.loss_partials), self.loss_partials.shape[0], A, self.mb
        f.entropy_coef, f.grad_scale, f.grad_head_bias, f.grad_logstd = (self.loss_cfg.entropy_coef, _p(self.scaler),
                                                                          _p(self.gbh), _p(self.gls))
        f.stats, f.stat_idx, f.kl_out = _p(self.stats), _p(self.stat_idx), _p(self.flat.extra)
        _check(L.ppo_weight_grads(C.byref(self._wgrad_args), s), "ppo_weight_grads")
        for i in range(6):
            w = self.h[i].shape[1]               # 72 or 264: [features | 1 | 0 ...]
            S = self.wg_splits[i]
            gw = self.wg_part[i]                 # (S, 256 | 32, w), trunk bias sums in column `ones`
            n_s = gw.numel() // S
            if i == 5:
                jobs.append(PpoReduceJob(gw.data_ptr(), self.gWh.data_ptr(), S, A + 1, w, 256, 256, n_s))
                continue
            m = self.linears[i]
            ones = 64 if i == 0 else 256
            jobs.append(PpoReduceJob(gw.data_ptr(), self.gW[i].data_ptr(), S, 256, w, m.in_features, m.in_features, n_s))
            jobs.append(PpoReduceJob(gw.data_ptr() + 4 * ones, self.gb[i].data_ptr(), S, 256, w, 1, 1, n_s))
        self._reduce(jobs, s)

    @torch.no_grad()
    def _optimizer_step(self) -> None:
        L, s, ag, fl = self.L, self._stream(), self.agent, self.flat
        n = fl.numel
        if self.fuse_norm:  # the reduce launch of graph A left the norm partials
            npart, nnp = self.red_norm, self._red_nblk.value
            if nnp <= 0:
                raise NativeError("fused gradient norm: step_b before step_a")
        else:
            _check(L.ppo_sqnorm(_p(fl.grads), n, _p(self.scaler), _p(self.norm_partials), _p(ag.lr),
                                _p(ag.optimizer.step_t), _p(self.opt_snap), s), "ppo_sqnorm")
            npart, nnp = self.norm_partials, self.norm_partials.numel() // 2
        opt = ag.optimizer
        if not self.fuse_tail:
            _check(L.ppo_adam(_p(fl.params), _p(fl.grads), _p(opt.exp_avg), _p(opt.exp_avg_sq), n, _p(npart), nnp,
                              ag.grad_norm if ag.truncate_grads else 0.0, _p(ag.lr), _p(opt.step_t), opt.beta1,
                              opt.beta2, opt.eps, self.segs, self.nseg, _p(self.mirror), self.dt_code if self.lp else 1,
                              _p(self.scaler), s), "ppo_adam")
            _check(L.ppo_tail(_p(ag.lr), _p(fl.extra), self.kl_thr if self.legacy else 0.0, self.min_lr, self.max_lr,
                              _p(opt.step_t), _p(self.mb_idx), self.n_mb, _p(self.stat_idx), _p(self.scaler),
                              _p(npart), nnp, SCALER_GROWTH_INTERVAL, s), "ppo_tail")
            return
        # clip + Adam + the tail (adaptive LR, GradScaler update, counters) in one launch
        a = PpoAdamStep(_p(fl.params), _p(fl.grads), _p(opt.exp_avg), _p(opt.exp_avg_sq), n, _p(npart), nnp,
                        ag.grad_norm if ag.truncate_grads else 0.0, opt.beta1, opt.beta2, opt.eps, self.segs,
                        self.nseg, _p(self.mirror), self.dt_code if self.lp else 1, _p(self.opt_snap),
                        _p(ag.lr), _p(fl.extra), self.kl_thr if self.legacy else 0.0, self.min_lr, self.max_lr,
                        _p(opt.step_t), _p(self.mb_idx), self.n_mb, _p(self.stat_idx), _p(self.scaler),
                        SCALER_GROWTH_INTERVAL)
        _check(L.ppo_adam_step(C.byref(a), s), "ppo_adam_step")

    # ------------------------------------------------------------------ graphs
    def _run(self, key, fn) -> None:
        """First call of a variant: run eagerly (real work; warms up hipBLASLt handles / workspaces and
        the allocator).  Second call: capture the graph (capture does not execute), then replay."""
        g = self.graphs.get(key)
        if g is None:
            fn()
            self.graphs[key] = "warm"
            return
        if g == "warm":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            self.graphs[key] = g
        g.replay()

    def begin_epoch(self) -> None:
        self.mb_idx.zero_()
        self.stat_idx.zero_()

    def step_a(self, rms_train: bool) -> None:
        if self.use_graphs:
            self._run(("a", rms_train), lambda: self._forward_backward(rms_train))
        else:
            self._forward_backward(rms_train)

    def step_b(self) -> None:
        if self.use_graphs:
            self._run(("b",), self._optimizer_step)
        else:
            self._optimizer_step()

    def run_minibatches(self, n: int, rms_train: bool) -> None:
        """n consecutive minibatch steps (graph A's then graph B's work, n times) as ONE graph, for a
        mini-epoch with nothing between A and B (no bucket all-reduce): the rows, the statistics slot and
        the LR are device counters, so the same n-step sequence serves every mini-epoch.  One graph launch
        per mini-epoch instead of 2 n: each launch boundary left ~5 us of idle GPU (r05w: update_s 54.1 ms
        against 50.5 ms of kernels)."""
        def body() -> None:
            for _ in range(n):
                self._forward_backward(rms_train)
                self._optimizer_step()

        if self.use_graphs:
            self._run(("mb", n, rms_train), body)
        else:
            body()
