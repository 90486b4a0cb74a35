"""Multi-GPU plumbing for the Allsteps step: one process per GPU, envs sharded, no data-path
collective inside ``env.step``.

* Env sharding.  Rank r of W owns global env ids ``[r N, (r+1) N)``: its ``AllstepsEnv`` is built with
  ``env_id_offset = r N`` so the in-kernel Philox reset draws are keyed by (seed, global env id): with
  one seed on every rank a sharded run is bit-identical to one GPU stepping all ``W N`` envs
  (tests/test_gpu_parity.py::test_shards_match_unsharded).  ``make_sharded_env`` follows train.py:100
  instead (``seed + rank``), which the reference does for its per-rank envs.
* The curriculum mean stays per process (allsteps_env.py:471 reads the process's own envs, which is
  what the reference does under ``--distributed``); ``global_curriculum_mean`` is the optional
  4-byte all-reduce variant.
* The only exchange is at the PPO update boundary: ``RolloutGather`` all-gathers a horizon of rollout
  tensors from every rank, one collective per tensor straight into its output buffer over RCCL (each
  is hundreds of KB to hundreds of MB, so the per-link bandwidth, not latency, is the bound).  With
  the gloo backend (CPU tests) the same code path runs.
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ShardInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    def env_offset(self, envs_per_rank: int) -> int:
        return self.rank * envs_per_rank

    def seed(self, base_seed: int) -> int:
        return base_seed + self.rank


def _local_device(local: int) -> int:
    """The device index of a local rank: itself, except in the shared-GPU rehearsal
    (ALLSTEPS_DIST_BACKEND=gloo: more ranks than GPUs), where ranks wrap onto the visible devices as
    bench.py maps them."""
    if os.environ.get("ALLSTEPS_DIST_BACKEND") == "gloo" and torch.cuda.is_available():
        return local % max(torch.cuda.device_count(), 1)
    return local


def shard_info() -> ShardInfo:
    """Rank / world / local rank (device index) from torch.distributed (or the launcher's environment)."""
    if dist.is_available() and dist.is_initialized():
        return ShardInfo(dist.get_rank(), dist.get_world_size(),
                         _local_device(int(os.environ.get("LOCAL_RANK", dist.get_rank()))))
    return ShardInfo(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                     _local_device(int(os.environ.get("LOCAL_RANK", 0))))


def init_process_group(backend: str | None = None) -> ShardInfo:
    """torch.distributed.run rendezvous (MASTER_ADDR defaults to 127.0.0.1); nccl = RCCL on ROCm."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    info = shard_info()
    if info.world > 1 and not dist.is_initialized():
        if backend is None:  # ALLSTEPS_DIST_BACKEND overrides (e.g. gloo for ranks sharing one GPU in tests)
            backend = os.environ.get("ALLSTEPS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        # a rank that dies or stalls ends the others' collectives after this long instead of hanging them
        kw = {"timeout": datetime.timedelta(seconds=float(os.environ.get("ALLSTEPS_DIST_TIMEOUT_S", "600")))}
        if backend == "nccl":
            torch.cuda.set_device(info.local_rank)
            kw["device_id"] = torch.device(f"cuda:{info.local_rank}")
        dist.init_process_group(backend, **kw)
        info = shard_info()
    return info


def make_sharded_env(cfg, info: ShardInfo | None = None, **kwargs):
    """AllstepsEnv for this rank's env shard (device cuda:local_rank, offset ids, seed + rank)."""
    from .envs.allsteps_env import AllstepsEnv

    info = info or shard_info()
    cfg.sim.device = f"cuda:{info.local_rank}"
    if cfg.seed is not None:
        cfg.seed = info.seed(cfg.seed)
    return AllstepsEnv(cfg, env_id_offset=info.env_offset(int(cfg.scene.num_envs)), **kwargs)


def global_curriculum_mean(env, group=None) -> float:
    """Mean curr_target_index over ALL ranks' envs (one 8-byte all-reduce) -- an opt-in variant of
    the per-process gate of allsteps_env.py:471."""
    idx = env.curr_target_index
    t = torch.stack([idx.sum().to(torch.float64), torch.tensor(float(idx.numel()), dtype=torch.float64,
                                                               device=idx.device)])
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
    return float(t[0] / t[1])


class RolloutGather:
    """All-gather of a PPO horizon of rollout tensors across ranks.

    ``gather({"obs": [N H, 59], "actions": [N H, 21], "dones": [N H] (bool), ...})`` returns the same keys
    with the env axis concatenated over ranks in rank order, i.e. global env order.  With the env axis
    outermost (``env_axis=0``: the trainer's env-major flattened batch) the rank-major receive buffer
    IS that concatenation, so every key is gathered straight into its own cached output tensor with one
    ``all_gather_into_tensor`` (RCCL) -- no send-side packing and no copy after the collective; the
    payloads are MB-sized, so the per-collective latency is negligible against the per-link
    bandwidth.  For another env axis ([H, N, ...]) the parts are concatenated along it (one copy).

    The returned tensors are this object's cached receive buffers (or views of them), keyed by
    (key, dtype, shape, device): they stay valid until the next ``gather`` with the same keys and shapes,
    which overwrites them in place.  A caller that keeps an earlier result across gathers passes
    ``copy=True`` (fresh tensors) or clones what it keeps; the trainer consumes each gathered batch
    (prepare_dataset copies it into the update's static buffers) before the next epoch's gather.
    """

    def __init__(self, group=None, env_axis: int = 0):
        self.group = group
        self.env_axis = env_axis
        self._recv: dict = {}

    def _world(self) -> int:
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def _out(self, key, t: torch.Tensor, world: int) -> torch.Tensor:
        shape = (world * t.shape[0],) + tuple(t.shape[1:])
        k = (key, t.dtype, shape, t.device)
        buf = self._recv.get(k)
        if buf is None:
            buf = torch.empty(shape, dtype=t.dtype, device=t.device)
            self._recv[k] = buf
        return buf

    def gather(self, tensors: dict[str, torch.Tensor], copy: bool = False) -> dict[str, torch.Tensor]:
        world = self._world()
        if world == 1:
            return {k: v.clone() for k, v in tensors.items()} if copy else dict(tensors)
        backend = dist.get_backend(self.group)
        out: dict[str, torch.Tensor] = {}
        for k, t in tensors.items():
            t = t.contiguous()
            src = t.movedim(self.env_axis, 0).contiguous() if self.env_axis != 0 else t
            buf = self._out(k, src, world)
            wire_src = src.view(torch.uint8) if src.dtype == torch.bool else src
            wire_buf = buf.view(torch.uint8) if buf.dtype == torch.bool else buf
            if backend == "nccl":
                dist.all_gather_into_tensor(wire_buf, wire_src, group=self.group)
            else:  # gloo (CPU tests, the shared-GPU rehearsal): views of the same buffer, no extra copy
                dist.all_gather(list(wire_buf.chunk(world)), wire_src, group=self.group)
            out[k] = buf if self.env_axis == 0 else buf.movedim(0, self.env_axis)
            if copy:
                out[k] = out[k].clone()
        return out
