"""Multi-process (gloo, world_size 2, CPU) coverage of the N > 1 path: rollout all-gather at the PPO
boundary, the optional global curriculum mean, and the per-rank shard layout."""

import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from allsteps_isaaclab_amd.distributed import RolloutGather, ShardInfo, global_curriculum_mean, shard_info


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_rollout(rank: int, H: int = 4, N: int = 6):
    g = torch.Generator().manual_seed(100 + rank)
    return {
        "obs": torch.randn(H, N, 59, generator=g),
        "actions": torch.randn(H, N, 21, generator=g),
        "rewards": torch.randn(H, N, generator=g),
        "dones": torch.rand(H, N, generator=g) < 0.3,
        "env_ids": (torch.arange(N, dtype=torch.int64) + rank * N).expand(H, N).contiguous(),
    }


def _flat(t):
    """swap_and_flatten01: [H, N, ...] -> env-major [N H, ...]"""
    return t.transpose(0, 1).reshape((t.shape[0] * t.shape[1],) + tuple(t.shape[2:]))


def _worker(rank: int, world: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        info = shard_info()
        gather = RolloutGather(env_axis=1)  # [H, N, ...] layout: parts concatenated along the env axis
        flat_gather = RolloutGather()       # env-major flattened [N H, ...] (the trainer's): direct receive
        res = {}
        for it in range(2):  # second call reuses the cached receive buffers
            res = gather.gather(_rank_rollout(rank))
            flat = flat_gather.gather({k: _flat(v) for k, v in _rank_rollout(rank).items()})
        # the results are the cached buffers: a later gather overwrites them in place; copy=True does not
        kept = flat_gather.gather({"obs": _flat(_rank_rollout(rank)["obs"])}, copy=True)["obs"]
        again = flat_gather.gather({"obs": torch.zeros_like(_flat(_rank_rollout(rank)["obs"]))})["obs"]
        assert again.data_ptr() == flat["obs"].data_ptr() and float(flat["obs"].abs().sum()) == 0.0
        assert float(kept.abs().sum()) > 0.0
        flat["obs"] = kept
        res.update({"flat/" + k: v for k, v in flat.items()})
        fake_env = types.SimpleNamespace(curr_target_index=torch.full((6,), 1 + 3 * rank, dtype=torch.int32))
        mean = global_curriculum_mean(fake_env)
        # numpy copies travel by value: torch tensors would be shared through /dev/shm files that vanish
        # when this process exits before the parent unpickles them
        q.put((rank, info.rank, info.world, {k: v.numpy().copy() for k, v in res.items()}, mean))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_rollout_gather_world2(world):
    """Both layouts at world 2, 3 (odd) and 4: every rank receives the rank-major
    concatenation, i.e. global env order, with rank r's shard at [r N, (r+1) N); receive buffers are
    reused across gathers."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = {k: torch.cat([_rank_rollout(r)[k] for r in range(world)], dim=1) for k in _rank_rollout(0)}
    # env-major flattened: rank-major concatenation along axis 0 is the global env order
    expect.update({"flat/" + k: torch.cat([_flat(_rank_rollout(r)[k]) for r in range(world)], dim=0)
                   for k in _rank_rollout(0)})
    for rank, info_rank, info_world, res, mean in out:
        res = {k: torch.from_numpy(v) for k, v in res.items()}
        assert info_rank == rank and info_world == world
        for k, v in expect.items():
            assert res[k].dtype == v.dtype and res[k].shape == v.shape, k
            torch.testing.assert_close(res[k], v, rtol=0, atol=0)
        # global env ids come out in order: rank r's shard is [r N, (r+1) N)
        assert torch.equal(res["env_ids"][0], torch.arange(6 * world))
        assert torch.equal(res["flat/env_ids"][::4], torch.arange(6 * world))  # env-major rows, H = 4 each
        assert mean == pytest.approx(sum(1 + 3 * r for r in range(world)) / world)


def test_single_process_gather_is_identity():
    t = _rank_rollout(0)
    out = RolloutGather().gather(t)
    assert all(out[k] is t[k] for k in t)


def test_shard_layout():
    info = ShardInfo(rank=3, world=8, local_rank=3)
    assert info.env_offset(32768) == 3 * 32768 and info.seed(42) == 45
