"""PPO trainer (rl_games 1.6.1 a2c_continuous semantics) on CPU.

rl_games is absent offline, so every formula is checked against an independent restatement (numpy /
torch.distributions / torch.optim.Adam) -- trainer parity vs rl_games itself is unpinned.  The
end-to-end runs use a toy point-mass env with the same VecEnv surface; the Allsteps env is GPU-only
(tests/test_gpu_learning.py)."""

import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from allsteps_isaaclab_amd.learning import a2c_continuous as A
from allsteps_isaaclab_amd.learning.models import FlatParams, ModelA2CContinuousLogStd, neglogp
from allsteps_isaaclab_amd.learning.running_mean_std import RunningMeanStd

from _toy_env import ToyReachEnv, agent_params


def test_running_mean_std_matches_pooled_moments():
    rms = RunningMeanStd((3,)).train()
    g = torch.Generator().manual_seed(0)
    xs = [torch.randn(n, 3, generator=g) * 2 + 1 for n in (5, 17, 64)]
    for x in xs:
        y = rms(x)
    # rl_games starts from mean 0, var 1, count 1 (a pseudo-sample); pooled with the batches
    allx = np.concatenate([x.numpy().astype(np.float64) for x in xs])
    cnt, mean, var = 1.0, np.zeros(3), np.ones(3)
    for x in xs:
        x = x.numpy().astype(np.float64)
        bm, bv, bc = x.mean(0), x.var(0, ddof=1), x.shape[0]
        d = bm - mean
        tot = cnt + bc
        mean, var, cnt = mean + d * bc / tot, (var * cnt + bv * bc + d ** 2 * cnt * bc / tot) / tot, tot
    np.testing.assert_allclose(rms.running_mean.numpy(), mean, rtol=1e-6)  # batch moments in fp32
    np.testing.assert_allclose(rms.running_var.numpy(), var, rtol=1e-6)
    assert float(rms.count) == 1 + len(allx)
    exp = np.clip((xs[-1].numpy() - mean.astype(np.float32)) / np.sqrt(var.astype(np.float32) + 1e-5), -5, 5)
    np.testing.assert_allclose(y.numpy(), exp, rtol=1e-5, atol=1e-6)
    rms.eval()
    before = rms.running_mean.clone()
    z = rms(xs[0])
    assert torch.equal(rms.running_mean, before)  # eval: no update
    back = rms(z, denorm=True)
    np.testing.assert_allclose(back.numpy(), np.clip(xs[0].numpy(), -1e9, 1e9), atol=5e-5 * 10)


def test_neglogp_entropy_kl_match_torch_distributions():
    g = torch.Generator().manual_seed(1)
    mu, logstd = torch.randn(32, 21, generator=g), torch.randn(21, generator=g) * 0.3
    x = torch.randn(32, 21, generator=g)
    sigma = torch.exp(logstd).expand_as(mu)
    d = torch.distributions.Normal(mu, sigma)
    torch.testing.assert_close(neglogp(x, mu, sigma, logstd.expand_as(mu)), -d.log_prob(x).sum(-1), rtol=1e-5, atol=1e-4)
    mu1, s1 = mu + 0.1 * torch.randn(32, 21, generator=g), sigma * 1.1
    kl = A.policy_kl(mu, sigma, mu1, s1, reduce=False)
    ref = torch.distributions.kl_divergence(torch.distributions.Normal(mu, sigma),
                                            torch.distributions.Normal(mu1, s1)).sum(-1)
    torch.testing.assert_close(kl, ref, rtol=1e-3, atol=1e-3)  # rl_games adds 1e-5 guards
    model = ModelA2CContinuousLogStd(5, 21, normalize_input=False, normalize_value=False, units=(8,))
    out = model({"is_train": True, "prev_actions": x[:, :21], "obs": torch.randn(32, 5, generator=g)})
    ref_ent = torch.distributions.Normal(out["mus"], out["sigmas"]).entropy().sum(-1)
    torch.testing.assert_close(out["entropy"], ref_ent)


def test_gae_matches_numpy_loop():
    H, N, gamma, tau = 7, 5, 0.99, 0.95
    g = torch.Generator().manual_seed(2)
    rew, val = torch.randn(H, N, 1, generator=g), torch.randn(H, N, 1, generator=g)
    mb_dones = (torch.rand(H, N, generator=g) < 0.3).float()
    fdones, last = (torch.rand(N, generator=g) < 0.3).float(), torch.randn(N, 1, generator=g)
    agent = A.A2CAgent.__new__(A.A2CAgent)
    agent.horizon_length, agent.gamma, agent.tau = H, gamma, tau
    adv = agent.discount_values(fdones, last, mb_dones, val, rew).numpy()[..., 0]
    r, v, d = rew.numpy()[..., 0], val.numpy()[..., 0], mb_dones.numpy()
    exp = np.zeros((H, N))
    for e in range(N):
        lg = 0.0
        for t in reversed(range(H)):
            nnt = 1.0 - (fdones[e].item() if t == H - 1 else d[t + 1, e])
            nv = last[e, 0].item() if t == H - 1 else v[t + 1, e]
            delta = r[t, e] + gamma * nv * nnt - v[t, e]
            lg = delta + gamma * tau * nnt * lg
            exp[t, e] = lg
    np.testing.assert_allclose(adv, exp, rtol=1e-5, atol=1e-5)


def test_flat_adam_matches_torch_adam():
    torch.manual_seed(3)
    ref = torch.nn.Sequential(torch.nn.Linear(6, 8), torch.nn.ELU(), torch.nn.Linear(8, 3))
    mine = torch.nn.Sequential(torch.nn.Linear(6, 8), torch.nn.ELU(), torch.nn.Linear(8, 3))
    mine.load_state_dict(ref.state_dict())
    flat = FlatParams(mine)
    lr = torch.tensor(3e-3, dtype=torch.float64)
    opt_m = A.FlatAdam(flat, lr)
    opt_r = torch.optim.Adam(ref.parameters(), lr=3e-3, eps=1e-8)
    for it in range(25):
        x = torch.randn(16, 6)
        y = torch.randn(16, 3)
        if it == 10:  # LR change mid-run (adaptive schedule)
            lr.fill_(1e-3)
            for gr in opt_r.param_groups:
                gr["lr"] = 1e-3
        flat.zero_grad()
        ((mine(x) - y) ** 2).mean().backward()
        opt_m.step()
        opt_r.zero_grad()
        ((ref(x) - y) ** 2).mean().backward()
        opt_r.step()
    for a, b in zip(mine.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # parameters really live in the flat buffer
    p0 = next(mine.parameters())
    assert p0.data_ptr() == flat.params.data_ptr() and p0.grad.data_ptr() == flat.grads.data_ptr()


def test_adaptive_scheduler_and_average_meter():
    sch = A.AdaptiveScheduler(0.008)
    lr = torch.tensor(3e-4, dtype=torch.float64)
    py = 3e-4
    for kl in [0.001, 0.02, 0.008, 0.0001, 0.5, 0.5, 0.0]:
        sch.update_(lr, torch.tensor(kl))
        if kl > 0.016:
            py = max(py / 1.5, 1e-6)
        if kl < 0.004:
            py = min(py * 1.5, 1e-2)
        assert float(lr) == pytest.approx(py, rel=1e-12)
    # AverageMeter: device-masked update == rl_games' indexed update
    m = A.AverageMeter(1, 5, "cpu")
    mean, cur = 0.0, 0
    g = torch.Generator().manual_seed(4)
    for _ in range(12):
        v = torch.randn(8, 1, generator=g)
        mask = torch.rand(8, generator=g) < 0.4
        m.update(v, mask)
        sel = v[mask]
        if sel.numel():
            size = min(sel.shape[0], 5)
            old = min(5 - size, cur)
            mean = (mean * old + sel.mean().item() * size) / (old + size)
            cur = old + size
        assert float(m.current_size) == cur
        assert float(m.mean[0]) == pytest.approx(mean, rel=1e-5, abs=1e-6)


def _make_agent(n=64, seed=0, **over):
    params = agent_params(n, **over)
    params["seed"] = seed
    params["config"]["vec_env"] = ToyReachEnv(n, seed=seed)
    torch.manual_seed(seed)
    return A.A2CAgent("run", params)


def test_loss_scaler_update_is_grad_scaler():
    """A2CAgent._scaler_update == torch.amp.GradScaler.update's rule (defaults: backoff 0.5, growth 2
    after 2000 good steps in a row, tracker reset on either event) -- the rule ppo_tail applies on the
    device in the fused path."""
    from allsteps_isaaclab_amd.learning.fused import SCALER_GROWTH_INTERVAL, SCALER_INIT

    class S:
        scaler_state = torch.tensor([SCALER_INIT, 0.0])

    s = S()
    A.A2CAgent._scaler_update(s, True)
    assert s.scaler_state.tolist() == [SCALER_INIT / 2, 0.0]
    for _ in range(SCALER_GROWTH_INTERVAL - 1):
        A.A2CAgent._scaler_update(s, False)
    assert s.scaler_state.tolist() == [SCALER_INIT / 2, SCALER_GROWTH_INTERVAL - 1]
    A.A2CAgent._scaler_update(s, False)
    assert s.scaler_state.tolist() == [SCALER_INIT, 0.0]
    import inspect

    d = inspect.signature(torch.amp.GradScaler.__init__).parameters  # the defaults rl_games gets
    assert (d["init_scale"].default, d["growth_factor"].default, d["backoff_factor"].default,
            d["growth_interval"].default) == (SCALER_INIT, 2.0, 0.5, SCALER_GROWTH_INTERVAL)


def test_state_dict_uses_rl_games_names(tmp_path):
    agent = _make_agent()
    keys = set(agent.model.state_dict())
    for k in ("a2c_network.sigma", "a2c_network.actor_mlp.0.weight", "a2c_network.actor_mlp.2.bias",
              "a2c_network.mu.weight", "a2c_network.value.bias", "running_mean_std.running_mean",
              "running_mean_std.count", "value_mean_std.running_var"):
        assert k in keys, k
    sd = agent.model.state_dict()
    assert torch.count_nonzero(sd["a2c_network.actor_mlp.0.bias"]) == 0  # biases zero-initialised
    assert torch.count_nonzero(sd["a2c_network.sigma"]) == 0  # const_initializer val 0


def test_ppo_trains_toy_env_and_checkpoints(tmp_path):
    agent = _make_agent(max_epochs=40, train_dir=str(tmp_path), save_best_after=5)
    agent.init_tensors()
    agent.obs = agent.env_reset()
    first = None
    rewards = []
    for ep in range(40):
        agent.update_epoch()
        agent.train_epoch()
        r = agent.tensor_dict["rewards"].mean().item()
        rewards.append(r)
        first = first if first is not None else r
    assert all(math.isfinite(x) for x in rewards)
    assert np.mean(rewards[-5:]) > np.mean(rewards[:5]) + 0.002, rewards  # the policy learns (shaped x0.01)
    assert float(agent.lr) != 3e-4  # adaptive schedule moved the LR
    fn = str(tmp_path / "ckpt")
    agent.save(fn)
    other = _make_agent(seed=1, train_dir=str(tmp_path))
    other.restore(fn + ".pth")
    for a, b in zip(agent.model.state_dict().values(), other.model.state_dict().values()):
        assert torch.equal(a, b)
    assert other.epoch_num == agent.epoch_num
    # restored parameters still live in the flat buffer (grads land where Adam reads them)
    p0 = next(other.model.parameters())
    assert p0.data_ptr() == other.flat.params.data_ptr()
    # the checkpoint records the env it was trained against; a changed action scaling is refused
    ck = torch.load(fn + ".pth", weights_only=True)
    assert ck["env_signature"]["obs_dim"] == agent.obs_shape[0] and ck["env_signature"]["actions_num"] == agent.actions_num
    ck["env_signature"]["action_scale"] = 0.5
    torch.save(ck, fn + "_other_env.pth")
    from allsteps_isaaclab_amd.learning.models import check_env_signature, env_signature

    cur = dict(env_signature(other.vec_env, other.obs_shape, other.actions_num), action_scale=1.0)
    with pytest.raises(ValueError, match="action_scale"):
        check_env_signature(ck["env_signature"], cur, fn)
    ck["env_signature"]["obs_dim"] += 1
    torch.save(ck, fn + "_other_env.pth")
    with pytest.raises(ValueError, match="obs_dim"):
        other.restore(fn + "_other_env.pth")


def test_runner_train_loop(tmp_path):
    from allsteps_isaaclab_amd.learning import Runner

    params = agent_params(32, max_epochs=2, train_dir=str(tmp_path))
    params["config"]["vec_env"] = ToyReachEnv(32)
    runner = Runner()
    runner.load({"params": params})
    runner.run({"train": True, "play": False, "sigma": "0.5"})
    agent = runner.agent
    assert agent.epoch_num == 2
    saved = [f for f in os.listdir(os.path.join(tmp_path, agent.experiment_name, "nn"))]
    assert saved and all(f.endswith(".pth") for f in saved)
    lines = open(os.path.join(tmp_path, agent.experiment_name, "summaries", "metrics.jsonl")).read().splitlines()
    assert len(lines) == 2 and '"a_loss"' in lines[0] and '"lr"' in lines[1]
    player = runner.create_player()
    player.restore(os.path.join(tmp_path, agent.experiment_name, "nn", saved[0]))
    res = player.run(max_steps=50)
    assert res["steps"] == 50


def test_mirror_agent_symmetry_off_is_a2c():
    from allsteps_isaaclab_amd.learning.a2c_ppo_mirroring import A2CAgentSymmetry

    params = agent_params(16)
    params["config"]["vec_env"] = ToyReachEnv(16)
    ag = A2CAgentSymmetry("run", params)
    assert not ag.symmetry and ag.batch_size == 16 * 16


# ---------------------------------------------------------------- multi-process (gloo, world 2)

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dist_worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(rank)  # different init per rank: train() must broadcast rank 0's
        params = agent_params(16, multi_gpu=True, multi_gpu_mode=mode, max_epochs=3, train_dir=f"/tmp/ppo_dist_{port}")
        params["seed"] = 5 + rank
        params["config"]["vec_env"] = ToyReachEnv(16, seed=rank)
        agent = A.A2CAgent("run", params)
        agent.train()
        # a numpy copy (pickled by value): a torch tensor would be shared through a file descriptor that
        # vanishes with this process if the parent reads the queue after it has exited
        q.put((rank, agent.flat.params.detach().numpy().copy(), float(agent.lr), agent.dataset.batch_size,
               agent.dataset.minibatch_size, agent.frame))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["allreduce", "allgather"])
def test_multi_gpu_modes_keep_ranks_identical(mode, world):
    """Both exchange modes at world 2 and 3 (odd): parameters and LR identical on
    every rank after 3 epochs, the allgather batch / minibatch scaled by the world size, frames counting
    every rank's env steps (the allreduce step's arithmetic: test_allreduce_minibatch_step_equals_mean_gradient_step)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, p0, lr0, bs0, mb0, fr0 = res[0]
    for rank, p1, lr1, bs1, mb1, fr1 in res[1:]:
        assert np.array_equal(p0, p1), f"{mode}: rank {rank} diverged from rank 0"
        assert (lr1, bs1, mb1, fr1) == (lr0, bs0, mb0, fr0)
    if mode == "allgather":
        assert (bs0, mb0) == (world * 16 * 16, world * 16 * 4)  # global batch, world-scaled minibatch
    else:
        assert (bs0, mb0) == (16 * 16, 16 * 4)
    assert fr0 == 3 * world * 16 * 16  # frames count every rank's env steps


# ------------------------------ the allreduce exchange vs a single-process step on the mean gradient

def _mb_batch(rank: int, B: int, device: str = "cpu") -> dict:
    g = torch.Generator(device=device).manual_seed(500 + rank)
    r = lambda *s: torch.randn(*s, device=device, generator=g)  # noqa: E731
    return {"obses": r(B, 5) * 2 + 0.5, "actions": r(B, 2), "neglogpacs": r(B).abs() * 2 + 3,
            "values": r(B, 1), "returns": r(B, 1) * 2, "mus": r(B, 2) * 0.3,
            "sigmas": torch.exp(r(B, 2) * 0.1), "dones": torch.zeros(B, dtype=torch.uint8, device=device)}


def _mb_agent(multi_gpu: bool):
    params = agent_params(16, multi_gpu=multi_gpu, multi_gpu_mode="allreduce", minibatch_size=16 * 16)
    params["config"]["vec_env"] = ToyReachEnv(16, seed=0)
    torch.manual_seed(3)  # identical initial parameters on every rank and in the reference
    ag = A.A2CAgent("run", params)
    ag.init_tensors()
    ag.model.train()
    return ag


def _allreduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ag = _mb_agent(True)
        ag.prepare_dataset(_mb_batch(rank, ag.batch_size))
        out = ag.calc_gradients(ag.dataset[0])  # backward, [grads | kl] all-reduce (mean), clip, Adam
        q.put((rank, ag.flat.params.detach().numpy().copy(), float(out[3]), ag.flat.grads.detach().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_minibatch_step_equals_mean_gradient_step(world):
    """one all-reduced minibatch step on W ranks (gloo; identical parameters,
    different minibatches) equals a single-process step whose [grads | kl] bucket is the mean of the W
    ranks' own buckets -- the clip (grad_norm 1.0, on the averaged gradient) and Adam included.  Two
    ranks applying the same WRONG gradient (an exchange at the wrong point, a bucket that misses a
    parameter, the KL left un-averaged) would pass "ranks stay identical" but fail this."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_allreduce_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    class _Stop(Exception):
        pass

    # the single-process statement: each rank's own bucket (backward only), then one step on their mean
    buckets = []
    for r in range(world):
        ag = _mb_agent(False)
        ag.prepare_dataset(_mb_batch(r, ag.batch_size))

        def grab(ag=ag):
            buckets.append(ag._bucket.clone())
            raise _Stop

        ag._exchange_grads = grab
        with pytest.raises(_Stop):
            ag.calc_gradients(ag.dataset[0])
    mean = torch.stack(buckets).sum(0) / world
    ref = _mb_agent(False)
    ref.prepare_dataset(_mb_batch(0, ref.batch_size))
    ref._exchange_grads = lambda: ref._bucket.copy_(mean)
    out = ref.calc_gradients(ref.dataset[0])
    p_ref = ref.flat.params.detach().numpy()
    assert float(torch.linalg.vector_norm(mean[:-1])) > ref.grad_norm  # the clip is active in this step
    for rank, p, kl, grads in res:
        assert np.array_equal(p, res[0][1]), f"rank {rank} diverged"
        np.testing.assert_allclose(p, p_ref, rtol=1e-6, atol=1e-7, err_msg=f"rank {rank} vs mean-gradient step")
        assert kl == pytest.approx(float(out[3]), rel=1e-6)  # the KL slot is averaged with the gradients
        np.testing.assert_allclose(grads, ref.flat.grads.detach().numpy(), rtol=1e-6, atol=1e-9)
