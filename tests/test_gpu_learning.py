"""PPO trainer on the HIP env: the reference's train.py flow end to end on
cuda:0 -- registry -> AllstepsEnv (native) -> RlGamesVecEnvWrapper -> Runner -> A2CAgentSymmetry."""

import math
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_train_script_runs_on_allsteps(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
    import train

    runner, _ = train.main(["--task", "Allsteps-v0", "--headless", "--num_envs", "1024", "--max_iterations", "3",
                            "--seed", "3", "--log_root", str(tmp_path)])
    agent = runner.agent
    st = agent.last_stats
    assert agent.epoch_num == 3 and agent.frame == 3 * 1024 * 32
    # rollout graphs: epoch 1 eager, epoch 2 captured, epoch 3 replayed; host counters still advance
    assert all(isinstance(g, torch.cuda.CUDAGraph) for g in agent._play_graphs.values())
    assert agent._uw.common_step_counter == 3 * 32
    # replayed env graphs keep the device step counters sane: no spurious curriculum bump (the gate
    # needs mean target index > 12; a random policy stays near 1) -- regression for a captured
    # hipMemsetAsync node that left garbage in the counter bank
    assert int(agent._uw.state["curriculum"][0]) == 0
    assert float(agent._uw.curr_target_index.float().mean()) < 3.0
    for k in ("a_loss", "c_loss", "kl", "entropy", "lr"):
        assert math.isfinite(st[k]), (k, st)
    assert torch.isfinite(agent.flat.params).all()
    # the native env really ran: the step counters advanced and observations are not all zero
    assert agent.tensor_dict["obses"].abs().sum() > 0
    nn_dir = os.path.join(agent.experiment_dir, "nn")
    assert any(f.endswith(".pth") for f in os.listdir(nn_dir))


@pytest.mark.gpu
def test_train_script_runs_on_c5_quadruped(tmp_path):
    """BASELINE C5 is trainable: train.py drives Allsteps-AnymalC-v0 (ANYmal-C's sim settings, DC motor,
    four foot sensors) through RlGamesVecEnvWrapper and the PPO agent of its registry cfg (3 x 128 ELU,
    horizon 24) -- the fused update on a non-walker trunk -- and writes a checkpoint."""
    sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
    import train

    runner, _ = train.main(["--task", "Allsteps-AnymalC-v0", "--headless", "--num_envs", "1024", "--max_iterations",
                            "2", "--seed", "3", "--log_root", str(tmp_path)])
    agent = runner.agent
    assert agent.epoch_num == 2 and agent.frame == 2 * 1024 * 24
    assert agent.obs_shape[0] == 64 and agent.actions_num == 12
    for k in ("a_loss", "c_loss", "kl", "entropy", "lr"):
        assert math.isfinite(agent.last_stats[k]), (k, agent.last_stats)
    assert torch.isfinite(agent.flat.params).all()
    assert agent.tensor_dict["obses"].abs().sum() > 0
    nn_dir = os.path.join(agent.experiment_dir, "nn")
    assert any(f.endswith(".pth") for f in os.listdir(nn_dir))


@pytest.mark.gpu
def test_symmetry_agent_doubles_batch(tmp_path):
    from allsteps_isaaclab_amd import registry
    from allsteps_isaaclab_amd.learning.a2c_ppo_mirroring import A2CAgentSymmetry
    from allsteps_isaaclab_amd.rl_games import RlGamesGpuEnv, RlGamesVecEnvWrapper, env_configurations, vecenv

    cfg = registry.load_cfg_from_registry("Allsteps-v0", "env_cfg_entry_point")
    cfg.scene.num_envs = 256
    env = RlGamesVecEnvWrapper(registry.make("Allsteps-v0", cfg=cfg), "cuda:0", math.inf, 1.0)
    vecenv.register("IsaacRlgWrapper", lambda n, a, **kw: RlGamesGpuEnv(n, a, **kw))
    env_configurations.register("rlgpu", {"vecenv_type": "IsaacRlgWrapper", "env_creator": lambda **kw: env})
    params = registry.load_cfg_from_registry("Allsteps-v0", "rl_games_cfg_entry_point")["params"]
    params["config"].update(num_actors=256, symmetry=True, minibatch_size=4096, max_epochs=1,
                            train_dir=str(tmp_path), print_stats=False)
    agent = A2CAgentSymmetry("run", params)
    agent.init_tensors()
    agent.obs = agent.env_reset()
    batch = agent.play_steps()
    assert batch["obses"].shape == (2 * 256 * 32, 59) and batch["actions"].shape == (2 * 256 * 32, 21)
    h = 256 * 32
    # mirrored half: left/right joint columns swapped
    uw = env.unwrapped
    r, l = uw.right_body_indices, uw.left_body_indices
    assert torch.equal(batch["actions"][h:, r], batch["actions"][:h, l])
    agent.model.train()
    agent.prepare_dataset({k: v for k, v in batch.items() if k not in ("played_frames", "step_time")})
    assert len(agent.dataset) == 2 * h // 4096
    env.close()


class _SpacesOnlyEnv:
    """VecEnv stand-in with the Allsteps spaces (59 obs, 21 actions) for update-only tests."""

    def __init__(self, n):
        from allsteps_isaaclab_amd.envs.spaces import Box

        self.n = n
        self._info = {"observation_space": Box(-math.inf, math.inf, (59,)), "action_space": Box(-1.0, 1.0, (21,)),
                      "state_space": None}

    def get_env_info(self):
        return self._info


def _agents_and_batch(n_envs, mixed, tmp, mp_dtype="float16"):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _toy_env import agent_params
    from allsteps_isaaclab_amd.learning.a2c_continuous import A2CAgent

    def make(fused):
        p = agent_params(n_envs, device="cuda:0", mixed_precision=mixed, fused_update=fused, train_dir=str(tmp),
                         minibatch_size=n_envs * 8, horizon_length=16)
        p["network"]["mlp"]["units"] = [256, 256, 256, 256, 256]
        p["config"]["vec_env"] = _SpacesOnlyEnv(n_envs)
        p["config"]["mixed_precision_dtype"] = mp_dtype
        torch.manual_seed(11)
        a = A2CAgent("run", p)
        a.init_tensors()
        return a

    ref, fus = make(False), make(True)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    B = n_envs * 16
    r = lambda *s: torch.randn(*s, device="cuda:0", generator=g)  # noqa: E731
    batch = {"obses": r(B, 59) * 2 + 0.5, "actions": r(B, 21), "neglogpacs": r(B).abs() * 5 + 20,
             "values": r(B, 1), "returns": r(B, 1) * 2, "mus": r(B, 21) * 0.3,
             "sigmas": torch.exp(r(B, 21) * 0.1), "dones": torch.zeros(B, dtype=torch.uint8, device="cuda:0")}
    for a in (ref, fus):
        a.model.train()
        a.prepare_dataset({k: v.clone() for k, v in batch.items()})
    return ref, fus


def _grads(agent):
    return {n: p.grad.detach().clone() for n, p in agent.model.named_parameters()}


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_fused_minibatch_step_matches_autograd_fp32(tmp_path, graphs):
    ref, fus = _agents_and_batch(256, mixed=False, tmp=tmp_path)
    fus.fused.fuse_norm = False  # this test writes the gradients between step_a and step_b
    fus.fused.use_graphs = graphs
    ref.truncate_grads = False  # compare raw gradients (the fused clip happens inside the Adam kernel)
    saved = ref.optimizer.step
    ref.optimizer.step = lambda: None
    out = ref.calc_gradients(ref.dataset[0])
    ref.optimizer.step = saved
    fus.fused.begin_epoch()
    if graphs:  # first call runs eagerly (warm-up); undo its side effects, then capture + replay
        rms = fus.model.running_mean_std
        keep = [t.clone() for t in (rms.running_mean, rms.running_var, rms.count, fus.fused.ds["mu"],
                                    fus.fused.ds["sigma"])]
        fus.fused.step_a(True)
        for t, v in zip((rms.running_mean, rms.running_var, rms.count, fus.fused.ds["mu"], fus.fused.ds["sigma"]),
                        keep):
            t.copy_(v)
        fus.flat.grads.zero_()
    fus.fused.step_a(True)
    torch.cuda.synchronize()
    if graphs:
        assert isinstance(fus.fused.graphs[("a", True)], torch.cuda.CUDAGraph)
    gr, gf = _grads(ref), _grads(fus)
    for k in gr:
        err = (gr[k] - gf[k]).abs().max().item()
        scale = gr[k].abs().max().item() + 1e-8
        assert err <= 2e-4 * scale + 1e-7, (k, err, scale)
    # obs normaliser (train-mode update of the first mini-epoch), KL and statistics
    for b in ("running_mean", "running_var", "count"):
        torch.testing.assert_close(getattr(fus.model.running_mean_std, b), getattr(ref.model.running_mean_std, b),
                                   rtol=1e-6, atol=1e-9)
    a_loss, c_loss, entropy, kl = out[0], out[1], out[2], out[3]
    st = fus.fused.stats[0]
    torch.testing.assert_close(st[0], a_loss, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(st[1], c_loss, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(st[3], entropy, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(st[4], kl.reshape(()), rtol=1e-3, atol=1e-6)
    # update_mu_sigma: the dataset rows of minibatch 0 now hold the current policy
    torch.testing.assert_close(fus.dataset.values_dict["mu"][:fus.minibatch_size], out[4], rtol=1e-5, atol=1e-5)
    # optimizer half: same gradients in -> same clipped Adam step out
    for (n, pf), (_, pr) in zip(fus.model.named_parameters(), ref.model.named_parameters()):
        pf.grad.copy_(pr.grad)
    ref.truncate_grads = True
    g = ref.flat.grads
    coef = torch.clamp(ref.grad_norm / (torch.linalg.vector_norm(g) + 1e-6), max=1.0)
    g.mul_(coef)
    ref.optimizer.step()
    fus.fused.step_b()
    torch.cuda.synchronize()
    for (n, pf), (_, pr) in zip(fus.model.named_parameters(), ref.model.named_parameters()):
        torch.testing.assert_close(pf, pr, rtol=1e-5, atol=2e-7, msg=n)
    assert int(fus.fused.mb_idx) == 1 % len(fus.dataset)


@pytest.mark.gpu
@pytest.mark.parametrize("mp_dtype,tol", [("float16", 1e-2), ("bfloat16", 3e-2)])
def test_fused_lowp_step_close_to_fp32_autograd(tmp_path, mp_dtype, tol):
    """mixed_precision (rl_games: fp16 autocast + GradScaler; bf16 selectable): the fused 16-bit
    trunk's gradients against the fp32 autograd step, after the loss scale is divided out (the fused
    step leaves scaled gradients in the bucket; the Adam kernel unscales them).  fp16 keeps 3 more
    mantissa bits than bf16, hence the tighter bound."""
    ref, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path, mp_dtype=mp_dtype)
    assert fus.fused.dt == (torch.float16 if mp_dtype == "float16" else torch.bfloat16)
    ref.mixed_precision = False
    ref.scaler_state = None
    ref.truncate_grads = False
    saved = ref.optimizer.step
    ref.optimizer.step = lambda: None
    ref.calc_gradients(ref.dataset[0])
    ref.optimizer.step = saved
    fus.fused.begin_epoch()
    fus.fused.step_a(True)
    torch.cuda.synchronize()
    scale = float(fus.scaler_state[0])
    assert scale == 2.0 ** 16
    gr, gf = _grads(ref), _grads(fus)
    for k in gr:
        g = gf[k] / scale
        rel = (gr[k] - g).norm().item() / (gr[k].norm().item() + 1e-12)
        assert rel < tol, (k, rel)


@pytest.mark.gpu
def test_fused_loss_scaler_skips_and_grows(tmp_path):
    """GradScaler semantics on the device (ppo_adam / ppo_tail): a non-finite gradient skips the whole
    Adam step (parameters, moments and the step count unchanged) and halves the scale; after
    SCALER_GROWTH_INTERVAL good steps in a row the scale doubles; a good step applies g / scale."""
    from allsteps_isaaclab_amd.learning.fused import SCALER_GROWTH_INTERVAL

    _, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path)
    fus.fused.fuse_norm = False  # this test writes the gradients between step_a and step_b
    fus.fused.use_graphs = False
    fus.fused.begin_epoch()
    fus.fused.step_a(True)
    torch.cuda.synchronize()
    p0 = fus.flat.params.clone()
    m0 = fus.optimizer.exp_avg.clone()
    step0 = float(fus.optimizer.step_t)
    good = fus.flat.grads.clone()
    fus.flat.grads[3] = float("inf")
    fus.fused.step_b()
    torch.cuda.synchronize()
    assert torch.equal(fus.flat.params, p0) and torch.equal(fus.optimizer.exp_avg, m0)
    assert float(fus.optimizer.step_t) == step0
    assert float(fus.scaler_state[0]) == 2.0 ** 15 and float(fus.scaler_state[1]) == 0.0
    # a good step at the end of a growth interval: unscaled update, then the scale doubles
    fus.flat.grads.copy_(good / 2.0)  # the gradients of the halved scale
    fus.scaler_state[1] = SCALER_GROWTH_INTERVAL - 1
    lr0 = fus.lr.clone()  # the adaptive LR moves after the Adam kernel, in ppo_tail
    fus.fused.step_b()
    torch.cuda.synchronize()
    assert float(fus.optimizer.step_t) == step0 + 1
    assert float(fus.scaler_state[0]) == 2.0 ** 16 and float(fus.scaler_state[1]) == 0.0
    assert not torch.equal(fus.flat.params, p0)
    # the update equals an fp32 Adam step on g / scale (FlatAdam, the same clip)
    ref = fus.flat.params.clone()
    fus.flat.params.copy_(p0)
    fus.optimizer.exp_avg.copy_(m0)
    fus.optimizer.exp_avg_sq.zero_()
    fus.optimizer.step_t.fill_(step0)
    fus.lr.copy_(lr0)
    g = good / 2.0 / 2.0 ** 15
    if fus.truncate_grads:
        g = g * torch.clamp(fus.grad_norm / (torch.linalg.vector_norm(g) + 1e-6), max=1.0)
    fus.flat.grads.copy_(g)
    fus.optimizer.step()
    torch.testing.assert_close(ref, fus.flat.params, rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_fused_loss_scaler_clips_finite_overflowing_norm(tmp_path):
    """found_inf is an OR over isfinite(g), not a test of the norm: finite scaled gradients whose
    squared sum overflows fp32 (||g|| * scale > 1.8e19) are unscaled, clipped and applied like
    torch's GradScaler + clip_grad_norm_ would, and the scale keeps growing (no skip)."""
    _, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path)
    fus.fused.fuse_norm = False  # this test writes the gradients between step_a and step_b
    fus.fused.use_graphs = False
    fus.fused.begin_epoch()
    fus.fused.step_a(True)
    torch.cuda.synchronize()
    p0 = fus.flat.params.clone()
    m0 = fus.optimizer.exp_avg.clone()
    step0 = float(fus.optimizer.step_t)
    scale = float(fus.scaler_state[0])
    tracker = float(fus.scaler_state[1])
    good = fus.flat.grads.clone()
    good[3] = 3e19  # finite; its square overflows fp32, its unscaled square does not
    assert torch.isinf((good * good).sum())
    fus.flat.grads.copy_(good)
    lr0 = fus.lr.clone()
    fus.fused.step_b()
    torch.cuda.synchronize()
    assert float(fus.optimizer.step_t) == step0 + 1
    assert float(fus.scaler_state[0]) == scale and float(fus.scaler_state[1]) == tracker + 1
    ref = fus.flat.params.clone()
    assert torch.isfinite(ref).all()
    fus.flat.params.copy_(p0)
    fus.optimizer.exp_avg.copy_(m0)
    fus.optimizer.exp_avg_sq.zero_()
    fus.optimizer.step_t.fill_(step0)
    fus.lr.copy_(lr0)
    g = good / scale
    if fus.truncate_grads:
        g = g * torch.clamp(fus.grad_norm / (torch.linalg.vector_norm(g) + 1e-6), max=1.0)
    fus.flat.grads.copy_(g)
    fus.optimizer.step()
    torch.testing.assert_close(ref, fus.flat.params, rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_fused_unscaled_nan_gradient_poisons_the_step_like_torch(tmp_path):
    """Without a scaler (fp32 trunk), clip_grad_norm_ of a NaN gradient gives a NaN norm and a NaN
    clip coefficient, so torch turns every parameter NaN; the fused path does the same instead of
    clipping the finite elements to zero."""
    _, fus = _agents_and_batch(256, mixed=False, tmp=tmp_path)
    fus.fused.fuse_norm = False  # this test writes the gradients between step_a and step_b
    if not fus.truncate_grads:
        pytest.skip("agent config without grad clipping")
    fus.fused.use_graphs = False
    fus.fused.begin_epoch()
    fus.fused.step_a(True)
    torch.cuda.synchronize()
    fus.flat.grads[3] = float("nan")
    fus.fused.step_b()
    torch.cuda.synchronize()
    assert torch.isnan(fus.flat.params).all()


@pytest.mark.gpu
def test_fused_gradient_norm_from_the_reduce_launch(tmp_path):
    """One GPU, no all-reduce: the reduce launch leaves the gradient-norm partials (ppo_reduce_rows_norm)
    and step B skips the separate norm pass.  Against the separate pass on the same minibatch: the same
    gradients bit for bit, the norm's partial count is the reduce's block count + 1, and the clipped Adam
    step agrees to fp32 rounding (the squares summed in another fixed order)."""
    outs = []
    for fuse in (False, True):
        _, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path / str(fuse))
        fus.fused.fuse_norm = fuse
        fus.fused.begin_epoch()
        fus.fused.step_a(True)
        g = fus.flat.grads.clone()
        fus.fused.step_b()
        torch.cuda.synchronize()
        outs.append((g, fus.flat.params.clone(), fus.scaler_state.clone(), fus.fused._red_nblk.value))
    (ga, pa, sa, _), (gb, pb, sb, nb) = outs
    assert torch.equal(ga, gb) and torch.equal(sa, sb)
    assert nb > 1
    torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
def test_fused_train_epoch_runs_graph_replays(tmp_path):
    ref, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path)
    fus.obs = None
    p0 = fus.flat.params.clone()
    fus.model.train()
    # one full fused epoch over the prepared dataset (mini_epochs x minibatches replays)
    out = fus._train_epoch_fused(0.0, 0.0, 0.0)
    stats = out[4]
    assert all(math.isfinite(float(v)) for v in stats.values()), stats
    assert not torch.equal(p0, fus.flat.params)
    n = fus.mini_epochs_num * len(fus.dataset)
    assert int(fus.fused.stat_idx) == n and int(fus.fused.mb_idx) == 0
    # the synthetic dataset's random old neglogp gives some rows a ratio of ~1e4: with the 16-bit head
    # gradient autocast hands the heads' Linear backward, such a minibatch overflows fp16 at scale 2^16 and
    # GradScaler skips it (scale halved, Adam's step count kept) -- the reference's behaviour too
    from allsteps_isaaclab_amd.learning.fused import SCALER_INIT
    skips = round(math.log2(SCALER_INIT / float(fus.scaler_state[0])))
    assert 0 <= skips < n
    assert float(fus.optimizer.step_t) == n - skips
    # one graph per mini-epoch: the normaliser-updating first mini-epoch ran once (eagerly, the warm-up
    # of its variant), the frozen ones ran eagerly, then were captured and replayed
    n_mb = len(fus.dataset)
    g = fus.fused.graphs
    assert set(g) == {("mb", n_mb, True), ("mb", n_mb, False)}
    assert g[("mb", n_mb, True)] == "warm" and isinstance(g[("mb", n_mb, False)], torch.cuda.CUDAGraph)
    fus._train_epoch_fused(0.0, 0.0, 0.0)
    assert all(isinstance(v, torch.cuda.CUDAGraph) for v in g.values())
    assert int(fus.fused.stat_idx) == n and int(fus.fused.mb_idx) == 0


@pytest.mark.gpu
def test_mini_epoch_graph_equals_per_minibatch_graphs(tmp_path):
    """run_minibatches (a mini-epoch's n minibatch steps as one graph) against the step_a / step_b graph
    pair per minibatch, over three mini-epochs (eager warm-up, capture + replay, replay): the same kernels
    in the same order, so parameters, Adam moments and count, scaler, LR, normaliser, statistics and the
    device counters agree bit for bit."""
    outs = []
    for whole in (False, True):
        _, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path / str(whole))
        f = fus.fused
        n_mb = len(fus.dataset)
        f.begin_epoch()
        for ep in range(3):
            if whole:
                f.run_minibatches(n_mb, ep == 0)
            else:
                for _ in range(n_mb):
                    f.step_a(ep == 0)
                    f.step_b()
        torch.cuda.synchronize()
        rms = fus.model.running_mean_std
        outs.append([t.clone() for t in (fus.flat.params, fus.optimizer.exp_avg, fus.optimizer.exp_avg_sq,
                                         fus.optimizer.step_t, fus.scaler_state, fus.lr, f.stats, f.mb_idx,
                                         f.stat_idx, rms.running_mean, rms.running_var, rms.count)])
        if whole:
            assert isinstance(f.graphs[("mb", n_mb, False)], torch.cuda.CUDAGraph)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert int(outs[1][8]) == 3 * n_mb


@pytest.mark.gpu
def test_env_step_replayed_from_graph_matches_eager():
    """AllstepsEnv.step captured once in a HIP graph (graph-safe counters) and replayed with fresh
    actions gives bit-identical obs / rewards / dones to eager stepping, resets included."""
    from allsteps_isaaclab_amd import registry

    envs = []
    for graph in (False, True):
        cfg = registry.load_cfg_from_registry("Allsteps-v0", "env_cfg_entry_point")
        cfg.scene.num_envs = 512
        e = registry.make("Allsteps-v0", cfg=cfg)
        e.set_graph_capture(graph)
        e.reset()
        envs.append(e)
    eager, ge = envs
    g = torch.Generator(device="cuda:0").manual_seed(9)
    acts = [torch.rand(512, 21, device="cuda:0", generator=g) * 2 - 1 for _ in range(150)]
    static = torch.zeros(512, 21, device="cuda:0")
    static.copy_(acts[0])
    ge.step(static)  # warm-up (eager) step 0
    graph = torch.cuda.CUDAGraph()
    static.copy_(acts[1])
    with torch.cuda.graph(graph):
        out = ge.step(static)
    resets = 0
    for k in range(150):
        o1, r1, t1, tr1, _ = eager.step(acts[k])
        if k == 0:
            continue
        static.copy_(acts[k])
        graph.replay()
        torch.cuda.synchronize()
        o2, r2, t2, tr2 = out[0]["policy"], out[1], out[2], out[3]
        assert torch.equal(o1["policy"], o2) and torch.equal(r1, r2), k
        assert torch.equal(t1, t2) and torch.equal(tr1, tr2), k
        resets += int((t1 | tr1).sum())
    assert resets > 0  # the in-kernel reset path ran inside the replays
    for e in envs:
        e.close()


@pytest.mark.gpu
def test_rollout_policy_sampling_kernel(tmp_path):
    """ppo_policy_sample: N(mu, sigma) draws (moments), neglogp / denormalised value formulas, and the
    same draw for the same step counter (graph replays are reproducible)."""
    ref, fus = _agents_and_batch(256, mixed=False, tmp=tmp_path)
    f = fus.fused
    n = 4096
    f.init_rollout(n, seed=123)
    with torch.no_grad():
        fus.model.a2c_network.sigma.fill_(-0.7)
        fus.model.value_mean_std.running_mean.fill_(0.3)
        fus.model.value_mean_std.running_var.fill_(4.0)
    obs = torch.randn(n, 59, device="cuda:0")
    out = {k: torch.empty(n, 21, device="cuda:0") for k in ("actions", "mus", "sigmas")}
    out["neglogpacs"] = torch.empty(n, device="cuda:0")
    out["values"] = torch.empty(n, 1, device="cuda:0")
    f.policy_act(obs, out)
    first = out["actions"].clone()
    fus.model.eval()
    ref_out = fus.model({"is_train": False, "prev_actions": None, "obs": obs})  # fp32 torch forward
    torch.testing.assert_close(out["mus"], ref_out["mus"], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out["values"], ref_out["values"], rtol=1e-4, atol=1e-4)
    sig = math.exp(-0.7)
    assert torch.allclose(out["sigmas"], torch.full_like(out["sigmas"], sig))
    z = (out["actions"] - out["mus"]) / sig
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1.0) < 0.01
    from allsteps_isaaclab_amd.learning.models import neglogp

    ls = torch.full_like(out["mus"], -0.7)
    torch.testing.assert_close(out["neglogpacs"], neglogp(out["actions"], out["mus"], out["sigmas"], ls),
                               rtol=1e-5, atol=1e-4)
    f.policy_act(obs, out)
    assert not torch.equal(first, out["actions"])  # counter advanced: fresh draws
    f.step_ctr.fill_(0)
    f.policy_act(obs, out)
    assert torch.equal(first, out["actions"])  # same counter, same draws


@pytest.mark.gpu
def test_play_script_restores_trained_checkpoint(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
    import play
    import train

    runner, _ = train.main(["--task", "Allsteps-v0", "--num_envs", "1024", "--max_iterations", "1", "--seed", "4",
                            "--log_root", str(tmp_path)])
    nn_dir = os.path.join(runner.agent.experiment_dir, "nn")
    ckpt = os.path.join(nn_dir, sorted(os.listdir(nn_dir))[0])
    out = play.main(["--task", "Allsteps-v0", "--num_envs", "256", "--checkpoint", ckpt, "--steps", "200"])
    assert out["steps"] == 200 and out["episodes"] > 0 and math.isfinite(out["mean_reward"])
    # --video (play.py:111-127): env 0's rgb_array frames from step 0, --video_length of them, then stop
    from PIL import Image

    out = play.main(["--task", "Allsteps-v0", "--num_envs", "64", "--checkpoint", ckpt, "--video",
                     "--video_length", "24"])
    assert out["steps"] == 24 and len(out["video"]) == 1
    assert os.path.dirname(out["video"][0]) == os.path.join(os.path.dirname(nn_dir), "videos", "play")
    im = Image.open(out["video"][0])
    assert im.n_frames == 24 and im.size == (640, 360)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,dt", [(32768, torch.bfloat16), (1000, torch.bfloat16), (32768, torch.float16),
                                     (1000, torch.float16)])
def test_fused_mlp_forward_kernel(rows, dt):
    """ppo_mlp_forward (weight-stationary MFMA, activations through LDS) vs an fp32 torch statement of the
    same rounding points: each of the five layers rounded to the 16-bit type once (as autocast keeps
    them); the heads as under autocast: 16-bit layer-5 activations, weights and bias, fp32 accumulation, a
    16-bit output."""
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    tol = 0.05 if dt == torch.bfloat16 else 0.01
    g = torch.Generator(device="cuda:0").manual_seed(3)
    dev = "cuda:0"
    x = torch.zeros(rows, 64, device=dev)
    x[:, :59] = torch.randn(rows, 59, device=dev, generator=g).clamp(-5, 5)
    xb = x.to(dt)
    ws = [(torch.randn(256, 64 if i == 0 else 256, device=dev, generator=g) / (8 if i == 0 else 16)).to(dt)
          for i in range(5)]
    ws[0][:, 59:] = 0
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(5)]
    wh = torch.randn(22, 256, device=dev, generator=g) / 16
    bh = torch.randn(22, device=dev, generator=g) * 0.1
    hs = [torch.empty(rows, 256, device=dev, dtype=dt) for _ in range(5)]
    head = torch.empty(rows, 22, device=dev)
    a = FU.PpoMlpFwd()
    a.x = xb.data_ptr()
    for i in range(5):
        a.w[i] = ws[i].data_ptr()
        a.b[i] = bs[i].data_ptr()
        a.h[i] = hs[i].data_ptr()
    a.wh, a.bh, a.head, a.rows, a.nh = wh.data_ptr(), bh.data_ptr(), head.data_ptr(), rows, 22
    a.x_stride, a.h_stride, a.dtype = 64, 256, FU.PPO_DT[dt]
    FU._check(L.ppo_mlp_forward(C.byref(a), torch.cuda.current_stream().cuda_stream), "ppo_mlp_forward")
    torch.cuda.synchronize()
    hin = xb.float()
    for i in range(5):
        z = hin @ ws[i].float().t() + bs[i]
        y = torch.nn.functional.elu(z)
        got = hs[i].float()
        yr = y.to(dt).float()
        assert (got - yr).abs().max().item() < tol, i
        frac = ((got - yr).abs() > 1e-6).float().mean().item()
        assert frac < 0.02, (i, frac)  # only rounding-boundary flips
        hin = got  # chain on the kernel's own rounding, as the kernel does
    ref_head = (hin @ wh.to(dt).float().t() + bh.to(dt).float()).to(dt).float()
    # one 16-bit rounding step apart at most (fp32 sums in another order)
    htol = 1e-2 if dt == torch.bfloat16 else 2e-3
    torch.testing.assert_close(head, ref_head, rtol=htol, atol=htol)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,dt", [(32768, torch.float16), (1000, torch.bfloat16)])
def test_fused_mlp_forward_normalises_its_input(rows, dt):
    """ppo_mlp_forward with `obs` set forms the layer-0 input in-kernel (minibatch `*mb_idx` of the fp32
    observations, the RunningMeanStd formula of ppo_obs_normalize): its x_out equals the separate
    normalisation kernel's output bit for bit, and the layer outputs equal those of a forward fed that
    output."""
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(5)
    obs = torch.randn(3 * rows, 59, device=dev, generator=g) * 3
    idx = torch.tensor([2], dtype=torch.int32, device=dev)
    mean = torch.randn(59, device=dev, generator=g, dtype=torch.float64)
    var = torch.rand(59, device=dev, generator=g, dtype=torch.float64) * 4
    s = torch.cuda.current_stream().cuda_stream
    x_ref = torch.zeros(rows, 72, device=dev, dtype=dt)
    FU._check(L.ppo_obs_normalize(obs.data_ptr(), idx.data_ptr(), rows, 59, mean.data_ptr(), var.data_ptr(), 1e-5,
                                  x_ref.data_ptr(), 64, 72, FU.PPO_DT[dt], s), "ppo_obs_normalize")
    ws = [(torch.randn(256, 64 if i == 0 else 256, device=dev, generator=g) / 16).to(dt) for i in range(5)]
    bs = [torch.randn(256, device=dev, generator=g) * 0.1 for _ in range(5)]
    wh, bh = torch.randn(22, 256, device=dev, generator=g) / 16, torch.zeros(22, device=dev)
    outs = []
    for fused_in in (False, True):
        x_out = torch.zeros(rows, 72, device=dev, dtype=dt)
        hs = [torch.zeros(rows, 264, device=dev, dtype=dt) for _ in range(5)]
        head = torch.zeros(rows, 22, device=dev)
        a = FU.PpoMlpFwd()
        for i in range(5):
            a.w[i], a.b[i], a.h[i] = ws[i].data_ptr(), bs[i].data_ptr(), hs[i].data_ptr()
        a.wh, a.bh, a.head, a.rows, a.nh = wh.data_ptr(), bh.data_ptr(), head.data_ptr(), rows, 22
        a.x_stride, a.h_stride, a.dtype = 72, 264, FU.PPO_DT[dt]
        if fused_in:
            a.obs, a.mb_idx, a.mean, a.var, a.eps, a.obs_dim = (obs.data_ptr(), idx.data_ptr(), mean.data_ptr(),
                                                                var.data_ptr(), 1e-5, 59)
            a.x_out = x_out.data_ptr()
        else:
            a.x = x_ref.data_ptr()
        FU._check(L.ppo_mlp_forward(C.byref(a), s), "ppo_mlp_forward")
        torch.cuda.synchronize()
        outs.append((x_out.clone(), [t.clone() for t in hs], head.clone()))
    (_, h_a, hd_a), (x_b, h_b, hd_b) = outs
    assert torch.equal(x_b[:, :64], x_ref[:, :64])
    assert all(torch.equal(p, q) for p, q in zip(h_a, h_b)) and torch.equal(hd_a, hd_b)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,A,dt", [(32768, 21, torch.float16), (1000, 12, torch.bfloat16)])
def test_fused_mlp_forward_runs_the_losses(rows, A, dt):
    """ppo_mlp_forward with loss.A set runs ppo_loss_grad's work in its epilogue: the 16-bit head gradient,
    the block partials and the dataset's updated mu / sigma equal a forward followed by ppo_loss_grad bit for
    bit (the same loss block, ppo_loss.h, on the same head values), and the activations are unchanged."""
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(12)
    r = lambda *sh: torch.randn(*sh, device=dev, generator=g)  # noqa: E731
    obs = r(2 * rows, 59) * 2
    idx = torch.tensor([1], dtype=torch.int32, device=dev)
    mean, var = r(59).double() * 0.1, torch.rand(59, device=dev, generator=g, dtype=torch.float64) + 0.5
    ws = [(r(256, 64 if i == 0 else 256) / 16).to(dt) for i in range(5)]
    bs = [r(256) * 0.1 for _ in range(5)]
    wh, bh = r(A + 1, 256) / 16, r(A + 1) * 0.1
    logstd = r(A) * 0.1
    ds0 = {"actions": r(2 * rows, A), "mu": r(2 * rows, A) * 0.3, "sigma": torch.exp(r(2 * rows, A) * 0.1),
           "nlp": r(2 * rows).abs() * 2 + 25, "adv": r(2 * rows), "v": r(2 * rows), "ret": r(2 * rows)}
    cfg = FU.PpoLossCfg(0.2, 4.0, 0.0, 1e-4, 1.1, 1, 1, 1)
    scale = torch.tensor([1024.0], device=dev)
    s = torch.cuda.current_stream().cuda_stream
    nblk = L.ppo_loss_blocks(rows)
    outs = []
    for fused in (False, True):
        ds = {k: v.clone() for k, v in ds0.items()}
        x_out = torch.zeros(rows, 72, device=dev, dtype=dt)
        hs = [torch.zeros(rows, 264, device=dev, dtype=dt) for _ in range(5)]
        head = torch.zeros(rows, A + 1, device=dev)
        dlp = torch.full((rows, 32), 7.0, device=dev, dtype=dt)
        part = torch.zeros(nblk, 2 * A + 1 + 5, device=dev)
        a = FU.PpoMlpFwd()
        for i in range(5):
            a.w[i], a.b[i], a.h[i] = ws[i].data_ptr(), bs[i].data_ptr(), hs[i].data_ptr()
        a.wh, a.bh, a.head, a.rows, a.nh = wh.data_ptr(), bh.data_ptr(), head.data_ptr(), rows, A + 1
        a.x_stride, a.h_stride, a.dtype = 72, 264, FU.PPO_DT[dt]
        a.obs, a.mb_idx, a.mean, a.var, a.eps, a.obs_dim = (obs.data_ptr(), idx.data_ptr(), mean.data_ptr(),
                                                            var.data_ptr(), 1e-5, 59)
        a.x_out = x_out.data_ptr()
        if fused:
            fl = a.loss
            fl.A, fl.logstd, fl.actions, fl.ds_mu, fl.ds_sigma = (A, logstd.data_ptr(), ds["actions"].data_ptr(),
                                                                  ds["mu"].data_ptr(), ds["sigma"].data_ptr())
            fl.old_neglogp, fl.advantages, fl.old_values, fl.returns = (ds["nlp"].data_ptr(), ds["adv"].data_ptr(),
                                                                        ds["v"].data_ptr(), ds["ret"].data_ptr())
            fl.cfg, fl.grad_scale, fl.dhead_lp, fl.partials = cfg, scale.data_ptr(), dlp.data_ptr(), part.data_ptr()
        FU._check(L.ppo_mlp_forward(C.byref(a), s), "ppo_mlp_forward")
        if not fused:
            FU._check(L.ppo_loss_grad(head.data_ptr(), logstd.data_ptr(), A, rows, idx.data_ptr(),
                                      ds["actions"].data_ptr(), ds["mu"].data_ptr(), ds["sigma"].data_ptr(),
                                      ds["nlp"].data_ptr(), ds["adv"].data_ptr(), ds["v"].data_ptr(),
                                      ds["ret"].data_ptr(), cfg, scale.data_ptr(), None, part.data_ptr(),
                                      dlp.data_ptr(), FU.PPO_DT[dt], s), "ppo_loss_grad")
        torch.cuda.synchronize()
        outs.append([x_out, *hs, head, dlp, part, ds["mu"], ds["sigma"]])
    for i, (p, q) in enumerate(zip(*outs)):
        assert torch.equal(p, q), i


@pytest.mark.gpu
@pytest.mark.parametrize("rows,splits,dt", [(32768, None, torch.bfloat16), (1000, [3, 2, 5, 1, 4, 3], torch.bfloat16),
                                            (64, [1] * 6, torch.bfloat16), (32768, None, torch.float16),
                                            (1000, [2, 3, 3, 3, 3, 7], torch.float16)])
def test_weight_grads_kernel(rows, splits, dt):
    """ppo_weight_grads (MFMA, transposed LDS reads) vs fp32 torch on the same 16-bit inputs: per job l and
    split s, part[l][s] = dz[rows of s]^T [hin | 1] over columns 0..kin for the trunk layers, dhead^T h5
    for the heads (job 5, 32 output rows, no bias column) -- the products of two bf16 or two fp16 values
    are exact in fp32; only the summation order differs.  Columns past the bias column stay untouched;
    ragged splits (rows not a multiple of splits or of the 64-row stage), per-job split counts and a
    trunk pair count that is not a multiple of 8 (the last XCD group) are covered; None = the trainer's
    splits (fused.wgrad_splits)."""
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    dev = "cuda:0"
    splits = splits or FU.wgrad_splits(rows)
    g = torch.Generator(device=dev).manual_seed(5)
    widths = [72] + [264] * 5
    dz = [torch.randn(rows, 256 if k < 5 else 32, device=dev, generator=g).to(dt) for k in range(6)]
    hin = [torch.randn(rows, w, device=dev, generator=g).to(dt) for w in widths]
    part = [torch.full((splits[k], 256 if k < 5 else 32, widths[k]), float("nan"), device=dev) for k in range(6)]
    a = FU.PpoWgrad()
    for k in range(6):
        a.dz[k], a.hin[k], a.part[k] = dz[k].data_ptr(), hin[k].data_ptr(), part[k].data_ptr()
        a.kin[k], a.hin_stride[k], a.splits[k] = 64 if k == 0 else 256, widths[k], splits[k]
    a.rows, a.layers, a.dtype = rows, 6, FU.PPO_DT[dt]
    FU._check(L.ppo_weight_grads(C.byref(a), torch.cuda.current_stream().cuda_stream), "ppo_weight_grads")
    torch.cuda.synchronize()
    for k in range(6):
        kin = 64 if k == 0 else 256
        nb = 1 if k < 5 else 0  # bias column
        for s in range(splits[k]):
            r0, r1 = rows * s // splits[k], rows * (s + 1) // splits[k]
            d, h = dz[k][r0:r1].double(), hin[k][r0:r1].double()
            ref = torch.cat([d.t() @ h[:, :kin], d.sum(0)[:, None]], 1).float()[:, :kin + nb]
            got = part[k][s, :, :kin + nb]
            torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * (r1 - r0) ** 0.5, msg=f"job {k} split {s}")
        assert torch.isnan(part[k][:, :, kin + nb:]).all(), k


@pytest.mark.gpu
def test_weight_grads_side_job_equals_loss_finalize():
    """ppo_weight_grads with the loss side job (ppo_wgrad_t.loss) writes what ppo_loss_finalize writes from
    the same loss-kernel partials -- head-bias and log-sigma gradients, the statistics row, the KL -- to fp32
    rounding (the blocks summed in another fixed order), and the weight-gradient partials are unchanged."""
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    dev, A, rows = "cuda:0", 21, 4096
    g = torch.Generator(device=dev).manual_seed(8)
    nblk = L.ppo_loss_blocks(rows)
    partials = torch.randn(nblk, 2 * A + 1 + 5, device=dev, generator=g)
    scale = torch.tensor([256.0], device=dev)
    sidx = torch.tensor([1], device=dev, dtype=torch.int32)
    s = torch.cuda.current_stream().cuda_stream
    outs = []
    for side in (False, True):
        ghb, gls, stats, kl = (torch.zeros(A + 1, device=dev), torch.zeros(A, device=dev), torch.zeros(3, 5, device=dev),
                               torch.zeros(1, device=dev))
        splits = FU.wgrad_splits(rows)
        widths = [72] + [264] * 5
        gg = torch.Generator(device=dev).manual_seed(2)
        dz = [torch.randn(rows, 256 if k < 5 else 32, device=dev, generator=gg).half() for k in range(6)]
        hin = [torch.randn(rows, w, device=dev, generator=gg).half() for w in widths]
        part = [torch.zeros(splits[k], 256 if k < 5 else 32, widths[k], device=dev) for k in range(6)]
        a = FU.PpoWgrad()
        for k in range(6):
            a.dz[k], a.hin[k], a.part[k] = dz[k].data_ptr(), hin[k].data_ptr(), part[k].data_ptr()
            a.kin[k], a.hin_stride[k], a.splits[k] = 64 if k == 0 else 256, widths[k], splits[k]
        a.rows, a.layers, a.dtype = rows, 6, FU.PPO_DT[torch.float16]
        if side:
            f = a.loss
            f.partials, f.nblk, f.A, f.mb_rows, f.entropy_coef = partials.data_ptr(), nblk, A, rows, 0.01
            f.grad_scale, f.grad_head_bias, f.grad_logstd = scale.data_ptr(), ghb.data_ptr(), gls.data_ptr()
            f.stats, f.stat_idx, f.kl_out = stats.data_ptr(), sidx.data_ptr(), kl.data_ptr()
        else:
            FU._check(L.ppo_loss_finalize(partials.data_ptr(), nblk, A, rows, 0.01, scale.data_ptr(), ghb.data_ptr(),
                                          gls.data_ptr(), stats.data_ptr(), sidx.data_ptr(), kl.data_ptr(), s),
                      "ppo_loss_finalize")
        FU._check(L.ppo_weight_grads(C.byref(a), s), "ppo_weight_grads")
        torch.cuda.synchronize()
        outs.append(([ghb, gls, stats, kl], part))
    (sa, pa), (sb, pb) = outs
    for x, y in zip(sa, sb):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-5)
    assert float(sb[2][1].abs().sum()) > 0 and float(sb[2][0].abs().sum()) == 0  # the stat_idx row only
    for x, y in zip(pa, pb):
        assert torch.equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["good_growth", "skip", "no_scaler"])
def test_adam_step_equals_adam_then_tail(case):
    """ppo_adam_step (Adam reading the norm launch's snapshot, the tail run by its first block) against
    ppo_sqnorm + ppo_adam + ppo_tail on the same inputs: parameters, moments, the 16-bit mirror, lr, step,
    the scaler and the counters bit for bit -- a good step that ends a growth interval (scale x2, KL above
    2x the threshold: lr / 1.5), a step skipped on a non-finite gradient (scale x0.5, step kept), and no
    scaler at all."""
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    dev = "cuda:0"
    gen = torch.Generator(device=dev).manual_seed(3)
    n = 300_001
    grads = torch.randn(n, device=dev, generator=gen) * 1e3
    if case == "skip":
        grads[12345] = float("inf")
    p0 = torch.randn(n, device=dev, generator=gen)
    m0 = torch.randn(n, device=dev, generator=gen) * 0.01
    v0 = torch.rand(n, device=dev, generator=gen) * 0.01
    segs = (FU.PpoSeg * 2)(FU.PpoSeg(0, 65536, 0, 256, 256, 0), FU.PpoSeg(65536, 65536, 65536, 256, 256, 1))
    nb = L.ppo_sqnorm_blocks()
    outs = []
    for fused in (False, True):
        p, m, v = p0.clone(), m0.clone(), v0.clone()
        mirror = torch.zeros(2 * 65536, device=dev, dtype=torch.float16)
        lr = torch.tensor([3e-4], device=dev, dtype=torch.float64)
        step = torch.tensor([7.0], device=dev, dtype=torch.float64)
        scaler = None if case == "no_scaler" else torch.tensor([65536.0, 1999.0], device=dev)
        kl = torch.tensor([0.02], device=dev)
        mb = torch.tensor([3], device=dev, dtype=torch.int32)
        st = torch.tensor([5], device=dev, dtype=torch.int32)
        part = torch.zeros(2 * nb, device=dev)
        snap = torch.zeros(4, device=dev, dtype=torch.float64)
        sp = None if scaler is None else scaler.data_ptr()
        if not fused:
            assert L.ppo_sqnorm(grads.data_ptr(), n, sp, part.data_ptr(), None, None, None, None) == 0
            assert L.ppo_adam(p.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), n, part.data_ptr(), nb,
                              1.0, lr.data_ptr(), step.data_ptr(), 0.9, 0.999, 1e-8, segs, 2, mirror.data_ptr(), 2,
                              sp, None) == 0
            assert L.ppo_tail(lr.data_ptr(), kl.data_ptr(), 0.008, 1e-6, 1e-2, step.data_ptr(), mb.data_ptr(), 4,
                              st.data_ptr(), sp, part.data_ptr(), nb, 2000, None) == 0
        else:
            assert L.ppo_sqnorm(grads.data_ptr(), n, sp, part.data_ptr(), lr.data_ptr(), step.data_ptr(),
                                snap.data_ptr(), None) == 0
            a = FU.PpoAdamStep(p.data_ptr(), grads.data_ptr(), m.data_ptr(), v.data_ptr(), n, part.data_ptr(), nb,
                               1.0, 0.9, 0.999, 1e-8, segs, 2, mirror.data_ptr(), 2, snap.data_ptr(), lr.data_ptr(),
                               kl.data_ptr(), 0.008, 1e-6, 1e-2, step.data_ptr(), mb.data_ptr(), 4, st.data_ptr(), sp,
                               2000)
            assert L.ppo_adam_step(C.byref(a), None) == 0
        torch.cuda.synchronize()
        outs.append([p, m, v, mirror, lr, step, kl, mb, st] + ([] if scaler is None else [scaler]))
    for x, y in zip(*outs):
        assert torch.equal(x, y)
    p, _, _, _, lr, step = outs[1][:6]
    assert int(outs[1][7]) == 0 and int(outs[1][8]) == 6  # mb_idx (3 + 1) % 4, stat_idx + 1
    if case == "skip":
        assert torch.equal(p, p0) and float(step) == 7.0 and float(outs[1][-1][0]) == 32768.0
    else:
        assert not torch.equal(p, p0) and float(step) == 8.0
        assert float(lr) == pytest.approx(3e-4 / 1.5)
        if case == "good_growth":
            assert float(outs[1][-1][0]) == 131072.0 and float(outs[1][-1][1]) == 0.0
    # without the snapshot pointer the step refuses to run
    a.snap = None
    assert L.ppo_adam_step(C.byref(a), None) != 0



def test_weight_grads_rejects_bad_arguments():
    import ctypes as C

    from allsteps_isaaclab_amd.learning import fused as FU

    L = FU.load()
    a = FU.PpoWgrad()
    a.rows, a.layers = 128, 1
    a.splits[0] = 1
    assert L.ppo_weight_grads(C.byref(a), None) == -1  # null pointers: refused before any launch
    assert b"bad arguments" in L.ppo_last_error()


@pytest.mark.gpu
def test_rollout_bookkeeping_kernel_matches_reference_ops(tmp_path):
    """ppo_rollout_post + ppo_meter_update == the play_steps tensor ops (shaping, value bootstrap,
    episode sums, AverageMeter updates, reset of the sums) over several steps."""
    from allsteps_isaaclab_amd.learning import a2c_continuous as A

    ref, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path)
    f = fus.fused
    n = 256
    fus.current_rewards = torch.zeros(n, 1, device="cuda:0")
    fus.current_shaped_rewards = torch.zeros(n, 1, device="cuda:0")
    fus.current_lengths = torch.zeros(n, device="cuda:0")
    fus.game_rewards = A.AverageMeter(1, 100, "cuda:0")
    fus.game_shaped_rewards = A.AverageMeter(1, 100, "cuda:0")
    fus.game_lengths = A.AverageMeter(1, 100, "cuda:0")
    f.init_bookkeeping(fus)
    cr, cs, cl = (torch.zeros(n, 1, device="cuda:0"), torch.zeros(n, 1, device="cuda:0"), torch.zeros(n, device="cuda:0"))
    meters = [A.AverageMeter(1, 100, "cuda:0") for _ in range(3)]
    g = torch.Generator(device="cuda:0").manual_seed(2)
    for step in range(40):
        rew = torch.randn(n, device="cuda:0", generator=g)
        done = torch.rand(n, device="cuda:0", generator=g) < (0.02 if step < 20 else 0.3)
        tout = done & (torch.rand(n, device="cuda:0", generator=g) < 0.5)
        val = torch.randn(n, 1, device="cuda:0", generator=g)
        out = torch.empty(n, device="cuda:0")
        f.rollout_post(fus, rew, done, tout, val.reshape(-1), out)
        shaped = fus.rewards_shaper(rew.unsqueeze(1)) + fus.gamma * val * tout.unsqueeze(1).float()
        torch.testing.assert_close(out, shaped.reshape(-1))
        cr += rew.unsqueeze(1)
        cs += shaped
        cl += 1
        meters[0].update(cr, done)
        meters[1].update(cs, done)
        meters[2].update(cl.unsqueeze(1), done)
        nd = 1.0 - done.float()
        cr *= nd.unsqueeze(1)
        cs *= nd.unsqueeze(1)
        cl *= nd
        torch.testing.assert_close(fus.current_rewards, cr)
        torch.testing.assert_close(fus.current_shaped_rewards, cs, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(fus.current_lengths, cl)
        for m, mm in zip(meters, (fus.game_rewards, fus.game_shaped_rewards, fus.game_lengths)):
            torch.testing.assert_close(mm.mean.reshape(-1), m.mean.reshape(-1), rtol=1e-5, atol=1e-5)
            assert float(mm.current_size) == float(m.current_size)


def _dist_train_worker(rank, port, mode, tmp, q, num_envs=1024, iters=3):
    import socket  # noqa: F401

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0", ALLSTEPS_DIST_BACKEND="gloo", ALLSTEPS_DIST_TIMEOUT_S="900")
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
    import torch.distributed as dist

    import train

    try:
        runner, _ = train.main(["--task", "Allsteps-v0", "--num_envs", str(num_envs), "--max_iterations", str(iters),
                                "--seed", "7", "--distributed", "--multi_gpu_mode", mode, "--log_root", f"{tmp}/r{rank}"])
        ag = runner.agent
        # a numpy copy (pickled by value), not a shared-memory tensor whose descriptor dies with this process
        q.put((rank, ag.flat.params.detach().cpu().numpy().copy(), float(ag.lr), ag.frame, ag.dataset.minibatch_size,
               int(ag._uw.env_id_offset), bool(ag.fused is not None and ag._play_graphs is not None),
               ag.dataset.batch_size, (ag.horizon_length, ag.minibatch_size, ag.mini_epochs_num)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _two_ranks(tmp_path, mode, num_envs=1024, iters=3, timeout=200):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_train_worker, args=(r, port, mode, str(tmp_path), q, num_envs, iters))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=timeout) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["allreduce", "allgather"])
def test_distributed_fused_trainer_two_ranks_one_gpu(tmp_path, mode):
    """The --distributed train.py path with the fused HIP-graph update and rollout graphs, two ranks
    (gloo, both on cuda:0): the gradient / rollout exchange keeps the ranks' parameters identical,
    env shards are offset, frames count both ranks."""
    res = _two_ranks(tmp_path, mode)
    (_, p0, lr0, f0, mb0, off0, fused0, _, _), (_, p1, lr1, f1, mb1, off1, _, _, _) = res
    assert fused0, "the fused update / rollout graphs must be the path under test"
    assert np.array_equal(p0, p1), f"{mode}: ranks diverged"
    assert lr0 == lr1 and f0 == f1 == 3 * 2 * 1024 * 32
    assert (off0, off1) == (0, 1024)
    assert mb0 == (2 * 32768 if mode == "allgather" else 32768)


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_c4_per_rank_workload_two_ranks_allgather(tmp_path):
    """BASELINE C4's per-rank workload -- 32768 envs per rank, the reference agent config (horizon 32,
    minibatch 32768, 10 mini-epochs: rl_games_ppo_cfg.yaml:48,69-71) -- through train.py --distributed in
    the north star's allgather mode, two ranks on cuda:0 over gloo, 2 epochs: the ranks stay
    bit-identical, each rank's update runs on the gathered 2 x per-rank batch with a 2 x minibatch, the
    env shards are offset by 32768 and the frame count covers both ranks."""
    n = 32768
    res = _two_ranks(tmp_path, "allgather", num_envs=n, iters=2, timeout=800)
    (_, p0, lr0, f0, mb0, off0, fused0, bs0, cfg0), (_, p1, lr1, f1, mb1, off1, _, bs1, _) = res
    assert cfg0 == (32, 32768, 10), cfg0  # the reference agent config, unmodified
    assert fused0
    assert np.array_equal(p0, p1), "C4 allgather: ranks diverged"
    assert lr0 == lr1
    assert bs0 == bs1 == 2 * 32 * n  # the gathered batch: both ranks' rollouts
    assert mb0 == mb1 == 2 * 32768
    assert (off0, off1) == (0, n)
    assert f0 == f1 == 2 * 2 * n * 32  # epochs x ranks x envs x horizon


@pytest.mark.gpu
def test_training_is_deterministic(tmp_path):
    """Same seed, same config -> bit-identical parameters after 3 epochs (env Philox resets, Philox
    policy sampling, deterministic kernels and graph replays; cf. the reference's
    test_environment_determinism.py for the env)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts", "reinforcement_learning", "rl_games"))
    import train

    out = []
    for k in range(2):
        runner, _ = train.main(["--task", "Allsteps-v0", "--num_envs", "1024", "--max_iterations", "3", "--seed", "11",
                                "--log_root", str(tmp_path / f"run{k}")])
        out.append((runner.agent.flat.params.clone(), runner.agent._uw.get_state()))
    assert torch.equal(out[0][0], out[1][0])
    for key in ("q", "qd", "root_pos", "idx", "episode"):
        assert torch.equal(out[0][1][key], out[1][1][key]), key


@pytest.mark.gpu
@pytest.mark.parametrize("mp_dtype,tol", [("float16", 4e-3), ("bfloat16", 3.5e-2)])  # r06c measured: 9.4e-4 / 8.9e-3
def test_rollout_heads_lowp_bounded_and_equal_to_training_forward(tmp_path, mp_dtype, tol):
    """with mixed_precision the rollout policy runs the same 16-bit trunk AND heads as
    the training forward (16-bit layer-5 activations and head weights, fp32 accumulation, a 16-bit
    rounded output: autocast's Linear).  rl_games' play_steps runs its policy in fp32 (no autocast), so
    the rollout's mu / value deviate from the fp32 policy by the 16-bit rounding: bounded here against the
    fp32 torch forward of the same parameters (max error over 2048 rows relative to the largest entry;
    the measured figure is printed).  In exchange the rollout's mu equals the training forward's mu bit
    for bit (the same kernel, the same rounding points), so the PPO ratio of an unchanged policy is
    exactly 1 -- under rl_games' fp32 rollout / fp16 training it carries the 16-bit noise instead."""
    _, fus = _agents_and_batch(256, mixed=True, tmp=tmp_path, mp_dtype=mp_dtype)
    f = fus.fused
    n = f.mb  # one minibatch of rows: the training forward's minibatch 0 is the same rows
    f.init_rollout(n, seed=1)
    obs = fus.dataset.values_dict["obs"][:n].contiguous()
    out = {k: torch.empty(n, 21, device="cuda:0") for k in ("actions", "mus", "sigmas")}
    out["neglogpacs"] = torch.empty(n, device="cuda:0")
    out["values"] = torch.empty(n, 1, device="cuda:0")
    f.policy_act(obs, out)
    v_norm = f.head_r[:, 21:].clone()
    fus.model.eval()
    with torch.no_grad():
        ref = fus.model({"is_train": False, "prev_actions": None, "obs": obs})  # fp32 torch forward
        net = fus.model.a2c_network
        x = fus.model.norm_obs(obs)
        h = x
        for m in net.actor_mlp:
            h = m(h)
        v_ref = net.value(h)  # normalised value head (what the training loss reads)
    emu = ((out["mus"] - ref["mus"]).abs().max() / ref["mus"].abs().max()).item()
    ev = ((out["values"] - ref["values"]).abs().max() / ref["values"].abs().max()).item()
    evn = ((v_norm - v_ref).abs().max() / v_ref.abs().max()).item()
    print(f"{mp_dtype}: rollout vs fp32 policy, max rel. error mu {emu:.2e}, value {ev:.2e}, normalised value {evn:.2e}")
    assert emu < tol and ev < tol and evn < tol
    # the training forward on the same rows: the same mu and value bits
    f.begin_epoch()
    f.use_graphs = False
    f.fuse_norm = False
    f.step_a(False)
    torch.cuda.synchronize()
    assert torch.equal(f.head[:, :21], out["mus"])
    assert torch.equal(f.head[:, 21:], v_norm)


@pytest.mark.gpu
def test_loss_head_gradient_vs_fp32_autograd(tmp_path):
    """the loss block multiplies by a correctly rounded 1/sigma where torch divides by
    sigma, so d loss / d [mu | value] (the head gradient that seeds the whole backward) and the loss
    statistics are within a few ulp of torch autograd, not bit-equal.  Pinned here on the fp32 path
    (ppo_loss_grad's fp32 dhead) against autograd of rl_games' loss (actor_loss, critic_loss, bound_loss,
    entropy) through the same head values; the measured error is printed and the bound is ~4x it."""
    from allsteps_isaaclab_amd.learning import a2c_continuous as AC
    from allsteps_isaaclab_amd.learning.models import neglogp

    _, fus = _agents_and_batch(256, mixed=False, tmp=tmp_path)
    f = fus.fused
    f.use_graphs = False
    f.fuse_norm = False
    mb = {k: v.clone() for k, v in fus.dataset[0].items() if torch.is_tensor(v)}
    f.begin_epoch()
    f.step_a(False)
    torch.cuda.synchronize()
    head, dhead = f.head.clone(), f.dhead.clone()
    A, B = 21, head.shape[0]
    mu = head[:, :A].clone().requires_grad_(True)
    value = head[:, A:].clone().requires_grad_(True)
    logstd = fus.model.a2c_network.sigma.detach().clone()
    sigma = torch.exp(logstd).expand_as(mu)
    nlp = neglogp(mb["actions"], mu, sigma, logstd.expand_as(mu))
    ent = (0.5 + 0.5 * math.log(2 * math.pi) + torch.log(sigma)).sum(dim=-1)
    a_loss = AC.actor_loss(mb["old_logp_actions"], nlp, mb["advantages"], fus.ppo, fus.e_clip).mean()
    c_loss = AC.critic_loss(mb["old_values"], value, fus.e_clip, mb["returns"], fus.clip_value).mean()
    b_loss = AC.bound_loss(mu).mean() if fus.bound_loss_type == "bound" else torch.zeros((), device=mu.device)
    loss = (a_loss + 0.5 * c_loss * fus.critic_coef - ent.mean() * fus.entropy_coef
            + b_loss * float(fus.bounds_loss_coef or 0.0))
    loss.backward()
    ref = torch.cat([mu.grad, value.grad], dim=1)
    err = ((dhead - ref).abs().max() / ref.abs().max()).item()
    st = f.stats[0]
    e_a = abs(st[0].item() - a_loss.item()) / max(abs(a_loss.item()), 1e-12)
    e_c = abs(st[1].item() - c_loss.item()) / max(abs(c_loss.item()), 1e-12)
    print(f"dhead max rel. error {err:.2e} (B = {B}); a_loss {e_a:.2e}, c_loss {e_c:.2e}")
    assert err < 2.5e-6, err  # r06c measured 6.5e-7 (B = 2048)
    assert e_a < 2e-6 and e_c < 2e-6  # r06c measured 4.0e-7 / 0
