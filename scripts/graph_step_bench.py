"""Eager env.step loop vs HIP-graph replay of G steps (graph-safe counters) at N envs."""
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402

from allsteps_isaaclab_amd import registry  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K, G = 1000, 10
res = {}
for mode in ("eager", "graph"):
    cfg = registry.load_cfg_from_registry("Allsteps-v0", "env_cfg_entry_point")
    cfg.scene.num_envs = N
    env = registry.make("Allsteps-v0", cfg=cfg)
    env.set_graph_capture(mode == "graph")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(1)
    acts = torch.rand(K + 50, N, 21, device="cuda:0", generator=g) * 2 - 1
    if mode == "eager":
        for t in range(50):
            env.step(acts[K + t])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(K):
            env.step(acts[t])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    else:
        static = torch.zeros(G, N, 21, device="cuda:0")
        for t in range(G):
            env.step(static[t])
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for t in range(G):
                env.step(static[t])
        for t in range(5):
            static.copy_(acts[K + G * t:K + G * (t + 1)])
            graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(K // G):
            static.copy_(acts[G * t:G * (t + 1)])
            graph.replay()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    res[mode] = {"ms_per_step": round(el / K * 1e3, 4), "env_steps_per_s": round(N * K / el)}
    env.close()
print(json.dumps(res))
