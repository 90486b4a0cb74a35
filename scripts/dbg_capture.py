import torch
dev = "cuda:0"
mu = torch.zeros(16, 4, device=dev); sig = torch.ones(16, 4, device=dev)
for name, gen in (("default", None), ("custom", torch.Generator(device=dev).manual_seed(1))):
    try:
        torch.normal(mu, sig, generator=gen)
        g = torch.cuda.CUDAGraph()
        if gen is not None and hasattr(g, "register_generator_state"):
            g.register_generator_state(gen)
        with torch.cuda.graph(g):
            out = torch.normal(mu, sig, generator=gen)
        g.replay(); a = out.clone(); g.replay(); b = out.clone()
        print(name, "ok", bool((a != b).any()))
    except Exception as e:
        print(name, "FAIL", str(e)[:200])
try:
    g = torch.cuda.CUDAGraph()
    x = torch.randn(16, 59, device=dev)
    lin = torch.nn.Linear(59, 256).to(dev)
    with torch.no_grad():
        lin(x)
        with torch.cuda.graph(g):
            y = lin(x)
    print("linear ok")
except Exception as e:
    print("linear FAIL", str(e)[:200])
