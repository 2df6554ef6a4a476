"""Per-kernel floor of a dependent kernel chain in a replayed graph (GPU): N tiny kernels (a one-
element add, one workgroup; and a 256-workgroup add over 256 K floats) captured in a torch CUDA graph,
replayed; prints the device time per kernel.  Sizes the launch overhead inside a one-image embed.
    python tools/graph_floor_probe.py"""
import json

import torch


def probe(n, numel):
    x = torch.zeros(numel, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                x.add_(1.0)
    ts = []
    for i in range(60):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        if i >= 10:
            ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2] / n, 3)


out = {f"us_per_kernel_n{n}_numel{m}": probe(n, m) for n in (10, 70) for m in (1, 1 << 18)}
print(json.dumps(out), flush=True)
