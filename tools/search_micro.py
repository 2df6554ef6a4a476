import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib, time, torch, json
M = importlib.import_module('end-to-end-image-retrieval-service-with-k8s-jenkins_amd.index')
for dtype, n in (("float32", 1_000_000), ("float16", 1_000_000), ("float16", 20_000_000)):
    d = M.DeviceIndex(512, dtype=dtype, capacity=n)
    d.fill_random(2, 0, n)
    q = torch.randn(1, 512, device='cuda')
    for _ in range(3): d.search(q, 10, n)
    torch.cuda.synchronize()
    d.timing(True)
    t = time.perf_counter()
    for _ in range(50): d.search(q, 10, n)
    torch.cuda.synchronize(); el = time.perf_counter() - t
    ms, cnt, b = d.timing_read()
    print(json.dumps({"dtype": dtype, "n": n, "wall_ms": el / 50 * 1e3, "scan_ms": ms / cnt, "scan_GBps": b / (ms / 1e3) / 1e9}))
    d.close()
