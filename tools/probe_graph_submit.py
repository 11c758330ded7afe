import time, torch
x = torch.zeros(16, device="cuda")
for nk in (1, 5, 10, 25, 50):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3): x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(nk):
            x.add_(1.0)
    torch.cuda.synchronize()
    for _ in range(20): g.replay()
    torch.cuda.synchronize()
    # host time per replay, GPU idle between (sync each)
    tt = 0.0
    for _ in range(200):
        t = time.perf_counter(); g.replay(); tt += time.perf_counter() - t
        torch.cuda.synchronize()
    # back-to-back
    t0 = time.perf_counter()
    for _ in range(500): g.replay()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"{nk:3d} kernels: replay host {tt/200*1e6:7.1f} us (idle GPU), back-to-back host {th/500*1e6:7.1f} us, wall {tw/500*1e6:7.1f} us", flush=True)
