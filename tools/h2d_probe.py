import torch, time
n = 2_380_051_469
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h.fill_(7)
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for rep in range(3):
    torch.cuda.synchronize(); t = time.perf_counter()
    d.copy_(h, non_blocking=True); torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print("1 stream: %.1f ms %.1f GB/s" % (dt * 1e3, n / dt / 1e9), flush=True)
ss = [torch.cuda.Stream() for _ in range(4)]
for k in (2, 4):
    for rep in range(2):
        torch.cuda.synchronize(); t = time.perf_counter()
        ch = (n + k - 1) // k
        for i in range(k):
            with torch.cuda.stream(ss[i]):
                d[i * ch:(i + 1) * ch].copy_(h[i * ch:(i + 1) * ch], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print("%d streams: %.1f ms %.1f GB/s" % (k, dt * 1e3, n / dt / 1e9), flush=True)
for rep in range(2):
    torch.cuda.synchronize(); t = time.perf_counter()
    h.copy_(d, non_blocking=True); torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print("D2H 1 stream: %.1f ms %.1f GB/s" % (dt * 1e3, n / dt / 1e9), flush=True)
