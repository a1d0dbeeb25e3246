"""Time the gzip method on cfg2 (device-resident input), report ratio."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import starch_amd
n = sum(starch_amd.gen_bed_sizes(0, 100_000_000))
host = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
starch_amd.gen_bed(0, 100_000_000, into=ctypes.c_void_p(host.data_ptr()))
dev = host.to("cuda")
for m in (starch_amd.K_BZIP2, starch_amd.K_GZIP):
    c = starch_amd.Starch(0)
    c.set_compression_method(m)
    c.compress_device(dev.data_ptr(), n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        c.compress_device(dev.data_ptr(), n)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    st = c.stats()
    print("method", m, "ms %.1f" % (dt * 1e3), "MB/s %.0f" % (n / dt / 1e6), "text", st["text_bytes"],
          "archive", c.archive_size() if hasattr(c, "archive_size") else "?", flush=True)
    c.close()
