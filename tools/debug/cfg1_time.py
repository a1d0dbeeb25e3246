"""cfg1 (10k-line chr1 BED3): host bytes -> archive in host memory, and device-resident."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import starch_amd
from tests import corpus, oracle_lib
d = corpus.cfg1_bed(10000)
c = starch_amd.Starch(0)
a = c.compress(d)
ts = []
for _ in range(20):
    t0 = time.perf_counter(); c.compress(d); ts.append(time.perf_counter() - t0)
st = c.stats()
idx, streams = starch_amd.parse_archive(a)
_, segs = oracle_lib.transform(d)
ok = all(s == oracle_lib.bz2(t, 9) for s, (_, _, t) in zip(streams, segs))
print({"cfg1_bytes": len(d), "stream_bytes": len(streams[0]), "e2e_ms_best": round(min(ts) * 1e3, 3),
       "e2e_MBps": round(len(d) / min(ts) / 1e6, 1), "device_ms": round(st["ms_total"], 3) if "ms_total" in st else None,
       "bit_identical": ok})
