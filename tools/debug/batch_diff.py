"""Debug: which streams differ from the oracle, default batch vs STARCH_BWT_BATCH."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import starch_amd
from tests import oracle_lib
data = bytes(starch_amd.gen_bed(int(os.environ.get("KIND", "0")), int(os.environ.get("LINES", "600000"))))
c = starch_amd.Starch(0)
arch = c.compress(data)
st = c.stats()
c.close()
idx, streams = starch_amd.parse_archive(arch)
_, osegs = oracle_lib.transform(data)
bad = 0
for k, (s, (ch, n, text)) in enumerate(zip(streams, osegs)):
    ok = s == oracle_lib.bz2(text, 9)
    if not ok:
        bad += 1
        import bz2
        try:
            d = bz2.decompress(s)
            print("stream", k, ch, "differs; decompresses", d == text, len(s), len(oracle_lib.bz2(text, 9)))
        except Exception as e:
            print("stream", k, ch, "differs; decompress error", e)
print("batch", os.environ.get("STARCH_BWT_BATCH"), "streams", len(streams), "bad", bad, "blocks", st.get("n_blocks"))
