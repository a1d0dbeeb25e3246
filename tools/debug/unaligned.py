import bz2, sys, os
sys.path.insert(0, os.getcwd())
import torch, starch_amd
from tests import corpus, oracle_lib
data = corpus.multi_chrom_bed(4, 1500, seed=8, kind="bed6")
_, osegs = oracle_lib.transform(data)
c = starch_amd.Starch(0)
for off in (0, 1, 3, 16):
    buf = torch.zeros(len(data) + 64, dtype=torch.uint8)
    buf[off:off + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    dev = buf.to("cuda")
    c.compress_device(dev.data_ptr() + off, len(data))
    idx, streams = starch_amd.parse_archive(c.archive())
    print("off", off, "nseg", len(streams), len(osegs), [m["chromosome"] for m in idx["streams"]], [m["uncompressedLineCount"] for m in idx["streams"]], [s[1] for s in osegs])
    for k, (st, (ch, ln, t)) in enumerate(zip(streams, osegs)):
        got = bz2.decompress(st)
        if got != t:
            i = next((j for j in range(min(len(got), len(t))) if got[j] != t[j]), min(len(got), len(t)))
            print("  seg", k, "len", len(got), len(t), "first diff", i, got[max(0,i-40):i+40], t[max(0,i-40):i+40])
