"""Debug (GPU box): per-position chromosomes generated on the device, then
transformed (MODE=tf) or encoded (MODE=enc) on torch's current stream as
tests/test_gpu_fullsize.py does; prints the segments.
usage: MODE=enc tf_perpos.py CHROM_ID [CHROM_ID ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import starch_amd  # noqa: E402

ids = [int(a) for a in sys.argv[1:]] or [10]
mode = os.environ.get("MODE", "tf")
cap = max(starch_amd.gen_perpos_device(c) for c in ids)
dev = torch.empty(cap + 64, dtype=torch.uint8, device="cuda")
c = starch_amd.Starch(0)
stream = torch.cuda.current_stream()
if os.environ.get("SETSTREAM", "1") == "1":
    c.set_stream(stream.cuda_stream)
for ci in ids:
    n = starch_amd.gen_perpos_device(ci, dev.data_ptr(), cap + 64, stream=stream.cuda_stream)
    if mode == "enc":
        c.compress_device(dev.data_ptr(), n)
    else:
        c.transform_device(dev.data_ptr(), n)
    segs = c.segments()
    print("chrom %d n %d segments %d" % (ci, n, len(segs)), flush=True)
    for name, s in segs[:6]:
        print("  %s lines %d off %d text %d" % (name, s.line_count, s.stream_offset, s.text_bytes), flush=True)
c.close()
