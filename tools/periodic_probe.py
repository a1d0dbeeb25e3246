"""Time single periodic 900 KB blocks (the test_gpu_periodic cases) with
STARCH_TRACE-free wall clocks, several repeats each, for a kernel-trace run:
  rocprofv3 --kernel-trace --stats -d gpurun_out/pprof -- python3 tools/periodic_probe.py p2 3
"""
import random
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import starch_amd  # noqa: E402

N = 899981


def periodic(unit):
    return unit * (N // len(unit))


def rand_unit(seed, p, alphabet):
    r = random.Random(seed)
    return bytes(r.choice(alphabet) for _ in range(p))


CASES = {
    "p2": lambda: periodic(b"0\n"),
    "p5_text": lambda: periodic(b"p1\n0\n"),
    "p997": lambda: periodic(rand_unit(1, 997, b"0123456789\n-p")),
    "p_half": lambda: periodic(rand_unit(3, N // 2, b"ACGTN")),
    "p_third": lambda: periodic(rand_unit(4, N // 3, b"ab")),
}

names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CASES)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
c = starch_amd.Starch(0)
c.bz2_compress(b"warm" * 1000, 9)
for nm in names:
    d = CASES[nm]()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        c.bz2_compress(d, 9)
        ts.append((time.perf_counter() - t0) * 1e3)
    st = c.stats()
    print("%s: %s ms  (blocks %s, periodic %s, rounds %s, tied %s, rle %s)" % (
        nm, " ".join("%.1f" % t for t in ts), st.get("n_blocks"), st.get("periodic_blocks"), st.get("bwt_rounds"),
        st.get("bwt_tied"), st.get("rle_bytes")), flush=True)
c.close()
