#!/usr/bin/env python3
"""Streamed-ingestion figures (dev tool; GPU box): the cfg2
input in pinned host memory, then
  api_feed     starch_stream_feed in PIECE-byte pieces (the library copies
               each piece into its pinned window)
  cli_file     starch3 < file > archive (read(2) straight into the window)
  cli_pipe     cat file | starch3 > archive (the same through a pipe)
each timed around the whole call / process; every archive is compared with
the one-call archive.  STARCH_TRACE=1 in the environment prints the
session timeline of the api_feed run on stderr.  Prints one JSON line."""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import starch_amd
    kind = int(os.environ.get("KIND", "0"))
    lines = int(os.environ.get("LINES", "100000000"))
    piece = int(os.environ.get("PIECE", str(64 << 20)))
    batch = int(os.environ.get("BATCH", "0"))
    n = sum(starch_amd.gen_bed_sizes(kind, lines))
    host = torch.empty(n + 64, dtype=torch.uint8, pin_memory=True)
    starch_amd.gen_bed(kind, lines, into=ctypes.c_void_p(host.data_ptr()))
    c = starch_amd.Starch(0)
    c.compress_host_ptr(host.data_ptr(), n)
    want = hashlib.sha256(c.archive()).hexdigest()
    res = {"input_bytes": n, "piece": piece, "batch": batch or (256 << 20)}

    cap = len(c.archive()) + (1 << 20)
    outb = torch.empty(cap, dtype=torch.uint8, pin_memory=True)

    def api_feed():
        # archive bytes drained straight into one pinned buffer (no Python copies)
        c.stream_begin(batch)
        o = c.stream_read(into=outb.data_ptr(), cap=cap)
        for off in range(0, n, piece):
            c.stream_feed(host.data_ptr() + off, min(piece, n - off))
            o += c.stream_read(into=outb.data_ptr() + o, cap=cap - o)
        c.stream_end()
        o += c.stream_read(into=outb.data_ptr() + o, cap=cap - o)
        return o

    api_feed()                                   # pins the session buffers once
    ts = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        t0 = time.perf_counter()
        got = api_feed()
        ts.append(time.perf_counter() - t0)
    same = hashlib.sha256(outb[:got].numpy().tobytes()).hexdigest() == want
    ts.sort()
    dt = ts[len(ts) // 2]
    res["api_feed"] = {"s_median": round(dt, 4), "mb_s": round(n / dt / 1e6, 1), "s_all": [round(x, 4) for x in ts],
                       "identical": same}
    c.close()

    tmp = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(tmp, "stream_bench_input.bed")
    with open(path, "wb") as f:
        f.write(host[:n].numpy().tobytes())
    exe = os.path.join(ROOT, "starch_amd", "_build", "starch3")
    extra = ["--batch-mb", str(batch >> 20)] if batch else []
    for name, cmd in (("cli_file", "%s --stats %s < %s" % (exe, " ".join(extra), path)),
                      ("cli_pipe", "cat %s | %s --stats %s" % (path, exe, " ".join(extra)))):
        out = os.path.join(tmp, "stream_bench_%s.starch" % name)
        for rep in range(2):                     # the first run pages the binary and the device in
            t0 = time.perf_counter()
            p = subprocess.run("%s > %s" % (cmd, out), shell=True, stderr=subprocess.PIPE, timeout=300)
            dt = time.perf_counter() - t0
            if p.returncode:
                raise SystemExit("%s failed: %s" % (name, p.stderr.decode()[-2000:]))
        with open(out, "rb") as f:
            got = hashlib.sha256(f.read()).hexdigest()
        os.unlink(out)
        res[name] = {"s": round(dt, 4), "mb_s": round(n / dt / 1e6, 1), "identical": got == want,
                     "stats": json.loads(p.stderr.decode().strip().splitlines()[-1])}
    os.unlink(path)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
