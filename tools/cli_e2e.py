#!/usr/bin/env python3
"""End-to-end CLI figure: the cfg2 input written to a file,
then `starch3 < file > archive` (streamed ingestion: reader thread, pinned
double buffer, encoder thread) and `starch3 --slurp file` (read all, one
call), each timed around the whole process (device open included), archives
compared byte for byte.  Prints one JSON line."""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import starch_amd
    kind = int(os.environ.get("KIND", "0"))
    lines = int(os.environ.get("LINES", "100000000"))
    tmp = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(tmp, "cli_e2e_input.bed")
    data = starch_amd.gen_bed(kind, lines)
    with open(path, "wb") as f:
        f.write(data)
    n = len(data)
    del data
    exe = os.path.join(ROOT, "starch_amd", "_build", "starch3")
    res = {"input_bytes": n, "kind": kind, "lines": lines}
    outs = {}
    for name, args in (("stream_stdin", [exe, "--stats"]), ("slurp_file", [exe, "--stats", "--slurp", path])):
        for rep in range(2):          # first run pages the binary + device in
            out = os.path.join(tmp, "cli_e2e_%s.starch" % name)
            t0 = time.perf_counter()
            with open(path, "rb") as fin, open(out, "wb") as fout:
                p = subprocess.run(args, stdin=fin if name == "stream_stdin" else subprocess.DEVNULL, stdout=fout,
                                   stderr=subprocess.PIPE, timeout=600)
            dt = time.perf_counter() - t0
            if p.returncode:
                raise SystemExit("%s failed: %s" % (name, p.stderr.decode()[-2000:]))
        st = json.loads(p.stderr.decode().strip().splitlines()[-1])
        outs[name] = hashlib.sha256(open(out, "rb").read()).hexdigest()
        res[name] = {"wall_s": round(dt, 3), "mb_s": round(n / dt / 1e6, 1), "stats": st}
        os.unlink(out)
    res["identical"] = outs["stream_stdin"] == outs["slurp_file"]
    os.unlink(path)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
