#!/usr/bin/env python3
"""tools/make_goldens.py -- regenerate tests/golden/ (TEST INFRASTRUCTURE).

Runs the REFERENCE itself, built from /root/reference by oracle/build_ref.sh
into oracle/_ref/, and records its outputs as small fixtures:

* transform goldens (tests/golden/transform_cases.json): for each input, the
  per-chromosome ``Chromosome/Lines/Content`` blocks that the reference binary
  prints from process_tf_buffer (hpp:393-407).  The binary is run under the
  zero-filling realloc shim (oracle/_ref/zrealloc.so) so the
  ``%s`` dump stops at tf_buffer_size, under ``timeout`` with retries because
  the reference can deadlock at EOF.
* bzip2 goldens (tests/golden/bz2_cases.json): streams produced by the
  reference's vendored, patched libbz2 1.0.6 (oracle/_ref/libbz2ref.so) for a
  corpus of small inputs (hex), including periodic blocks whose origPtr
  depends on fallbackSort's tie order, run-heavy inputs and
  multi-block inputs (sha256 + seeded generator for the large ones).
* the bzip2 known-answer files sample{1,2,3}.bz2 (data files the reference's
  vendored bzip2 tests hold, bz:Makefile:55-70) copied to tests/golden/kat/.

Usage: python tools/make_goldens.py   (needs /root/reference; CPU only)
"""
import base64
import ctypes
import hashlib
import json
import os
import random
import re
import subprocess
import sys
import tarfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests import corpus  # noqa: E402  (shared seeded generators)

REF = "/root/reference"
GOLD = os.path.join(ROOT, "tests", "golden")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "starch3")
SHIM = os.path.join(ROOT, "oracle", "_ref", "zrealloc.so")
LIBBZ2REF = os.path.join(ROOT, "oracle", "_ref", "libbz2ref.so")

SEG_RE = re.compile(rb"Chromosome \[(.*?)\]\nLines \[(\d+)\]\nContent \[(.*?)\]\n---", re.S)


def run_reference(data: bytes, tries: int = 12):
    env = dict(os.environ, LD_PRELOAD=SHIM)
    for _ in range(tries):
        try:
            p = subprocess.run([REF_BIN], input=data, capture_output=True, timeout=20, env=env)
        except subprocess.TimeoutExpired:
            continue                      # EOF deadlock: retry
        if p.returncode != 0:
            raise RuntimeError("reference exited %d" % p.returncode)
        segs = [{"chr": base64.b64encode(m.group(1)).decode(),
                 "lines": int(m.group(2)),
                 "content": base64.b64encode(m.group(3)).decode()}
                for m in SEG_RE.finditer(p.stderr)]
        return p.stdout, segs
    raise RuntimeError("reference hung %d times" % tries)


def transform_cases():
    cases = []
    for name, data in corpus.edge_cases():
        cases.append((name, data))
    for name, gen in corpus.TRANSFORM_GENERATORS.items():
        cases.append((name, gen()))
    for k in range(40):
        cases.append(("fuzz%02d" % k, corpus.fuzz_bed(seed=1000 + k, nlines=60)))
    return cases


def main():
    if not os.path.exists(REF_BIN):
        subprocess.check_call(["bash", os.path.join(ROOT, "oracle", "build_ref.sh")])
    os.makedirs(os.path.join(GOLD, "kat"), exist_ok=True)

    # ---- transform goldens from the reference binary ------------------------
    out = []
    for name, data in transform_cases():
        if not data:
            continue                      # empty input: reference may hang; covered by unit tests
        stdout, segs = run_reference(data)
        assert stdout == b"\xca\x5c\xad\x1a", (name, stdout[:8])
        if name in corpus.TRANSFORM_GENERATORS:   # large: regenerate input, pin text by sha256
            for sg in segs:
                txt = base64.b64decode(sg.pop("content"))
                sg["len"] = len(txt)
                sg["sha256"] = hashlib.sha256(txt).hexdigest()
            out.append({"name": name, "gen": name, "sha256_in": hashlib.sha256(data).hexdigest(),
                        "segments": segs})
        else:
            out.append({"name": name, "input": base64.b64encode(data).decode(), "segments": segs})
        print("transform", name, len(data), "bytes ->", len(segs), "segments", file=sys.stderr)
    with open(os.path.join(GOLD, "transform_cases.json"), "w") as f:
        json.dump({"source": "reference oracle/_ref/starch3 under zrealloc shim (tools/make_goldens.py)",
                   "cases": out}, f, indent=0)

    # ---- bzip2 goldens from the reference's vendored libbz2 ------------------
    lib = ctypes.CDLL(LIBBZ2REF)
    lib.ref_bz2_compress.restype = ctypes.c_int
    lib.ref_bz2_version.restype = ctypes.c_char_p

    def ref_bz2(data, bs=9):
        cap = len(data) + len(data) // 50 + 1024
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_size_t(0)
        rc = lib.ref_bz2_compress(data, ctypes.c_size_t(len(data)), bs, 30, buf, ctypes.c_size_t(cap),
                                  ctypes.byref(n))
        assert rc == 0, rc
        return buf.raw[:n.value]

    bz = []
    for name, data, bs in corpus.bz2_small_cases():
        s = ref_bz2(data, bs)
        bz.append({"name": name, "bs": bs, "input": base64.b64encode(data).decode(),
                   "stream": s.hex()})
    for name, gen, bs in corpus.bz2_large_cases():
        data = gen()
        s = ref_bz2(data, bs)
        bz.append({"name": name, "bs": bs, "gen": name, "n": len(data),
                   "sha256_in": hashlib.sha256(data).hexdigest(),
                   "sha256": hashlib.sha256(s).hexdigest(), "len": len(s)})
        print("bz2", name, len(data), "->", len(s), file=sys.stderr)
    with open(os.path.join(GOLD, "bz2_cases.json"), "w") as f:
        json.dump({"source": "reference vendored libbz2 %s via oracle/_ref/libbz2ref.so" %
                   lib.ref_bz2_version().decode(), "cases": bz}, f, indent=0)

    # ---- bzip2's own KAT files ---------------------------------------------
    with tarfile.open(os.path.join(REF, "third-party", "bzip2-1.0.6.tar.gz")) as t:
        for k in (1, 2, 3):
            m = t.getmember("bzip2-1.0.6/sample%d.bz2" % k)
            with open(os.path.join(GOLD, "kat", "sample%d.bz2" % k), "wb") as f:
                f.write(t.extractfile(m).read())


if __name__ == "__main__":
    main()
