"""Loading of the committed golden fixtures (tests/golden/)."""
import base64
import json
import os

from tests import corpus

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def transform_cases():
    """-> [(name, input bytes, [(chr, lines, content-or-None, sha256-or-None, len-or-None)])]"""
    with open(os.path.join(GOLD, "transform_cases.json")) as f:
        j = json.load(f)
    out = []
    for c in j["cases"]:
        data = corpus.TRANSFORM_GENERATORS[c["gen"]]() if "gen" in c else base64.b64decode(c["input"])
        segs = []
        for s in c["segments"]:
            segs.append((base64.b64decode(s["chr"]), s["lines"],
                         base64.b64decode(s["content"]) if "content" in s else None,
                         s.get("sha256"), s.get("len")))
        out.append((c["name"], data, segs))
    return out


def bz2_cases(include_large=True):
    """-> [(name, input, bs, stream-or-None, sha256-or-None)]"""
    with open(os.path.join(GOLD, "bz2_cases.json")) as f:
        j = json.load(f)
    out = []
    for c in j["cases"]:
        if "gen" in c:
            if not include_large:
                continue
            gen, bs = corpus.LARGE_GENERATORS[c["gen"]]
            out.append((c["name"], gen(), c["bs"], None, c["sha256"]))
        else:
            out.append((c["name"], base64.b64decode(c["input"]), c["bs"], bytes.fromhex(c["stream"]), None))
    return out


def kat_files():
    """bzip2's own known-answer tests (bz:Makefile:55-70): (level, input, expected stream)."""
    import bz2 as _bz2
    out = []
    for k in (1, 2, 3):
        with open(os.path.join(GOLD, "kat", "sample%d.bz2" % k), "rb") as f:
            s = f.read()
        out.append((k, _bz2.decompress(s), s))
    return out
