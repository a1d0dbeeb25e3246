"""The starch3 CLI and the C++ class surface on the MI355X: stdout is the
archive Starch.compress produces (cfg1, stdin and file input), the
--reference-compat output is exactly the reference's stdout (the 4 magic
bytes, hpp:765-769), and the reference-shaped main() over
include/starch3_amd.hpp -- both the whole-path call and the per-chromosome
process_tf_buffer hook -- writes the same bytes."""
import os
import subprocess

import pytest

from tests import corpus, oracle_lib

pytestmark = pytest.mark.gpu

BUILD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "starch_amd", "_build")


def _run(exe, args, data):
    r = subprocess.run([os.path.join(BUILD, exe)] + args, input=data, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_cli_stdout_is_the_archive_cfg1(tmp_path):
    import starch_amd
    data = corpus.cfg1_bed(10000)
    c = starch_amd.Starch(0)
    want = c.compress(data)
    c.close()
    assert _run("starch3", [], data) == want
    f = tmp_path / "cfg1.bed"
    f.write_bytes(data)
    assert _run("starch3", [str(f)], b"") == want
    idx, streams = starch_amd.parse_archive(want)
    _, segs = oracle_lib.transform(data)
    assert streams[0] == oracle_lib.bz2(segs[0][2], 9)


def test_cli_reference_compat_is_magic_only():
    assert _run("starch3", ["--reference-compat"], corpus.cfg1_bed(500)) == b"\xca\x5c\xad\x1a"


def test_cli_note_and_level():
    import starch_amd
    data = corpus.multi_chrom_bed(3, 300, seed=4)
    out = _run("starch3", ["--note=run 7", "--level", "3"], data)
    idx, streams = starch_amd.parse_archive(out)
    assert idx["archive"]["note"] == "run 7" and idx["archive"]["blockSize100k"] == 3
    _, segs = oracle_lib.transform(data)
    assert [s for s in streams] == [oracle_lib.bz2(t, 3) for _, _, t in segs]


@pytest.mark.parametrize("hook", [False, True])
def test_hpp_main_matches_cli(hook):
    data = corpus.multi_chrom_bed(5, 700, seed=12, kind="bed6") + corpus.fuzz_bed(2, 300)
    want = _run("starch3", [], data)
    got = _run("starch3_hpp_example", ["--hook"] if hook else [], data)
    assert got == want
