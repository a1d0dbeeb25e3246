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


def test_cli_file_whose_size_reads_zero():
    """A regular file whose st_size is 0 but which has content (/proc) is read
    to EOF, not taken as empty: same archive as its bytes piped in."""
    path = "/proc/version"
    data = open(path, "rb").read()
    assert os.stat(path).st_size == 0 and data
    got = _run("starch3", [path], b"")
    assert got == _run("starch3", [], data)
    assert len(got) > 4 + 32


def test_cli_reference_compat_is_magic_only():
    assert _run("starch3", ["--reference-compat"], corpus.cfg1_bed(500)) == b"\xca\x5c\xad\x1a"


@pytest.mark.parametrize("args", [[], ["--vdev", "2"], ["--vdev", "3"]])
def test_hpp_reference_compat_is_magic_only(args):
    """compress_in_stream under --reference-compat writes the magic alone on
    one device and on the multi-device batch path alike (the reference's
    stdout, hpp:765-769)."""
    data = corpus.multi_chrom_bed(5, 700, seed=12, kind="bed6")
    assert _run("starch3_hpp_example", ["--reference-compat"] + args, data) == b"\xca\x5c\xad\x1a"


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


@pytest.mark.parametrize("args", [["--hook"], ["--vdev", "2"], ["--vdev", "3"]])
def test_hpp_batches_of_chromosome_runs(args, monkeypatch):
    """transform_and_flush_in_stream and the multi-device compress_in_stream
    read the input in batches of whole chromosome runs (bounded memory): with
    64 KiB batches (many batches; runs longer than a batch held whole; stale
    sscanf values and revisited chromosomes across batch cuts; a 0xFF that
    ends the input) the archive is the CLI's byte for byte."""
    import starch_amd
    monkeypatch.setenv("STARCH_HPP_BATCH", str(64 << 10))
    runs = corpus.multi_chrom_bed(9, 900, seed=31, kind="bed6")
    stale = b"chrQ\t10\t20\nchrQ\t30\t45\n" + b"chrR\tq\tz\nchrR\t7\tw\n" * 40 + b"chrS\t5\t9\n"
    for data in (runs + stale + corpus.fuzz_bed(4, 400) + runs[:30000],
                 starch_amd.gen_bed(0, 60_000, chroms=[13, 14]) + b"chrZ\t1\t2\n\xffchrZ\t3\t4\n"):
        want = _run("starch3", [], data)
        got = _run("starch3_hpp_example", args, data)
        if got != want:
            wi, ws = starch_amd.parse_archive(want)
            gi, gs = starch_amd.parse_archive(got)
            assert [len(x) for x in gs] == [len(x) for x in ws]
            assert gs == ws
            for a, b in zip(gi["streams"], wi["streams"]):
                assert a == b
            assert gi == wi
        assert got == want


def test_hpp_hook_large_chromosomes():
    """Chromosomes whose text passes the bzlib ABI's 16 MiB direct-DMA
    threshold (the caller's buffer registered for the call) through the
    asynchronous process_tf_buffer hand-off: same archive as the CLI, and the
    synchronous hand-off (STARCH_HOOK_SYNC=1) too."""
    import starch_amd
    data = starch_amd.gen_bed(0, 100_000_000, chroms=[13, 14])   # ~19-21 MB of text each
    want = _run("starch3", [], data)
    assert _run("starch3_hpp_example", ["--hook"], data) == want
    env = dict(os.environ, STARCH_HOOK_SYNC="1")
    r = subprocess.run([os.path.join(BUILD, "starch3_hpp_example"), "--hook"], input=data, capture_output=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout == want
    # the text pool capped at nothing: every page-locked buffer is released
    # when its chromosome is done (no reuse), the archive is the same
    env = dict(os.environ, STARCH_HOOK_POOL_MAX="0")
    r = subprocess.run([os.path.join(BUILD, "starch3_hpp_example"), "--hook"], input=data, capture_output=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout == want


@pytest.mark.parametrize("args", [[], ["--hook"], ["--reference-compat"]])
def test_hpp_mapped_file_input(args, tmp_path):
    """stdin redirected from a regular file: compress_in_stream (one
    starch_encode_host_into over the mapping) and the hook's
    transform_and_flush_in_stream (runs planned over the mapping, batches
    DMA'd from it, tf_buffers from the page-locked pool) take the mapped
    paths (STARCH_HPP_MAP_MIN lowers their size floor); same bytes as the
    CLI, with and without a 0xFF that ends the input, as the unmapped paths
    (STARCH_HPP_MAP=0), and in 1 MiB batches (the hook's transform of batch
    k on its second context while batch k-1 is handed off)."""
    import starch_amd
    base = starch_amd.gen_bed(0, 400_000, chroms=[13, 14, 21]) + corpus.multi_chrom_bed(4, 500, seed=5, kind="bed6")
    for k, data in enumerate((base, base + b"chrZ\t1\t2\n\xffchrZ\t3\t4\n")):
        f = tmp_path / ("in%d.bed" % k)
        f.write_bytes(data)
        want = _run("starch3", ["--reference-compat"] if "--reference-compat" in args else [], data)
        for env_extra in ({"STARCH_HPP_MAP_MIN": "4096"}, {"STARCH_HPP_MAP": "0"},
                          {"STARCH_HPP_MAP_MIN": "4096", "STARCH_HPP_BATCH": str(1 << 20)}):
            env = dict(os.environ, **env_extra)
            with open(f, "rb") as fh:
                r = subprocess.run([os.path.join(BUILD, "starch3_hpp_example")] + args, stdin=fh,
                                   capture_output=True, timeout=300, env=env)
            assert r.returncode == 0, r.stderr[-2000:]
            assert r.stdout == want, (args, k, env_extra)


@pytest.mark.parametrize("pipe_reader", ["1", "0"])
def test_cli_pipe_larger_than_reader_pool(pipe_reader):
    """A pipe on stdin larger than the reader's buffer pool (8 x 32 MiB): the
    early-start reader thread (F_SETPIPE_SZ, pooled buffers fed to the
    session) and the plain read(2)-into-window loop (STARCH_CLI_PIPE=0) both
    give the one-call archive."""
    import starch_amd
    data = bytes(starch_amd.gen_bed(0, 14_000_000))
    assert len(data) > 300 << 20
    c = starch_amd.Starch(0)
    want = c.compress(data)
    c.close()
    env = dict(os.environ, STARCH_CLI_PIPE=pipe_reader)
    r = subprocess.run([os.path.join(BUILD, "starch3")], input=data, capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout == want
