"""The C++ boundary on the CPU: (1) the reference's own CLI and engine
(/root/reference/src/starch3.cpp + include/starch3api.hpp) compile and link
against this repo's bzlib.h / libstarch_amd.so instead of the vendored
libbz2 (build and link only -- never run, and only where /root/reference
exists); (2) include/starch3_amd.hpp compiles as C++11 and its host-only
members behave like the reference's; (3) the starch3 CLI's exit-code contract
for everything decided before a device is opened (src/starch3.cpp:72-167,
include/starch3api.hpp:747-754, 777-779, 890-905)."""
import os
import subprocess
import tarfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "starch_amd", "_build")
REF = "/root/reference"
CLI = os.path.join(BUILD, "starch3")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference sources not present")
def test_reference_cli_links_against_gpu_bzlib(tmp_path):
    # jansson's headers come from the reference's own tarball (the engine includes jansson.h)
    with tarfile.open(os.path.join(REF, "third-party", "jansson-2.9.tar.gz")) as t:
        for m in ("jansson-2.9/src/jansson.h", "jansson-2.9/android/jansson_config.h"):
            t.extract(m, tmp_path)
    exe = tmp_path / "starch3_on_mi355x"
    cmd = ["g++", "-std=c++11", "-O1", "-w", "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(REF, "include"),
           "-I" + str(tmp_path / "jansson-2.9" / "src"), "-I" + str(tmp_path / "jansson-2.9" / "android"),
           os.path.join(REF, "src", "starch3.cpp"), "-L" + BUILD, "-lstarch_amd", "-lpthread",
           "-Wl,-rpath," + BUILD, "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    und = subprocess.run(["nm", "-D", "--undefined-only", str(exe)], capture_output=True, text=True).stdout
    for sym in ("BZ2_bzCompressInit", "BZ2_bzCompressEnd"):
        assert sym in und          # resolved from libstarch_amd.so, not a static libbz2
    needed = subprocess.run(["readelf", "-d", str(exe)], capture_output=True, text=True).stdout
    assert "libstarch_amd.so" in needed


def test_starch3_amd_hpp_compiles_cxx11(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include "starch3_amd.hpp"
#include <cassert>
int main() {
    starch3::Starch s;
    assert(s.get_note().empty());
    assert(s.get_compression_method() == starch3::Starch::k_compression_method_undefined);
    s.set_note("hello");
    assert(s.get_note() == "hello");
    s.set_compression_method(starch3::Starch::k_bzip2);
    assert(s.get_compression_method() == starch3::Starch::k_bzip2);
    const unsigned char* m = s.get_header_magic_bytes();
    assert(m[0] == 0xca && m[1] == 0x5c && m[2] == 0xad && m[3] == 0x1a);
    std::vector<unsigned char> out;
    int rc = s.compress("chr1\t1\t2\n", 10, &out);   // no MI355X here: a status, not a crash
    return rc == STARCH_OK ? 0 : (rc == STARCH_ERR_DEVICE ? 3 : 1);
}
''')
    exe = tmp_path / "t"
    r = subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), str(src),
                        "-L" + BUILD, "-lstarch_amd", "-Wl,-rpath," + BUILD, "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rc = subprocess.run([str(exe)], capture_output=True).returncode
    try:
        import torch
        gpu = torch.cuda.is_available()
    except Exception:
        gpu = False
    assert rc == (0 if gpu else 3)


def _cli(args, stdin=None, input_bytes=None):
    return subprocess.run([CLI] + args, input=input_bytes, stdin=stdin, capture_output=True, timeout=60)


def test_cli_missing_file_exits_61(tmp_path):
    r = _cli([str(tmp_path / "nope.bed")], input_bytes=b"")
    assert r.returncode == 61 and b"does not exist" in r.stderr and r.stdout == b""


def test_cli_two_methods_exits_1():
    r = _cli(["-b", "-g"], input_bytes=b"chr1\t1\t2\n")
    assert r.returncode == 1 and b"Only one compression method" in r.stderr


def test_cli_gzip_reference_compat_writes_magic_then_exits_38():
    """--reference-compat keeps the reference's gzip behaviour (hpp:765-769, 777-779)."""
    r = _cli(["-g", "--reference-compat"], input_bytes=b"chr1\t1\t2\n")
    assert r.returncode == 38 and r.stdout == b"\xca\x5c\xad\x1a"


def test_cli_tty_stdin_without_file_exits_61():
    import pty
    m, s = pty.openpty()
    try:
        r = _cli([], stdin=s)
    finally:
        os.close(m)
        os.close(s)
    assert r.returncode == 61 and b"No input is specified" in r.stderr


def test_cli_help_and_bad_level():
    assert _cli(["-h"]).returncode == 0
    assert b"Usage" in _cli(["--help"]).stdout
    assert _cli(["--level", "0"], input_bytes=b"").returncode == 22
