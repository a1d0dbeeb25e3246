"""Host check of bz2_mtf.hip's byte-wide MTF value writer (Out8 + put_run):
the struct is compiled with g++ straight from the kernel source (device
qualifiers defined away) and fuzzed against a plain restatement of the
RUNA/RUNB coder (bz:compress.c:213-227) -- random chunk starts (every
alignment of the 16-byte window), empty chunks, long zero runs carried in,
bytes outside the chunk left untouched."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HDR = r'''
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define __device__
#define __forceinline__ inline
struct uint4 { uint32_t x, y, z, w; };
static uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return {a, b, c, d}; }
'''

MAIN = r'''
int main() {
  srand(1);
  for (int trial = 0; trial < 20000; ++trial) {
    const int n = rand() % 300;
    const uint32_t start = rand() % 64;
    const uint32_t z0 = (rand() % 4 == 0) ? rand() % 2000 : rand() % 5;
    std::vector<uint32_t> xs(n);
    for (auto& x : xs) { const int r = rand() % 10; x = r < 6 ? 0 : 1 + rand() % 30; }
    if (rand() % 50 == 0) for (auto& x : xs) x = 0;
    std::vector<int> ref(start + 5000, -1);
    uint32_t o = start, z = z0;
    for (auto x : xs) {
      if (!x) { ++z; continue; }
      while (z) { const uint32_t d = ((z - 1) & 1u) ? 1 : 0; ref[o++] = d; z = (z - (d + 1)) >> 1; }
      ref[o++] = x + 1;
      z = 0;
    }
    const uint32_t oend = o;
    std::vector<uint8_t> buf(start + 5000 + 32, 0xEE);
    bz::Out8 out;
    out.init(buf.data(), start);
    z = z0;
    for (auto x : xs) {
      if (!x) { ++z; continue; }
      bz::put_run(out, z);
      out.put(x + 1);
      z = 0;
    }
    out.flush();
    if (out.o != oend) { printf("length %u != %u (trial %d)\n", out.o, oend, trial); return 1; }
    for (uint32_t i = 0; i < buf.size(); ++i) {
      const int want = (i >= start && i < oend) ? ref[i] : 0xEE;
      if (buf[i] != want) { printf("byte %u: %d != %d (trial %d)\n", i, buf[i], want, trial); return 1; }
    }
  }
  printf("ok\n");
  return 0;
}
'''


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_out8_writer_matches_run_coder(tmp_path):
    src = open(os.path.join(ROOT, "starch_amd", "csrc", "bz2_mtf.hip")).read()
    a = src.index("struct Out8 {")
    b = src.index("// ---- alphabets <= 32: five launches")
    cpp = tmp_path / "out8.cpp"
    cpp.write_text(HDR + "namespace bz {\n" + src[a:b] + "}\n" + MAIN)
    exe = tmp_path / "out8"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(cpp)], check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == b"ok", r.stdout + r.stderr
