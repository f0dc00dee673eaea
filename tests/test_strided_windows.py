"""The windowed strided walk of device.hpp (for_each_strided), run on the host: a lane visits exactly
the units tid, tid + nthreads, ... below n, in order, and each offset handed to a buffer descriptor is
(i - w0) * Unit < 2 GiB with w0 a window start shared by every lane -- across the 4 GiB boundary and
at ragged ends.  CPU only (hipcc builds a host program; no GPU call)."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SRC = r'''
#include <cstdio>
#include <cstdint>
#include "mscclpp_amd/device.hpp"
using namespace mscclpp_amd;
template <uint32_t Unit>
static int check(uint64_t n, uint64_t nthreads, uint64_t tid) {
  uint64_t expect = tid, visits = 0;
  int bad = 0;
  const uint64_t win = (1ull << 31) / Unit;
  const bool single = n * Unit <= 0xFFFFFFFFull;
  for_each_strided<Unit>(n, tid, nthreads, [&](uint64_t i, uint64_t w0, uint32_t off) {
    if (i != expect) ++bad;                                   // every unit of this lane, in order
    if ((uint64_t)off != (i - w0) * Unit) ++bad;              // the offset is relative to w0
    if (single ? w0 != 0 : (w0 % win != 0 || i < w0 || i - w0 >= win)) ++bad;  // a shared window start
    expect = i + nthreads;
    ++visits;
  });
  const uint64_t want = tid < n ? (n - tid + nthreads - 1) / nthreads : 0;
  if (visits != want) ++bad;
  return bad;
}
int main() {
  int bad = 0;
  const uint64_t G = 1ull << 30;
  // 16-byte units: 4 GiB + 80 bytes, a grid of 2^26 lanes (4-5 visits each), lanes at both ends
  for (uint64_t tid : {0ull, 1ull, 5ull, (1ull << 26) - 1}) bad += check<16>((4 * G + 80) / 16, 1ull << 26, tid);
  // 4-byte units over 9 GiB with a grid that does not divide the window (odd stride)
  for (uint64_t tid : {0ull, 7ull, 999999ull}) bad += check<4>(9 * G / 4 + 3, 1000003, tid);
  // 8-byte units just under and just over the single-window limit
  for (uint64_t tid : {0ull, 3ull}) bad += check<8>((4 * G - 8) / 8, 1ull << 24, tid);
  for (uint64_t tid : {0ull, 3ull}) bad += check<8>((4 * G + 8) / 8, 1ull << 24, tid);
  // a lane beyond n visits nothing
  bad += check<16>(10, 64, 20);
  std::printf("bad %d\n", bad);
  return bad != 0;
}
'''


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
def test_for_each_strided_windows():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "w.hip"), os.path.join(d, "w")
        open(src, "w").write(SRC)
        r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                            src, "-o", exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-3000:]
        r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120)
        assert r.returncode == 0 and "bad 0" in r.stdout, r.stdout[-2000:]
