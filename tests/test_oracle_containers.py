"""The reference's preprocessing result depends on libstdc++ container iteration orders
(reference/mesh.cpp:224-239 iterates a std::unordered_set<uint32_t>; :292-307 sums over an
unordered_multimap equal_range).  The oracle (plain C) emulates them; this test compiles a tiny C++
program against the real containers of this toolchain and checks the emulation agrees."""
import ctypes
import subprocess

import numpy as np
import pytest

PROG = r"""
#include <cstdio>
#include <cstdint>
#include <unordered_map>
#include <unordered_set>
int main() {
  uint32_t n, k;
  while (std::scanf("%u", &n) == 1) {
    std::unordered_set<uint32_t> s;
    for (uint32_t i = 0; i < n; ++i) { std::scanf("%u", &k); s.insert(k); }
    for (auto x : s) std::printf("%u ", x);
    std::printf("\n");
  }
  std::unordered_multimap<int, int> m;   // equal_range order: newest first
  for (int i = 0; i < 40; ++i) m.emplace(i % 5, i);
  auto r = m.equal_range(2);
  for (auto it = r.first; it != r.second; ++it) std::printf("%d ", it->second);
  std::printf("\n");
}
"""


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    d = tmp_path_factory.mktemp("uset")
    src = d / "u.cpp"
    src.write_text(PROG)
    exe = d / "u"
    subprocess.run(["g++", "-O1", "-std=c++17", str(src), "-o", str(exe)], check=True)
    return exe


def test_unordered_set_iteration_order(orc, prog):
    rng = np.random.default_rng(0)
    cases = [list(range(10)), [100, 5, 37, 101, 12, 999, 3]]
    for size in (1, 5, 13, 14, 29, 30, 60, 200):
        cases.append(list(rng.integers(0, 5000, size)))
    cases.append([int(x) for x in rng.permutation(100000)[:300]])
    inp = "".join(f"{len(c)} " + " ".join(map(str, c)) + "\n" for c in cases)
    out = subprocess.run([str(prog)], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    for c, line in zip(cases, out):
        keys = np.asarray(c, np.uint32)
        res = np.zeros(len(keys), np.uint32)
        cnt = orc.lib().orc_debug_uset_order(keys.ctypes.data, len(keys), res.ctypes.data)
        assert list(res[:cnt]) == [int(x) for x in line.split()], c[:10]
    assert out[-1].split() == [str(i) for i in range(37, -1, -5)]  # 37 32 ... 2: newest first
