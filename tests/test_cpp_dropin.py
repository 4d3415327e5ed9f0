"""Build a reference-style C++ caller against the drop-in headers (include/bzr/*.h) and run it:
on CPU the googleTest L1 cases + preprocessing; on a GPU box also the hot-path calls vs the oracle."""
import subprocess

import pytest

from conftest import PKG, REPO


def build(tmp_path):
    exe = tmp_path / "dropin_test"
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", str(REPO / "tests" / "cpp" / "dropin_test.cpp"),
           f"-I{REPO / 'include' / 'bzr'}", f"-I{REPO / 'include'}", f"-I{REPO / 'oracle'}",
           f"-L{PKG / 'lib'}", "-lbzr", f"-L{REPO / 'oracle'}", "-loracle",
           f"-Wl,-rpath,{PKG / 'lib'}", f"-Wl,-rpath,{REPO / 'oracle'}", "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_dropin_cpu_parts(built, tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


@pytest.mark.gpu
def test_dropin_with_gpu(built, tmp_path):
    exe = build(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hot path:" in r.stdout and "0 failed" in r.stdout
