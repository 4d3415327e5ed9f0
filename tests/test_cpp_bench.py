"""The C++ host path's frame bench (tests/cpp/tiled_bench.cpp): it builds against the
drop-in headers and libbzr on CPU; on a GPU box a short run through bzr::TiledChain (one device: the DIRECT
plan) must reproduce the committed oracle digests of the whole cfg4 4096^2 frame, tile for tile, so the
frames the C++ bench times are the bit-exact ones."""
import importlib.util
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

from conftest import PKG, REPO

GOLDEN = Path(__file__).resolve().parent / "golden"


def build(out: Path) -> Path:
    exe = out / "tiled_bench"
    cmd = ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__",
           str(REPO / "tests" / "cpp" / "tiled_bench.cpp"),
           f"-I{REPO / 'include' / 'bzr'}", f"-I{REPO / 'include'}", "-I/opt/rocm/include",
           f"-L{PKG / 'lib'}", "-lbzr", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{PKG / 'lib'}", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_cpp_bench_builds(built, tmp_path):
    assert build(tmp_path).exists()


@pytest.mark.gpu
def test_cpp_bench_frame_matches_oracle_digests(built, tmp_path):
    exe = build(tmp_path)
    dump = tmp_path / "frame.bin"
    r = subprocess.run([str(exe), "--frames", "3", "--warmup", "1", "--prewarm-s", "0", "--dump", str(dump)],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ))
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["transport"] == "direct" and line["segments_per_frame"] == 49913901
    raw = dump.read_bytes()
    side, n = np.frombuffer(raw[:16], np.uint64)
    assert side == 4096 and n == 4096 * 4096
    body = np.frombuffer(raw[16:], np.uint32)
    rays, status, seg = body[:6 * n].reshape(6, n), body[6 * n:7 * n], body[7 * n:]
    spec = importlib.util.spec_from_file_location("tile_digest", GOLDEN / "tile_digest.py")
    td = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(td)
    want = np.load(GOLDEN / "d_cfg4_4096.npz")
    assert np.array_equal(want["tiles"], np.arange(4096))
    got = td.chain_digests(rays, status, seg)
    bad = np.flatnonzero((got != want["digests"]).any(axis=1))
    assert bad.size == 0, f"{bad.size} of 4096 tiles differ from the oracle digests, first {bad[:8]}"
