"""Build-variant libraries (cuda-bezier-triangle-raytracer_amd/Makefile `variants`, built by build()).

stack4: libbzr with a 4-entry traversal stack (-DBZR_STACK=4).  Lanes whose walk runs out of stack
mid-walk switch to the reference's in-order full scan (reference/bezierMesh.cpp:206-227) while keeping
what the walk already found -- duplicates must collapse under the (t, scanned index) key and parked /
joined retry state must stay valid across the switch.  The default 64-entry stack never overflows on the
bench configs, so only this build exercises that path: fused == staged == brute force (and == the oracle
on cfg2), bit for bit, with the device counters reporting overflow rays.

dense1 / dense64: libbzr with the staged pair layout's two extremes (-DBZR_DENSE_MIN=1: every bucket's last
partial chunk padded, no sparse region; =64: no padding, every remainder in the sparse region): staged ==
brute force (== the oracle on cfg2 and the cfg4 chain) through only the dense or mostly the sparse kernel.

rpl2 / rpl4: libbzr whose fused kernel is k_trace_r (trace_pool.inc): 2 or 4 rays per lane, the Newton passes
pooled over a wave's 128 / 256 rays (-DBZR_TRACE_RPL); the same checks plus cfg4's two-lens chain and origins
beyond s_max (the in-order scan inside the pooled kernel), fused == brute force == the oracle.

tracebundle / traceperlane: libbzr with k_trace's wave-bundle walk one tree level per batch (-DBZR_TRACE_WIDE=0;
the default takes two) and with k_trace's per-lane walk (-DBZR_TRACE_BUNDLE=0, round 3's default): the same
checks, fused == staged == brute force (== the oracle on cfg2), including the incoherent cfg5 rays whose wide
bundles take the per-lane node tests.

The variant runs in a child process (BZR_LIBRARY selects the library; one process = one libbzr).
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "cuda-bezier-triangle-raytracer_amd"

WORKER = r"""
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import bzr_amd as bzr
from bzr_amd.configs import CONFIGS, build_lens, grid_rays, pixel_coords, rays_for
from oracle import pyoracle as orc

def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)

ctx = bzr.Context(0)
out = {}
# cfg2: one lens, the refraction chain, 256^2 primaries (oracle too)
lens = build_lens(bzr.TriMesh, CONFIGS["cfg2"].lenses[0]).bezier_patches()
dm = bzr.DeviceMesh(ctx, lens)
rays = grid_rays(CONFIGS["cfg2"], side=256)
want = orc.trace_chain([lens], [1.3], rays)
for name, mode in (("fused", bzr.PIPELINE_FUSED), ("staged", bzr.PIPELINE_STAGED), ("brute", bzr.ACCEL_NONE)):
    ctx.counters(True); ctx.counters_report()
    got = bzr.trace_chain(ctx, [dm], [1.3], rays, mode=mode)
    c = ctx.counters_report(); ctx.counters(False)
    out[f"cfg2_{name}_equal"] = all(np.array_equal(bits(g), bits(w)) for g, w in zip(got, want))
    out[f"cfg2_{name}_overflow_rays"] = c["overflow_rays"]
# cfg5: 301 056 patches, BezierMesh::intersect on 65 536 grid rays from the lens's middle rows
cfg = CONFIGS["cfg5"]
p5 = build_lens(bzr.TriMesh, cfg.lenses[0]).bezier_patches()
dm5 = bzr.DeviceMesh(ctx, p5)
r, c = pixel_coords(cfg, side=8192, order="tiles")
mid = len(r) // 2
rays5 = rays_for(cfg, r[mid:mid + 65536], c[mid:mid + 65536], side=8192)
# plus incoherent rays from all around the lens (deep, diverging walks: the ones that overflow a tiny stack)
rng = np.random.default_rng(41)
o = rng.uniform(-12, 12, (16384, 3)) + np.array([10.0, 0.0, 0.0])
tgt = np.array([10.0, 0.0, 0.0]) + rng.uniform(-1, 1, (16384, 3)) * np.array([1.0, 4.0, 2.0])
dd = (tgt - o) / np.linalg.norm(tgt - o, axis=1, keepdims=True)
rays5 = np.concatenate([rays5, np.concatenate([o.T, dd.T]).astype(np.float32)], axis=1)
ref = bits(bzr.intersect(ctx, dm5, rays5, mode=bzr.ACCEL_NONE))
out["cfg5_hits"] = int((ref[11] == 4).sum())
for name, mode in (("fused", bzr.PIPELINE_FUSED), ("staged", bzr.PIPELINE_STAGED)):
    ctx.counters(True); ctx.counters_report()
    got = bits(bzr.intersect(ctx, dm5, rays5, mode=mode))
    cnt = ctx.counters_report(); ctx.counters(False)
    out[f"cfg5_{name}_equal"] = bool(np.array_equal(got, ref))
    out[f"cfg5_{name}_overflow_rays"] = cnt["overflow_rays"]
    out[f"cfg5_{name}_lane_chunks"] = cnt["lane_chunks"]
    out[f"cfg5_{name}_pairs"] = cnt["pairs"]
if "--more" in sys.argv:
    # cfg4: two lenses, the chain, 256^2 primaries: fused == brute force == the oracle
    l4 = [build_lens(bzr.TriMesh, l).bezier_patches() for l in CONFIGS["cfg4"].lenses]
    d4 = [bzr.DeviceMesh(ctx, p) for p in l4]
    r4 = grid_rays(CONFIGS["cfg4"], side=256)
    w4 = orc.trace_chain(l4, [1.3, 1.3], r4)
    for name, mode in (("fused", bzr.PIPELINE_FUSED), ("staged", bzr.PIPELINE_STAGED), ("brute", bzr.ACCEL_NONE)):
        g4 = bzr.trace_chain(ctx, d4, [1.3, 1.3], r4, mode=mode)
        out[f"cfg4_{name}_equal"] = all(np.array_equal(bits(g), bits(w)) for g, w in zip(g4, w4))
    # origins beyond s_max mixed into the waves (the in-order scan): robot.stl, 25 % far
    lr = build_lens(bzr.TriMesh, CONFIGS["cfg3"].lenses[0].__class__("stl", split=1)).bezier_patches()
    dr = bzr.DeviceMesh(ctx, lr)
    rng = np.random.default_rng(11)
    o = rng.uniform(-30, 30, (3, 4096)).astype(np.float32)
    far = rng.random(4096) < 0.25
    o[0, far] = np.float32(-5e4)
    t = rng.uniform(-20, 20, (3, 4096)).astype(np.float32)
    dd = t - o
    dd /= np.sqrt((dd * dd).sum(axis=0, keepdims=True)).astype(np.float32)
    rr = np.concatenate([o, dd.astype(np.float32)]).astype(np.float32)
    ctx.counters(True); ctx.counters_report()
    gf = bits(bzr.intersect(ctx, dr, rr, mode=bzr.PIPELINE_FUSED))
    cnt = ctx.counters_report(); ctx.counters(False)
    out["far_fused_equal"] = bool(np.array_equal(gf, bits(orc.intersect(lr, rr))))
    out["far_overflow_rays"] = cnt["overflow_rays"]
    out["far_count"] = int(far.sum())
print(json.dumps(out))
"""


@pytest.mark.gpu
def test_tiny_stack_overflow_path_is_exact():
    lib = PKG / "lib" / "stack4" / "libbzr.so"
    if not lib.exists():
        pytest.fail(f"{lib} missing: build() makes the `variants` target")
    env = dict(os.environ, BZR_LIBRARY=str(lib))
    res = subprocess.run([sys.executable, "-c", WORKER, str(PKG), str(REPO)], env=env, capture_output=True,
                         text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    for k, v in out.items():
        if k.endswith("_equal"):
            assert v, (k, out)
    # the tiny stack really overflowed on both pipelines (the brute-force scan has no stack)
    for k in ("cfg2_fused", "cfg2_staged", "cfg5_fused", "cfg5_staged"):
        assert out[f"{k}_overflow_rays"] > 0, (k, out)
    assert out["cfg5_hits"] > 10000


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["tracebundle", "traceperlane"])
def test_trace_bundle_walk_is_exact(variant):
    """k_trace's other walks (one level per batch; per lane): exact, and only the far origins take the in-order
    scan (round 3's 4096-of-1026 count came from a pre-release bundle walk whose full-stack batches sent whole
    incoherent waves to the scan; the released one tests wide bundles per lane --
    profiles/r04_bundle_overflow_probe.jsonl)."""
    lib = PKG / "lib" / variant / "libbzr.so"
    if not lib.exists():
        pytest.fail(f"{lib} missing: build() makes the `variants` target")
    env = dict(os.environ, BZR_LIBRARY=str(lib))
    res = subprocess.run([sys.executable, "-c", WORKER, str(PKG), str(REPO), "--more"], env=env, capture_output=True,
                         text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    for k, v in out.items():
        if k.endswith("_equal"):
            assert v, (k, out)
    assert out["far_overflow_rays"] == out["far_count"]
    assert out["cfg2_fused_overflow_rays"] == 0
    assert out["cfg5_hits"] > 10000


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["rpl2", "rpl4"])
def test_pooled_passes_are_exact(variant):
    """k_trace_r (2 / 4 rays per lane, Newton passes pooled over the wave's rays): bit-identical to the
    brute-force scan and the oracle on cfg2 / cfg4 chains, cfg5 intersect and far origins."""
    lib = PKG / "lib" / variant / "libbzr.so"
    if not lib.exists():
        pytest.fail(f"{lib} missing: build() makes the `variants` target")
    env = dict(os.environ, BZR_LIBRARY=str(lib))
    res = subprocess.run([sys.executable, "-c", WORKER, str(PKG), str(REPO), "--more"], env=env,
                         capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    for k, v in out.items():
        if k.endswith("_equal"):
            assert v, (k, out)
    assert out["cfg2_fused_overflow_rays"] == 0 and out["cfg5_fused_overflow_rays"] == 0
    assert out["far_overflow_rays"] == out["far_count"]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["dense1", "dense64"])
def test_staged_pair_layout_extremes_are_exact(variant):
    """The staged path with every remainder padded (dense1) or none (dense64): bit-identical to the brute-force
    scan and the oracle; dense1 runs no sparse chunk, dense64 runs every bucket remainder per lane."""
    lib = PKG / "lib" / variant / "libbzr.so"
    if not lib.exists():
        pytest.fail(f"{lib} missing: build() makes the `variants` target")
    env = dict(os.environ, BZR_LIBRARY=str(lib))
    res = subprocess.run([sys.executable, "-c", WORKER, str(PKG), str(REPO), "--more"], env=env,
                         capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    for k, v in out.items():
        if k.endswith("_equal"):
            assert v, (k, out)
    if variant == "dense1":
        assert out["cfg5_staged_lane_chunks"] == 0, out
    else:
        assert out["cfg5_staged_lane_chunks"] > 0, out
