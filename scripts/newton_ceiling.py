#!/usr/bin/env python3
"""Inputs for scripts/newton_ceiling.hip: the patch records of cfg4's first lens (3 072 patches, L2-resident) and of
cfg5's lens (301 056 patches, 80 MB) as raw [n][66] float32 files under gpurun_out/ (host code only, no GPU) -- only
the records whose plane faces the probe's +x rays (|n.x| >= 0.3), so every pass takes the Newton site's usual path
(a grazing plane would send the bracket quotients and normalisations down their full-range sequences).

usage: python scripts/newton_ceiling.py   -> prints "<file> <npatches>" per line
"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "cuda-bezier-triangle-raytracer_amd"), str(REPO)]

import numpy as np  # noqa: E402

import bzr_amd  # noqa: E402
from bzr_amd.configs import CONFIGS, build_lens  # noqa: E402

out = REPO / "gpurun_out"
out.mkdir(exist_ok=True)
for name in ("cfg4", "cfg5"):
    p = np.ascontiguousarray(build_lens(bzr_amd.TriMesh, CONFIGS[name].lenses[0]).bezier_patches(), dtype=np.float32)
    p = p[np.abs(p[:, 0]) >= 0.3]  # rec::kUnder: the plane normal's x
    f = out / f"nc_{name}.f32"
    p.tofile(f)
    print(f, p.shape[0], flush=True)
