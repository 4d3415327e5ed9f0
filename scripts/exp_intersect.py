"""Experiment helper: per-kernel timing of one BezierMesh::intersect stage over the cfg2 ray grid
(fixed workload, so kernel variants can be compared without changing downstream stages)."""
import os, sys, json
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cuda-bezier-triangle-raytracer_amd")]
import torch
import bzr_amd
from bzr_amd.configs import CONFIGS, build_lens, grid_rays
cfg = CONFIGS["cfg2"]
patches = build_lens(bzr_amd.TriMesh, cfg.lenses[0]).bezier_patches()
ctx = bzr_amd.Context(0)
mesh = bzr_amd.DeviceMesh(ctx, patches)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
ctx.use_torch_stream(stream)
rays = torch.from_numpy(grid_rays(cfg)).cuda()
hits = torch.empty((13, rays.shape[1]), dtype=torch.float32, device="cuda")
for _ in range(3):
    bzr_amd.intersect(ctx, mesh, rays, hits)
torch.cuda.synchronize()
ctx.timing(True); ctx.timing_report()
for _ in range(20):
    bzr_amd.intersect(ctx, mesh, rays, hits)
rep = ctx.timing_report()
print(json.dumps({k: round(ms / c, 4) for k, (ms, c) in rep.items()}))
