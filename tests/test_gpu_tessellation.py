"""Device tessellation: BezierMesh::interpolate (reference/bezierMesh.cpp:55-66) as a HIP kernel.

The reference tessellates every lens with interpolate(5) for its STL dumps (reference/test.cpp:265,
299, 372).  The GPU result must equal, bit for bit, the host product path (TriMesh.bezier_interpolate)
and the oracle's restatement (oracle/bzr_oracle.c orc_bezier_interpolate_mesh) of the same mesh,
and the STL written from it must equal the host path's STL byte for byte.
"""
import numpy as np
import pytest

from bzr_amd.configs import CONFIGS, build_lens

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg_name,divisor", [("cfg1", 1), ("cfg1", 3), ("cfg2", 5), ("cfg3", 2)])
def test_interpolate_matches_host_and_oracle(bzr, orc, ctx, cfg_name, divisor):
    lens = CONFIGS[cfg_name].lenses[0]
    mesh = build_lens(bzr.TriMesh, lens)
    patches = mesh.bezier_patches()
    got = bzr.interpolate(ctx, bzr.DeviceMesh(ctx, patches), divisor)
    assert got.shape == (divisor * divisor * len(patches), 3, 3)
    host = mesh.bezier_interpolate(divisor).triangles
    assert np.array_equal(got.view(np.uint32), host.view(np.uint32))
    oracle = build_lens(orc.OMesh, lens).bezier_interpolate(divisor).triangles
    assert np.array_equal(got.view(np.uint32), np.asarray(oracle, np.float32).view(np.uint32))


def test_interpolate_device_buffer_and_stl(bzr, ctx, tmp_path):
    torch = pytest.importorskip("torch")
    mesh = build_lens(bzr.TriMesh, CONFIGS["cfg2"].lenses[0])
    patches = mesh.bezier_patches()
    dm = bzr.DeviceMesh(ctx, patches)
    out = torch.empty((25 * len(patches), 3, 3), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.use_torch_stream()
    try:
        bzr.interpolate(ctx, dm, 5, out=out)
        torch.cuda.synchronize()
    finally:
        ctx.use_own_stream()
    gpu_mesh = bzr.TriMesh()
    gpu_mesh.triangles = out.cpu().numpy()
    gpu_mesh.write_stl(tmp_path / "gpu.stl")
    mesh.bezier_interpolate(5).write_stl(tmp_path / "host.stl")
    assert (tmp_path / "gpu.stl").read_bytes() == (tmp_path / "host.stl").read_bytes()


def test_interpolate_rejects_bad_divisor(bzr, ctx):
    dm = bzr.DeviceMesh(ctx, build_lens(bzr.TriMesh, CONFIGS["cfg1"].lenses[0]).bezier_patches())
    with pytest.raises(bzr.BzrError):
        bzr.interpolate(ctx, dm, 0)
