"""The exact normalized() (Eigen `a / sqrt(a.a)`, reference/3dGeomUtil.h via bezierTriangle.cpp:164,233)
with one square root and a shared reciprocal (patch_math.hpp `unit`) returns the same bits as one
correctly rounded division per component, and as numpy's IEEE float32 arithmetic, over vectors whose
components span the whole float range (the guard's fallback included).  Called through the C-ABI test
hook bzr_debug_unit (include/bzr_debug.h)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _vectors(torch, n, gen, kind):
    if kind == "unitish":  # what the Newton site normalizes: tangent crosses, hit - plane point
        mag = torch.exp2(torch.empty(n, 1, device="cuda").uniform_(-40.0, 20.0, generator=gen))
        return (torch.randn(n, 3, device="cuda", generator=gen) * mag).T.contiguous()
    if kind == "wide":  # every exponent, both signs, per component
        e = torch.randint(-150, 128, (3, n), device="cuda", generator=gen).float()
        m = torch.empty(3, n, device="cuda").uniform_(1.0, 2.0, generator=gen)
        s = torch.randint(0, 2, (3, n), device="cuda", generator=gen).float() * 2 - 1
        return (s * m * torch.exp2(e)).float().contiguous()
    if kind == "zeros":  # axis-aligned and signed-zero components
        v = torch.randn(3, n, device="cuda", generator=gen)
        z = torch.randint(0, 4, (3, n), device="cuda", generator=gen)
        v = torch.where(z == 0, torch.zeros_like(v), v)
        v = torch.where(z == 1, -torch.zeros_like(v), v)
        return v.contiguous()
    # guard edges: |a_k| near 2^-100, z near 2^-96 and 2^40
    base = torch.randn(3, n, device="cuda", generator=gen)
    pick = torch.randint(0, 4, (1, n), device="cuda", generator=gen).float()
    scale = torch.where(pick == 0, 2.0 ** -100, torch.where(pick == 1, 2.0 ** -48, torch.where(pick == 2, 2.0 ** 20, 2.0 ** -101)))
    jitter = torch.exp2(torch.empty(3, n, device="cuda").uniform_(-2.0, 2.0, generator=gen))
    return (base * scale * jitter).float().contiguous()


def _numpy_unit(a):
    x, y, z = a.astype(np.float32)
    with np.errstate(all="ignore"):
        zz = x * x + (y * y + z * z)
        s = np.sqrt(zz)
        out = np.stack([x / s, y / s, z / s])
    keep = ~(zz > 0)
    out[:, keep] = a[:, keep]
    return out


@pytest.mark.parametrize("kind", ["unitish", "wide", "zeros", "edges"])
def test_shared_reciprocal_unit_is_bit_exact(bzr, ctx, kind):
    torch = pytest.importorskip("torch")
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234 + len(kind))
    L = bzr.lib()
    n = 1 << 22
    ctx.use_torch_stream()
    for rep in range(4):
        a = _vectors(torch, n, gen, kind)
        out = torch.empty(6, n, device="cuda")
        assert L.bzr_debug_unit(ctx.handle, ctypes.c_void_p(a.data_ptr()), n, ctypes.c_void_p(out.data_ptr())) == 0
        torch.cuda.synchronize()
        got, ref = out[:3].view(torch.int32), out[3:].view(torch.int32)
        bad = (got != ref).any(dim=0)
        assert int(bad.sum()) == 0, (kind, rep, a[:, bad][:, :4].cpu().numpy(), out[:, bad][:, :4].cpu().numpy())
        if rep == 0:  # IEEE float32 on the CPU: the oracle's arithmetic
            k = 1 << 16
            host = a[:, :k].cpu().numpy()
            want = _numpy_unit(host)
            gotk = out[:3, :k].cpu().numpy()
            same = (gotk.view(np.uint32) == want.view(np.uint32)) | (np.isnan(gotk) & np.isnan(want))
            assert same.all(), (kind, host[:, ~same.all(axis=0)][:, :4])


def _heights(torch, n, gen, kind):
    """(hIn, hOut, cos) rows: the dome heights are record constants, cos a lane's plane cosine."""
    if kind == "lens":  # what the Newton site sees: heights ~1e-3..1, |cos| in [1e-5, 1]
        h = torch.exp2(torch.empty(2, n, device="cuda").uniform_(-12.0, 0.0, generator=gen))
        h = h * (torch.randint(0, 2, (2, n), device="cuda", generator=gen).float() * 2 - 1)
        c = torch.exp2(torch.empty(1, n, device="cuda").uniform_(-16.6, 0.0, generator=gen))
        c = c * (torch.randint(0, 2, (1, n), device="cuda", generator=gen).float() * 2 - 1)
        return torch.cat([h, c]).contiguous()
    # every exponent (the guard's fallback), zeros of both signs
    e = torch.randint(-150, 128, (3, n), device="cuda", generator=gen).float()
    m = torch.empty(3, n, device="cuda").uniform_(1.0, 2.0, generator=gen)
    s = torch.randint(0, 2, (3, n), device="cuda", generator=gen).float() * 2 - 1
    v = (s * m * torch.exp2(e)).float()
    z = torch.randint(0, 16, (3, n), device="cuda", generator=gen)
    v = torch.where(z == 0, torch.zeros_like(v), torch.where(z == 1, -torch.zeros_like(v), v))
    return v.contiguous()


@pytest.mark.parametrize("kind", ["lens", "wide"])
def test_shared_reciprocal_heights_are_bit_exact(bzr, ctx, kind):
    """newton_tail's din = hIn / cos, dout = hOut / cos (reference/bezierTriangle.cpp:132-133) with one shared
    reciprocal (patch_math.hpp div_heights) == one correctly rounded division each == numpy float32."""
    torch = pytest.importorskip("torch")
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4321 + len(kind))
    L = bzr.lib()
    n = 1 << 22
    ctx.use_torch_stream()
    for rep in range(4):
        a = _heights(torch, n, gen, kind)
        out = torch.empty(4, n, device="cuda")
        assert L.bzr_debug_div_heights(ctx.handle, ctypes.c_void_p(a.data_ptr()), n, ctypes.c_void_p(out.data_ptr())) == 0
        torch.cuda.synchronize()
        got, ref = out[:2].view(torch.int32), out[2:].view(torch.int32)
        bad = (got != ref).any(dim=0) & ~(torch.isnan(out[:2]).any(dim=0) & torch.isnan(out[2:]).any(dim=0))
        assert int(bad.sum()) == 0, (kind, rep, a[:, bad][:, :4].cpu().numpy())
        if rep == 0:
            k = 1 << 16
            host = a[:, :k].cpu().numpy()
            with np.errstate(all="ignore"):
                want = np.stack([host[0] / host[2], host[1] / host[2]]).astype(np.float32)
            gotk = out[:2, :k].cpu().numpy()
            same = (gotk.view(np.uint32) == want.view(np.uint32)) | (np.isnan(gotk) & np.isnan(want))
            assert same.all(), (kind, host[:, ~same.all(axis=0)][:, :4])
