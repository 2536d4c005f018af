"""Every conv of the headline ResNet-50/CIFAR step at its REAL batch-256 shape, forward / data
gradient / weight gradient (+ the fused-BN epilogue variants the step uses), against a plain
PyTorch fp32 reference of the same op.

The small-shape tests in test_kernels_gpu.py never reach the tile / pipeline branches the bench
takes at these sizes: 256x64 tiles (M >= 65 536), the 128x64 under-fill policy, the LDS-DMA ring
depths, single-k-tile kernels, the in-block split-K weight gradients, the stride-2 parity-class
data gradients and the last-arriver BN finalize.  One test per distinct layer shape covers them all
(the shapes are the ones bench.py runs; see scripts/conv_bench.py)."""
import math
import os
import sys

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))


def _shapes(B=256):
    from conv_bench import resnet50_convs
    seen, out = set(), []
    for sh in resnet50_convs(B):
        if sh not in seen:
            seen.add(sh)
            out.append(sh)
    return out


# batch 256 (bench.py's default) and 128 (a second per-GPU batch: a non-256 ``--batch`` must not
# reach a tile / ring pick that no test ran)
SHAPES = _shapes(256) + _shapes(128)


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _ids(sh):
    N, H, W, C, K, R, st = sh
    return "%dx%dx%d_c%d_k%d_r%d_s%d" % (N, H, W, C, K, R, st)


@pytest.mark.parametrize("shape", SHAPES, ids=[_ids(s) for s in SHAPES])
def test_conv_production_shape(gpu, shape):
    N, H, W, C, Ko, R, st = shape
    pad = R // 2
    g = torch.Generator(device=gpu).manual_seed(hash(shape) & 0xffff)
    x = _bf(torch.randn(N, H, W, C, device=gpu, generator=g))
    if C == 8:  # padded-RGB stem: channels 3..7 are zero
        x[..., 3:] = 0
    w = _bf(torch.randn(Ko, R, R, C, device=gpu, generator=g) * (1.0 / math.sqrt(R * R * C)))
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pad)
    y = torch.ops.tfx.conv_fwd(x, w, st, pad, 1)
    assert _rel(y, yr.permute(0, 2, 3, 1)) < 1e-2

    gy = _bf(torch.randn(y.shape, device=gpu, generator=g))
    yr.backward(gy.float().permute(0, 3, 1, 2))
    dx = torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None)
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    dw = torch.zeros(Ko, R, R, C, device=gpu)
    torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, False)
    assert _rel(dw, wr.grad.permute(0, 2, 3, 1)) < 5e-3

    # fused-BN forward epilogue (statistics + last-arriver finalize), as after_conv runs it
    gamma = torch.rand(Ko, device=gpu, generator=g) + 0.5
    beta = torch.randn(Ko, device=gpu, generator=g)
    ws = torch.zeros(64 * 2 * Ko + 64, device=gpu)
    yb, save = torch.ops.tfx.conv_fwd_bn(x, w, st, pad, 1, ws, gamma, beta, None, None, 0.1, 1e-5)
    torch.cuda.synchronize()
    assert _rel(yb, y) < 1e-3
    yf = yb.float().reshape(-1, Ko)
    mean, var = yf.mean(0), yf.var(0, unbiased=False)
    assert torch.allclose(save[:Ko], mean, rtol=1e-3, atol=1e-3)
    assert torch.allclose(save[Ko:2 * Ko], torch.rsqrt(var + 1e-5), rtol=2e-3, atol=1e-3)
    assert ws.abs().max().item() == 0.0

    # fused-BN backward reduction in the data-gradient epilogue (stride-1 convs only, as the model)
    if st == 1:
        xb = _bf(torch.randn(N, H, W, C, device=gpu, generator=g) * 1.5 + 0.3)
        gam, bet = torch.rand(C, device=gpu, generator=g) + 0.5, torch.randn(C, device=gpu, generator=g)
        wsb = torch.zeros(64 * 2 * C + 64, device=gpu)
        _, sv, _ = torch.ops.tfx.bn_fwd_train(xb, gam, bet, None, None, 0.1, 1e-5, None, True, wsb, False)
        dx2, red = torch.ops.tfx.conv_dgrad_bn(gy, w, list(x.shape), st, pad, 1, None, xb, sv, None, True, wsb,
                                               None, None)
        assert _rel(dx2, dx) < 1e-3
        _, _, red_ref = torch.ops.tfx.bn_bwd(dx2, xb, None, sv, True, torch.zeros_like(wsb), None, None, None)
        assert _rel(red, red_ref) < 2e-3
        assert wsb.abs().max().item() == 0.0


PW_FWD = [s for s in SHAPES if s[5] == 1 and s[6] == 1 and s[0] == 256]


@pytest.mark.parametrize("shape", PW_FWD, ids=[_ids(s) for s in PW_FWD])
def test_persistent_pointwise_forward_matches_per_tile_kernel(gpu, shape):
    """The persistent 1x1 forward (igemm_persist.hip: one LDS-DMA ring over all of a block's tiles, ring
    depth 2 or 3) against the one-tile-per-block kernel and fp32: output and the fused BN statistics
    (saved mean / invstd) at every production 1x1 shape."""
    N, H, W, C, Ko, R, st = shape
    g = torch.Generator(device=gpu).manual_seed(7 + C + Ko)
    x = _bf(torch.randn(N, H, W, C, device=gpu, generator=g))
    w = _bf(torch.randn(Ko, 1, 1, C, device=gpu, generator=g) * (1.0 / math.sqrt(C)))
    yr = torch.einsum("nhwc,kc->nhwk", x.float(), w.float().reshape(Ko, C))
    gamma = torch.rand(Ko, device=gpu, generator=g) + 0.5
    beta = torch.randn(Ko, device=gpu, generator=g)
    res = {}
    prev = torch.ops.tfx.igemm_persist_mode(0)
    try:
        for mode in (0, 2, 3):
            torch.ops.tfx.igemm_persist_mode(mode)
            ws = torch.zeros(64 * 2 * Ko + 64, device=gpu)
            yb, save = torch.ops.tfx.conv_fwd_bn(x, w, 1, 0, 1, ws, gamma, beta, None, None, 0.1, 1e-5)
            y = torch.ops.tfx.conv_fwd(x, w, 1, 0, 1)
            torch.cuda.synchronize()
            assert float(ws[:64 * 2 * Ko].abs().max()) == 0.0, "statistics slots left dirty"
            res[mode] = (yb, save.clone(), y)
    finally:
        torch.ops.tfx.igemm_persist_mode(prev)
    mean_r = yr.reshape(-1, Ko).mean(0)
    for mode in (2, 3):
        yb, save, y = res[mode]
        assert _rel(yb, yr) < 1e-2 and _rel(y, yr) < 1e-2
        # (the per-tile kernel splits K over two wave groups at some shapes: summation order differs)
        assert _rel(yb, res[0][0]) < 2e-3 and _rel(y, res[0][2]) < 2e-3
        assert _rel(save[:Ko], res[0][1][:Ko]) < 1e-4 and _rel(save[Ko:2 * Ko], res[0][1][Ko:2 * Ko]) < 1e-4
        assert _rel(save[:Ko], mean_r) < 2e-2
