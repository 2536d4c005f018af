"""Slot-consuming BN passes (csrc/kernels/batchnorm.hip "slot-consuming passes") against an fp32
PyTorch reference: the forward apply reduces the forward statistics slots itself, the backward
apply reduces the backward partials itself, and each direction leaves the OTHER direction's slots
zero.  Shapes include the ResNet-50/CIFAR batch-256 layers (slab grid with many row groups, the
4-slab / 8-slab channel splits of the stage-3/4 tails).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

NSLOT = 64


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _ref(x, r, gamma, beta, relu):
    xr = x.float().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if r is not None else None
    mean, var = xr.mean(0), xr.var(0, unbiased=False)
    yr = (xr - mean) / torch.sqrt(var + 1e-5) * gr + br
    if rr is not None:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    return xr, gr, br, rr, yr, mean, var


@pytest.mark.parametrize("M,C,res,relu", [
    (512, 64, False, True),
    (512, 128, False, False),
    (1024, 256, True, True),
    (512, 512, True, True),
    (256, 2048, True, True),
    (256 * 32 * 32, 64, False, True),     # stage-1 bn1/bn2, batch 256
    (256 * 32 * 32, 256, True, True),     # stage-1 block tail
    (256 * 4 * 4, 2048, True, True),      # stage-4 block tail (8 slabs)
])
def test_bn_slots_fwd_bwd(gpu, M, C, res, relu):
    torch.manual_seed(11)
    x = _bf(torch.randn(M, C, device=gpu) * 2 + 0.5)
    r = _bf(torch.randn(M, C, device=gpu)) if res else None
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    sf = torch.zeros(NSLOT * 2 * C + 64, device=gpu)
    sb = torch.full((NSLOT * 2 * C + 64,), 7.0, device=gpu)  # stale partials: the forward must clear them
    sb[NSLOT * 2 * C:] = 0
    y, save, mask = torch.ops.tfx.bn_fwd_slots(x, gamma, beta, rm, rv, 0.1, 1e-5, r, relu, sf, sb, False)
    assert sb.abs().max().item() == 0.0, "forward apply must zero the backward slots"
    xr, gr, br, rr, yr, mean, var = _ref(x, r, gamma, beta, relu)
    assert _rel(y, yr) < 1e-2
    assert _rel(save[:C], mean) < 1e-4
    assert torch.allclose(rm, 0.1 * mean.detach(), atol=1e-4)
    assert torch.allclose(rv, 0.9 + 0.1 * var.detach() * M / (M - 1), atol=1e-3)
    if res and relu:
        bits = torch.stack([(mask.long() >> k) & 1 for k in range(8)], 1).reshape(M, C)
        assert torch.equal(bits.bool(), y.float() > 0)
    g = _bf(torch.randn(M, C, device=gpu))
    yr.backward(g.float())
    dgam, dbet = torch.ones(C, device=gpu), torch.zeros(C, device=gpu)
    assert sf.abs().max().item() > 0  # statistics still in S_f until the backward apply
    dx, dres = torch.ops.tfx.bn_bwd_slots(g, x, res, save, relu, mask if (res and relu) else None, sb, sf,
                                          dgam, dbet, False, True)
    assert sf.abs().max().item() == 0.0, "backward apply must zero the forward slots"
    assert sb.abs().max().item() > 0  # partials stay until the next forward
    assert _rel(dx, xr.grad) < 2e-2
    assert _rel(dgam - 1, gr.grad) < 1e-3 and _rel(dbet, br.grad) < 1e-3
    if res:
        assert _rel(dres, rr.grad) < 1e-2
    # a second forward (next step) sees clean S_f (stats pass refills it) and clears S_b again
    y2, _, _ = torch.ops.tfx.bn_fwd_slots(x, gamma, beta, None, None, 0.1, 1e-5, r, relu, sf, sb, False)
    assert sb.abs().max().item() == 0.0
    assert _rel(y2, y) < 1e-3  # same statistics up to the float-atomic summation order


def test_bn_slots_consumer_dgrad_partials(gpu):
    """conv_dgrad_bn(reduce=False) leaves the BN-backward partials in S_b; bn_bwd_slots(have_partials)
    reduces them and matches the standalone reduce path (batch-256 stage-2 bn2 shape)."""
    torch.manual_seed(12)
    N, H, W, C, Ko = 256, 16, 16, 128, 128
    M = N * H * W
    xb = _bf(torch.randn(N, H, W, C, device=gpu) + 0.3)
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu) * 0.1
    sf = torch.zeros(NSLOT * 2 * C + 64, device=gpu)
    sb = torch.zeros_like(sf)
    _, save, _ = torch.ops.tfx.bn_fwd_slots(xb, gamma, beta, None, None, 0.1, 1e-5, None, True, sf, sb, False)
    w = _bf(torch.randn(Ko, 3, 3, C, device=gpu) * 0.05)
    dy = _bf(torch.randn(N, H, W, Ko, device=gpu))
    dx, red = torch.ops.tfx.conv_dgrad_bn(dy, w, [N, H, W, C], 1, 1, 1, None, xb, save, None, True, sb, None,
                                          None, None, False)
    assert red is None or red.numel() == 0
    dg1, db1 = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    sf1 = sf.clone()
    d1, _ = torch.ops.tfx.bn_bwd_slots(dx, xb, False, save, True, None, sb, sf1, dg1, db1, True, False)
    sb2, sf2 = torch.zeros_like(sb), sf.clone()
    dg2, db2 = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    d2, _ = torch.ops.tfx.bn_bwd_slots(dx, xb, False, save, True, None, sb2, sf2, dg2, db2, False, False)
    assert _rel(d1, d2) < 1e-2
    assert _rel(dg1, dg2) < 1e-3 and _rel(db1, db2) < 1e-3
    assert sf1.abs().max().item() == 0.0 and sf2.abs().max().item() == 0.0
