"""Stride-2 compact addend (igemm epilogue ``addend_s2``): a 1x1 stride-2 projection's input gradient
exists only at the even pixels, is computed on the strided grid, and conv1's data-gradient epilogue
adds it there.  Checked against the full zero-filled gradient summed in fp32, plain and with the
fused BN-backward epilogue, at the ResNet-50/CIFAR batch-256 stage-2 entry shape."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("shape", [(256, 32, 32, 256, 128, 512), (4, 7, 9, 64, 32, 64)])
@pytest.mark.parametrize("bn", [False, True])
def test_addend_s2(gpu, shape, bn):
    torch.manual_seed(31)
    N, H, W, C, K1, Ksc = shape
    P, Q = (H + 1) // 2, (W + 1) // 2
    dy1 = torch.randn(N, H, W, K1, device=gpu).bfloat16()           # conv1 (1x1, stride 1) output grad
    w1 = (torch.randn(K1, 1, 1, C, device=gpu) * 0.05).bfloat16()
    dysc = torch.randn(N, P, Q, Ksc, device=gpu).bfloat16()         # shortcut (1x1, stride 2) output grad
    wsc = (torch.randn(Ksc, 1, 1, C, device=gpu) * 0.05).bfloat16()
    dxc = torch.ops.tfx.conv_dgrad(dysc, wsc, [N, P, Q, C], 1, 0, 1, None)
    full = torch.ops.tfx.conv_dgrad(dysc, wsc, [N, H, W, C], 2, 0, 1, None)  # zero-filled reference path
    ref = dy1.float().reshape(-1, K1) @ w1.float().reshape(K1, C)
    ref = ref.reshape(N, H, W, C) + full.float()
    assert full[:, 1::2].float().abs().max().item() == 0 and full[:, :, 1::2].float().abs().max().item() == 0
    if not bn:
        dx = torch.ops.tfx.conv_dgrad(dy1, w1, [N, H, W, C], 1, 0, 1, dxc, None, True)
    else:
        xb = torch.randn(N, H, W, C, device=gpu).bfloat16()
        save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(gpu)
        ws = torch.zeros(64 * 2 * C + 64, device=gpu)
        dx, red = torch.ops.tfx.conv_dgrad_bn(dy1, w1, [N, H, W, C], 1, 0, 1, dxc, xb, save, None, True, ws, None,
                                              None, None, True, True)
        g = dx.float() * (xb.float() > 0)
        assert _rel(red[:C], g.sum((0, 1, 2))) < 1e-2
    assert _rel(dx, ref) < 1e-2
