"""CIFAR stem weight gradient (csrc/kernels/stem.hip: one block per 32x32 image, im2col^T built in LDS
per row) against the generic implicit-GEMM weight gradient and a plain fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("N", [256, 3])
def test_stem_wgrad_matches_generic_and_fp32(gpu, N):
    torch.manual_seed(41)
    x = torch.zeros(N, 32, 32, 8, device=gpu)
    x[..., :3] = torch.randn(N, 32, 32, 3, device=gpu)  # RGB in channels 0..2, the pad channels zero
    x = x.to(torch.bfloat16)
    dy = torch.randn(N, 32, 32, 64, device=gpu).to(torch.bfloat16)
    dw = torch.full((64, 3, 3, 8), 0.25, device=gpu)  # accumulates into an existing gradient
    dw_gen = dw.clone()
    ws = torch.zeros(int(torch.ops.tfx.stem_wgrad_ws_floats(64)), device=gpu)
    torch.ops.tfx.stem_wgrad(dy, x, dw, ws)
    torch.ops.tfx.conv_wgrad(dy, x, dw_gen, 1, 1, 1, True)
    torch.cuda.synchronize()
    xr = x.float().permute(0, 3, 1, 2)
    wr = torch.zeros(64, 8, 3, 3, device=gpu, requires_grad=True)
    F.conv2d(xr, wr, padding=1).backward(dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(0, 2, 3, 1) + 0.25
    assert _rel(dw, ref) < 1e-4
    assert _rel(dw, dw_gen) < 1e-4
    assert torch.all(dw[..., 3:] == 0.25), "padded input channels get exactly zero gradient"
    assert ws.abs().max().item() == 0.0, "workspace copies re-zeroed"


def test_resnet_stem_routes_to_stem_kernel(gpu):
    from tensorflow_examples_amd import ops
    from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input
    from tensorflow_examples_amd.ops import nn as nnops
    img = torch.randint(0, 256, (8, 32, 32, 3), dtype=torch.uint8, device=gpu)
    lab = torch.randint(0, 10, (8,), device=gpu)
    st, m = build_resnet_cifar(device=gpu, depth=50, dtype=torch.bfloat16, seed=3)
    st.zero_grad()
    n0 = nnops.STEM_WGRAD_CALLS[0]
    m.training_loss(to_model_input(img), lab, unit_seed=True).backward()
    torch.cuda.synchronize()
    assert nnops.STEM_WGRAD_CALLS[0] - n0 == 1
    g = st.grad[m.stem.w.offset:m.stem.w.offset + m.stem.w.numel].view(64, 3, 3, 8)
    assert torch.isfinite(g).all() and g[..., :3].abs().sum() > 0 and torch.all(g[..., 3:] == 0)


@pytest.mark.parametrize("N", [256, 3])
def test_stem_forward_with_bn_stats_matches_generic_and_fp32(gpu, N):
    """conv_fwd_bn routes the stem to stem.hip: outputs and BN statistics vs the generic implicit GEMM
    (torch.ops.tfx.conv_stem_fwd(False)) and fp32 PyTorch."""
    torch.manual_seed(43)
    x = torch.zeros(N, 32, 32, 8, device=gpu)
    x[..., :3] = torch.randn(N, 32, 32, 3, device=gpu)
    x = x.to(torch.bfloat16)
    w = torch.zeros(64, 3, 3, 8, device=gpu)
    w[..., :3] = torch.randn(64, 3, 3, 3, device=gpu) * 0.2
    w = w.to(torch.bfloat16)
    g, b = torch.rand(64, device=gpu) + 0.5, torch.randn(64, device=gpu) * 0.2

    def run(on):
        prev = torch.ops.tfx.conv_stem_fwd(on)
        try:
            ws = torch.zeros(64 * 2 * 64, device=gpu)
            rm, rv = torch.zeros(64, device=gpu), torch.ones(64, device=gpu)
            y, save = torch.ops.tfx.conv_fwd_bn(x, w, 1, 1, 1, ws, g, b, rm, rv, 0.1, 1e-5)
            torch.cuda.synchronize()
            return y, save, ws, rm, rv
        finally:
            torch.ops.tfx.conv_stem_fwd(prev)

    y, save, ws, rm, rv = run(True)
    y0, save0, _, rm0, rv0 = run(False)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 5e-3
    assert _rel(y, y0) < 5e-3
    assert ws.abs().max().item() == 0.0
    yf = y.float().reshape(-1, 64)
    assert torch.allclose(save[:64], yf.mean(0), rtol=1e-3, atol=1e-3)
    assert torch.allclose(save, save0, rtol=2e-3, atol=2e-3)
    assert torch.allclose(rm, rm0, rtol=1e-3, atol=1e-5) and torch.allclose(rv, rv0, rtol=1e-3, atol=1e-5)
