"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

All tests are ``@pytest.mark.gpu`` (run on the MI355X box via gpurun).  Inputs are
bf16-representable so the only error left is accumulation order / output rounding.
"""
import math

import pytest
import torch
import torch.nn.functional as F
from tensorflow_examples_amd import ops

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_SHAPES = [
    # N, H, W, C, Ko, R, stride, pad
    (4, 8, 8, 64, 64, 1, 1, 0),
    (2, 8, 8, 64, 128, 3, 1, 1),
    (3, 9, 7, 32, 64, 3, 2, 1),
    (2, 8, 8, 64, 256, 1, 2, 0),
    (2, 32, 32, 8, 64, 3, 1, 1),  # padded-RGB stem
    (1, 5, 5, 16, 24, 3, 1, 1),   # ragged M / N
    # stride-2 data gradients run as 4 output-parity-class GEMMs (even / odd grids, empty classes)
    (2, 16, 16, 128, 128, 3, 2, 1),
    (2, 10, 10, 64, 32, 5, 2, 2),
    (2, 7, 9, 32, 64, 1, 2, 0),
    (2, 16, 16, 64, 128, 1, 2, 0),
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd_dgrad_wgrad(gpu, shape):
    N, H, W, C, Ko, R, st, pad = shape
    torch.manual_seed(0)
    x = _bf(torch.randn(N, H, W, C, device=gpu))
    w = _bf(torch.randn(Ko, R, R, C, device=gpu) * (1.0 / math.sqrt(R * R * C)))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pad)
    y = torch.ops.tfx.conv_fwd(x, w, st, pad, 1)
    assert y.shape == (N, yr.shape[2], yr.shape[3], Ko)
    assert _rel(y, yr.permute(0, 2, 3, 1)) < 1e-2
    gy = _bf(torch.randn_like(y.float()))
    yr.backward(gy.float().permute(0, 3, 1, 2))
    dx = torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, None)
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    add = _bf(torch.randn_like(dx.float()))
    ref_sum = dx.float() + add.float()
    dx2 = torch.ops.tfx.conv_dgrad(gy, w, list(x.shape), st, pad, 1, add)  # epilogue-fused sum, in place
    assert dx2.data_ptr() == add.data_ptr() and _rel(dx2, ref_sum) < 1e-2
    dw = torch.zeros(Ko, R, R, C, device=gpu)
    torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, False)
    assert _rel(dw, wr.grad.permute(0, 2, 3, 1)) < 5e-3
    # accumulate mode adds on top
    torch.ops.tfx.conv_wgrad(gy, x, dw, st, pad, 1, True)
    assert _rel(dw, 2 * wr.grad.permute(0, 2, 3, 1)) < 5e-3


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("mnk", [(256, 128, 64), (200, 136, 328), (64, 16, 1024)])
def test_gemm_layouts(gpu, ta, tb, mnk):
    M, N, K = mnk
    torch.manual_seed(1)
    A = torch.randn(M, K, device=gpu)
    B = torch.randn(K, N, device=gpu) + torch.arange(N, device=gpu)[None, :] * 0.01  # asymmetric
    a = _bf(A.t().contiguous() if ta else A)
    b = _bf(B.t().contiguous() if tb else B)
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    out = torch.ops.tfx.gemm(a, b, ta, tb, None, False, True)
    assert _rel(out, ref) < 1e-5 * math.sqrt(K) + 1e-5
    acc = torch.ones(M, N, device=gpu)
    torch.ops.tfx.gemm_into(a, b, ta, tb, acc, True)
    assert _rel(acc, ref + 1) < 1e-4


def test_gemm_identity_asymmetric(gpu):
    # A = I with an asymmetric B catches a transposed C-write (cdna_hip_programming.md §3)
    I = _bf(torch.eye(128, device=gpu))
    B = _bf(torch.arange(128 * 128, device=gpu, dtype=torch.float32).view(128, 128) % 97)
    out = torch.ops.tfx.gemm(I, B, False, False, None, False, True)
    assert torch.equal(out, B.float())


def test_gemm_bias_relu_bf16(gpu):
    a = _bf(torch.randn(64, 256, device=gpu))
    w = _bf(torch.randn(96, 256, device=gpu))
    b = torch.randn(96, device=gpu)
    out = torch.ops.tfx.gemm(a, w, False, True, b, True, False)
    ref = torch.relu(a.float() @ w.float().t() + b)
    assert out.dtype == torch.bfloat16 and _rel(out, ref) < 1e-2


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,N,K,split", [(64, 128, 4096, True), (4096, 64, 128, True), (4096, 128, 64, False),
                                         (100, 784, 100, False), (37, 61, 1029, True)])
def test_sgemm_shapes(gpu, ta, tb, M, N, K, split):
    """The word2vec sampled-loss GEMMs (neg = E Ws^T, dE += dn Ws, dWs = dn^T E with split-K f32
    atomics) and ragged shapes that take the scalar (non-16-byte) staging path."""
    torch.manual_seed(5)
    A = torch.randn(M, K, device=gpu)
    B = torch.randn(K, N, device=gpu)
    a = A.t().contiguous() if ta else A
    b = B.t().contiguous() if tb else B
    out = torch.ops.tfx.sgemm(a, b, ta, tb, None, 0, split)
    ref = (A.double() @ B.double()).float()
    tol = 1e-4 * max(1.0, K / 100) ** 0.5
    assert (out - ref).abs().max().item() < 10 * tol
    acc = torch.randn(M, N, device=gpu)
    acc0 = acc.clone()
    torch.ops.tfx.sgemm_into(a, b, ta, tb, acc, True, split)
    assert (acc - (acc0 + ref)).abs().max().item() < 10 * tol


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True)])
def test_sgemm_exact_f32(gpu, ta, tb):
    torch.manual_seed(2)
    M, N, K = 100, 10, 100
    A = torch.randn(M, K, device=gpu)
    B = torch.randn(K, N, device=gpu)
    a = A.t().contiguous() if ta else A
    b = B.t().contiguous() if tb else B
    out = torch.ops.tfx.sgemm(a, b, ta, tb, None, 0)
    ref = (A.double() @ B.double()).float()
    assert (out - ref).abs().max().item() < 1e-4
    bias = torch.randn(N, device=gpu)
    sig = torch.ops.tfx.sgemm(a, b, ta, tb, bias, 2)
    assert torch.allclose(sig, torch.sigmoid(ref + bias), atol=1e-5)


@pytest.mark.parametrize("C", [64, 256, 2048, 6, 120])
@pytest.mark.parametrize("res,relu", [(False, False), (False, True), (True, True)])
def test_batchnorm_train(gpu, C, res, relu):
    torch.manual_seed(3)
    M = 512
    x = _bf(torch.randn(M, C, device=gpu) * 2 + 0.5)
    r = _bf(torch.randn(M, C, device=gpu)) if res else None
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    ws = torch.zeros(64 * 2 * C, device=gpu)
    y, save, mask = torch.ops.tfx.bn_fwd_train(x, gamma, beta, rm, rv, 0.1, 1e-5, r, relu, ws, False)
    assert ws.abs().max().item() == 0.0  # consumed workspace is re-zeroed
    if res and relu and C % 8 == 0 and 256 % (C // 8) == 0:  # 1-bit ReLU mask of y, one byte per 8 channels
        bits = torch.stack([(mask.long() >> k) & 1 for k in range(8)], 1).reshape(M, C)
        assert torch.equal(bits.bool(), y.float() > 0)
    else:
        assert mask is None or mask.numel() == 0
    xr = x.float().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rr = r.float().requires_grad_(True) if res else None
    mean, var = xr.mean(0), xr.var(0, unbiased=False)
    yr = (xr - mean) / torch.sqrt(var + 1e-5) * gr + br
    if res:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    assert _rel(y, yr) < 1e-2
    assert torch.allclose(rm, 0.1 * mean.detach(), atol=1e-4)
    assert torch.allclose(rv, 0.9 + 0.1 * var.detach() * M / (M - 1), atol=1e-3)
    g = _bf(torch.randn(M, C, device=gpu))
    yr.backward(g.float())
    dgam, dbet = torch.ones(C, device=gpu), torch.zeros(C, device=gpu)
    has_mask = mask is not None and mask.numel() > 0
    dx, dres, red = torch.ops.tfx.bn_bwd(g, x, None if has_mask else r, save, relu, ws, dgam, dbet,
                                         mask if has_mask else None)
    assert ws.abs().max().item() == 0.0
    if has_mask:  # the residual-tensor path (generic kernels) gives the same gradients
        dx2, dres2, _ = torch.ops.tfx.bn_bwd(g, x, r, save, relu, ws, None, None, None)
        assert _rel(dx2, dx) < 1e-2 and _rel(dres2, dres) < 1e-2
    assert _rel(dx, xr.grad) < 2e-2
    assert _rel(red[C:], gr.grad) < 1e-3 and _rel(red[:C], br.grad) < 1e-3
    assert _rel(dgam - 1, gr.grad) < 1e-3 and _rel(dbet, br.grad) < 1e-3  # accumulated in place
    if res:
        assert _rel(dres, rr.grad) < 1e-2


@pytest.mark.parametrize("naive", [False, True])
@pytest.mark.parametrize("dense", [False, True])
def test_softmax_xent(gpu, naive, dense):
    torch.manual_seed(4)
    B, C = 100, 10
    z = torch.randn(B, C, device=gpu) * 3
    lab = torch.randint(0, C, (B,), device=gpu)
    y = F.one_hot(lab, C).float()
    loss_rows, dz = torch.ops.tfx.softmax_xent(z, None if dense else lab, y if dense else None, naive, 1.0 / B, True)
    zr = z.clone().requires_grad_(True)
    if naive:
        lr = -(y * torch.log(torch.softmax(zr, 1))).sum(1)
    else:
        lr = -(y * torch.log_softmax(zr, 1)).sum(1)
    lr.mean().backward()
    assert torch.allclose(loss_rows, lr.detach(), atol=1e-4, rtol=1e-4)
    assert torch.allclose(dz, zr.grad, atol=1e-5, rtol=1e-3)
    cnt = torch.ops.tfx.accuracy_count(z, lab, None)
    assert cnt.item() == (z.argmax(1) == lab).sum().item()


@pytest.mark.parametrize("naive", [False, True])
@pytest.mark.parametrize("dense", [False, True])
@pytest.mark.parametrize("B,C,bf16", [(256, 10, True), (100, 10, False), (1024, 10, True), (300, 40, True), (7, 130, True)])
def test_softmax_xent_mean(gpu, naive, dense, B, C, bf16):
    """Single-launch mean loss + dz (the training step's loss): fp32 reference of the same op, and
    the unit-seed autograd path returns the same gradient as the scaled one."""
    torch.manual_seed(5)
    z = (torch.randn(B, C, device=gpu) * 3)
    if bf16:
        z = z.bfloat16()
    lab = torch.randint(0, C, (B,), device=gpu)
    y = F.one_hot(lab, C).float()
    for native_dz in (False, True):
        loss, dz = torch.ops.tfx.softmax_xent_mean(z, None if dense else lab, y if dense else None, naive, True,
                                                   native_dz)
        assert loss.dim() == 0 and dz.dtype == (z.dtype if native_dz else torch.float32)
        zr = z.float().clone().requires_grad_(True)
        if naive:
            lr = (-(y * torch.log(torch.softmax(zr, 1))).sum(1)).mean()
        else:
            lr = (-(y * torch.log_softmax(zr, 1)).sum(1)).mean()
        lr.backward()
        assert abs(loss.item() - lr.item()) < 1e-4 * max(1.0, abs(lr.item()))
        tol = 4e-3 if dz.dtype == torch.bfloat16 else 1e-3
        assert torch.allclose(dz.float(), zr.grad, atol=1e-5, rtol=tol)
    # autograd: unit-seed gradient (ready in the forward) == the scaled/cast backward
    grads = []
    for unit in (False, True):
        zz = z.clone().requires_grad_(True)
        ops.softmax_cross_entropy(zz, y if dense else lab, naive=naive, unit_seed=unit).backward()
        grads.append(zz.grad.float())
    assert torch.allclose(grads[0], grads[1], atol=1e-6, rtol=1e-2)


@pytest.mark.parametrize("shape", [(4, 4, 4, 2048), (256, 4, 4, 2048), (3, 5, 3, 12), (2, 8, 8, 64)])
def test_global_avg_pool(gpu, shape):
    """8-channel vector kernels (C % 8 == 0) and the scalar fallback, bf16 / f32 in and out."""
    N, H, W, C = shape
    x = _bf(torch.randn(N, H, W, C, device=gpu))
    y = torch.ops.tfx.gap_fwd(x, False)
    assert y.dtype == torch.bfloat16 and _rel(y, x.float().mean((1, 2))) < 1e-2
    y32 = torch.ops.tfx.gap_fwd(x, True)
    assert y32.dtype == torch.float32 and _rel(y32, x.float().mean((1, 2))) < 1e-5
    for g in (_bf(torch.randn(N, C, device=gpu)), torch.randn(N, C, device=gpu)):
        dx = torch.ops.tfx.gap_bwd(g, H, W)
        assert _rel(dx, (g.float() / (H * W))[:, None, None, :].expand(N, H, W, C)) < 1e-2


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_optimizer_kernels(gpu, kind):
    from tensorflow_examples_amd.optim import Optimizer
    from tensorflow_examples_amd.variables import RandomNormal, VariableStore

    def make(dev):
        st = VariableStore(dev, torch.bfloat16 if dev.type == "cuda" else torch.float32, seed=7)
        st.variable([37, 5], RandomNormal())
        st.variable([11], RandomNormal())
        st.finalize()
        st.grad.copy_(torch.linspace(-1, 1, st.total))
        o = Optimizer.__new__(Optimizer)
        o.kind = kind
        Optimizer.__init__(o, st, 0.05, weight_decay=0.01, beta1=0.9, beta2=0.99, eps=1e-6)
        return st, o

    sg, og = make(gpu)
    sc, oc = make(torch.device("cpu"))
    for _ in range(3):
        og.apply_gradients(grad_scale=0.5)
        oc.apply_gradients(grad_scale=0.5)
    assert torch.allclose(sg.master.cpu(), sc.master, atol=1e-5, rtol=1e-5)
    assert torch.allclose(sg.shadow.float().cpu(), sc.master, atol=1e-2, rtol=1e-2)


def test_sumsq_and_clip(gpu):
    g = torch.randn(4096, device=gpu)
    s = torch.ops.tfx.sumsq(g)
    assert abs(s.item() - (g.double() ** 2).sum().item()) / s.item() < 1e-5


@pytest.mark.parametrize("shape", [(4, 8, 8, 64, 64, 1, 1, 0), (3, 9, 7, 32, 136, 3, 2, 1)])
def test_conv_fwd_fused_bn_stats(gpu, shape):
    """BN statistics produced by the conv epilogue == statistics of the conv output."""
    N, H, W, C, Ko, R, st, pad = shape
    x = _bf(torch.randn(N, H, W, C, device=gpu))
    w = _bf(torch.randn(Ko, R, R, C, device=gpu) * 0.1)
    slots = torch.zeros(64 * 2 * Ko, device=gpu)
    y = torch.ops.tfx.conv_fwd_stats(x, w, st, pad, 1, slots)
    s = slots.view(64, 2, Ko).sum(0)
    yf = y.float().reshape(-1, Ko)
    assert torch.allclose(s[0], yf.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(s[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
    gamma, beta = torch.ones(Ko, device=gpu), torch.zeros(Ko, device=gpu)
    y1, _, _ = torch.ops.tfx.bn_fwd_train(y, gamma, beta, None, None, 0.1, 1e-5, None, True, slots, True)
    y2, _, _ = torch.ops.tfx.bn_fwd_train(y, gamma, beta, None, None, 0.1, 1e-5, None, True, slots, False)
    assert _rel(y1, y2) < 1e-3


@pytest.mark.parametrize("shape", [(4, 8, 8, 64, 64, 1, 1, 0), (2, 8, 8, 64, 128, 3, 1, 1), (2, 9, 7, 256, 64, 1, 1, 0)])
def test_conv_dgrad_masked_addend(gpu, shape):
    """dX = dgrad(dY) + addend * relu_mask (the identity block's residual gradient consumed as
    (gradient, mask bits) without materialising the masked tensor); the addend stays intact."""
    N, H, W, C, Ko, R, st, pad = shape
    torch.manual_seed(7)
    w = _bf(torch.randn(Ko, R, R, C, device=gpu) * 0.1)
    dy = _bf(torch.randn(N, H, W, Ko, device=gpu))
    add = _bf(torch.randn(N, H, W, C, device=gpu))
    keep = torch.rand(N, H, W, C, device=gpu) > 0.4
    bits = keep.reshape(-1, 8).to(torch.uint8) << torch.arange(8, device=gpu, dtype=torch.uint8)
    mask = bits.sum(1, dtype=torch.int32).to(torch.uint8).contiguous()
    add0 = add.clone()
    ref = torch.ops.tfx.conv_dgrad(dy, w, [N, H, W, C], st, pad, 1, None).float() + add.float() * keep
    dx = torch.ops.tfx.conv_dgrad(dy, w, [N, H, W, C], st, pad, 1, add, mask)
    assert dx.data_ptr() != add.data_ptr() and torch.equal(add, add0)
    assert _rel(dx, ref) < 1e-2
    # the BN-backward-fused data gradient takes the same masked addend
    xb = _bf(torch.randn(N, H, W, C, device=gpu))
    gamma, beta = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    ws = torch.zeros(64 * 2 * C + 64, device=gpu)
    _, save, _ = torch.ops.tfx.bn_fwd_train(xb, gamma, beta, None, None, 0.1, 1e-5, None, True, ws, False)
    dx2, red = torch.ops.tfx.conv_dgrad_bn(dy, w, [N, H, W, C], st, pad, 1, add, xb, save, None, True, ws,
                                           None, None, mask)
    assert _rel(dx2, ref) < 1e-2 and torch.equal(add, add0)
    _, _, red_ref = torch.ops.tfx.bn_bwd(dx2, xb, None, save, True, torch.zeros_like(ws), None, None, None)
    assert _rel(red, red_ref) < 1e-3


def test_image_normalize_matches_reference(gpu):
    """Fused input kernel == the PyTorch formulation of to_model_input (padded channels exactly 0)."""
    from tensorflow_examples_amd.models.resnet import to_model_input
    img = torch.randint(0, 256, (5, 32, 32, 3), dtype=torch.uint8)
    ref = to_model_input(img)  # CPU path
    out = to_model_input(img.to(gpu))
    assert out.shape == (5, 32, 32, 8) and out.dtype == torch.bfloat16
    assert torch.equal(out[..., 3:].cpu(), torch.zeros(5, 32, 32, 5, dtype=torch.bfloat16))
    assert (out.float().cpu() - ref.float()).abs().max().item() <= 0.02


def test_bn_bwd_without_dres(gpu):
    """want_dres=False: same dx / statistics, no residual-gradient tensor."""
    torch.manual_seed(8)
    M, C = 512, 64
    x = _bf(torch.randn(M, C, device=gpu))
    r = _bf(torch.randn(M, C, device=gpu))
    g = _bf(torch.randn(M, C, device=gpu))
    gamma, beta = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    ws = torch.zeros(64 * 2 * C, device=gpu)
    y, save, mask = torch.ops.tfx.bn_fwd_train(x, gamma, beta, None, None, 0.1, 1e-5, r, True, ws, False)
    dx1, dres1, red1 = torch.ops.tfx.bn_bwd(g, x, None, save, True, ws, None, None, mask)
    dx2, dres2, red2 = torch.ops.tfx.bn_bwd(g, x, None, save, True, ws, None, None, mask, False)
    assert dres1 is not None and dres2 is None
    assert torch.equal(dx1, dx2) and torch.allclose(red1, red2, rtol=1e-5, atol=1e-5)
    bx, bres = torch.ops.tfx.bn_bwd_apply(g, x, None, save, red1, True, mask, False)
    assert bres is None and _rel(bx, dx1) < 1e-3


FUSED_BN_SHAPES = [
    # N, H, W, C, Ko, R, stride, pad: 1x1 pointwise (dense loaders), 3x3 im2col, stride 2, ragged M
    (4, 8, 8, 64, 64, 1, 1, 0),
    (2, 8, 8, 64, 128, 3, 1, 1),
    (3, 9, 7, 32, 136, 3, 2, 1),
    (64, 16, 16, 64, 256, 1, 1, 0),  # many row tiles per column tile: the last-arriver path
]


@pytest.mark.parametrize("shape", FUSED_BN_SHAPES)
def test_conv_fwd_bn_finalize(gpu, shape):
    """conv_fwd_bn: the epilogue's last block per column tile finalizes the BN ([mean | invstd |
    scale | shift] + running stats) and leaves the workspace (slots + counters) zero."""
    N, H, W, C, Ko, R, st, pad = shape
    torch.manual_seed(5)
    x = _bf(torch.randn(N, H, W, C, device=gpu))
    w = _bf(torch.randn(Ko, R, R, C, device=gpu) * 0.1)
    gamma = torch.rand(Ko, device=gpu) + 0.5
    beta = torch.randn(Ko, device=gpu)
    rm, rv = torch.zeros(Ko, device=gpu), torch.ones(Ko, device=gpu)
    ws = torch.zeros(64 * 2 * Ko + 64, device=gpu)
    for it in range(2):  # twice: the counters must have been reset by the first launch
        y, save = torch.ops.tfx.conv_fwd_bn(x, w, st, pad, 1, ws, gamma, beta, rm, rv, 0.1, 1e-5)
        torch.cuda.synchronize()
        assert ws.abs().max().item() == 0.0, "workspace not restored to zero"
        assert _rel(y, torch.ops.tfx.conv_fwd(x, w, st, pad, 1)) < 1e-3
        yf = y.float().reshape(-1, Ko)
        mean, var = yf.mean(0), yf.var(0, unbiased=False)
        invstd = torch.rsqrt(var + 1e-5)
        assert torch.allclose(save[:Ko], mean, rtol=1e-4, atol=1e-4)
        assert torch.allclose(save[Ko:2 * Ko], invstd, rtol=1e-3, atol=1e-4)
        assert torch.allclose(save[2 * Ko:3 * Ko], gamma * invstd, rtol=1e-3, atol=1e-4)
        assert torch.allclose(save[3 * Ko:], beta - mean * gamma * invstd, rtol=1e-3, atol=1e-3)
    M = yf.shape[0]
    unb = var * M / (M - 1)
    assert torch.allclose(rm, 0.19 * mean, atol=1e-4, rtol=1e-3)  # two momentum-0.1 updates from 0
    assert torch.allclose(rv, 0.81 + 0.19 * unb, atol=1e-3, rtol=1e-3)
    # the BN apply over the conv's save == the unfused BN forward
    y1, _ = torch.ops.tfx.bn_apply_train(y, None, save, True)
    ws2 = torch.zeros(64 * 2 * Ko, device=gpu)
    y2, _, _ = torch.ops.tfx.bn_fwd_train(y, gamma, beta, None, None, 0.1, 1e-5, None, True, ws2, False)
    assert _rel(y1, y2) < 1e-2


@pytest.mark.parametrize("shape", [s for s in FUSED_BN_SHAPES if s[6] == 1])
@pytest.mark.parametrize("variant", ["relu", "res_mask", "plain", "addend"])
def test_conv_dgrad_bn_reduce(gpu, shape, variant):
    """conv_dgrad_bn: dx of the conv + the backward reduction of the BN that produced the conv's
    input (sum g', sum g' xhat, dgamma / dbeta), vs the unfused conv_dgrad -> bn_bwd."""
    N, H, W, C, Ko, R, st, pad = shape
    torch.manual_seed(6)
    xb = _bf(torch.randn(N, H, W, C, device=gpu) * 1.5 + 0.3)  # BN input
    res = _bf(torch.randn(N, H, W, C, device=gpu)) if variant == "res_mask" else None
    relu = variant != "plain"
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu)
    ws = torch.zeros(64 * 2 * C + 64, device=gpu)
    y, save, mask = torch.ops.tfx.bn_fwd_train(xb, gamma, beta, None, None, 0.1, 1e-5, res, relu, ws, False)
    if mask is not None and mask.numel() == 0:
        mask = None
    assert (mask is not None) == (variant == "res_mask")
    w = _bf(torch.randn(Ko, R, R, C, device=gpu) * 0.1)
    P = (H + 2 * pad - R) // st + 1
    Q = (W + 2 * pad - R) // st + 1
    dy = _bf(torch.randn(N, P, Q, Ko, device=gpu))
    add = _bf(torch.randn(N, H, W, C, device=gpu)) if variant == "addend" else None
    ref_dx = torch.ops.tfx.conv_dgrad(dy, w, list(y.shape), st, pad, 1, add.clone() if add is not None else None)
    wsr = torch.zeros(64 * 2 * C, device=gpu)
    dgr, dbr = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    ref_bx, ref_dres, ref_red = torch.ops.tfx.bn_bwd(ref_dx, xb, None if mask is not None else res, save, relu, wsr,
                                                     dgr, dbr, mask)
    dg, db = torch.ones(C, device=gpu), torch.zeros(C, device=gpu)
    for it in range(2):
        dx, red = torch.ops.tfx.conv_dgrad_bn(dy, w, list(y.shape), st, pad, 1,
                                              add.clone() if add is not None else None, xb, save, mask, relu, ws,
                                              dg, db)
        torch.cuda.synchronize()
        assert ws.abs().max().item() == 0.0, "workspace not restored to zero"
        assert _rel(dx, ref_dx) < 1e-3
        assert _rel(red, ref_red) < 1e-3
    assert _rel(dg - 1, 2 * dgr) < 1e-3 and _rel(db, 2 * dbr) < 1e-3  # accumulated in place, twice
    bx, dres = torch.ops.tfx.bn_bwd_apply(dx, xb, None if mask is not None else res, save, red, relu, mask)
    assert _rel(bx, ref_bx) < 1e-2
    if mask is not None:
        assert _rel(dres, ref_dres) < 1e-2


@pytest.mark.parametrize("B,I,O", [(256, 2048, 10), (100, 84, 10), (64, 520, 64)])
def test_linear_small_bwd(gpu, B, I, O):
    """Classifier-head backward in one launch: dx = g W, dW += g^T x, db += colsum(g)."""
    torch.manual_seed(41)
    g = _bf(torch.randn(B, O, device=gpu))
    x = _bf(torch.randn(B, I, device=gpu))
    w = _bf(torch.randn(O, I, device=gpu) * 0.1)
    dw = torch.ones(O, I, device=gpu)
    db = torch.ones(O, device=gpu)
    dx = torch.ops.tfx.linear_small_bwd(g, x, w, True, dw, db)
    assert _rel(dx, g.float() @ w.float()) < 1e-2
    assert _rel(dw - 1, g.float().t() @ x.float()) < 1e-3
    assert _rel(db - 1, g.float().sum(0)) < 1e-3


@pytest.mark.parametrize("shape", [(256, 32, 32, 64, 64, 1, 1), (256, 32, 32, 64, 64, 3, 1),
                                   (256, 16, 16, 128, 128, 3, 1), (256, 8, 8, 1024, 256, 1, 1),
                                   (256, 4, 4, 512, 2048, 1, 1), (256, 16, 16, 256, 256, 3, 2), (4, 5, 5, 24, 40, 3, 1)])
def test_conv_wgrad_slot_reduce_tail_blocks(gpu, shape):
    """conv_wgrad_sr: the weight gradient plus, in tail blocks of the same grid, another BN layer's
    backward slot reduction (red = slot sums, dgamma / dbeta +=, slots re-zeroed) -- every wgrad
    family (dense pair, im2col, transposed) at production shapes, vs conv_wgrad + a torch reduction."""
    N, H, W, C, K, R, st = shape
    pad = R // 2
    torch.manual_seed(23)
    x = _bf(torch.randn(N, H, W, C, device=gpu))
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    gy = _bf(torch.randn(N, P, Q, K, device=gpu))
    dw_ref = torch.zeros(K, R, R, C, device=gpu)
    torch.ops.tfx.conv_wgrad(gy, x, dw_ref, st, pad, 1, True)
    slots = torch.zeros(64 * 2 * C + 64, device=gpu)
    slots[: 64 * 2 * C] = torch.randn(64 * 2 * C, device=gpu)
    red_ref = slots[: 64 * 2 * C].view(64, 2, C).sum(0).reshape(-1)
    dg, db = torch.full((C,), 0.5, device=gpu), torch.full((C,), -0.25, device=gpu)
    dw = torch.zeros(K, R, R, C, device=gpu)
    red = torch.ops.tfx.conv_wgrad_sr(gy, x, dw, st, pad, 1, True, slots, dg, db)
    torch.cuda.synchronize()
    assert _rel(dw, dw_ref) < 1e-5
    assert torch.allclose(red, red_ref, rtol=1e-5, atol=1e-4)
    assert torch.allclose(db, red_ref[:C] - 0.25, rtol=1e-5, atol=1e-4)
    assert torch.allclose(dg, red_ref[C:] + 0.5, rtol=1e-5, atol=1e-4)
    assert slots.abs().max().item() == 0.0, "slots not re-zeroed"
    red2 = torch.ops.tfx.conv_wgrad_sr(gy, x, dw, st, pad, 1, True, slots, None, None)  # no parameter grads
    torch.cuda.synchronize()
    assert red2.abs().max().item() == 0.0 and _rel(dw, 2 * dw_ref) < 1e-5


@pytest.mark.parametrize("shape,C2", [((256, 16, 16, 128, 128, 3, 2), 512), ((256, 8, 8, 256, 1024, 1, 1), 1024),
                                      ((256, 4, 4, 512, 2048, 1, 1), 2048)])
def test_conv_wgrad_two_tail_reductions(gpu, shape, C2):
    """conv_wgrad_sr2: two BN layers' deferred slot reductions in one weight-gradient grid's tail
    (the conv's own input BN, and a pending one: a projection-shortcut BN), vs torch; plus the
    reduce-only BN backward (bn_bwd_reduce_into) and the standalone bn_slots_reduce it pairs with."""
    N, H, W, C, K, R, st = shape
    pad = R // 2
    torch.manual_seed(29)
    x = _bf(torch.randn(N, H, W, C, device=gpu))
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    gy = _bf(torch.randn(N, P, Q, K, device=gpu))
    dw_ref = torch.zeros(K, R, R, C, device=gpu)
    torch.ops.tfx.conv_wgrad(gy, x, dw_ref, st, pad, 1, True)
    # set 1: partials written by bn_bwd_reduce_into from a BN with ReLU (checked against bn_bwd's red)
    xb = _bf(torch.randn(N, H, W, C, device=gpu) + 0.2)
    gamma, beta = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    ws = torch.zeros(64 * 2 * C + 64, device=gpu)
    _, save, _ = torch.ops.tfx.bn_fwd_train(xb, gamma, beta, None, None, 0.1, 1e-5, None, True, ws, False)
    g = _bf(torch.randn(N, H, W, C, device=gpu))
    wsr = torch.zeros(64 * 2 * C, device=gpu)
    _, _, red_ref = torch.ops.tfx.bn_bwd(g, xb, None, save, True, wsr, None, None, None)
    slots1 = torch.zeros(64 * 2 * C + 64, device=gpu)
    torch.ops.tfx.bn_bwd_reduce_into(g, xb, save, True, None, slots1)
    # set 2: arbitrary partials
    slots2 = torch.zeros(64 * 2 * C2 + 64, device=gpu)
    slots2[: 64 * 2 * C2] = torch.randn(64 * 2 * C2, device=gpu)
    red2_ref = slots2[: 64 * 2 * C2].view(64, 2, C2).sum(0).reshape(-1)
    dg1, db1 = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
    dg2, db2 = torch.zeros(C2, device=gpu), torch.zeros(C2, device=gpu)
    dw = torch.zeros(K, R, R, C, device=gpu)
    r1, r2 = torch.ops.tfx.conv_wgrad_sr2(gy, x, dw, st, pad, 1, True, slots1, dg1, db1, slots2, C2, dg2, db2)
    torch.cuda.synchronize()
    assert _rel(dw, dw_ref) < 1e-5
    assert _rel(r1, red_ref) < 1e-4 and _rel(db1, red_ref[:C]) < 1e-4 and _rel(dg1, red_ref[C:]) < 1e-4
    assert torch.allclose(r2, red2_ref, rtol=1e-5, atol=1e-4)
    assert torch.allclose(db2, red2_ref[:C2], rtol=1e-5, atol=1e-4)
    assert slots1.abs().max().item() == 0.0 and slots2.abs().max().item() == 0.0
    # only the second set; then the standalone reduction
    slots2[: 64 * 2 * C2] = torch.randn(64 * 2 * C2, device=gpu)
    ref = slots2[: 64 * 2 * C2].view(64, 2, C2).sum(0).reshape(-1)
    r1b, r2b = torch.ops.tfx.conv_wgrad_sr2(gy, x, dw, st, pad, 1, True, None, None, None, slots2, C2, None, None)
    torch.cuda.synchronize()
    assert r1b.numel() == 0 and torch.allclose(r2b, ref, rtol=1e-5, atol=1e-4)
    slots2[: 64 * 2 * C2] = torch.randn(64 * 2 * C2, device=gpu)
    ref = slots2[: 64 * 2 * C2].view(64, 2, C2).sum(0).reshape(-1)
    r3 = torch.ops.tfx.bn_slots_reduce(slots2, C2, None, None)
    torch.cuda.synchronize()
    assert torch.allclose(r3, ref, rtol=1e-5, atol=1e-4) and slots2.abs().max().item() == 0.0
