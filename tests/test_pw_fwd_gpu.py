"""Fused block tail + next squeezing 1x1 conv forward (csrc/kernels/pw_fwd.hip): the kernel against
the layer-wise pair (bn_apply + conv_fwd_bn) and an fp32 PyTorch reference, and the whole ResNet-50
first step with the deferred tails on vs off."""
import pytest
import torch

from tensorflow_examples_amd.models.resnet import build_resnet_cifar, to_model_input

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("shape", [(256, 32, 32), (256, 16, 16), (4, 8, 8), (3, 4, 8), (1, 1, 16)])
@pytest.mark.parametrize("ci,co", [(256, 64), (256, 128), (512, 128)])
@pytest.mark.parametrize("rbn", [False, True])
def test_pw_fwd_squeeze_matches_layerwise(gpu, shape, ci, co, rbn):
    N, H, W = shape
    CI, M = ci, N * H * W
    if not torch.ops.tfx.pw_fwd_squeeze_supported(CI, co, M):
        pytest.skip("rows not a multiple of the m-tile")
    torch.manual_seed(11)
    y3 = _bf(torch.randn(N, H, W, CI, device=gpu) * 1.2 + 0.1)
    res = _bf(torch.randn(N, H, W, CI, device=gpu) * 0.8 - 0.2)
    g3, b3 = torch.rand(CI, device=gpu) + 0.5, torch.randn(CI, device=gpu) * 0.3
    ws3 = torch.zeros(64 * 2 * CI, device=gpu)
    _, save3, _ = torch.ops.tfx.bn_fwd_train(y3, g3, b3, None, None, 0.1, 1e-5, None, False, ws3, False)
    save_r = None
    if rbn:  # the residual is a shortcut BN's (never written) output: res = its input
        gr, br = torch.rand(CI, device=gpu) + 0.5, torch.randn(CI, device=gpu) * 0.3
        wsr = torch.zeros(64 * 2 * CI, device=gpu)
        _, save_r, _ = torch.ops.tfx.bn_fwd_train(res, gr, br, None, None, 0.1, 1e-5, None, False, wsr, False)
    w1 = _bf(torch.randn(co, 1, 1, CI, device=gpu) * 0.06)
    gam1, bet1 = torch.rand(co, device=gpu) + 0.5, torch.randn(co, device=gpu) * 0.2

    # layer-wise: tail apply, then conv1 with the fused BN1 statistics + finalize
    if rbn:
        out_ref, mask_ref = torch.ops.tfx.bn_apply_res_bn(y3, res, save3, save_r, True)
    else:
        out_ref, mask_ref = torch.ops.tfx.bn_apply_train(y3, res, save3, True)
    ws1a = torch.zeros(64 * 2 * co, device=gpu)
    rm_a, rv_a = torch.zeros(co, device=gpu), torch.ones(co, device=gpu)
    y1_ref, save1_ref = torch.ops.tfx.conv_fwd_bn(out_ref, w1, 1, 0, 1, ws1a, gam1, bet1, rm_a, rv_a, 0.1, 1e-5)

    out = torch.empty_like(y3)
    mask = torch.empty(M * CI // 8, dtype=torch.uint8, device=gpu)
    ws1 = torch.zeros(64 * 2 * co, device=gpu)
    rm, rv = torch.zeros(co, device=gpu), torch.ones(co, device=gpu)
    y1, save1 = torch.ops.tfx.pw_fwd_squeeze(y3, save3, res, save_r, w1, out, mask, ws1, gam1, bet1, rm, rv,
                                             0.1, 1e-5)
    torch.cuda.synchronize()
    # the tail: bit-identical to the apply pass
    assert torch.equal(out, out_ref)
    assert torch.equal(mask, mask_ref.reshape(-1))
    # conv1 vs fp32 PyTorch on the same bf16 input, and vs the layer-wise kernel
    ref = out.float().reshape(M, CI) @ w1.float().reshape(co, CI).t()
    assert _rel(y1.reshape(M, co), ref) < 8e-3
    assert _rel(y1, y1_ref) < 8e-3
    assert ws1.abs().max().item() == 0.0, "BN1 slots not restored to zero"
    y1f = y1.float().reshape(M, co)
    mean, var = y1f.mean(0), y1f.var(0, unbiased=False)
    assert torch.allclose(save1[:co], mean, rtol=1e-3, atol=1e-3)
    assert torch.allclose(save1[co:2 * co], torch.rsqrt(var + 1e-5), rtol=2e-3, atol=1e-3)
    assert torch.allclose(rm, rm_a, rtol=1e-3, atol=1e-4) and torch.allclose(rv, rv_a, rtol=1e-3, atol=1e-4)


def test_resnet50_deferred_tails_match_layerwise(gpu):
    """ResNet-50 first step: stage-1/2 tails applied inside the next conv1 (pw_fwd_squeeze) vs their own
    apply pass, in the deterministic-reduction mode: the same loss bits and every variable within the
    fixed gate (det_util.DET_TOL); the fused kernel's tail output scaled by 0.95 must fail it."""
    from det_util import assert_gate_catches, assert_within_gate, scaled_output
    from tensorflow_examples_amd import ops
    from tensorflow_examples_amd.ops import nn as nnops

    g = torch.Generator().manual_seed(9)
    img = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, generator=g)
    lab = torch.randint(0, 10, (32,), generator=g).to(gpu)
    xin = to_model_input(img.to(gpu))

    def run():
        st, m = build_resnet_cifar(device=gpu, depth=50, dtype=torch.bfloat16, seed=4)
        st.zero_grad()
        loss = ops.softmax_cross_entropy(m(xin, training=True), lab)
        loss.backward()
        torch.cuda.synchronize()
        return float(loss.detach()), st.grad.clone(), st

    from tensorflow_examples_amd.ops import fusion
    with fusion.override(), ops.deterministic():  # the default knobs, restored after
        n0 = nnops.PW_SQUEEZE_CALLS[0]
        l0, g0, st = run()
        assert nnops.PW_SQUEEZE_CALLS[0] - n0 == 6, "stage-1 and stage-2 tails fused into the next conv1 (3 + 3 boundaries)"
        with fusion.override(defer_tail=False):
            l2, g2, _ = run()
        # negative control: the tail output the fused kernel writes (its `out` argument) x0.95
        with scaled_output("pw_fwd_squeeze", lambda a, o: [a[5]]):
            ln, gn, _ = run()
    assert l0 == l2, (l0, l2)
    assert ln != l0
    assert_within_gate(g0, g2, st, "defer_tail off")
    assert_gate_catches(g0, gn, st, "fused tail output x0.95")
