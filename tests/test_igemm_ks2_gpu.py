"""In-block split-K (two 4-wave groups per 8-wave block, igemm_impl.h KS = 2) on the bf16-output
families with the fused-BN epilogues: forced launch configurations against the default
configuration and an fp32 PyTorch reference, at ResNet-50/CIFAR batch-256 production shapes.
Group 1 hands its accumulators over and exits; group 0 runs the statistics / BN-backward epilogue."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

FAM_FWD_PW, FAM_FWD_X, FAM_DGRAD_PW, FAM_DGRAD_X = 0, 1, 2, 3
NS = 64


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture
def unforce():
    yield
    torch.ops.tfx.igemm_tune_force(-1, 0, 0, -1, 0)


@pytest.mark.parametrize("cfg", [(1, 2, 0, 0), (1, 2, 2, 0), (2, 2, 0, 0), (2, 2, 2, 0)])
@pytest.mark.parametrize("shape", [(256, 8, 8, 256, 256, 3), (256, 4, 4, 512, 512, 3), (256, 8, 8, 1024, 256, 1)])
def test_fwd_stats_ks2(gpu, unforce, cfg, shape):
    torch.manual_seed(21)
    N, H, W, C, K, R = shape
    pad = R // 2
    x = torch.randn(N, H, W, C, device=gpu).bfloat16()
    w = (torch.randn(K, R, R, C, device=gpu) * 0.05).bfloat16()
    s0 = torch.zeros(NS * 2 * K + 64, device=gpu)
    y0 = torch.ops.tfx.conv_fwd_stats(x, w, 1, pad, 1, s0)
    torch.ops.tfx.igemm_tune_force(FAM_FWD_X if R > 1 else FAM_FWD_PW, *cfg)
    s1 = torch.zeros_like(s0)
    y1 = torch.ops.tfx.conv_fwd_stats(x, w, 1, pad, 1, s1)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=pad).permute(0, 2, 3, 1)
    assert _rel(y1, ref) < 1e-2
    assert _rel(y1, y0) < 1e-2
    tot0 = s0[: NS * 2 * K].view(NS, 2, K).sum(0)
    tot1 = s1[: NS * 2 * K].view(NS, 2, K).sum(0)
    assert _rel(tot1, tot0) < 1e-3


@pytest.mark.parametrize("cfg", [(1, 2, 0, 0), (1, 2, 2, 0), (2, 2, 2, 0)])
@pytest.mark.parametrize("shape,addend", [((256, 8, 8, 256, 256, 3), False), ((256, 8, 8, 256, 1024, 1), True),
                                          ((256, 4, 4, 512, 2048, 1), False)])
def test_dgrad_bn_ks2(gpu, unforce, cfg, shape, addend):
    torch.manual_seed(22)
    N, H, W, C, K, R = shape
    pad = R // 2
    dy = torch.randn(N, H, W, K, device=gpu).bfloat16()
    w = (torch.randn(K, R, R, C, device=gpu) * 0.05).bfloat16()
    xb = (torch.randn(N, H, W, C, device=gpu) + 0.2).bfloat16()
    save = torch.cat([torch.full((C,), 0.2), torch.ones(C), torch.full((C,), 1.3), torch.full((C,), -0.1)]).to(gpu)
    add = torch.randn(N, H, W, C, device=gpu).bfloat16() if addend else None
    amask = torch.randint(0, 256, (N * H * W * C // 8,), device=gpu, dtype=torch.uint8) if addend else None

    def run():
        ws = torch.zeros(NS * 2 * C + 64, device=gpu)
        dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
        dx, red = torch.ops.tfx.conv_dgrad_bn(dy, w, [N, H, W, C], 1, pad, 1, add, xb, save, None, True, ws, dg, db,
                                              amask)
        return dx, red, dg, db

    dx0, red0, dg0, db0 = run()
    torch.ops.tfx.igemm_tune_force(FAM_DGRAD_X if R > 1 else FAM_DGRAD_PW, *cfg)
    dx1, red1, dg1, db1 = run()
    torch.cuda.synchronize()
    assert _rel(dx1, dx0) < 1e-2
    assert _rel(red1, red0) < 1e-3
    assert _rel(dg1, dg0) < 1e-3 and _rel(db1, db0) < 1e-3
