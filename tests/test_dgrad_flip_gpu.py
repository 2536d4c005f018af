"""Stride-1 3x3 data gradient as the forward conv of dY with the flipped, transposed filter
(igemm_dgrad_flip.hip) and the one-launch refresh of every layer's flipped copy (wflip.hip):
bitwise copy against torch flip/permute, and the data gradient against the gathered kernel and an
fp32 PyTorch reference, plain, with an addend and with the fused BN-backward epilogue."""
import pytest
import torch
import torch.nn.functional as F

from tensorflow_examples_amd.variables import HeNormal, VariableStore

pytestmark = pytest.mark.gpu
NS = 64


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_wflip_store_refresh(gpu):
    st = VariableStore(device=gpu, compute_dtype=torch.bfloat16, seed=1)
    shapes = [(64, 3, 3, 64), (128, 3, 3, 64), (64, 1, 1, 64), (256, 3, 3, 512), (8, 3, 3, 8)]
    vs = [st.variable(list(s), HeNormal(), name=f"w{i}") for i, s in enumerate(shapes)]
    st.finalize()
    assert st.flip_index(vs[2]) is None and st.flip_index(vs[4]) is None  # 1x1; channels not % 64
    for v in (vs[0], vs[1], vs[3]):
        wf = st.flipped3x3(v)
        assert torch.equal(wf, v.value.flip(1, 2).permute(3, 1, 2, 0).contiguous())
    # weights change -> stale -> refreshed on the next request
    vs[3].assign(torch.randn(vs[3].shape))
    st.flip_stale = True
    assert torch.equal(st.flipped3x3(vs[3]), vs[3].value.flip(1, 2).permute(3, 1, 2, 0).contiguous())


@pytest.mark.parametrize("shape", [(256, 8, 8, 256), (4, 5, 7, 64), (2, 4, 4, 128)])
@pytest.mark.parametrize("mode", ["plain", "addend", "bn"])
def test_dgrad_flip_matches_gathered(gpu, shape, mode):
    torch.manual_seed(51)
    N, H, W, C = shape
    Ko = C
    dy = torch.randn(N, H, W, Ko, device=gpu).bfloat16()
    w = (torch.randn(Ko, 3, 3, C, device=gpu) * 0.05).bfloat16()
    wf = w.flip(1, 2).permute(3, 1, 2, 0).contiguous()
    ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1)
    ref = ref.permute(0, 2, 3, 1)
    if mode == "bn":
        xb = (torch.randn(N, H, W, C, device=gpu) + 0.2).bfloat16()
        save = torch.cat([torch.full((C,), 0.2), torch.ones(C), torch.full((C,), 1.3),
                          torch.full((C,), -0.1)]).to(gpu)

        def run(f):
            ws = torch.zeros(NS * 2 * C + 64, device=gpu)
            dg, db = torch.zeros(C, device=gpu), torch.zeros(C, device=gpu)
            dx, red = torch.ops.tfx.conv_dgrad_bn(dy, w, [N, H, W, C], 1, 1, 1, None, xb, save, None, True, ws, dg,
                                                  db, None, True, False, f)
            return dx, red, dg, db
        a, b = run(None), run(wf)
        torch.cuda.synchronize()
        assert _rel(b[0], ref) < 1e-2 and _rel(b[0], a[0]) < 1e-2
        for u, v in zip(a[1:], b[1:]):
            assert _rel(v, u) < 1e-3
        return
    add = torch.randn(N, H, W, C, device=gpu).bfloat16() if mode == "addend" else None
    a = torch.ops.tfx.conv_dgrad(dy, w, [N, H, W, C], 1, 1, 1, None if add is None else add.clone(), None, False,
                                 None)
    b = torch.ops.tfx.conv_dgrad(dy, w, [N, H, W, C], 1, 1, 1, None if add is None else add.clone(), None, False,
                                 wf)
    torch.cuda.synchronize()
    if add is not None:
        ref = ref + add.float()
    assert _rel(b, ref) < 1e-2 and _rel(b, a) < 1e-2
