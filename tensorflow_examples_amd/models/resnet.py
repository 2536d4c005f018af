"""ResNet for CIFAR-10 (north-star config 3 of BASELINE.json: ResNet-50/CIFAR-10 bf16 DP).

CIFAR adaptation of ResNet-50 v1.5: 3x3 stride-1 stem (no max-pool), bottleneck stages
[3, 4, 6, 3] with widths 64/128/256/512 (x4 expansion), stride on the 3x3 conv, 1x1
projection shortcuts, global average pool, FC 2048 -> 10.  23.5 M parameters.

MI355X layout: activations NHWC bf16 end to end, conv weights [Ko][R][S][C] so every conv
is an implicit GEMM with the channel axis contiguous (csrc/kernels/igemm.hip); each BN
pass fuses ReLU and, at a block's tail, the residual add (csrc/kernels/batchnorm.hip).
The 3-channel RGB input is carried as 8 channels (zeros in 3..7) so the stem conv meets
the 16-byte vector-load granularity; its weights for channels 3..7 stay exactly zero.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from .. import ops
from ..ops import _native, fusion
from ..ops.nn import BNWorkspace
from ..variables import Constant, HeNormal, VariableStore, Zeros

STAGES = {
    18: ("basic", [2, 2, 2, 2]),
    34: ("basic", [3, 4, 6, 3]),
    50: ("bottleneck", [3, 4, 6, 3]),
    101: ("bottleneck", [3, 4, 23, 3]),
    152: ("bottleneck", [3, 8, 36, 3]),
}
IN_CH_PAD = 8
_MEAN = (0.4914, 0.4822, 0.4465)  # CIFAR-10 per-channel statistics
_STD = (0.2470, 0.2435, 0.2616)
# GPU training fusions (each measured as an interleaved A/B when introduced, README ledger), read
# from the fusion config (ops/fusion.py knobs): the residual-gradient sum in conv1's data-gradient
# epilogue (GradSink, "sink"); the conv<->BN epilogue fusions (BN statistics in the producing conv's
# epilogue, BN backward reduction in the consuming conv's data-gradient epilogue: igemm.hip
# EPI_STATS / EPI_BNB, "fuse_bn"); identity blocks hand conv1 the residual BN's (gradient, ReLU mask)
# instead of the masked gradient tensor ("masked_res"); a 1x1 stride-2 projection parks its input
# gradient compact (even pixels only) for conv1's epilogue to add ("s2_addend").  Which kernel each
# layer runs is the model's fusion plan (ResNetCifar.plan_for, fusion.plan_resnet).


class _BN:
    def __init__(self, store: VariableStore, c: int, name: str, zero_gamma: bool = False):
        with store.scope(name):
            self.gamma = store.variable([c], Constant(0.0 if zero_gamma else 1.0), name="gamma")
            self.beta = store.variable([c], Zeros(), name="beta")
            self.mean = store.add_state("moving_mean", torch.zeros(c))
            self.var = store.add_state("moving_variance", torch.ones(c))
        self.ws = BNWorkspace(c, store)

    def __call__(self, x, training, relu=False, residual=None, stats_ready=False, residual_sink=None, ws_obj=False,
                 residual_is_bn=False, defer_output=False, lazy_backward=False, defer_apply=False):
        ws = (self.ws if ws_obj else self.ws.get(x.device)) if x.device.type == "cuda" else None
        return ops.batch_norm(x, self.gamma, self.beta, self.mean, self.var, training=training, momentum=0.1,
                              eps=1e-5, residual=residual, relu=relu, workspace=ws, stats_ready=stats_ready,
                              residual_grad_sink=residual_sink, fuse_residual_bn_backward=residual_is_bn,
                              defer_output=defer_output, lazy_backward=lazy_backward, defer_apply=defer_apply)

    def after_conv(self, conv, x, training, relu=False, residual=None, sink=None, residual_sink=None,
                   fuse_input_bn_backward=False, residual_is_bn=False, defer_output=False, defer_apply=False):
        """conv -> BN with the BN statistics produced (and, with knob fuse_bn, finalized) by the conv's
        epilogue (GPU, training).  ``fuse_input_bn_backward``: the conv's data gradient is the
        complete gradient of ``x`` -- reduce x's producing BN's backward in its epilogue.  The BN's
        input gradient may reach ``conv`` unmaterialised (ops.nn.LazyBNGrad): it is its only producer.
        ``defer_apply``: the output's first reader is the next bottleneck's conv1, which applies this
        (tail) BN while loading it (ops.nn.TailPending)."""
        fused = training and x.device.type == "cuda"
        if fused and fusion.knob("fuse_bn"):
            self.ws.finalize_args = (self.gamma.master, self.beta.master, self.mean, self.var, 0.1, 1e-5)
            y = conv(x, self.ws, sink, fuse_input_bn_backward and fusion.knob("fuse_bn"))
            return self(y, training, relu=relu, residual=residual, stats_ready=True, residual_sink=residual_sink,
                        ws_obj=True, residual_is_bn=residual_is_bn, defer_output=defer_output, lazy_backward=True,
                        defer_apply=defer_apply)
        y = conv(x, self.ws.get(x.device) if fused else None, sink)
        return self(y, training, relu=relu, residual=residual, stats_ready=fused, residual_sink=residual_sink,
                    residual_is_bn=residual_is_bn)


class _Conv:
    def __init__(self, store: VariableStore, cin: int, cout: int, k: int, stride: int, name: str):
        self.w = store.variable([cout, k, k, cin], HeNormal(), name=name)
        self.stride, self.pad = stride, k // 2

    def __call__(self, x, bn_stats_into=None, grad_sink=None, fuse_input_bn_backward=False):
        return ops.conv2d(x, self.w, self.stride, self.pad, bn_stats_into=bn_stats_into, grad_sink=grad_sink,
                          fuse_input_bn_backward=fuse_input_bn_backward)


class Bottleneck:
    expansion = 4

    def __init__(self, store, cin, width, stride, name, zero_init_residual=False):
        cout = width * 4
        with store.scope(name):
            self.c1 = _Conv(store, cin, width, 1, 1, "conv1")
            self.b1 = _BN(store, width, "bn1")
            self.c2 = _Conv(store, width, width, 3, stride, "conv2")
            self.b2 = _BN(store, width, "bn2")
            self.c3 = _Conv(store, width, cout, 1, 1, "conv3")
            self.b3 = _BN(store, cout, "bn3", zero_gamma=zero_init_residual)
            self.proj = None
            if stride != 1 or cin != cout:
                self.proj = _Conv(store, cin, cout, 1, stride, "shortcut")
                self.bp = _BN(store, cout, "shortcut_bn")

    def __call__(self, x, training, defer_tail=False):
        # defer_tail: the output feeds the next bottleneck, whose conv1 runs first -- that conv applies
        # this block's tail BN while loading its input (pw_fwd.hip)
        # x feeds conv1 and the shortcut: the shortcut's input-gradient is folded into conv1's
        # dgrad epilogue (GradSink) instead of an autograd add kernel
        gpu_train = training and x.device.type == "cuda"
        prod, cons = ops.GradSink.pair() if (gpu_train and fusion.knob("sink")) else (None, None)
        if prod is not None and fusion.knob("masked_res"):
            prod.accept_masked = True  # conv1 (1x1, stride 1) applies the residual ReLU mask itself
        if prod is not None and fusion.knob("s2_addend"):
            prod.accept_s2 = True  # ... and a 1x1 stride-2 projection's compact gradient
        # conv1 is x's last consumer in backward only when the GradSink carries the other branch
        # BN1's apply is left to conv2 (a stage-1 3x3 conv applies it on load: conv3x3_fused.hip)
        o = self.b1.after_conv(self.c1, x, training, relu=True, sink=cons, fuse_input_bn_backward=cons is not None,
                               defer_apply=True)
        # BN2's apply is left to conv3 too (a single-k-tile 1x1 conv applies it on load; else materialised)
        o = self.b2.after_conv(self.c2, o, training, relu=True, fuse_input_bn_backward=True, defer_apply=True)
        o3_fuse = True
        if self.proj is None:
            return self.b3.after_conv(self.c3, o, training, relu=True, residual=x, residual_sink=prod,
                                      fuse_input_bn_backward=o3_fuse, defer_apply=defer_tail)
        # sc (the shortcut BN's output) is used only as the tail's residual: never written (the tail
        # normalizes the shortcut conv's output on the fly), and its BN backward rides along
        sc = self.bp.after_conv(self.proj, x, training, sink=prod, defer_output=True)
        return self.b3.after_conv(self.c3, o, training, relu=True, residual=sc, fuse_input_bn_backward=o3_fuse,
                                  residual_is_bn=True, defer_apply=defer_tail)


class Basic:
    expansion = 1

    def __init__(self, store, cin, width, stride, name, zero_init_residual=False):
        with store.scope(name):
            self.c1 = _Conv(store, cin, width, 3, stride, "conv1")
            self.b1 = _BN(store, width, "bn1")
            self.c2 = _Conv(store, width, width, 3, 1, "conv2")
            self.b2 = _BN(store, width, "bn2", zero_gamma=zero_init_residual)
            self.proj = None
            if stride != 1 or cin != width:
                self.proj = _Conv(store, cin, width, 1, stride, "shortcut")
                self.bp = _BN(store, width, "shortcut_bn")

    def __call__(self, x, training):
        gpu_train = training and x.device.type == "cuda"
        prod, cons = ops.GradSink.pair() if (gpu_train and fusion.knob("sink")) else (None, None)
        if prod is not None and fusion.knob("masked_res") and self.c1.stride == 1:
            prod.accept_masked = True
        o = self.b1.after_conv(self.c1, x, training, relu=True, sink=cons)
        if self.proj is None:
            return self.b2.after_conv(self.c2, o, training, relu=True, residual=x, residual_sink=prod)
        sc = self.bp.after_conv(self.proj, x, training, sink=prod, defer_output=True)
        return self.b2.after_conv(self.c2, o, training, relu=True, residual=sc, residual_is_bn=True)


_ENV_APPLIED = False


class ResNetCifar:
    def __init__(self, store: VariableStore, depth: int = 50, num_classes: int = 10, base_width: int = 64,
                 zero_init_residual: bool = False, plan_batch: int = 256):
        """``zero_init_residual``: the last BN of every residual branch starts with gamma = 0, so each block
        is the identity (plus its shortcut) at init -- the well-conditioned start of Goyal et al.'s large-batch
        recipe; without it the randomly initialised 50-layer net is ill-conditioned at lr 0.1 and 3-epoch runs
        end anywhere between 42 % and 99 % (profiles/r04_conv).  Off by default: the kernel / gradient tests
        compare every layer's gradient, which zero gammas would make zero inside the blocks."""
        global _ENV_APPLIED
        if not _ENV_APPLIED:  # TFX_FUSION profile (ops/fusion.py), once per process
            _ENV_APPLIED = True
            fusion.apply_env()
        kind, blocks = STAGES[depth]
        Block = Bottleneck if kind == "bottleneck" else Basic
        self.store = store
        with store.scope("resnet%d" % depth):
            self.stem = _Conv(store, IN_CH_PAD, base_width, 3, 1, "conv0")
            self.stem_bn = _BN(store, base_width, "bn0")
            self.blocks: List = []
            cin = base_width
            for si, n in enumerate(blocks):
                width = base_width * (2 ** si)
                for bi in range(n):
                    stride = 2 if (bi == 0 and si > 0) else 1
                    blk = Block(store, cin, width, stride, "stage%d_block%d" % (si + 1, bi + 1),
                                zero_init_residual=zero_init_residual)
                    self.blocks.append(blk)
                    cin = width * Block.expansion
            with store.scope("fc"):
                self.fc_w = store.variable([num_classes, cin], HeNormal(gain=1.0), name="kernel")
                self.fc_b = store.variable([num_classes], Zeros(), name="bias")
        self.num_classes = num_classes
        self.feat = cin
        self._plans = {}
        # the fusion plan of a training step, built with the model for the bench batch at CIFAR size
        # (GPU stores); other batch sizes get theirs on first use (plan_for)
        self.fusion_plan = self.plan_for(plan_batch) if str(store.device).startswith("cuda") else None

    def plan_for(self, batch: int, hw: Tuple[int, int] = (32, 32)) -> Optional["fusion.FusionPlan"]:
        """The fusion plan (ops/fusion.py) of a training step at ``batch`` images of ``hw``, for the
        current fusion config; None where the native library (whose kernel-support predicates the
        planner asks) is absent."""
        key = (int(batch), tuple(hw), fusion.CONFIG.signature)
        plan = self._plans.get(key)
        if plan is None:
            if not _native.load():
                return None
            plan = self._plans[key] = fusion.plan_resnet(self, int(batch), tuple(hw))
        return plan

    def post_init(self):
        """Zero the stem weights of the padded input channels (3..7)."""
        with torch.no_grad():
            self.stem.w.master[..., 3:] = 0
        self.store.refresh_shadow()

    def features(self, x: torch.Tensor, training: bool = True, defer_last: bool = False) -> torch.Tensor:
        """Stem and residual stages: the NHWC input of the classifier head.  ``defer_last``: the caller's
        head applies the last block's tail BN itself (ops.classifier_head_xent); anything else that reads
        the output first materialises it (ops.nn.TailPending).  A GPU training step runs under this
        batch's fusion plan: the ops consult its per-layer entries (fusion.layer_plan)."""
        native = training and x.is_cuda and _native.use_native(x)
        self.store.fusion_plan = self.plan_for(x.shape[0], tuple(x.shape[1:3])) if native else None
        o = self.stem_bn.after_conv(self.stem, x, training, relu=True)
        for i, blk in enumerate(self.blocks):
            if isinstance(blk, Bottleneck):
                nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
                o = blk(o, training, defer_tail=isinstance(nxt, Bottleneck) or (nxt is None and defer_last))
            else:
                o = blk(o, training)
        return o

    def __call__(self, x: torch.Tensor, training: bool = True) -> torch.Tensor:
        f = ops.global_avg_pool(self.features(x, training))
        return ops.linear(f, self.fc_w, self.fc_b)

    def training_loss(self, x: torch.Tensor, labels: torch.Tensor, naive: bool = False,
                      unit_seed: bool = False) -> torch.Tensor:
        """Mean softmax cross-entropy of a training forward; the head (pool, FC, loss and, for a unit
        seed, its input gradient) is one launch on the GPU (ops.classifier_head_xent)."""
        return ops.classifier_head_xent(self.features(x, True, defer_last=True), self.fc_w, self.fc_b, labels,
                                        naive=naive, unit_seed=unit_seed)


def build_resnet_cifar(device="cuda", depth=50, num_classes=10, dtype=torch.bfloat16, seed=0,
                       zero_init_residual: bool = False) -> Tuple[VariableStore, ResNetCifar]:
    store = VariableStore(device=device, compute_dtype=dtype, seed=seed)
    model = ResNetCifar(store, depth=depth, num_classes=num_classes, zero_init_residual=zero_init_residual)
    store.finalize()
    model.post_init()
    return store, model


def to_model_batch(images: torch.Tensor, labels: torch.Tensor, dtype=torch.bfloat16, device=None,
                   out: Optional[torch.Tensor] = None, labels_out: Optional[torch.Tensor] = None):
    """(images, labels) -> (model input, device labels).  With both static buffers (a captured step's
    :meth:`ClassifierTrainer.input_buffer` / :meth:`label_buffer`) and uint8 images on the GPU or in
    pinned host memory, the one input kernel writes both (no separate label copy launch); otherwise
    :func:`to_model_input` plus a label copy."""
    if out is not None and labels_out is not None and images.dtype == torch.uint8 and out.is_cuda and \
            out.dtype == torch.bfloat16 and labels.dtype == torch.int64 and labels_out.is_cuda and \
            (images.is_cuda or images.is_pinned()) and (labels.is_cuda or labels.is_pinned()) and \
            _native.use_native_device(out.device):
        torch.ops.tfx.image_normalize_into(images.contiguous(), list(_MEAN), list(_STD), out, labels.contiguous(),
                                           labels_out)
        return out, labels_out
    x = to_model_input(images, dtype=dtype, device=device, out=out)
    dev = torch.device(device) if device is not None else x.device
    y = labels.to(dev, non_blocking=True) if labels.device != dev else labels
    return x, y


def to_model_input(images_nhwc_u8_or_f: torch.Tensor, dtype=torch.bfloat16, device=None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[N,32,32,3] images -> [N,32,32,8] normalised NHWC compute tensor (channels 3..7 zero).
    GPU uint8 input: one fused HIP kernel (csrc/kernels/image.hip).  A pinned host uint8 batch with
    ``device`` = a GPU: the same kernel reads it over the host link (zero-copy input).  ``out``: a bf16
    GPU tensor of the output shape to write into (e.g. a captured graph's static input buffer)."""
    x = images_nhwc_u8_or_f
    if out is not None and x.dtype == torch.uint8 and out.is_cuda and out.dtype == torch.bfloat16 and \
            (x.is_cuda or x.is_pinned()) and _native.use_native_device(out.device):
        torch.ops.tfx.image_normalize_into(x.contiguous(), list(_MEAN), list(_STD), out, None, None)
        return out
    if x.dtype == torch.uint8 and dtype == torch.bfloat16 and x.device.type == "cuda" and _native.use_native(x):
        return torch.ops.tfx.image_normalize(x.contiguous(), list(_MEAN), list(_STD), IN_CH_PAD)
    if device is not None and torch.device(device).type == "cuda" and x.device.type == "cpu" and \
            x.dtype == torch.uint8 and dtype == torch.bfloat16 and x.is_pinned():
        # zero-copy input: the kernel reads the pinned host batch directly (no H2D staging copy)
        out = torch.empty((*x.shape[:-1], IN_CH_PAD), dtype=dtype, device=device)
        torch.ops.tfx.image_normalize_into(x.contiguous(), list(_MEAN), list(_STD), out, None, None)
        return out
    if x.dtype == torch.uint8:
        x = x.float() / 255.0
    mean = torch.tensor(_MEAN, device=x.device)
    std = torch.tensor(_STD, device=x.device)
    x = (x - mean) / std
    out = torch.zeros(*x.shape[:-1], IN_CH_PAD, device=x.device, dtype=dtype)
    out[..., :3] = x.to(dtype)
    return out
