"""The cross-op fusion plan of the GPU training path: named fusion groups, one switch each, and a
recorder that reports which group took which layer and on which kernel.

The reference builds its model op by op and runs it unfused (R/distributed/distributed.py:94-108,
SURVEY §2.7).  Here the ResNet step fuses across op and layer boundaries; every fusion is a named
GROUP with a kernel and a fallback (the layer-wise path that runs when the group is off or a shape
is unsupported):

=====================  ==========================================================  ===============================
group                  what it fuses (kernel)                                        fallback
=====================  ==========================================================  ===============================
bn_epilogue            BN statistics + finalize in the producing conv's epilogue;   bn_fwd_train / bn_bwd passes
                       BN-backward partials in the consuming dgrad's epilogue
                       (igemm EPI_STATS / EPI_BNB)
grad_sink              residual-branch gradient sum in conv1's dgrad epilogue       autograd add
masked_res             residual ReLU mask applied by that epilogue (no masked g)     masked gradient tensor
s2_addend              stride-2 projection gradient added compact (even pixels)     zero-filled full-size addend
deferred_slot_reduce   BN-backward slot reductions in weight-gradient tail blocks   bn_slot_reduce launches
block_boundary_fwd     tail BN apply + next conv1 in one launch (pw_fwd_squeeze)    bn_apply + conv
bn_on_load             plain ReLU BN applied by its 3x3 / single-k-tile 1x1          bn_apply pass
                       consumer (conv3x3_fwd_fused, igemm a_scale)
lazy_bn_bwd            BN backward apply formed by the producer conv's backward     bn_bwd_apply pass
                       (pw_bwd_expand / pw_bwd_squeeze / conv3x3_bwd_fused)
conv3_fused_bwd        stage-1 3x3 conv backward in one launch (conv3x3_bwd_fused)  dgrad + wgrad launches
stem_kernels           CIFAR stem forward / weight gradient (stem.hip)              generic implicit GEMM
fused_head             pool + FC + softmax-xent + input gradient (head.hip)         three composed ops
head_tail              last tail BN applied inside the fused head (TAIL mode)       bn_apply before the head
bn_finalize_fold       stage 2-4 BN finalize inside the layer-wise apply: every     bn_finalize launch after the
                       block reduces the conv epilogue's few statistics rows         conv (conv_fwd_bn)
                       itself (bn_apply_fin); the rows live in the store's
                       gradient scratch, re-zeroed by VariableStore.zero_grad
=====================  ==========================================================  ===============================

``TFX_FUSION`` selects a profile at import: ``all`` (default: every group but the opt-in
``bn_finalize_fold``), ``r2`` (the round-2 level: epilogue
fusions only, no cross-layer kernels), ``none`` (layer-wise), or a comma list of ``-group`` /
``+group`` edits applied to ``all`` (e.g. ``-head_tail,-bn_on_load``).  :func:`set_groups` switches
them at run time (tests, A/B runs); :class:`record` collects what one traced step actually ran.
"""
from __future__ import annotations

import os
from collections import Counter, OrderedDict
from typing import Dict, Iterable, List, Optional, Tuple

GROUPS = ("bn_epilogue", "grad_sink", "masked_res", "s2_addend", "deferred_slot_reduce", "block_boundary_fwd",
          "bn_on_load", "lazy_bn_bwd", "conv3_fused_bwd", "stem_kernels", "fused_head", "head_tail",
          "bn_finalize_fold")
# bn_finalize_fold is opt-in (``TFX_FUSION=+bn_finalize_fold``): measured neutral, profiles/r04_fold
PROFILES = {
    "all": set(GROUPS) - {"bn_finalize_fold"},
    "r2": {"bn_epilogue", "grad_sink", "masked_res", "s2_addend", "deferred_slot_reduce", "fused_head"},
    "none": set(),
}


def _bind() -> Dict[str, List[Tuple[object, str]]]:
    """group -> the module switches that implement it (imported lazily: no import cycle)."""
    from . import nn
    from ..models import resnet
    return {
        "bn_epilogue": [(resnet, "_FUSE_BN")],
        "grad_sink": [(resnet, "_SINK")],
        "masked_res": [(resnet, "_MASKED_RES")],
        "s2_addend": [(resnet, "_S2_ADDEND")],
        "deferred_slot_reduce": [(nn, "_SR_TAKE_PENDING"), (nn, "_SR_DEFER")],
        "block_boundary_fwd": [(nn, "_DEFER_TAIL")],
        "bn_on_load": [(nn, "_DEFER_BN_IN"), (nn, "_BN_ON_LOAD_1X1")],
        "lazy_bn_bwd": [(nn, "_LAZY_BN_BWD")],
        "conv3_fused_bwd": [(nn, "_FUSE_CONV3_BWD")],
        "stem_kernels": [(nn, "_STEM_WGRAD")],
        "fused_head": [(nn, "_FUSE_HEAD")],
        "head_tail": [(nn, "_HEAD_TAIL")],
        "bn_finalize_fold": [(nn, "_FOLD_FIN")],
    }


def parse_profile(spec: str) -> set:
    spec = (spec or "all").strip()
    if spec in PROFILES:
        return set(PROFILES[spec])
    on = set(PROFILES["all"])
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok:
            continue
        name = tok.lstrip("+-")
        if name not in GROUPS:
            raise ValueError("TFX_FUSION: unknown fusion group %r (groups: %s)" % (name, ", ".join(GROUPS)))
        (on.discard if tok.startswith("-") else on.add)(name)
    return on


def enabled() -> Dict[str, bool]:
    b = _bind()
    return {g: all(bool(getattr(m, a)) for m, a in b[g]) for g in GROUPS}


def set_groups(on: Iterable[str]) -> Dict[str, bool]:
    """Enable exactly the groups in ``on``; returns the previous state (pass it to :func:`restore`)."""
    prev = enabled()
    on = set(on)
    for g, sw in _bind().items():
        for m, a in sw:
            setattr(m, a, g in on)
    _stem_fwd("stem_kernels" in on)
    return prev


def restore(state: Dict[str, bool]) -> None:
    set_groups([g for g, v in state.items() if v])


def _stem_fwd(on: bool) -> None:
    try:
        import torch
        from . import _native
        if _native.load():
            torch.ops.tfx.conv_stem_fwd(bool(on))
    except Exception:  # pragma: no cover - no native library (CPU-only tree)
        pass


def apply_env() -> None:
    spec = os.environ.get("TFX_FUSION", "")
    if spec and spec != "all":
        set_groups(parse_profile(spec))


# ---------------------------------------------------------------- recorder
_REC: Optional["record"] = None


def note(group: str, layer: str, kernel: str) -> None:
    """Called at each fusion decision point of ops/nn.py (a dict lookup when nothing records)."""
    if _REC is not None:
        _REC.events.append((group, layer, kernel))


class record:
    """``with fusion.record() as r: <one training step>`` -> ``r.events`` = [(group, layer, kernel)]
    in launch order; ``r.plan()`` groups them; ``r.table()`` formats the plan for the log."""

    def __init__(self):
        self.events: List[Tuple[str, str, str]] = []

    def __enter__(self):
        global _REC
        self._prev, _REC = _REC, self
        return self

    def __exit__(self, *exc):
        global _REC
        _REC = self._prev
        return False

    def plan(self) -> "OrderedDict[str, List[Tuple[str, str]]]":
        out: "OrderedDict[str, List[Tuple[str, str]]]" = OrderedDict((g, []) for g in GROUPS)
        out["layerwise"] = []
        for g, layer, k in self.events:
            out.setdefault(g, []).append((layer, k))
        return out

    def counts(self) -> Counter:
        return Counter((g, k) for g, _, k in self.events)

    def table(self) -> str:
        lines = ["fusion plan (%d decisions):" % len(self.events)]
        for g, items in self.plan().items():
            if not items:
                continue
            ks = Counter(k for _, k in items)
            lines.append("  %-22s %4d  %s" % (g, len(items), ", ".join("%s x%d" % kv for kv in sorted(ks.items()))))
        return "\n".join(lines)


__all__ = ["GROUPS", "PROFILES", "parse_profile", "enabled", "set_groups", "restore", "apply_env", "note", "record"]
