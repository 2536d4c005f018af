"""The cross-op fusion plan of the GPU training path.

The reference builds its model op by op and runs it unfused (R/distributed/distributed.py:94-108,
SURVEY §2.7).  Here the ResNet step fuses across op and layer boundaries.  Every fusion is a named
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
=====================  ==========================================================  ===============================

Three parts:

* :class:`FusionConfig` (``CONFIG``): which groups are on, as named knobs (one or two per group) that
  the ops read through :func:`knob`.  ``TFX_FUSION`` selects a profile at import: ``all`` (default:
  every group), ``r2`` (epilogue fusions only), ``none``
  (layer-wise), or a comma list of ``-group`` / ``+group`` edits applied to ``all``.  :func:`set_groups`
  / :func:`override` switch them at run time (tests, A/B runs).
* :class:`FusionPlan`: the per-layer plan, built when the model is constructed
  (:func:`plan_resnet`, ``ResNetCifar.fusion_plan``) from the architecture, the batch size and the
  kernels' own support predicates (the native library's ``*_supported`` entry points, host code that
  runs without a GPU).  For every conv it names the forward kernel, what happens to its deferred
  input (applied on load, formed by a fused boundary kernel, or materialised), and the fused backward
  kernel.  The conv op consults its layer's entry (:func:`layer_plan`) and runs the planned kernel;
  a layer without a plan (a conv used outside a planned model) takes the same decision from the
  same rules at call time.  A planned choice that the run-time state cannot honour is recorded as a
  ``plan_miss`` event and falls back -- the GPU test asserts there are none.
* Carriers (:func:`carry` / :func:`carried`): the run-time DATA a fused pair hands over between ops
  (a deferred BN apply, a BN's backward-fusion record, an unmaterialised BN input gradient), riding
  with the tensor they belong to.  They carry no decisions: whether a layer fuses is the plan's.

:class:`record` collects what one traced step actually ran, for comparison with the plan.
"""
from __future__ import annotations

import contextlib
import os
from collections import Counter, OrderedDict
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Tuple

GROUPS = ("bn_epilogue", "grad_sink", "masked_res", "s2_addend", "deferred_slot_reduce", "block_boundary_fwd",
          "bn_on_load", "lazy_bn_bwd", "conv3_fused_bwd", "stem_kernels", "fused_head", "head_tail")
# (a BN-finalize-folded-into-the-apply group was measured neutral and removed: profiles/r04_fold)
PROFILES = {
    "all": set(GROUPS),
    "r2": {"bn_epilogue", "grad_sink", "masked_res", "s2_addend", "deferred_slot_reduce", "fused_head"},
    "none": set(),
}

# group -> the knobs the ops read (a group is on when all its knobs are)
GROUP_KNOBS: Dict[str, Tuple[str, ...]] = {
    "bn_epilogue": ("fuse_bn",),
    "grad_sink": ("sink",),
    "masked_res": ("masked_res",),
    "s2_addend": ("s2_addend",),
    # take: a weight-gradient launch takes the pending reductions; defer: BNs leave them pending
    "deferred_slot_reduce": ("sr_take", "sr_defer"),
    "block_boundary_fwd": ("defer_tail",),
    # defer_bn_in: plain ReLU BNs leave their apply to the consumer; bn_on_load_1x1: ... incl. a 1x1 one
    "bn_on_load": ("defer_bn_in", "bn_on_load_1x1"),
    "lazy_bn_bwd": ("lazy_bn_bwd",),
    "conv3_fused_bwd": ("fuse_conv3_bwd",),
    "stem_kernels": ("stem_wgrad",),
    "fused_head": ("fuse_head",),
    "head_tail": ("head_tail",),
}
KNOBS = tuple(k for g in GROUPS for k in GROUP_KNOBS[g])


class FusionConfig:
    """The fusion switches: one boolean knob per decision point family (``GROUP_KNOBS``).  ``signature``
    (the knob values) keys the plans built under it: a plan is valid only under its own signature."""

    def __init__(self, groups: Iterable[str]):
        on = set(groups)
        self.knobs: Dict[str, bool] = {k: g in on for g in GROUPS for k in GROUP_KNOBS[g]}
        self.signature = tuple(self.knobs[k] for k in KNOBS)

    def set(self, name: str, value: bool) -> None:
        if name not in self.knobs:
            raise KeyError("unknown fusion knob %r (knobs: %s)" % (name, ", ".join(KNOBS)))
        self.knobs[name] = bool(value)
        self.signature = tuple(self.knobs[k] for k in KNOBS)

    def group_on(self, group: str) -> bool:
        return all(self.knobs[k] for k in GROUP_KNOBS[group])


CONFIG = FusionConfig(PROFILES["all"])


def knob(name: str) -> bool:
    """The ops' read of one fusion switch."""
    return CONFIG.knobs[name]


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
    return {g: CONFIG.group_on(g) for g in GROUPS}


def knobs() -> Dict[str, bool]:
    return dict(CONFIG.knobs)


def set_groups(on: Iterable[str]) -> Dict[str, bool]:
    """Enable exactly the groups in ``on``; returns the previous knob state (pass it to :func:`restore`)."""
    prev = knobs()
    on = set(on)
    for g in GROUPS:
        for k in GROUP_KNOBS[g]:
            CONFIG.set(k, g in on)
    _stem_fwd("stem_kernels" in on)
    return prev


def restore_knobs(state: Dict[str, bool]) -> None:
    """Restore a COMPLETE knob state, as returned by :func:`knobs` / :func:`set_groups`."""
    if set(state) != set(KNOBS):
        raise ValueError("restore_knobs needs every knob (%s); got %s" % (", ".join(KNOBS), sorted(state)))
    for k, v in state.items():
        CONFIG.set(k, v)
    _stem_fwd(CONFIG.knobs["stem_wgrad"])


def restore_groups(state: Dict[str, bool]) -> None:
    """Restore a COMPLETE group state, as returned by :func:`enabled`."""
    if set(state) != set(GROUPS):
        raise ValueError("restore_groups needs every group (%s); got %s" % (", ".join(GROUPS), sorted(state)))
    set_groups([g for g, v in state.items() if v])


def restore(state: Dict[str, bool]) -> None:
    """Restore a complete state returned by :func:`set_groups` / :func:`knobs` (knob dict) or
    :func:`enabled` (group dict).  Three knob names are also group names (masked_res, s2_addend,
    lazy_bn_bwd), so a partial dict is ambiguous: anything but a complete one raises."""
    if set(state) == set(KNOBS):
        restore_knobs(state)
    elif set(state) == set(GROUPS):
        restore_groups(state)
    else:
        raise ValueError("fusion.restore: neither a complete knob dict nor a complete group dict: %s" % sorted(state))


@contextlib.contextmanager
def override(**kv: bool):
    """``with fusion.override(sr_defer=False): ...`` -- knobs set for the block, then restored."""
    prev = knobs()
    try:
        for k, v in kv.items():
            CONFIG.set(k, v)
        if "stem_wgrad" in kv:
            _stem_fwd(CONFIG.knobs["stem_wgrad"])
        yield CONFIG
    finally:
        restore(prev)


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


# ---------------------------------------------------------------- carriers
CARRIER_KINDS = ("tail", "bnb", "lazy_bnbwd")
_CARRY_ATTR = {k: "_tfx_carry_" + k for k in CARRIER_KINDS}


def carry(t, kind: str, obj) -> None:
    """Hand ``obj`` over with tensor ``t`` (``kind``: "tail" = a deferred BN apply (TailPending), "bnb"
    = a BN's backward-fusion record (BNBackwardFusion), "lazy_bnbwd" = an unmaterialised BN input
    gradient (LazyBNGrad)).  The object rides on the tensor's Python object, which PyTorch keeps
    (with it) for as long as autograd holds the tensor -- a gradient returned by one backward reaches
    the next backward as the same object.  Only these two functions touch the attribute."""
    setattr(t, _CARRY_ATTR[kind], obj)


def carried(t, kind: str):
    """The object handed over with ``t`` under ``kind``, or None."""
    return getattr(t, _CARRY_ATTR[kind], None) if t is not None else None


# ---------------------------------------------------------------- the per-layer plan
# forward kernels of a conv, as the recorder names them
FWD_KERNELS = ("igemm_fwd_stats", "stem_fwd", "pw_fwd_squeeze", "conv3x3_fwd_fused", "igemm_fwd_a_scale",
               "igemm_fwd", "igemm_fwd_stats_only")
# the kernel -> group of every fused forward / backward choice
KERNEL_GROUP = {
    "igemm_fwd_stats": "bn_epilogue", "stem_fwd": "bn_epilogue", "igemm_fwd_stats_only": "bn_epilogue",
    "pw_fwd_squeeze": "block_boundary_fwd", "conv3x3_fwd_fused": "bn_on_load", "igemm_fwd_a_scale": "bn_on_load",
    "igemm_fwd": "conv", "conv3x3_bwd_fused": "conv3_fused_bwd", "pw_bwd_expand": "lazy_bn_bwd",
    "pw_bwd_squeeze": "lazy_bn_bwd", "stem_wgrad": "stem_kernels", "igemm_dgrad_compact": "s2_addend",
    "head_xent": "fused_head", "head_xent_tail": "head_tail", "bn_apply_into": "layerwise",
}


@dataclass
class LayerPlan:
    """One conv's plan.  ``input``: what produces its input -- "tensor" (a written tensor), "plain" (a
    plain ReLU BN whose apply was deferred to this conv) or "tail" (a residual + ReLU block tail BN
    deferred to it).  ``pre``: the kernel that materialises a deferred input first (None when the
    forward kernel consumes it).  ``fwd`` / ``bwd``: the forward kernel and the fused backward kernel
    (``bwd`` None = the layer-wise implicit-GEMM data / weight gradients, whose epilogue flavours --
    BN-backward partials, residual addend, slot-reduce tail blocks -- follow the run-time gradient
    sinks).  ``extra``: further planned fused events of the layer (e.g. its compact stride-2 input
    gradient)."""
    name: str
    role: str
    cin: int
    cout: int
    k: int
    stride: int
    hw: Tuple[int, int]
    rows: int
    input: str = "tensor"
    pre: Optional[str] = None
    fwd: str = "igemm_fwd_stats"
    bwd: Optional[str] = None
    extra: List[str] = field(default_factory=list)

    def events(self) -> List[Tuple[str, str, str]]:
        ev = []
        if self.pre is not None:
            ev.append((KERNEL_GROUP[self.pre], self.name, self.pre))
        ev.append((KERNEL_GROUP[self.fwd], self.name, self.fwd))
        if self.bwd is not None:
            ev.append((KERNEL_GROUP[self.bwd], self.name, self.bwd))
        for k in self.extra:
            ev.append((KERNEL_GROUP[k], self.name, k))
        return ev


class FusionPlan:
    """The fusion plan of one model at one batch size: ``layers`` (conv weight name -> LayerPlan, in
    forward order) and ``head`` (the classifier head's planned kernels)."""

    def __init__(self, batch: int, config_signature: Tuple[bool, ...]):
        self.batch = batch
        self.config_signature = config_signature
        self.layers: "OrderedDict[str, LayerPlan]" = OrderedDict()
        self.head: List[Tuple[str, str, str]] = []

    def add(self, lp: LayerPlan) -> LayerPlan:
        self.layers[lp.name] = lp
        return lp

    def events(self) -> List[Tuple[str, str, str]]:
        ev = [e for lp in self.layers.values() for e in lp.events()]
        return ev + list(self.head)

    def counts(self) -> Counter:
        return Counter((g, k) for g, _, k in self.events())

    def fused_counts(self) -> Counter:
        """Counts of the fused-group decisions (the layer-wise fallbacks and plain convs left out)."""
        return Counter({gk: n for gk, n in self.counts().items() if gk[0] not in ("layerwise", "conv")})

    def table(self) -> str:
        lines = ["fusion plan, batch %d (%d conv layers):" % (self.batch, len(self.layers))]
        for lp in self.layers.values():
            lines.append("  %-40s %-9s %4d->%-4d k%d s%d  in=%-6s %s%s%s" % (
                lp.name, lp.role, lp.cin, lp.cout, lp.k, lp.stride, lp.input,
                (lp.pre + " + ") if lp.pre else "", lp.fwd, ("  | bwd " + lp.bwd) if lp.bwd else ""))
        for g, name, k in self.head:
            lines.append("  %-40s head      %s (%s)" % (name, k, g))
        return "\n".join(lines)


def layer_plan(w) -> Optional[LayerPlan]:
    """The active plan's entry for conv weight ``w`` (None: no planned model owns it).  The plan is the
    one its model set on the store for the current batch (``ResNetCifar.features``)."""
    plan = getattr(getattr(w, "store", None), "fusion_plan", None)
    if plan is None or plan.config_signature != CONFIG.signature:
        return None
    return plan.layers.get(w.name)


def miss(layer: str, planned: str, reason: str) -> None:
    """A planned choice the run-time state could not honour (recorded; the op falls back)."""
    note("plan_miss", layer, "%s (%s)" % (planned, reason))


# ---- the decision rules: used by the planner (architecture known) and by unplanned calls (run time)
def _sup(name: str, *args) -> bool:
    import torch
    return bool(getattr(torch.ops.tfx, name)(*args))


def conv_rows(batch: int, hw: Tuple[int, int], k: int, stride: int) -> int:
    pad = k // 2
    p = (hw[0] + 2 * pad - (k - 1) - 1) // stride + 1
    q = (hw[1] + 2 * pad - (k - 1) - 1) // stride + 1
    return batch * p * q


def fwd_rule(input_kind: str, cin: int, cout: int, k: int, stride: int, batch: int, hw: Tuple[int, int],
             ws: str = "obj", stem: bool = False) -> Tuple[Optional[str], str]:
    """(pre, fwd) of a conv whose input is ``input_kind`` ("tensor" / "plain" / "tail", LayerPlan) and
    whose output statistics go to ``ws``: "obj" (a BNWorkspace: statistics + finalize in the epilogue),
    "raw" (a slot tensor: statistics only) or "none".  A deferred input is consumed by the fused kernel
    that takes this shape, else materialised first (``pre``)."""
    pre = None
    rows_in = batch * hw[0] * hw[1]
    fused_ok = ws == "obj"
    if input_kind == "plain":
        if k == 3 and stride == 1 and fused_ok and _sup("conv3x3_fused_supported", batch, hw[0], hw[1], cin, cout):
            return None, "conv3x3_fwd_fused"
        if k == 1 and stride == 1 and fused_ok and cin <= 64 and cin % 8 == 0 and knob("defer_bn_in") \
                and knob("bn_on_load_1x1"):
            return None, "igemm_fwd_a_scale"
        pre = "bn_apply_into"
    elif input_kind == "tail":
        if k == 1 and stride == 1 and fused_ok and _sup("pw_fwd_squeeze_supported", cin, cout, rows_in):
            return None, "pw_fwd_squeeze"
        pre = "bn_apply_into"
    if ws == "obj":
        return pre, ("stem_fwd" if stem else "igemm_fwd_stats")
    return pre, ("igemm_fwd_stats_only" if ws == "raw" else "igemm_fwd")


def stem_ok(cin: int, cout: int, k: int, stride: int, batch: int, hw: Tuple[int, int]) -> bool:
    return k == 3 and stride == 1 and _sup("stem_wgrad_supported", batch, hw[0], hw[1], cin, cout)


def plan_resnet(model, batch: int, hw: Tuple[int, int] = (32, 32)) -> FusionPlan:
    """The fusion plan of a CIFAR ResNet (models/resnet.py) training step at ``batch`` images of
    ``hw``: walks the stem, the blocks and the head in forward order, tracking what each conv's
    input is (a written tensor, or a BN output deferred to it) with the same knobs the ops read."""
    from ..models import resnet as R
    plan = FusionPlan(batch, CONFIG.signature)
    fuse_bn = knob("fuse_bn")
    lazy = fuse_bn and knob("lazy_bn_bwd")
    sink_on = knob("sink")
    st = model.stem
    stem = knob("stem_wgrad") and stem_ok(st.w.shape[3], st.w.shape[0], st.w.shape[1], st.stride, batch, hw)
    lp = plan.add(LayerPlan(st.w.name, "stem", st.w.shape[3], st.w.shape[0], st.w.shape[1], st.stride, hw,
                            conv_rows(batch, hw, st.w.shape[1], st.stride)))
    wsk = "obj" if fuse_bn else "raw"
    lp.pre, lp.fwd = fwd_rule("tensor", lp.cin, lp.cout, lp.k, lp.stride, batch, hw, ws=wsk, stem=stem and fuse_bn)
    if stem:
        lp.bwd = "stem_wgrad"
    cur_hw, cur_kind = hw, "tensor"
    nblk = len(model.blocks)
    for i, blk in enumerate(model.blocks):
        if isinstance(blk, R.Bottleneck):
            nxt = model.blocks[i + 1] if i + 1 < nblk else None
            defer_tail = fuse_bn and knob("defer_tail") and (isinstance(nxt, R.Bottleneck) or nxt is None)
            prev_tail = i > 0 and isinstance(model.blocks[i - 1], R.Bottleneck)
            cur_hw, cur_kind = _plan_bottleneck(plan, blk, batch, cur_hw, cur_kind, prev_tail, defer_tail, lazy,
                                                sink_on)
        else:
            cur_hw, cur_kind = _plan_basic(plan, blk, batch, cur_hw, cur_kind)
    if knob("fuse_head"):
        fc = model.fc_w.name
        if cur_kind == "tail" and knob("head_tail"):
            plan.head.append(("head_tail", fc, "head_xent_tail"))
        plan.head.append(("fused_head", fc, "head_xent"))
    return plan


def _conv_lp(c, role, batch, hw) -> LayerPlan:
    k, s = c.w.shape[1], c.stride
    return LayerPlan(c.w.name, role, c.w.shape[3], c.w.shape[0], k, s, hw, conv_rows(batch, hw, k, s))


def _plan_bottleneck(plan, blk, batch, hw, in_kind, prev_tail, defer_tail, lazy, sink_on):
    """One bottleneck: conv1 (1x1) <- the block input; conv2 (3x3, the block's stride) <- BN1;
    conv3 (1x1 expand) <- BN2; shortcut (1x1 projection) <- the block input."""
    fuse_bn = knob("fuse_bn")
    wsk = "obj" if fuse_bn else "raw"
    plain = fuse_bn and knob("defer_bn_in")
    masked = sink_on and knob("masked_res")
    c1 = plan.add(_conv_lp(blk.c1, "conv1", batch, hw))
    c1.input = in_kind
    c1.pre, c1.fwd = fwd_rule(in_kind, c1.cin, c1.cout, 1, 1, batch, hw, ws=wsk)
    # conv1's backward: BN1's lazy input gradient formed on load, the identity branch's parked
    # (gradient, mask) added, the previous tail BN's partials reduced (pw_bwd_squeeze) -- needs that
    # tail BN (its mask bits) as the input and an identity block's masked sink
    if lazy and masked and prev_tail and blk.proj is None \
            and _sup("pw_bwd_squeeze_supported", c1.cin, c1.cout, c1.rows):
        c1.bwd = "pw_bwd_squeeze"
    c2 = plan.add(_conv_lp(blk.c2, "conv2", batch, hw))
    c2.input = "plain" if plain else "tensor"
    c2.pre, c2.fwd = fwd_rule(c2.input, c2.cin, c2.cout, 3, c2.stride, batch, hw, ws=wsk)
    if c2.fwd == "conv3x3_fwd_fused" and lazy and knob("fuse_conv3_bwd"):
        c2.bwd = "conv3x3_bwd_fused"
    hw2 = (hw[0] // blk.c2.stride, hw[1] // blk.c2.stride)
    c3 = plan.add(_conv_lp(blk.c3, "conv3", batch, hw2))
    c3.input = "plain" if plain else "tensor"
    c3.pre, c3.fwd = fwd_rule(c3.input, c3.cin, c3.cout, 1, 1, batch, hw2, ws=wsk)
    # conv3's backward: the tail BN's lazy input gradient (identity block: its residual gradient
    # parked masked in the sink; projection block: the shortcut BN's reduction rides along)
    tail_lazy = lazy and (blk.proj is not None or masked)
    if tail_lazy and c3.cout == 4 * c3.cin and _sup("pw_bwd_expand_supported", c3.cin, c3.rows):
        c3.bwd = "pw_bwd_expand"
    if blk.proj is not None:
        sc = plan.add(_conv_lp(blk.proj, "shortcut", batch, hw))
        # the block input is written by conv1's launch (or its materialising apply) before this runs
        sc.pre, sc.fwd = fwd_rule("tensor", sc.cin, sc.cout, 1, sc.stride, batch, hw, ws=wsk)
        if sink_on and knob("s2_addend") and sc.stride == 2 and sc.cin % 8 == 0:
            sc.extra.append("igemm_dgrad_compact")
    return hw2, ("tail" if defer_tail else "tensor")


def _plan_basic(plan, blk, batch, hw, in_kind):
    """One basic block: conv1 (3x3, the block's stride), conv2 (3x3), shortcut (1x1 projection); no
    deferred BN applies (a basic block's BNs apply as they go)."""
    wsk = "obj" if knob("fuse_bn") else "raw"
    c1 = plan.add(_conv_lp(blk.c1, "conv1", batch, hw))
    c1.input = in_kind
    c1.pre, c1.fwd = fwd_rule(in_kind, c1.cin, c1.cout, 3, c1.stride, batch, hw, ws=wsk)
    hw2 = (hw[0] // blk.c1.stride, hw[1] // blk.c1.stride)
    c2 = plan.add(_conv_lp(blk.c2, "conv2", batch, hw2))
    c2.pre, c2.fwd = fwd_rule("tensor", c2.cin, c2.cout, 3, 1, batch, hw2, ws=wsk)
    if blk.proj is not None:
        sc = plan.add(_conv_lp(blk.proj, "shortcut", batch, hw))
        sc.pre, sc.fwd = fwd_rule("tensor", sc.cin, sc.cout, 1, sc.stride, batch, hw, ws=wsk)
    return hw2, "tensor"


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

    def misses(self) -> List[Tuple[str, str]]:
        return [(layer, k) for g, layer, k in self.events if g == "plan_miss"]

    def table(self) -> str:
        lines = ["fusion plan (%d decisions):" % len(self.events)]
        for g, items in self.plan().items():
            if not items:
                continue
            ks = Counter(k for _, k in items)
            lines.append("  %-22s %4d  %s" % (g, len(items), ", ".join("%s x%d" % kv for kv in sorted(ks.items()))))
        return "\n".join(lines)


__all__ = ["GROUPS", "PROFILES", "GROUP_KNOBS", "KNOBS", "FusionConfig", "CONFIG", "knob", "parse_profile",
           "enabled", "knobs", "set_groups", "restore", "override", "apply_env", "carry", "carried",
           "LayerPlan", "FusionPlan", "layer_plan", "plan_resnet", "fwd_rule", "note", "record"]
