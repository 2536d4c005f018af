"""Flat variable store: every trainable tensor of a model is a view into ONE contiguous
f32 master buffer, with a matching flat gradient buffer and (for bf16 models) a flat
bf16 compute shadow.

This replaces TF1's per-variable ``VariableV2`` ops (R/distributed/distributed.py:68-91,
R/simple/simple.py:11-12) with a layout designed for MI355X:

* one fused optimizer launch updates the whole model and refreshes the bf16 shadow
  (csrc/kernels/optim.hip);
* gradient all-reduce works on large contiguous buckets of the flat grad buffer
  (parallel/allreduce.py) -- few, big RCCL calls over xGMI;
* the parameter server (cluster/ps.py) ships the flat buffer (or shards of it) in one
  message instead of one RPC per variable;
* weight-gradient kernels accumulate straight into their grad view (f32 atomics), so
  there is no per-parameter ``.grad`` allocation or copy.

Variables keep their TF names (``weights/Variable``, ``biases/Variable_1``, ...) so
checkpoints and the PS shard map match the reference's naming.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch

ALIGN = 64  # elements; keeps every view 128-B aligned in f32 and bf16 buffers


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


# ---------------------------------------------------------------- initializers
class Initializer:
    def __call__(self, shape: Sequence[int], gen: torch.Generator) -> torch.Tensor:  # pragma: no cover
        raise NotImplementedError

    def philox_spec(self, shape) -> Optional[tuple]:
        """(dist, a, b) for the Philox generator (random.py), or None for a host-side initializer."""
        return None


@dataclass
class Zeros(Initializer):
    def __call__(self, shape, gen):
        return torch.zeros(shape, dtype=torch.float32)


@dataclass
class Constant(Initializer):
    value: float = 0.0

    def __call__(self, shape, gen):
        return torch.full(shape, float(self.value), dtype=torch.float32)


@dataclass
class RandomNormal(Initializer):
    """tf.random_normal(shape, mean, stddev) -- R/distributed/distributed.py:85-86 (stddev 1.0)."""
    mean: float = 0.0
    stddev: float = 1.0

    def __call__(self, shape, gen):
        return torch.randn(shape, generator=gen, dtype=torch.float32) * self.stddev + self.mean

    def philox_spec(self, shape):
        return (1, self.mean, self.stddev)


@dataclass
class TruncatedNormal(Initializer):
    mean: float = 0.0
    stddev: float = 1.0

    def __call__(self, shape, gen):
        t = torch.randn(shape, generator=gen, dtype=torch.float32)
        bad = t.abs() > 2
        while bad.any():
            t[bad] = torch.randn(int(bad.sum()), generator=gen, dtype=torch.float32)
            bad = t.abs() > 2
        return t * self.stddev + self.mean

    def philox_spec(self, shape):
        return (2, self.mean, self.stddev)


@dataclass
class Uniform(Initializer):
    low: float = -1.0
    high: float = 1.0

    def __call__(self, shape, gen):
        return torch.rand(shape, generator=gen, dtype=torch.float32) * (self.high - self.low) + self.low

    def philox_spec(self, shape):
        return (0, self.low, self.high)


@dataclass
class HeNormal(Initializer):
    """Kaiming normal with fan_in = prod(shape[1:]) (conv weights stored [Ko,R,S,C])."""
    gain: float = math.sqrt(2.0)

    def __call__(self, shape, gen):
        fan_in = int(math.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
        return torch.randn(shape, generator=gen, dtype=torch.float32) * (self.gain / math.sqrt(fan_in))

    def philox_spec(self, shape):
        fan_in = int(math.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
        return (1, 0.0, self.gain / math.sqrt(fan_in))


@dataclass
class GlorotUniform(Initializer):
    @staticmethod
    def _lim(shape):
        if len(shape) == 2:
            fan_out, fan_in = shape[0], shape[1]
        else:
            rf = int(math.prod(shape[1:-1])) if len(shape) > 2 else 1
            fan_out, fan_in = shape[0] * rf, shape[-1] * rf
        return math.sqrt(6.0 / (fan_in + fan_out))

    def __call__(self, shape, gen):
        lim = self._lim(shape)
        return (torch.rand(shape, generator=gen, dtype=torch.float32) * 2 - 1) * lim

    def philox_spec(self, shape):
        lim = self._lim(shape)
        return (0, -lim, lim)


@dataclass
class Padded(Initializer):
    """Initialise the leading ``real_shape`` corner with ``inner`` and zero the padding.

    Used for layers whose channel counts are padded to the 8-element (16-B) granularity of the
    MFMA kernels (LeNet-5's 1 -> 6 -> 16 channels are carried as 8 -> 8 -> 16): padded weights,
    BN scales and shifts start at exactly zero and, because every gradient that reaches them is
    exactly zero too, stay zero under SGD / momentum / Adam -- the padded network computes the
    same function as the unpadded one."""
    inner: Initializer = field(default_factory=Zeros)
    real_shape: tuple = ()

    def __call__(self, shape, gen):
        out = torch.zeros(shape, dtype=torch.float32)
        out[tuple(slice(0, r) for r in self.real_shape)] = self.inner(tuple(self.real_shape), gen)
        return out


# ---------------------------------------------------------------- variables
@dataclass
class Variable:
    name: str
    shape: tuple
    initializer: Initializer
    trainable: bool = True
    index: int = 0
    offset: int = 0
    numel: int = 0
    store: Optional["VariableStore"] = field(default=None, repr=False)

    @property
    def master(self) -> torch.Tensor:
        """f32 master value (view into the flat buffer)."""
        return self.store.master[self.offset:self.offset + self.numel].view(self.shape)

    @property
    def value(self) -> torch.Tensor:
        """Compute copy: bf16 shadow view for bf16 stores, the f32 master otherwise."""
        buf = self.store.shadow if self.store.shadow is not None else self.store.master
        return buf[self.offset:self.offset + self.numel].view(self.shape)

    @property
    def grad(self) -> torch.Tensor:
        return self.store.grad[self.offset:self.offset + self.numel].view(self.shape)

    def assign(self, t: torch.Tensor) -> None:
        self.master.copy_(t.to(self.master.dtype).view(self.shape))
        if self.store.shadow is not None:
            self.value.copy_(self.master)


class SparseVariable:
    """A large, sparsely-updated table (word2vec embeddings, NCE weights/biases).

    Lives OUTSIDE the flat store: a 1M x 128 f32 table is 512 MB, and only the ~B rows a step
    touches change, so it has no dense gradient buffer and no dense optimizer pass.  Backward
    ops append ``(ids, rows)`` pairs to :attr:`pending` (TF's ``IndexedSlices``); the optimizer
    applies them with the scatter-add kernel (TF ``ScatterSub`` / sparse ``ApplyGradientDescent``
    semantics: duplicates are summed).  Initialised on the device (no host round trip)."""

    def __init__(self, name, shape, initializer: Initializer, store: "VariableStore", trainable=True, index=0):
        self.name, self.shape, self.initializer = name, tuple(int(s) for s in shape), initializer
        self.store, self.trainable, self.index = store, trainable, index
        self.table: Optional[torch.Tensor] = None
        self.pending: List[tuple] = []

    def materialize(self) -> None:
        dev = self.store.device
        spec = self.initializer.philox_spec(self.shape)
        if self.store.init_mode == "philox" and (spec is not None or isinstance(self.initializer, (Zeros, Constant))):
            from .random import philox_fill
            t = torch.empty(self.shape, dtype=torch.float32, device=dev)
            if spec is None:
                t.fill_(float(getattr(self.initializer, "value", 0.0)))
            else:
                philox_fill(t, self.store.seed, (1 << 40) + self.index, *spec)
            self.table = t
            return
        g = torch.Generator(device=dev).manual_seed(self.store.seed * 1000003 + 7919 + self.index)
        t = torch.empty(self.shape, dtype=torch.float32, device=dev)
        ini = self.initializer
        if isinstance(ini, Uniform):
            t.uniform_(ini.low, ini.high, generator=g)
        elif isinstance(ini, (RandomNormal, TruncatedNormal)):
            t.normal_(ini.mean, ini.stddev, generator=g)
            if isinstance(ini, TruncatedNormal):
                lo, hi = ini.mean - 2 * ini.stddev, ini.mean + 2 * ini.stddev
                bad = (t < lo) | (t > hi)
                while bool(bad.any()):
                    t[bad] = torch.empty(int(bad.sum()), device=dev).normal_(ini.mean, ini.stddev, generator=g)
                    bad = (t < lo) | (t > hi)
        elif isinstance(ini, Constant):
            t.fill_(float(ini.value))
        elif isinstance(ini, Zeros):
            t.zero_()
        else:
            t.copy_(ini(self.shape, torch.Generator().manual_seed(self.store.seed * 1000003 + 7919 + self.index)))
        self.table = t

    @property
    def master(self) -> torch.Tensor:
        return self.table

    value = master

    def add_sparse_grad(self, ids: torch.Tensor, rows: torch.Tensor) -> None:
        self.pending.append((ids.reshape(-1), rows.reshape(ids.numel(), -1).float().contiguous()))

    def clear(self) -> None:
        self.pending.clear()

    def assign(self, t: torch.Tensor) -> None:
        self.table.copy_(t.to(self.table.dtype).view(self.shape))


class VariableStore:
    """Creates variables (TF naming, creation order preserved) and lays them out flat."""

    def __init__(self, device="cpu", compute_dtype=torch.float32, seed: int = 0, init: str = "philox"):
        """``init``: "philox" (default) runs every random initializer through the Philox4x32-10
        generator of random.py -- on the device for GPU stores, identical streams on CPU and GPU;
        "torch" uses host torch.Generator draws (kept for reproducing older runs)."""
        self.init_mode = init
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.seed = seed
        self.vars: List[Variable] = []
        self.sparse: List[SparseVariable] = []
        self.by_name: Dict[str, Variable] = {}
        self.state: Dict[str, torch.Tensor] = {}  # non-trainable state (BN running stats, global_step)
        self.master: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        # True while the gradient buffer is known to be all zeros (a fresh buffer, or the optimizer
        # cleared it in its pass: Optimizer.apply_gradients(zero_grad=True)); zero_grad then skips the fill
        self.grads_clean = True
        self.grad_epoch = 0  # bumped by zero_grad (a step counter for gradient consumers)
        # per-model runtime state of the fused ops (ops/nn.py _model_state): the stem / head workspaces and
        # the BN-backward reductions deferred to a later launch of THIS model's backward -- never shared
        # between two models of one process
        self.fused_state: Dict[str, object] = {}
        self.shadow: Optional[torch.Tensor] = None
        self._flip = None          # flipped 3x3 filter copies (flip_index / flipped3x3)
        self.flip_stale = True
        self.total = 0
        # autograd anchor: a leaf that requires grad, passed to every parameterised op so the
        # graph is recorded even when no input activation requires grad (params are not
        # autograd leaves -- their grads are written into the flat buffer by the ops).
        self.anchor = torch.zeros((), device=self.device, requires_grad=True)
        self.grad_ready_hook = None
        self._scopes: List[str] = []
        self._name_counts: Dict[str, int] = {}

    # -- naming (tf.name_scope + tf.Variable auto-naming "Variable", "Variable_1", ...)
    def scope(self, name: str):
        store = self

        class _S:
            def __enter__(self):
                store._scopes.append(name)

            def __exit__(self, *a):
                store._scopes.pop()

        return _S()

    def unique_name(self, base: str) -> str:
        prefix = "/".join(self._scopes)
        full = f"{prefix}/{base}" if prefix else base
        n = self._name_counts.get(full, 0)
        self._name_counts[full] = n + 1
        return full if n == 0 else f"{full}_{n}"

    def variable(self, shape, initializer: Initializer, name: str = "Variable", trainable=True) -> Variable:
        if self.master is not None:
            raise RuntimeError("VariableStore already finalized")
        full = self.unique_name(name)
        v = Variable(full, tuple(int(s) for s in shape), initializer, trainable, index=len(self.vars), store=self)
        self.vars.append(v)
        self.by_name[full] = v
        return v

    def sparse_variable(self, shape, initializer: Initializer, name: str = "Variable",
                        trainable=True) -> SparseVariable:
        """A table updated through sparse (IndexedSlices) gradients -- see :class:`SparseVariable`."""
        if self.master is not None:
            raise RuntimeError("VariableStore already finalized")
        full = self.unique_name(name)
        v = SparseVariable(full, shape, initializer, self, trainable, index=len(self.vars) + len(self.sparse))
        self.sparse.append(v)
        self.by_name[full] = v
        return v

    def add_state(self, name: str, t: torch.Tensor) -> torch.Tensor:
        full = self.unique_name(name)
        t = t.to(self.device)
        self.state[full] = t
        return t

    # -- layout
    def finalize(self, init: bool = True) -> "VariableStore":
        off = 0
        for v in self.vars:
            v.numel = int(math.prod(v.shape)) if v.shape else 1
            v.offset = off
            off = _round_up(off + v.numel, ALIGN)
        self.total = max(off, ALIGN)
        self.master = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=self.device)
        self.grads_clean = True  # all zeros (see zero_grad)
        if self.compute_dtype != torch.float32:
            self.shadow = torch.zeros(self.total, dtype=self.compute_dtype, device=self.device)
        if init:
            self.initialize()
        else:
            for sv in self.sparse:
                sv.table = torch.zeros(sv.shape, dtype=torch.float32, device=self.device)
        return self

    def initialize(self) -> None:
        """Run every initializer (TF global_variables_initializer). Deterministic per (seed, index)."""
        if self.init_mode == "philox":
            self._initialize_philox()
        else:
            host = torch.zeros(self.total, dtype=torch.float32)
            for v in self.vars:
                g = torch.Generator().manual_seed(self.seed * 1000003 + v.index)
                host[v.offset:v.offset + v.numel] = v.initializer(v.shape, g).reshape(-1)
            self.master.copy_(host)
        self.refresh_shadow()
        for sv in self.sparse:
            sv.materialize()

    def _initialize_philox(self) -> None:
        from .random import philox_fill
        self.master.zero_()
        for v in self.vars:
            ini, view, shape = v.initializer, self.master[v.offset:v.offset + v.numel], v.shape
            if isinstance(ini, Padded):
                inner = ini.inner.philox_spec(tuple(ini.real_shape))
                if inner is None:
                    src = ini.inner(tuple(ini.real_shape), torch.Generator().manual_seed(self.seed * 1000003 + v.index))
                else:
                    src = torch.empty(tuple(ini.real_shape), dtype=torch.float32, device=self.device)
                    philox_fill(src, self.seed, v.index, *inner)
                view.view(shape)[tuple(slice(0, r) for r in ini.real_shape)] = src.to(self.device)
                continue
            spec = ini.philox_spec(shape)
            if spec is not None:
                philox_fill(view, self.seed, v.index, *spec)
            else:
                g = torch.Generator().manual_seed(self.seed * 1000003 + v.index)
                view.copy_(ini(shape, g).reshape(-1).to(self.device))

    def refresh_shadow(self) -> None:
        if self.shadow is not None:
            self.shadow.copy_(self.master)
        self.flip_stale = True

    # -- flipped 3x3 filters (the stride-1 3x3 data gradient runs as a forward conv with them)
    def flip_index(self, v: "Variable"):
        """Slot of ``v`` in the flipped-filter buffer, or None (not a [Ko, 3, 3, C] filter with
        Ko, C multiples of 64 in a bf16 GPU store)."""
        if self._flip is None:
            self._build_flip()
        return self._flip["slot"].get(v.name)

    def _build_flip(self) -> None:
        slot, rows, doff, tiles = {}, [], 0, 0
        if self.shadow is not None and self.shadow.is_cuda:
            for v in self.vars:
                sh = v.shape
                if len(sh) == 4 and sh[1] == 3 and sh[2] == 3 and sh[0] % 64 == 0 and sh[3] % 64 == 0:
                    slot[v.name] = (doff, tuple(int(d) for d in (sh[3], 3, 3, sh[0])))
                    rows.append([v.offset, doff, sh[0], sh[3], tiles])
                    doff += _round_up(v.numel, ALIGN)
                    tiles += 9 * (sh[0] // 64) * (sh[3] // 64)
        self._flip = {"slot": slot, "tiles": tiles, "buf": None, "desc": None}
        if rows:
            self._flip["buf"] = torch.zeros(doff, dtype=self.shadow.dtype, device=self.device)
            self._flip["desc"] = torch.tensor(rows, dtype=torch.int64).to(self.device)

    def flipped3x3(self, v: "Variable") -> torch.Tensor:
        """Wf[c][r][s][ko] = W[ko][2-r][2-s][c] of ``v`` (bf16), every layer's copy refreshed from
        the shadow in one launch when ``flip_stale`` (set by each forward conv that will want it)."""
        off, shape = self._flip["slot"][v.name]
        f = self._flip
        if self.flip_stale:
            torch.ops.tfx.wflip3x3(self.shadow, f["buf"], f["desc"], f["tiles"])
            self.flip_stale = False
        return f["buf"][off:off + v.numel].view(shape)

    def zero_grad(self) -> None:
        """Clear the gradients before a backward.  Skipped when the previous optimizer launch already
        cleared them in its pass (``Optimizer.apply_gradients(zero_grad=True)`` sets ``grads_clean``):
        the graphed training step then holds no separate fill."""
        if not self.grads_clean:
            self.grad.zero_()
        self.grads_clean = False  # the caller is about to accumulate into them
        self.grad_epoch += 1

    def trainable(self) -> List[Variable]:
        return [v for v in self.vars if v.trainable]

    def num_params(self) -> int:
        return sum(v.numel for v in self.vars if v.trainable) + \
            sum(int(math.prod(v.shape)) for v in self.sparse if v.trainable)

    # -- checkpoint helpers (name -> f32 tensor)
    def named_values(self) -> Dict[str, torch.Tensor]:
        out = {v.name: v.master.detach() for v in self.vars}
        out.update({v.name: v.table.detach() for v in self.sparse})
        out.update({k: t.detach() for k, t in self.state.items()})
        return out

    def load_named(self, values: Dict[str, torch.Tensor], strict: bool = True) -> None:
        for v in self.vars:
            if v.name in values:
                v.master.copy_(values[v.name].to(self.device, torch.float32).view(v.shape))
            elif strict:
                raise KeyError(f"missing variable {v.name}")
        for v in self.sparse:
            if v.name in values:
                v.table.copy_(values[v.name].to(self.device, torch.float32).view(v.shape))
            elif strict:
                raise KeyError(f"missing variable {v.name}")
        for k, t in self.state.items():
            if k in values:
                t.copy_(values[k].to(t.device, t.dtype).view(t.shape))
            elif strict:
                raise KeyError(f"missing state {k}")
        self.refresh_shadow()
