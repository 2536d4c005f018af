"""Sparse ops: embedding lookup, the log-uniform candidate sampler and sampled losses (NCE /
sampled softmax) -- the word2vec skip-gram workload (BASELINE.json config 4) and the char-LSTM
input embedding (config 5).

TF1 equivalents: ``tf.nn.embedding_lookup`` (gather + IndexedSlices gradient),
``tf.nn.log_uniform_candidate_sampler``, ``tf.nn.nce_loss`` and ``tf.nn.sampled_softmax_loss``.

GPU path (csrc/kernels/sparse_rnn.hip + sgemm.hip), per step with B examples, S shared
negatives, D-wide rows:

    ids_s, logQ_s  = log_uniform_sample(S)               (counter-hash RNG, no state)
    E, Wt, bt      = gather(emb, x), gather(W, y), gather(b, y)
    neg            = E @ Ws^T + bs                        (f32 MFMA GEMM, bias in the epilogue)
    loss, dn, dE, dWt, dbt = sampled_loss(E, Wt, bt, neg)  (one fused kernel: true dot, logQ,
                                                           accidental hits, loss, all row grads)
    dE            += dn @ Ws                              (GEMM accumulating into dE)
    dWs            = dn^T @ E                             (GEMM)
    table[ids]    -= lr * rows                            (scatter-add, whole-row f32 atomics)

CPU path: the same math in PyTorch (the numerics oracle of tests/test_sparse_*).
"""
from __future__ import annotations

import math
from typing import Optional, Union

import torch

from . import _native
from ..variables import SparseVariable, Variable

Table = Union[Variable, SparseVariable]


# ---------------------------------------------------------------- raw row ops
def gather_rows(table: torch.Tensor, ids: torch.Tensor, bf16: bool = False) -> torch.Tensor:
    """rows[i] = table[ids[i]] (ids clamped into range like TF's GPU gather)."""
    if _native.use_native(table):
        return torch.ops.tfx.embedding_gather(table, ids.reshape(-1).contiguous(), bf16)
    out = table.index_select(0, ids.reshape(-1).clamp(0, table.shape[0] - 1))
    return out.to(torch.bfloat16) if bf16 else out


def scatter_add_rows(table: torch.Tensor, ids: torch.Tensor, rows: torch.Tensor, alpha: float = 1.0) -> None:
    """table[ids[i]] += alpha * rows[i] (duplicates summed)."""
    ids = ids.reshape(-1)
    rows = rows.reshape(ids.numel(), -1).float().contiguous()
    if _native.use_native(table):
        torch.ops.tfx.embedding_scatter_add(table, ids.contiguous(), rows, float(alpha))
    else:
        table.index_add_(0, ids, rows, alpha=alpha)


# ---------------------------------------------------------------- sampler
def log_uniform_logq(ids: torch.Tensor, range_max: int, num_expected: int) -> torch.Tensor:
    """log(expected count) of ``ids`` under the Zipfian sampler:
    log(num_expected * log((k+2)/(k+1)) / log(range_max+1))."""
    if _native.use_native(ids):
        return torch.ops.tfx.log_uniform_logq(ids.reshape(-1).contiguous(), range_max, num_expected)
    k = ids.reshape(-1).double()
    p = torch.log((k + 2) / (k + 1)) / math.log(range_max + 1.0)
    return torch.log(p * num_expected).float()


def log_uniform_sample(num_sampled: int, range_max: int, seed: int, device,
                       seed_tensor: Optional[torch.Tensor] = None) -> tuple:
    """tf.nn.log_uniform_candidate_sampler(unique=False): (ids int64 [S], log expected counts [S]).
    GPU: stateless counter-hash RNG keyed by ``seed`` plus, if given, the device int64 counter
    ``seed_tensor`` (so a captured HIP graph draws new candidates on each replay)."""
    device = torch.device(device)
    if device.type == "cuda" and _native.load():
        return torch.ops.tfx.log_uniform_sample(num_sampled, range_max, int(seed) & 0x7FFFFFFFFFFFFFFF,
                                                num_sampled, device, seed_tensor)
    if seed_tensor is not None:
        seed = int(seed) + int(seed_tensor.reshape(-1)[0])
    g = torch.Generator().manual_seed(int(seed))
    u = torch.rand(num_sampled, generator=g, dtype=torch.float64)
    ids = (torch.exp(u * math.log(range_max + 1.0)).floor().long() - 1).clamp(0, range_max - 1).to(device)
    return ids, log_uniform_logq(ids, range_max, num_sampled)


# ---------------------------------------------------------------- embedding lookup
class _EmbeddingLookup(torch.autograd.Function):
    """Gather rows of a table.  Backward: an IndexedSlices gradient -- for a :class:`SparseVariable`
    it is queued for the sparse optimizer; for a dense flat-store :class:`Variable` it is scattered
    (f32 atomics) straight into the variable's slice of the flat grad buffer."""

    @staticmethod
    def forward(ctx, ids, anchor, table: Table, bf16: bool):
        ctx.table, ctx.ids = table, ids
        t = table.master
        out = gather_rows(t, ids, bf16)
        return out.view(*ids.shape, t.shape[1])

    @staticmethod
    def backward(ctx, g):
        table, ids = ctx.table, ctx.ids
        if table.trainable:
            rows = g.reshape(ids.numel(), -1).float().contiguous()
            if isinstance(table, SparseVariable):
                table.add_sparse_grad(ids, rows)
            else:
                scatter_add_rows(table.grad, ids, rows, 1.0)
                hook = getattr(table.store, "grad_ready_hook", None)
                if hook is not None:
                    hook(table)
        return None, None, None, None


def embedding_lookup(table: Table, ids: torch.Tensor, bf16: bool = False) -> torch.Tensor:
    """tf.nn.embedding_lookup(params, ids): [..] int64 -> [.., D] (f32, or bf16 when ``bf16``)."""
    return _EmbeddingLookup.apply(ids, table.store.anchor, table, bf16)


# ---------------------------------------------------------------- sampled losses
def sampled_loss_grads(E: torch.Tensor, Wt: torch.Tensor, bt: Optional[torch.Tensor], Ws: torch.Tensor,
                       bs: Optional[torch.Tensor], logq_t: Optional[torch.Tensor], logq_s: Optional[torch.Tensor],
                       true_ids: Optional[torch.Tensor] = None, sampled_ids: Optional[torch.Tensor] = None,
                       softmax: bool = False, gscale: float = 1.0):
    """Per-example sampled loss and every gradient it needs, without autograd.

    ``E`` [B,D] inputs, ``Wt``/``bt`` true-class rows, ``Ws``/``bs`` the S sampled rows (shared by the
    batch, as in tf.nn.nce_loss). Passing both id tensors removes accidental hits
    (remove_accidental_hits=True). Returns (loss_rows [B], dE [B,D], dWt [B,D], dbt [B], dWs [S,D],
    dbs [S]); gradients are of ``gscale * sum(loss_rows)``."""
    if _native.use_native(E):
        neg = torch.ops.tfx.sgemm(E, Ws, False, True, bs, 0, True)
        loss, dn, dE, dWt, dbt = torch.ops.tfx.sampled_loss(E, Wt, bt, neg, logq_t, logq_s, true_ids, sampled_ids,
                                                             gscale, softmax)
        torch.ops.tfx.sgemm_into(dn, Ws, False, False, dE, True)
        # dWs = dn^T E reduces over the whole batch into 64 x D: split-K over blocks (f32 atomics)
        dWs = torch.ops.tfx.sgemm(dn, E, True, False, None, 0, True)
        dbs = dn.sum(0)
        return loss, dE, dWt, dbt, dWs, dbs
    return _sampled_ref(E, Wt, bt, Ws, bs, logq_t, logq_s, true_ids, sampled_ids, softmax, gscale)


def _sampled_ref(E, Wt, bt, Ws, bs, logq_t, logq_s, true_ids, sampled_ids, softmax, gscale):
    with torch.enable_grad():
        E_, Wt_, Ws_ = (t.detach().float().requires_grad_(True) for t in (E, Wt, Ws))
        bt_ = bt.detach().float().requires_grad_(True) if bt is not None else None
        bs_ = bs.detach().float().requires_grad_(True) if bs is not None else None
        t = (E_ * Wt_).sum(1)
        if bt_ is not None:
            t = t + bt_
        n = E_ @ Ws_.t()
        if bs_ is not None:
            n = n + bs_
        if logq_t is not None:
            t = t - logq_t
        if logq_s is not None:
            n = n - logq_s
        hit = None
        if true_ids is not None and sampled_ids is not None:
            hit = true_ids.reshape(-1, 1) == sampled_ids.reshape(1, -1)
        if softmax:
            if hit is not None:
                n = n.masked_fill(hit, float("-inf"))
            logits = torch.cat([t[:, None], n], 1)
            loss = torch.logsumexp(logits, 1) - t
        else:
            sp = torch.nn.functional.softplus(n)
            if hit is not None:
                sp = sp.masked_fill(hit, 0.0)
            loss = torch.nn.functional.softplus(-t) + sp.sum(1)
        leaves = [E_, Wt_, Ws_] + [x for x in (bt_, bs_) if x is not None]
        grads = torch.autograd.grad(loss.sum() * gscale, leaves, allow_unused=True)
    dE, dWt, dWs = grads[:3]
    rest = list(grads[3:])
    dbt = rest.pop(0) if bt_ is not None else torch.zeros(E.shape[0], dtype=torch.float32, device=E.device)
    dbs = rest.pop(0) if bs_ is not None else torch.zeros(Ws.shape[0], dtype=torch.float32, device=E.device)
    return loss.detach(), dE, dWt, dbt, dWs, dbs


def _squeeze_bias(b: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if b is None else b.reshape(-1).contiguous()


class _SampledLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, anchor, weights: Table, biases: Optional[Table], labels, num_sampled, num_classes,
                softmax, remove_hits, seed):
        labels = labels.reshape(-1)
        B = labels.numel()
        E = inputs.float().contiguous()
        sid, logq_s = log_uniform_sample(num_sampled, num_classes, seed, E.device)
        logq_t = log_uniform_logq(labels, num_classes, num_sampled)
        Wt = gather_rows(weights.master, labels)
        Ws = gather_rows(weights.master, sid)
        bt = _squeeze_bias(gather_rows(biases.master, labels)) if biases is not None else None
        bs = _squeeze_bias(gather_rows(biases.master, sid)) if biases is not None else None
        loss, dE, dWt, dbt, dWs, dbs = sampled_loss_grads(
            E, Wt, bt, Ws, bs, logq_t, logq_s, labels if remove_hits else None, sid if remove_hits else None,
            softmax, 1.0 / B)
        ctx.weights, ctx.biases, ctx.dtype = weights, biases, inputs.dtype
        ctx.grads = (labels, sid, dE, dWt, dbt, dWs, dbs)
        return loss.mean()

    @staticmethod
    def backward(ctx, g):
        labels, sid, dE, dWt, dbt, dWs, dbs = ctx.grads
        ctx.grads = None
        gs = g.float()
        for tab, rows_t, rows_s in ((ctx.weights, dWt, dWs), (ctx.biases, dbt, dbs)):
            if tab is None or not tab.trainable:
                continue
            rt, rs = (rows_t * gs).reshape(labels.numel(), -1), (rows_s * gs).reshape(sid.numel(), -1)
            if isinstance(tab, SparseVariable):
                tab.add_sparse_grad(labels, rt)
                tab.add_sparse_grad(sid, rs)
            else:
                scatter_add_rows(tab.grad, labels, rt)
                scatter_add_rows(tab.grad, sid, rs)
        return (dE * gs).to(ctx.dtype), None, None, None, None, None, None, None, None, None


def nce_loss(weights: Table, biases: Optional[Table], labels: torch.Tensor, inputs: torch.Tensor, num_sampled: int,
             num_classes: int, remove_accidental_hits: bool = False, seed: int = 0) -> torch.Tensor:
    """tf.nn.nce_loss(...) averaged over the batch (word2vec_basic's ``tf.reduce_mean(nce_loss)``).
    ``weights`` [num_classes, D], ``biases`` [num_classes, 1] (or None); shared log-uniform negatives,
    sampled with replacement (``unique=False``), varied per call through ``seed``."""
    return _SampledLoss.apply(inputs, weights.store.anchor, weights, biases, labels, num_sampled, num_classes,
                              False, remove_accidental_hits, seed)


def sampled_softmax_loss(weights: Table, biases: Optional[Table], labels: torch.Tensor, inputs: torch.Tensor,
                         num_sampled: int, num_classes: int, remove_accidental_hits: bool = True,
                         seed: int = 0) -> torch.Tensor:
    """tf.nn.sampled_softmax_loss(...) averaged over the batch."""
    return _SampledLoss.apply(inputs, weights.store.anchor, weights, biases, labels, num_sampled, num_classes,
                              True, remove_accidental_hits, seed)


__all__ = ["embedding_lookup", "gather_rows", "scatter_add_rows", "log_uniform_sample", "log_uniform_logq",
           "sampled_loss_grads", "nce_loss", "sampled_softmax_loss"]
