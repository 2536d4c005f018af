"""word2vec skip-gram (BASELINE.json config 4: "word2vec skip-gram 1M-row embedding on one
MI355X (embedding-lookup + sampled-softmax HIP)").

TF ``word2vec_basic`` model: ``embeddings`` [V,D] ~ U(-1,1), ``nce_weights`` [V,D] ~
truncated_normal(stddev=1/sqrt(D)), ``nce_biases`` [V] = 0; loss ``reduce_mean(nce_loss(...,
num_sampled=64))`` with log-uniform negatives; ``GradientDescentOptimizer(1.0)`` applied as
sparse (IndexedSlices) updates; cosine-similarity nearest neighbours for evaluation.

Two equivalent training paths:

* :meth:`SkipGram.loss` -- composable autograd ops (``embedding_lookup`` + ``nce_loss``),
  then ``optimizer.apply_gradients()`` applies the queued sparse gradients;
* :meth:`SkipGram.train_step` -- the MI355X fast path: one explicit forward+backward+update
  with no autograd bookkeeping: ~12 kernel launches, all on the current stream, HIP-graph
  capturable (device step counter drives the batch generator and the sampler).

Tables are :class:`~tensorflow_examples_amd.variables.SparseVariable` s: 1M x 128 f32 = 512 MB
each, resident in HBM; only the ~B + S touched rows are read or written per step.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from .. import ops
from ..ops.sparse import gather_rows, log_uniform_logq, log_uniform_sample, sampled_loss_grads, scatter_add_rows
from ..variables import TruncatedNormal, Uniform, VariableStore, Zeros


class SkipGram:
    def __init__(self, store: VariableStore, vocab_size: int = 1_000_000, embedding_size: int = 128,
                 num_sampled: int = 64, loss: str = "nce"):
        assert loss in ("nce", "sampled_softmax")
        self.store, self.V, self.D, self.S, self.kind = store, vocab_size, embedding_size, num_sampled, loss
        self.embeddings = store.sparse_variable([vocab_size, embedding_size], Uniform(-1.0, 1.0), name="embeddings")
        self.nce_weights = store.sparse_variable([vocab_size, embedding_size],
                                                 TruncatedNormal(stddev=1.0 / math.sqrt(embedding_size)),
                                                 name="nce_weights")
        self.nce_biases = store.sparse_variable([vocab_size, 1], Zeros(), name="nce_biases")

    # -- autograd path
    def loss(self, centers: torch.Tensor, labels: torch.Tensor, seed: int = 0) -> torch.Tensor:
        embed = ops.embedding_lookup(self.embeddings, centers)
        fn = ops.nce_loss if self.kind == "nce" else ops.sampled_softmax_loss
        return fn(self.nce_weights, self.nce_biases, labels.reshape(-1), embed, self.S, self.V, seed=seed)

    # -- fused path
    def train_step(self, centers: torch.Tensor, labels: torch.Tensor, lr: float, seed: int = 0,
                   seed_tensor: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One SGD step (forward, backward, sparse update); returns the mean loss (device scalar)."""
        emb, W, b = self.embeddings.table, self.nce_weights.table, self.nce_biases.table
        x, y = centers.reshape(-1), labels.reshape(-1)
        B = x.numel()
        sid, logq_s = log_uniform_sample(self.S, self.V, seed, x.device, seed_tensor)
        logq_t = log_uniform_logq(y, self.V, self.S)
        E = gather_rows(emb, x)
        Wt, Ws = gather_rows(W, y), gather_rows(W, sid)
        bt, bs = gather_rows(b, y).reshape(-1), gather_rows(b, sid).reshape(-1)
        softmax = self.kind == "sampled_softmax"
        loss, dE, dWt, dbt, dWs, dbs = sampled_loss_grads(E, Wt, bt, Ws, bs, logq_t, logq_s,
                                                          y if softmax else None, sid if softmax else None,
                                                          softmax, 1.0 / B)
        scatter_add_rows(emb, x, dE, -lr)
        scatter_add_rows(W, y, dWt, -lr)
        scatter_add_rows(W, sid, dWs, -lr)
        scatter_add_rows(b, y, dbt, -lr)
        scatter_add_rows(b, sid, dbs, -lr)
        return loss.mean()

    # -- evaluation
    @torch.no_grad()
    def nearest(self, ids: torch.Tensor, k: int = 8, chunk: int = 1 << 18) -> torch.Tensor:
        """Top-k cosine neighbours (excluding self) of ``ids`` -- word2vec_basic's similarity op,
        computed in row chunks so the [len(ids), V] similarity matrix never materialises whole."""
        emb = self.embeddings.table
        q = emb[ids]
        q = q / q.norm(dim=1, keepdim=True).clamp_min(1e-12)
        best_v = torch.full((ids.numel(), k + 1), -2.0, device=emb.device)
        best_i = torch.zeros((ids.numel(), k + 1), dtype=torch.long, device=emb.device)
        for lo in range(0, self.V, chunk):
            blk = emb[lo:lo + chunk]
            blk = blk / blk.norm(dim=1, keepdim=True).clamp_min(1e-12)
            sim = q @ blk.t()
            v, i = sim.topk(min(k + 1, sim.shape[1]), dim=1)
            allv, alli = torch.cat([best_v, v], 1), torch.cat([best_i, i + lo], 1)
            best_v, sel = allv.topk(k + 1, dim=1)
            best_i = alli.gather(1, sel)
        out = []
        for r in range(ids.numel()):
            row = [int(j) for j in best_i[r] if int(j) != int(ids[r])][:k]
            out.append(row)
        return torch.tensor(out, dtype=torch.long)


def build_skipgram(device="cuda", vocab_size=1_000_000, embedding_size=128, num_sampled=64, loss="nce",
                   seed=0) -> Tuple[VariableStore, SkipGram]:
    store = VariableStore(device=device, compute_dtype=torch.float32, seed=seed)
    model = SkipGram(store, vocab_size, embedding_size, num_sampled, loss)
    store.finalize()
    return store, model
