"""CPU (PyTorch reference path) tests of the LeNet-5, word2vec and char-LSTM model families and
their input pipelines."""
import numpy as np
import torch

from tensorflow_examples_amd import ops
from tensorflow_examples_amd.data.text import (CharCorpus, SkipGramBatcher, build_dataset, device_skipgram_batch,
                                               ptb_batches, synthetic_zipf_corpus)
from tensorflow_examples_amd.optim import AdamOptimizer, GradientDescentOptimizer, MomentumOptimizer
from tensorflow_examples_amd.ops import sparse as sp
from tensorflow_examples_amd.variables import Uniform, VariableStore


def test_lenet5_cpu_trains_and_padding_stays_zero():
    from tensorflow_examples_amd.models.lenet import build_lenet5, to_model_input
    from tensorflow_examples_amd.train import ClassifierTrainer
    store, m = build_lenet5(device="cpu", dtype=torch.float32)
    assert m.effective_params() == 61728
    tr = ClassifierTrainer(store, m, MomentumOptimizer(store, 0.05, 0.9))
    torch.manual_seed(0)
    x, y = to_model_input(torch.rand(32, 784), torch.float32), torch.randint(0, 10, (32,))
    first = float(tr.step(x, y))
    for _ in range(15):
        last = float(tr.step(x, y))
    assert last < 0.3 * first
    assert m.c1.w.master[6:].abs().sum() == 0 and m.c1.w.master[..., 1:].abs().sum() == 0
    assert m.c1.beta.master[6:].abs().sum() == 0 and m.c2.w.master[..., 6:].abs().sum() == 0


def test_pool_ops_cpu_grad():
    x = torch.randn(2, 6, 6, 8, requires_grad=True)
    y = ops.max_pool2d(x, 2)
    assert y.shape == (2, 3, 3, 8)
    y.sum().backward()
    assert x.grad.sum().item() == 2 * 9 * 8
    x2 = torch.randn(1, 5, 5, 8, requires_grad=True)
    ops.avg_pool2d(x2, 3, 2, 1).sum().backward()
    assert torch.isfinite(x2.grad).all()


def test_skipgram_batcher_matches_word2vec_basic_layout():
    b = SkipGramBatcher(np.arange(20), batch_size=8, num_skips=2, skip_window=1, seed=0)
    batch, labels = b.next()
    assert batch.tolist() == [1, 1, 2, 2, 3, 3, 4, 4]
    for c, l in zip(batch, labels[:, 0]):
        assert abs(int(l) - int(c)) == 1
    pairs = {(int(c), int(l)) for c, l in zip(batch, labels[:, 0])}
    assert len(pairs) == 8  # num_skips distinct contexts per center
    batch2, _ = b.next()
    assert batch2.tolist() == [5, 5, 6, 6, 7, 7, 8, 8]


def test_build_dataset_unk():
    words = "a b a c a b d e".split()
    data, count, d, rd = build_dataset(words, 3)
    assert count[0][0] == "UNK" and d["a"] == 1 and d["b"] == 2
    assert count[0][1] == 3  # c, d, e -> UNK
    assert rd[1] == "a" and data.tolist() == [1, 2, 1, 0, 1, 2, 0, 0]


def test_device_skipgram_batch_cpu_and_corpus():
    corpus = torch.from_numpy(synthetic_zipf_corpus(10000, 100, 0))
    assert corpus.dtype == torch.int32 and int(corpus.max()) < 100
    assert (corpus == 0).float().mean() > (corpus == 50).float().mean()
    c, l = device_skipgram_batch(corpus, 64, 2, seed=1)
    assert c.shape == l.shape == (64,)


def test_sampled_losses_cpu_reference_consistency():
    torch.manual_seed(0)
    B, S, D = 16, 8, 12
    E, Wt, Ws = torch.randn(B, D) * 0.3, torch.randn(B, D) * 0.3, torch.randn(S, D) * 0.3
    # NCE without corrections == explicit sigmoid cross-entropies
    loss, dE, *_ = sp._sampled_ref(E, Wt, None, Ws, None, None, None, None, None, False, 1.0)
    t = (E * Wt).sum(1)
    n = E @ Ws.t()
    ref = -torch.log(torch.sigmoid(t)) - torch.log(1 - torch.sigmoid(n)).sum(1)
    assert torch.allclose(loss, ref, atol=1e-4)
    # sampled softmax == full softmax xent over [true, sampled] with label 0
    loss2, *_ = sp._sampled_ref(E, Wt, None, Ws, None, None, None, None, None, True, 1.0)
    ref2 = torch.nn.functional.cross_entropy(torch.cat([t[:, None], n], 1), torch.zeros(B, dtype=torch.long),
                                             reduction="none")
    assert torch.allclose(loss2, ref2, atol=1e-5)


def test_word2vec_cpu_paths_agree_and_learn():
    from tensorflow_examples_amd.models.word2vec import build_skipgram
    sa, ma = build_skipgram("cpu", vocab_size=500, embedding_size=16, num_sampled=8, seed=2)
    sb, mb = build_skipgram("cpu", vocab_size=500, embedding_size=16, num_sampled=8, seed=2)
    opt = GradientDescentOptimizer(sb, 1.0)
    c, l = torch.randint(0, 500, (64,)), torch.randint(0, 500, (64,))
    la = ma.train_step(c, l, 1.0, seed=3)
    sb.zero_grad()
    lb = mb.loss(c, l, seed=3)
    lb.backward()
    opt.apply_gradients()
    assert abs(float(la) - float(lb)) < 1e-5
    for va, vb in zip(sa.sparse, sb.sparse):
        assert torch.allclose(va.table, vb.table, atol=1e-6)
    corpus = torch.from_numpy(synthetic_zipf_corpus(50000, 500, 1))
    losses = []
    for i in range(150):
        c, l = device_skipgram_batch(corpus, 128, 1, seed=i)
        losses.append(float(ma.train_step(c, l, 1.0, seed=100 + i)))
    assert np.mean(losses[-10:]) < 0.5 * np.mean(losses[:5])


def test_sparse_variable_checkpoint_roundtrip():
    store = VariableStore("cpu", seed=1)
    t = store.sparse_variable([10, 4], Uniform(-1, 1), name="emb")
    store.finalize()
    vals = {k: v.clone() for k, v in store.named_values().items()}
    t.table.zero_()
    store.load_named(vals)
    assert torch.equal(t.table, vals["emb"])
    assert store.num_params() == 40


def test_char_lstm_cpu_learns_pattern_with_clip():
    from tensorflow_examples_amd.models.char_lstm import LMTrainer, build_char_lstm
    rng = np.random.default_rng(0)
    ids = np.tile(rng.integers(0, 16, 30), 200)
    store, m = build_char_lstm("cpu", vocab_size=16, embed=16, hidden=32, layers=1, dtype=torch.float32)
    tr = LMTrainer(m, AdamOptimizer(store, 0.02), max_grad_norm=1.0)
    st, losses = None, []
    for _ in range(2):
        for x, y in ptb_batches(ids, 8, 15):
            l, st = tr.step(torch.from_numpy(x), torch.from_numpy(y), st)
            losses.append(float(l))
    assert losses[-1] < 0.3 * losses[0]


def test_char_corpus_and_ptb_batches():
    cc = CharCorpus("hello world")
    assert cc.decode(cc.ids) == "hello world"
    ids = np.arange(101)
    wins = list(ptb_batches(ids, 4, 5))
    assert len(wins) == 4 and wins[0][0].shape == (5, 4)
    x, y = wins[1]
    assert (y == x + 1).all() and x[0, 0] == 5 and x[0, 1] == 30
