#!/usr/bin/env python3
"""Throughput of the non-headline BASELINE.json configs, ours vs stock PyTorch-ROCm, one JSON line each.

    python scripts/bench_models.py --model lenet5   [--impl native|torch] [--graph]
    python scripts/bench_models.py --model word2vec [--impl native|torch] [--graph]
    python scripts/bench_models.py --model char_lstm [--impl native|torch] [--graph]
    python scripts/bench_models.py --model resnet50 --impl torch [--graph]   (stock PyTorch comparison)
    python scripts/bench_models.py --model mnist_softmax   (CPU, config 1)

Same timing discipline as bench.py: W untimed warmup steps, synchronize, K timed steps,
synchronize.  Synthetic data of the config's shape, random-init weights.  ``--impl torch`` is
the stock eager PyTorch formulation of the same model (nn.Conv2d/BatchNorm/MaxPool, nn.Embedding
+ manual NCE with sparse SGD, nn.LSTM = MIOpen RNN) for a labelled comparison.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(step, steps, warmup, cuda=True):
    for i in range(warmup):
        step(i)
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        out = step(i)
    if cuda:
        torch.cuda.synchronize()
    return time.perf_counter() - t0, out


def graphed(step_fn):
    """Capture ``step_fn()`` into a HIP graph; returns a replay callable."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step_fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = step_fn()
    return lambda: (g.replay(), out)[1]


# ---------------------------------------------------------------- LeNet-5
def bench_lenet(a, dev):
    B = a.batch or 256
    x = torch.rand(B, 784, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    if a.impl == "native":
        from tensorflow_examples_amd.models.lenet import build_lenet5, to_model_input
        from tensorflow_examples_amd.optim import MomentumOptimizer
        from tensorflow_examples_amd.train import ClassifierTrainer
        store, m = build_lenet5(device=dev)
        tr = ClassifierTrainer(store, m, MomentumOptimizer(store, 0.05, 0.9), fuse_zero_grad=True)
        xi = to_model_input(x)
        if a.graph:
            tr.capture(xi, y)
        step = lambda i: tr.step(xi, y)  # noqa: E731
    else:
        import torch.nn as nn
        net = nn.Sequential(nn.Conv2d(1, 6, 5, padding=2, bias=False), nn.BatchNorm2d(6), nn.ReLU(), nn.MaxPool2d(2),
                            nn.Conv2d(6, 16, 5, bias=False), nn.BatchNorm2d(16), nn.ReLU(), nn.MaxPool2d(2),
                            nn.Flatten(), nn.Linear(400, 120), nn.ReLU(), nn.Linear(120, 84), nn.ReLU(),
                            nn.Linear(84, 10)).to(dev)
        opt = torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9, foreach=True)
        xi = x.view(B, 1, 28, 28)

        def one():
            opt.zero_grad(set_to_none=False)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = nn.functional.cross_entropy(net(xi), y)
            loss.backward()
            opt.step()
            return loss.detach()
        run = graphed(one) if a.graph else one
        step = lambda i: run()  # noqa: E731
    dt, loss = timed(step, a.steps, a.warmup)
    return dict(metric="images/sec LeNet-5 MNIST bf16 (1 GPU)", value=B * a.steps / dt, unit="images/sec",
                ms_per_step=dt * 1e3 / a.steps, config=dict(model="LeNet-5 (BN)", global_batch=B, seq_len=None),
                final_loss=float(loss))


# ---------------------------------------------------------------- word2vec
def bench_word2vec(a, dev):
    B, V, D, S = a.batch or 4096, a.vocab or 1_000_000, 128, 64
    from tensorflow_examples_amd.data.text import device_skipgram_batch, synthetic_zipf_corpus
    corpus = torch.from_numpy(synthetic_zipf_corpus(10_000_000, V, 0)).to(dev)
    counter = torch.zeros(1, dtype=torch.long, device=dev)
    if a.impl == "native":
        from tensorflow_examples_amd.models.word2vec import build_skipgram
        store, m = build_skipgram(dev, V, D, S)

        def one():
            c, l = device_skipgram_batch(corpus, B, 1, seed=1, seed_tensor=counter)
            loss = m.train_step(c, l, 1.0, seed=2, seed_tensor=counter)
            counter.add_(1)
            return loss
    else:
        import torch.nn as nn
        emb = nn.Embedding(V, D, sparse=True).to(dev)
        nn.init.uniform_(emb.weight, -1, 1)
        w = nn.Embedding(V, D, sparse=True).to(dev)
        nn.init.trunc_normal_(w.weight, std=1 / math.sqrt(D))
        b = nn.Embedding(V, 1, sparse=True).to(dev)
        nn.init.zeros_(b.weight)
        opt = torch.optim.SGD(list(emb.parameters()) + list(w.parameters()) + list(b.parameters()), lr=1.0)
        lrange = math.log(V + 1)

        def one():
            c, l = device_skipgram_batch(corpus, B, 1, seed=1, seed_tensor=counter)
            u = torch.rand(S, device=dev, dtype=torch.float64)
            sid = (torch.exp(u * lrange).floor().long() - 1).clamp(0, V - 1)
            lq = lambda k: torch.log(S * torch.log((k.double() + 2) / (k.double() + 1)) / lrange).float()  # noqa
            e = emb(c)
            t = (e * w(l)).sum(1) + b(l).squeeze(1) - lq(l)
            n = e @ w(sid).t() + b(sid).squeeze(1) - lq(sid)
            loss = (nn.functional.softplus(-t) + nn.functional.softplus(n).sum(1)).mean()
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            counter.add_(1)
            return loss.detach()
    run = graphed(one) if (a.graph and a.impl == "native") else one
    dt, loss = timed(lambda i: run(), a.steps, a.warmup)
    return dict(metric="examples/sec word2vec skip-gram NCE, 1M x 128 embedding (1 GPU)", value=B * a.steps / dt,
                unit="examples/sec", ms_per_step=dt * 1e3 / a.steps,
                config=dict(model="skip-gram NCE V=%d D=%d S=%d" % (V, D, S), global_batch=B, seq_len=None),
                final_loss=float(loss))


# ---------------------------------------------------------------- char-LSTM
def bench_char_lstm(a, dev):
    B, T, H, E, L, V = a.batch or 64, a.seq or 100, 512, 128, 2, 65
    x = torch.randint(0, V, (T, B), device=dev)
    y = torch.randint(0, V, (T, B), device=dev)
    if a.impl == "native":
        from tensorflow_examples_amd.models.char_lstm import LMTrainer, build_char_lstm
        from tensorflow_examples_amd.optim import GradientDescentOptimizer
        store, m = build_char_lstm(dev, V, E, H, L)
        tr = LMTrainer(m, GradientDescentOptimizer(store, 1.0), max_grad_norm=5.0)
        state = [m.zero_state(B, dev)]

        def one():
            loss, st = tr.step(x, y, state[0])
            return loss
    else:
        import torch.nn as nn

        class Net(nn.Module):
            def __init__(self):
                super().__init__()
                self.emb = nn.Embedding(V, E)
                self.rnn = nn.LSTM(E, H, L)
                self.out = nn.Linear(H, V)

            def forward(self, x, st):
                o, st = self.rnn(self.emb(x), st)
                return self.out(o).view(-1, V), st

        net = Net().to(dev)
        opt = torch.optim.SGD(net.parameters(), lr=1.0, foreach=True)
        st0 = (torch.zeros(L, B, H, device=dev), torch.zeros(L, B, H, device=dev))

        def one():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits, _ = net(x, st0)
                loss = nn.functional.cross_entropy(logits.float(), y.view(-1))
            loss.backward()
            torch.nn.utils.clip_grad_norm_(net.parameters(), 5.0, foreach=True)
            opt.step()
            return loss.detach()
    run = graphed(one) if a.graph else one
    dt, loss = timed(lambda i: run(), a.steps, a.warmup)
    return dict(metric="tokens/sec char-LSTM 2x512 (1 GPU)", value=B * T * a.steps / dt, unit="tokens/sec",
                ms_per_step=dt * 1e3 / a.steps,
                config=dict(model="char-LSTM V=%d E=%d H=%d L=%d" % (V, E, H, L), global_batch=B, seq_len=T),
                final_loss=float(loss))


# ---------------------------------------------------------------- ResNet-50/CIFAR (stock PyTorch only)
def bench_resnet50(a, dev):
    """The headline step in stock PyTorch-ROCm (torch.nn + MIOpen, channels_last, bf16 autocast,
    torch.optim.SGD foreach), optionally captured into a HIP graph -- a stronger comparison point than the
    eager baseline of ``bench.py --impl torch`` (the native step is ``bench.py``).  The batch is a fixed
    device-resident normalised image tensor."""
    assert a.impl == "torch", "the native ResNet-50 step is bench.py"
    import torch.nn as nn
    from tensorflow_examples_amd.models.torch_baseline import TorchResNet50Cifar
    B = a.batch or 256
    torch.manual_seed(0)
    net = TorchResNet50Cifar().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4, foreach=True)
    x = torch.randn(B, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (B,), device=dev)

    def one():
        opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = nn.functional.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
        return loss.detach()
    run = graphed(one) if a.graph else one
    dt, loss = timed(lambda i: run(), a.steps, a.warmup)
    return dict(metric="images/sec ResNet-50/CIFAR-10 bf16 (1 GPU)", value=B * a.steps / dt, unit="images/sec",
                ms_per_step=dt * 1e3 / a.steps,
                config=dict(model="ResNet-50 (CIFAR-10 adaptation: 3x3 stem, bottleneck [3,4,6,3])", global_batch=B,
                            seq_len=None), final_loss=float(loss))


# ---------------------------------------------------------------- MNIST softmax (CPU)
def bench_mnist_softmax(a, dev):
    from tensorflow_examples_amd.models.mnist_mlp import MnistSoftmax
    from tensorflow_examples_amd.optim import GradientDescentOptimizer
    from tensorflow_examples_amd.variables import VariableStore
    B = a.batch or 64
    store = VariableStore("cpu", seed=0)
    m = MnistSoftmax(store)
    store.finalize()
    opt = GradientDescentOptimizer(store, 0.5)
    x = torch.rand(B, 784)
    y = torch.nn.functional.one_hot(torch.randint(0, 10, (B,)), 10).float()

    def one(i):
        store.zero_grad()
        loss = m.loss(x, y)
        loss.backward()
        opt.apply_gradients()
        return loss.detach()
    dt, loss = timed(one, a.steps, a.warmup, cuda=False)
    return dict(metric="examples/sec MNIST softmax regression CPU", value=B * a.steps / dt, unit="examples/sec",
                ms_per_step=dt * 1e3 / a.steps, config=dict(model="softmax 784->10", global_batch=B, seq_len=None),
                final_loss=float(loss))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", required=True, choices=["lenet5", "word2vec", "char_lstm", "mnist_softmax", "resnet50"])
    ap.add_argument("--impl", choices=["native", "torch"], default="native")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--seq", type=int, default=0)
    ap.add_argument("--vocab", type=int, default=0)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args(argv)
    dev = torch.device("cpu") if a.model == "mnist_softmax" else torch.device("cuda", 0)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    fn = {"lenet5": bench_lenet, "word2vec": bench_word2vec, "char_lstm": bench_char_lstm,
          "mnist_softmax": bench_mnist_softmax, "resnet50": bench_resnet50}[a.model]
    rec = fn(a, dev)
    rec.update(impl=a.impl, hip_graph=bool(a.graph), steps=a.steps, warmup=a.warmup, n_gpus=1 if dev.type == "cuda" else 0,
               dtype="bf16" if a.model in ("lenet5", "char_lstm", "resnet50") else "fp32", data="synthetic")
    rec["value"] = round(rec["value"], 1)
    rec["ms_per_step"] = round(rec["ms_per_step"], 3)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
