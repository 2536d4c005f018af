"""Text pipelines for word2vec (skip-gram) and the char-LSTM language model.

* :func:`build_dataset` / :class:`SkipGramBatcher` -- TF ``word2vec_basic`` semantics
  (``[['UNK', -1]] + most_common(n-1)`` vocabulary, sequential ``generate_batch`` with a
  sliding window, ``num_skips`` distinct contexts per center);
* :func:`device_skipgram_batch` -- the MI355X path: the corpus lives in HBM as int32 and each
  batch is drawn by one HIP kernel (random center + random in-window context, counter-hash RNG;
  HIP-graph capturable through a device step counter);
* :func:`synthetic_zipf_corpus` -- Zipfian word ids (there is no text8 download on the box);
* :class:`CharCorpus` / :func:`ptb_batches` -- PTB-style ``[batch, num_steps]`` windows over a
  character stream with carried state (truncated BPTT), like ``reader.ptb_producer``.
"""
from __future__ import annotations

import collections
import random
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import _native


# ---------------------------------------------------------------- word level
def synthetic_zipf_corpus(n_words: int, vocab_size: int, seed: int = 0, s: float = 1.0) -> np.ndarray:
    """int32 word ids with P(k) ~ 1/(k+1)^s (k = frequency rank), like natural text."""
    rng = np.random.default_rng(seed)
    ranks = np.arange(1, vocab_size + 1, dtype=np.float64)
    p = ranks ** -s
    p /= p.sum()
    return rng.choice(vocab_size, size=n_words, p=p).astype(np.int32)


def build_dataset(words: Sequence[str], n_words: int):
    """word2vec_basic.build_dataset: (data ids, count, dictionary, reversed_dictionary)."""
    count = [["UNK", -1]]
    count.extend(collections.Counter(words).most_common(n_words - 1))
    dictionary: Dict[str, int] = {w: i for i, (w, _) in enumerate(count)}
    data = np.fromiter((dictionary.get(w, 0) for w in words), dtype=np.int32, count=len(words))
    count[0][1] = int((data == 0).sum())
    reversed_dictionary = {i: w for w, i in dictionary.items()}
    return data, count, dictionary, reversed_dictionary


class SkipGramBatcher:
    """word2vec_basic.generate_batch: slide a (2*skip_window+1) window over ``data``; for every
    center emit ``num_skips`` distinct context words.  Host-side, deterministic per ``seed``."""

    def __init__(self, data: np.ndarray, batch_size: int, num_skips: int, skip_window: int, seed: int = 0):
        assert batch_size % num_skips == 0 and num_skips <= 2 * skip_window
        self.data = np.asarray(data, dtype=np.int64)
        self.batch_size, self.num_skips, self.skip_window = batch_size, num_skips, skip_window
        self.data_index = 0
        self.rng = random.Random(seed)

    def next(self) -> Tuple[np.ndarray, np.ndarray]:
        span = 2 * self.skip_window + 1
        batch = np.empty(self.batch_size, dtype=np.int64)
        labels = np.empty((self.batch_size, 1), dtype=np.int64)
        n = len(self.data)
        buf = collections.deque(maxlen=span)
        if self.data_index + span > n:
            self.data_index = 0
        buf.extend(self.data[self.data_index:self.data_index + span])
        self.data_index += span
        for i in range(self.batch_size // self.num_skips):
            context = [w for w in range(span) if w != self.skip_window]
            for j, cw in enumerate(self.rng.sample(context, self.num_skips)):
                batch[i * self.num_skips + j] = buf[self.skip_window]
                labels[i * self.num_skips + j, 0] = buf[cw]
            if self.data_index == n:
                buf.extend(self.data[0:span])
                self.data_index = span
            else:
                buf.append(self.data[self.data_index])
                self.data_index += 1
        self.data_index = (self.data_index + n - span) % n  # backtrack (word2vec_basic)
        return batch, labels


def device_skipgram_batch(corpus: torch.Tensor, batch_size: int, skip_window: int, seed: int = 0,
                          seed_tensor: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Random (center, context) int64 pairs from an int32 corpus tensor (one HIP kernel on GPU)."""
    if _native.use_native(corpus):
        return torch.ops.tfx.skipgram_batch(corpus, batch_size, skip_window, int(seed) & 0x7FFFFFFFFFFFFFFF,
                                            seed_tensor)
    if seed_tensor is not None:
        seed = int(seed) + int(seed_tensor.reshape(-1)[0])
    g = torch.Generator().manual_seed(int(seed))
    n = corpus.numel()
    p = torch.randint(skip_window, n - skip_window, (batch_size,), generator=g)
    o = torch.randint(1, skip_window + 1, (batch_size,), generator=g)
    sign = torch.randint(0, 2, (batch_size,), generator=g) * 2 - 1
    c = corpus.cpu().long()
    return c[p].to(corpus.device), c[p + sign * o].to(corpus.device)


# ---------------------------------------------------------------- char level
class CharCorpus:
    """Character vocabulary + id stream (``reader._build_vocab`` / ``_file_to_word_ids``, per char)."""

    def __init__(self, text: str):
        self.chars: List[str] = sorted(set(text))
        self.vocab = {c: i for i, c in enumerate(self.chars)}
        self.ids = np.fromiter((self.vocab[c] for c in text), dtype=np.int64, count=len(text))

    @property
    def vocab_size(self) -> int:
        return len(self.chars)

    def decode(self, ids) -> str:
        return "".join(self.chars[int(i)] for i in ids)


def synthetic_char_ids(n: int, vocab_size: int = 65, seed: int = 0) -> np.ndarray:
    """A learnable synthetic character stream: a random order-2 Markov chain over the vocabulary
    (peaked transitions), so a trained LSTM's loss falls well below log(vocab)."""
    rng = np.random.default_rng(seed)
    trans = rng.dirichlet(np.full(vocab_size, 0.05), size=(vocab_size, vocab_size))
    cdf = np.cumsum(trans, axis=-1)
    out = np.empty(n, dtype=np.int64)
    out[0], out[1] = 0, 1
    u = rng.random(n)
    for i in range(2, n):
        out[i] = min(int(np.searchsorted(cdf[out[i - 2], out[i - 1]], u[i])), vocab_size - 1)
    return out


def ptb_batches(ids: np.ndarray, batch_size: int, num_steps: int) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
    """reader.ptb_producer: split the stream into ``batch_size`` rows, yield [num_steps, batch]
    (time-major) input/target windows in order, so the LSTM state carries across windows."""
    n = len(ids) // batch_size
    data = np.asarray(ids[:n * batch_size]).reshape(batch_size, n)
    epoch = (n - 1) // num_steps
    for i in range(epoch):
        x = data[:, i * num_steps:(i + 1) * num_steps]
        y = data[:, i * num_steps + 1:(i + 1) * num_steps + 1]
        yield np.ascontiguousarray(x.T), np.ascontiguousarray(y.T)
