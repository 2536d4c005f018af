"""word2vec skip-gram with NCE / sampled-softmax loss (BASELINE.json config 4: "word2vec skip-gram
1M-row embedding on one MI355X").

TF ``word2vec_basic`` on this framework: 1M x 128 embedding + NCE tables resident in HBM as
sparse variables, log-uniform negatives (64 per batch), fused loss/gradient kernel, sparse SGD
(scatter-add) updates.  The corpus is a text file (``--train_data``, e.g. text8) when present, else a
synthetic Zipfian corpus; batches are drawn on the GPU by one kernel (random center + in-window
context).  ``--graph`` captures the whole step (batch generation, sampling, forward, backward,
update) in a HIP graph and replays it.  ``--logs_path`` writes the average-loss scalar and the graph to
an event file, ``--logdir`` checkpoints the tables (and the batch-generator counter) periodically and
resumes (utils/runlog.py; the reference's conventions, R/distributed/distributed.py:120-138).

    python examples/word2vec.py --vocabulary_size=1000000 --batch_size=128 --num_steps=100001
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorflow_examples_amd import app  # noqa: E402
from tensorflow_examples_amd.data.text import build_dataset, device_skipgram_batch, synthetic_zipf_corpus  # noqa: E402
from tensorflow_examples_amd.models.word2vec import build_skipgram  # noqa: E402
from tensorflow_examples_amd.utils import runlog  # noqa: E402

flags = app.flags
flags.DEFINE_string("train_data", "", "whitespace-tokenised text corpus (synthetic Zipf corpus if absent)")
flags.DEFINE_integer("vocabulary_size", 1000000, "vocabulary (embedding rows)")
flags.DEFINE_integer("embedding_size", 128, "embedding width")
flags.DEFINE_integer("num_sampled", 64, "negative samples per batch")
flags.DEFINE_integer("batch_size", 128, "examples per step")
flags.DEFINE_integer("skip_window", 1, "context words on each side")
flags.DEFINE_integer("num_steps", 20001, "training steps")
flags.DEFINE_float("learning_rate", 1.0, "SGD learning rate")
flags.DEFINE_string("loss", "nce", "nce | sampled_softmax")
flags.DEFINE_integer("corpus_words", 20000000, "synthetic corpus length")
flags.DEFINE_boolean("graph", False, "capture the training step in a HIP graph")
flags.DEFINE_integer("log_every", 2000, "print the average loss every N steps")
runlog.define_flags(flags, save_steps_default=10000)
FLAGS = flags.FLAGS


def main(_):
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    V = FLAGS.vocabulary_size
    rev = None
    if FLAGS.train_data and os.path.exists(FLAGS.train_data):
        with open(FLAGS.train_data) as f:
            words = f.read().split()
        data, count, dictionary, rev = build_dataset(words, V)
        V = min(V, len(count))
        print("corpus %s: %d words, vocabulary %d" % (FLAGS.train_data, len(data), V))
    else:
        data = synthetic_zipf_corpus(FLAGS.corpus_words, V, seed=0)
        print("synthetic Zipf corpus: %d words, vocabulary %d" % (len(data), V))
    corpus = torch.from_numpy(np.ascontiguousarray(data, dtype=np.int32)).to(dev)
    store, model = build_skipgram(dev, V, FLAGS.embedding_size, FLAGS.num_sampled, FLAGS.loss, seed=0)
    counter = torch.zeros(1, dtype=torch.long, device=dev)
    lr, B = FLAGS.learning_rate, FLAGS.batch_size
    # the device counter seeds the batch generator and the sampler: checkpointed with the tables, so a
    # resumed run continues the same stream
    log = runlog.RunLog(store, None, FLAGS.logs_path, FLAGS.logdir, FLAGS.save_checkpoint_steps,
                        extra_state={"skipgram/step_counter": counter})
    start = log.restore()

    def step():
        c, l = device_skipgram_batch(corpus, B, FLAGS.skip_window, seed=1, seed_tensor=counter)
        loss = model.train_step(c, l, lr, seed=2, seed_tensor=counter)
        counter.add_(1)
        return loss

    if FLAGS.graph and dev.type == "cuda":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static_loss = step()
        run = lambda: (g.replay(), static_loss)[1]  # noqa: E731
    else:
        run = step
    avg = torch.zeros((), device=dev)
    t0 = time.time()
    t_last = t0
    for i in range(start, FLAGS.num_steps):
        avg += run()
        if (i + 1) % FLAGS.log_every == 0:
            a = float(avg) / FLAGS.log_every
            now = time.time()
            print("Average loss at step %d: %.4f  (%.0f examples/sec)" %
                  (i + 1, a, FLAGS.log_every * B / (now - t_last)), flush=True)
            log.scalars(i + 1, loss=a)
            avg.zero_()
            t_last = now
        log.maybe_save(i + 1)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    valid = torch.arange(0, 16 * 6, 6, device=dev)
    near = model.nearest(valid, 8)
    for r, w in enumerate(valid.tolist()[:4]):
        name = (lambda k: rev.get(k, str(k))) if rev else str
        print("Nearest to %s: %s" % (name(w), ", ".join(name(int(k)) for k in near[r])))
    print("examples/sec %.1f" % (max(FLAGS.num_steps - start, 0) * B / max(dt, 1e-9)))
    saved = log.close(max(FLAGS.num_steps, start))
    if saved:
        print("saved", saved)
    return 0


if __name__ == "__main__":
    app.run(main)
