"""MNIST softmax regression (BASELINE.json config 1: "MNIST softmax regression on CPU, batch=64").

The TF "MNIST for beginners" model -- y = softmax(x W + b), cross-entropy, plain SGD -- on this
framework's CPU path (PyTorch reference ops over the flat variable store); ``--device cuda`` runs
the same script on the HIP kernels (f32 MFMA GEMM + fused softmax-xent).  Reads the MNIST IDX
files from ``--data_dir`` when present, else deterministic synthetic MNIST.  ``--logs_path`` writes
``cost`` / ``accuracy`` scalars and the graph to a TensorBoard event file, ``--logdir`` checkpoints
periodically and resumes (the reference's conventions, R/distributed/distributed.py:120-138;
utils/runlog.py).

    python examples/mnist_softmax.py --batch_size=64 --train_steps=1000 --logs_path=/tmp/mnist_softmax
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_examples_amd import app, ops  # noqa: E402
from tensorflow_examples_amd.data.mnist import read_data_sets  # noqa: E402
from tensorflow_examples_amd.models.mnist_mlp import MnistSoftmax  # noqa: E402
from tensorflow_examples_amd.optim import GradientDescentOptimizer  # noqa: E402
from tensorflow_examples_amd.utils import runlog  # noqa: E402
from tensorflow_examples_amd.variables import VariableStore  # noqa: E402

flags = app.flags
flags.DEFINE_string("data_dir", "MNIST_data", "MNIST IDX directory (synthetic MNIST if absent)")
flags.DEFINE_integer("batch_size", 64, "batch size")
flags.DEFINE_integer("train_steps", 1000, "SGD steps")
flags.DEFINE_float("learning_rate", 0.5, "SGD learning rate")
flags.DEFINE_string("device", "cpu", "cpu | cuda")
flags.DEFINE_boolean("naive_xent", False, "TF1 reduce_mean(-reduce_sum(y_*log(softmax))) loss")
flags.DEFINE_integer("log_every", 100, "print every N steps")
runlog.define_flags(flags)
FLAGS = flags.FLAGS


def main(_):
    dev = torch.device(FLAGS.device)
    mnist = read_data_sets(FLAGS.data_dir, one_hot=True, seed=0)
    store = VariableStore(device=dev, compute_dtype=torch.float32, seed=0)
    model = MnistSoftmax(store)
    store.finalize()
    opt = GradientDescentOptimizer(store, FLAGS.learning_rate)
    log = runlog.RunLog(store, opt, FLAGS.logs_path, FLAGS.logdir, FLAGS.save_checkpoint_steps)
    start = log.restore()  # global step of the latest checkpoint in --logdir (0: fresh run)
    t0 = time.time()
    for step in range(start, FLAGS.train_steps):
        bx, by = mnist.train.next_batch(FLAGS.batch_size)
        x = torch.as_tensor(bx, device=dev)
        y = torch.as_tensor(by, device=dev)
        store.zero_grad()
        loss = model.loss(x, y, naive=FLAGS.naive_xent)
        loss.backward()
        opt.apply_gradients()
        if (step + 1) % FLAGS.log_every == 0:
            with torch.no_grad():
                acc = float(ops.accuracy(model.logits(x), y))
            print("step %d loss %.4f" % (step + 1, float(loss)), flush=True)
            log.scalars(step + 1, cost=float(loss), accuracy=acc)
        log.maybe_save(step + 1)
    dt = time.time() - t0
    with torch.no_grad():
        xt = torch.as_tensor(mnist.test.images, device=dev)
        yt = torch.as_tensor(mnist.test.labels, device=dev)
        acc = float(ops.accuracy(model.logits(xt), yt))
    print("accuracy %.4f" % acc)
    print("examples/sec %.1f" % (max(FLAGS.train_steps - start, 0) * FLAGS.batch_size / max(dt, 1e-9)))
    log.scalars(FLAGS.train_steps, test_accuracy=acc)
    saved = log.close(max(FLAGS.train_steps, start))
    if saved:
        print("saved", saved)
    return 0


if __name__ == "__main__":
    app.run(main)
