"""LeNet-5 on MNIST (BASELINE.json config 2: "MNIST LeNet-5 CNN bf16 on one MI355X").

bf16 NHWC conv (implicit-GEMM MFMA) + fused BN/ReLU + max-pool + bf16 FC GEMMs, momentum SGD
fused over the flat store; optional HIP-graph capture of the whole step (``--graph``: LeNet is
launch-bound at small batch).  MNIST IDX files from ``--data_dir`` when present, else synthetic.
``--logs_path`` / ``--logdir`` / ``--save_checkpoint_steps``: event-file scalars and periodic
checkpoints with resume (utils/runlog.py; R/distributed/distributed.py:120-138).

    python examples/lenet5.py --batch_size=256 --epochs=2
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorflow_examples_amd import app, ops  # noqa: E402
from tensorflow_examples_amd.data.mnist import read_data_sets  # noqa: E402
from tensorflow_examples_amd.data.pipeline import DevicePrefetcher, batches  # noqa: E402
from tensorflow_examples_amd.models.lenet import build_lenet5, to_model_input  # noqa: E402
from tensorflow_examples_amd.optim import MomentumOptimizer  # noqa: E402
from tensorflow_examples_amd.train import ClassifierTrainer  # noqa: E402
from tensorflow_examples_amd.utils import runlog  # noqa: E402

flags = app.flags
flags.DEFINE_string("data_dir", "MNIST_data", "MNIST IDX directory (synthetic MNIST if absent)")
flags.DEFINE_integer("batch_size", 256, "batch size")
flags.DEFINE_integer("epochs", 2, "training epochs")
flags.DEFINE_integer("max_steps", 0, "stop after N steps (0 = full epochs)")
flags.DEFINE_float("learning_rate", 0.05, "momentum-SGD learning rate")
flags.DEFINE_string("device", "auto", "auto | cuda | cpu")
flags.DEFINE_boolean("graph", False, "capture the training step in a HIP graph")
flags.DEFINE_integer("log_every", 100, "print / log scalars every N steps")
runlog.define_flags(flags)
FLAGS = flags.FLAGS


def main(_):
    use_cuda = FLAGS.device == "cuda" or (FLAGS.device == "auto" and torch.cuda.is_available())
    dev = torch.device("cuda", 0) if use_cuda else torch.device("cpu")
    dtype = torch.bfloat16 if use_cuda else torch.float32
    mnist = read_data_sets(FLAGS.data_dir, one_hot=False, seed=0)
    store, model = build_lenet5(device=dev, dtype=dtype, seed=0)
    print("LeNet-5: %d parameters (%d padded)" % (model.effective_params(), store.num_params()))
    opt = MomentumOptimizer(store, FLAGS.learning_rate, 0.9)
    trainer = ClassifierTrainer(store, model, opt, fuse_zero_grad=True)  # optimizer clears the grads
    log = runlog.RunLog(store, opt, FLAGS.logs_path, FLAGS.logdir, FLAGS.save_checkpoint_steps)
    start = log.restore()  # resume from --logdir's latest checkpoint (0: fresh run)
    xtr, ytr = mnist.train.images, mnist.train.labels.astype(np.int64)
    total = FLAGS.max_steps or FLAGS.epochs * (len(xtr) // FLAGS.batch_size)
    step, t0, seen = start, time.time(), 0
    for ep in range(FLAGS.epochs):
        if step >= total:
            break
        for xb, yb in DevicePrefetcher(batches([xtr, ytr], FLAGS.batch_size, seed=ep), dev):
            x = to_model_input(xb, dtype)
            if FLAGS.graph and use_cuda and trainer.graph is None:
                trainer.capture(x, yb)
            loss = trainer.step(x, yb)
            step += 1
            seen += xb.shape[0]
            if step % FLAGS.log_every == 0:
                with torch.no_grad():  # training-batch accuracy, as the reference's summary op
                    acc = float(ops.accuracy(model(x, training=False), yb))
                print("epoch %d step %d loss %.4f" % (ep + 1, step, float(loss)), flush=True)
                log.scalars(step, cost=float(loss), accuracy=acc)
            log.maybe_save(step)
            if step >= total:
                break
    if use_cuda:
        torch.cuda.synchronize()
    dt = time.time() - t0
    correct = 0.0
    xte, yte = mnist.test.images, mnist.test.labels.astype(np.int64)
    with torch.no_grad():
        for i in range(0, len(xte), 1000):
            x = to_model_input(torch.as_tensor(xte[i:i + 1000], device=dev), dtype)
            y = torch.as_tensor(yte[i:i + 1000], device=dev)
            correct += float(ops.accuracy(model(x, training=False), y)) * len(y)
    print("test accuracy %.4f" % (correct / len(xte)))
    print("images/sec %.1f (%d steps, batch %d)" % (seen / max(dt, 1e-9), step - start, FLAGS.batch_size))
    log.scalars(step, test_accuracy=correct / len(xte))
    saved = log.close(step)
    if saved:
        print("saved", saved)
    return 0


if __name__ == "__main__":
    app.run(main)
