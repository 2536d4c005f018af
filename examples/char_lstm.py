"""Character-level LSTM language model (BASELINE.json config 5: "PTB-shaped char-LSTM language model
DP on 4xMI355X").

ptb_word_lm-style training per character: [num_steps, batch] windows with the LSTM state carried
across windows (truncated BPTT), stacked LSTM layers with the four gates in one MFMA GEMM,
softmax projection, SGD with clip_by_global_norm and LR decay after ``--max_epoch`` epochs.  One
process per GPU under torchrun: each rank takes its own slice of the batch rows; gradients are
all-reduced in buckets overlapped with backward.  Text from ``--data_path`` when present, else a
synthetic order-2 Markov character stream.  ``--logs_path`` writes cost / perplexity scalars and the
graph to an event file, ``--logdir`` checkpoints periodically and resumes (utils/runlog.py; the
reference's conventions, R/distributed/distributed.py:120-138).

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/char_lstm.py --batch_size=64
"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tensorflow_examples_amd import app  # noqa: E402
from tensorflow_examples_amd.data.text import CharCorpus, ptb_batches, synthetic_char_ids  # noqa: E402
from tensorflow_examples_amd.data.pipeline import DevicePrefetcher  # noqa: E402
from tensorflow_examples_amd.models.char_lstm import LMTrainer, build_char_lstm  # noqa: E402
from tensorflow_examples_amd.optim import GradientDescentOptimizer  # noqa: E402
from tensorflow_examples_amd.parallel import GradAllReduce, broadcast_variables, init_distributed  # noqa: E402
from tensorflow_examples_amd.utils import runlog  # noqa: E402

flags = app.flags
flags.DEFINE_string("data_path", "", "text file to model (synthetic character stream if absent)")
flags.DEFINE_integer("batch_size", 64, "sequences per GPU")
flags.DEFINE_integer("num_steps", 100, "unrolled time steps (truncated BPTT window)")
flags.DEFINE_integer("hidden_size", 512, "LSTM width")
flags.DEFINE_integer("embed_size", 128, "character embedding width")
flags.DEFINE_integer("num_layers", 2, "stacked LSTM layers")
flags.DEFINE_float("learning_rate", 1.0, "SGD learning rate")
flags.DEFINE_float("lr_decay", 0.5, "LR multiplier per epoch after max_epoch")
flags.DEFINE_integer("max_epoch", 4, "epochs at the initial learning rate")
flags.DEFINE_integer("max_max_epoch", 6, "total epochs")
flags.DEFINE_float("max_grad_norm", 5.0, "clip_by_global_norm bound")
flags.DEFINE_integer("max_steps", 0, "stop after N steps (0 = full epochs)")
flags.DEFINE_integer("synthetic_chars", 2000000, "synthetic stream length")
flags.DEFINE_integer("log_every", 50, "print / log scalars every N steps")
runlog.define_flags(flags)
FLAGS = flags.FLAGS


def main(_):
    dev = init_distributed(device="cuda" if torch.cuda.is_available() else "cpu")
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if FLAGS.data_path and os.path.exists(FLAGS.data_path):
        with open(FLAGS.data_path) as f:
            cc = CharCorpus(f.read())
        ids, vocab = cc.ids, cc.vocab_size
    else:
        vocab = 65
        ids = synthetic_char_ids(FLAGS.synthetic_chars, vocab, seed=0)
    n_val = len(ids) // 20
    train, valid = ids[:-n_val], ids[-n_val:]
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    store, model = build_char_lstm(dev, vocab_size=vocab, embed=FLAGS.embed_size, hidden=FLAGS.hidden_size,
                                   layers=FLAGS.num_layers, dtype=dtype, seed=0)
    opt = GradientDescentOptimizer(store, FLAGS.learning_rate)
    log = runlog.RunLog(store, opt, FLAGS.logs_path, FLAGS.logdir, FLAGS.save_checkpoint_steps, rank=rank)
    start = log.restore()  # every rank restores; the broadcast below keeps them identical
    broadcast_variables(store)
    dp = GradAllReduce(store) if world > 1 else None
    trainer = LMTrainer(model, opt, dp, FLAGS.max_grad_norm)
    if rank == 0:
        print("char-LSTM: vocab %d, %d x %d LSTM, %d params, %d GPU(s)" %
              (vocab, FLAGS.num_layers, FLAGS.hidden_size, store.num_params(), world))
    B, T = FLAGS.batch_size, FLAGS.num_steps
    steps_per_epoch = max(1, (len(train) // (B * world) - 1) // T)
    step, tokens, t0 = start, 0, time.time()
    for ep in range(start // steps_per_epoch, FLAGS.max_max_epoch):
        opt.set_learning_rate(FLAGS.learning_rate * FLAGS.lr_decay ** max(ep + 1 - FLAGS.max_epoch, 0))
        state, costs, iters = None, 0.0, 0
        # global batch = B * world rows; rank r trains rows [r*B, (r+1)*B).  Windows reach the GPU
        # through the pinned ring (async H2D on a copy stream, two windows ahead of the step).  A resumed
        # run skips the windows of the epoch its checkpoint had already trained on
        skip = step - ep * steps_per_epoch
        shard = ((x[:, rank * B:(rank + 1) * B], y[:, rank * B:(rank + 1) * B])
                 for k, (x, y) in enumerate(ptb_batches(train, B * world, T)) if k >= skip)
        for xs, ys in DevicePrefetcher(shard, dev, depth=2):
            loss, state = trainer.step(xs, ys, state)
            step += 1
            tokens += B * T * world
            if step % FLAGS.log_every == 0:
                costs += float(loss)
                iters += 1
                trainer.check()  # a timed-out persistent-LSTM hand-off: steps skipped, per-step kernels from here
                if rank == 0:
                    print("epoch %d step %d perplexity %.3f  %.0f tokens/sec" %
                          (ep + 1, step, math.exp(costs / iters), tokens / (time.time() - t0)), flush=True)
                    log.scalars(step, cost=float(loss), perplexity=math.exp(float(loss)))
            log.maybe_save(step)
            if FLAGS.max_steps and step >= FLAGS.max_steps:
                break
        if FLAGS.max_steps and step >= FLAGS.max_steps:
            break
    if dev.type == "cuda":
        torch.cuda.synchronize()
        trainer.check()
    dt = time.time() - t0
    # validation perplexity (rank 0's model; all ranks hold identical weights)
    from tensorflow_examples_amd import ops
    vstate, vcost, vn = None, 0.0, 0
    with torch.no_grad():
        for x, y in ptb_batches(valid, B, T):
            logits, vstate = model(torch.as_tensor(x, device=dev), vstate)
            vcost += float(ops.softmax_cross_entropy(logits, torch.as_tensor(y, device=dev).reshape(-1)))
            vn += 1
    if rank == 0:
        print("valid perplexity %.3f" % math.exp(vcost / max(vn, 1)))
        print("tokens/sec (all GPUs) %.1f" % (tokens / max(dt, 1e-9)))
        log.scalars(step, valid_perplexity=math.exp(vcost / max(vn, 1)))
    saved = log.close(step)
    if saved:
        print("saved", saved)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    app.run(main)
