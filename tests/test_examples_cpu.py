"""The examples/ scripts (BASELINE.json configs 1-5) run end to end on the CPU path with tiny settings,
as subprocesses exactly as a user would run them; the DP examples also run as 2 gloo ranks."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")


def _run(script, *args, timeout=600):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), *args], capture_output=True,
                       text=True, timeout=timeout, env=ENV, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return p.stdout


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(script, n, *args, timeout=900):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "examples", script), *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=ENV, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    return p.stdout


def test_mnist_softmax_example():
    out = _run("mnist_softmax.py", "--train_steps=200", "--log_every=100", "--data_dir=/nonexistent")
    acc = float([l for l in out.splitlines() if l.startswith("accuracy")][0].split()[1])
    assert acc > 0.8


def test_lenet5_example(tmp_path):
    out = _run("lenet5.py", "--max_steps=40", "--batch_size=64", "--data_dir=/nonexistent", f"--logdir={tmp_path}")
    acc = float([l for l in out.splitlines() if l.startswith("test accuracy")][0].split()[2])
    assert acc > 0.5
    assert os.path.exists(tmp_path / "checkpoint")


def test_resnet_cifar_example_dp2(tmp_path):
    out = _torchrun("resnet_cifar.py", 2, "--depth=18", "--batch_size=8", "--max_steps=2", "--synthetic_train=256", "--eval_examples=100",
                    f"--logdir={tmp_path}")
    assert "test accuracy" in out and "images/sec (all GPUs)" in out
    assert os.path.exists(tmp_path / "checkpoint")
    # TF1 Supervisor layout: graph.pbtxt + a MetaGraphDef .meta, parsed by the repo's readers
    from tensorflow_examples_amd import ckpt
    nodes = ckpt.read_graph(str(tmp_path / "graph.pbtxt"))
    assert len(nodes) > 50 and all(n["op"] == "VariableV2" for n in nodes)
    first = ckpt.latest_checkpoint(str(tmp_path))
    mg = ckpt.read_meta_graph(first)
    assert len(mg["trainable_variables"]) > 50 and mg["saver"]["version"] == 2
    # resume: the second run restores the checkpoint and continues from its global step
    out2 = _torchrun("resnet_cifar.py", 2, "--depth=18", "--batch_size=8", "--max_steps=2", "--synthetic_train=256",
                     "--eval_examples=100", f"--logdir={tmp_path}", f"--export_dir={tmp_path / 'export'}")
    second = ckpt.latest_checkpoint(str(tmp_path))
    assert int(first.rsplit("-", 1)[1]) == 2 and int(second.rsplit("-", 1)[1]) == 4, (first, second, out2[-500:])
    # SavedModel export: a SavedModel protobuf with the serving signature + the variables directory
    sm = ckpt.read_saved_model(str(tmp_path / "export"))
    assert sm["tags"] == ["serve"] and sm["schema_version"] == 1
    assert sm["signature_defs"]["serving_default"]["inputs"]["images"]["shape"] == [-1, 32, 32, 3]
    assert os.path.exists(tmp_path / "export" / "variables" / "variables.data-00000-of-00001")


def test_word2vec_example():
    out = _run("word2vec.py", "--vocabulary_size=2000", "--num_steps=200", "--log_every=100",
               "--corpus_words=50000", "--embedding_size=32", "--num_sampled=16")
    assert "Nearest to" in out and "examples/sec" in out
    losses = [float(l.split(":")[1].split()[0]) for l in out.splitlines() if l.startswith("Average loss")]
    assert losses[-1] < losses[0]


def test_char_lstm_example_dp2():
    out = _torchrun("char_lstm.py", 2, "--hidden_size=32", "--embed_size=16", "--batch_size=4", "--num_steps=10",
                    "--max_steps=60", "--synthetic_chars=20000")
    assert "valid perplexity" in out and "tokens/sec (all GPUs)" in out
