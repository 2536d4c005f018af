"""Per-kernel cost of a chain of dependent launches inside one HIP graph (the ResNet step is ~310
of them): a 1-block torch add, the BN slot reduction (the shape of bn_finalize: NSLOT x 2 x C
floats in, 2C out), and a stage-3/4-sized BN apply.  Prints microseconds per launch for each.

    python scripts/launch_floor.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_examples_amd.ops import _native  # noqa: E402


def timed_graph(fn, n=100, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * n)


def main():
    assert _native.load(), "native library missing"
    dev = torch.device("cuda", 0)
    nslot = int(torch.ops.tfx.bn_nslot())
    one = torch.zeros(1, device=dev)
    out = {"add_1elem": timed_graph(lambda: one.add_(1.0))}
    for C in (64, 256, 1024, 2048):
        sl = torch.zeros(nslot * 2 * C, device=dev)
        out["slot_reduce_C%d" % C] = timed_graph(lambda: torch.ops.tfx.bn_slots_reduce(sl, C, None, None))
    for M, C in ((4096, 512), (16384, 256), (65536, 128)):
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        save = torch.cat([torch.zeros(C), torch.ones(C), torch.ones(C), torch.zeros(C)]).to(dev)
        y = torch.empty_like(x)
        out["bn_apply_%dx%d" % (M, C)] = timed_graph(lambda: torch.ops.tfx.bn_apply_into(x, None, save, None, y, None))
    for k, v in out.items():
        print("%-24s %7.2f us/launch" % (k, v))


if __name__ == "__main__":
    main()
