"""Kernel-boundary cost of a producer's stores by cache policy (csrc/probes/store_flush_probe.hip): a
16-byte store sweep of S bytes (plain / nt / sc1 write-through / sc0 sc1), then a dependent 1-block kernel
or a full read of the bytes, HIP-graph replayed (20 pairs, best of 3).  If a kernel boundary pays for
writing back the producer's dirty L2 lines, write-through stores should shorten store -> tiny.

    bash scripts/dev/build_probes.sh && python scripts/dev/store_flush_probe.py"""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "tensorflow_examples_amd", "_lib", "libtfx_probe.so"))
V = ctypes.c_void_p
lib.tfx_probe_store.argtypes = [ctypes.c_int, V, ctypes.c_uint, ctypes.c_int, V]
lib.tfx_probe_read.argtypes = [V, ctypes.c_uint, V, ctypes.c_int, V]
lib.tfx_probe_tiny.argtypes = [V, V]
dev = torch.device("cuda")
ITER = 20


def graph_us(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(ITER):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / ITER * 1e3)
    return best


out = torch.zeros(4096, device=dev)
names = {0: "plain", 2: "nt", 16: "sc1", 17: "sc0 sc1"}
for mb in (8, 32, 64, 128):
    buf = torch.empty(mb << 20, dtype=torch.uint8, device=dev)
    n = buf.numel()
    for blocks in (1024,):
        row = []
        for aux in (0, 2, 16, 17):
            st = lambda: lib.tfx_probe_store(aux, buf.data_ptr(), n, blocks, torch.cuda.current_stream().cuda_stream)
            tiny = lambda: lib.tfx_probe_tiny(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            rd = lambda: lib.tfx_probe_read(buf.data_ptr(), n, out.data_ptr(), blocks,
                                            torch.cuda.current_stream().cuda_stream)
            t_s = graph_us(st)
            t_st = graph_us(lambda: (st(), tiny()))
            t_sr = graph_us(lambda: (st(), rd()))
            row.append("%-7s store %6.2f | +tiny %6.2f (%+5.2f) | +read %6.2f" % (names[aux], t_s, t_st, t_st - t_s, t_sr))
        print("%4d MB: " % mb + "\n         ".join(row), flush=True)
    t_tiny = graph_us(lambda: lib.tfx_probe_tiny(out.data_ptr(), torch.cuda.current_stream().cuda_stream))
print("tiny alone %.2f us" % t_tiny)
