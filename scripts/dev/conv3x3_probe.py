"""Where the stage-1 fused 3x3 conv kernels (conv3x3_fused.hip) spend their time: the production kernels
instantiated with PROBE bits that skip one phase each (csrc/probes/conv3x3_probe.hip), HIP-graph replayed at
the bench shape (batch 256, 32x32x64).  Outputs of the probe variants are wrong; only their time is read.

    bash scripts/dev/build_probes.sh && python scripts/dev/conv3x3_probe.py
"""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "tensorflow_examples_amd", "_lib", "libtfx_probe.so"))
V = ctypes.c_void_p
lib.tfx_probe_conv3_fwd.argtypes = [ctypes.c_int, V, V, V, V, V, ctypes.c_int, ctypes.c_int, V]
lib.tfx_probe_conv3_bwd.argtypes = [ctypes.c_int] + [V] * 10 + [ctypes.c_int, ctypes.c_int, V]
dev = torch.device("cuda")
ITER = 20
N, H = 256, 32


def graph_us(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(ITER):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / ITER * 1e3)
    return best


def save(c=64):
    mu, istd = torch.randn(c, device=dev) * 0.1, torch.rand(c, device=dev) + 0.5
    sc, sh = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
    return torch.cat([mu, istd, sc, sh]).contiguous()


t = lambda: torch.randn(N, H, 32, 64, device=dev).bfloat16()
x, y1, y2, g2 = t(), t(), t(), t()
w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).bfloat16()
y, dx = torch.empty_like(x), torch.empty_like(x)
s1, s2 = save(), save()
red2 = torch.randn(128, device=dev)
slots = torch.zeros(64 * 2 * 64, device=dev)
slab = torch.zeros(256, 64 * 576, device=dev)
st = lambda: torch.cuda.current_stream().cuda_stream

FWD = {0: "production", 1: "no MFMA", 2: "no BN transform", 3: "no MFMA, no transform", 4: "no epilogue",
       7: "loads + LDS only"}
for p, name in FWD.items():
    us = graph_us(lambda: lib.tfx_probe_conv3_fwd(p, x.data_ptr(), s1.data_ptr(), w.data_ptr(), y.data_ptr(),
                                                 slots.data_ptr(), N, H, st()))
    print(f"fwd  probe {p:2d} {name:32s} {us:7.2f} us", flush=True)
BWD = {0: "production", 1: "no dgrad MFMA", 2: "no wgrad MFMA", 3: "no MFMA at all", 4: "no BN transforms",
       8: "no dgrad epilogue", 16: "no slab store", 24: "no dgrad epilogue, no slab", 7: "no MFMA, no transforms",
       28: "no transforms/epilogue/slab", 27: "no MFMA/epilogue/slab", 31: "loads + LDS staging only"}
for p, name in BWD.items():
    us = graph_us(lambda: lib.tfx_probe_conv3_bwd(p, g2.data_ptr(), y2.data_ptr(), s2.data_ptr(), red2.data_ptr(),
                                                 y1.data_ptr(), s1.data_ptr(), w.data_ptr(), dx.data_ptr(),
                                                 slots.data_ptr(), slab.data_ptr(), N, H, st()))
    print(f"bwd  probe {p:2d} {name:32s} {us:7.2f} us", flush=True)
