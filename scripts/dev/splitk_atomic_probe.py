"""What the split-K f32 atomic epilogue costs the 1x1 weight gradient: the production kernel and launch
configuration (128x64 tile, KS=2, LDS-DMA ring 3, 256 blocks) built twice into the probe library
(csrc/probes, scripts/dev/build_probes.sh) -- with the atomics and with plain stores in their place --
HIP-graph replayed, interleaved A/B.  The atomic build is checked against an fp32 reference first.

    bash scripts/dev/build_probes.sh && python scripts/dev/splitk_atomic_probe.py
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "tensorflow_examples_amd", "_lib", "libtfx_probe.so"))
fns = {}
for v in ("atomic", "store"):
    f = getattr(lib, "tfx_probe_wgrad_" + v)
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    fns[v] = f
dev = torch.device("cuda")
ITER = 20


def call(v, dy, x, dw, npix, ko, c):
    rc = fns[v](dy.data_ptr(), x.data_ptr(), dw.data_ptr(), npix, ko, c, 256, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


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
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * ITER) * 1e3


# (N, H, W, C, Ko): dW[Ko][C] = sum over pixels dy[p][Ko] x[p][C]
for (N, H, W, C, Ko) in [(256, 8, 8, 1024, 256), (256, 8, 8, 256, 1024), (256, 16, 16, 128, 512),
                         (256, 16, 16, 512, 128), (256, 4, 4, 512, 2048), (256, 4, 4, 2048, 512)]:
    npix = N * H * W
    x = torch.randn(npix, C, device=dev).bfloat16()
    dy = torch.randn(npix, Ko, device=dev).bfloat16()
    dw = torch.zeros(Ko, C, device=dev)
    call("atomic", dy, x, dw, npix, Ko, C)
    ref = dy.float().t() @ x.float()
    err = float((dw - ref).abs().max() / ref.abs().max())
    assert err < 1e-3, (N, H, W, C, Ko, err)
    ta, ts = [], []
    for _ in range(3):
        ta.append(graph_us(lambda: call("atomic", dy, x, dw, npix, Ko, C)))
        ts.append(graph_us(lambda: call("store", dy, x, dw, npix, Ko, C)))
    a, s = min(ta), min(ts)
    mb = 256 * 128 * 64 * 4 / 2 ** 20
    print(f"x={N}x{H}x{W}x{C} Ko={Ko}: atomic epilogue {a:6.2f} us  plain-store epilogue {s:6.2f} us  "
          f"-> atomics cost {a - s:5.2f} us ({100 * (a - s) / a:4.1f} %) for {mb:.0f} MB of partial tiles "
          f"[rel err {err:.1e}; runs {', '.join(f'{t:.1f}' for t in ta)} / {', '.join(f'{t:.1f}' for t in ts)}]",
          flush=True)
