// Parameter-server transport over xGMI peer memory ("parity mode, intra-node").
//
// The reference moves every variable between worker and ps with gRPC RecvTensor/RunGraph each
// step (R/distributed/distributed.py:148-150) and applies
// ApplyGradientDescent + AssignAdd(global_step) on the ps (:107-108).  Here the ps owns one
// hipMalloc'd arena on its GPU and exports it with hipIpcGetMemHandle; a worker on any GPU of
// the node maps it with hipIpcOpenMemHandle and then
//   * PULL  = one device-to-device copy out of the peer arena (xGMI read, no host hop),
//   * PUSH  = ps_peer_sgd below: the worker's own kernel writes p -= lr*g straight into the
//             peer arena (lock-free like TF's use_locking=False: concurrent workers may tear a
//             float update, never a pointer) and bumps the 64-bit global step with one device
//             atomic, returning the new value into worker-local memory.
//
// Arena header (64-bit words): [0] global step, [1] ready flag (chief sets 1 after init),
// [2] layout fingerprint, [3..7] reserved; parameters start at byte 256 in the worker's flat
// VariableStore layout (every replica builds the identical layout).
#include <cstring>

#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

// One pass over a contiguous parameter range: float4 body (arena and store are 16-byte
// aligned at matching offsets for the whole-store range) + scalar tail; grid-stride.
__global__ void __launch_bounds__(256) ps_peer_sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                          int64_t n, float lr,
                                                          unsigned long long* __restrict__ step,
                                                          long long* __restrict__ step_out) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g)) & 15) == 0;
  int64_t done = 0;
  if (vec) {
    const int64_t n4 = n >> 2;
    for (int64_t i = tid; i < n4; i += stride) {
      float4 pv = reinterpret_cast<float4*>(p)[i];
      const float4 gv = reinterpret_cast<const float4*>(g)[i];
      pv.x -= lr * gv.x; pv.y -= lr * gv.y; pv.z -= lr * gv.z; pv.w -= lr * gv.w;
      reinterpret_cast<float4*>(p)[i] = pv;
    }
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += stride) p[i] -= lr * g[i];
  if (step && tid == 0) {
    // AssignAdd(global_step, 1) after this worker's update was issued; device-scope atomic on
    // the (possibly remote) arena, system scope so a peer GPU's increments are ordered too.
    __threadfence_system();
    const unsigned long long old = atomicAdd(step, 1ull);
    *step_out = (long long)(old + 1);
  }
}

void ps_peer_sgd(float* p, const float* g, int64_t n, float lr, void* step, int64_t* step_out, hipStream_t s) {
  if (n <= 0 && !step) return;
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(ps_peer_sgd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, n, lr,
                     reinterpret_cast<unsigned long long*>(step), reinterpret_cast<long long*>(step_out));
}

// ---------------------------------------------------------------- IPC arena management
int ipc_alloc(int device, int64_t nbytes, void** ptr) {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return -1;
  if (hipSetDevice(device) != hipSuccess) return -1;
  // plain hipMalloc (not the caching allocator): hipIpcGetMemHandle needs an allocation base
  hipError_t e = hipMalloc(ptr, (size_t)nbytes);
  if (e == hipSuccess) e = hipMemset(*ptr, 0, (size_t)nbytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  hipSetDevice(prev);
  return e == hipSuccess ? 0 : -(int)e;
}

int ipc_free(int device, void* ptr) {
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  const hipError_t e = hipFree(ptr);
  hipSetDevice(prev);
  return e == hipSuccess ? 0 : -(int)e;
}

int ipc_get_handle(void* ptr, uint8_t* out64) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) return -(int)e;
  static_assert(sizeof(h) <= 64, "IPC handle size");
  memcpy(out64, &h, sizeof(h));
  return (int)sizeof(h);
}

int ipc_open(int device, const uint8_t* handle64, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(device);
  const hipError_t e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
  hipSetDevice(prev);
  return e == hipSuccess ? 0 : -(int)e;
}

int ipc_close(void* ptr) {
  const hipError_t e = hipIpcCloseMemHandle(ptr);
  return e == hipSuccess ? 0 : -(int)e;
}

}  // namespace tfx
