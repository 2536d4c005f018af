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
// aligned at matching offsets) + scalar tail; grid-stride.  zero_g: the worker-local gradient is
// cleared as it is consumed (the next step's backward accumulates into a zero buffer without a
// separate fill launch).
__global__ void __launch_bounds__(256) ps_peer_sgd_kernel(float* __restrict__ p, float* __restrict__ g, int64_t n,
                                                          float lr, int zero_g) {
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
      if (zero_g) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += stride) {
    p[i] -= lr * g[i];
    if (zero_g) g[i] = 0.f;
  }
}

// AssignAdd(global_step, 1) (R/distributed/distributed.py:108), ordered AFTER this worker's whole
// update: it is its own single-thread launch behind the SGD kernel on the same stream, so every
// block's writes to the (possibly peer) arena have completed first; the fence writes them back at
// system scope before the increment becomes visible, and the increment itself is a SYSTEM-scope
// atomic (other GPUs of the node bump the same word).
__global__ void ps_step_inc_kernel(unsigned long long* __restrict__ step, long long* __restrict__ step_out) {
  __threadfence_system();
  const unsigned long long old =
      __hip_atomic_fetch_add(step, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  *step_out = (long long)(old + 1);
}

// PULL: peer arena -> worker-local store (xGMI reads), float4 grid-stride copy
__global__ void __launch_bounds__(256) ps_peer_copy_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                           int64_t n) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const bool vec = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0;
  int64_t done = 0;
  if (vec) {
    const int64_t n4 = n >> 2;
    for (int64_t i = tid; i < n4; i += stride) reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += stride) dst[i] = src[i];
}

static int ps_blocks(int64_t n) {
  int64_t blocks = (n / 4 + 255) / 256;
  return (int)(blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks));
}

void ps_peer_sgd(float* p, float* g, int64_t n, float lr, bool zero_g, void* step, int64_t* step_out,
                 hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(ps_peer_sgd_kernel, dim3(ps_blocks(n)), dim3(256), 0, s, p, g, n, lr, zero_g ? 1 : 0);
  if (step)
    hipLaunchKernelGGL(ps_step_inc_kernel, dim3(1), dim3(1), 0, s, reinterpret_cast<unsigned long long*>(step),
                       reinterpret_cast<long long*>(step_out));
}

void ps_peer_copy(float* dst, const float* src, int64_t n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(ps_peer_copy_kernel, dim3(ps_blocks(n)), dim3(256), 0, s, dst, src, n);
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
