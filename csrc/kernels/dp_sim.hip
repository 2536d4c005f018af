// One-GPU stand-in for the CU footprint of an 8-rank RCCL ring all-reduce (scripts/dp_contention.py): a
// bucket's collective, issued on a side stream at the bucket's ready point in the graphed backward, is
// replaced by `nblocks` workgroups that stream the bucket through the vector memory path (read, write
// back the same bytes; `passes` sweeps ~ the ring's local traffic) and hold their CUs for the ring's
// modelled duration, the way RCCL's channel blocks do.  What it measures is the slowdown the backward kernels -- each sized to fill the chip -- suffer
// from sharing CUs, L2 and HBM with the collective, which the round-4 link-time model ignored.
// The bytes written back are the bytes read (the bucket is complete at launch and read only after the
// join), so the gradients are unchanged.  Reference: the sync-replicas remnant
// R/distributed/distributed.py:110-113 (the reference has no synchronous DP).
#include "tfx_common.h"

namespace tfx {
namespace {

constexpr int SIM_NT = 256;

// s_memrealtime: the constant 100 MHz clock (MI355X_MICROARCH.md DVFS item 6), read by the scalar unit
__device__ __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void __launch_bounds__(SIM_NT) dp_ring_sim_kernel(uint4* __restrict__ buf, int64_t nvec, uint64_t ticks,
                                                               int passes) {
  // a static LDS reservation like a collective kernel's staging: the block cannot share its CU with a
  // 147 KB GEMM block (nor could RCCL's)
  __shared__ uint4 stage[2048];
  const uint64_t t0 = realtime();
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = lo + per < nvec ? lo + per : nvec;
  // `passes` read + write-back sweeps of this block's share of the bucket (the ring's local memory
  // traffic: ~2 S(N-1)/N read and written per collective), then hold the CU polling the clock until the
  // modelled ring time is up, as RCCL's blocks do while they wait on their peers
  for (int pass = 0; pass < passes && realtime() - t0 < ticks; ++pass) {
    for (int64_t i = lo + threadIdx.x; i < hi; i += SIM_NT) {
      const uint4 v = buf[i];
      stage[(threadIdx.x + pass) & 2047] = v;
      buf[i] = stage[(threadIdx.x + pass) & 2047];
    }
  }
  while (realtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

}  // namespace

void dp_ring_sim(void* buf, int64_t nbytes, int nblocks, double duration_us, int passes, hipStream_t s) {
  const int64_t nvec = nbytes / 16;
  if (nvec <= 0 || nblocks <= 0) return;
  if (duration_us > 10000.0) duration_us = 10000.0;  // a bounded spin: every wave exits
  if (nblocks > 1024) nblocks = 1024;
  const uint64_t ticks = (uint64_t)(duration_us * 100.0);  // 100 MHz
  dp_ring_sim_kernel<<<nblocks, SIM_NT, 0, s>>>(static_cast<uint4*>(buf), nvec, ticks, passes < 0 ? (1 << 30) : passes);
}

}  // namespace tfx
