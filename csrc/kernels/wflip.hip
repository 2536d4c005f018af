// Flipped, channel-transposed copies of the 3x3 conv filters, all layers in one launch:
// Wf[c][r][s][ko] = W[ko][2-r][2-s][c] (bf16).  The stride-1 3x3 data gradients run as the forward
// conv of dY with Wf (igemm_dgrad_flip.hip); this refreshes every Wf of the model once per step
// (ops/nn.py: after the optimizer rewrote the bf16 shadow).
// Per (layer, tap, 64x64 [ko][c] tile): 16-byte coalesced loads along c, an LDS transpose, 16-byte
// coalesced stores along ko.  Layer descriptors: {src_off, dst_off, Ko, C, first_tile} (elements).
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

__global__ void __launch_bounds__(256) wflip3x3_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                       const int64_t* __restrict__ desc, int nlayers) {
  __shared__ uint16_t tile[64][64 + 8];  // [ko][c]; 144-byte rows keep 16-byte alignment
  int L = 0;
  while (L + 1 < nlayers && desc[(L + 1) * 5 + 4] <= blockIdx.x) ++L;
  const int64_t* d = desc + L * 5;
  const int Ko = (int)d[2], C = (int)d[3];
  const int local = blockIdx.x - (int)d[4];
  const int tc = C / 64, tk = Ko / 64;
  const int tap = local / (tk * tc), rem = local % (tk * tc);
  const int k0 = (rem / tc) * 64, c0 = (rem % tc) * 64;
  const int r = tap / 3, s = tap % 3;
  const int t = threadIdx.x;
  // load rows ko of W[ko][2-r][2-s][c0 .. c0+63]: 4 threads per row, 16 channels each
  {
    const int row = t >> 2, q = (t & 3) * 16;
    const uint16_t* p = src + d[0] + ((int64_t)(k0 + row) * 9 + (2 - r) * 3 + (2 - s)) * C + c0 + q;
    const U4 v0 = reinterpret_cast<const U4*>(p)[0], v1 = reinterpret_cast<const U4*>(p)[1];
    *reinterpret_cast<U4*>(&tile[row][q]) = v0;
    *reinterpret_cast<U4*>(&tile[row][q + 8]) = v1;
  }
  __syncthreads();
  // store rows c of Wf[c][r][s][k0 .. k0+63]: 4 threads per row, 16 ko each
  {
    const int c = t >> 2, q = (t & 3) * 16;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      w[i] = (uint32_t)tile[q + 2 * i][c] | ((uint32_t)tile[q + 2 * i + 1][c] << 16);
    uint16_t* p = dst + d[1] + ((int64_t)(c0 + c) * 9 + r * 3 + s) * Ko + k0 + q;
    reinterpret_cast<U4*>(p)[0] = U4{w[0], w[1], w[2], w[3]};
    reinterpret_cast<U4*>(p)[1] = U4{w[4], w[5], w[6], w[7]};
  }
}

}  // namespace

void wflip3x3(const uint16_t* src, uint16_t* dst, const int64_t* desc, int nlayers, int ntiles, hipStream_t s) {
  if (ntiles > 0) wflip3x3_kernel<<<ntiles, 256, 0, s>>>(src, dst, desc, nlayers);
}

}  // namespace tfx
