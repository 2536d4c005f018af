// Sparse and recurrent hot ops (BASELINE.json configs 4 and 5).
//
// word2vec skip-gram (TF's word2vec_basic: embedding_lookup + nce_loss + GradientDescent):
//   embedding_gather    rows[i] = table[ids[i]]            (one wave per row, 16-B loads)
//   embedding_scatter   table[ids[i]] += alpha * rows[i]    (sparse SGD apply / IndexedSlices
//                       accumulate; whole-row f32 atomics: each wave instruction adds 256
//                       contiguous bytes -- the fast shape of MI355X_MICROARCH.md "Global float
//                       atomics"; duplicates in ids are summed, Hogwild like TF's sparse apply)
//   log_uniform_sample  Zipfian candidate sampler (tf.random.log_uniform_candidate_sampler):
//                       k = floor(exp(u * ln(range+1))) - 1, counter-based hash RNG (no state)
//   sampled_loss        fused NCE (sigmoid) / sampled-softmax loss: true-logit dot product, logQ
//                       correction, accidental hits, loss and all per-example gradients
// char-LSTM:
//   lstm_cell_fwd       gates = gx + gh (+b) -> i,f,o = sigmoid, g = tanh; c = f*c' + i*g;
//                       h = o*tanh(c); stores the activated gates for backward (f32 state)
//   lstm_cell_bwd       dgates, dc' from dh, dc (+ the carried dc of the next step)
#include "tfx_common.h"
#include "tfx_kernels.h"

namespace tfx {

namespace {

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// ------------------------------------------------------------------ embedding
template <typename TO, bool VEC>
__global__ void __launch_bounds__(256) emb_gather_kernel(const float* __restrict__ table, int64_t V, int D,
                                                         const int64_t* __restrict__ ids, int64_t n,
                                                         TO* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    int64_t id = ids[r];
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);  // clamp like tf.gather on GPU (no fault)
    const float* src = table + id * D;
    TO* dst = out + r * D;
    if constexpr (VEC) {  // D % 4 == 0: 16-B loads, a 128-wide row is one wave instruction (512 B)
      for (int c = lane * 4; c < D; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(src + c);
        if constexpr (sizeof(TO) == 4) {
          *reinterpret_cast<float4*>(dst + c) = v;
        } else {
          uint2 o;
          o.x = pack_bf16x2(v.x, v.y);
          o.y = pack_bf16x2(v.z, v.w);
          *reinterpret_cast<uint2*>(dst + c) = o;
        }
      }
    } else {
      for (int c = lane; c < D; c += 64) {
        if constexpr (sizeof(TO) == 4)
          dst[c] = src[c];
        else
          dst[c] = f32_to_bf16(src[c]);
      }
    }
  }
}

__global__ void __launch_bounds__(256) emb_scatter_kernel(float* __restrict__ table, int64_t V, int D,
                                                          const int64_t* __restrict__ ids, int64_t n,
                                                          const float* __restrict__ rows, float alpha) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    if (id < 0 || id >= V) continue;
    float* dst = table + id * D;
    const float* src = rows + r * D;
    for (int c = lane; c < D; c += 64) atomicAdd(dst + c, alpha * src[c]);
  }
}

// ------------------------------------------------------------------ sampler
// ids_in == nullptr: draw n candidates; else: only compute logq of the given ids (true labels)
// seed_dev (optional): a device step counter added to ``seed`` -- a captured HIP graph then draws
// fresh candidates on every replay.
__global__ void log_uniform_kernel(int64_t n, int64_t range, uint64_t seed, const int64_t* __restrict__ seed_dev,
                                   const int64_t* __restrict__ ids_in, int64_t* __restrict__ out,
                                   float* __restrict__ logq, int num_expected) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (seed_dev) seed += (uint64_t)(*seed_dev) * 0x9E3779B97F4A7C15ull;
  const double lr = log((double)range + 1.0);
  int64_t k;
  if (ids_in) {
    k = ids_in[i];
  } else {
    const uint32_t h = hash32((uint32_t)i * 0x9E3779B1u ^ hash32((uint32_t)seed) ^ (uint32_t)(seed >> 32));
    const double u = (h + 0.5) / 4294967296.0;
    k = (int64_t)floor(exp(u * lr)) - 1;
    k = k < 0 ? 0 : (k >= range ? range - 1 : k);
    out[i] = k;
  }
  if (logq) {
    // log(expected count) = log(num_expected * P(k)), P(k) = log((k+2)/(k+1)) / log(range+1)
    const double p = log(((double)k + 2.0) / ((double)k + 1.0)) / lr;
    logq[i] = (float)log(p * (double)num_expected);
  }
}

// ------------------------------------------------------------------ skip-gram batch generator
// Random (center, context) pairs from a device-resident corpus: position p uniform in
// [window, N-window), context offset uniform in [-window, window] \ {0} (word2vec_basic's
// generate_batch with num_skips = 1 per draw; every pair is drawn independently).
__global__ void skipgram_batch_kernel(const int32_t* __restrict__ corpus, int64_t N, int B, int window, uint64_t seed,
                                      const int64_t* __restrict__ seed_dev, int64_t* __restrict__ centers,
                                      int64_t* __restrict__ labels) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (seed_dev) seed += (uint64_t)(*seed_dev) * 0x9E3779B97F4A7C15ull;
  const uint32_t s0 = hash32((uint32_t)seed ^ 0x68bc21ebu) ^ hash32((uint32_t)(seed >> 32) + 0x02e5be93u);
  const uint32_t h1 = hash32((uint32_t)i * 2u + 1u + s0);
  const uint32_t h2 = hash32((uint32_t)i * 2u + 2u + hash32(s0));
  const uint64_t span = (uint64_t)(N - 2 * window);
  const int64_t p = window + (int64_t)((((uint64_t)h1 << 20) ^ h2) % span);
  const int o = 1 + (int)((h2 >> 1) % (uint32_t)window);
  const int64_t q = (h2 & 1u) ? p + o : p - o;
  centers[i] = corpus[p];
  labels[i] = corpus[q];
}

// ------------------------------------------------------------------ sampled loss (NCE / sampled softmax)
// One wave per example b.  Fused: the true logit t = e_b . w_t + b_t (dot over D in-wave), the logQ
// corrections, accidental-hit removal, the loss and every gradient of the example:
//   nce (sigmoid):  loss = softplus(-t') + sum_s softplus(n'_s);  dt = sig(t') - 1;  dn_s = sig(n'_s)
//   sampled softmax: loss = logsumexp([t', n']) - t';              dt = p_0 - 1;     dn_s = p_s
// dt is folded straight into the true-branch rows: dE_b = dt * w_t (the later GEMM adds dn @ Ws on top),
// dWt_b = dt * e_b, dbt_b = dt.  All gradients are pre-multiplied by gscale (1/B for a mean loss).
template <bool SOFTMAX>
__global__ void __launch_bounds__(256) sampled_loss_kernel(const float* __restrict__ E, const float* __restrict__ Wt,
                                                           const float* __restrict__ bt, const float* __restrict__ nl,
                                                           int B, int S, int D, const float* __restrict__ logq_t,
                                                           const float* __restrict__ logq_n,
                                                           const int64_t* __restrict__ tid,
                                                           const int64_t* __restrict__ sid, float gscale,
                                                           float* __restrict__ loss, float* __restrict__ dn,
                                                           float* __restrict__ dE, float* __restrict__ dWt,
                                                           float* __restrict__ dbt) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* e = E + (int64_t)b * D;
  const float* w = Wt + (int64_t)b * D;
  float dot = 0.f;
  for (int c = lane; c < D; c += 64) dot = fmaf(e[c], w[c], dot);
  const float t = wave_sum(dot) + (bt ? bt[b] : 0.f) - (logq_t ? logq_t[b] : 0.f);
  const int64_t myid = tid ? tid[b] : -1;
  const float* nrow = nl + (int64_t)b * S;
  float* drow = dn + (int64_t)b * S;
  float lsum, dt;
  if constexpr (SOFTMAX) {
    float m = t;
    for (int s = lane; s < S; s += 64) {
      const bool hit = sid && sid[s] == myid;
      if (!hit) m = fmaxf(m, nrow[s] - (logq_n ? logq_n[s] : 0.f));
    }
    m = wave_max(m);
    float z = 0.f;
    for (int s = lane; s < S; s += 64) {
      const bool hit = sid && sid[s] == myid;
      if (!hit) z += __expf(nrow[s] - (logq_n ? logq_n[s] : 0.f) - m);
    }
    z = wave_sum(z) + __expf(t - m);
    const float inv = 1.f / z;
    for (int s = lane; s < S; s += 64) {
      const bool hit = sid && sid[s] == myid;
      drow[s] = hit ? 0.f : gscale * __expf(nrow[s] - (logq_n ? logq_n[s] : 0.f) - m) * inv;
    }
    lsum = logf(z) + m - t;
    dt = gscale * (__expf(t - m) * inv - 1.f);
  } else {
    float acc = 0.f;
    for (int s = lane; s < S; s += 64) {
      const bool hit = sid && sid[s] == myid;
      const float v = nrow[s] - (logq_n ? logq_n[s] : 0.f);
      if (!hit) acc += fmaxf(v, 0.f) + log1pf(__expf(-fabsf(v)));
      drow[s] = hit ? 0.f : gscale / (1.f + __expf(-v));
    }
    lsum = wave_sum(acc) + fmaxf(-t, 0.f) + log1pf(__expf(-fabsf(t)));
    dt = gscale * (1.f / (1.f + __expf(-t)) - 1.f);
  }
  for (int c = lane; c < D; c += 64) {
    dE[(int64_t)b * D + c] = dt * w[c];
    dWt[(int64_t)b * D + c] = dt * e[c];
  }
  if (lane == 0) {
    loss[b] = lsum;
    dbt[b] = dt;
  }
}

// ------------------------------------------------------------------ LSTM cell (gate order i, f, g, o)
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ void __launch_bounds__(256) lstm_fwd_kernel(const float* __restrict__ gx, const float* __restrict__ gh,
                                                       const float* __restrict__ bias, const float* __restrict__ c_prev,
                                                       int B, int H, float* __restrict__ act, float* __restrict__ c,
                                                       float* __restrict__ h, uint16_t* __restrict__ h16) {
  const int64_t total = (int64_t)B * H;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t b = idx / H;
    const int j = (int)(idx - b * H);
    const int64_t g0 = b * 4 * H + j;
    float z[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      z[q] = gx[g0 + q * H] + (gh ? gh[g0 + q * H] : 0.f) + (bias ? bias[q * H + j] : 0.f);
    }
    const float ig = sigm(z[0]), fg = sigm(z[1]), gg = tanhf(z[2]), og = sigm(z[3]);
    const float cp = c_prev ? c_prev[idx] : 0.f;
    const float cn = fmaf(fg, cp, ig * gg);
    const float hn = og * tanhf(cn);
    act[g0] = ig;
    act[g0 + H] = fg;
    act[g0 + 2 * H] = gg;
    act[g0 + 3 * H] = og;
    c[idx] = cn;
    h[idx] = hn;
    if (h16) h16[idx] = f32_to_bf16(hn);
  }
}

// dh: gradient w.r.t. h_t (from the output layer + the recurrent path); dc_next: carried from t+1
__global__ void __launch_bounds__(256) lstm_bwd_kernel(const float* __restrict__ act, const float* __restrict__ c,
                                                       const float* __restrict__ c_prev, const float* __restrict__ dh,
                                                       const float* __restrict__ dc_next, int B, int H,
                                                       float* __restrict__ dgates, uint16_t* __restrict__ dg16,
                                                       float* __restrict__ dc_prev) {
  const int64_t total = (int64_t)B * H;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t b = idx / H;
    const int j = (int)(idx - b * H);
    const int64_t g0 = b * 4 * H + j;
    const float ig = act[g0], fg = act[g0 + H], gg = act[g0 + 2 * H], og = act[g0 + 3 * H];
    const float cn = c[idx], cp = c_prev ? c_prev[idx] : 0.f;
    const float tc = tanhf(cn);
    const float dhv = dh ? dh[idx] : 0.f;
    const float dc = fmaf(dhv * og, 1.f - tc * tc, dc_next ? dc_next[idx] : 0.f);
    const float d0 = dc * gg * ig * (1.f - ig), d1 = dc * cp * fg * (1.f - fg);
    const float d2 = dc * ig * (1.f - gg * gg), d3 = dhv * tc * og * (1.f - og);
    if (dgates) {
      dgates[g0] = d0;
      dgates[g0 + H] = d1;
      dgates[g0 + 2 * H] = d2;
      dgates[g0 + 3 * H] = d3;
    }
    if (dg16) {
      dg16[g0] = f32_to_bf16(d0);
      dg16[g0 + H] = f32_to_bf16(d1);
      dg16[g0 + 2 * H] = f32_to_bf16(d2);
      dg16[g0 + 3 * H] = f32_to_bf16(d3);
    }
    if (dc_prev) dc_prev[idx] = dc * fg;
  }
}

int egrid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, 16384)); }
int pgrid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

}  // namespace

void embedding_gather(const float* table, int64_t V, int D, const int64_t* ids, int64_t n, void* out, bool out_bf16,
                      hipStream_t s) {
  const bool vec = D % 4 == 0 && (reinterpret_cast<uintptr_t>(table) & 15) == 0;
  if (out_bf16) {
    if (vec) emb_gather_kernel<uint16_t, true><<<egrid(n), 256, 0, s>>>(table, V, D, ids, n, (uint16_t*)out);
    else emb_gather_kernel<uint16_t, false><<<egrid(n), 256, 0, s>>>(table, V, D, ids, n, (uint16_t*)out);
  } else {
    if (vec) emb_gather_kernel<float, true><<<egrid(n), 256, 0, s>>>(table, V, D, ids, n, (float*)out);
    else emb_gather_kernel<float, false><<<egrid(n), 256, 0, s>>>(table, V, D, ids, n, (float*)out);
  }
}

void embedding_scatter_add(float* table, int64_t V, int D, const int64_t* ids, int64_t n, const float* rows,
                           float alpha, hipStream_t s) {
  emb_scatter_kernel<<<egrid(n), 256, 0, s>>>(table, V, D, ids, n, rows, alpha);
}

void log_uniform_sample(int64_t n, int64_t range, uint64_t seed, const int64_t* seed_dev, const int64_t* ids_in,
                        int64_t* out, float* logq, int num_expected, hipStream_t s) {
  log_uniform_kernel<<<(int)((n + 255) / 256), 256, 0, s>>>(n, range, seed, seed_dev, ids_in, out, logq,
                                                              num_expected);
}

void skipgram_batch(const int32_t* corpus, int64_t N, int B, int window, uint64_t seed, const int64_t* seed_dev,
                    int64_t* centers, int64_t* labels, hipStream_t s) {
  skipgram_batch_kernel<<<(B + 255) / 256, 256, 0, s>>>(corpus, N, B, window, seed, seed_dev, centers, labels);
}

void sampled_loss(bool softmax, const float* E, const float* Wt, const float* bt, const float* nl, int B, int S, int D,
                  const float* logq_t, const float* logq_n, const int64_t* tid, const int64_t* sid, float gscale,
                  float* loss, float* dn, float* dE, float* dWt, float* dbt, hipStream_t s) {
  if (softmax)
    sampled_loss_kernel<true><<<(B + 3) / 4, 256, 0, s>>>(E, Wt, bt, nl, B, S, D, logq_t, logq_n, tid, sid, gscale,
                                                          loss, dn, dE, dWt, dbt);
  else
    sampled_loss_kernel<false><<<(B + 3) / 4, 256, 0, s>>>(E, Wt, bt, nl, B, S, D, logq_t, logq_n, tid, sid, gscale,
                                                           loss, dn, dE, dWt, dbt);
}

void lstm_cell_fwd(const float* gx, const float* gh, const float* bias, const float* c_prev, int B, int H,
                   float* act, float* c, float* h, uint16_t* h16, hipStream_t s) {
  lstm_fwd_kernel<<<pgrid((int64_t)B * H), 256, 0, s>>>(gx, gh, bias, c_prev, B, H, act, c, h, h16);
}

void lstm_cell_bwd(const float* act, const float* c, const float* c_prev, const float* dh, const float* dc_next,
                   int B, int H, float* dgates, uint16_t* dg16, float* dc_prev, hipStream_t s) {
  lstm_bwd_kernel<<<pgrid((int64_t)B * H), 256, 0, s>>>(act, c, c_prev, dh, dc_next, B, H, dgates, dg16, dc_prev);
}

}  // namespace tfx
