// Dropout with a counter-based hash mask (gfx950).
//
//  dropout_apply          y = keep(seed, i) ? x * 1/keep : 0   (bf16 or fp32, 16 B per lane)
//                         -- the backward is the same op on dy with the same seed
//  softmax_dropout_fwd    p = softmax(z) per row (saved), pd = p * keep(seed, r*S + c) / keep
//  softmax_dropout_bwd    dz = p * (dp - sum_c p dp),  dp = dpd * keep(seed, r*S + c) / keep
//
// Flax nn.Dropout on the FF hidden / outputs and on the attention probabilities
// (reference src/modeling.py:133-148).  No mask tensor is ever stored: the keep bit of element i
// is a pure function of (seed, i), so the backward -- and the recompute of an activation-
// checkpointed layer, which redraws the same seed from the restored generator -- regenerates it.
// The seed lives on the device (int64 [1], drawn from the layer's torch.Generator), so a step
// captured in a HIP graph draws a fresh mask per replay without a host round trip.
// The keep decision (common.h drop_hash / drop_keep: one hash per pair of elements, 16-bit
// thresholds) is mirrored bit for bit by ops/dropout.py::keep_mask (the CPU path and the GPU
// tests' oracle).  Attention probabilities [rows = (b h, q), S] index their mask transposed,
// ((b h) S + c) SE + q with SE = S rounded up to even (the fused attention kernels' convention).
#include "common.h"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void dropout_apply_kernel(const T* __restrict__ x, T* __restrict__ y, long n8,
                                                            const int64_t* __restrict__ seed_p, uint32_t thr,
                                                            float scale) {
  const uint64_t seed = (uint64_t)seed_p[0];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {  // one hash per pair of elements
      const uint32_t h = drop_hash((uint32_t)(i * 4 + j / 2), seed);
      v[j] = drop_keep_half(h, 0, thr) ? v[j] * scale : 0.f;
      v[j + 1] = drop_keep_half(h, 1, thr) ? v[j + 1] * scale : 0.f;
    }
    store8(y + i * 8, v);
  }
}

// FF hidden dropout of the fused blocks (reference modeling.py:147): the saved gelu'(h) and the
// FF2 input gelu(h) of the same elements both times keep(i) / keep, so the FF2 data-gradient
// epilogue (EPI_DMUL) and the FF2 weight gradient see the dropped activations unchanged.
// PAIR: g, gp in place; else from the pre-activation h: g = gelu(h) m, gp = gelu'(h) m.
template <bool PAIR>
__global__ __launch_bounds__(256) void gelu_drop_kernel(const uint16_t* __restrict__ h, uint16_t* __restrict__ g,
                                                        uint16_t* __restrict__ gp, long n8,
                                                        const int64_t* __restrict__ seed_p, uint32_t thr,
                                                        float scale) {
  const uint64_t seed = (uint64_t)seed_p[0];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float a[8], d[8];
    if (PAIR) {
      load8(g + i * 8, a);
      load8(gp + i * 8, d);
    } else {
      float x[8];
      load8(h + i * 8, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) gelu_and_grad_f(x[j], a[j], d[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const uint32_t hs = drop_hash((uint32_t)(i * 4 + j / 2), seed);
      const float m0 = drop_keep_half(hs, 0, thr) ? scale : 0.f, m1 = drop_keep_half(hs, 1, thr) ? scale : 0.f;
      a[j] *= m0;
      d[j] *= m0;
      a[j + 1] *= m1;
      d[j + 1] *= m1;
    }
    store8(g + i * 8, a);
    store8(gp + i * 8, d);
  }
}

// one wave per row of S fp32 logits; lanes stride the columns (any S)
__global__ __launch_bounds__(256) void softmax_dropout_fwd_kernel(const float* __restrict__ z, float* __restrict__ p,
                                                                  float* __restrict__ pd, long rows, int S,
                                                                  const int64_t* __restrict__ seed_p, uint32_t thr,
                                                                  float scale) {
  const uint64_t seed = (uint64_t)seed_p[0];
  const int lane = threadIdx.x & 63;
  const long SE = S + (S & 1);
  for (long r = blockIdx.x * 4L + (threadIdx.x >> 6); r < rows; r += (long)gridDim.x * 4) {
    const float* zr = z + r * S;
    const long q = r % S;  // mask index ((r - q) + c) SE + q (attention.hip convention)
    float m = -INFINITY;
    for (int c = lane; c < S; c += 64) m = fmaxf(m, zr[c]);
    m = wave_max(m);
    float s = 0.f;
    for (int c = lane; c < S; c += 64) s += __expf(zr[c] - m);
    const float inv = 1.f / wave_sum(s);
    for (int c = lane; c < S; c += 64) {
      const float v = __expf(zr[c] - m) * inv;
      p[r * S + c] = v;
      pd[r * S + c] = drop_keep(seed, (uint64_t)((r - q + c) * SE + q), thr) ? v * scale : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void softmax_dropout_bwd_kernel(const float* __restrict__ dpd,
                                                                  const float* __restrict__ p, float* __restrict__ dz,
                                                                  long rows, int S, const int64_t* __restrict__ seed_p,
                                                                  uint32_t thr, float scale) {
  const uint64_t seed = (uint64_t)seed_p[0];
  const int lane = threadIdx.x & 63;
  const long SE = S + (S & 1);
  for (long r = blockIdx.x * 4L + (threadIdx.x >> 6); r < rows; r += (long)gridDim.x * 4) {
    const long o = r * S, q = r % S, om = r - q;  // mask index (om + c) SE + q (attention.hip)
    float s = 0.f;
    for (int c = lane; c < S; c += 64) {
      const float dp = drop_keep(seed, (uint64_t)((om + c) * SE + q), thr) ? dpd[o + c] * scale : 0.f;
      s += p[o + c] * dp;
    }
    s = wave_sum(s);
    for (int c = lane; c < S; c += 64) {
      const float dp = drop_keep(seed, (uint64_t)((om + c) * SE + q), thr) ? dpd[o + c] * scale : 0.f;
      dz[o + c] = p[o + c] * (dp - s);
    }
  }
}

int grid_rows(long rows) {
  long b = (rows + 3) / 4;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

int grid_elems(long n8) {
  long b = (n8 + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

// x, y: n elements (n % 8 == 0, 16-B aligned); bf16 != 0: uint16 bf16 data, else fp32
int jm_dropout_apply(const void* x, void* y, long n, int bf16, const int64_t* seed, uint32_t thr, float scale,
                     hipStream_t st) {
  if (n % 8) return -1;
  if (n == 0) return 0;
  if (bf16)
    dropout_apply_kernel<uint16_t><<<grid_elems(n / 8), 256, 0, st>>>((const uint16_t*)x, (uint16_t*)y, n / 8, seed,
                                                                      thr, scale);
  else
    dropout_apply_kernel<float><<<grid_elems(n / 8), 256, 0, st>>>((const float*)x, (float*)y, n / 8, seed, thr,
                                                                   scale);
  return 0;
}

// h null: g, gp (bf16, n elements) masked in place; else g = gelu(h) m, gp = gelu'(h) m
int jm_gelu_drop(const uint16_t* h, uint16_t* g, uint16_t* gp, long n, const int64_t* seed, uint32_t thr, float scale,
                 hipStream_t st) {
  if (n % 8) return -1;
  if (n == 0) return 0;
  if (h == nullptr)
    gelu_drop_kernel<true><<<grid_elems(n / 8), 256, 0, st>>>(nullptr, g, gp, n / 8, seed, thr, scale);
  else
    gelu_drop_kernel<false><<<grid_elems(n / 8), 256, 0, st>>>(h, g, gp, n / 8, seed, thr, scale);
  return 0;
}

int jm_softmax_dropout_fwd(const float* z, float* p, float* pd, long rows, int S, const int64_t* seed, uint32_t thr,
                           float scale, hipStream_t st) {
  if (S <= 0) return -1;
  if (rows == 0) return 0;
  softmax_dropout_fwd_kernel<<<grid_rows(rows), 256, 0, st>>>(z, p, pd, rows, S, seed, thr, scale);
  return 0;
}

int jm_softmax_dropout_bwd(const float* dpd, const float* p, float* dz, long rows, int S, const int64_t* seed,
                           uint32_t thr, float scale, hipStream_t st) {
  if (S <= 0) return -1;
  if (rows == 0) return 0;
  softmax_dropout_bwd_kernel<<<grid_rows(rows), 256, 0, st>>>(dpd, p, dz, rows, S, seed, thr, scale);
  return 0;
}

JM_DEBUG_EXPORT(dropout)
