// Multi-tensor optimizer kernels over the flat fp32 master / grad / state buffers (gfx950).
//
// One launch covers every parameter: the grid walks a host-built chunk table
// [start, length, segment] (<= 64Ki elements per chunk), each segment = one Flax leaf with
// metadata [decay flag, layer-wise LR scale, trust-ratio flag, trainable].  The same pass writes
// the bf16 shadow copy read by the GEMMs, so weights are never re-cast per step.
// Per-step scalars come from a device tensor hyper = [lr, 1-b1^t, 1-b2^t, clip, b1, b2, eps, wd]
// and the optional global grad norm^2 (negative = clipping off), so the step is graph-capturable.
// Semantics: optax adamw / modified LAMB / lars / sgd (see optim/flat.py for the reference map).
#include "common.h"

namespace {

struct Chunk {
  int start, len, seg;
};

JM_DEVICE float clip_factor(const float* hyper, const float* gnorm_sq) {
  const float gs = gnorm_sq[0];
  if (gs < 0.f) return 1.f;
  const float gn = sqrtf(gs);
  const float c = hyper[3];
  return gn < c ? 1.f : c / gn;
}

JM_DEVICE float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += sh[i];
  }
  return r;
}

// Norm partials: every chunk block stores its sums in cpart[chunk][NC] and chunk_sums_kernel adds
// them per segment in chunk order -- the same bits on every run (the round-1..3 kernels added the
// block sums with float atomics, whose order varies).
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, const Chunk* __restrict__ chunks,
                                                    float* __restrict__ cpart) {
  __shared__ float sh[8];
  const Chunk c = chunks[blockIdx.x];
  float s = 0.f;
  for (int i = threadIdx.x; i < c.len; i += 256) {
    const float v = x[c.start + i];
    s += v * v;
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) cpart[blockIdx.x] = s;
}

// out[seg * NC + k] += sum over the run of chunks of seg (chunks sorted by segment) of
// cpart[chunk * NC + k]; PER_SEG = false: one sum over all chunks into out[k].  One block per chunk:
// the first chunk of each run reduces the run (thread-strided in order, then a fixed tree).
template <int NC, bool PER_SEG>
__global__ __launch_bounds__(256) void chunk_sums_kernel(const Chunk* __restrict__ chunks, int nchunks,
                                                         const float* __restrict__ cpart, float* __restrict__ out) {
  __shared__ float red[NC][256];
  const int i0 = PER_SEG ? (int)blockIdx.x : 0;
  const int seg = chunks[i0].seg;
  if (PER_SEG && i0 > 0 && chunks[i0 - 1].seg == seg) return;  // not a run start (block-uniform)
  float a[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) a[k] = 0.f;
  for (int j = i0 + threadIdx.x; j < nchunks; j += 256) {
    if (PER_SEG && chunks[j].seg != seg) break;  // runs are contiguous: nothing of seg beyond
#pragma unroll
    for (int k = 0; k < NC; ++k) a[k] += cpart[(long)j * NC + k];
  }
#pragma unroll
  for (int k = 0; k < NC; ++k) red[k][threadIdx.x] = a[k];
  __syncthreads();
#pragma unroll
  for (int h = 128; h >= 1; h >>= 1) {
    if ((int)threadIdx.x < h) {
#pragma unroll
      for (int k = 0; k < NC; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NC; ++k) out[(PER_SEG ? seg * NC : 0) + k] += red[k][0];
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ mu, float* __restrict__ nu,
                                                    uint16_t* __restrict__ shadow, const Chunk* __restrict__ chunks,
                                                    const float* __restrict__ meta, const float* __restrict__ hyper,
                                                    const float* __restrict__ gnorm_sq) {
  const Chunk c = chunks[blockIdx.x];
  const float* m = meta + 4 * c.seg;
  if (m[3] == 0.f) return;
  const float lr = hyper[0], bc1 = hyper[1], bc2 = hyper[2], b1 = hyper[4], b2 = hyper[5], eps = hyper[6];
  const float wd = hyper[7] * m[0];
  const float step = -lr * m[1];
  const float f = clip_factor(hyper, gnorm_sq);
  const float ib1 = 1.f / bc1, ib2 = 1.f / bc2;
  // one element: moments in place, returns the new parameter
  auto upd = [&](float gv, float& mm, float& vv, float pv) {
    const float gg = gv * f;
    mm = b1 * mm + (1.f - b1) * gg;
    vv = b2 * vv + (1.f - b2) * gg * gg;
    const float u = (mm * ib1) / (sqrtf(vv * ib2) + eps) + wd * pv;
    return pv + step * u;
  };
  // 16 B per lane (chunk starts are multiples of 64 elements).  Same step time as the r1
  // 4-B-per-lane loop in a same-process A/B (profiles/r2_adamw_vector.txt: the pass is HBM-bound
  // either way; its 2.1-2.4 ms spread is box to box)
  const int n4 = c.len >> 2;
  for (int i = threadIdx.x; i < n4; i += 256) {
    const long k = (long)c.start + 4L * i;
    float gv[4], mm[4], vv[4], pv[4], np[4];
    load4(g + k, gv);
    load4(mu + k, mm);
    load4(nu + k, vv);
    load4(p + k, pv);
#pragma unroll
    for (int j = 0; j < 4; ++j) np[j] = upd(gv[j], mm[j], vv[j], pv[j]);
    store4(mu + k, mm);
    store4(nu + k, vv);
    store4(p + k, np);
    if (shadow) store4(shadow + k, np);
  }
  for (int i = 4 * n4 + threadIdx.x; i < c.len; i += 256) {
    const long k = (long)c.start + i;
    float mm = mu[k], vv = nu[k];
    const float np = upd(g[k], mm, vv, p[k]);
    mu[k] = mm;
    nu[k] = vv;
    p[k] = np;
    if (shadow) shadow[k] = f2bf(np);
  }
}

__global__ __launch_bounds__(256) void lamb_phase1_kernel(const float* __restrict__ p, const float* __restrict__ g,
                                                          float* __restrict__ mu, float* __restrict__ nu,
                                                          float* __restrict__ u_out, const Chunk* __restrict__ chunks,
                                                          const float* __restrict__ meta,
                                                          const float* __restrict__ hyper,
                                                          const float* __restrict__ gnorm_sq, float* __restrict__ cpart) {
  __shared__ float sh[8];
  const Chunk c = chunks[blockIdx.x];
  const float* m = meta + 4 * c.seg;
  const float bc1 = hyper[1], bc2 = hyper[2], b1 = hyper[4], b2 = hyper[5], eps = hyper[6];
  const float wd = hyper[7] * m[0];
  const float f = clip_factor(hyper, gnorm_sq);
  float sp = 0.f, su = 0.f;
  for (int i = threadIdx.x; i < c.len; i += 256) {
    const long k = (long)c.start + i;
    const float gg = g[k] * f;
    const float mm = b1 * mu[k] + (1.f - b1) * gg;
    const float vv = b2 * nu[k] + (1.f - b2) * gg * gg;
    mu[k] = mm;
    nu[k] = vv;
    const float pv = p[k];
    const float u = (mm / bc1) / (sqrtf(vv / bc2) + eps) + wd * pv;
    u_out[k] = u;
    sp += pv * pv;
    su += u * u;
  }
  sp = block_sum(sp, sh);
  su = block_sum(su, sh);
  if (threadIdx.x == 0) {
    cpart[2 * blockIdx.x] = sp;
    cpart[2 * blockIdx.x + 1] = su;
  }
}

__global__ __launch_bounds__(256) void lars_norms_kernel(const float* __restrict__ p, const float* __restrict__ g,
                                                         const Chunk* __restrict__ chunks,
                                                         const float* __restrict__ hyper,
                                                         const float* __restrict__ gnorm_sq, float* __restrict__ cpart) {
  __shared__ float sh[8];
  const Chunk c = chunks[blockIdx.x];
  const float f = clip_factor(hyper, gnorm_sq);
  float sp = 0.f, su = 0.f;
  for (int i = threadIdx.x; i < c.len; i += 256) {
    const long k = (long)c.start + i;
    const float pv = p[k], u = g[k] * f;
    sp += pv * pv;
    su += u * u;
  }
  sp = block_sum(sp, sh);
  su = block_sum(su, sh);
  if (threadIdx.x == 0) {
    cpart[2 * blockIdx.x] = sp;
    cpart[2 * blockIdx.x + 1] = su;
  }
}

// mode 0: LAMB apply  p += -lr*llrd*tr*u          (u precomputed by phase 1)
// mode 1: LARS        t = -lr*tr*(f*g) + mom*t;  p += llrd*t
__global__ __launch_bounds__(256) void apply_trust_kernel(float* __restrict__ p, const float* __restrict__ u_or_g,
                                                          float* __restrict__ trace, uint16_t* __restrict__ shadow,
                                                          const Chunk* __restrict__ chunks,
                                                          const float* __restrict__ meta,
                                                          const float* __restrict__ hyper,
                                                          const float* __restrict__ norms,
                                                          const float* __restrict__ gnorm_sq, int mode, float momentum,
                                                          float trust_coef) {
  const Chunk c = chunks[blockIdx.x];
  const float* m = meta + 4 * c.seg;
  if (m[3] == 0.f) return;
  const float lr = hyper[0];
  const float pn = sqrtf(norms[2 * c.seg]), un = sqrtf(norms[2 * c.seg + 1]);
  float tr = 1.f;
  if (m[2] != 0.f && pn != 0.f && un != 0.f) tr = (mode == 1 ? trust_coef : 1.f) * pn / un;
  const float f = mode == 1 ? clip_factor(hyper, gnorm_sq) : 1.f;
  for (int i = threadIdx.x; i < c.len; i += 256) {
    const long k = (long)c.start + i;
    float np;
    if (mode == 0) {
      np = p[k] - lr * m[1] * tr * u_or_g[k];
    } else {
      const float t = -lr * tr * (f * u_or_g[k]) + momentum * trace[k];
      trace[k] = t;
      np = p[k] + m[1] * t;
    }
    p[k] = np;
    if (shadow) shadow[k] = f2bf(np);
  }
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ trace, uint16_t* __restrict__ shadow,
                                                  const Chunk* __restrict__ chunks, const float* __restrict__ meta,
                                                  const float* __restrict__ hyper, const float* __restrict__ gnorm_sq,
                                                  float momentum) {
  const Chunk c = chunks[blockIdx.x];
  const float* m = meta + 4 * c.seg;
  if (m[3] == 0.f) return;
  const float lr = hyper[0];
  const float f = clip_factor(hyper, gnorm_sq);
  for (int i = threadIdx.x; i < c.len; i += 256) {
    const long k = (long)c.start + i;
    const float t = f * g[k] + momentum * trace[k];
    trace[k] = t;
    const float np = p[k] - lr * m[1] * t;
    p[k] = np;
    if (shadow) shadow[k] = f2bf(np);
  }
}

}  // namespace

// cpart: nchunks (sumsq) / 2 * nchunks (LAMB / LARS norms) floats of chunk partials
void jm_opt_sumsq(const float* x, const int* chunks, int nchunks, float* out, float* cpart, hipStream_t st) {
  if (nchunks < 1) return;
  sumsq_kernel<<<nchunks, 256, 0, st>>>(x, (const Chunk*)chunks, cpart);
  chunk_sums_kernel<1, false><<<1, 256, 0, st>>>((const Chunk*)chunks, nchunks, cpart, out);
}

void jm_opt_adamw(float* p, const float* g, float* mu, float* nu, uint16_t* shadow, const int* chunks, int nchunks,
                  const float* meta, const float* hyper, const float* gnorm_sq, hipStream_t st) {
  adamw_kernel<<<nchunks, 256, 0, st>>>(p, g, mu, nu, shadow, (const Chunk*)chunks, meta, hyper, gnorm_sq);
}

void jm_opt_lamb_phase1(const float* p, const float* g, float* mu, float* nu, float* u, const int* chunks,
                        int nchunks, const float* meta, const float* hyper, const float* gnorm_sq, float* norms,
                        float* cpart, hipStream_t st) {
  if (nchunks < 1) return;
  lamb_phase1_kernel<<<nchunks, 256, 0, st>>>(p, g, mu, nu, u, (const Chunk*)chunks, meta, hyper, gnorm_sq, cpart);
  chunk_sums_kernel<2, true><<<nchunks, 256, 0, st>>>((const Chunk*)chunks, nchunks, cpart, norms);
}

void jm_opt_lars_norms(const float* p, const float* g, const int* chunks, int nchunks, const float* hyper,
                       const float* gnorm_sq, float* norms, float* cpart, hipStream_t st) {
  if (nchunks < 1) return;
  lars_norms_kernel<<<nchunks, 256, 0, st>>>(p, g, (const Chunk*)chunks, hyper, gnorm_sq, cpart);
  chunk_sums_kernel<2, true><<<nchunks, 256, 0, st>>>((const Chunk*)chunks, nchunks, cpart, norms);
}

void jm_opt_apply_trust(float* p, const float* u_or_g, float* trace, uint16_t* shadow, const int* chunks, int nchunks,
                        const float* meta, const float* hyper, const float* norms, const float* gnorm_sq, int mode,
                        float momentum, float trust_coef, hipStream_t st) {
  apply_trust_kernel<<<nchunks, 256, 0, st>>>(p, u_or_g, trace, shadow, (const Chunk*)chunks, meta, hyper, norms,
                                              gnorm_sq, mode, momentum, trust_coef);
}

void jm_opt_sgd(float* p, const float* g, float* trace, uint16_t* shadow, const int* chunks, int nchunks,
                const float* meta, const float* hyper, const float* gnorm_sq, float momentum, hipStream_t st) {
  sgd_kernel<<<nchunks, 256, 0, st>>>(p, g, trace, shadow, (const Chunk*)chunks, meta, hyper, gnorm_sq, momentum);
}

JM_DEBUG_EXPORT(optim)
