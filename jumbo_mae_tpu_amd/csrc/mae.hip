// MAE data-path kernels (gfx950).
//
// patchify_normalize: uint8 NCHW images -> fp32 [B, N, p*p*3] patches of the normalized image,
// element order (ph, pw, c) == extract_patches(NHWC) of the reference (utils_mae.py:67-73) after
// ((x/255) - mean) / std (pretraining.py:90-91).  One workgroup per (image, patch row): the
// 3 x p x W uint8 strip is staged through LDS with 4-byte loads, then written out coalesced.
#include "common.h"

namespace {

__constant__ float c_mean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float c_istd[3] = {1.f / 0.229f, 1.f / 0.224f, 1.f / 0.225f};

__global__ __launch_bounds__(256) void patchify_kernel(const uint8_t* __restrict__ img, float* __restrict__ out, int H,
                                                       int W, int p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t strip[];  // [3][p][W]
  const int g = W / p;
  const int gh = H / p;
  const int b = blockIdx.x / gh, gy = blockIdx.x - (blockIdx.x / gh) * gh;
  const int W4 = W / 4;
  for (int i = threadIdx.x; i < 3 * p * W4; i += 256) {
    const int c = i / (p * W4);
    const int rem = i - c * p * W4;
    const int ph = rem / W4, x4 = rem - ph * W4;
    const uint32_t v =
        *reinterpret_cast<const uint32_t*>(img + (((long)b * 3 + c) * H + gy * p + ph) * W + x4 * 4);
    *reinterpret_cast<uint32_t*>(strip + (c * p + ph) * W + x4 * 4) = v;
  }
  __syncthreads();
  const int KP = p * p * 3;
  float* o = out + ((long)b * gh * g + (long)gy * g) * KP;
  for (int idx = threadIdx.x; idx < g * KP; idx += 256) {
    const int gx = idx / KP;
    const int k = idx - gx * KP;
    const int ph = k / (p * 3);
    const int r2 = k - ph * p * 3;
    const int pw = r2 / 3, c = r2 - (r2 / 3) * 3;
    const float v = (float)strip[(c * p + ph) * W + gx * p + pw];
    o[idx] = (v * (1.f / 255.f) - c_mean[c]) * c_istd[c];
  }
}

}  // namespace

int jm_patchify_normalize(const uint8_t* img, float* out, int B, int H, int W, int p, hipStream_t st) {
  if ((W % 4) || (H % p) || (W % p)) return -1;
  const size_t sm = (size_t)3 * p * W;
  patchify_kernel<<<B * (H / p), 256, sm, st>>>(img, out, H, W, p);
  return 0;
}

// ----------------------------------------------------------------------------------------------
// Mask-first MAE glue.  Index tensors are int32 with a batch
// stride: 0 for the reference's per-rank shared permutation (utils_mae.py:88-102, quirk Q1), N
// (or K) for per-sample masks.  None of these kernels materialises the fp32 patch tensor: the
// encoder input and the loss target are both read straight from the uint8 images.
namespace {

// normalized pixel o (in (ph, pw, c) order) of patch (gy, gx) of image b
JM_DEVICE float patch_pixel(const uint8_t* __restrict__ img, int b, int H, int W, int p, int gy, int gx, int o) {
  const int ph = o / (3 * p);
  const int r = o - ph * 3 * p;
  const int pw = r / 3, c = r - (r / 3) * 3;
  const float v = (float)img[(((long)b * 3 + c) * H + gy * p + ph) * W + gx * p + pw];
  return (v * (1.f / 255.f) - c_mean[c]) * c_istd[c];
}

// p = 16 (768 outputs per patch, one 64-lane row group per patch): lane l produces the 12
// consecutive outputs 12 l .. 12 l + 11 = patch row l / 4, pixels 4 (l % 4) .. + 3, channels 0-2,
// from one 4-byte load per channel (W % 4 == 0 and a 4-byte aligned image: host checks) instead
// of twelve byte loads; raw pixel bytes, channel c in byte k of px[c] = pixel 4 (l % 4) + k
JM_DEVICE void p16_raw(const uint8_t* __restrict__ img, int b, int H, int W, int gy, int gx, int lane, uint32_t* px) {
  const int ph = lane >> 2, pw0 = (lane & 3) * 4;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    px[c] = *reinterpret_cast<const uint32_t*>(img + (((long)b * 3 + c) * H + gy * 16 + ph) * W + gx * 16 + pw0);
}

JM_DEVICE float p16_norm(const uint32_t* px, int j) {  // output j = 3 k + c of the lane
  const int k = j / 3, c = j - (j / 3) * 3;
  return ((float)((px[c] >> (8 * k)) & 0xffu) * (1.f / 255.f) - c_mean[c]) * c_istd[c];
}

JM_DEVICE void p16_store12(uint16_t* o, const float* f) {
  uint2* d = reinterpret_cast<uint2*>(o);
#pragma unroll
  for (int q = 0; q < 3; ++q)
    d[q] = make_uint2(pack_bf2(f[4 * q], f[4 * q + 1]), pack_bf2(f[4 * q + 2], f[4 * q + 3]));
}

// K1+K3: kept patches of the normalized image as the bf16 patch-embed GEMM operand [B*K, 3p^2].
// One thread writes 4 consecutive outputs (8-byte store).
__global__ __launch_bounds__(256) void gather_patches_kernel(const uint8_t* __restrict__ img,
                                                             const int* __restrict__ ids, long idsB,
                                                             uint16_t* __restrict__ out, int B, int K, int H,
                                                             int W, int p) {
  const int P3 = 3 * p * p, q = P3 / 4, g = W / p;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * K * q) return;
  const long row = i / q;
  const int o = (int)(i - row * q) * 4;
  const int b = (int)(row / K), k = (int)(row - (long)b * K);
  const int n = ids[b * idsB + k];
  JM_DASSERT(n >= 0 && n < (H / p) * g);
  const int gy = n / g, gx = n - (n / g) * g;
  float f[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = patch_pixel(img, b, H, W, p, gy, gx, o + j);
  store4(out + row * P3 + o, f);
}

// p = 16 form of gather_patches_kernel: 12 outputs per thread from 3 word loads (p16_raw)
__global__ __launch_bounds__(256) void gather_patches16_kernel(const uint8_t* __restrict__ img,
                                                               const int* __restrict__ ids, long idsB,
                                                               uint16_t* __restrict__ out, int B, int K, int H, int W) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * K * 64) return;
  const long row = i >> 6;
  const int lane = (int)(i & 63);
  const int b = (int)(row / K), k = (int)(row - (long)b * K);
  const int g = W / 16;
  const int n = ids[b * idsB + k];
  JM_DASSERT(n >= 0 && n < (H / 16) * g);
  uint32_t px[3];
  p16_raw(img, b, H, W, n / g, n - (n / g) * g, lane, px);
  float f[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) f[j] = p16_norm(px, j);
  p16_store12(out + row * 768 + 12 * lane, f);
}

// K2 epilogue + K4: x[b, t] = cls[t] (t < C); e[b*K + t - C] + pos[ids[t - C]] (t >= C), fp32.
__global__ __launch_bounds__(256) void embed_finish_kernel(const uint16_t* __restrict__ e, const float* __restrict__ pos,
                                                           const int* __restrict__ ids, long idsB,
                                                           const float* __restrict__ cls, float* __restrict__ out,
                                                           int B, int C, int K, int D) {
  const int q = D / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * (C + K) * q) return;
  const long row = i / q;
  const int col = (int)(i - row * q) * 4;
  const int b = (int)(row / (C + K)), t = (int)(row - (long)b * (C + K));
  float f[4];
  if (t < C) {
    load4(cls + (long)t * D + col, f);
  } else {
    load4(e + ((long)b * K + t - C) * D + col, f);
    if (pos != nullptr) {
      float pp[4];
      load4(pos + (long)ids[b * idsB + t - C] * D + col, pp);
#pragma unroll
      for (int j = 0; j < 4; ++j) f[j] += pp[j];
    }
  }
  store4(out + row * D + col, f);
}

// K13 forward: decoder input [B, C+N, d] fp32 = cat(cls, unshuffle(cat(kept, mask_token)) + pos).
__global__ __launch_bounds__(256) void unshuffle_fwd_kernel(const uint16_t* __restrict__ y, const float* __restrict__ tok,
                                                            const int* __restrict__ restore, long rsB,
                                                            const float* __restrict__ pos, float* __restrict__ out,
                                                            int B, int C, int K, int N, int d) {
  const int q = d / 4;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * (C + N) * q) return;
  const long row = i / q;
  const int col = (int)(i - row * q) * 4;
  const int b = (int)(row / (C + N)), t = (int)(row - (long)b * (C + N));
  float f[4];
  if (t < C) {
    load4(y + ((long)b * (C + K) + t) * d + col, f);
  } else {
    const int n = t - C;
    const int j = restore[b * rsB + n];
    JM_DASSERT(j >= 0 && j < N);
    if (j < K) load4(y + ((long)b * (C + K) + C + j) * d + col, f);
    else load4(tok + col, f);
    float pp[4];
    load4(pos + (long)n * d + col, pp);
#pragma unroll
    for (int u = 0; u < 4; ++u) f[u] += pp[u];
  }
  store4(out + row * d + col, f);
}

// K13 backward in one pass over dout [B, C+N, d]: kept and CLS rows are gathered into dy
// [B, C+K, d] (bf16, the decoder_proj GEMM operand); mask-token rows are summed into per-block
// column partials part[blockIdx.x][d] (atomic-free, reduced by the caller).  Each block owns a
// contiguous range of ``rows_per_block`` rows; threads cover 4 columns each.
__global__ __launch_bounds__(256) void unshuffle_bwd_kernel(const float* __restrict__ dout, const int* __restrict__ restore,
                                                            long rsB, uint16_t* __restrict__ dy, float* __restrict__ part,
                                                            int B, int C, int K, int N, int d, int rows_per_block) {
  extern __shared__ float red[];  // [256 / q][d]
  const int q = d / 4;
  const int lanes = (256 / q) * q;
  const int col = (threadIdx.x % q) * 4;
  const int rg = threadIdx.x / q, nrg = 256 / q;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const long total = (long)B * (C + N);
  const long r0 = (long)blockIdx.x * rows_per_block;
  if (threadIdx.x < lanes) {
    for (long row = r0 + rg; row < r0 + rows_per_block && row < total; row += nrg) {
      const int b = (int)(row / (C + N)), t = (int)(row - (long)b * (C + N));
      float f[4];
      load4(dout + row * d + col, f);
      if (t < C) {
        store4(dy + ((long)b * (C + K) + t) * d + col, f);
      } else {
        const int j = restore[b * rsB + t - C];
        if (j < K) {
          store4(dy + ((long)b * (C + K) + C + j) * d + col, f);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[u] += f[u];
        }
      }
    }
    store4(red + rg * d + col, acc);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 256) {
    float s = 0.f;
    for (int g = 0; g < nrg; ++g) s += red[g * d + c];
    part[(long)blockIdx.x * d + c] = s;
  }
}

// target pixels of one patch row for a wave: lane holds elements o = lane + 64 * j.  The patch's
// 3 x p x p uint8 pixels are first staged into the wave's LDS slice with coalesced row loads
// (p = 16: 48 lanes x 16 B), then each lane picks its (ph, pw, c) elements from LDS.
template <int NJ, bool P16>
JM_DEVICE void patch_target(const uint8_t* __restrict__ img, long row, int N, int H, int W, int p_, int P3_,
                            bool norm_pix, uint8_t* lds, float* t) {
  const int p = P16 ? 16 : p_, P3 = P16 ? 768 : P3_;
  const int g = W / p;
  const int b = (int)(row / N), n = (int)(row - (long)b * N);
  const int gy = n / g, gx = n - (n / g) * g;
  const int lane = threadIdx.x & 63;
  const uint8_t* src = img + ((long)b * 3 * H + gy * p) * W + gx * p;  // channel 0, first patch row
  if (p == 16) {
    if (lane < 48) {
      const int c = lane >> 4, ph = lane & 15;
      *reinterpret_cast<uint4*>(lds + lane * 16) =
          *reinterpret_cast<const uint4*>(src + ((long)c * H + ph) * W);
    }
  } else {
    for (int i = lane; i < P3; i += 64) {
      const int c = i / (p * p), r = i - c * p * p;
      const int ph = r / p, pw = r - (r / p) * p;
      lds[i] = src[((long)c * H + ph) * W + pw];
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int o = lane + 64 * j;
    float v = 0.f;
    if (o < P3) {
      const int ph = o / (3 * p), r = o - ph * 3 * p;
      const int pw = r / 3, c = r - (r / 3) * 3;
      v = ((float)lds[(c * p + ph) * p + pw] * (1.f / 255.f) - c_mean[c]) * c_istd[c];
    }
    t[j] = v;
  }
  if (norm_pix) {  // per-patch (t - mean) / sqrt(var + 1e-6), biased var (pretraining.py:114-117)
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) s += t[j];
    const float mean = wave_sum(s) / P3;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int o = lane + 64 * j;
      const float dlt = o < P3 ? t[j] - mean : 0.f;
      v += dlt * dlt;
    }
    const float rs = rsqrtf(wave_sum(v) / P3 + 1e-6f);
#pragma unroll
    for (int j = 0; j < NJ; ++j) t[j] = (t[j] - mean) * rs;
  }
}

// p = 16 rows (768 = 64 lanes x 12): lane l owns the 12 CONSECUTIVE elements o = 12 l + j, i.e.
// patch row ph = l / 4, pixels pw = 4 (l % 4) + j / 3, channel c = j % 3 -- so pred / dpred move as
// three 8-byte accesses per lane instead of twelve 2-byte ones, the pred loads are issued before
// the pixel staging (both HBM round trips overlap), and each channel's 4 pixels come out of the
// staged patch in one 4-byte LDS read.
JM_DEVICE void p16_load_pred(const uint16_t* __restrict__ pr, float* f) {
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint2 v = *reinterpret_cast<const uint2*>(pr + 4 * q);
    f[4 * q + 0] = __uint_as_float(v.x << 16);
    f[4 * q + 1] = __uint_as_float(v.x & 0xffff0000u);
    f[4 * q + 2] = __uint_as_float(v.y << 16);
    f[4 * q + 3] = __uint_as_float(v.y & 0xffff0000u);
  }
}

JM_DEVICE void p16_target(const uint8_t* __restrict__ img, long row, int N, int H, int W, bool norm_pix, uint8_t* lds,
                          float* t) {
  const int g = W / 16;
  const int b = (int)(row / N), n = (int)(row - (long)b * N);
  const int gy = n / g, gx = n - (n / g) * g;
  const int lane = threadIdx.x & 63;
  const uint8_t* src = img + ((long)b * 3 * H + gy * 16) * W + gx * 16;
  if (lane < 48) {
    const int c = lane >> 4, ph = lane & 15;
    *reinterpret_cast<uint4*>(lds + lane * 16) = *reinterpret_cast<const uint4*>(src + ((long)c * H + ph) * W);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
  const int ph = lane >> 2, pw0 = (lane & 3) * 4;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const uint32_t px = *reinterpret_cast<const uint32_t*>(lds + (c * 16 + ph) * 16 + pw0);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      t[3 * k + c] = ((float)((px >> (8 * k)) & 0xffu) * (1.f / 255.f) - c_mean[c]) * c_istd[c];
  }
  if (norm_pix) {  // per-patch (t - mean) / sqrt(var + 1e-6), biased var (pretraining.py:114-117)
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 12; ++j) s += t[j];
    const float mean = wave_sum(s) * (1.f / 768.f);
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < 12; ++j) v += (t[j] - mean) * (t[j] - mean);
    const float rs = rsqrtf(wave_sum(v) * (1.f / 768.f) + 1e-6f);
#pragma unroll
    for (int j = 0; j < 12; ++j) t[j] = (t[j] - mean) * rs;
  }
}

// K14 forward: per-patch mean squared error of the prediction vs the normalized target, one wave
// per (image, patch) row.  mse[row] = mean_pix (t - pred)^2 (utils_mae.py:51-64 before masking).
template <int NJ, bool P16>
__global__ __launch_bounds__(256) void patch_mse_fwd_kernel(const uint16_t* __restrict__ pred, long ldp,
                                                            const uint8_t* __restrict__ img, float* __restrict__ mse,
                                                            long rows, int N, int H, int W, int p, int norm_pix) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int P3 = 3 * p * p;
  __shared__ __attribute__((aligned(16))) uint8_t pix[4][64 * NJ];
  float t[NJ];
  const int lane = threadIdx.x & 63;
  if constexpr (P16) {  // ldp % 4 == 0 (host)
    float f[12];
    p16_load_pred(pred + row * ldp + 12 * lane, f);
    p16_target(img, row, N, H, W, norm_pix != 0, pix[threadIdx.x >> 6], t);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 12; ++j) s += (t[j] - f[j]) * (t[j] - f[j]);
    s = wave_sum(s);
    if (lane == 0) mse[row] = s * (1.f / 768.f);
    return;
  }
  patch_target<NJ, P16>(img, row, N, H, W, p, P3, norm_pix != 0, pix[threadIdx.x >> 6], t);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int o = lane + 64 * j;
    if (o < P3) {
      const float dlt = t[j] - bf2f(pred[row * ldp + o]);
      s += dlt * dlt;
    }
  }
  s = wave_sum(s);
  if (lane == 0) mse[row] = s / P3;
}

// K14 backward: dpred[row] = dmse[row] * 2 / P3 * (pred - t); rows with dmse == 0 (the kept,
// unmasked patches) are written as zeros without reading pred or the image.
template <int NJ, bool P16>
__global__ __launch_bounds__(256) void patch_mse_bwd_kernel(const uint16_t* __restrict__ pred, long ldp,
                                                            const uint8_t* __restrict__ img,
                                                            const float* __restrict__ dmse, uint16_t* __restrict__ dpred,
                                                            long rows, int N, int H, int W, int p, int norm_pix) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int P3 = 3 * p * p;
  const int lane = threadIdx.x & 63;
  const float gsc = dmse[row];
  __shared__ __attribute__((aligned(16))) uint8_t pix[4][64 * NJ];
  float t[NJ];
  if constexpr (P16) {  // ldp % 4 == 0 (host)
    uint2* o = reinterpret_cast<uint2*>(dpred + row * 768 + 12 * lane);
    if (gsc == 0.f) {
#pragma unroll
      for (int q = 0; q < 3; ++q) o[q] = make_uint2(0u, 0u);
      return;
    }
    float f[12];
    p16_load_pred(pred + row * ldp + 12 * lane, f);
    p16_target(img, row, N, H, W, norm_pix != 0, pix[threadIdx.x >> 6], t);
    const float k = 2.f * gsc * (1.f / 768.f);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      o[q] = make_uint2(pack_bf2(k * (f[4 * q] - t[4 * q]), k * (f[4 * q + 1] - t[4 * q + 1])),
                        pack_bf2(k * (f[4 * q + 2] - t[4 * q + 2]), k * (f[4 * q + 3] - t[4 * q + 3])));
    return;
  }
  if (gsc == 0.f) {
    for (int o = lane; o < P3; o += 64) dpred[row * P3 + o] = 0;
    return;
  }
  patch_target<NJ, P16>(img, row, N, H, W, p, P3, norm_pix != 0, pix[threadIdx.x >> 6], t);
  const float k = 2.f * gsc / P3;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int o = lane + 64 * j;
    if (o < P3) dpred[row * P3 + o] = f2bf(k * (bf2f(pred[row * ldp + o]) - t[j]));
  }
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace

int jm_gather_patches(const uint8_t* img, const int* ids, long idsB, uint16_t* out, int B, int K, int H, int W, int p,
                      hipStream_t st) {
  if ((3 * p * p) % 4 || H % p || W % p) return -1;
  const long n = (long)B * K * (3 * p * p / 4);
  if (n == 0) return 0;
  if (p == 16 && W % 4 == 0 && (reinterpret_cast<uintptr_t>(img) & 3) == 0) {
    gather_patches16_kernel<<<cdiv((long)B * K * 64, 256), 256, 0, st>>>(img, ids, idsB, out, B, K, H, W);
    return 0;
  }
  gather_patches_kernel<<<cdiv(n, 256), 256, 0, st>>>(img, ids, idsB, out, B, K, H, W, p);
  return 0;
}

int jm_embed_finish(const uint16_t* e, const float* pos, const int* ids, long idsB, const float* cls, float* out,
                    int B, int C, int K, int D, hipStream_t st) {
  if (D % 4) return -1;
  const long n = (long)B * (C + K) * (D / 4);
  if (n == 0) return 0;
  embed_finish_kernel<<<cdiv(n, 256), 256, 0, st>>>(e, pos, ids, idsB, cls, out, B, C, K, D);
  return 0;
}

int jm_unshuffle_fwd(const uint16_t* y, const float* tok, const int* restore, long rsB, const float* pos, float* out,
                     int B, int C, int K, int N, int d, hipStream_t st) {
  if (d % 4) return -1;
  const long n = (long)B * (C + N) * (d / 4);
  if (n == 0) return 0;
  unshuffle_fwd_kernel<<<cdiv(n, 256), 256, 0, st>>>(y, tok, restore, rsB, pos, out, B, C, K, N, d);
  return 0;
}

// returns the number of partial rows written to ``part`` (caller sizes part with jm_unshuffle_bwd_blocks)
int jm_unshuffle_bwd_blocks(int B, int C, int N, int rows_per_block) {
  return cdiv((long)B * (C + N), rows_per_block);
}

int jm_unshuffle_bwd(const float* dout, const int* restore, long rsB, uint16_t* dy, float* part, int B, int C, int K,
                     int N, int d, int rows_per_block, hipStream_t st) {
  if (d % 4 || d / 4 > 256) return -1;
  const int nb = jm_unshuffle_bwd_blocks(B, C, N, rows_per_block);
  const size_t sm = (size_t)(256 / (d / 4)) * d * sizeof(float);
  unshuffle_bwd_kernel<<<nb, 256, sm, st>>>(dout, restore, rsB, dy, part, B, C, K, N, d, rows_per_block);
  return 0;
}

int jm_patch_mse_fwd(const uint16_t* pred, long ldp, const uint8_t* img, float* mse, long rows, int N, int H, int W,
                     int p, int norm_pix, hipStream_t st) {
  const int P3 = 3 * p * p;
  if (H % p || W % p || P3 > 64 * 16) return -1;
  const int nb = cdiv(rows, 4);
  if (p == 16 && ldp % 4 == 0 && (reinterpret_cast<uintptr_t>(pred) & 7) == 0)
    patch_mse_fwd_kernel<12, true><<<nb, 256, 0, st>>>(pred, ldp, img, mse, rows, N, H, W, p, norm_pix);
  else if (P3 <= 64 * 4)
    patch_mse_fwd_kernel<4, false><<<nb, 256, 0, st>>>(pred, ldp, img, mse, rows, N, H, W, p, norm_pix);
  else if (P3 <= 64 * 12)
    patch_mse_fwd_kernel<12, false><<<nb, 256, 0, st>>>(pred, ldp, img, mse, rows, N, H, W, p, norm_pix);
  else patch_mse_fwd_kernel<16, false><<<nb, 256, 0, st>>>(pred, ldp, img, mse, rows, N, H, W, p, norm_pix);
  return 0;
}

int jm_patch_mse_bwd(const uint16_t* pred, long ldp, const uint8_t* img, const float* dmse, uint16_t* dpred, long rows,
                     int N, int H, int W, int p, int norm_pix, hipStream_t st) {
  const int P3 = 3 * p * p;
  if (H % p || W % p || P3 > 64 * 16) return -1;
  const int nb = cdiv(rows, 4);
  if (p == 16 && ldp % 4 == 0 && (reinterpret_cast<uintptr_t>(pred) & 7) == 0)
    patch_mse_bwd_kernel<12, true><<<nb, 256, 0, st>>>(pred, ldp, img, dmse, dpred, rows, N, H, W, p, norm_pix);
  else if (P3 <= 64 * 4)
    patch_mse_bwd_kernel<4, false><<<nb, 256, 0, st>>>(pred, ldp, img, dmse, dpred, rows, N, H, W, p, norm_pix);
  else if (P3 <= 64 * 12)
    patch_mse_bwd_kernel<12, false><<<nb, 256, 0, st>>>(pred, ldp, img, dmse, dpred, rows, N, H, W, p, norm_pix);
  else
    patch_mse_bwd_kernel<16, false><<<nb, 256, 0, st>>>(pred, ldp, img, dmse, dpred, rows, N, H, W, p, norm_pix);
  return 0;
}

// ----------------------------------------------------------------------------------------------
// K19 (finetune input): all patches of the normalized, Mixup- or CutMix-blended batch as the bf16
// patch-embed operand [B*N, 3p^2], straight from uint8 (utils.py:66-111 semantics):
//   mode 0: x[b];  mode 1 (mixup): r x[b] + (1 - r) x[perm[b]];
//   mode 2 (cutmix): x[perm[b]] inside the pixel box [y0, y1) x [x0, x1), else x[b].
// The per-batch decisions live in DEVICE buffers (prm = [mode, ratio, ...], box = [y0, y1, x0, x1],
// perm), written by the host step feeder: the launch has no host-varying arguments and can be
// replayed from a HIP graph.  prm == nullptr: no mixing.
namespace {
__global__ __launch_bounds__(256) void mix_patches_kernel(const uint8_t* __restrict__ img, const int* __restrict__ perm,
                                                          const float* __restrict__ prm, const int* __restrict__ box,
                                                          uint16_t* __restrict__ out, int B, int H, int W, int p) {
  const int P3 = 3 * p * p, q = P3 / 4, g = W / p, N = (H / p) * g;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * N * q) return;
  const int mode = prm ? (int)prm[0] : 0;
  const float r = prm ? prm[1] : 1.f;
  int y0 = 0, y1 = 0, x0 = 0, x1 = 0;
  if (mode == 2) {
    y0 = box[0];
    y1 = box[1];
    x0 = box[2];
    x1 = box[3];
  }
  const long row = i / q;
  const int o0 = (int)(i - row * q) * 4;
  const int b = (int)(row / N), n = (int)(row - (long)b * N);
  const int gy = n / g, gx = n - (n / g) * g;
  const int bo = mode ? perm[b] : b;
  float f[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = o0 + j;
    const int ph = o / (3 * p);
    const int rr = o - ph * 3 * p;
    const int pw = rr / 3;
    const int y = gy * p + ph, x = gx * p + pw;
    const float a = patch_pixel(img, b, H, W, p, gy, gx, o);
    if (mode == 1) {
      f[j] = r * a + (1.f - r) * patch_pixel(img, bo, H, W, p, gy, gx, o);
    } else if (mode == 2 && y >= y0 && y < y1 && x >= x0 && x < x1) {
      f[j] = patch_pixel(img, bo, H, W, p, gy, gx, o);
    } else {
      f[j] = a;
    }
  }
  store4(out + row * P3 + o0, f);
}

// p = 16 form of mix_patches_kernel: 12 outputs per thread from 3 word loads per source image
__global__ __launch_bounds__(256) void mix_patches16_kernel(const uint8_t* __restrict__ img,
                                                            const int* __restrict__ perm,
                                                            const float* __restrict__ prm,
                                                            const int* __restrict__ box,
                                                            uint16_t* __restrict__ out, int B, int H, int W) {
  const int g = W / 16, N = (H / 16) * g;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * N * 64) return;
  const int mode = prm ? (int)prm[0] : 0;
  const float r = prm ? prm[1] : 1.f;
  const long row = i >> 6;
  const int lane = (int)(i & 63);
  const int b = (int)(row / N), n = (int)(row - (long)b * N);
  const int gy = n / g, gx = n - (n / g) * g;
  uint32_t pa[3], pb[3];
  p16_raw(img, b, H, W, gy, gx, lane, pa);
  float f[12];
  if (mode == 0) {
#pragma unroll
    for (int j = 0; j < 12; ++j) f[j] = p16_norm(pa, j);
  } else {
    p16_raw(img, perm[b], H, W, gy, gx, lane, pb);
    if (mode == 1) {
#pragma unroll
      for (int j = 0; j < 12; ++j) f[j] = r * p16_norm(pa, j) + (1.f - r) * p16_norm(pb, j);
    } else {  // cutmix: the permuted image inside the pixel box [y0, y1) x [x0, x1)
      const int y = gy * 16 + (lane >> 2), x0 = gx * 16 + (lane & 3) * 4;
      const bool yin = y >= box[0] && y < box[1];
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const int x = x0 + j / 3;
        f[j] = (yin && x >= box[2] && x < box[3]) ? p16_norm(pb, j) : p16_norm(pa, j);
      }
    }
  }
  p16_store12(out + row * 768 + 12 * lane, f);
}
}  // namespace

int jm_mix_patches(const uint8_t* img, const int* perm, const float* prm, const int* box, uint16_t* out, int B, int H,
                   int W, int p, hipStream_t st) {
  if ((3 * p * p) % 4 || H % p || W % p) return -1;
  if (prm != nullptr && (perm == nullptr || box == nullptr)) return -2;
  const long n = (long)B * (H / p) * (W / p) * (3 * p * p / 4);
  if (n == 0) return 0;
  if (p == 16 && W % 4 == 0 && (reinterpret_cast<uintptr_t>(img) & 3) == 0) {
    mix_patches16_kernel<<<cdiv((long)B * (H / 16) * (W / 16) * 64, 256), 256, 0, st>>>(img, perm, prm, box, out, B,
                                                                                         H, W);
    return 0;
  }
  mix_patches_kernel<<<cdiv(n, 256), 256, 0, st>>>(img, perm, prm, box, out, B, H, W, p);
  return 0;
}

// ------------------------------------------------------------------ random masking ids
// random_masking's permutation algebra (utils_mae.py:88-102) for rows of uniform noise [R, N]
// (R = 1: one permutation shared by the rank's batch; R = B: per-sample), one workgroup per row:
// the rank of element i is the number of elements that sort before it (ties broken by index: a
// stable argsort), so ids_shuffle[rank_i] = i, ids_restore[i] = rank_i and mask[i] = rank_i >= keep.
// Written as int64 (the API's dtype) and int32 (the gather kernels' operand, keep32 = the first
// ``keep`` of each row contiguous) -- replaces two radix sorts, their copies and the scatter of the
// torch composition (a dozen small launches per step).
namespace {
__global__ __launch_bounds__(256) void mask_ids_kernel(const float* __restrict__ noise, int N, int keep,
                                                       int64_t* __restrict__ shuffle, int64_t* __restrict__ restore,
                                                       int* __restrict__ keep32, int* __restrict__ restore32,
                                                       float* __restrict__ mask) {
  __shared__ float v[1024];
  const long r = blockIdx.x;
  for (int i = threadIdx.x; i < N; i += 256) v[i] = noise[r * N + i];
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += 256) {
    const float x = v[i];
    int rank = 0;
    for (int j = 0; j < N; ++j) {
      const float y = v[j];
      rank += (y < x) || (y == x && j < i);
    }
    shuffle[r * N + rank] = i;
    restore[r * N + i] = rank;
    restore32[r * N + i] = rank;
    if (rank < keep) keep32[r * keep + rank] = i;
    mask[r * N + i] = rank >= keep ? 1.f : 0.f;
  }
}
}  // namespace

int jm_mask_ids(const float* noise, int R, int N, int keep, int64_t* shuffle, int64_t* restore, int* keep32,
                int* restore32, float* mask, hipStream_t st) {
  if (N > 1024 || keep > N || keep < 0 || R <= 0) return -1;
  mask_ids_kernel<<<R, 256, 0, st>>>(noise, N, keep, shuffle, restore, keep32, restore32, mask);
  return 0;
}

JM_DEBUG_EXPORT(mae)
