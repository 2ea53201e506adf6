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
