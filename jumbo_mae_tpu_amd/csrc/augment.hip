// Device-side RandomResizedCrop (bicubic) + horizontal flip of decoded uint8 images (gfx950).
//
// The pretraining input transform (reference src/dataset.py:56-82: RandomResizedCrop(224,
// scale=(0.2, 1), bicubic) -> RandomHorizontalFlip -> PILToTensor) costs a loader worker ~1.4 ms
// per ImageNet-sized picture in PIL's resampler, as much as the JPEG decode itself
// (profiles/r5_data_rate.txt).  With the device augment the workers only decode, draw the crop /
// flip parameters from the same per-sample RNG and ship the crop window (data/loader.py
// DeviceAugment); these kernels then produce the uint8 CHW batch on the GPU, BIT-EXACT to PIL:
// the same coefficient arithmetic as Pillow's Resample.c (precompute_coeffs in double, bicubic
// a = -0.5, support scaled by the downscale factor, normalisation by the running sum, 22-bit fixed
// point, horizontal pass into 8-bit rows, then the vertical pass, clip8 rounding), evaluated in
// the ORIGINAL image coordinates (the window only offsets the pixel reads), with floating-point
// contraction off so every double operation rounds like the host's.
//
//   rrc_h_kernel  block (image, row block): thread = output column; its <= RRC_KMAX taps in
//                 registers; writes the 8-bit horizontal pass of the rows the vertical pass needs
//   rrc_v_kernel  block (image, 16 output rows): the rows' vertical taps in LDS; thread = output
//                 column; writes out[b][c][y][flip ? S-1-x : x]
//
// Per-image table (int64 x RRC_TAB): src offset, window rows / cols, window origin y0 / x0, image
// H / W, crop i / j / h / w (PIL box (j, i, j + w, i + h)), flip, offset of its rows in tmp.
#include "common.h"

namespace {

constexpr int PB = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2
constexpr int RRC_TAB = 13;
constexpr int RRC_KMAX = 24;  // taps: support 2 x scale -> crops up to 5.75 x the output size
constexpr int RRC_VROWS = 16;

#pragma clang fp contract(off)

JM_DEVICE double bicubic_w(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

struct Axis {
  double scale, support, ss;
  float in0;
  int in_size;
};

JM_DEVICE Axis make_axis(int in_size, float in0, float in1, int out_size) {
  Axis a;
  a.scale = (double)(in1 - in0) / out_size;
  const double filterscale = a.scale < 1.0 ? 1.0 : a.scale;
  a.support = 2.0 * filterscale;  // bicubic support 2
  a.ss = 1.0 / filterscale;
  a.in0 = in0;
  a.in_size = in_size;
  return a;
}

// first input index and tap count of output coordinate xx
JM_DEVICE int axis_bounds(const Axis& a, int xx, double& center, int& xmin) {
  center = a.in0 + (xx + 0.5) * a.scale;
  xmin = (int)(center - a.support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + a.support + 0.5);
  if (xmax > a.in_size) xmax = a.in_size;
  return xmax - xmin;
}

// the fixed-point taps of output coordinate xx -> k[0 .. n) (n <= RRC_KMAX, checked by the host)
JM_DEVICE int axis_taps(const Axis& a, int xx, int* k, int& xmin) {
  double center;
  const int n = axis_bounds(a, xx, center, xmin);
  double ww = 0.0;
#pragma unroll
  for (int x = 0; x < RRC_KMAX; ++x)
    if (x < n) ww += bicubic_w(((double)(x + xmin) - center + 0.5) * a.ss);
#pragma unroll
  for (int x = 0; x < RRC_KMAX; ++x) {
    if (x < n) {
      double w = bicubic_w(((double)(x + xmin) - center + 0.5) * a.ss);
      if (ww != 0.0) w /= ww;
      k[x] = w < 0 ? (int)(-0.5 + w * (1 << PB)) : (int)(0.5 + w * (1 << PB));
    } else {
      k[x] = 0;
    }
  }
  return n;
}

JM_DEVICE uint8_t clip8(int v) {
  if (v >= (1 << PB << 8)) return 255;
  if (v <= 0) return 0;
  return (uint8_t)(v >> PB);
}

struct Img {
  long src, tmp;
  int wh, ww, y0, x0, H, W, i, j, ch, cw, flip;
};

JM_DEVICE Img load_img(const int64_t* __restrict__ tab, int b) {
  const int64_t* t = tab + (long)b * RRC_TAB;
  Img m;
  m.src = t[0];
  m.wh = (int)t[1];
  m.ww = (int)t[2];
  m.y0 = (int)t[3];
  m.x0 = (int)t[4];
  m.H = (int)t[5];
  m.W = (int)t[6];
  m.i = (int)t[7];
  m.j = (int)t[8];
  m.ch = (int)t[9];
  m.cw = (int)t[10];
  m.flip = (int)t[11];
  m.tmp = t[12];
  return m;
}

// rows [first, last) of the source that the vertical pass reads
JM_DEVICE void vrows(const Img& m, int S, int& first, int& last) {
  const Axis av = make_axis(m.H, (float)m.i, (float)(m.i + m.ch), S);
  double c;
  int y;
  axis_bounds(av, 0, c, first);
  const int n = axis_bounds(av, S - 1, c, y);
  last = y + n;
}

__global__ __launch_bounds__(256) void rrc_h_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ tab,
                                                    uint8_t* __restrict__ tmp, int S, int rows_per_blk) {
  const Img m = load_img(tab, blockIdx.x);
  int first, last;
  vrows(m, S, first, last);
  const int r0 = first + blockIdx.y * rows_per_blk;
  const int r1 = min(last, r0 + rows_per_blk);
  if (r0 >= r1) return;
  const Axis ah = make_axis(m.W, (float)m.j, (float)(m.j + m.cw), S);
  for (int xx = threadIdx.x; xx < S; xx += blockDim.x) {
    int k[RRC_KMAX], xmin;
    const int n = axis_taps(ah, xx, k, xmin);
    const uint8_t* base = src + m.src + (long)(xmin - m.x0) * 3;
    for (int r = r0; r < r1; ++r) {
      const uint8_t* p = base + (long)(r - m.y0) * m.ww * 3;
      int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
#pragma unroll
      for (int x = 0; x < RRC_KMAX; ++x) {
        if (x < n) {
          s0 += (int)p[3 * x] * k[x];
          s1 += (int)p[3 * x + 1] * k[x];
          s2 += (int)p[3 * x + 2] * k[x];
        }
      }
      uint8_t* o = tmp + m.tmp + ((long)(r - first) * S + xx) * 3;
      o[0] = clip8(s0);
      o[1] = clip8(s1);
      o[2] = clip8(s2);
    }
  }
}

__global__ __launch_bounds__(256) void rrc_v_kernel(const uint8_t* __restrict__ tmp, const int64_t* __restrict__ tab,
                                                    uint8_t* __restrict__ out, int S) {
  __shared__ int kv[RRC_VROWS][RRC_KMAX];
  __shared__ int vmin[RRC_VROWS], vn[RRC_VROWS];
  const int b = blockIdx.x;
  const Img m = load_img(tab, b);
  int first, last;
  vrows(m, S, first, last);
  const int yy0 = blockIdx.y * RRC_VROWS;
  if (threadIdx.x < RRC_VROWS && yy0 + (int)threadIdx.x < S) {
    const Axis av = make_axis(m.H, (float)m.i, (float)(m.i + m.ch), S);
    int k[RRC_KMAX], ymin;
    const int n = axis_taps(av, yy0 + threadIdx.x, k, ymin);
#pragma unroll
    for (int x = 0; x < RRC_KMAX; ++x) kv[threadIdx.x][x] = k[x];
    vmin[threadIdx.x] = ymin - first;
    vn[threadIdx.x] = n;
  }
  __syncthreads();
  const long plane = (long)S * S;
  uint8_t* ob = out + (long)b * 3 * plane;
  for (int r = 0; r < RRC_VROWS && yy0 + r < S; ++r) {
    const int yy = yy0 + r, n = vn[r];
    const uint8_t* base = tmp + m.tmp + (long)vmin[r] * S * 3;
    for (int xx = threadIdx.x; xx < S; xx += blockDim.x) {
      int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
      const uint8_t* p = base + xx * 3;
      for (int y = 0; y < n; ++y) {
        const int kk = kv[r][y];
        s0 += (int)p[0] * kk;
        s1 += (int)p[1] * kk;
        s2 += (int)p[2] * kk;
        p += (long)S * 3;
      }
      const int ox = m.flip ? S - 1 - xx : xx;
      ob[(long)yy * S + ox] = clip8(s0);
      ob[plane + (long)yy * S + ox] = clip8(s1);
      ob[2 * plane + (long)yy * S + ox] = clip8(s2);
    }
  }
}

}  // namespace

// src: concatenated HWC uint8 crop windows; tab: [B, RRC_TAB] int64 (see top); tmp: >= sum over
// images of (their vertical-pass rows) x S x 3 bytes at the table's offsets; out: [B, 3, S, S] uint8.
// tmp_rows_max: the largest per-image row count (grid height).  Returns 0, or <0 on bad arguments.
int jm_rrc_resize(const uint8_t* src, const int64_t* tab, int B, int S, uint8_t* tmp, int tmp_rows_max,
                  uint8_t* out, hipStream_t st) {
  if (B <= 0 || S <= 0 || S > 4096 || tmp_rows_max <= 0) return -1;
  const int rows_per_blk = 32;
  rrc_h_kernel<<<dim3(B, (tmp_rows_max + rows_per_blk - 1) / rows_per_blk), 256, 0, st>>>(src, tab, tmp, S,
                                                                                         rows_per_blk);
  rrc_v_kernel<<<dim3(B, (S + RRC_VROWS - 1) / RRC_VROWS), 256, 0, st>>>(tmp, tab, out, S);
  return 0;
}

int jm_rrc_kmax() { return RRC_KMAX; }

JM_DEBUG_EXPORT(augment)
