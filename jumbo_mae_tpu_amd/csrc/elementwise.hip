// Fused elementwise kernels of the transformer blocks (gfx950).
//
//  gelu_fwd           a = gelu_tanh(h)                         (flax nn.gelu, approximate=True)
//  gelu_bwd_colsum    dh = da * gelu'(h);  bias_grad += sum_rows dh     (fused bias-grad of w1)
//  colsum             acc += sum_rows dy                                (bias-grad of plain Dense)
//  residual_fwd       out[b,t,:] = x[b,t,:] + m[b] * s[:] * y[b*T+t,:] (droppath + LayerScale)
//  residual_bwd       dy = m[b]*s[:]*dout (bf16);  ds += sum_rows m[b]*dout*y
//
// All loads/stores are 16 B per lane (8 x bf16 or 2 x float4): hipcc does not vectorise bf16.
// Column reductions use a 2-D decomposition: each thread owns 8 adjacent columns and walks a
// slab of rows, keeps the 8 partial sums in registers, merges the block's row-slots through LDS
// float atomics and issues one global atomicAdd per column per block into the fp32 grad buffer.
#include "common.h"

namespace {

constexpr float GELU_C = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float GELU_A = 0.044715f;

JM_DEVICE float gelu_f(float h) {
  const float u = GELU_C * (h + GELU_A * h * h * h);
  return 0.5f * h * (1.f + tanhf(u));
}

JM_DEVICE float gelu_grad(float h) {
  const float u = GELU_C * (h + GELU_A * h * h * h);
  const float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * h * (1.f - t * t) * GELU_C * (1.f + 3.f * GELU_A * h * h);
}

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const uint16_t* __restrict__ h, uint16_t* __restrict__ a,
                                                       long n8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    load8(h + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_f(v[j]);
    store8(a + i * 8, v);
  }
}

// Row/column decomposition shared by the column-reduction kernels.
struct ColPlan {
  int cgs, tpr, rps;
};

JM_DEVICE ColPlan col_plan(int N) {
  ColPlan p;
  p.cgs = N / 8;
  p.tpr = p.cgs < 256 ? p.cgs : 256;
  p.rps = 256 / p.tpr;
  return p;
}

// MODE 0: colsum(dy)          -> acc
// MODE 1: gelu_bwd(h, da)     -> out (bf16), acc += colsum(out)
// MODE 2: residual_bwd        -> out = m*s*dout (bf16, dout fp32), acc += colsum(m*dout*y)
template <int MODE>
__global__ __launch_bounds__(256) void rowcol_kernel(const void* __restrict__ in0, const uint16_t* __restrict__ in1,
                                                     uint16_t* __restrict__ out, float* __restrict__ acc,
                                                     const float* __restrict__ scale, const float* __restrict__ mask,
                                                     int M, int N, int T, int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [N]
  const ColPlan p = col_plan(N);
  const int slot = threadIdx.x / p.tpr, c = threadIdx.x % p.tpr;
  const bool active = slot < p.rps;
  if (acc) {
    for (int i = threadIdx.x; i < N; i += 256) red[i] = 0.f;
    __syncthreads();
  }
  const int r_begin = blockIdx.x * rows_per_block;
  int r_end = r_begin + rows_per_block;
  if (r_end > M) r_end = M;
  if (active) {
    for (int cg = c; cg < p.cgs; cg += p.tpr) {
      const int col = cg * 8;
      float s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = 0.f;
      float sc[8];
      if (MODE == 2) {
        if (scale) {
          load8(scale + col, sc);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) sc[j] = 1.f;
        }
      }
      for (int r = r_begin + slot; r < r_end; r += p.rps) {
        const long off = (long)r * N + col;
        if (MODE == 0) {
          float v[8];
          load8((const uint16_t*)in0 + off, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += v[j];
        } else if (MODE == 1) {
          float hv[8], dv[8];
          load8((const uint16_t*)in0 + off, hv);
          load8(in1 + off, dv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            // round dh to bf16 first so the bias grad equals the colsum of what the GEMMs consume
            dv[j] = bf2f(f2bf(dv[j] * gelu_grad(hv[j])));
            s[j] += dv[j];
          }
          store8(out + off, dv);
        } else {
          float dv[8], yv[8], o[8];
          load8((const float*)in0 + off, dv);
          const float m = mask ? mask[r / T] : 1.f;
          if (scale) load8(in1 + off, yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float md = m * dv[j];
            o[j] = md * sc[j];
            if (scale) s[j] += md * yv[j];
          }
          store8(out + off, o);
        }
      }
      if (acc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(&red[col + j], s[j]);
      }
    }
  }
  if (acc) {
    __syncthreads();
    for (int i = threadIdx.x; i < N; i += 256) atomicAdd(&acc[i], red[i]);
  }
}

__global__ __launch_bounds__(256) void residual_fwd_kernel(const float* __restrict__ x, long sB, long sT, int T,
                                                           const uint16_t* __restrict__ y,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ mask, float* __restrict__ out,
                                                           int rows, int D) {
  const int cgs = D / 8;
  const long total = (long)rows * cgs;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int row = (int)(i / cgs);
    const int col = (int)(i - (long)row * cgs) * 8;
    const int b = row / T, t = row - b * T;
    float xv[8], yv[8], sc[8];
    load8(x + b * sB + t * sT + col, xv);
    load8(y + (long)row * D + col, yv);
    const float m = mask ? mask[b] : 1.f;
    if (scale) {
      load8(scale + col, sc);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[j] = 1.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] += m * sc[j] * yv[j];
    store8(out + (long)row * D + col, xv);
  }
}

int grid_for(long work, int per_thread_items = 1) {
  long b = (work + 256L * per_thread_items - 1) / (256L * per_thread_items);
  if (b > 256L * 16) b = 256L * 16;
  if (b < 1) b = 1;
  return (int)b;
}

template <int MODE>
void launch_rowcol(const void* in0, const uint16_t* in1, uint16_t* out, float* acc, const float* scale,
                   const float* mask, int M, int N, int T, hipStream_t st) {
  // each row-slot should walk >= 16 rows; cap the grid so the per-block atomics stay cheap
  const int cgs = N / 8;
  const int tpr = cgs < 256 ? cgs : 256;
  const int rps = 256 / tpr;
  int rows_per_block = rps * 16;
  int nb = (M + rows_per_block - 1) / rows_per_block;
  if (nb > 2048) {
    nb = 2048;
    rows_per_block = (M + nb - 1) / nb;
  }
  if (nb < 1) nb = 1;
  const size_t smem = acc ? N * sizeof(float) : 0;
  rowcol_kernel<MODE><<<nb, 256, smem, st>>>(in0, in1, out, acc, scale, mask, M, N, T, rows_per_block);
}

}  // namespace

int jm_gelu_fwd(const uint16_t* h, uint16_t* a, long n, hipStream_t st) {
  if (n % 8) return -1;
  gelu_fwd_kernel<<<grid_for(n / 8), 256, 0, st>>>(h, a, n / 8);
  return 0;
}

int jm_gelu_bwd(const uint16_t* h, const uint16_t* da, uint16_t* dh, float* bias_grad, int M, int N,
                hipStream_t st) {
  if (N % 8) return -1;
  launch_rowcol<1>(h, da, dh, bias_grad, nullptr, nullptr, M, N, 1, st);
  return 0;
}

int jm_colsum_bf16(const uint16_t* x, float* acc, int M, int N, hipStream_t st) {
  if (N % 8) return -1;
  launch_rowcol<0>(x, nullptr, nullptr, acc, nullptr, nullptr, M, N, 1, st);
  return 0;
}

int jm_residual_fwd(const float* x, long sB, long sT, int B, int T, int D, const uint16_t* y, const float* scale,
                    const float* mask, float* out, hipStream_t st) {
  if (D % 8) return -1;
  const long work = (long)B * T * (D / 8);
  residual_fwd_kernel<<<grid_for(work), 256, 0, st>>>(x, sB, sT, T, y, scale, mask, out, B * T, D);
  return 0;
}

int jm_residual_bwd(const float* dout, const uint16_t* y, const float* scale, const float* mask, float* dscale,
                    uint16_t* dy, int B, int T, int D, hipStream_t st) {
  if (D % 8) return -1;
  launch_rowcol<2>(dout, y, dy, dscale, scale, mask, B * T, D, T, st);
  return 0;
}
