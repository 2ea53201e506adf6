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
// in slot order and stores one partial row per block; a row-lane column sum (colsum_rows_kernel)
// adds the partial rows into the fp32 grad buffer in a fixed order (no float atomics: the same
// bits on every run).
#include "common.h"

namespace {

// one GELU implementation for every kernel (common.h, sigmoid form)
JM_DEVICE float gelu_f(float h) { return gelu_tanh_f(h); }
JM_DEVICE float gelu_grad(float h) { return gelu_grad_f(h); }

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
// MODE 3: as MODE 1 with in0 = the saved gelu'(h) (a multiply instead of the derivative)
// MODE 2: residual_bwd        -> out = m*s*dout (bf16, dout fp32), acc += colsum(m*dout*y),
//                                acc2 += colsum(out)  (bias gradient of the Dense that produced y)
template <int MODE>
__global__ __launch_bounds__(256) void rowcol_kernel(const void* __restrict__ in0, const uint16_t* __restrict__ in1,
                                                     uint16_t* __restrict__ out, float* __restrict__ acc,
                                                     const float* __restrict__ scale, const float* __restrict__ mask,
                                                     int M, int N, int T, int rows_per_block, long sB, long sT,
                                                     float* __restrict__ acc2, long yB, long yT, int cw,
                                                     DropIO drop, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) float red_s[];  // [2][rps][nc] slot partials
  // 2-D grid: blockIdx.y picks a chunk of cw (<= 2048, % 8 == 0) columns, blockIdx.x a slab of rows
  const int c0 = blockIdx.y * cw;
  const int nc = (N - c0) < cw ? (N - c0) : cw;
  const ColPlan p = col_plan(nc);
  const int slot = threadIdx.x / p.tpr, c = threadIdx.x % p.tpr;
  const bool active = slot < p.rps;
  // rps * nc <= 2048 (tpr = nc / 8 up to 256 threads): one plain store per (slot, column)
  float* red = red_s + slot * nc - c0;  // index with absolute column
  float* red2 = red_s + 2048 + slot * nc - c0;
  const int r_begin = blockIdx.x * rows_per_block;
  int r_end = r_begin + rows_per_block;
  if (r_end > M) r_end = M;
  if (active) {
    for (int cg = c; cg < p.cgs; cg += p.tpr) {
      const int col = c0 + cg * 8;
      float s[8], s2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = s2[j] = 0.f;
      float sc[8];
      if (MODE == 2) {
        if (scale) {
          load8(scale + col, sc);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) sc[j] = 1.f;
        }
      }
      // U rows per trip: all loads of a trip are issued before any use (memory-level parallelism;
      // one load per trip left this loop latency-bound at ~55 % of HBM bandwidth)
      constexpr int U = 4;
      for (int r0 = r_begin + slot; r0 < r_end; r0 += U * p.rps) {
        float a[U][8], b[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = r0 + u * p.rps;
          if (r < r_end) {
            const long off = (long)r * N + col;
            if (MODE == 0) {
              load8((const uint16_t*)in0 + off, a[u]);
            } else if (MODE == 1 || MODE == 3) {
              load8((const uint16_t*)in0 + off, a[u]);
              load8(in1 + off, b[u]);
            } else {  // dout is a [B, T, D] view with strides (sB, sT, 1)
              load8((const float*)in0 + (r / T) * sB + (r % T) * sT + col, a[u]);
              if (scale) load8(in1 + (r / T) * yB + (r % T) * yT + col, b[u]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = r0 + u * p.rps;
          if (r >= r_end) break;
          const long off = (long)r * N + col;
          if (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += a[u][j];
          } else if (MODE == 1 || MODE == 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              // round dh to bf16 first so the bias grad equals the colsum of what the GEMMs consume
              b[u][j] = bf2f(f2bf(b[u][j] * (MODE == 3 ? a[u][j] : gelu_grad(a[u][j]))));
              s[j] += b[u][j];
            }
            store8(out + off, b[u]);
          } else {
            float o[8], f[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
            const float m = mask ? mask[r / T] : 1.f;
            if (drop.seed) drop_factors<8>(drop, drop.ioff + (r / T) * yB + (r % T) * yT + col, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float md = m * a[u][j] * f[j];  // f: the dropout of y
              o[j] = md * sc[j];
              if (scale) s[j] += md * b[u][j];
              s2[j] += bf2f(f2bf(o[j]));  // colsum of the bf16 values the GEMMs consume
            }
            store8(out + (r / T) * yB + (r % T) * yT + col, o);
          }
        }
      }
      if (acc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[col + j] = s[j];
      }
      if (MODE == 2 && acc2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red2[col + j] = s2[j];
      }
    }
  }
  if (!acc && !acc2) return;
  __syncthreads();
  // the block's partial row (slots summed in order) -> ws[blockIdx.x][c0 ..), acc2's after acc's
  const long wrow = (long)blockIdx.x * N + c0;
  for (int i = threadIdx.x; i < nc; i += 256) {
    if (acc) {
      float a = 0.f;
      for (int k = 0; k < p.rps; ++k) a += red_s[k * nc + i];
      ws[wrow + i] = a;
    }
    if (MODE == 2 && acc2) {
      float a = 0.f;
      for (int k = 0; k < p.rps; ++k) a += red_s[2048 + k * nc + i];
      ws[(long)gridDim.x * N + wrow + i] = a;
    }
  }
}

__global__ __launch_bounds__(256) void residual_fwd_kernel(const float* __restrict__ x, long sB, long sT, int T,
                                                           const uint16_t* __restrict__ y,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ mask, float* __restrict__ out,
                                                           int rows, int D, long oB, long oT, DropIO drop) {
  const int cgs = D / 8;
  const long total = (long)rows * cgs;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int row = (int)(i / cgs);
    const int col = (int)(i - (long)row * cgs) * 8;
    const int b = row / T, t = row - b * T;
    float xv[8], yv[8], sc[8];
    load8(x + b * sB + t * sT + col, xv);
    load8(y + (long)row * D + col, yv);
    if (drop.seed) {
      float f[8];
      drop_factors<8>(drop, drop.ioff + (long)row * D + col, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) yv[j] *= f[j];
    }
    const float m = mask ? mask[b] : 1.f;
    if (scale) {
      load8(scale + col, sc);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) sc[j] = 1.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] += m * sc[j] * yv[j];
    store8(out + b * oB + t * oT + col, xv);
  }
}

int grid_for(long work, int per_thread_items = 1) {
  long b = (work + 256L * per_thread_items - 1) / (256L * per_thread_items);
  if (b > 256L * 16) b = 256L * 16;
  if (b < 1) b = 1;
  return (int)b;
}

void launch_colsum(const float* part, float* g, long n4, int S, long ld, int store, hipStream_t st);

// rowcol launch geometry: column chunks of cw <= 2048 x nb row slabs of rows_per_block rows
struct RowcolGeom {
  int cw, ncol, nb, rows_per_block;
};

RowcolGeom rowcol_geom(int M, int N) {
  // each row-slot walks >= 16 rows, at most 1024 blocks in total (their partial rows are summed
  // by a second pass).  Few rows (< 8192): chunks narrowed so ~256 blocks keep >= 32 rows each.
  int cw = N < 2048 ? N : 2048;
  if (M < 32 * 256) {
    const int nbr = M / 32 > 1 ? M / 32 : 1;
    int nch = (256 + nbr - 1) / nbr;
    if (nch > N / 64) nch = N / 64 > 1 ? N / 64 : 1;
    const int w = ((N + nch - 1) / nch + 7) / 8 * 8;
    if (w < cw) cw = w;
  }
  const int ncol = (N + cw - 1) / cw;
  const int cgs = cw / 8;
  const int tpr = cgs < 256 ? cgs : 256;
  const int rps = 256 / tpr;
  int rows_per_block = rps * 16;
  int nb = (M + rows_per_block - 1) / rows_per_block;
  // few rows (the jumbo residual / GELU backward: 512 x 3072 / 512 x 12288, the CLS-row residual:
  // 1536 x 1024): spread over >= 256 blocks in total, one per CU -- 16 rows per slot gave 48-192
  // blocks and a latency-bound 16-20 us per call
  const int want = (256 + ncol - 1) / ncol;
  if (nb < want) {
    rows_per_block = (M + want - 1) / want;
    if (rows_per_block < rps) rows_per_block = rps;
    nb = (M + rows_per_block - 1) / rows_per_block;
  }
  const int cap = 1024 / ncol > 1 ? 1024 / ncol : 1;
  if (nb > cap) {
    nb = cap;
    rows_per_block = (M + nb - 1) / nb;
  }
  if (nb < 1) nb = 1;
  return RowcolGeom{cw, ncol, nb, rows_per_block};
}

// ws: the block partial rows, rowcol_ws_floats(M, N, 2 if acc2 else 1) floats
template <int MODE>
void launch_rowcol(const void* in0, const uint16_t* in1, uint16_t* out, float* acc, const float* scale,
                   const float* mask, int M, int N, int T, hipStream_t st, float* ws, long sB = 0, long sT = 0,
                   float* acc2 = nullptr, long yB = -1, long yT = -1, JmDrop drop = JmDrop{nullptr, 0u, 1.f, 0}) {
  if (yB < 0) {  // y / out contiguous [M, N]
    yB = (long)T * N;
    yT = N;
  }
  const RowcolGeom g = rowcol_geom(M, N);
  const size_t smem = (acc || acc2) ? 4096 * sizeof(float) : 0;
  rowcol_kernel<MODE><<<dim3(g.nb, g.ncol), 256, smem, st>>>(in0, in1, out, acc, scale, mask, M, N, T,
                                                              g.rows_per_block, sB, sT, acc2, yB, yT, g.cw, drop, ws);
  if (acc) launch_colsum(ws, acc, N / 4, g.nb, N, 0, st);
  if (MODE == 2 && acc2) launch_colsum(ws + (long)g.nb * N, acc2, N / 4, g.nb, N, 0, st);
}

}  // namespace

int jm_gelu_fwd(const uint16_t* h, uint16_t* a, long n, hipStream_t st) {
  if (n % 8) return -1;
  gelu_fwd_kernel<<<grid_for(n / 8), 256, 0, st>>>(h, a, n / 8);
  return 0;
}

// floats of the partial-row workspace of a column-reducing elementwise call (nacc: 1, or 2 for
// residual_bwd with both dscale and dbias); 0 when N is not supported
long jm_rowcol_ws_floats(int M, int N, int nacc) {
  if (N % 8 || M < 1) return 0;
  return (long)rowcol_geom(M, N).nb * N * nacc;
}

int jm_gelu_bwd(const uint16_t* h, const uint16_t* da, uint16_t* dh, float* bias_grad, int M, int N,
                hipStream_t st, int deriv, float* ws) {
  if (N % 8 || (bias_grad && !ws)) return -1;
  if (deriv)
    launch_rowcol<3>(h, da, dh, bias_grad, nullptr, nullptr, M, N, 1, st, ws);
  else
    launch_rowcol<1>(h, da, dh, bias_grad, nullptr, nullptr, M, N, 1, st, ws);
  return 0;
}

int jm_colsum_bf16(const uint16_t* x, float* acc, int M, int N, hipStream_t st, float* ws) {
  if (N % 8 || !ws) return -1;
  launch_rowcol<0>(x, nullptr, nullptr, acc, nullptr, nullptr, M, N, 1, st, ws);
  return 0;
}

int jm_residual_fwd(const float* x, long sB, long sT, int B, int T, int D, const uint16_t* y, const float* scale,
                    const float* mask, float* out, long oB, long oT, hipStream_t st, JmDrop drop) {
  if (D % 8) return -1;
  const long work = (long)B * T * (D / 8);
  residual_fwd_kernel<<<grid_for(work), 256, 0, st>>>(x, sB, sT, T, y, scale, mask, out, B * T, D, oB, oT, drop);
  return 0;
}

int jm_residual_bwd(const float* dout, long dB, long dT, const uint16_t* y, const float* scale, const float* mask,
                    float* dscale, uint16_t* dy, int B, int T, int D, float* dbias, long yB, long yT, hipStream_t st,
                    JmDrop drop, float* ws) {
  if (D % 8) return -1;
  if ((dscale || dbias) && !ws) return -1;
  launch_rowcol<2>(dout, y, dy, dscale, scale, mask, B * T, D, T, st, ws, dB, dT, dbias, yB, yT, drop);
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Split-K epilogue of the weight-gradient GEMMs: g[i] += sum_s part[s][i] (fp32), one pass.
void jm_zero_f32(float* p, long n, hipStream_t st);
namespace {
// g[i] += sum_s part[s][i], one thread per float4 column walking all S rows (n large).
// ``ld``: row stride of part in floats (n for the packed partial slices, a strided view otherwise).
__global__ __launch_bounds__(256) void splitk_reduce_add_kernel(const float* __restrict__ part,
                                                                float* __restrict__ g, long n4, int S, long ld) {
  const long n = ld;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 1 < S; s += 2) {
      float v[4], w[4];
      load4(part + (long)s * n + i * 4, v);
      load4(part + (long)(s + 1) * n + i * 4, w);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += v[j] + w[j];
    }
    if (s < S) {
      float v[4];
      load4(part + (long)s * n + i * 4, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += v[j];
    }
    float o[4];
    load4(g + i * 4, o);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] += acc[j];
    store4(g + i * 4, o);
  }
}

// The same for few columns and many rows (per-sample bias partials: n = 3D, S = batch; token
// partials): RL row lanes per column, each summing every RL-th row (4 loads in flight), then a
// fixed-order LDS tree over the lanes -- the same bits on every run (the round-3 form split the
// rows over grid.y slices summed with float atomics, whose order varies).
// One workgroup per 256 / RL float4 columns; STORE: g = sum (g not read).
template <int RL>
__global__ __launch_bounds__(256) void colsum_rows_kernel(const float* __restrict__ part, float* __restrict__ g,
                                                          long n4, int S, long ld, int store) {
  constexpr int CW = 256 / RL;
  __shared__ float4 red[256];
  const int c = threadIdx.x % CW, rl = threadIdx.x / CW;
  const long i = blockIdx.x * (long)CW + c;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    const float4* p = reinterpret_cast<const float4*>(part) + i;
    const long l4 = ld / 4;
    int s = rl;
    for (; s + 3 * RL < S; s += 4 * RL) {
      const float4 a = p[(long)s * l4], b = p[(long)(s + RL) * l4];
      const float4 e = p[(long)(s + 2 * RL) * l4], f = p[(long)(s + 3 * RL) * l4];
      acc.x += (a.x + b.x) + (e.x + f.x);
      acc.y += (a.y + b.y) + (e.y + f.y);
      acc.z += (a.z + b.z) + (e.z + f.z);
      acc.w += (a.w + b.w) + (e.w + f.w);
    }
    for (; s < S; s += RL) {
      const float4 a = p[(long)s * l4];
      acc.x += a.x;
      acc.y += a.y;
      acc.z += a.z;
      acc.w += a.w;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
#pragma unroll
  for (int h = RL / 2; h >= 1; h >>= 1) {
    if (rl < h) {
      const float4 o = red[threadIdx.x + h * CW];
      float4& r = red[threadIdx.x];
      r.x += o.x;
      r.y += o.y;
      r.z += o.z;
      r.w += o.w;
    }
    __syncthreads();
  }
  if (rl == 0 && i < n4) {
    float4* gp = reinterpret_cast<float4*>(g) + i;
    float4 o = store ? make_float4(0.f, 0.f, 0.f, 0.f) : *gp;
    const float4 r = red[c];
    o.x += r.x;
    o.y += r.y;
    o.z += r.z;
    o.w += r.w;
    *gp = o;
  }
}

// column sums over S rows of stride ld into g (store: g = sum): the one-pass kernel when the
// columns alone fill the chip, else colsum_rows_kernel with the row lanes sized to ~32 rows each
void launch_colsum(const float* part, float* g, long n4, int S, long ld, int store, hipStream_t st) {
  const long blocks = (n4 + 255) / 256;
  if (blocks >= 512 || S < 16) {
    if (store) jm_zero_f32(g, n4 * 4, st);
    splitk_reduce_add_kernel<<<(unsigned)(blocks > 4096 ? 4096 : blocks), 256, 0, st>>>(part, g, n4, S, ld);
    return;
  }
  int rl = 16;
  while (rl < 256 && S > 32 * rl) rl *= 2;
  const unsigned nb = (unsigned)((n4 * rl + 255) / 256);
  switch (rl) {
    case 16: colsum_rows_kernel<16><<<nb, 256, 0, st>>>(part, g, n4, S, ld, store); break;
    case 32: colsum_rows_kernel<32><<<nb, 256, 0, st>>>(part, g, n4, S, ld, store); break;
    case 64: colsum_rows_kernel<64><<<nb, 256, 0, st>>>(part, g, n4, S, ld, store); break;
    case 128: colsum_rows_kernel<128><<<nb, 256, 0, st>>>(part, g, n4, S, ld, store); break;
    default: colsum_rows_kernel<256><<<nb, 256, 0, st>>>(part, g, n4, S, ld, store); break;
  }
}

// The same with S a template constant, one float4 per thread and every load of the thread -- the S
// partial slices and g -- issued before the first add: the loop form kept two 16-B loads in flight
// per thread and ran the weight-gradient reductions at ~4.8 TB/s although the slices were just
// written (MALL-resident).
// STORE: g = sum (g is not read: the first gradient contribution of a step, see jm_zero_ranges)
template <int S, bool STORE = false>
__global__ __launch_bounds__(256) void splitk_reduce_add_s_kernel(const float* __restrict__ part,
                                                                  float* __restrict__ g, long n4) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n4) return;
  const long n = n4 * 4;
  float v[S][4], o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < S; ++s) load4(part + (long)s * n + i * 4, v[s]);
  if (!STORE) load4(g + i * 4, o);
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] += v[s][j];
  store4(g + i * 4, o);
}
}  // namespace

// g[i] (+)= sum_s part[s][i]; store: g[i] = sum (g not read; smaller / longer-S shapes zero g first)
namespace {
__global__ __launch_bounds__(256) void zero_f32_kernel(float* __restrict__ p, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = 0.f;
}
}  // namespace

// g[0:n] = 0 by a kernel, not hipMemsetAsync: a memset captured into a HIP graph left store-mode
// gradients as garbage on replay (tests/test_graph_gpu.py, tools/graph_grad_diag.py)
void jm_zero_f32(float* p, long n, hipStream_t st) {
  if (n <= 0) return;
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  zero_f32_kernel<<<(unsigned)blocks, 256, 0, st>>>(p, n);
}

int jm_splitk_reduce_add(const float* part, float* g, long n, int S, hipStream_t st, int store) {
  if (n % 4) return -1;
  const long n4 = n / 4;
  if (S >= 1 && S <= 16 && n4 >= 256L * 256) {  // large slices: the all-loads-first kernel
    const unsigned nb = (unsigned)((n4 + 255) / 256);
    switch (S) {
#define JM_SKR(SS)                                                                     \
  case SS:                                                                             \
    if (store) splitk_reduce_add_s_kernel<SS, true><<<nb, 256, 0, st>>>(part, g, n4);  \
    else splitk_reduce_add_s_kernel<SS><<<nb, 256, 0, st>>>(part, g, n4);              \
    return 0;
      JM_SKR(1) JM_SKR(2) JM_SKR(3) JM_SKR(4) JM_SKR(5) JM_SKR(6) JM_SKR(7) JM_SKR(8)
      JM_SKR(9) JM_SKR(10) JM_SKR(11) JM_SKR(12) JM_SKR(13) JM_SKR(14) JM_SKR(15) JM_SKR(16)
#undef JM_SKR
      default: break;
    }
  }
  launch_colsum(part, g, n4, S, n, store, st);
  return 0;
}

// g[i] += sum_r x[r * ld + i], i < n: column sums of a row-strided fp32 view (token-parameter
// gradients: the CLS rows of dx, the mask-token partials) added straight into the flat gradient
int jm_colsum_add_f32(const float* x, long ld, int rows, long n, float* g, hipStream_t st) {
  if (n % 4 || ld % 4 || ld < n || rows < 1) return -1;
  launch_colsum(x, g, n / 4, rows, ld, 0, st);
  return 0;
}

// ------------------------------------------------------------------ zero ranges
// The per-step gradient reset of every flat-buffer range NOT written by a store-mode weight
// gradient (ParamStore.zero_grad): desc int64 [n][2] = (offset, count) in floats, one launch;
// block b zeroes 4096 floats of the range that owns it (first block of range r: desc-order prefix).
namespace {
__global__ __launch_bounds__(256) void zero_ranges_kernel(float* __restrict__ base, const long long* __restrict__ desc,
                                                          int n) {
  long long b = blockIdx.x;
  int r = 0;
  for (; r < n; ++r) {
    const long long nb = (desc[2 * r + 1] + 4095) / 4096;
    if (b < nb) break;
    b -= nb;
  }
  if (r >= n) return;
  const long long off = desc[2 * r], cnt = desc[2 * r + 1];
  for (long long i = b * 4096 + threadIdx.x; i < (b + 1) * 4096 && i < cnt; i += 256) base[off + i] = 0.f;
}
}  // namespace

int jm_zero_ranges(float* base, const long long* desc, int n, long long blocks, hipStream_t st) {
  if (n <= 0 || blocks <= 0) return 0;
  zero_ranges_kernel<<<(unsigned)blocks, 256, 0, st>>>(base, desc, n);
  return 0;
}

// ------------------------------------------------------------------ bf16 transpose
// dst[C][R] = src[R][C]^T through a 64 x 64 LDS tile: 16-byte coalesced reads and writes on both
// sides (the transposed weight copies read by the data-gradient MFMA GEMM).  The LDS tile rows
// are padded by one 4-byte word so the column reads of 2-byte elements do not pile onto a bank.
namespace {
constexpr int TT = 64;
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                             int R, int C) {
  __shared__ uint16_t tile[TT][TT + 2];
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
  const int t = threadIdx.x;
  // read: 64 rows x 64 cols = 512 chunks of 8 -> 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = t + k * 256;
    const int r = i >> 3, c = (i & 7) * 8;
    if (r0 + r < R && c0 + c < C) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + (long)(r0 + r) * C + c0 + c);
      const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[r][c + j] = h[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = t + k * 256;
    const int c = i >> 3, r = (i & 7) * 8;  // output row c (source column), 8 source rows
    if (c0 + c < C && r0 + r < R) {
      uint4 v;
      uint16_t* h = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = tile[r + j][c];
      *reinterpret_cast<uint4*>(dst + (long)(c0 + c) * R + r0 + r) = v;
    }
  }
}
}  // namespace

int jm_transpose_bf16(const uint16_t* src, uint16_t* dst, int R, int C, hipStream_t st) {
  if (R % 8 || C % 8) return -1;
  dim3 grid((C + TT - 1) / TT, (R + TT - 1) / TT);
  transpose_bf16_kernel<<<grid, 256, 0, st>>>(src, dst, R, C);
  return 0;
}

// Batched form: every transposed weight copy of a step in ONE launch.  desc[i] = {src, dst, R, C,
// first tile, tiles along C} (int64); workgroup b finds its matrix by binary search over the first
// tiles (the per-call launch gaps of ~120 small transposes per ViT-L step go away).
namespace {
__global__ __launch_bounds__(256) void transpose_bf16_batch_kernel(const long long* __restrict__ desc, int n) {
  __shared__ uint16_t tile[TT][TT + 2];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {  // last i with first_tile(i) <= b
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * 6 + 4] <= b) lo = mid;
    else hi = mid - 1;
  }
  const long long* d = desc + lo * 6;
  const uint16_t* src = reinterpret_cast<const uint16_t*>(d[0]);
  uint16_t* dst = reinterpret_cast<uint16_t*>(d[1]);
  const int R = (int)d[2], C = (int)d[3], local = b - (int)d[4], ntc = (int)d[5];
  const int r0 = (local / ntc) * TT, c0 = (local % ntc) * TT;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = t + k * 256;
    const int r = i >> 3, c = (i & 7) * 8;
    if (r0 + r < R && c0 + c < C) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + (long)(r0 + r) * C + c0 + c);
      const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[r][c + j] = h[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = t + k * 256;
    const int c = i >> 3, r = (i & 7) * 8;
    if (c0 + c < C && r0 + r < R) {
      uint4 v;
      uint16_t* h = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = tile[r + j][c];
      *reinterpret_cast<uint4*>(dst + (long)(c0 + c) * R + r0 + r) = v;
    }
  }
}
}  // namespace

int jm_transpose_bf16_batch(const long long* desc, int n, int tiles, hipStream_t st) {
  if (n <= 0 || tiles <= 0) return -1;
  transpose_bf16_batch_kernel<<<tiles, 256, 0, st>>>(desc, n);
  return 0;
}

// ------------------------------------------------------------------ split-K finish
// out[m][n] (bf16) = sum_s part[s][m][n] (+ bias[n]): the epilogue of a split-K NT GEMM
namespace {
// SC > 0: S == SC at compile time and every partial load of a thread is issued before the first
// add (the runtime loop kept one or two loads in flight: ~5 TB/s on MALL-resident slices)
template <int SC>
__global__ __launch_bounds__(256) void splitk_reduce_bf16_kernel(const float* __restrict__ part, int S, long n8,
                                                                 int N, const float* __restrict__ bias,
                                                                 uint16_t* __restrict__ out) {
  const long total = n8 * 8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float acc[8];
    if constexpr (SC > 0) {
      float v[SC][8];
#pragma unroll
      for (int s = 0; s < SC; ++s) load8(part + (long)s * total + i * 8, v[s]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = v[0][j];
#pragma unroll
      for (int s = 1; s < SC; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[s][j];
    } else {
      load8(part + i * 8, acc);
      for (int s = 1; s < S; ++s) {
        float v[8];
        load8(part + (long)s * total + i * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += v[j];
      }
    }
    if (bias) {
      float b[8];
      load8(bias + (i * 8) % N, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += b[j];
    }
    store8(out + i * 8, acc);
  }
}
}  // namespace

// out[m][n] (fp32, contiguous) = sum_s part[s][m][n] (+ bias[n]) + add[m * add_ld + n]: a split-K NT
// GEMM whose result is summed into an fp32 residual-stream gradient (the shared jumbo MLP's input
// gradient d hc = dx2_cls + W1 dpre) without a bf16 round trip and a separate add pass
namespace {
template <int SC>
__global__ __launch_bounds__(256) void splitk_reduce_f32_kernel(const float* __restrict__ part, int S, long n4, int N,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ add, long add_ld,
                                                                float* __restrict__ out) {
  const long total = n4 * 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float acc[4];
    if constexpr (SC > 0) {
      float v[SC][4];
#pragma unroll
      for (int s = 0; s < SC; ++s) load4(part + (long)s * total + i * 4, v[s]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = v[0][j];
#pragma unroll
      for (int s = 1; s < SC; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += v[s][j];
    } else {
      load4(part + i * 4, acc);
      for (int s = 1; s < S; ++s) {
        float v[4];
        load4(part + (long)s * total + i * 4, v);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += v[j];
      }
    }
    const long m = (i * 4) / N, n = (i * 4) - m * N;
    if (bias) {
      float b[4];
      load4(bias + n, b);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += b[j];
    }
    if (add) {
      float a[4];
      load4(add + m * add_ld + n, a);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += a[j];
    }
    store4(out + i * 4, acc);
  }
}
}  // namespace

int jm_splitk_reduce_f32(const float* part, int S, int M, int N, const float* bias, const float* add, long add_ld,
                         float* out, hipStream_t st) {
  if (N % 4 || add_ld % 4) return -1;
  const long n = (long)M * N;
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
#define JM_SKF(SS) \
  case SS: splitk_reduce_f32_kernel<SS><<<(int)blocks, 256, 0, st>>>(part, S, n / 4, N, bias, add, add_ld, out); break;
  switch (S) {
    JM_SKF(2) JM_SKF(3) JM_SKF(4) JM_SKF(5) JM_SKF(6) JM_SKF(7) JM_SKF(8) JM_SKF(9) JM_SKF(10) JM_SKF(11)
    JM_SKF(12) JM_SKF(13) JM_SKF(14) JM_SKF(15) JM_SKF(16)
    default: splitk_reduce_f32_kernel<0><<<(int)blocks, 256, 0, st>>>(part, S, n / 4, N, bias, add, add_ld, out);
  }
#undef JM_SKF
  return 0;
}

int jm_splitk_reduce_bf16(const float* part, int S, long n, int N, const float* bias, uint16_t* out, hipStream_t st) {
  if (n % 8 || N % 8) return -1;
  long blocks = (n / 8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
#define JM_SKB(SS) \
  case SS: splitk_reduce_bf16_kernel<SS><<<(int)blocks, 256, 0, st>>>(part, S, n / 8, N, bias, out); break;
  switch (S) {
    JM_SKB(2) JM_SKB(3) JM_SKB(4) JM_SKB(5) JM_SKB(6) JM_SKB(7) JM_SKB(8) JM_SKB(9) JM_SKB(10) JM_SKB(11)
    JM_SKB(12) JM_SKB(13) JM_SKB(14) JM_SKB(15) JM_SKB(16)
    default: splitk_reduce_bf16_kernel<0><<<(int)blocks, 256, 0, st>>>(part, S, n / 8, N, bias, out);
  }
#undef JM_SKB
  return 0;
}

JM_DEBUG_EXPORT(elementwise)

// debug-build self test: the check fails when v != 0 (exercises the soft-assert path end to end)
namespace {
__global__ __launch_bounds__(64) void debug_selftest_kernel(int v) { JM_DASSERT(v == 0); }
}  // namespace

void jm_debug_selftest(int v, hipStream_t st) { debug_selftest_kernel<<<1, 64, 0, st>>>(v); }
