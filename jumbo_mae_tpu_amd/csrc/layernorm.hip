// LayerNorm forward / backward for gfx950 (Flax LayerNorm semantics: eps inside rsqrt, biased
// variance, scale + bias; reference modeling.py:155-156,177-179,238,282).
//
// Layout: input x is the fp32 residual stream viewed as [B, T, D] with arbitrary batch / token
// strides (so the CLS rows x[:, :3] reshaped to [B, 1, 3D] and the patch rows x[:, 3:] are read
// in place, no gather copies).  One 64-lane wave owns one row; each lane keeps V float4 of the
// row in registers (D <= 256*V), so x is read exactly once.  Output rows are contiguous [B*T, D]
// in bf16 (GEMM operand) or fp32.
//
// Backward: one wave per row for dx (two half-wave rows at D <= 512), while dgamma/dbeta (and the
// fused residual's dscale/dbias) are reduced per wave in registers over a grid-stride row loop,
// then across the block's waves through LDS in a fixed order into one partial row per block, and
// the partial rows are summed by ln_param_reduce_kernel (no float atomics: bit-reproducible).
#include <type_traits>

#include "common.h"
#include "jm_api.h"

namespace {

template <int V, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, long sB, long sT, int T,
                                                     int rows, int D, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     TO* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, uint16_t* __restrict__ y2) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int b = row / T, t = row - b * T;
  const float* xr = x + b * sB + t * sT;
  float v[V][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
      load4(xr + col, v[i]);
    } else {
      v[i][0] = v[i][1] = v[i][2] = v[i][3] = 0.f;
    }
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mean = wave_sum(s) / D;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(s2) / D + eps);
  TO* yr = y + (long)row * D;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
      float gg[4], bb[4], o[4];
      load4(gamma + col, gg);
      load4(beta + col, bb);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * gg[j] + bb[j];
      store4(yr + col, o);
      if (y2 != nullptr) store4(y2 + (long)row * D + col, o);  // bf16 copy (GEMM operand)
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Residual add fused with the LayerNorm that reads its result (the block's second LN):
//   x1[b,t] = x[b,t] + mask[b] * scale * y[b*T+t]          (written, the residual stream)
//   h[b, t-T0] = LN(x1[b,t]) for t >= T0 (bf16), with its mean / rstd
// Rows t < T0 (the Jumbo CLS tokens, normalized jointly by LN3 elsewhere) only get the add.
// Saves the LN's re-read of x1 from HBM.
struct ResLnIO {
  const float* x;
  long sB, sT;
  const uint16_t* y;  // [B*T, D] bf16
  const float* scale;
  const float* mask;
  float* x1;
  long oB, oT;
  uint16_t* h;        // [B*(T-T0), D]
  float* mean;
  float* rstd;
  DropIO drop;        // dropout of y (mask index: y's own element offset)
};

// R0 > 0: only rows t >= R0 are residual targets (y holds [B*(T-R0), D] rows); rows t < R0 of x1
// are already final and are only normalised (read from x1 itself) -- the jumbo block's CLS rows,
// whose residual is the jumbo branch's, when the NEXT block's LN1 rides on this pass.
template <int V>
__global__ __launch_bounds__(256) void res_ln_fwd_kernel(ResLnIO io, int T, int T0, int R0, int rows, int D,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float eps) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const int b = row / T, t = row - b * T;
  const bool rrow = t >= R0;  // wave-uniform
  float* x1r = io.x1 + b * io.oB + t * io.oT;
  const float* xr = rrow ? io.x + b * io.sB + t * io.sT : x1r;
  const uint16_t* yr = io.y + ((long)b * (T - R0) + (t - R0)) * D;
  const float m = io.mask ? io.mask[b] : 1.f;
  float v[V][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
      float xv[4];
      load4(xr + col, xv);
      if (rrow) {
        float yv[4], sc[4] = {1.f, 1.f, 1.f, 1.f};
        load4(yr + col, yv);
        if (io.scale) load4(io.scale + col, sc);
        if (io.drop.seed) {
          float f[4];
          drop_factors<4>(io.drop, io.drop.ioff + (yr - io.y) + col, f);
#pragma unroll
          for (int j = 0; j < 4; ++j) yv[j] *= f[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = xv[j] + m * sc[j] * yv[j];
        store4(x1r + col, v[i]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = xv[j];
      }
    } else {
      v[i][0] = v[i][1] = v[i][2] = v[i][3] = 0.f;
    }
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  if (t < T0) return;  // wave-uniform
  const float mean = wave_sum(s) / D;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(s2) / D + eps);
  const long hrow = (long)b * (T - T0) + (t - T0);
  uint16_t* hr = io.h + hrow * D;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int col = (i * 64 + lane) * 4;
    if (col < D) {
      float gg[4], bb[4], o[4];
      load4(gamma + col, gg);
      load4(beta + col, bb);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * gg[j] + bb[j];
      store4(hr + col, o);
    }
  }
  if (lane == 0) {
    io.mean[hrow] = mean;
    io.rstd[hrow] = rstd;
  }
}

// dx output and optional residual-gradient input, both [B, T, D] views with their own strides:
// dx = LN'(dy) (+ dres), i.e. the residual-stream gradient add is fused into the LN backward.
// hx / beta (optional): the forward's bf16 LN output h = bf16(gamma x-hat + beta), contiguous rows
// like dy.  x-hat is then rebuilt as (h - beta) / gamma from 2 bytes per element instead of
// re-reading the fp32 residual-stream input (4 bytes) and its (mean, rstd) -- for the columns
// where that is accurate: |beta| <= |gamma| (x-hat error <= 2^-9 (|x-hat| + |beta / gamma|), i.e.
// within 2x of bf16's own rounding of x-hat).  With any column outside that bound the launch reads
// x as before (every block sees the same gamma / beta, so every block takes the same path).
struct LnBwdIO {
  float* dx;
  long oB, oT;
  const float* dres;
  long rB, rT;
  const uint16_t* hx;
  const float* beta;
};

// a column where x-hat may be rebuilt from h: |beta| <= |gamma|, gamma not tiny
JM_DEVICE bool ln_h_ok(float g, float b) { return fabsf(g) >= 1e-20f && fabsf(b) <= fabsf(g); }

// Optional fused residual backward of the branch that FEEDS on dx (the next op of the backward
// pass): rows t >= T0 of the LN's [B, T] grid are residual targets,
//   dyr(b, t) = bf16(mask[b] * scale * dx(b, t))        at y/dy + b * yB + (t - T0) * yT,
//   dscale += colsum(mask * dx * y),  dbias += colsum(dyr)   (bias of the Dense that produced y).
// Replaces a separate residual_bwd pass that re-read dx from HBM.
struct LnResIO {
  const uint16_t* y;
  uint16_t* dy;
  long yB, yT;
  const float* scale;
  const float* mask;
  int T0;
  DropIO drop;
};

// parameter-gradient outputs (null entries skipped): dgamma, dbeta, dscale, dbias
struct ParamOuts {
  float* p[4];
};

// partial rows in ws: [dgamma | dbeta] (NP = 2) or [dgamma | dbeta | dscale | dbias] (NP = 4)
// ER (early residual-gradient load): dres is loaded together with x / dy in the first pass (one
// HBM round trip per row instead of two) while the parameter partials stay in registers.
// SC: the residual branch has a LayerScale (rio.scale); without one (every ViT-L / ViT-B preset)
// the scale registers, the branch-output loads and the dscale partials are compiled out (ViT-L
// encoder variant 200 -> 152 VGPRs: 3 waves per SIMD instead of 2).
// R rows per wave (1 or 2): at R = 2 each half-wave owns a row (the decoder's 512-wide rows: 16
// elements per lane instead of 8, two rows' loads in flight per wave, half-wave sums), and the
// halves' parameter partials are added across lanes before the block merge.
template <int V, typename TI, bool RES, bool ER = false, bool SC = true, int R = 1>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const TI* __restrict__ dy, const float* __restrict__ x,
                                                     long sB, long sT, int T, int rows, int D,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma, LnBwdIO io, LnResIO rio,
                                                     float* __restrict__ ws, int accum_params, ParamOuts outs) {
  JM_DGUARD(blockDim.x == 256 && D % 4 == 0 && D <= V * 256);
  static_assert(R == 1 || R == 2, "rows per wave");
  constexpr int NP = RES ? 4 : 2;
  constexpr int LPR = 64 / R, VL = V * R;  // lanes per row, float4 chunks per lane
  extern __shared__ __attribute__((aligned(16))) float red[];  // [NP*D]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane / LPR, l = lane % LPR;
  const bool partials = accum_params || RES;
  auto acc_add = [&](float (&acc)[NP][VL][4], int k, int i, int j, float v) { acc[k][i][j] += v; };
  // the row sum of this lane's row: the whole wave (R = 1) or its half (R = 2)
  auto row_sum = [&](float v) {
    if constexpr (R == 1) {
      return wave_sum(v);
    } else {
      v = row16_sum(v);
      const int iv = __builtin_bit_cast(int, v);
      const float lo = __builtin_bit_cast(float, __builtin_amdgcn_readlane(iv, 0)) +
                       __builtin_bit_cast(float, __builtin_amdgcn_readlane(iv, 16));
      const float hi = __builtin_bit_cast(float, __builtin_amdgcn_readlane(iv, 32)) +
                       __builtin_bit_cast(float, __builtin_amdgcn_readlane(iv, 48));
      return sub ? hi : lo;
    }
  };
  float acc[NP][VL][4], gg[VL][4], sc[VL][4];
  // h path: beta and 1 / gamma per column in LDS (after the [NP*D] merge area), read per row
  float* hbi = red + (partials ? NP * D : 0);  // [D] beta, then [D] 1 / gamma
  const bool use_h = io.hx != nullptr;
  uint32_t xchunk = 0;  // bit i: chunk i of this lane reads x (a column outside the h bound)
#pragma unroll
  for (int i = 0; i < VL; ++i) {
    const int col = (i * LPR + l) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < NP; ++k) acc[k][i][j] = 0.f;
      sc[i][j] = 1.f;
    }
    if (col < D) {
      load4(gamma + col, gg[i]);
      if constexpr (RES && SC) {
        if (rio.scale) load4(rio.scale + col, sc[i]);
      }
      if (use_h) {
        float bb[4], ig[4];
        load4(io.beta + col, bb);
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ok = ok && ln_h_ok(gg[i][j], bb[j]);
          ig[j] = 1.f / gg[i][j];
        }
        if (!ok) xchunk |= 1u << i;
        if (wave == 0 && sub == 0) {
          store4(hbi + col, bb);
          store4(hbi + D + col, ig);
        }
      }
    }
  }
  // one path per block: h when no column of the row needs x (every block sees the same gamma / beta,
  // so every block takes the same path); a per-chunk choice serialised each chunk's loads
  const bool hpath = use_h && !__syncthreads_or(xchunk != 0u);
  // the row loop, compiled once per path (a runtime branch per chunk serialised the loads)
  auto row_loop = [&](auto hp) {
    constexpr bool HP = decltype(hp)::value;
    for (int rw = blockIdx.x * 4 + wave; rw * R < rows; rw += gridDim.x * 4) {
      const int row = rw * R + sub;
      const bool valid = R == 1 || row < rows;  // R = 2: the second half of an odd tail has no row
      const int b = row / T, t = row - b * T;
      const float* xr = x + b * sB + t * sT;
      const TI* dyr = dy + (long)row * D;
      const float mu = valid ? mean[row] : 0.f, rs = valid ? rstd[row] : 0.f;
      const bool rrow = RES && t >= rio.T0;
      const long yoff = RES ? b * rio.yB + (long)(t - rio.T0) * rio.yT : 0;
      float xh[VL][4], g[VL][4], yv[VL][4];
      float rvp[ER ? VL : 1][4];
      const float* rr = io.dres ? io.dres + b * io.rB + t * io.rT : nullptr;
      float sg = 0.f, sgx = 0.f;
      // the row's x (or h) first, in one run of loads; then dy / dres with the math below
      if constexpr (HP) {
        const uint16_t* hr = io.hx + (long)row * D;
#pragma unroll
        for (int i = 0; i < VL; ++i) {
          const int col = (i * LPR + l) * 4;
          if (valid && col < D) load4(hr + col, xh[i]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < VL; ++i) {
          const int col = (i * LPR + l) * 4;
          if (valid && col < D) load4(xr + col, xh[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < VL; ++i) {
        const int col = (i * LPR + l) * 4;
        if (valid && col < D) {
          float dv[4];
          if constexpr (HP) {  // x-hat = (h - beta) / gamma
            float bb[4], ig[4];
            load4(hbi + col, bb);
            load4(hbi + D + col, ig);
#pragma unroll
            for (int j = 0; j < 4; ++j) xh[i][j] = (xh[i][j] - bb[j]) * ig[j];
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) xh[i][j] = (xh[i][j] - mu) * rs;
          }
          load4(dyr + col, dv);
          if constexpr (RES && SC) {
            if (rrow && rio.scale) load4(rio.y + yoff + col, yv[i]);
          }
          if constexpr (ER) {
            if (rr) load4(rr + col, rvp[i]);
            else rvp[i][0] = rvp[i][1] = rvp[i][2] = rvp[i][3] = 0.f;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            g[i][j] = dv[j] * gg[i][j];
            sg += g[i][j];
            sgx += g[i][j] * xh[i][j];
            acc_add(acc, 0, i, j, dv[j] * xh[i][j]);
            acc_add(acc, 1, i, j, dv[j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) xh[i][j] = g[i][j] = 0.f;
        }
      }
      sg = row_sum(sg) / D;
      sgx = row_sum(sgx) / D;
      float* dxr = io.dx + b * io.oB + t * io.oT;
      const float m = (RES && rio.mask) ? rio.mask[valid ? b : 0] : 1.f;
#pragma unroll
      for (int i = 0; i < VL; ++i) {
        const int col = (i * LPR + l) * 4;
        if (valid && col < D) {
          float o[4], rv[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (ER) {
#pragma unroll
            for (int j = 0; j < 4; ++j) rv[j] = rvp[i][j];
          } else if (rr) {
            load4(rr + col, rv);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = rs * (g[i][j] - sg - xh[i][j] * sgx) + rv[j];
          store4(dxr + col, o);
          if (RES && rrow) {
            float d[4], f[4] = {1.f, 1.f, 1.f, 1.f};
            if (rio.drop.seed) drop_factors<4>(rio.drop, rio.drop.ioff + yoff + col, f);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float md = m * o[j] * f[j];  // f: the dropout of y (d(y_pre) and dscale see it)
              d[j] = SC ? md * sc[i][j] : md;
              if constexpr (SC) {
                if (rio.scale) acc_add(acc, 2, i, j, md * yv[i][j]);
              }
              acc_add(acc, 3 % NP, i, j, bf2f(f2bf(d[j])));  // colsum of the bf16 values the GEMMs consume
            }
            store4(rio.dy + yoff + col, d);
          }
        }
      }
    }
  };
  if (hpath) row_loop(std::true_type{});
  else row_loop(std::false_type{});
  if (!partials) return;
  if constexpr (R == 2) {  // both halves hold the same columns: add them (lane l gets lane l + 32's)
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int i = 0; i < VL; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[k][i][j] += __shfl_xor(acc[k][i][j], 32, WAVE);
  }
  // merge the 4 waves' partials through LDS in turn (float4, conflict-free, no atomics), then
  // one coalesced store of the block partial row into the workspace
  for (int w = 0; w < 4; ++w) {
    if (wave == w && sub == 0) {
#pragma unroll
      for (int i = 0; i < VL; ++i) {
        const int col = (i * LPR + l) * 4;
        if (col < D) {
#pragma unroll
          for (int k = 0; k < NP; ++k) {
            float a[4] = {0.f, 0.f, 0.f, 0.f};
            if (w > 0) load4(red + k * D + col, a);
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] += acc[k][i][j];
            store4(red + k * D + col, a);
          }
        }
      }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x * 4; i < NP * D; i += 256 * 4) {
    float a[4];
    load4(red + i, a);
    store4(ws + (long)blockIdx.x * NP * D + i, a);
  }
}

// out_k[c] += sum_b ws[b][k*D + c] for the NP partial vectors (null outputs skipped).  RL row
// lanes per float4 column, each summing every RL-th partial row (4 loads in flight), then a
// fixed-order LDS tree over the lanes and ONE plain read-add-write per output column: the same
// bits on every run.  (Rounds 1-3 split the rows over grid.y slices and added the slice sums with
// float atomics, whose order varies from run to run.)
template <int RL>
__global__ __launch_bounds__(256) void ln_param_reduce_kernel(const float* __restrict__ ws, int nb, int D, int NP,
                                                              ParamOuts outs) {
  constexpr int CW = 256 / RL;
  __shared__ float4 red[256];
  const int c = threadIdx.x % CW, rl = threadIdx.x / CW;
  const int i4 = blockIdx.x * CW + c;
  const int n4 = NP * D / 4;
  const long l4 = (long)NP * D / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    const float4* p = reinterpret_cast<const float4*>(ws) + i4;
    int b = rl;
    for (; b + 3 * RL < nb; b += 4 * RL) {
      const float4 a0 = p[b * l4], a1 = p[(b + RL) * l4], a2 = p[(b + 2 * RL) * l4], a3 = p[(b + 3 * RL) * l4];
      acc.x += (a0.x + a1.x) + (a2.x + a3.x);
      acc.y += (a0.y + a1.y) + (a2.y + a3.y);
      acc.z += (a0.z + a1.z) + (a2.z + a3.z);
      acc.w += (a0.w + a1.w) + (a2.w + a3.w);
    }
    for (; b < nb; b += RL) {
      const float4 a0 = p[b * l4];
      acc.x += a0.x;
      acc.y += a0.y;
      acc.z += a0.z;
      acc.w += a0.w;
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
  if (rl == 0 && i4 < n4) {
    const float4 r = red[c];
    const float v[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // D % 4 == 0: the 4 columns share one output vector
      const int col = i4 * 4 + j;
      float* dst = outs.p[col / D];
      if (dst != nullptr) dst[col % D] += v[j];
    }
  }
}

// ln_param_reduce_kernel over nb partial rows of NP * D floats: row lanes sized to ~32 rows each
void launch_param_reduce(const float* ws, int nb, int D, int NP, ParamOuts outs, hipStream_t st) {
  int rl = 16;
  while (rl < 256 && nb > 32 * rl) rl *= 2;
  const unsigned grid = (unsigned)((NP * D / 4) * rl + 255) / 256;
  switch (rl) {
    case 16: ln_param_reduce_kernel<16><<<grid, 256, 0, st>>>(ws, nb, D, NP, outs); break;
    case 32: ln_param_reduce_kernel<32><<<grid, 256, 0, st>>>(ws, nb, D, NP, outs); break;
    case 64: ln_param_reduce_kernel<64><<<grid, 256, 0, st>>>(ws, nb, D, NP, outs); break;
    case 128: ln_param_reduce_kernel<128><<<grid, 256, 0, st>>>(ws, nb, D, NP, outs); break;
    default: ln_param_reduce_kernel<256><<<grid, 256, 0, st>>>(ws, nb, D, NP, outs); break;
  }
}

template <typename TO>
void launch_fwd(int V, dim3 grid, hipStream_t st, const float* x, long sB, long sT, int T, int rows, int D,
                const float* g, const float* b, float eps, TO* y, float* m, float* r, uint16_t* y2) {
#define JM_LNF(VV) \
  case VV: ln_fwd_kernel<VV, TO><<<grid, 256, 0, st>>>(x, sB, sT, T, rows, D, g, b, eps, y, m, r, y2); break;
  switch (V) {
    JM_LNF(1) JM_LNF(2) JM_LNF(3) JM_LNF(4) JM_LNF(6) JM_LNF(8) JM_LNF(9) JM_LNF(12) JM_LNF(16)
    default: break;
  }
#undef JM_LNF
}

// ------------------------------------------------------------------ wide rows, few of them
// The jumbo branch's LN3 normalises B rows of J = 3D (2304 / 3072) values: with one row per wave
// that is only B / 4 workgroups (128 for B = 512) and a 12-float4-per-lane chain per wave.  Here a
// whole 256-thread workgroup owns a row (VW float4 per thread, block reduction through LDS), so
// the grid has one workgroup per row.

// sum over the 256 threads of the workgroup (every thread gets it); red: >= 4 floats of LDS
JM_DEVICE float block_sum256(float v, float* red) {
  const int wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();  // red may still be read from a previous call
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

template <int VW, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_wide_kernel(const float* __restrict__ x, long sB, long sT, int T,
                                                          int rows, int D, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          TO* __restrict__ y, float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out, uint16_t* __restrict__ y2) {
  JM_DGUARD(blockDim.x == 256 && D % 4 == 0 && D <= VW * 1024);
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int b = row / T, t = row - b * T;
  const float* xr = x + b * sB + t * sT;
  float v[VW][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VW; ++i) {
    const int col = (i * 256 + threadIdx.x) * 4;
    if (col < D) {
      load4(xr + col, v[i]);
    } else {
      v[i][0] = v[i][1] = v[i][2] = v[i][3] = 0.f;
    }
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
  const float mean = block_sum256(s, red) / D;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VW; ++i) {
    const int col = (i * 256 + threadIdx.x) * 4;
    if (col < D) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        s2 += d * d;
      }
    }
  }
  const float rstd = rsqrtf(block_sum256(s2, red) / D + eps);
#pragma unroll
  for (int i = 0; i < VW; ++i) {
    const int col = (i * 256 + threadIdx.x) * 4;
    if (col < D) {
      float gg[4], bb[4], o[4];
      load4(gamma + col, gg);
      load4(beta + col, bb);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * gg[j] + bb[j];
      store4(y + (long)row * D + col, o);
      if (y2 != nullptr) store4(y2 + (long)row * D + col, o);
    }
  }
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = LN'(dy) (+ dres); per-workgroup [dgamma | dbeta] partial rows in ws (grid-stride rows)
template <int VW, typename TI>
__global__ __launch_bounds__(256) void ln_bwd_wide_kernel(const TI* __restrict__ dy, const float* __restrict__ x,
                                                          long sB, long sT, int T, int rows, int D,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma, LnBwdIO io,
                                                          float* __restrict__ ws, int accum_params) {
  JM_DGUARD(blockDim.x == 256 && D % 4 == 0 && D <= VW * 1024);
  __shared__ float red[4];
  float ag[VW][4], ab[VW][4], gg[VW][4];
#pragma unroll
  for (int i = 0; i < VW; ++i) {
    const int col = (i * 256 + threadIdx.x) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) ag[i][j] = ab[i][j] = gg[i][j] = 0.f;
    if (col < D) load4(gamma + col, gg[i]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {  // workgroup-uniform
    const int b = row / T, t = row - b * T;
    const float* xr = x + b * sB + t * sT;
    const TI* dyr = dy + (long)row * D;
    const float* rr = io.dres ? io.dres + b * io.rB + t * io.rT : nullptr;
    const float mu = mean[row], rs = rstd[row];
    float xh[VW][4], g[VW][4], rv[VW][4];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const int col = (i * 256 + threadIdx.x) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) xh[i][j] = g[i][j] = rv[i][j] = 0.f;
      if (col < D) {
        float xv[4], dv[4];
        load4(xr + col, xv);
        load4(dyr + col, dv);
        if (rr) load4(rr + col, rv[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xh[i][j] = (xv[j] - mu) * rs;
          g[i][j] = dv[j] * gg[i][j];
          sg += g[i][j];
          sgx += g[i][j] * xh[i][j];
          ag[i][j] += dv[j] * xh[i][j];
          ab[i][j] += dv[j];
        }
      }
    }
    sg = block_sum256(sg, red) / D;
    sgx = block_sum256(sgx, red) / D;
    float* dxr = io.dx + b * io.oB + t * io.oT;
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const int col = (i * 256 + threadIdx.x) * 4;
      if (col < D) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = rs * (g[i][j] - sg - xh[i][j] * sgx) + rv[i][j];
        store4(dxr + col, o);
      }
    }
  }
  if (!accum_params) return;
#pragma unroll
  for (int i = 0; i < VW; ++i) {
    const int col = (i * 256 + threadIdx.x) * 4;
    if (col < D) {
      store4(ws + (long)blockIdx.x * 2 * D + col, ag[i]);
      store4(ws + (long)blockIdx.x * 2 * D + D + col, ab[i]);
    }
  }
}

// wide-row path: D > 1024 with at most this many rows (enough workgroups, few enough partials)
constexpr int LN_WIDE_MAX_ROWS = 8192;
int pick_vw(int D) { return D <= 2048 ? 2 : D <= 3072 ? 3 : D <= 4096 ? 4 : -1; }
bool use_wide(int rows, int D) { return D > 1024 && rows <= LN_WIDE_MAX_ROWS && pick_vw(D) > 0; }

// LN backward parameter partials: per-block workspace rows + ln_param_reduce_kernel.  Measured
// and removed: float atomics from each block straight into the outputs (the same step time, ViT-L
// 94.05 vs 93.90 ms -- 512 adders per address cost what the reduce launch did;
// profiles/r2_ln_param_reduce.txt), and folding the rows in the kernel by the last block of each
// group of 8 (2.7 ms/step slower, r3e_summary_vitl_b512_fused_reductions.txt)

// the residual-gradient input is loaded with x / dy (ER) where the registers allow it (V <= 4:
// 97.96 -> 97.75 ms/step, profiles/r1_ab_ln_bwd_early_dres.txt).  Measured and removed: LDS-
// accumulated parameter partials (r1_ab_ln_bwd_lds_acc.txt), a next-row prefetch variant
// (r2_ln_bwd_prefetch.txt).
// rows per wave of the row-loop backward: two half-wave rows at V = 2 (D <= 512, the decoder)
#define LN_BWD_R(VV) ((VV) == 2 ? 2 : 1)
template <typename TI, bool RES, bool SC = true>
void launch_bwd(int V, dim3 grid, size_t smem, hipStream_t st, const TI* dy, const float* x, long sB, long sT,
                int T, int rows, int D, const float* m, const float* r, const float* g, LnBwdIO dx, LnResIO rio,
                float* ws, int acc, ParamOuts outs) {
#define JM_LNB(VV)                                                                                          \
  case VV:                                                                                                  \
    ln_bwd_kernel<VV, TI, RES, (VV >= 2 && VV <= 4), SC, LN_BWD_R(VV)><<<grid, 256, smem, st>>>(             \
        dy, x, sB, sT, T, rows, D, m, r, g, dx, rio, ws, acc, outs);                                         \
    break;
  switch (V) {
    JM_LNB(1) JM_LNB(2) JM_LNB(3) JM_LNB(4) JM_LNB(6) JM_LNB(8) JM_LNB(9) JM_LNB(12) JM_LNB(16)
    default: break;
  }
#undef JM_LNB
}

int pick_v(int D) {
  const int need = (D + 255) / 256;
  const int opts[] = {1, 2, 3, 4, 6, 8, 9, 12, 16};
  for (int o : opts)
    if (o >= need) return o;
  return -1;
}

}  // namespace

// ------------------------------------------------------------------------- host entry points
int jm_layernorm_fwd(const float* x, long sB, long sT, int B, int T, int D, const float* gamma,
                     const float* beta, float eps, void* y, int out_bf16, float* mean, float* rstd,
                     hipStream_t st, uint16_t* y2) {
  const int V = pick_v(D);
  if (V < 0 || (D % 4) != 0) return -1;
  const int rows = B * T;
  if (use_wide(rows, D)) {
    const int VW = pick_vw(D);
#define JM_LNFW(VV, TO, YP, Y2)                                                                                    \
  case VV:                                                                                                         \
    ln_fwd_wide_kernel<VV, TO><<<rows, 256, 0, st>>>(x, sB, sT, T, rows, D, gamma, beta, eps, YP, mean, rstd, Y2); \
    break;
    if (out_bf16) {
      switch (VW) { JM_LNFW(2, uint16_t, (uint16_t*)y, nullptr) JM_LNFW(3, uint16_t, (uint16_t*)y, nullptr)
                    JM_LNFW(4, uint16_t, (uint16_t*)y, nullptr) default: return -1; }
    } else {
      switch (VW) { JM_LNFW(2, float, (float*)y, y2) JM_LNFW(3, float, (float*)y, y2) JM_LNFW(4, float, (float*)y, y2)
                    default: return -1; }
    }
#undef JM_LNFW
    return 0;
  }
  dim3 grid((rows + 3) / 4);
  if (out_bf16)
    launch_fwd<uint16_t>(V, grid, st, x, sB, sT, T, rows, D, gamma, beta, eps, (uint16_t*)y, mean, rstd, nullptr);
  else
    launch_fwd<float>(V, grid, st, x, sB, sT, T, rows, D, gamma, beta, eps, (float*)y, mean, rstd, y2);
  return 0;
}

int jm_residual_ln_fwd(const float* x, long sB, long sT, const uint16_t* y, const float* scale, const float* mask,
                       float* x1, long oB, long oT, uint16_t* h, float* mean, float* rstd, int B, int T, int T0,
                       int D, const float* gamma, const float* beta, float eps, hipStream_t st, int R0,
                       JmDrop drop) {
  const ResLnIO io{x, sB, sT, y, scale, mask, x1, oB, oT, h, mean, rstd, drop};
  if (R0 < 0 || R0 >= T) return -2;
  const int V = pick_v(D);
  if (V < 0 || (D % 4) != 0) return -1;
  const int rows = B * T;
  dim3 grid((rows + 3) / 4);
#define JM_RLN(VV) \
  case VV: res_ln_fwd_kernel<VV><<<grid, 256, 0, st>>>(io, T, T0, R0, rows, D, gamma, beta, eps); break;
  switch (V) {
    JM_RLN(1) JM_RLN(2) JM_RLN(3) JM_RLN(4) JM_RLN(6) JM_RLN(8) JM_RLN(9) JM_RLN(12) JM_RLN(16)
    default: return -1;
  }
#undef JM_RLN
  return 0;
}

// most row-loop blocks of the (non-wide) LN backward: one resident round of the fused-residual
// kernel without LayerScale -- 3 blocks per CU at V = 4 (147 VGPRs, D = 1024) and at V = 2 with
// two rows per wave (148, D = 512), 4 at V = 1, 2 beyond.  A second round only adds partial rows
// (r2: 1024 blocks at 2 per CU lost 0.3 ms/step to 512, r2_ln_bwd_blocks.txt).
constexpr int LN_BWD_CUS = 256;
int ln_bwd_blocks_per_cu(int V) { return V <= 1 ? 4 : V <= 4 ? 3 : 2; }

int jm_layernorm_bwd_blocks(int rows, int D) {
  // wide rows: one workgroup per row (at most 1024 workgroups, grid-stride beyond)
  if (use_wide(rows, D)) return rows > 1024 ? 1024 : rows;
  // grid-stride over rows, 4 waves per block; each block writes one [NP*D] partial (no atomics in
  // the hot kernel)
  const int V = pick_v(D), cap = LN_BWD_CUS * ln_bwd_blocks_per_cu(V < 0 ? 16 : V);
  const int rpb = 4 * LN_BWD_R(V);  // rows per block and loop step
  int nb = (rows + rpb - 1) / rpb;
  return nb > cap ? cap : nb;
}

int jm_layernorm_bwd(const void* dy, int dy_bf16, const float* x, long sB, long sT, int B, int T, int D,
                     const float* mean, const float* rstd, const float* gamma, float* dx_ptr, long oB, long oT,
                     const float* dres, long rB, long rT, float* dgamma, float* dbeta, int accum_params, float* ws,
                     const JmLnRes* res, hipStream_t st, const uint16_t* hx, const float* beta) {
  if (hx != nullptr && beta == nullptr) return -3;
  const LnBwdIO dx{dx_ptr, oB, oT, dres, rB, rT, hx, beta};
  const int V = pick_v(D);
  if (V < 0 || (D % 4) != 0) return -1;
  const int rows = B * T;
  const int nb = jm_layernorm_bwd_blocks(rows, D);
  dim3 grid(nb);
  const int NP = res ? 4 : 2;
  const bool partials = accum_params || res;
  if (!res && use_wide(rows, D)) {
    const int VW = pick_vw(D);
#define JM_LNBW(VV, TI)                                                                                     \
  case VV:                                                                                                  \
    ln_bwd_wide_kernel<VV, TI><<<nb, 256, 0, st>>>((const TI*)dy, x, sB, sT, T, rows, D, mean, rstd, gamma, \
                                                   dx, ws, accum_params);                                   \
    break;
    if (dy_bf16) {
      switch (VW) { JM_LNBW(2, uint16_t) JM_LNBW(3, uint16_t) JM_LNBW(4, uint16_t) default: return -1; }
    } else {
      switch (VW) { JM_LNBW(2, float) JM_LNBW(3, float) JM_LNBW(4, float) default: return -1; }
    }
#undef JM_LNBW
    if (accum_params) {
      ParamOuts outs{{dgamma, dbeta, nullptr, nullptr}};
      launch_param_reduce(ws, nb, D, 2, outs, st);
    }
    return 0;
  }
  const size_t smem = ((partials ? NP * D : 0) + (hx ? 2 * D : 0)) * sizeof(float);
  const ParamOuts outs{{accum_params ? dgamma : nullptr, accum_params ? dbeta : nullptr,
                        res ? res->dscale : nullptr, res ? res->dbias : nullptr}};
  float* wsk = ws;
  LnResIO rio{nullptr, nullptr, 0, 0, nullptr, nullptr, 0, JmDrop{nullptr, 0u, 1.f, 0}};
  if (res) rio = LnResIO{res->y, res->dy, res->yB, res->yT, res->scale, res->mask, res->T0, res->drop};
  if (dy_bf16) {
    if (res && res->scale)
      launch_bwd<uint16_t, true>(V, grid, smem, st, (const uint16_t*)dy, x, sB, sT, T, rows, D, mean, rstd, gamma,
                                 dx, rio, wsk, accum_params, outs);
    else if (res)
      launch_bwd<uint16_t, true, false>(V, grid, smem, st, (const uint16_t*)dy, x, sB, sT, T, rows, D, mean, rstd,
                                        gamma, dx, rio, wsk, accum_params, outs);
    else
      launch_bwd<uint16_t, false>(V, grid, smem, st, (const uint16_t*)dy, x, sB, sT, T, rows, D, mean, rstd, gamma,
                                  dx, rio, wsk, accum_params, outs);
  } else {
    if (res && res->scale)
      launch_bwd<float, true>(V, grid, smem, st, (const float*)dy, x, sB, sT, T, rows, D, mean, rstd, gamma, dx, rio,
                              wsk, accum_params, outs);
    else if (res)
      launch_bwd<float, true, false>(V, grid, smem, st, (const float*)dy, x, sB, sT, T, rows, D, mean, rstd, gamma,
                                     dx, rio, wsk, accum_params, outs);
    else
      launch_bwd<float, false>(V, grid, smem, st, (const float*)dy, x, sB, sT, T, rows, D, mean, rstd, gamma, dx, rio,
                               wsk, accum_params, outs);
  }
  if (partials)
    launch_param_reduce(ws, nb, D, NP, outs, st);
  return 0;
}

JM_DEBUG_EXPORT(layernorm)
