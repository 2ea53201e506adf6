// Host-side argument structs shared by the kernel translation units and bindings.cpp.
#pragma once
#include <cstdint>

// Dense-output dropout applied by the residual kernels that consume the branch output y (ops/blocks.py
// Drops): the element at y + o (y's own element offset o) is kept with common.h drop_keep(seed, ioff + o),
// kept values scaled by 1 / keep.  seed null: no dropout.
struct JmDrop {
  const int64_t* seed;
  uint32_t thr;
  float scale;
  long ioff;
};

// Fused residual backward riding on the LayerNorm backward (layernorm.hip, LnResIO):
// for rows t >= T0, dy(b, t) = bf16(mask[b] * scale * dx(b, t)) at y/dy + b * yB + (t - T0) * yT,
// dscale += colsum(mask * dx * y), dbias += colsum(dy).  scale / mask / dscale / dbias may be null.
struct JmLnRes {
  const uint16_t* y;
  uint16_t* dy;
  long yB, yT;
  const float* scale;
  const float* mask;
  int T0;
  float* dscale;
  float* dbias;
  JmDrop drop;  // y's dropout (dy and dscale use the masked y)
};

// Grouped weight-gradient launch (gemm_tn.hip jm_gemm_tn_group): n <= 4 independent TN problems
// G_p[N_p][K_p] (+)= A_p[M][N_p]^T . B_p[M][K_p] over the SAME M rows in one grid; tile0 = prefix
// sums of the problems' 256 x 256 output tiles; out[p] = G_p (one split) or its [S][N_p K_p]
// fp32 partial slices.
struct TnGroup {
  const uint16_t* a[4];
  const uint16_t* b[4];
  long lda[4], ldb[4];
  int N[4], K[4];
  float* out[4];
  int tile0[5];
  int n;
};

// Epilogue / output description of an NT GEMM launch (gemm.hip, bindings.cpp).
struct GemmEpi {
  const float* bias;     // [N] fp32 or null
  uint16_t* out;         // bf16 [M, ldo] (EPI_GELU_D: unused, see dq)
  long ldo;
  uint16_t* out2;        // EPI_GELU: gelu(out) bf16 [M, ldo]
  const uint16_t* aux;   // EPI_DGELU: pre-activation h bf16 [M, ldo]
  float* colpart;        // EPI_DGELU: per-row-tile column sums of out, [ceil(M/256) (+ 8 * tail tiles)][N] fp32
  float* part;           // EPI_PARTIAL: [splits][M][N] fp32 split-K partial products
  int splits;            // K splits (1 = none)
  // tail split (jm_gemm_nt_tail_plan): the last, partly filled wave of output tiles is computed
  // split-K into the compact workspace tail[tail_S][tail_r][256][256] and finished by a reduce
  // kernel that applies the epilogue; t_begin / t_count restrict a launch to a tile range.
  float* tail;
  int tail_S;
  int t_begin;
  int t_count;
  // EPI_GELU_D: FF hidden dropout (ops/blocks.py Drops) -- gelu(h) times keep(seed, m * ldo + n) / keep
  // (common.h drop_keep), gelu'(h) times the keep bit alone (its 1 / keep travels as dqs); dseed null: none
  const int64_t* dseed;
  uint32_t dthr;
  float dscale;
  // gelu'(h) as 8-bit codes (common.h gd_code): EPI_GELU_D writes dq [M, ldo] u8, EPI_DMUL reads dqa and
  // decodes code q as (q - GD_Z) * dqs (dqs = keep scale / GD_Q)
  uint8_t* dq;
  const uint8_t* dqa;
  float dqs;
};
