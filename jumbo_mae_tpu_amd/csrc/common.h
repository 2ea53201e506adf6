// Shared device helpers for the jumbo_mae_tpu_amd CDNA4 (gfx950) kernels.
// Wave size is 64 on CDNA: every reduction below is a 64-lane butterfly.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "jm_api.h"

#define JM_DEVICE __device__ __forceinline__

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef uint16_t bf16_raw;

constexpr int WAVE = 64;

JM_DEVICE float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Dropout keep decisions, shared by every dropout site (dropout.hip, the attention kernels, the
// GELU and residual kernels) and mirrored bit for bit by ops/dropout.py keep_mask.  Element idx
// takes bits [16 * (idx & 1), +16) of ONE 32-bit hash per pair j = idx >> 1 (lowbias32 finalizer
// of j + seed; j taken mod 2^32) and is kept iff they are below thr = round(keep * 65536).
JM_DEVICE uint32_t drop_hash(uint32_t j, uint64_t seed) {
  uint32_t x = (j + (uint32_t)seed) ^ (uint32_t)(seed >> 32);
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
JM_DEVICE bool drop_keep_half(uint32_t h, int odd, uint32_t thr) { return (odd ? (h >> 16) : (h & 0xffffu)) < thr; }
JM_DEVICE bool drop_keep(uint64_t seed, uint64_t idx, uint32_t thr) {
  return drop_keep_half(drop_hash((uint32_t)(idx >> 1), seed), (int)(idx & 1), thr);
}

// Dense-output dropout applied where the branch output is consumed (the residual kernels): the
// element at y + o (o = y's own element offset) has mask index ioff + o in the branch tensor.
using DropIO = JmDrop;  // seed null: no dropout; scale = 1 / keep
// f[j] = keep(idx + j) / keep for W consecutive elements (idx even, W even)
template <int W>
JM_DEVICE void drop_factors(const DropIO& d, long idx, float* f) {
  const uint64_t seed = (uint64_t)d.seed[0];
#pragma unroll
  for (int j = 0; j < W; j += 2) {
    const uint32_t h = drop_hash((uint32_t)((idx + j) >> 1), seed);
    f[j] = drop_keep_half(h, 0, d.thr) ? d.scale : 0.f;
    f[j + 1] = drop_keep_half(h, 1, d.thr) ? d.scale : 0.f;
  }
}

JM_DEVICE uint16_t f2bf(float f) {
  // round-to-nearest-even; hipcc lowers the builtin conversion to v_cvt_pk_bf16_f32 on gfx950,
  // which keeps NaNs NaN (MI355X_MICROARCH.md "Correctness boundaries").
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// two floats -> one dword of two bf16 (a low): built as a 2-vector so that it lowers to ONE
// v_cvt_pk_bf16_f32 (the shift-or form became two single-operand conversions + lshl + or)
JM_DEVICE uint32_t pack_bf2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) short s16x2_t;
  s16x2_t s;
  s[0] = (short)f2bf(a);
  s[1] = (short)f2bf(b);
  return __builtin_bit_cast(uint32_t, s);
}

template <typename T> JM_DEVICE float to_f(T v);
template <> JM_DEVICE float to_f<float>(float v) { return v; }
template <> JM_DEVICE float to_f<uint16_t>(uint16_t v) { return bf2f(v); }

template <typename T> JM_DEVICE T from_f(float v);
template <> JM_DEVICE float from_f<float>(float v) { return v; }
template <> JM_DEVICE uint16_t from_f<uint16_t>(float v) { return f2bf(v); }

// tanh through one v_exp_f32 + one reciprocal (libm tanhf is a long software sequence);
// saturates correctly at +-inf, absolute error ~1e-7
JM_DEVICE float jm_tanh(float u) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u)); }

// flax nn.gelu(approximate=True): 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))).  With
// p = 0.5 (1 + tanh u) = sigmoid(2u) = 1 / (1 + exp(-2u)) this is x * p -- one v_exp_f32 and one
// reciprocal -- and the derivative is p + x p (1 - p) 2c (1 + 3a x^2); both saturate cleanly
// (exp -> inf gives p = 0, exp -> 0 gives p = 1).
JM_DEVICE float gelu_p_f(float x) {
  const float m2u = x * (-1.5957691216057308f - 0.07135481627260025f * x * x);  // -2u
  return __builtin_amdgcn_rcpf(1.f + __expf(m2u));
}

JM_DEVICE float gelu_tanh_f(float x) { return x * gelu_p_f(x); }

// d/dx of gelu_tanh_f
JM_DEVICE float gelu_grad_f(float x) {
  const float p = gelu_p_f(x);
  return __builtin_fmaf(x * p * (1.f - p), __builtin_fmaf(0.21406444881780076f, x * x, 1.5957691216057308f), p);
}

// gelu_tanh_f and its derivative sharing one exp / reciprocal (the forward epilogue that saves
// gelu' for the backward instead of the pre-activation)
JM_DEVICE void gelu_and_grad_f(float x, float& g, float& d) {
  const float p = gelu_p_f(x);
  g = x * p;
  d = __builtin_fmaf(g * (1.f - p), __builtin_fmaf(0.21406444881780076f, x * x, 1.5957691216057308f), p);
}

// The same on element pairs as 2-vectors: mul / add / fma lower to v_pk_*_f32 (2 elements per
// 4-cycle issue; for epilogue phases, not beside MFMAs -- MI355X_MICROARCH.md prices packed f32
// there as an anti-lever), log2(e) folded into the polynomial (one v_exp_f32, no pre-multiply),
// x^2 shared by p and the derivative.  Per element pair: 9 packed ops + 4 transcendentals.
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
constexpr float GELU_C1 = -1.5957691216057308f * 1.4426950408889634f;   // -2 sqrt(2/pi) log2(e)
constexpr float GELU_C2 = -0.07135481627260025f * 1.4426950408889634f;  // -2 sqrt(2/pi) 0.044715 log2(e)

JM_DEVICE f32x2_t gelu_p2(f32x2_t x, f32x2_t x2) {
  const f32x2_t m = x * (x2 * GELU_C2 + GELU_C1);  // -2u log2(e)
  f32x2_t e = {__builtin_amdgcn_exp2f(m.x), __builtin_amdgcn_exp2f(m.y)};
  e = e + 1.f;
  return f32x2_t{__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}

// n (even) elements: g = gelu(x) and/or d = gelu'(x) (null pointers skipped at compile time)
template <int NE, bool G, bool D>
JM_DEVICE void gelu_n(const float* x, float* g, float* d) {
#pragma unroll
  for (int j = 0; j < NE; j += 2) {
    const f32x2_t xv = {x[j], x[j + 1]};
    const f32x2_t x2 = xv * xv;
    const f32x2_t p = gelu_p2(xv, x2);
    const f32x2_t gv = xv * p;
    if (G) {
      g[j] = gv.x;
      g[j + 1] = gv.y;
    }
    if (D) {
      const f32x2_t dv = (gv * (1.f - p)) * (x2 * 0.21406444881780076f + 1.5957691216057308f) + p;
      d[j] = dv.x;
      d[j + 1] = dv.y;
    }
  }
}

// gelu'(h) of the tanh GELU lies in [-0.1701, 1.1290].  The FF1 forward saves it for the FF2 data
// gradient as an 8-bit code q = round(GD_Q gelu') + GD_Z -- step 1 / 195 = 0.0051, |error| <= 0.0026
// (bf16 rounds values near 1 by up to 0.002), 0 and 1 exact (codes 34 and 229), codes 1..254 used --
// half the bytes of a bf16 copy on both sides of the round trip (ops/prims.py GD_Q / GD_Z mirror).
constexpr float GD_Q = 195.f;
constexpr int GD_Z = 34;
// v_cvt_pk_u8_f32 rounds to nearest even and saturates to [0, 255] (probed on gfx950:
// tools/probes/cvt_pk_u8_probe.hip) and writes its byte into a word: one instruction per code
// instead of the clamp / truncating convert / shift / or sequence -- the FF1 forward epilogue is
// VALU-issue bound (profiles/r6h_gelu_code_cvt.txt).  Ties round to even (the torch mirror
// gd_encode rounds them up: codes may differ by one at exact ties).
JM_DEVICE uint32_t gd_code(float d) { return __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fmaf(d, GD_Q, (float)GD_Z), 0, 0u); }
template <int B>
JM_DEVICE uint32_t gd_put(float d, uint32_t w) { return __builtin_amdgcn_cvt_pk_u8_f32(__builtin_fmaf(d, GD_Q, (float)GD_Z), B, w); }
// 8 derivatives -> 8 codes, 4 per 32-bit word, element 0 in the low byte
JM_DEVICE uint2 gd_pack8(const float* d) {
  uint2 v;
  v.x = gd_put<3>(d[3], gd_put<2>(d[2], gd_put<1>(d[1], gd_put<0>(d[0], 0u))));
  v.y = gd_put<3>(d[7], gd_put<2>(d[6], gd_put<1>(d[5], gd_put<0>(d[4], 0u))));
  return v;
}
// codes -> (q - GD_Z) * s: v_cvt_f32_ubyte0..3, an exact subtraction, one multiply -- code GD_Z
// (dropped elements, gelu' underflow) decodes to exactly 0, which an fma with -GD_Z s would not
JM_DEVICE void gd_unpack4(uint32_t w, float s, float* d) {
  d[0] = ((float)(w & 255u) - (float)GD_Z) * s;
  d[1] = ((float)((w >> 8) & 255u) - (float)GD_Z) * s;
  d[2] = ((float)((w >> 16) & 255u) - (float)GD_Z) * s;
  d[3] = ((float)(w >> 24) - (float)GD_Z) * s;
}

// DPP lane moves (VALU, no LDS round trip like __shfl_xor's ds_bpermute)
template <int CTRL>
JM_DEVICE float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}

template <int CTRL>
JM_DEVICE uint32_t dpp_mov_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}

// sum over the 16 lanes of each DPP row; every lane of the row gets the result.
// Requires the whole row active.
JM_DEVICE float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// full-wave sum (wave-uniform result); requires all 64 lanes active
JM_DEVICE float wave_sum(float v) {
  v = row16_sum(v);
  const int i = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 48)));
}

JM_DEVICE float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, WAVE));
  return v;
}

// 8 x bf16 <-> 8 x float through one 16-byte access
struct bf16x8_u {
  union {
    uint4 u;
    uint16_t h[8];
  };
};

JM_DEVICE void load8(const uint16_t* p, float* f) {
  bf16x8_u v;
  v.u = *reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf2f(v.h[i]);
}

JM_DEVICE void store8(uint16_t* p, const float* f) {
  bf16x8_u v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v.h[i] = f2bf(f[i]);
  *reinterpret_cast<uint4*>(p) = v.u;
}

JM_DEVICE void load8(const float* p, float* f) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

JM_DEVICE void store8(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}

JM_DEVICE void load4(const float* p, float* f) {
  float4 a = *reinterpret_cast<const float4*>(p);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
}
JM_DEVICE void store4(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
}
JM_DEVICE void load4(const uint16_t* p, float* f) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
}
JM_DEVICE void store4(uint16_t* p, const float* f) {
  uint2 v;
  v.x = pack_bf2(f[0], f[1]);
  v.y = pack_bf2(f[2], f[3]);
  *reinterpret_cast<uint2*>(p) = v;
}

// ------------------------------------------------------------------ debug build
// build.py --debug compiles every kernel with -DJM_DEBUG into _C_debug.so.  Device checks there are
// SOFT: a failing check records its source line in a per-translation-unit device word (first
// failure wins) instead of trapping -- a trapping wave can take the whole GPU down -- and the host
// reads and clears the words through debug_lines().  JM_DGUARD additionally returns from the kernel;
// use it only at kernel entry on workgroup-uniform launch invariants (before any barrier), where a
// violated assumption would otherwise turn into out-of-bounds accesses.
#ifdef JM_DEBUG
static __device__ int jm_dbg_line;
JM_DEVICE void jm_dbg_fail(int line) { atomicCAS(&jm_dbg_line, 0, line); }
#define JM_DASSERT(c)                     \
  do {                                    \
    if (!(c)) jm_dbg_fail(__LINE__);      \
  } while (0)
#define JM_DGUARD(c)                      \
  do {                                    \
    if (!(c)) {                           \
      jm_dbg_fail(__LINE__);              \
      return;                             \
    }                                     \
  } while (0)
#define JM_DEBUG_EXPORT(tu)                                                         \
  int jm_debug_line_##tu() {                                                        \
    int v = 0, z = 0;                                                               \
    (void)hipDeviceSynchronize();                                                   \
    (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(jm_dbg_line), sizeof(int));            \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(jm_dbg_line), &z, sizeof(int));              \
    return v;                                                                       \
  }
#else
#define JM_DASSERT(c) \
  do {                \
  } while (0)
#define JM_DGUARD(c) \
  do {               \
  } while (0)
#define JM_DEBUG_EXPORT(tu) \
  int jm_debug_line_##tu() { return 0; }
#endif

#define JM_CHECK(x)                                                                  \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
    }                                                                                \
  } while (0)
