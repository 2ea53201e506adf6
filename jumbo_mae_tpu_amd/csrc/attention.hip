// Fused short-sequence multi-head attention, forward + backward, for gfx950 MFMA.
//
// Shapes of this workload: encoder S=52 (3 CLS + 49 kept patches), hd=64;
// MAE decoder S=199, hd=32; finetune S=199, hd=64.  The whole sequence of one (batch, head)
// fits in LDS, so one 256-thread workgroup (4 waves) owns one (b, h): no online softmax, no
// S x S matrix in HBM, one pass over q/k/v.
//
// MFMA: v_mfma_f32_16x16x32_bf16 (fp32 accumulate).  Orientation ("key on the lane"):
//   forward   S^T = K Q^T  -> the C tile holds one query per lane column and 4 keys per lane
//             group, so the softmax column reduction is in-register + 2 cross-lane shuffles and
//             P^T is *already* the B operand of O^T = V^T P^T (k-permuted; V^T is read with the
//             same permutation) -- no LDS round trip for P.
//   backward  S = Q K^T and dP = dO V^T with the key on the lane; their C tiles are directly the
//             B operands of dV^T += dO^T P and dK^T += Q^T dS.  dS crosses LDS once (per 64-query
//             chunk) for dQ^T = K^T dS^T.  Each wave keeps dK^T/dV^T of its key tiles in
//             registers across the whole query sweep: no atomics, deterministic.
//
// Sequence is padded to SP (multiple of 32) inside LDS; padded keys get P = 0, padded queries
// get lse = +inf (P = 0) and zero dO, so they contribute nothing.
//
// Memory layout: qkv [B, S, 3, H, hd] (output of the fused QKV GEMM, read in place),
// o / do [B, S, H, hd], lse [B, H, S] (natural log), dqkv [B, S, 3, H, hd].
#include "common.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

JM_DEVICE bf16x8_t pack8(const float* f) {
  s16x8_t s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = (short)f2bf(f[j]);
  return __builtin_bit_cast(bf16x8_t, s);
}

JM_DEVICE bf16x8_t cat44(s16x4_t lo, s16x4_t hi) {
  s16x8_t s;
  s[0] = lo[0]; s[1] = lo[1]; s[2] = lo[2]; s[3] = lo[3];
  s[4] = hi[0]; s[5] = hi[1]; s[6] = hi[2]; s[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, s);
}

JM_DEVICE bf16x8_t ld8(const uint16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }
// Range-checked loads: a buffer resource over [base, base + bytes) returns zeros past its end, so
// the rows of padded queries / keys need no branch around their loads (a branch leaves each loaded
// value behind a phi copy whose wait splits the load burst into several round trips)
JM_DEVICE __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
JM_DEVICE uint4 bld16(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
JM_DEVICE s16x4_t ld4(const uint16_t* p) { return *reinterpret_cast<const s16x4_t*>(p); }

// ds_read_b64_tr_b16 (gfx950): per 16-lane group, lane 4q+p supplies the address of row q,
// columns 4p..4p+3 of a 4 x 16 block of 16-bit elements; lane i receives column i of the 4 rows.
// Lets row-major LDS images serve as transposed MFMA operands (no second, transposed copy).
JM_DEVICE s16x4_t tr4(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(p));
}

// 8 bf16 values (one 16-byte chunk) times f, rounded back to bf16
JM_DEVICE uint4 scale_bf16x8(uint4 v, float f) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = pack_bf2(__uint_as_float(w[j] << 16) * f, __uint_as_float(w[j] & 0xffff0000u) * f);
  return v;
}

JM_DEVICE f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Workgroup -> (b, h) order: the dispatcher deals consecutive workgroups round-robin over the 8
// XCDs, so heads h and h + 1 of one token row -- the two halves of a 128-B line at hd = 32 --
// would be read (and written) through two different L2s.  With remap the grid is relabelled
// bijectively so that consecutive (b, h) share an XCD (the GEMM tile remap); placement only
// changes speed, never results (dec fwd 175 -> 163 us, bwd 361 -> 340 us with the forward's
// batched staging below; profiles/r2_attn_remap.txt).
JM_DEVICE int xcd_bid() {
  const int orig = blockIdx.x, nwg = gridDim.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// XOR swizzle of 16-byte chunks shared by every whole-sequence kernel's LDS images (the backward's
// comment below has the details)
JM_DEVICE int aswz(int row) {
  return ((row >> 2) & 1) | ((((row >> 2) ^ (row >> 3)) & 1) << 1) | (((row >> 1) & 1) << 2);
}

// element offset of (row, col) in a swizzled image of NCH 16-byte chunks per row
template <int NCH>
JM_DEVICE int swo(int row, int col) {
  return row * (NCH * 8) + ((((col >> 3) ^ aswz(row)) & (NCH - 1)) << 3) + (col & 7);
}

// ---------------------------------------------------------------- forward softmax (fast form)
// The forward is VALU-bound (PMC: ~80 % of SIMD cycles in VALU at S = 199, hd = 32, ~10 VALU
// instructions per score), so per score it now issues only an fma (scale and max subtraction in
// one), the exp2, half a max3 and half a bf16 pack:
//  * padded keys are masked through the QK^T accumulator init (-1e30 for keys >= S, only in the
//    key tiles that straddle S) instead of a compare + select per score;
//  * the max is taken over raw scores and the scale folded into the exp2 argument;
//  * the row sum comes out of the MFMA: an all-ones A operand next to V^T sums the same bf16 P
//    the P.V product uses (7 extra MFMAs per query tile instead of one add per score);
//  * query tiles past S (fully padded) are skipped.
JM_DEVICE f32x4_t key_init(int kt, int g, int S) {
  f32x4_t a = {0.f, 0.f, 0.f, 0.f};
  if (kt * 16 + 16 > S) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = kt * 16 + 4 * g + i < S ? 0.f : -1e30f;
  }
  return a;
}

JM_DEVICE bf16x8_t bf16_ones() {
  s16x8_t s;
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = (short)0x3F80;
  return __builtin_bit_cast(bf16x8_t, s);
}

// sc: raw S^T tiles (key on the lane group) of one query tile, NTv of them real; va(s, dt): the
// V^T A operand of key pair s, d tile dt.  Returns O^T (unnormalised), ms = scaled row max (log2
// domain) and l = row sum of the bf16 P.
// Attention-probability dropout (reference modeling.py:133): keep bit of P[b, h, q, k] from
// common.h drop_keep at index ((b * H + h) * S + k) * SE + q, SE = S rounded up to even, so that
// queries 2m, 2m + 1 of a key share one hash: the backward's lanes hold 4 consecutive queries of
// one key (2 hashes per 4 scores), the forward's 4 keys of one query (2 hashes, the other 2 from
// the partner query's lane).  ops/dropout.py
// keep_mask_rows mirrors it.  The row statistics (lse, row sum) are those of the undropped P; the
// forward scales O by 1 / keep, the backward folds the mask into dP and P^T dO.
struct AttnDrop {
  const int64_t* seed;  // int64 [1] on the device; null: no dropout
  uint32_t thr;         // round(keep * 65536)
  float scale;          // 1 / keep
};

// DROP: P.V uses the masked P (keys of pair s: 32 s + 4 g + i, 32 s + 16 + 4 g + i; hash index
// jq + key * seh, half qodd); the row sum l stays the undropped one.  Every lane of the wave must be
// active (the partner-lane DPP exchange).
template <int NT, int DT, bool DROP = false, class VA>
JM_DEVICE void softmax_pv(const f32x4_t (&sc)[NT], float sl2, VA&& va, f32x4_t (&oacc)[DT], float& ms, float& l,
                          uint64_t dseed = 0, uint32_t dthr = 0, uint32_t jq = 0, uint32_t seh = 0, int qodd = 0,
                          int g = 0) {
  float m = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < NT; ++kt) {  // two v_max3 per tile
    m = fmaxf(fmaxf(m, sc[kt][0]), sc[kt][1]);
    m = fmaxf(fmaxf(m, sc[kt][2]), sc[kt][3]);
  }
  m = fmaxf(m, __shfl_xor(m, 16, WAVE));
  m = fmaxf(m, __shfl_xor(m, 32, WAVE));
  ms = m * sl2;
  const bf16x8_t ones = bf16_ones();
  f32x4_t lacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) oacc[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NT / 2; ++s) {
    float pf[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pf[i] = __builtin_amdgcn_exp2f(fmaf(sc[2 * s][i], sl2, -ms));
      pf[4 + i] = __builtin_amdgcn_exp2f(fmaf(sc[2 * s + 1][i], sl2, -ms));
    }
    const bf16x8_t pb = pack8(pf);
    lacc = mfma(ones, pb, lacc);
    if constexpr (DROP) {
      // queries q and q ^ 1 (lanes l16, l16 ^ 1 of one lane group) share each key's hash (the pair
      // convention): a lane hashes two of its four keys per tile -- the pair half 2 qodd, 2 qodd + 1
      // -- and takes the other two from its partner (DPP quad_perm [1,0,3,2], every lane active
      // here): 4 hashes per 8 scores instead of 8
      uint32_t hm[4], hp[4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        hm[u] = drop_hash(jq + (uint32_t)(32 * s + 4 * g + 2 * qodd + u) * seh, dseed);
        hm[2 + u] = drop_hash(jq + (uint32_t)(32 * s + 16 + 4 * g + 2 * qodd + u) * seh, dseed);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) hp[u] = dpp_mov_u32<0xB1>(hm[u]);
      bool k0[4], k1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool own = (i >> 1) == qodd;
        k0[i] = drop_keep_half(own ? hm[i & 1] : hp[i & 1], qodd, dthr);
        k1[i] = drop_keep_half(own ? hm[2 + (i & 1)] : hp[2 + (i & 1)], qodd, dthr);
      }
      float pd[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pd[i] = k0[i] ? pf[i] : 0.f;
        pd[4 + i] = k1[i] ? pf[4 + i] : 0.f;
      }
      const bf16x8_t pbd = pack8(pd);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[dt] = mfma(va(s, dt), pbd, oacc[dt]);
    } else {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[dt] = mfma(va(s, dt), pb, oacc[dt]);
    }
  }
  l = lacc[0];
}

// QK^T tile init: keys >= S get -1e30 (P = 0).  EX (S > SP - 32): only the last two key tiles
// can hold padded keys, so every other tile starts from zero with no per-score work.
template <int NT, bool EX>
JM_DEVICE f32x4_t qk_init(int kt, int g, int S) {
  if (EX && kt < NT - 2) return f32x4_t{0.f, 0.f, 0.f, 0.f};
  return key_init(kt, g, S);
}

// --------------------------------------------------------------------------------- forward
// One (b, h) per workgroup.  LDS holds row-major K and V images (V^T operands come out of the
// transposing ds_read_b64_tr_b16); the Q fragments of every query tile of a wave and all of a
// thread's K / V chunks are loaded up front, one HBM round trip instead of one per chunk.
template <int HD, int SP, bool EX = false, bool DROP = false>
// waves per SIMD: the padded-row layout's occupancy, kept with the swizzled images
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(HD == 64 && SP > 128 && !DROP ? 4 : 2))) void attn_fwd_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ o,
                                                       float* __restrict__ lse, int S, int H, float scale,
                                                       AttnDrop drop) {
  JM_DGUARD(S >= 1 && S <= SP && blockDim.x == 256);
  constexpr int NT = SP / 16;
  constexpr int KK = HD / 32;
  constexpr int DT = HD / 16;
  constexpr int NCH = HD / 8;  // 16-byte chunks per row; K / V images XOR-swizzled (swo)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;
  uint16_t* Vs = smem + SP * HD;

  const int bh = xcd_bid();
  const int b = bh / H, h = bh - (bh / H) * H;
  const long ts = 3L * H * HD;  // token stride in qkv
  const uint16_t* base = qkv + (long)b * S * ts;
  const uint16_t* Qg = base + h * HD;
  const uint16_t* Kg = base + (H + h) * HD;
  const uint16_t* Vg = base + (2 * H + h) * HD;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l16 = lane & 15, g = lane >> 4;
  constexpr int NQW = (SP / 16 + 3) / 4;
  bf16x8_t qpre[NQW][KK];
#pragma unroll
  for (int i = 0; i < NQW; ++i) {
    const int q = (wave + 4 * i) * 16 + l16;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
      qpre[i][kk] = q < S ? ld8(Qg + (long)q * ts + 32 * kk + 8 * g) : __builtin_bit_cast(bf16x8_t, z);
    }
  }
  constexpr int CPR = HD / 8;
  {
    constexpr int NIT = (SP * CPR + 255) / 256;
    uint4 kv[NIT], vv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = it * 256 + threadIdx.x, r = i / CPR, c = (i % CPR) * 8;
      kv[it] = vv[it] = make_uint4(0, 0, 0, 0);
      if (i < SP * CPR && r < S) {
        kv[it] = *reinterpret_cast<const uint4*>(Kg + r * ts + c);
        vv[it] = *reinterpret_cast<const uint4*>(Vg + r * ts + c);
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = it * 256 + threadIdx.x, r = i / CPR, c = (i % CPR) * 8;
      if (i < SP * CPR) {
        *reinterpret_cast<uint4*>(Ks + swo<NCH>(r, c)) = kv[it];
        *reinterpret_cast<uint4*>(Vs + swo<NCH>(r, c)) = vv[it];
      }
    }
  }
  __syncthreads();

  const float sl2 = scale * LOG2E;
  const int NTv = (S + 15) >> 4;
  // per-lane swizzled offsets within 16- / 32-row blocks; the other column blocks XOR into the
  // chunk bits and rows r and r + 16 share a swizzle (aswz reads row bits 1-3): two registers
  const int of0 = swo<NCH>(l16, 8 * g), ot0 = swo<NCH>(4 * g + (l16 >> 2), 4 * (l16 & 3));
#pragma unroll
  for (int it = 0; it < NQW; ++it) {
    const int qt = wave + 4 * it;
    if (qt >= NTv) break;
    const int q = qt * 16 + l16;
    f32x4_t sc[NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
      f32x4_t acc = qk_init<NT, EX>(kt, g, S);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) acc = mfma(ld8(Ks + kt * 16 * HD + (of0 ^ (kk << 5))), qpre[it][kk], acc);
      sc[kt] = acc;
    }
    f32x4_t oacc[DT];
    float ms, l;
    const uint32_t seh = (uint32_t)((S + 1) >> 1), jq = (uint32_t)(bh * S) * seh + (uint32_t)(q >> 1);
    softmax_pv<NT, DT, DROP>(sc, sl2,
                             [&](int s, int dt) {
                               const uint16_t* vr = Vs + 32 * s * HD + (ot0 ^ (dt << 4));
                               return cat44(tr4(vr), tr4(vr + 16 * HD));
                             },
                             oacc, ms, l, DROP ? (uint64_t)drop.seed[0] : 0, drop.thr, jq, seh, q & 1, g);
    if (q < S) {
      const float inv = (DROP ? drop.scale : 1.f) / l;
      uint16_t* orow = o + ((long)b * S + q) * H * HD + h * HD;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        float v[4] = {oacc[dt][0] * inv, oacc[dt][1] * inv, oacc[dt][2] * inv, oacc[dt][3] * inv};
        store4(orow + dt * 16 + 4 * g, v);
      }
      if (g == 0) lse[((long)b * H + h) * S + q] = (ms + log2f(l)) * LN2;
    }
  }
}

// ------------------------------------------------------------------ forward, multi-head loop
// Same math and LDS images as attn_fwd_kernel, but one workgroup walks ``hpw``
// consecutive (b, h) pairs: the next pair's K / V rows are loaded into registers right after
// the current pair's images are in LDS, so their HBM latency hides behind the current pair's
// MFMA / softmax work (the one-pair kernel stalls on every load phase); Q fragments of the next
// query tile are prefetched the same way.
template <int HD, int SP, bool EX = false, bool DROP = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SP <= 64 && !DROP ? 5 : 2))) void attn_fwd_ml_kernel(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ o,
                                                          float* __restrict__ lse, int S, int H, int BH, int hpw,
                                                          float scale, AttnDrop drop) {
  JM_DGUARD(S >= 1 && S <= SP && hpw >= 1 && blockDim.x == 256);
  constexpr int NT = SP / 16;
  constexpr int KK = HD / 32;
  constexpr int DT = HD / 16;
  constexpr int CPR = HD / 8;
  constexpr int LPT = (SP * CPR + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;
  uint16_t* Vt = smem + SP * HD;
  const long ts = 3L * H * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const float sl2 = scale * LOG2E;

  uint4 kr[LPT], vr[LPT];
  auto load = [&](int bh) {
    const int b = bh / H, h = bh - (bh / H) * H;
    const uint16_t* base = qkv + (long)b * S * ts;
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int r = i / CPR, c = (i % CPR) * 8;
      kr[j] = make_uint4(0, 0, 0, 0);
      vr[j] = make_uint4(0, 0, 0, 0);
      if (i < SP * CPR && r < S) {
        kr[j] = *reinterpret_cast<const uint4*>(base + (long)r * ts + (H + h) * HD + c);
        vr[j] = *reinterpret_cast<const uint4*>(base + (long)r * ts + (2 * H + h) * HD + c);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < LPT; ++j) {
      const int i = threadIdx.x + 256 * j;
      const int r = i / CPR, c = (i % CPR) * 8;
      if (i < SP * CPR) {
        *reinterpret_cast<uint4*>(Ks + swo<CPR>(r, c)) = kr[j];
        *reinterpret_cast<uint4*>(Vt + swo<CPR>(r, c)) = vr[j];
      }
    }
  };
  auto load_q = [&](const uint16_t* Qg, int qt, bf16x8_t (&qf)[KK]) {
    const int q = qt * 16 + l16;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      if (q < S) {
        qf[kk] = ld8(Qg + (long)q * ts + 32 * kk + 8 * g);
      } else {
        s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
        qf[kk] = __builtin_bit_cast(bf16x8_t, z);
      }
    }
  };

  const int of0 = swo<CPR>(l16, 8 * g), ot0 = swo<CPR>(4 * g + (l16 >> 2), 4 * (l16 & 3));  // see attn_fwd_kernel
  const int bh0 = xcd_bid() * hpw;
  load(bh0);
  for (int j = 0; j < hpw; ++j) {
    const int bh = bh0 + j;
    if (bh >= BH) break;
    if (j > 0) __syncthreads();  // every wave is done reading the previous pair's images
    store();
    __syncthreads();
    if (j + 1 < hpw && bh + 1 < BH) load(bh + 1);
    const int b = bh / H, h = bh - (bh / H) * H;
    const uint16_t* Qg = qkv + (long)b * S * ts + h * HD;
    bf16x8_t qn[KK];
    if (wave < NT) load_q(Qg, wave, qn);
    for (int qt = wave; qt < NT; qt += 4) {
      const int q = qt * 16 + l16;
      bf16x8_t qf[KK];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) qf[kk] = qn[kk];
      if (qt + 4 < NT) load_q(Qg, qt + 4, qn);
      f32x4_t sc[NT];
#pragma unroll
      for (int kt = 0; kt < NT; ++kt) {
        f32x4_t acc = qk_init<NT, EX>(kt, g, S);
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) acc = mfma(ld8(Ks + kt * 16 * HD + (of0 ^ (kk << 5))), qf[kk], acc);
        sc[kt] = acc;
      }
      f32x4_t oacc[DT];
      float ms, l;
      const uint32_t seh = (uint32_t)((S + 1) >> 1), jq = (uint32_t)(bh * S) * seh + (uint32_t)(q >> 1);
      softmax_pv<NT, DT, DROP>(sc, sl2,
                               [&](int s, int dt) {
                                 const uint16_t* vr2 = Vt + 32 * s * HD + (ot0 ^ (dt << 4));
                                 return cat44(tr4(vr2), tr4(vr2 + 16 * HD));
                               },
                               oacc, ms, l, DROP ? (uint64_t)drop.seed[0] : 0, drop.thr, jq, seh, q & 1, g);
      if (q < S) {
        const float inv = (DROP ? drop.scale : 1.f) / l;
        uint16_t* orow = o + ((long)b * S + q) * H * HD + h * HD;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          float v[4] = {oacc[dt][0] * inv, oacc[dt][1] * inv, oacc[dt][2] * inv, oacc[dt][3] * inv};
          store4(orow + dt * 16 + 4 * g, v);
        }
        if (g == 0) lse[((long)b * H + h) * S + q] = (ms + log2f(l)) * LN2;
      }
    }
  }
}

// -------------------------------------------------------------------------------- backward
// (the r1 one-workgroup-per-(b, h) backward with padded LDS images was replaced by the compact and
// batched kernels below: profiles/r1_attn_bench_v3.txt, r1_attn_bwd3.txt; removed)
// ------------------------------------------------------------------ backward, compact variant
// S = softmax(Q K^T) recomputed from the saved lse, dV = P^T dO, dS = P (dP - delta), dK = dS^T Q,
// dQ = dS K; laid out so that two or more workgroups fit a
// CU (their barriers and staging then overlap each other's MFMA work):
//  * Q, dO, K images are unpadded [SP][HD] rows with the 16-byte chunks XOR-swizzled by aswz(row)
//    (a GF(2) map found by exhaustive search: conflict-free for the ds_read_b128 fragment reads AND
//    the ds_read_b64_tr_b16 transposed reads, 64 B and 128 B rows alike);
//  * V never enters LDS: each wave only needs V rows of its own key tiles -> registers;
//  * dS is stored TRANSPOSED ([key][64 queries], same swizzle): one ds_write_b64 of 4 consecutive
//    queries per lane instead of four 2-byte stores, read back for dQ with the transposing read.
// 4 waves, 64-query chunks, one 16-query dQ tile per wave per chunk.
template <int HD, int SP, int QC = 64>
constexpr size_t bwd2_smem() {
  return (size_t)(3 * SP * HD + SP * QC) * 2 + (2 * SP + (QC / 16) * 3 * HD) * sizeof(float);
}


template <int HD, int SP, bool DROP = false>
__global__ __launch_bounds__(256, 2) void attn_bwd2_kernel(const uint16_t* __restrict__ qkv,
                                                        const uint16_t* __restrict__ o,
                                                        const uint16_t* __restrict__ dO,
                                                        const float* __restrict__ lse,
                                                        uint16_t* __restrict__ dqkv, int S, int H, float scale,
                                                        float* __restrict__ dbp, int B, int ppw, AttnDrop drop) {
  JM_DGUARD(S >= 1 && S <= SP && blockDim.x == 256 && ppw >= 1);
  constexpr int NW = 4, NTH = 256, QC = 64;
  constexpr int NT = SP / 16, KK = HD / 32, DT = HD / 16;
  constexpr int NKW = (NT + NW - 1) / NW;
  constexpr int NCH = HD / 8;  // 16-byte chunks per Q / dO / K row
  constexpr int IMG = SP * HD;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Qs = smem;
  uint16_t* dOs = Qs + IMG;
  uint16_t* Ks = dOs + IMG;
  uint16_t* dSt = smem + 3 * IMG;  // [SP][QC], 8 chunks per row
  float* lse_s = reinterpret_cast<float*>(dSt + SP * QC);
  float* delta_s = lse_s + SP;
  float* bsum = delta_s + SP;

  // one workgroup walks ``ppw`` batch elements of ONE head (blockIdx = bg * H + h): the QKV bias
  // gradient partials stay in registers across them and are reduced across lanes once
  const int bid = xcd_bid();
  const int h = bid % H, bg = bid / H;
  const long ts = 3L * H * HD;
  const long os = (long)H * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const float sl2 = scale * LOG2E;
  const uint64_t dseed = DROP ? (uint64_t)drop.seed[0] : 0;
  // Every swizzled address below is (16-row-aligned base) + (per-lane constant): aswz depends on
  // row bits 1-3 only, and all bases are multiples of 16 rows.
  int o_frag[KK];  // fragment row l16, chunk 4kk + g
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) o_frag[kk] = swo<NCH>(l16, 32 * kk + 8 * g);
  int o_tr[DT][2];  // transposing reads of rows 4g + l16/4 (+16), columns dt*16 + 4 (l16 & 3)
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    o_tr[dt][0] = swo<NCH>(4 * g + (l16 >> 2), dt * 16 + 4 * (l16 & 3));
    o_tr[dt][1] = swo<NCH>(4 * g + (l16 >> 2) + 16, dt * 16 + 4 * (l16 & 3));
  }
  int o_dsw[QC / 16];  // dS^T store: row l16, queries 16 j + 4 g .. + 3
#pragma unroll
  for (int j = 0; j < QC / 16; ++j) o_dsw[j] = swo<8>(l16, 16 * j + 4 * g);
  const int krow = 8 * g + (l16 >> 2);  // dQ transposing reads: rows 32 s + krow (+4)
  int o_dsr[2], o_kt[DT][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    o_dsr[u] = swo<8>(krow + 4 * u, wave * 16 + 4 * (l16 & 3));
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o_kt[dt][u] = swo<NCH>(krow + 4 * u, dt * 16 + 4 * (l16 & 3));
  }
  // per-lane bias-gradient partials (columns dt * 16 + 4 g + i), summed over this lane's rows
  float qb[DT][4], kb[DT][4], vb[DT][4];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) qb[dt][i] = kb[dt][i] = vb[dt][i] = 0.f;

  constexpr int NIT = (SP * NCH + NTH - 1) / NTH;
  uint4 qv[NIT], kv[NIT], dv[NIT], ov[NIT];
  bf16x8_t vf[NKW][KK], vfn[NKW][KK];  // vfn: as loaded, vf: the element being computed
  float lsen = 0.f;
  // every global load of batch element b into registers in one burst -- V fragments of this
  // wave's key tiles (the B operand of dP = dO V^T), the Q / K / dO / O rows of the staging and
  // this thread's lse -- one exposed round trip per element instead of two (enc bwd 132 -> 112 us,
  // profiles/r2_attn_remap.txt); prefetching the NEXT element's burst during this element's MFMAs
  // measured slower (occupancy step: 118 us enc, 401 vs 247 us at S = 199)
  auto load_regs = [&](int b) {
    const uint16_t* base = qkv + (long)b * S * ts;
    // range-checked resources: rows at and past S read as zeros, no branch around the loads
    const __amdgpu_buffer_rsrc_t rq = rsrc(base + h * HD, (long)S * ts * 2), rk = rsrc(base + (H + h) * HD, (long)S * ts * 2),
                                 rv = rsrc(base + (2 * H + h) * HD, (long)S * ts * 2),
                                 ro = rsrc(o + (long)b * S * os + h * HD, (long)S * os * 2),
                                 rdo = rsrc(dO + (long)b * S * os + h * HD, (long)S * os * 2),
                                 rl = rsrc(lse + ((long)b * H + h) * S, (long)S * 4);
#pragma unroll
    for (int w = 0; w < NKW; ++w) {
      const int key = (wave + NW * w) * 16 + l16;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) vfn[w][kk] = __builtin_bit_cast(bf16x8_t, bld16(rv, (key * (int)ts + 32 * kk + 8 * g) * 2));
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int i = it * NTH + threadIdx.x;
      const int r = i / NCH, c = (i % NCH) * 8;  // r >= SP >= S past the image: zeros
      qv[it] = bld16(rq, (r * (int)ts + c) * 2);
      kv[it] = bld16(rk, (r * (int)ts + c) * 2);
      dv[it] = bld16(rdo, (r * (int)os + c) * 2);
      ov[it] = bld16(ro, (r * (int)os + c) * 2);
    }
    const int i = threadIdx.x;
    const float lraw = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rl, i * 4, 0, 0));
    lsen = (i < SP && i < S) ? -lraw * LOG2E : -INFINITY;
  };

  // one batch element
  auto pair = [&](const int pj) -> bool {
  const int b = bg * ppw + pj;
  if (b >= B) return false;  // workgroup-uniform
  uint16_t* dQg = dqkv + (long)b * S * ts + h * HD;
  uint16_t* dKg = dqkv + (long)b * S * ts + (H + h) * HD;
  uint16_t* dVg = dqkv + (long)b * S * ts + (2 * H + h) * HD;

  load_regs(b);
#pragma unroll
  for (int w = 0; w < NKW; ++w)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) vf[w][kk] = vfn[w][kk];
  if (threadIdx.x < SP) lse_s[threadIdx.x] = lsen;  // -lse (log2 domain): the S accumulator init
  __syncthreads();
  // LDS images from the registers; delta = O . dO
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = it * NTH + threadIdx.x;
    const int r = i / NCH, c = (i % NCH) * 8;
    if (i < SP * NCH) {
      const int off = swo<NCH>(r, c);
      *reinterpret_cast<uint4*>(Qs + off) = scale_bf16x8(qv[it], sl2);  // P = exp2(S) (see attn_bwd3_kernel)
      *reinterpret_cast<uint4*>(Ks + off) = kv[it];
      *reinterpret_cast<uint4*>(dOs + off) = dv[it];
    }
    // delta = O . dO: the NCH chunks of row r sit in NCH consecutive lanes (whole groups in or out
    // of range) -> butterfly sum and one plain store: the same value on every run, no atomics
    float dsum = 0.f;
    if (i < SP * NCH && r < S) {
      const uint32_t* ow = reinterpret_cast<const uint32_t*>(&ov[it]);
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(&dv[it]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dsum += __uint_as_float(ow[j] << 16) * __uint_as_float(dw[j] << 16);
        dsum += __uint_as_float(ow[j] & 0xffff0000u) * __uint_as_float(dw[j] & 0xffff0000u);
      }
    }
#pragma unroll
    for (int m = 1; m < NCH; m <<= 1) dsum += __shfl_xor(dsum, m, WAVE);
    if (i < SP * NCH && c == 0) delta_s[r] = -dsum;  // -delta: the dP accumulator init; padded rows 0
  }
  __syncthreads();

  bf16x8_t kf[NKW][KK];
  f32x4_t dvacc[NKW][DT], dkacc[NKW][DT];
#pragma unroll
  for (int w = 0; w < NKW; ++w) {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) kf[w][kk] = ld8(Ks + (wave + NW * w) * 16 * HD + o_frag[kk]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dvacc[w][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dkacc[w][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  }

  for (int qc = 0; qc * QC < SP; ++qc) {
    // one key tile; ``kneg`` = -1e30 on padded keys (only in the tile that holds them)
    auto tile = [&](int w, int kt, float kneg) {
      uint16_t* dsw = dSt + kt * 16 * QC;
#pragma unroll
      for (int r = 0; r < QC / 32; ++r) {
        const int qbase = qc * QC + 32 * r;
        if (qbase < SP) {
          float pf[8], df[8];
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int q0 = qbase + 16 * half;
            const float4 l4 = *reinterpret_cast<const float4*>(lse_s + q0 + 4 * g);
            const float4 d4 = *reinterpret_cast<const float4*>(delta_s + q0 + 4 * g);
            f32x4_t sacc = {l4.x + kneg, l4.y + kneg, l4.z + kneg, l4.w + kneg};
            f32x4_t dp = DROP ? f32x4_t{0.f, 0.f, 0.f, 0.f} : f32x4_t{d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
              sacc = mfma(ld8(Qs + q0 * HD + o_frag[kk]), kf[w][kk], sacc);
              dp = mfma(ld8(dOs + q0 * HD + o_frag[kk]), vf[w][kk], dp);
            }
            // sacc[i] = S[q = q0 + 4g + i][key] (log2 domain, minus lse)
            const float nd[4] = {d4.x, d4.y, d4.z, d4.w};  // -delta
            uint32_t dh[2] = {0u, 0u};  // one hash per query pair (q0 + 4g even)
            if constexpr (DROP) {
              const uint32_t seh = (uint32_t)((S + 1) >> 1);
              const uint32_t jk = (uint32_t)((b * H + h) * S + kt * 16 + l16) * seh + (uint32_t)((q0 + 4 * g) >> 1);
              dh[0] = drop_hash(jk, dseed);
              dh[1] = drop_hash(jk + 1, dseed);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float p = __builtin_amdgcn_exp2f(sacc[i]);
              if constexpr (DROP) {  // dS = P (M dP' / keep - delta); P^T dO uses M P (1 / keep at the end)
                const bool kp = drop_keep_half(dh[i >> 1], i & 1, drop.thr);
                pf[4 * half + i] = kp ? p : 0.f;
                df[4 * half + i] = p * ((kp ? dp[i] * drop.scale : 0.f) + nd[i]);
              } else {
                pf[4 * half + i] = p;
                df[4 * half + i] = p * dp[i];
              }
            }
            uint2 pk;
            pk.x = pack_bf2(df[4 * half], df[4 * half + 1]);
            pk.y = pack_bf2(df[4 * half + 2], df[4 * half + 3]);
            *reinterpret_cast<uint2*>(dsw + o_dsw[2 * r + half]) = pk;
          }
          const bf16x8_t pb = pack8(pf);
          const bf16x8_t dsb = pack8(df);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const uint16_t* dor = dOs + qbase * HD;
            const uint16_t* qr = Qs + qbase * HD;
            const bf16x8_t a_do = cat44(tr4(dor + o_tr[dt][0]), tr4(dor + o_tr[dt][1]));
            const bf16x8_t a_q = cat44(tr4(qr + o_tr[dt][0]), tr4(qr + o_tr[dt][1]));
            dvacc[w][dt] = mfma(a_do, pb, dvacc[w][dt]);
            dkacc[w][dt] = mfma(a_q, dsb, dkacc[w][dt]);
          }
        }
      }
    };
#pragma unroll
    for (int w = 0; w < NKW; ++w) {
      const int kt = wave + NW * w;
      if (kt * 16 + 16 <= S) {
        tile(w, kt, 0.f);
      } else if (kt < NT) {  // wave-uniform
        asm volatile("" ::: "memory");  // keeps the two paths apart: no per-score selects
        tile(w, kt, kt * 16 + l16 < S ? 0.f : -1e30f);
      }
    }
    __syncthreads();
    // dQ^T[d][q] = sum_key K^T[d][key] dS^T[key][q] for this wave's 16 queries of the chunk
    {
      const int qt = qc * (QC / 16) + wave;
      if (qt < NT) {
        f32x4_t dq[DT];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dq[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SP / 32; ++s) {
          const uint16_t* dsr = dSt + 32 * s * QC;
          const uint16_t* kr = Ks + 32 * s * HD;
          const bf16x8_t bop = cat44(tr4(dsr + o_dsr[0]), tr4(dsr + o_dsr[1]));
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const bf16x8_t ka = cat44(tr4(kr + o_kt[dt][0]), tr4(kr + o_kt[dt][1]));
            dq[dt] = mfma(ka, bop, dq[dt]);
          }
        }
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int i = 0; i < 4; ++i) qb[dt][i] += dq[dt][i];
        const int q = qt * 16 + l16;
        if (q < S) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            float v[4] = {dq[dt][0] * scale, dq[dt][1] * scale, dq[dt][2] * scale, dq[dt][3] * scale};
            store4(dQg + (long)q * ts + dt * 16 + 4 * g, v);
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int w = 0; w < NKW; ++w) {
    const int kt = wave + NW * w;
    const int key = kt * 16 + l16;
    if (kt < NT && key < S) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        float kv[4] = {dkacc[w][dt][0] * LN2, dkacc[w][dt][1] * LN2, dkacc[w][dt][2] * LN2,
                       dkacc[w][dt][3] * LN2};  // Q staged times scale * log2(e)
        const float vs = DROP ? drop.scale : 1.f;
        float vv[4] = {dvacc[w][dt][0] * vs, dvacc[w][dt][1] * vs, dvacc[w][dt][2] * vs, dvacc[w][dt][3] * vs};
        store4(dKg + (long)key * ts + dt * 16 + 4 * g, kv);
        store4(dVg + (long)key * ts + dt * 16 + 4 * g, vv);
      }
    }
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int w = 0; w < NKW; ++w) {
        kb[dt][i] += dkacc[w][dt][i];
        vb[dt][i] += dvacc[w][dt][i];
      }
  return true;
  };  // batch element
  for (int pj = 0; pj < ppw; ++pj)
    if (!pair(pj)) break;
  if (dbp != nullptr) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sq = row16_sum(qb[dt][i]), sk = row16_sum(kb[dt][i]), sv = row16_sum(vb[dt][i]);
        if (l16 == 0) {  // one slot per wave, summed in wave order below: deterministic
          float* bw = bsum + wave * 3 * HD;
          const int d = dt * 16 + 4 * g + i;
          bw[d] = sq * scale;
          bw[HD + d] = sk * LN2;
          bw[2 * HD + d] = DROP ? sv * drop.scale : sv;
        }
      }
    __syncthreads();
    float* dst = dbp + (long)bg * ts + h * HD;
    for (int i = threadIdx.x; i < 3 * HD; i += NTH) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) a += bsum[w * 3 * HD + i];
      dst[(i / HD) * H * HD + (i % HD)] = a;
    }
  }
}

// ------------------------------------------------------------------ backward, batched variant
// attn_bwd2_kernel's layout with the per-key-tile work batched for instruction-level parallelism
// (the decoder's hd = 32 backward was latency-bound: each 16-query slice ran LDS read -> MFMA ->
// VALU -> LDS write in series).  Per 64-query chunk a wave now
//  * loads ONCE the fragments that do not depend on the key tile -- Q / dO rows for S and dP, the
//    transposed dO / Q fragments of the dV / dK products, lse and delta -- instead of once per key
//    tile (NKW = 4 key tiles per wave at S = 199);
//  * per key tile issues the 8 independent S / dP MFMAs back to back, then the softmax-gradient
//    VALU of all four 16-query slices, then the 8 dV / dK MFMAs;
//  * runs the softmax gradient on two VALU instructions per score besides the bf16 packs: Q is
//    staged pre-multiplied by scale * log2(e) and the S accumulator starts at -lse (log2
//    domain), so P = exp2(S) with no per-score fma; the dP accumulator starts at -delta, so
//    dS = P * dP with no per-score subtraction (dK then scales by ln 2 instead of the softmax
//    scale).  Padded keys (only in the last key tile) add -1e30 to that init.
// NWV waves per workgroup: 4 (the default), or 8 for hd 64 at long S, where the 4-wave form needs
// more than 256 VGPRs (one wave per SIMD): 8 waves own half the key tiles each (half the dK / dV
// accumulators) and sweep 128-query chunks (one 16-query dQ tile per wave), two waves per SIMD.
template <int HD, int SP, int NWV = 4, bool DROP = false>
__global__ __launch_bounds__(64 * NWV, 2) void attn_bwd3_kernel(const uint16_t* __restrict__ qkv,
                                                        const uint16_t* __restrict__ o,
                                                        const uint16_t* __restrict__ dO,
                                                        const float* __restrict__ lse,
                                                        uint16_t* __restrict__ dqkv, int S, int H, float scale,
                                                        float* __restrict__ dbp, AttnDrop drop) {
  JM_DGUARD(S >= 1 && S <= SP && blockDim.x == 64 * NWV);
  constexpr int NW = NWV, NTH = 64 * NWV, QC = 16 * NWV;
  constexpr int QB = QC / 32;   // 32-query blocks per chunk
  constexpr int DCH = QC / 8;   // 16-byte chunks per dS^T row
  constexpr int NT = SP / 16, KK = HD / 32, DT = HD / 16;
  constexpr int NKW = (NT + NW - 1) / NW;
  constexpr int NCH = HD / 8;
  // smallest S dispatched to this SP (dispatch_sp buckets 32 / 64 / 128 / 224)
  constexpr int SMIN = SP <= 32 ? 1 : (SP <= 64 ? 33 : (SP <= 128 ? 65 : 129));
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Qs = smem;
  uint16_t* dOs = Qs + SP * HD;
  uint16_t* Ks = dOs + SP * HD;
  uint16_t* dSt = Ks + SP * HD;  // [SP][QC]
  float* lse_s = reinterpret_cast<float*>(dSt + SP * QC);
  float* delta_s = lse_s + SP;
  float* bsum = delta_s + SP;

  const int bh = xcd_bid();
  const int b = bh / H, h = bh - (bh / H) * H;
  const long ts = 3L * H * HD;
  const long os = (long)H * HD;
  const uint16_t* base = qkv + (long)b * S * ts;
  const uint16_t* Qg = base + h * HD;
  const uint16_t* Kg = base + (H + h) * HD;
  const uint16_t* Vg = base + (2 * H + h) * HD;
  const uint16_t* Og = o + (long)b * S * os + h * HD;
  const uint16_t* dOg = dO + (long)b * S * os + h * HD;
  uint16_t* dQg = dqkv + (long)b * S * ts + h * HD;
  uint16_t* dKg = dqkv + (long)b * S * ts + (H + h) * HD;
  uint16_t* dVg = dqkv + (long)b * S * ts + (2 * H + h) * HD;

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l16 = lane & 15, g = lane >> 4;

  bf16x8_t vf[NKW][KK];
  float kneg[NKW];  // -1e30 on padded keys
#pragma unroll
  for (int w = 0; w < NKW; ++w) {
    const int key = (wave + NW * w) * 16 + l16;
    kneg[w] = key < S ? 0.f : -1e30f;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
      vf[w][kk] = __builtin_bit_cast(bf16x8_t, z);
      if (key < S) vf[w][kk] = ld8(Vg + (long)key * ts + 32 * kk + 8 * g);
    }
  }
  // every global load in one burst (V fragments above, lse, the staging rows): one exposed round
  // trip instead of two
  static_assert(SP <= NTH, "one lse per thread");
  // -lse in the log2 domain (the S accumulator init); padded queries -inf (P = 0)
  const float nlse = (int)threadIdx.x < S ? -lse[((long)b * H + h) * S + threadIdx.x] * LOG2E : -INFINITY;
  constexpr int NIT = (SP * NCH + NTH - 1) / NTH;
  uint4 qv[NIT], kv[NIT], dv[NIT], ov[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = it * NTH + threadIdx.x;
    const int r = i / NCH, c = (i % NCH) * 8;
    qv[it] = kv[it] = dv[it] = ov[it] = make_uint4(0, 0, 0, 0);
    if (i < SP * NCH && r < S) {
      qv[it] = *reinterpret_cast<const uint4*>(Qg + r * ts + c);
      kv[it] = *reinterpret_cast<const uint4*>(Kg + r * ts + c);
      dv[it] = *reinterpret_cast<const uint4*>(dOg + r * os + c);
      ov[it] = *reinterpret_cast<const uint4*>(Og + r * os + c);
    }
  }
  for (int i = threadIdx.x; i < NW * 3 * HD; i += NTH) bsum[i] = 0.f;  // one slot per wave
  // dS^T rows of the key tiles past S: never written (those tiles are skipped), read by the dQ
  // product against zero K rows -- zero, not whatever the LDS held
  for (int i = ((S + 15) / 16) * 16 * QC + 8 * (int)threadIdx.x; i < SP * QC; i += 8 * NTH)
    *reinterpret_cast<uint4*>(dSt + i) = make_uint4(0, 0, 0, 0);
  const float sl2 = scale * LOG2E;
  const uint64_t dseed = DROP ? (uint64_t)drop.seed[0] : 0;
  if ((int)threadIdx.x < SP) lse_s[threadIdx.x] = nlse;
  __syncthreads();
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = it * NTH + threadIdx.x;
    const int r = i / NCH, c = (i % NCH) * 8;
    if (i < SP * NCH) {
      const int off = swo<NCH>(r, c);
      *reinterpret_cast<uint4*>(Qs + off) = scale_bf16x8(qv[it], sl2);
      *reinterpret_cast<uint4*>(Ks + off) = kv[it];
      // dropout: dO staged times 1 / keep, so dP and P^T dO come out scaled (delta below is taken
      // from the unscaled dO)
      *reinterpret_cast<uint4*>(dOs + off) = DROP ? scale_bf16x8(dv[it], drop.scale) : dv[it];
    }
    // delta = O . dO: the NCH chunks of row r sit in NCH consecutive lanes (whole groups in or out
    // of range) -> butterfly sum and one plain store: the same value on every run, no atomics
    float dsum = 0.f;
    if (i < SP * NCH && r < S) {
      const uint32_t* ow = reinterpret_cast<const uint32_t*>(&ov[it]);
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(&dv[it]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dsum += __uint_as_float(ow[j] << 16) * __uint_as_float(dw[j] << 16);
        dsum += __uint_as_float(ow[j] & 0xffff0000u) * __uint_as_float(dw[j] & 0xffff0000u);
      }
    }
#pragma unroll
    for (int m = 1; m < NCH; m <<= 1) dsum += __shfl_xor(dsum, m, WAVE);
    if (i < SP * NCH && c == 0) delta_s[r] = -dsum;  // -delta: the dP accumulator init; padded rows 0
  }
  __syncthreads();

  int o_frag[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) o_frag[kk] = swo<NCH>(l16, 32 * kk + 8 * g);
  int o_tr[DT][2];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    o_tr[dt][0] = swo<NCH>(4 * g + (l16 >> 2), dt * 16 + 4 * (l16 & 3));
    o_tr[dt][1] = swo<NCH>(4 * g + (l16 >> 2) + 16, dt * 16 + 4 * (l16 & 3));
  }
  int o_dsw[QC / 16];
#pragma unroll
  for (int j = 0; j < QC / 16; ++j) o_dsw[j] = swo<DCH>(l16, 16 * j + 4 * g);
  const int krow = 8 * g + (l16 >> 2);
  int o_dsr[2], o_kt[DT][2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    o_dsr[u] = swo<DCH>(krow + 4 * u, wave * 16 + 4 * (l16 & 3));
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o_kt[dt][u] = swo<NCH>(krow + 4 * u, dt * 16 + 4 * (l16 & 3));
  }

  bf16x8_t kf[NKW][KK];
  f32x4_t dvacc[NKW][DT], dkacc[NKW][DT];
#pragma unroll
  for (int w = 0; w < NKW; ++w) {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) kf[w][kk] = ld8(Ks + (wave + NW * w) * 16 * HD + o_frag[kk]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dvacc[w][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      dkacc[w][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
  }

  for (int qc = 0; qc * QC < SP; ++qc) {
    const int q0 = qc * QC;
    const int nr = (SP - q0) >= QC ? QB : (SP - q0) / 32;  // 32-query blocks in this chunk (SP % 32 == 0)
    // (not unrolled at 8 waves: the 4-block chunk would keep every block's fragments live)
#pragma unroll(NWV == 4 ? QB : 1)
    for (int r = 0; r < QB; ++r) {
      if (r < nr) {
        // ---- key-tile independent fragments of this 32-query block
        const int qb = q0 + 32 * r;
        bf16x8_t qf[2][KK], dof[2][KK], a_do[DT], a_q[DT];
        f32x4_t lv[2], dl[2];  // accumulator inits: -lse (log2 domain) and -delta
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if constexpr (!(DROP && NWV == 8)) {
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
              qf[hh][kk] = ld8(Qs + (qb + 16 * hh) * HD + o_frag[kk]);
              dof[hh][kk] = ld8(dOs + (qb + 16 * hh) * HD + o_frag[kk]);
            }
            const float4 l4 = *reinterpret_cast<const float4*>(lse_s + qb + 16 * hh + 4 * g);
            const float4 d4 = *reinterpret_cast<const float4*>(delta_s + qb + 16 * hh + 4 * g);
            lv[hh] = f32x4_t{l4.x, l4.y, l4.z, l4.w};
            dl[hh] = f32x4_t{d4.x, d4.y, d4.z, d4.w};
          }
        }
        // the transposed dO / Q operands of the dV / dK products: loaded once per block, or per
        // key tile in the 8-wave dropout variant (whose mask work would otherwise spill)
        constexpr bool TILE_AOP = DROP && NWV == 8;
        auto load_aop = [&]() {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            a_do[dt] = cat44(tr4(dOs + qb * HD + o_tr[dt][0]), tr4(dOs + qb * HD + o_tr[dt][1]));
            a_q[dt] = cat44(tr4(Qs + qb * HD + o_tr[dt][0]), tr4(Qs + qb * HD + o_tr[dt][1]));
          }
        };
        if constexpr (!TILE_AOP) load_aop();
        // one key tile: S / dP products from the accumulator inits, softmax gradient, dV / dK
        // TILE_AOP: -lse / -delta re-read from LDS per tile too (kn: the padded-key init), so no
        // per-block vectors stay live across the key tiles
        auto tile = [&](int w, int kt, const f32x4_t (&ini)[2], float kn) {
          f32x4_t sacc[2], dp[2], dlt[2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            if constexpr (TILE_AOP) {
              const float4 l4 = *reinterpret_cast<const float4*>(lse_s + qb + 16 * hh + 4 * g);
              const float4 d4 = *reinterpret_cast<const float4*>(delta_s + qb + 16 * hh + 4 * g);
              sacc[hh] = f32x4_t{l4.x + kn, l4.y + kn, l4.z + kn, l4.w + kn};
              dlt[hh] = f32x4_t{d4.x, d4.y, d4.z, d4.w};
            } else {
              sacc[hh] = ini[hh];
              dlt[hh] = dl[hh];
            }
            dp[hh] = dlt[hh];
            if constexpr (TILE_AOP) {  // the Q / dO fragments too: nothing per block stays live
#pragma unroll
              for (int kk = 0; kk < KK; ++kk) {
                qf[hh][kk] = ld8(Qs + (qb + 16 * hh) * HD + o_frag[kk]);
                dof[hh][kk] = ld8(dOs + (qb + 16 * hh) * HD + o_frag[kk]);
              }
            }
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
              sacc[hh] = mfma(qf[hh][kk], kf[w][kk], sacc[hh]);
              dp[hh] = mfma(dof[hh][kk], vf[w][kk], dp[hh]);
            }
          }
          float pf[8], df[8];
          uint16_t* dsw = dSt + kt * 16 * QC;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            uint32_t dh[2] = {0u, 0u};  // one hash per query pair (qb + 16 hh + 4 g even)
            if constexpr (DROP) {
              const uint32_t seh = (uint32_t)((S + 1) >> 1);
              const uint32_t jk = (uint32_t)(bh * S + kt * 16 + l16) * seh + (uint32_t)((qb + 16 * hh + 4 * g) >> 1);
              dh[0] = drop_hash(jk, dseed);
              dh[1] = drop_hash(jk + 1, dseed);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float p = __builtin_amdgcn_exp2f(sacc[hh][i]);
              if constexpr (DROP) {  // dS = P (M dP' / keep - delta), dp = dP' / keep - delta (dO
                                     // staged scaled, -delta init); P^T dO uses M P
                const bool kp = drop_keep_half(dh[i >> 1], i & 1, drop.thr);
                pf[4 * hh + i] = kp ? p : 0.f;
                df[4 * hh + i] = p * (kp ? dp[hh][i] : dlt[hh][i]);
              } else {
                pf[4 * hh + i] = p;
                df[4 * hh + i] = p * dp[hh][i];
              }
            }
            uint2 pk;
            pk.x = pack_bf2(df[4 * hh], df[4 * hh + 1]);
            pk.y = pack_bf2(df[4 * hh + 2], df[4 * hh + 3]);
            *reinterpret_cast<uint2*>(dsw + (NWV == 4 ? o_dsw[2 * r + hh] : swo<DCH>(l16, 16 * (2 * r + hh) + 4 * g))) = pk;
          }
          const bf16x8_t pb = pack8(pf);
          const bf16x8_t dsb = pack8(df);
          if constexpr (TILE_AOP) load_aop();
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            dvacc[w][dt] = mfma(a_do[dt], pb, dvacc[w][dt]);
            dkacc[w][dt] = mfma(a_q[dt], dsb, dkacc[w][dt]);
          }
        };
#pragma unroll
        for (int w = 0; w < NKW; ++w) {
          const int kt = wave + NW * w;
          if (NWV == 4 && NW * 16 * (w + 1) <= SMIN) {  // compile-time after the unroll (8 waves: spills)
            // full for every S of this instantiation: no branch around it, so the scheduler
            // interleaves these tiles' MFMA -> exp -> MFMA chains
            tile(w, kt, lv, 0.f);
          } else if (kt * 16 + 16 <= S) {
            tile(w, kt, lv, 0.f);
          } else if (kt * 16 < S) {  // the tile holding padded keys (wave-uniform branch); tiles
                                     // past S are skipped (their dS^T rows stay zero)
            asm volatile("" ::: "memory");  // keeps the two paths apart: no per-tile selects
            if constexpr (TILE_AOP) {
              tile(w, kt, lv, kneg[w]);
            } else {
              const f32x4_t lm[2] = {lv[0] + kneg[w], lv[1] + kneg[w]};
              tile(w, kt, lm, 0.f);
            }
          }
        }
      }
    }
    __syncthreads();
    {
      const int qt = qc * (QC / 16) + wave;
      if (qt < NT) {
        f32x4_t dq[DT];
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dq[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < SP / 32; ++s2) {
          const uint16_t* dsr = dSt + 32 * s2 * QC;
          const uint16_t* kr = Ks + 32 * s2 * HD;
          const bf16x8_t bop = cat44(tr4(dsr + o_dsr[0]), tr4(dsr + o_dsr[1]));
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const bf16x8_t ka = cat44(tr4(kr + o_kt[dt][0]), tr4(kr + o_kt[dt][1]));
            dq[dt] = mfma(ka, bop, dq[dt]);
          }
        }
        if (dbp != nullptr) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float v = row16_sum(dq[dt][i]);
              if (l16 == 0) bsum[wave * 3 * HD + dt * 16 + 4 * g + i] += v * scale;  // this wave's slot
            }
        }
        const int q = qt * 16 + l16;
        if (q < S) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            float v[4] = {dq[dt][0] * scale, dq[dt][1] * scale, dq[dt][2] * scale, dq[dt][3] * scale};
            store4(dQg + (long)q * ts + dt * 16 + 4 * g, v);
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int w = 0; w < NKW; ++w) {
    const int kt = wave + NW * w;
    const int key = kt * 16 + l16;
    if (kt < NT && key < S) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        float kv2[4] = {dkacc[w][dt][0] * LN2, dkacc[w][dt][1] * LN2, dkacc[w][dt][2] * LN2,
                        dkacc[w][dt][3] * LN2};
        float vv[4] = {dvacc[w][dt][0], dvacc[w][dt][1], dvacc[w][dt][2], dvacc[w][dt][3]};  // dO staged scaled
        store4(dKg + (long)key * ts + dt * 16 + 4 * g, kv2);
        store4(dVg + (long)key * ts + dt * 16 + 4 * g, vv);
      }
    }
  }
  if (dbp != nullptr) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float sk = 0.f, sv = 0.f;
#pragma unroll
        for (int w = 0; w < NKW; ++w) {
          sk += dkacc[w][dt][i];
          sv += dvacc[w][dt][i];
        }
        sk = row16_sum(sk);
        sv = row16_sum(sv);
        if (l16 == 0) {
          float* bw = bsum + wave * 3 * HD;
          const int d = dt * 16 + 4 * g + i;
          bw[HD + d] = sk * LN2;
          bw[2 * HD + d] = sv;
        }
      }
    __syncthreads();
    float* dst = dbp + (long)b * ts + h * HD;
    for (int i = threadIdx.x; i < 3 * HD; i += NTH) {
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) a += bsum[w * 3 * HD + i];  // wave order: deterministic
      dst[(i / HD) * H * HD + (i % HD)] = a;
    }
  }
}

// forward images: row-major K and V, XOR-swizzled (V^T operands through ds_read_b64_tr_b16)
template <int HD, int SP>
size_t fwd_smem() { return (size_t)(2 * SP * HD) * 2; }

// one (b, h) per workgroup (S > 64; the short encoder sequences take the multi-pair kernel)
template <int HD, int SP, bool DROP>
int run_fwd(const uint16_t* qkv, uint16_t* out, float* lse_out, int B, int S, int H, float scale, AttnDrop dr,
            hipStream_t st) {
  dim3 grid(B * H);
  const size_t sm = fwd_smem<HD, SP>();
  if (sm > 160 * 1024) return -3;
  if (S > SP - 32) {
    static bool attr_ex = false;
    if (sm > 64 * 1024 && !attr_ex) {
      (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<HD, SP, true, DROP>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
      attr_ex = true;
    }
    attn_fwd_kernel<HD, SP, true, DROP><<<grid, 256, sm, st>>>(qkv, out, lse_out, S, H, scale, dr);
  } else {
    static bool attr = false;
    if (sm > 64 * 1024 && !attr) {
      (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<HD, SP, false, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sm);
      attr = true;
    }
    attn_fwd_kernel<HD, SP, false, DROP><<<grid, 256, sm, st>>>(qkv, out, lse_out, S, H, scale, dr);
  }
  return 0;
}

// The backward kernel per shape -- the single source of that choice for run_bwd and
// jm_attn_bwd_part_rows:
//  * hd 32 (decoder): the batched bwd3, 4 waves (profiles/r1_attn_bwd3.txt);
//  * hd 64, S > 64 (finetune S = 199): bwd3 with 8 waves, two per SIMD (the 4-wave form needs
//    more than 256 VGPRs there): 249 -> 177 us (profiles/r2_attn_ft_bwd.txt);
//  * hd 64, S <= 64 (the ViT-L encoder): the compact bwd2, BWD2_PPW batch elements per workgroup.
bool uses_bwd3(int S, int hd) { return hd == 32 || (hd == 64 && S > 64); }
// ViT-L encoder (S 52): 160 -> 140 us at 8 batch elements per bwd2 workgroup (profiles/r1_attn_bwd_ppw.txt)
// (16 at the 2048-image micro-batch: enc bwd 399.8 -> 403.0 us, tools/attn_bench.py enc2k, gpurun r4pp)
constexpr int BWD2_PPW = 8;

template <int HD, int SP, bool DROP>
int run_bwd(const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse_in, uint16_t* out,
            float* dbias_part, int B, int S, int H, float scale, AttnDrop dr, hipStream_t st) {
  if constexpr (HD == 64 && SP > 64) {
    constexpr size_t sm8 = bwd2_smem<HD, SP, 128>();
    static_assert(sm8 <= 160 * 1024, "8-wave backward LDS");
    static bool attr8 = false;
    if (!attr8) {
      (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<HD, SP, 8, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sm8);
      attr8 = true;
    }
    attn_bwd3_kernel<HD, SP, 8, DROP><<<dim3(B * H), 512, sm8, st>>>(qkv, o, dO, lse_in, out, S, H, scale, dbias_part, dr);
  } else {
    constexpr size_t sm = bwd2_smem<HD, SP>();
    static_assert(sm <= 160 * 1024, "backward LDS");
    static bool attr = false;
    if constexpr (HD == 32) {
      if (sm > 64 * 1024 && !attr) {
        (void)hipFuncSetAttribute((const void*)attn_bwd3_kernel<HD, SP, 4, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sm);
        attr = true;
      }
      attn_bwd3_kernel<HD, SP, 4, DROP><<<dim3(B * H), 256, sm, st>>>(qkv, o, dO, lse_in, out, S, H, scale, dbias_part, dr);
    } else {
      if (sm > 64 * 1024 && !attr) {
        (void)hipFuncSetAttribute((const void*)attn_bwd2_kernel<HD, SP, DROP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)sm);
        attr = true;
      }
      attn_bwd2_kernel<HD, SP, DROP><<<dim3(((B + BWD2_PPW - 1) / BWD2_PPW) * H), 256, sm, st>>>(
          qkv, o, dO, lse_in, out, S, H, scale, dbias_part, B, BWD2_PPW, dr);
    }
  }
  return 0;
}

// forward: the multi-pair kernel (4 (b, h) per workgroup) for the short encoder sequences
// (SP <= 64: 43 -> 39 us), the one-pair kernel for the decoder, where the extra prefetch registers
// cost an occupancy step (199 -> 215 us; profiles/r1_attn_fwd_ml.txt)
// (8 pairs at the 2048-image micro-batch: enc fwd 186.6 -> 191.2 us, gpurun r4pp)
constexpr int FWD_ML_PAIRS = 4;

template <int HD, int SP, bool DROP>
int run_fwd_ml(const uint16_t* qkv, uint16_t* out, float* lse_out, int B, int S, int H, float scale, AttnDrop dr,
               hipStream_t st) {
  const size_t sm = fwd_smem<HD, SP>();
  static bool attr_set[2] = {false, false};
  const bool ex = S > SP - 32;
  const void* fn = ex ? (const void*)attn_fwd_ml_kernel<HD, SP, true, DROP> : (const void*)attn_fwd_ml_kernel<HD, SP, false, DROP>;
  if (sm > 64 * 1024 && !attr_set[ex]) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    attr_set[ex] = true;
  }
  const int BH = B * H;
  const int grid = (BH + FWD_ML_PAIRS - 1) / FWD_ML_PAIRS;
  if (ex)
    attn_fwd_ml_kernel<HD, SP, true, DROP><<<grid, 256, sm, st>>>(qkv, out, lse_out, S, H, BH, FWD_ML_PAIRS, scale, dr);
  else
    attn_fwd_ml_kernel<HD, SP, false, DROP><<<grid, 256, sm, st>>>(qkv, out, lse_out, S, H, BH, FWD_ML_PAIRS, scale, dr);
  return 0;
}

template <int HD, int SP>
int run(bool fwd, const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse_in, uint16_t* out,
        float* lse_out, int B, int S, int H, float scale, AttnDrop dr, hipStream_t st) {
  if (dr.seed != nullptr) {
    if (!fwd) return run_bwd<HD, SP, true>(qkv, o, dO, lse_in, out, lse_out, B, S, H, scale, dr, st);
    if constexpr (SP <= 64) return run_fwd_ml<HD, SP, true>(qkv, out, lse_out, B, S, H, scale, dr, st);
    return run_fwd<HD, SP, true>(qkv, out, lse_out, B, S, H, scale, dr, st);
  }
  if (!fwd) return run_bwd<HD, SP, false>(qkv, o, dO, lse_in, out, lse_out, B, S, H, scale, dr, st);
  if constexpr (SP <= 64) return run_fwd_ml<HD, SP, false>(qkv, out, lse_out, B, S, H, scale, dr, st);
  return run_fwd<HD, SP, false>(qkv, out, lse_out, B, S, H, scale, dr, st);
}

template <int HD>
int dispatch_sp(bool fwd, const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse_in,
                uint16_t* out, float* lse_out, int B, int S, int H, float scale, AttnDrop dr, hipStream_t st) {
  if (S <= 32) return run<HD, 32>(fwd, qkv, o, dO, lse_in, out, lse_out, B, S, H, scale, dr, st);
  if (S <= 64) return run<HD, 64>(fwd, qkv, o, dO, lse_in, out, lse_out, B, S, H, scale, dr, st);
  if (S <= 128) return run<HD, 128>(fwd, qkv, o, dO, lse_in, out, lse_out, B, S, H, scale, dr, st);
  if (S <= 224) return run<HD, 224>(fwd, qkv, o, dO, lse_in, out, lse_out, B, S, H, scale, dr, st);
  return -2;
}

// ------------------------------------------------------ long sequences (S > 224): tile-streamed
// Past 224 tokens one (b, h) no longer fits a workgroup's register/LDS budget (finetuning at
// 448 px: S = 787), so 64-row tiles stream through LDS instead.  The MFMA
// orientations are the ones of the fused kernels above:
//   attn_fwd_long_kernel  WG = 64 queries of one (b, h) (one 16-query tile per wave, query on the
//                         lane); online softmax over 64-key tiles; O^T = V^T P^T with P^T straight
//                         from the S^T accumulators.
//   attn_bwd_dq_kernel    WG = 64 queries; P^T recomputed from lse; dQ^T = K^T dS^T; also writes
//                         delta = rowsum(dO * O) for the next kernel.
//   attn_bwd_dkv_kernel   WG = 64 keys (key on the lane, K / V fragments kept in registers);
//                         sweeps 64-query tiles: dV^T += dO^T P, dK^T += Q^T dS.
// Every output element has one writer: no atomics, deterministic.  Grid x = (b, h) major, tile
// minor, so the WGs sharing one (b, h)'s K / V (or Q / dO) rows are dispatched together.
constexpr int LT = 64;

// a 64 x HD bf16 tile moves HBM -> registers (issued one tile ahead, so its latency hides behind
// the current tile's MFMA work) -> LDS (row stride HD + 8); rows past S are zero
template <int HD>
struct TileRegs {
  uint4 v[HD / 32];
};

template <int HD>
JM_DEVICE void tile_fetch(TileRegs<HD>& t, const uint16_t* src, long rs, int r0, int S) {
  constexpr int CPR = HD / 8;
#pragma unroll
  for (int j = 0; j < HD / 32; ++j) {
    const int i = threadIdx.x + 256 * j, r = i / CPR, c = (i % CPR) * 8;
    t.v[j] = r0 + r < S ? *reinterpret_cast<const uint4*>(src + (long)(r0 + r) * rs + c) : make_uint4(0, 0, 0, 0);
  }
}

template <int HD>
JM_DEVICE void tile_store(uint16_t* dst, const TileRegs<HD>& t) {
  constexpr int CPR = HD / 8, KS = HD + 8;
#pragma unroll
  for (int j = 0; j < HD / 32; ++j) {
    const int i = threadIdx.x + 256 * j, r = i / CPR, c = (i % CPR) * 8;
    *reinterpret_cast<uint4*>(dst + r * KS + c) = t.v[j];
  }
}

// A operand of X^T (d on the lane) for a 32-row chunk of a row-major LDS tile, rows permuted
// like the packed P^T / dS^T fragments (rows 4g..4g+3, then 16+4g..16+4g+3)
template <int HD>
JM_DEVICE bf16x8_t tr_frag(const uint16_t* t, int s, int dt, int l16, int g) {
  constexpr int KS = HD + 8;
  const uint16_t* p = t + (32 * s + 4 * g + (l16 >> 2)) * KS + dt * 16 + 4 * (l16 & 3);
  return cat44(tr4(p), tr4(p + 16 * KS));
}

template <int HD>
__global__ __launch_bounds__(256, 2) void attn_fwd_long_kernel(const uint16_t* __restrict__ qkv,
                                                            uint16_t* __restrict__ o, float* __restrict__ lse,
                                                            int S, int H, float scale) {
  constexpr int KS = HD + 8, KK = HD / 32, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LT * KS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[LT * KS];
  const int nq = (S + LT - 1) / LT;
  const int bh = blockIdx.x / nq, qb = blockIdx.x - bh * nq;
  const int b = bh / H, h = bh - b * H;
  const long ts = 3L * H * HD;
  const uint16_t* base = qkv + (long)b * S * ts;
  const uint16_t* Kg = base + (H + h) * HD;
  const uint16_t* Vg = base + (2 * H + h) * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, l16 = lane & 15, g = lane >> 4;
  const int q = qb * LT + wave * 16 + l16;
  const float sl2 = scale * LOG2E;

  bf16x8_t qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
    qf[kk] = q < S ? ld8(base + (long)q * ts + h * HD + 32 * kk + 8 * g) : __builtin_bit_cast(bf16x8_t, z);
  }
  f32x4_t oacc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) oacc[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  TileRegs<HD> kr, vr;
  tile_fetch<HD>(kr, Kg, ts, 0, S);
  tile_fetch<HD>(vr, Vg, ts, 0, S);
  for (int k0 = 0; k0 < S; k0 += LT) {
    __syncthreads();
    tile_store<HD>(Ks, kr);
    tile_store<HD>(Vs, vr);
    __syncthreads();
    if (k0 + LT < S) {
      tile_fetch<HD>(kr, Kg, ts, k0 + LT, S);
      tile_fetch<HD>(vr, Vg, ts, k0 + LT, S);
    }
    f32x4_t sc[4];
    float mt = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) acc = mfma(ld8(Ks + (kt * 16 + l16) * KS + 32 * kk + 8 * g), qf[kk], acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = k0 + kt * 16 + 4 * g + i < S ? acc[i] * sl2 : -INFINITY;
        sc[kt][i] = v;
        mt = fmaxf(mt, v);
      }
    }
    mt = fmaxf(mt, __shfl_xor(mt, 16, WAVE));
    mt = fmaxf(mt, __shfl_xor(mt, 32, WAVE));
    const float mn = fmaxf(m, mt);  // finite: every tile holds at least one valid key
    const float alpha = __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) oacc[dt] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = __builtin_amdgcn_exp2f(sc[kt][i] - m);
        sc[kt][i] = p;
        l += p;
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float pf[8] = {sc[2 * s][0], sc[2 * s][1], sc[2 * s][2], sc[2 * s][3],
                     sc[2 * s + 1][0], sc[2 * s + 1][1], sc[2 * s + 1][2], sc[2 * s + 1][3]};
      const bf16x8_t pb = pack8(pf);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[dt] = mfma(tr_frag<HD>(Vs, s, dt, l16, g), pb, oacc[dt]);
    }
  }
  l += __shfl_xor(l, 16, WAVE);
  l += __shfl_xor(l, 32, WAVE);
  if (q < S) {
    const float inv = 1.f / l;
    uint16_t* orow = o + ((long)b * S + q) * H * HD + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      float v[4] = {oacc[dt][0] * inv, oacc[dt][1] * inv, oacc[dt][2] * inv, oacc[dt][3] * inv};
      store4(orow + dt * 16 + 4 * g, v);
    }
    if (g == 0) lse[((long)b * H + h) * S + q] = (m + log2f(l)) * LN2;
  }
}

template <int HD>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(const uint16_t* __restrict__ qkv,
                                                          const uint16_t* __restrict__ o,
                                                          const uint16_t* __restrict__ dO,
                                                          const float* __restrict__ lse,
                                                          uint16_t* __restrict__ dqkv, float* __restrict__ delta,
                                                          int S, int H, float scale) {
  constexpr int KS = HD + 8, KK = HD / 32, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) uint16_t Ks[LT * KS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[LT * KS];
  const int nq = (S + LT - 1) / LT;
  const int bh = blockIdx.x / nq, qb = blockIdx.x - bh * nq;
  const int b = bh / H, h = bh - b * H;
  const long ts = 3L * H * HD;
  const uint16_t* base = qkv + (long)b * S * ts;
  const uint16_t* Kg = base + (H + h) * HD;
  const uint16_t* Vg = base + (2 * H + h) * HD;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, l16 = lane & 15, g = lane >> 4;
  const int q = qb * LT + wave * 16 + l16;
  const float sl2 = scale * LOG2E;

  bf16x8_t qf[KK], df[KK];
  float dl = 0.f;
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
    qf[kk] = df[kk] = __builtin_bit_cast(bf16x8_t, z);
    if (q < S) {
      const long orow = ((long)b * S + q) * H * HD + h * HD + 32 * kk + 8 * g;
      qf[kk] = ld8(base + (long)q * ts + h * HD + 32 * kk + 8 * g);
      df[kk] = ld8(dO + orow);
      const s16x8_t dv = __builtin_bit_cast(s16x8_t, df[kk]);
      const s16x8_t ov = __builtin_bit_cast(s16x8_t, ld8(o + orow));
#pragma unroll
      for (int j = 0; j < 8; ++j) dl += bf2f((uint16_t)dv[j]) * bf2f((uint16_t)ov[j]);
    }
  }
  dl += __shfl_xor(dl, 16, WAVE);
  dl += __shfl_xor(dl, 32, WAVE);
  const long lrow = ((long)b * H + h) * S;
  const float l2 = q < S ? lse[lrow + q] * LOG2E : INFINITY;
  if (q < S && g == 0) delta[lrow + q] = dl;

  f32x4_t dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  TileRegs<HD> kr, vr;
  tile_fetch<HD>(kr, Kg, ts, 0, S);
  tile_fetch<HD>(vr, Vg, ts, 0, S);
  for (int k0 = 0; k0 < S; k0 += LT) {
    __syncthreads();
    tile_store<HD>(Ks, kr);
    tile_store<HD>(Vs, vr);
    __syncthreads();
    if (k0 + LT < S) {
      tile_fetch<HD>(kr, Kg, ts, k0 + LT, S);
      tile_fetch<HD>(vr, Vg, ts, k0 + LT, S);
    }
    float ds[4][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4_t sa = {0.f, 0.f, 0.f, 0.f}, pa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        sa = mfma(ld8(Ks + (kt * 16 + l16) * KS + 32 * kk + 8 * g), qf[kk], sa);
        pa = mfma(ld8(Vs + (kt * 16 + l16) * KS + 32 * kk + 8 * g), df[kk], pa);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = k0 + kt * 16 + 4 * g + i < S ? __builtin_amdgcn_exp2f(sa[i] * sl2 - l2) : 0.f;
        ds[kt][i] = p * (pa[i] - dl);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float f[8] = {ds[2 * s][0], ds[2 * s][1], ds[2 * s][2], ds[2 * s][3],
                    ds[2 * s + 1][0], ds[2 * s + 1][1], ds[2 * s + 1][2], ds[2 * s + 1][3]};
      const bf16x8_t db = pack8(f);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) dq[dt] = mfma(tr_frag<HD>(Ks, s, dt, l16, g), db, dq[dt]);
    }
  }
  if (q < S) {
    uint16_t* row = dqkv + ((long)b * S + q) * ts + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      float v[4] = {dq[dt][0] * scale, dq[dt][1] * scale, dq[dt][2] * scale, dq[dt][3] * scale};
      store4(row + dt * 16 + 4 * g, v);
    }
  }
}

template <int HD>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_kernel(const uint16_t* __restrict__ qkv,
                                                           const uint16_t* __restrict__ dO,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           uint16_t* __restrict__ dqkv, int S, int H, float scale) {
  constexpr int KS = HD + 8, KK = HD / 32, DT = HD / 16;
  __shared__ __attribute__((aligned(16))) uint16_t Qs[LT * KS];
  __shared__ __attribute__((aligned(16))) uint16_t Ds[LT * KS];
  __shared__ float Ls[LT], Dl[LT];
  const int nk = (S + LT - 1) / LT;
  const int bh = blockIdx.x / nk, kb = blockIdx.x - bh * nk;
  const int b = bh / H, h = bh - b * H;
  const long ts = 3L * H * HD;
  const uint16_t* base = qkv + (long)b * S * ts;
  const uint16_t* Qg = base + h * HD;
  const uint16_t* dOg = dO + (long)b * S * H * HD + h * HD;
  const long lrow = ((long)b * H + h) * S;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, l16 = lane & 15, g = lane >> 4;
  const int key = kb * LT + wave * 16 + l16;
  const bool kv = key < S;
  const float sl2 = scale * LOG2E;

  bf16x8_t kf[KK], vf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    s16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
    kf[kk] = vf[kk] = __builtin_bit_cast(bf16x8_t, z);
    if (kv) {
      kf[kk] = ld8(base + (long)key * ts + (H + h) * HD + 32 * kk + 8 * g);
      vf[kk] = ld8(base + (long)key * ts + (2 * H + h) * HD + 32 * kk + 8 * g);
    }
  }
  f32x4_t dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dk[dt] = dv[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  TileRegs<HD> qr, dr;
  float lr = INFINITY, dlr = 0.f;
  auto fetch = [&](int r0) {
    tile_fetch<HD>(qr, Qg, ts, r0, S);
    tile_fetch<HD>(dr, dOg, (long)H * HD, r0, S);
    const int r = r0 + threadIdx.x;
    if (threadIdx.x < LT && r < S) {
      lr = lse[lrow + r] * LOG2E;
      dlr = delta[lrow + r];
    } else {
      lr = INFINITY;
      dlr = 0.f;
    }
  };
  fetch(0);
  for (int q0 = 0; q0 < S; q0 += LT) {
    __syncthreads();
    tile_store<HD>(Qs, qr);
    tile_store<HD>(Ds, dr);
    if (threadIdx.x < LT) {
      Ls[threadIdx.x] = lr;
      Dl[threadIdx.x] = dlr;
    }
    __syncthreads();
    if (q0 + LT < S) fetch(q0 + LT);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float pf[8], df[8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int qt = 2 * s + t;
        f32x4_t sa = {0.f, 0.f, 0.f, 0.f}, pa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          sa = mfma(ld8(Qs + (qt * 16 + l16) * KS + 32 * kk + 8 * g), kf[kk], sa);
          pa = mfma(ld8(Ds + (qt * 16 + l16) * KS + 32 * kk + 8 * g), vf[kk], pa);
        }
        // sa[i] = S[query = qt*16 + 4g + i][key = l16]
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = qt * 16 + 4 * g + i;
          const float p = kv ? __builtin_amdgcn_exp2f(sa[i] * sl2 - Ls[qq]) : 0.f;
          pf[4 * t + i] = p;
          df[4 * t + i] = p * (pa[i] - Dl[qq]);
        }
      }
      const bf16x8_t pb = pack8(pf), db = pack8(df);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        dv[dt] = mfma(tr_frag<HD>(Ds, s, dt, l16, g), pb, dv[dt]);
        dk[dt] = mfma(tr_frag<HD>(Qs, s, dt, l16, g), db, dk[dt]);
      }
    }
  }
  // dk[dt][i] = dK^T[d = dt*16 + 4g + i][key]
  if (kv) {
    uint16_t* row = dqkv + ((long)b * S + key) * ts;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      float a[4] = {dk[dt][0] * scale, dk[dt][1] * scale, dk[dt][2] * scale, dk[dt][3] * scale};
      float c[4] = {dv[dt][0], dv[dt][1], dv[dt][2], dv[dt][3]};
      store4(row + (H + h) * HD + dt * 16 + 4 * g, a);
      store4(row + (2 * H + h) * HD + dt * 16 + 4 * g, c);
    }
  }
}

template <int HD>
int run_long_fwd(const uint16_t* qkv, uint16_t* o, float* lse, int B, int S, int H, float scale, hipStream_t st) {
  const long grid = (long)B * H * ((S + LT - 1) / LT);
  if (grid > 0x7fffffffL) return -5;
  attn_fwd_long_kernel<HD><<<dim3((unsigned)grid), 256, 0, st>>>(qkv, o, lse, S, H, scale);
  return 0;
}

template <int HD>
int run_long_bwd(const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse, uint16_t* dqkv,
                 float* delta, int B, int S, int H, float scale, hipStream_t st) {
  const long grid = (long)B * H * ((S + LT - 1) / LT);
  if (grid > 0x7fffffffL) return -5;
  attn_bwd_dq_kernel<HD><<<dim3((unsigned)grid), 256, 0, st>>>(qkv, o, dO, lse, dqkv, delta, S, H, scale);
  attn_bwd_dkv_kernel<HD><<<dim3((unsigned)grid), 256, 0, st>>>(qkv, dO, lse, delta, dqkv, S, H, scale);
  return 0;
}

}  // namespace

// longest sequence on the whole-sequence-in-LDS kernels (every flagship shape); the
// tile-streamed kernels take longer ones
constexpr int ATTN_MAX_SEQ = 224;
int jm_attn_max_seq() { return ATTN_MAX_SEQ; }

// rows of the dbias_part workspace that jm_attn_bwd writes: the bwd2 kernel folds BWD2_PPW batch
// elements into one row, every other backward writes one row per batch element.
int jm_attn_bwd_part_rows(int B, int S, int hd) {
  if (uses_bwd3(S, hd) || S > ATTN_MAX_SEQ || hd != 64) return B;
  return (B + BWD2_PPW - 1) / BWD2_PPW;
}

// dseed (int64 [1] on the device) non-null: dropout on the attention probabilities with keep
// threshold dthr = round(keep * 65536) and dscale = 1 / keep (whole-sequence kernels, S <= 224)
int jm_attn_fwd(const uint16_t* qkv, uint16_t* o, float* lse, int B, int S, int H, int hd, const int64_t* dseed,
                uint32_t dthr, float dscale, hipStream_t st) {
  const float scale = 1.f / sqrtf((float)hd);
  const AttnDrop dr{dseed, dthr, dscale};
  if (S > jm_attn_max_seq()) {
    if (dseed != nullptr) return -5;
    if (hd == 32) return run_long_fwd<32>(qkv, o, lse, B, S, H, scale, st);
    if (hd == 64) return run_long_fwd<64>(qkv, o, lse, B, S, H, scale, st);
    return -1;
  }
  if (hd == 32) return dispatch_sp<32>(true, qkv, nullptr, nullptr, nullptr, o, lse, B, S, H, scale, dr, st);
  if (hd == 64) return dispatch_sp<64>(true, qkv, nullptr, nullptr, nullptr, o, lse, B, S, H, scale, dr, st);
  return -1;
}

// dbias_part: optional [B][3*H*hd] fp32 per-sample column sums of dqkv (see attn_bwd_kernel)
int jm_attn_bwd(const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse, uint16_t* dqkv, int B,
                int S, int H, int hd, float* dbias_part, const int64_t* dseed, uint32_t dthr, float dscale,
                hipStream_t st) {
  const float scale = 1.f / sqrtf((float)hd);
  const AttnDrop dr{dseed, dthr, dscale};
  if (hd == 32) return dispatch_sp<32>(false, qkv, o, dO, lse, dqkv, dbias_part, B, S, H, scale, dr, st);
  if (hd == 64) return dispatch_sp<64>(false, qkv, o, dO, lse, dqkv, dbias_part, B, S, H, scale, dr, st);
  return -1;
}

// S > jm_attn_max_seq(): tile-streamed backward; delta = fp32 [B][H][S] workspace.  No fused
// bias colsum on this path (the caller takes colsum(dqkv)).
int jm_attn_bwd_long(const uint16_t* qkv, const uint16_t* o, const uint16_t* dO, const float* lse, uint16_t* dqkv,
                     float* delta, int B, int S, int H, int hd, hipStream_t st) {
  const float scale = 1.f / sqrtf((float)hd);
  if (hd == 32) return run_long_bwd<32>(qkv, o, dO, lse, dqkv, delta, B, S, H, scale, st);
  if (hd == 64) return run_long_bwd<64>(qkv, o, dO, lse, dqkv, delta, B, S, H, scale, st);
  return -1;
}

JM_DEBUG_EXPORT(attention)
