// MFMA GEMM for gfx950 with fused epilogues: C[M, N] = A[M, K] . B[N, K]^T (+ epilogue).
//
// Both operands are K-contiguous ("NT"), which is the layout of every forward Dense of the model
// (activations [tokens, in] x weights [out, in]) and of the data-gradient GEMMs when they are fed
// the transposed bf16 weight shadow.  bf16 in, fp32 accumulate.
//
// Tiling (CDNA4, 64-wide waves): one 512-thread workgroup (8 waves, 2 along M x 4 along N) owns a
// 256 x 256 output tile; each wave a 128 x 64 sub-tile = 8 x 4 v_mfma_f32_16x16x32_bf16 tiles
// (128 accumulator VGPRs).  Operands are staged global -> LDS with buffer_load_dwordx4 ... lds (no
// VGPR round trip).  Two main loops:
//   * p4 (K % 128 == 0, the default): 64-deep K-tiles cut into half-tile LDS slots whose loads stay
//     in flight ACROSS barriers (counted vmcnt), four phases per K-tile (see p4_mainloop);
//   * nt64 (K % 128 == 64, tail-split partial tiles): 64-deep stages through two 64 KB slots.
// MFMA orientation: the B fragment is the MFMA "A" operand, so each lane's accumulator holds four
// consecutive output COLUMNS of one row -- bias / activation / residual epilogues work on float4
// runs.  Epilogues stage the bf16 tile through LDS and stream full 128-byte rows out.
//
// Workgroup -> tile map: bijective XCD remap (consecutive tile ids share an XCD and its L2), then
// groups of 8 row-tiles sweep the column tiles.
//
// Measured and removed (records in profiles/, code in git history): the r1 32-deep ring kernel,
// 4-wave (one wave per SIMD) tiles, 256 x 128 tiles at 2 workgroups per CU (with and without a
// staggered start), persistent launches with the next tile's loads under the epilogue, persistent
// data-parallel + stream-K with in-kernel fix-up, per-phase priority / in-stream glds schedules.
#include <type_traits>

#include "common.h"
#include "jm_api.h"

namespace {

constexpr int BM = 256, BN = 256;
constexpr size_t GEMM_SMEM = 128 * 1024;  // p4: 8 x 16 KB slots; nt64: 2 x 64 KB slots

typedef __attribute__((address_space(3))) void lds_void_t;

// buffer_load_dwordx4 ... lds: 16 B per lane straight into LDS (wave-uniform LDS base + 16 * lane).
// Buffer addressing keeps ONE 32-bit VGPR per load (SGPR base + per-step SGPR offset), and the
// range check zero-fills rows past the operand's end (ragged M / N tiles need no clamping).
JM_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const uint16_t* base, long bytes) {
  const int n = bytes >= 0xffffffffL ? -1 : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, n, 0x00020000);
}

JM_DEVICE void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint16_t* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(l), 16, voff, soff, 0, 0);
}

JM_DEVICE bf16x8_t lds8(const uint16_t* p) { return *reinterpret_cast<const bf16x8_t*>(p); }

JM_DEVICE f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int NTW>
struct Frags {
  bf16x8_t b[NTW], a[8];
};

}  // namespace


// EPI_STORE: out = acc (+bias); EPI_GELU: out = acc (+bias), out2 = gelu(out);
// EPI_DGELU: out = bf16(acc) * gelu'(aux) -- the data gradient through the FF GELU -- with the
// following Dense's bias gradient (column sums of out) as per-tile partials.
// EPI_PARTIAL: split-K -- each (tile, split) workgroup stores its fp32 partial tile; the sum (+bias,
// bf16) is taken by jm_splitk_reduce_bf16.  For small-M, long-K GEMMs (the jumbo MLP: 512 rows,
// K = 12288) whose 24 output tiles would otherwise occupy 24 of 256 CUs.
// EPI_GELU_ONLY: out = gelu(bf16(acc + bias)) alone -- inference (no backward needs the
// pre-activation), half the epilogue bytes of EPI_GELU.
// EPI_TAIL: split-K partial tile of a tail-split launch, stored compact in ep.tail (see GemmEpi).
// EPI_GELU_D: dq = gelu'(h) as 8-bit codes (common.h gd_code), out2 = gelu(h) for h = bf16(acc + bias):
// the FF1 forward saves the GELU derivative for the backward instead of h (one shared exp here, no
// transcendental in the backward epilogue), in 1 byte per element instead of 2.
// EPI_DMUL: out = bf16(acc) * gelu'(h) decoded from dqa, + column partials as EPI_DGELU.
enum { EPI_STORE = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_PARTIAL = 3, EPI_GELU_ONLY = 4, EPI_TAIL = 5, EPI_GELU_D = 6,
       EPI_DMUL = 7 };

namespace {

// FF hidden dropout of the EPI_GELU_D outputs (GemmEpi::dseed): W consecutive elements from flat
// index idx0 (even); gelu(h) times the keep bit / keep, gelu'(h) times the keep bit (its 1 / keep is
// applied when EPI_DMUL decodes the 8-bit code, GemmEpi::dqs, so the code range stays [-0.17, 1.13])
template <int W>
JM_DEVICE void gelu_d_drop(const GemmEpi& ep, long idx0, float* g, float* d) {
  const uint64_t seed = (uint64_t)ep.dseed[0];
#pragma unroll
  for (int j = 0; j < W; j += 2) {
    const uint32_t h = drop_hash((uint32_t)((idx0 + j) >> 1), seed);
    const bool k0 = drop_keep_half(h, 0, ep.dthr), k1 = drop_keep_half(h, 1, ep.dthr);
    g[j] = k0 ? g[j] * ep.dscale : 0.f;
    d[j] = k0 ? d[j] : 0.f;
    g[j + 1] = k1 ? g[j + 1] * ep.dscale : 0.f;
    d[j + 1] = k1 ? d[j + 1] : 0.f;
  }
}

// acc[mt][nt][i] = C[mb + mt*16 + l16][nb + nt*16 + 4g + i]  (mt < MTW)
template <int EPI, int NTW, int MTW = 8>
JM_DEVICE void epilogue(const f32x4_t (&acc)[8][NTW], const GemmEpi& ep, int M, int N, int mb, int nb, int l16,
                        int g) {
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt) {
    const int n = nb + nt * 16 + 4 * g;
    if (n >= N) continue;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (ep.bias) load4(ep.bias + n, bv);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int m = mb + mt * 16 + l16;
      if (m >= M) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[mt][nt][i] + bv[i];
      if (EPI == EPI_GELU_ONLY) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = gelu_tanh_f(bf2f(f2bf(v[i])));
      }
      if (EPI == EPI_GELU_D) {
        float gv[4], dv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) gelu_and_grad_f(bf2f(f2bf(v[i])), gv[i], dv[i]);
        if (ep.dseed) gelu_d_drop<4>(ep, (long)m * ep.ldo + n, gv, dv);
        *reinterpret_cast<uint32_t*>(ep.dq + (long)m * ep.ldo + n) =
            gd_put<3>(dv[3], gd_put<2>(dv[2], gd_put<1>(dv[1], gd_put<0>(dv[0], 0u))));
        store4(ep.out2 + (long)m * ep.ldo + n, gv);
        continue;
      }
      store4(ep.out + (long)m * ep.ldo + n, v);
      if (EPI == EPI_GELU) {
        float gv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) gv[i] = gelu_tanh_f(bf2f(f2bf(v[i])));
        store4(ep.out2 + (long)m * ep.ldo + n, gv);
      }
    }
  }
}

// TR = tile rows (256, or 224 / 192 for the short-row p4 launches, see tile_rows)
template <int BNT = BN, int TR = BM>
JM_DEVICE void tile_of(int M, int N, int GROUP_M, int& m0, int& n0, int splits = 1, int* split = nullptr) {
  const int nM = (M + TR - 1) / TR, nN = (N + BNT - 1) / BNT;
  const int nwg = nM * nN * splits;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  if (split) {  // split-major: concurrently running blocks work on the same K range
    *split = wg / (nM * nN);
    wg -= *split * (nM * nN);
  }
  const int per_group = GROUP_M * nN;
  const int first_m = (wg / per_group) * GROUP_M;
  const int gsz = min(nM - first_m, GROUP_M);
  m0 = (first_m + (wg % per_group) % gsz) * TR;
  n0 = ((wg % per_group) / gsz) * BNT;
}

// tile g (grouped order: GROUP_M row tiles sweep the column tiles) -> (m0, n0)
JM_DEVICE void tile_coords(int g, int M, int N, int GROUP_M, int& m0, int& n0) {
  const int nM = (M + BM - 1) / BM, nN = (N + BN - 1) / BN;
  const int per_group = GROUP_M * nN;
  const int first_m = (g / per_group) * GROUP_M;
  const int gsz = min(nM - first_m, GROUP_M);
  m0 = (first_m + (g % per_group) % gsz) * BM;
  n0 = ((g % per_group) / gsz) * BN;
}

// launch restricted to tiles [t_begin, t_begin + t_count) (x splits, split-major): bijective XCD
// remap over this launch's grid, then the global grouped order
JM_DEVICE void tile_of_range(int M, int N, int GROUP_M, int t_begin, int t_count, int splits, int& m0, int& n0,
                             int& split, int& tg) {
  const int nwg = t_count * splits;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  split = wg / t_count;
  tg = wg - split * t_count;
  tile_coords(t_begin + tg, M, N, GROUP_M, m0, n0);
}

// WN waves along N (2 along M): WN = 4 -> 8 waves of 128 x 64 (2 waves / SIMD);
// WN = 2 -> 4 waves of 128 x 128 (1 wave / SIMD, accumulators in AGPRs)
// Coalesced epilogue through LDS (the staging ring is free once the K loop has drained):
// (1) every wave adds the bias to its accumulators, rounds to bf16 and writes its sub-tile into
//     a [256][256] bf16 image whose 16-byte chunks are XOR-swizzled by (row & 15) -- the
//     ds_write_b64 of 16 rows x 8 B and the ds_read_b128 row reads are both conflict-free;
// (2) the workgroup streams the tile out row by row, 16 B per lane, 512 B per row: full 128 B
//     lines instead of 16 rows x 32 B per store instruction.  GELU is applied in (2) to the
//     rounded pre-activation, which is exactly what the backward will see.
template <typename T>
JM_DEVICE void st16(T* p, uint4 v, bool nts) {
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
  if (nts) __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(p));
  else *reinterpret_cast<uint4*>(p) = v;
}

JM_DEVICE void st8(uint8_t* p, uint2 v, bool nts) {
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
  if (nts) __builtin_nontemporal_store(u32x2_t{v.x, v.y}, reinterpret_cast<u32x2_t*>(p));
  else *reinterpret_cast<uint2*>(p) = v;
}

JM_DEVICE uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack_bf2(f[0], f[1]);
  v.y = pack_bf2(f[2], f[3]);
  v.z = pack_bf2(f[4], f[5]);
  v.w = pack_bf2(f[6], f[7]);
  return v;
}

template <int EPI, int NTW, int NTH, int BNT = BN, bool NTS = false, int TR = BM>
JM_DEVICE void epilogue_lds(const f32x4_t (&acc)[8][NTW], const GemmEpi& ep, uint16_t* cs, int M, int N, int m0,
                            int n0, int wr, int wc, int l16, int g) {
  constexpr int RB = BNT;  // elements per LDS image row
  constexpr int HR = TR / 2, MTW = HR / 16;  // rows and 16-row MFMA tiles per wave row
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  constexpr int LPR = BNT / 8;        // lanes per row (16 B each)
  constexpr int RPP = NTH / LPR;      // rows per pass
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));  // not hoisted out of a persistent kernel's item loop
  const int c = tid % LPR;
  const bool col_ok = n0 + c * 8 < N;
  // EPI_DGELU / EPI_DMUL: the first PF of this thread's aux rows are loaded before the accumulators
  // are staged through LDS (their latency hides behind the staging) and each row pass then issues
  // the load PF passes ahead -- a register ring instead of one exposed load per pass
  constexpr bool PRE = EPI == EPI_DGELU || EPI == EPI_DMUL;
  constexpr int NPASS = PRE ? TR / RPP : 1;
  constexpr int PF = NPASS < 8 ? NPASS : 8;
  uint4 auxv[PF];
  auto aux_load = [&](int i) {
    const int m = m0 + tid / LPR + i * RPP;
    uint4 a = make_uint4(0, 0, 0, 0);
    if (m < M && col_ok) {
      if constexpr (EPI == EPI_DMUL) {  // 8 gelu' codes
        const uint2 q = *reinterpret_cast<const uint2*>(ep.dqa + (long)m * ep.ldo + n0 + c * 8);
        a.x = q.x;
        a.y = q.y;
      } else {
        a = *reinterpret_cast<const uint4*>(ep.aux + (long)m * ep.ldo + n0 + c * 8);
      }
    }
    return a;
  };
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < PF; ++i) auxv[i] = aux_load(i);
  }
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt) {
    const int nl = wc * NTW * 16 + nt * 16 + 4 * g;  // tile-local column
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (ep.bias && n0 + nl < N) load4(ep.bias + n0 + nl, bv);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int r = wr * HR + mt * 16 + l16;
      uint2 pk;
      pk.x = pack_bf2(acc[mt][nt][0] + bv[0], acc[mt][nt][1] + bv[1]);
      pk.y = pack_bf2(acc[mt][nt][2] + bv[2], acc[mt][nt][3] + bv[3]);
      const int chunk = (nl >> 3) ^ (r & 15);
      *reinterpret_cast<uint2*>(cs + r * RB + chunk * 8 + (nl & 7)) = pk;
    }
  }
  __syncthreads();
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // one row pass: row r of the tile; av = the prefetched aux row (PRE epilogues)
  auto pass = [&](int r, const uint4& av) {
    const int m = m0 + r;
    const uint4 v = *reinterpret_cast<const uint4*>(cs + r * RB + ((c ^ (r & 15)) << 3));
    if (m < M && col_ok) {
      if (EPI == EPI_DGELU || EPI == EPI_DMUL) {
        float f[8], hp[8], gd[8];
        const uint16_t* dg = reinterpret_cast<const uint16_t*>(&v);
        if constexpr (EPI == EPI_DMUL) {
          gd_unpack4(av.x, ep.dqs, hp);
          gd_unpack4(av.y, ep.dqs, hp + 4);
        } else {
          const uint16_t* ah = reinterpret_cast<const uint16_t*>(&av);
#pragma unroll
          for (int j = 0; j < 8; ++j) hp[j] = bf2f(ah[j]);
          gelu_n<8, false, true>(hp, nullptr, gd);
        }
        // round the products to bf16 once (one v_cvt_pk_bf16_f32 per pair), then the column sums
        // read the rounded values back from the packed words (shift / mask) -- the epilogue is
        // VALU-issue bound, a second conversion per pair for the store cost issue slots
        uint4 o;
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const float a0 = bf2f(dg[j]) * (EPI == EPI_DMUL ? hp[j] : gd[j]);
          const float a1 = bf2f(dg[j + 1]) * (EPI == EPI_DMUL ? hp[j + 1] : gd[j + 1]);
          ow[j / 2] = pack_bf2(a0, a1);
          f[j] = __uint_as_float(ow[j / 2] << 16);
          f[j + 1] = __uint_as_float(ow[j / 2] & 0xffff0000u);
          csum[j] += f[j];
          csum[j + 1] += f[j + 1];
        }
        st16(ep.out + (long)m * ep.ldo + n0 + c * 8, o, NTS);
      } else if (EPI == EPI_GELU_D) {
        float fh[8], fg[8], fd[8];
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) fh[j] = bf2f(h[j]);
        gelu_n<8, true, true>(fh, fg, fd);
        if (ep.dseed) gelu_d_drop<8>(ep, (long)m * ep.ldo + n0 + c * 8, fg, fd);
        st8(ep.dq + (long)m * ep.ldo + n0 + c * 8, gd_pack8(fd), NTS);
        st16(ep.out2 + (long)m * ep.ldo + n0 + c * 8, pack8(fg), NTS);
      } else if (EPI == EPI_GELU_ONLY) {
        float fh[8], f[8];
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) fh[j] = bf2f(h[j]);
        gelu_n<8, true, false>(fh, f, nullptr);
        st16(ep.out + (long)m * ep.ldo + n0 + c * 8, pack8(f), NTS);
      } else {
        st16(ep.out + (long)m * ep.ldo + n0 + c * 8, v, NTS);
      }
      if (EPI == EPI_GELU) {
        float fh[8], f[8];
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) fh[j] = bf2f(h[j]);
        gelu_n<8, true, false>(fh, f, nullptr);
        st16(ep.out2 + (long)m * ep.ldo + n0 + c * 8, pack8(f), NTS);
      }
    }
  };
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      pass(tid / LPR + i * RPP, auxv[i % PF]);
      if (i + PF < NPASS) auxv[i % PF] = aux_load(i + PF);
    }
  } else {
#pragma unroll 4
    for (int r = tid / LPR; r < TR; r += RPP) pass(r, auxv[0]);
  }
  if ((EPI == EPI_DGELU || EPI == EPI_DMUL) && ep.colpart != nullptr) {
    // column sums of this row tile: RPP threads share a column chunk -> reduce through LDS
    float* red = reinterpret_cast<float*>(cs);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = csum[j];
    __syncthreads();
    for (int col = tid; col < BNT; col += NTH) {
      const int cc = col >> 3, j = col & 7;
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < RPP; ++q) acc += red[(cc + q * LPR) * 8 + j];
      if (n0 + col < N) ep.colpart[(long)(m0 / TR) * N + n0 + col] = acc;
    }
  }
}


// ------------------------------------------------------------------ 128-byte-row variant
// Same tile, waves and epilogues as gemm_nt_kernel, but K is staged 64 deep: every operand row of
// a stage is 128 contiguous bytes, so each global_load_lds piece maps to full 128 B L2 requests
// (the 64 B rows of the 32-deep ring issue twice the requests for the same bytes).  Two 64 KB
// slots (the LDS budget), one barrier per 64-deep stage placed in the middle of its second half:
//   half A: MFMAs of k 0-31 (registers), reads of k 32-63 of the same slot beside them;
//   half B: MFMAs of k 32-63 rows 0-3 | vmcnt(0) + barrier (stage u+1 landed, slot u free) |
//           issue stage u+2 into slot u, reads of stage u+1's k 0-31 beside rows 4-7.
// Chunks of a 128 B row are XOR-swizzled by (row >> 1) & 7: conflict-free ds_read_b128 for both
// halves (brute-forced over the four lane groups).
JM_DEVICE int swz64(int row) { return (row >> 1) & 7; }

template <int EPI, bool NTS>
__attribute__((always_inline)) JM_DEVICE void nt64_body(const uint16_t* __restrict__ A, long lda,
                                                        const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                        int K, const GemmEpi& ep, int GROUP_M, uint16_t* smem) {
  constexpr int NW = 8, NTW = 4, BK2 = 64;
  constexpr int STG = (BM + BN) * BK2;  // elements per slot: 64 KB

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const int wr = wave >> 2, wc = wave & 3;

  int m0, n0, split = 0, tg = 0;
  if (ep.t_count > 0)
    tile_of_range(M, N, GROUP_M, ep.t_begin, ep.t_count, EPI == EPI_TAIL ? ep.tail_S : 1, m0, n0, split, tg);
  else
    tile_of(M, N, GROUP_M, m0, n0, EPI == EPI_PARTIAL ? ep.splits : 1, EPI == EPI_PARTIAL ? &split : nullptr);
  int k_begin = 0;
  if (EPI == EPI_PARTIAL || EPI == EPI_TAIL) {
    const int ns = EPI == EPI_TAIL ? ep.tail_S : ep.splits;
    const int ku = K / 64;
    const int ku0 = split * ku / ns, ku1 = (split + 1) * ku / ns;
    k_begin = ku0 * 64;
    K = (ku1 - ku0) * 64;
  }
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A + (long)m0 * lda + k_begin, (long)(M - m0) * lda * 2 - 2L * k_begin);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B + (long)n0 * ldb + k_begin, (long)(N - n0) * ldb * 2 - 2L * k_begin);
  // one glds piece = 8 rows x 128 B; per operand and stage 32 pieces, 4 per wave
  uint32_t a_src[4], b_src[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = rr * 64 + wave * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz64(row);
    a_src[rr] = (uint32_t)((row * lda + c * 8) * 2);
    b_src[rr] = (uint32_t)((row * ldb + c * 8) * 2);
  }
  auto issue = [&](int u) {
    const uint32_t k0b = u * BK2 * 2;
    uint16_t* la = smem + (u & 1) * STG;
    uint16_t* lb = la + BM * BK2;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      blds16(ra, a_src[rr], k0b, la + (rr * 64 + wave * 8) * BK2);
      blds16(rb, b_src[rr], k0b, lb + (rr * 64 + wave * 8) * BK2);
    }
  };
  const int ch0 = ((0 * 4 + g) ^ swz64(l16)) * 8, ch1 = ((1 * 4 + g) ^ swz64(l16)) * 8;
  const int a_row = (wr * 128 + l16) * BK2, b_row = BM * BK2 + (wc * 64 + l16) * BK2;
  auto read = [&](int u, auto half, Frags<NTW>& f) {
    const int ch = decltype(half)::value ? ch1 : ch0;
    const uint16_t* base = smem + (u & 1) * STG;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) f.b[nt] = lds8(base + b_row + nt * 16 * BK2 + ch);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) f.a[mt] = lds8(base + a_row + mt * 16 * BK2 + ch);
  };
  f32x4_t acc[8][NTW];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto mfma_rows = [&](auto lo, const Frags<NTW>& f) {
    constexpr int R0 = decltype(lo)::value;
#pragma unroll
    for (int mt = R0; mt < R0 + 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) acc[mt][nt] = mfma16(f.b[nt], f.a[mt], acc[mt][nt]);
  };
  auto interleave = [&]() {  // 12 reads beside 16 MFMAs
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  };
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;
  using R0 = std::integral_constant<int, 0>;
  using R4 = std::integral_constant<int, 4>;
  // KIND 2: steady (issue u + 2), 1: stage u + 1 exists but nothing left to issue, 0: last stage
  auto stage = [&](auto kind, int u, Frags<NTW>& f0, Frags<NTW>& f1) {
    constexpr int KIND = decltype(kind)::value;
    mfma_rows(R0{}, f0);
    __builtin_amdgcn_sched_barrier(0);
    read(u, H1{}, f1);
    mfma_rows(R4{}, f0);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    mfma_rows(R0{}, f1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (KIND > 0) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (KIND == 2) issue(u + 2);
      read(u + 1, H0{}, f0);
      mfma_rows(R4{}, f1);
      interleave();
    } else {
      mfma_rows(R4{}, f1);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using K2 = std::integral_constant<int, 2>;
  using K1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;

  const int nst = K / BK2;  // >= 1 (host checks K % 64 == 0)
  issue(0);
  if (nst > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0);
  Frags<NTW> f0, f1;
  read(0, H0{}, f0);
  int u = 0;
  for (; u + 2 < nst; ++u) stage(K2{}, u, f0, f1);
  if (u + 1 < nst) stage(K1{}, u++, f0, f1);
  stage(K0{}, u, f0, f1);

  if (EPI == EPI_TAIL) {  // compact fp32 partial tile: tail[split][tg][256][256] (rows past M unused)
    float* dst = ep.tail + ((long)split * ep.t_count + tg) * (BM * BN);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int ml = wr * 128 + mt * 16 + l16;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int nl = wc * NTW * 16 + nt * 16 + 4 * g;
        float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
        store4(dst + ml * BN + nl, v);
      }
    }
  } else if (EPI == EPI_PARTIAL) {
    float* dst = ep.part + (long)split * M * N;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int m = m0 + wr * 128 + mt * 16 + l16;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n = n0 + wc * NTW * 16 + nt * 16 + 4 * g;
        if (n >= N) continue;
        float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
        store4(dst + (long)m * N + n, v);
      }
    }
  } else if (N % 8 == 0)
    epilogue_lds<EPI, NTW, 512, BN, NTS>(acc, ep, smem, M, N, m0, n0, wr, wc, l16, g);
  else
    epilogue<EPI, NTW>(acc, ep, M, N, m0 + wr * 128, n0 + wc * NTW * 16, l16, g);
}

template <int EPI, bool NTS>
__global__ __launch_bounds__(512, 1) void gemm_nt64_kernel(const uint16_t* __restrict__ A, long lda,
                                                           const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                           int K, GemmEpi ep, int GROUP_M) {
  JM_DGUARD(blockDim.x == 512 && K % 64 == 0 && M > 0 && N > 0);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  nt64_body<EPI, NTS>(A, lda, B, ldb, M, N, K, ep, GROUP_M, smem);
}

// ------------------------------------------------------------------ 4-phase counted-vmcnt variant
// Same 256 x 256 tile, 8 waves (2 x 4, 128 x 64 each) and epilogues as nt64_body; the K loop is
// cut into half-tile LDS slots so that loads stay in flight ACROSS barriers (counted vmcnt, never
// 0 in steady state) instead of draining every stage:
//   * a K-tile (64 deep) is 4 slots of 128 rows x 128 B: a0 / a1 = the A rows of the waves' upper
//     / lower 64-row halves (rows wr*128 + mh*64 + [0,64) for both wr), b0 / b1 = the B rows of the
//     waves' left / right 32-column halves (wc*64 + nh*32 + [0,32) for all wc);
//   * 8 slots = two K-tiles in LDS (128 KB); each wave runs 4 phases per K-tile, one 64 x 32
//     quadrant (mh, nh) x K = 64 = 16 MFMAs each, in the order (0,0) (0,1) (1,1) (1,0), so a
//     phase needs at most one new operand half;
//   * fragments are read one phase ahead of their MFMAs (registers: A_X/A_Y, two B sets whose
//     roles swap every K-tile -- hence 2 K-tiles per loop trip): q4 reads a0,b0 of the next
//     tile, q1 reads b1, q2 reads a1, q3 reads nothing;
//   * every phase starts with [vmcnt(N) lgkmcnt(0) s_barrier] and then issues ONE slot load (2
//     glds per thread) for the tile after next: q1 a0, q2 b1, q3 a1, q4 b0 -- each slot is
//     refilled the phase after its last read, A slots 7 phases and b0 (weights, L2-resident) 4
//     phases before they are read;
//   * N per phase start (loads issued after the one that must have landed): q1 12, q2 12, q3 none,
//     q4 6; the last two K-tiles issue nothing and count down (12 10 - 0 | 4 2 - -).
// Slot rows are 128 B; 16-B chunks XOR-swizzled by swz64(slot row) on the per-lane global source
// and on the ds_read address (conflict-free ds_read_b128, the nt64 image).
// Waves 4-7 (the younger half, SIMD partners of waves 0-3) run at priority 1 throughout (static
// young-half priority, MI355X_MICROARCH.md "Two waves per SIMD" item 4; profiles/r2_gemm_p4.txt).
// acc = A[m0:m0+TR, k_begin:k_begin+K] . B[n0:n0+256, same]^T  (K % 128 == 0, K > 0); every LDS
// slot is free on entry (caller's barrier) and the ring is drained on exit except for the reads
// of the last K-tile's MFMAs (caller's epilogue barriers before reusing LDS).
// Short-row tiles (MTL < 4: TR = 128 + 32 * MTL = 224 / 192 / 160 rows) keep the slot layout and the
// counted-vmcnt schedule unchanged: each wave row owns 64 + 16 * MTL rows, the a1 slot's unused
// rows are loaded from an out-of-range buffer offset (no memory traffic) and never read, and the
// lower-half phases q3 / q4 run MTL instead of 4 row MFMA tiles.  They exist for wave fill
// (tile_rows): e.g. M = 25088, N = 4096 is 6.1 waves of 256-row tiles but exactly 7 of 224.
template <int MTL>
__attribute__((always_inline)) JM_DEVICE void p4_mainloop(const uint16_t* __restrict__ A, long lda,
                                                          const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                          int m0, int n0, int k_begin, int K,
                                                          f32x4_t (&acc)[8][4], uint16_t* smem) {
  // 2 x 4 waves of 128 x 64 (2 waves / SIMD)
  constexpr int WN = 4;               // waves along N
  constexpr int QC = 128 / WN;        // columns of a wave's quadrant (32)
  constexpr int NTQ = QC / 16;        // 16-wide n tiles per quadrant (2)
  constexpr int NTW = 2 * NTQ;        // per wave (4)
  constexpr int P = 2;                // glds pieces per wave and slot
  constexpr int BK2 = 64, SLOT = 128 * BK2;  // elements per slot (16 KB)
  constexpr int HR = 64 + 16 * MTL;   // tile rows per wave row
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const int wr = wave / WN, wc = wave % WN;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A + (long)m0 * lda + k_begin, (long)(M - m0) * lda * 2 - 2L * k_begin);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B + (long)n0 * ldb + k_begin, (long)(N - n0) * ldb * 2 - 2L * k_begin);
  // glds pieces: slot rows q*8 + (lane >> 3), q = P * wave + r; slot row -> tile row / column
  uint32_t a_src[2][P], b_src[2][P];  // [half][r] byte offsets
#pragma unroll
  for (int r = 0; r < P; ++r) {
    const int srow = (P * wave + r) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz64(srow);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int arow = (srow >> 6) * HR + h * 64 + (srow & 63);
      const int bcol = (srow / QC) * (2 * QC) + h * QC + (srow % QC);
      const bool aok = h == 0 || (srow & 63) < 16 * MTL;  // host: A bytes < 2^31 (offset out of range)
      a_src[h][r] = aok ? (uint32_t)((arow * lda + c * 8) * 2) : 0x80000000u;
      b_src[h][r] = (uint32_t)((bcol * ldb + c * 8) * 2);
    }
  }
  // slot index within a K-tile set: 0 = a0, 1 = a1, 2 = b0, 3 = b1
  auto issue = [&](int t, auto slot) {
    constexpr int S = decltype(slot)::value;
    const uint32_t k0b = t * BK2 * 2;
    uint16_t* l = smem + ((t & 1) * 4 + S) * SLOT + (P * wave) * 8 * BK2;
#pragma unroll
    for (int r = 0; r < P; ++r) {
      if constexpr (S < 2) blds16(ra, a_src[S][r], k0b, l + r * 8 * BK2);
      else blds16(rb, b_src[S - 2][r], k0b, l + r * 8 * BK2);
    }
  };
  const int ch0 = ((0 * 4 + g) ^ swz64(l16)) * 8, ch1 = ((1 * 4 + g) ^ swz64(l16)) * 8;
  const int a_row = (wr * 64 + l16) * BK2, b_row = (wc * QC + l16) * BK2;
  typedef bf16x8_t AF[4][2];    // [mt within the half][k32 step]
  typedef bf16x8_t BF[NTQ][2];  // [nt within the half][k32 step]
  auto read_a = [&](int t, auto half, AF& f) {
    constexpr int NMT = decltype(half)::value ? MTL : 4;
    const uint16_t* base = smem + ((t & 1) * 4 + decltype(half)::value) * SLOT + a_row;
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) {
      f[mt][0] = lds8(base + mt * 16 * BK2 + ch0);
      f[mt][1] = lds8(base + mt * 16 * BK2 + ch1);
    }
  };
  auto read_b = [&](int t, auto half, BF& f) {
    const uint16_t* base = smem + ((t & 1) * 4 + 2 + decltype(half)::value) * SLOT + b_row;
#pragma unroll
    for (int nt = 0; nt < NTQ; ++nt) {
      f[nt][0] = lds8(base + nt * 16 * BK2 + ch0);
      f[nt][1] = lds8(base + nt * 16 * BK2 + ch1);
    }
  };
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto mfma_q = [&](auto mh, auto nh, const AF& a, const BF& b) {
    constexpr int MH = decltype(mh)::value, NH = decltype(nh)::value;
    constexpr int NMT = MH ? MTL : 4;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTQ; ++nt)
          acc[MH * 4 + mt][NH * NTQ + nt] = mfma16(b[nt][kk], a[mt][kk], acc[MH * 4 + mt][NH * NTQ + nt]);
  };
  // vmcnt(n * P) lgkmcnt(0) s_barrier (n in phase units of P glds); n < 0: no vmcnt wait
  auto sync = [&](auto n) {
    constexpr int V = decltype(n)::value * P;
    if constexpr (V >= 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(V) : "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // the phase's instruction order: its NR ds_reads spread evenly over its NM MFMAs
  auto interleave = [&](auto nreads, auto mh) {
    constexpr int NM = (decltype(mh)::value ? MTL : 4) * 2 * NTQ;
    constexpr int NR = decltype(nreads)::value;
    constexpr int PER = NR >= NM ? 1 : NM / (NR > 0 ? NR : 1);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (i % PER == 0 && i / PER < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I5 = std::integral_constant<int, 5>;
  using I6 = std::integral_constant<int, 6>;
  using I8 = std::integral_constant<int, 8>;
  using IN = std::integral_constant<int, -1>;
  using RB = std::integral_constant<int, 2 * NTQ>;      // fragment reads of a B half
  using RQ4 = std::integral_constant<int, 8 + 2 * NTQ>;  // q4: a0 + b0 of the next tile
  using RA1 = std::integral_constant<int, 2 * MTL>;      // q2: a1

  AF ax, ay;
  BF bp, bq;
  // one K-tile: b0 holds its b0 fragments (read during the previous tile's q4), b1 receives b1 and
  // then the next tile's b0.  KIND 2 = steady (issues tile t + 2), 1 = next-to-last, 0 = last.
  // Counted waits (phases of P glds issued after the one that must have landed): q1 6, q2 6,
  // q3 none, q4 3; next-to-last 6 5 - 0; last 2 1 - -.
  auto tile = [&](auto kind, int t, BF& b0, BF& b1) {
    constexpr int KIND = decltype(kind)::value;
    // q1 (0,0): read b1(t)
    sync(std::conditional_t<KIND == 0, I2, I6>{});
    if constexpr (KIND == 2) issue(t + 2, I0{});
    read_b(t, I1{}, b1);
    mfma_q(I0{}, I0{}, ax, b0);
    interleave(RB{}, I0{});
    // q2 (0,1): read a1(t)
    sync(std::conditional_t<KIND == 0, I1, std::conditional_t<KIND == 1, I5, I6>>{});
    if constexpr (KIND == 2) issue(t + 2, I3{});
    read_a(t, I1{}, ay);
    mfma_q(I0{}, I1{}, ax, b1);
    interleave(RA1{}, I0{});
    // q3 (1,1): no reads
    sync(IN{});
    if constexpr (KIND == 2) issue(t + 2, I1{});
    mfma_q(I1{}, I1{}, ay, b1);
    interleave(I0{}, I1{});
    // q4 (1,0): read a0(t+1), b0(t+1) (into b1, free after q3)
    if constexpr (KIND > 0) {
      sync(std::conditional_t<KIND == 1, I0, I3>{});
        if constexpr (KIND == 2) issue(t + 2, I2{});
      read_a(t + 1, I0{}, ax);
      read_b(t + 1, I0{}, b1);
      mfma_q(I1{}, I0{}, ay, b0);
      interleave(RQ4{}, I1{});
      } else {
      mfma_q(I1{}, I0{}, ay, b0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using K2 = std::integral_constant<int, 2>;
  using K1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;

  const int nk = K / BK2;  // even, >= 2
  // prologue: tiles 0 and 1 in the steady-state issue order (a0 b1 a1 | b0), so the counted
  // waits of the first tiles hold unchanged
  issue(0, I0{});
  issue(0, I3{});
  issue(0, I1{});
  issue(0, I2{});
  issue(1, I0{});
  issue(1, I3{});
  issue(1, I1{});
  sync(I3{});
  issue(1, I2{});
  read_a(0, I0{}, ax);
  read_b(0, I0{}, bp);
  int t = 0;
  for (; t + 4 <= nk; t += 2) {  // tiles t, t+1 with t + 3 < nk: both steady
    tile(K2{}, t, bp, bq);
    tile(K2{}, t + 1, bq, bp);
  }
  // nk - t == 2: the last two tiles (nk - 2 -> KIND 1, nk - 1 -> KIND 0)
  tile(K1{}, t, bp, bq);
  tile(K0{}, t + 1, bq, bp);
}

// the 256 x 256 tile's epilogue from the p4 accumulators (EPI_PARTIAL: fp32 split slice)
template <int EPI, int MTL>
__attribute__((always_inline)) JM_DEVICE void p4_epilogue(const f32x4_t (&acc)[8][4], const GemmEpi& ep, int M,
                                                          int N, int m0, int n0, int split, uint16_t* smem) {
  constexpr int NTW = 4, WN = 4;
  constexpr int HR = 64 + 16 * MTL, MTW = 4 + MTL;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const int wr = wave / WN, wc = wave % WN;
  if (EPI == EPI_PARTIAL) {
    float* dst = ep.part + (long)split * M * N;
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
      const int m = m0 + wr * HR + mt * 16 + l16;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n = n0 + wc * NTW * 16 + nt * 16 + 4 * g;
        if (n >= N) continue;
        float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
        store4(dst + (long)m * N + n, v);
      }
    }
  } else if (N % 8 == 0)
    epilogue_lds<EPI, NTW, 512, BN, true, 2 * HR>(acc, ep, smem, M, N, m0, n0, wr, wc, l16, g);
  else
    epilogue<EPI, NTW, MTW>(acc, ep, M, N, m0 + wr * HR, n0 + wc * NTW * 16, l16, g);
}

template <int EPI, int MTL = 4>
__global__ __launch_bounds__(512, 1) void gemm_p4_kernel(const uint16_t* __restrict__ A, long lda,
                                                         const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                         int K, GemmEpi ep, int GROUP_M) {
  JM_DGUARD(blockDim.x == 512 && K % 128 == 0 && M > 0 && N > 0);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);  // young half
  int m0, n0, split = 0;
  if (EPI != EPI_PARTIAL && ep.t_count > 0) {  // main part of a tail-split launch: tiles [t_begin, +t_count)
    int tg;
    tile_of_range(M, N, GROUP_M, ep.t_begin, ep.t_count, 1, m0, n0, split, tg);
  } else {
    tile_of<BN, 128 + 32 * MTL>(M, N, GROUP_M, m0, n0, EPI == EPI_PARTIAL ? ep.splits : 1,
                                EPI == EPI_PARTIAL ? &split : nullptr);
  }
  int k_begin = 0;
  if (EPI == EPI_PARTIAL) {
    const int ku = K / 128;  // splits take whole 128-deep units (even tile count per split)
    const int ku0 = split * ku / ep.splits, ku1 = (split + 1) * ku / ep.splits;
    k_begin = ku0 * 128;
    K = (ku1 - ku0) * 128;
  }
  f32x4_t acc[8][4];
  p4_mainloop<MTL>(A, lda, B, ldb, M, N, m0, n0, k_begin, K, acc, smem);
  p4_epilogue<EPI, MTL>(acc, ep, M, N, m0, n0, split, smem);
}

// ------------------------------------------------------------------ narrow tiles (M < 4096)
// Skinny-M GEMMs -- the shared jumbo MLP (512 rows per GPU in pretraining, 128 in finetuning),
// the classifier head, small batches -- get too few 256 x 256 tiles to fill 256 CUs.  Here one
// 512-thread workgroup owns a 128 x 192 tile: 8 waves, 2 along M x 4 along N, each 64 x 48 =
// 4 x 3 v_mfma_f32_16x16x32_bf16 tiles (48 accumulator VGPRs).  M = 512, N = 12288 (the jumbo
// W1 forward / W2 data gradient, K = 3072) is then exactly 4 x 64 = 256 tiles: one full wave.
// K moves in 64-deep K-tiles (A 128 x 128 B + B 192 x 128 B = 40 KB) through a 3-slot LDS ring
// by buffer_load ... lds with the nt64 chunk swizzle; one barrier per K-tile, the next-but-one
// K-tile issued right after it (counted vmcnt keeps one K-tile in flight across the barrier).
// Epilogues: the tile is staged as bf16 through a padded LDS image ([128][200]: conflict-free
// 8-byte writes) and streamed out 16 B per lane by 384 threads (24 per row, 16 rows per pass),
// each on fixed columns, so the DGELU / DMUL column sums stay in registers until one LDS reduce.
// EPI_PARTIAL: split-K fp32 slices straight from the accumulators.
constexpr int NBM = 128, NBN = 192, NKT = 64;
constexpr int N_AEL = NBM * NKT, N_BEL = NBN * NKT, N_STAGE = N_AEL + N_BEL;  // elements (40 KB / K-tile)
constexpr int N_RING = 3;
constexpr int N_LD = NBN + 8;  // epilogue image row stride (elements)
static_assert(N_RING * N_STAGE * 2 <= (int)GEMM_SMEM, "narrow ring exceeds the LDS budget");

// bijective XCD remap, split-major, then GROUP_M row tiles sweep the column tiles
JM_DEVICE void narrow_tile(int M, int N, int GROUP_M, int splits, int& m0, int& n0, int& split) {
  const int nM = (M + NBM - 1) / NBM, nN = (N + NBN - 1) / NBN;
  const int tiles = nM * nN, nwg = tiles * splits;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  split = wg / tiles;
  wg -= split * tiles;
  const int per_group = GROUP_M * nN;
  const int first_m = (wg / per_group) * GROUP_M;
  const int gsz = min(nM - first_m, GROUP_M);
  m0 = (first_m + (wg % per_group) % gsz) * NBM;
  n0 = ((wg % per_group) / gsz) * NBN;
}

template <int EPI>
JM_DEVICE void narrow_epilogue(const f32x4_t (&acc)[4][3], const GemmEpi& ep, uint16_t* cs, int M, int N, int m0,
                               int n0, int split, int wr, int wc, int l16, int g) {
  if constexpr (EPI == EPI_PARTIAL) {
    float* dst = ep.part + (long)split * M * N;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int m = m0 + wr * 64 + mt * 16 + l16;
      if (m >= M) continue;
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) {
        const int n = n0 + wc * 48 + nt * 16 + 4 * g;
        if (n >= N) continue;
        float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
        store4(dst + (long)m * N + n, v);
      }
    }
    return;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // ring drained and free
#pragma unroll
  for (int nt = 0; nt < 3; ++nt) {
    const int nl = wc * 48 + nt * 16 + 4 * g;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (ep.bias && n0 + nl < N) load4(ep.bias + n0 + nl, bv);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int r = wr * 64 + mt * 16 + l16;
      uint2 pk;
      pk.x = pack_bf2(acc[mt][nt][0] + bv[0], acc[mt][nt][1] + bv[1]);
      pk.y = pack_bf2(acc[mt][nt][2] + bv[2], acc[mt][nt][3] + bv[3]);
      *reinterpret_cast<uint2*>(cs + r * N_LD + nl) = pk;
    }
  }
  __syncthreads();
  const int tid = threadIdx.x;
  constexpr bool PRE = EPI == EPI_DGELU || EPI == EPI_DMUL;
  const bool active = tid < 384;
  const int c = tid % 24, rr = tid / 24;  // column chunk, first row (active threads: rr < 16)
  const int n = n0 + c * 8;
  const bool col_ok = active && n < N;
  uint4 auxv[8];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + rr + 16 * i;
      auxv[i] = make_uint4(0, 0, 0, 0);
      if (col_ok && m < M) {
        if constexpr (EPI == EPI_DMUL) {  // 8 gelu' codes
          const uint2 q = *reinterpret_cast<const uint2*>(ep.dqa + (long)m * ep.ldo + n);
          auxv[i].x = q.x;
          auxv[i].y = q.y;
        } else {
          auxv[i] = *reinterpret_cast<const uint4*>(ep.aux + (long)m * ep.ldo + n);
        }
      }
    }
  }
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = rr + 16 * i, m = m0 + r;
      if (m >= M || !col_ok) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(cs + r * N_LD + c * 8);
      uint16_t* o = ep.out + (long)m * ep.ldo + n;
      const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
      if constexpr (PRE) {
        float f[8], hp[8], gd[8];
        if constexpr (EPI == EPI_DMUL) {
          gd_unpack4(auxv[i].x, ep.dqs, hp);
          gd_unpack4(auxv[i].y, ep.dqs, hp + 4);
        } else {
          const uint16_t* ah = reinterpret_cast<const uint16_t*>(&auxv[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) hp[j] = bf2f(ah[j]);
          gelu_n<8, false, true>(hp, nullptr, gd);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          f[j] = bf2f(f2bf(bf2f(h[j]) * (EPI == EPI_DMUL ? hp[j] : gd[j])));
          csum[j] += f[j];
        }
        st16(o, pack8(f), false);
      } else if constexpr (EPI == EPI_GELU_D) {
        float fh[8], fg[8], fd[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) fh[j] = bf2f(h[j]);
        gelu_n<8, true, true>(fh, fg, fd);
        if (ep.dseed) gelu_d_drop<8>(ep, (long)m * ep.ldo + n, fg, fd);
        st8(ep.dq + (long)m * ep.ldo + n, gd_pack8(fd), false);
        st16(ep.out2 + (long)m * ep.ldo + n, pack8(fg), false);
      } else if constexpr (EPI == EPI_GELU_ONLY) {
        float fh[8], f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) fh[j] = bf2f(h[j]);
        gelu_n<8, true, false>(fh, f, nullptr);
        st16(o, pack8(f), false);
      } else {
        st16(o, v, false);
        if constexpr (EPI == EPI_GELU) {
          float fh[8], f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) fh[j] = bf2f(h[j]);
          gelu_n<8, true, false>(fh, f, nullptr);
          st16(ep.out2 + (long)m * ep.ldo + n, pack8(f), false);
        }
      }
    }
  }
  if constexpr (PRE) {
    if (ep.colpart != nullptr) {  // column sums of this row tile: 16 row threads per column chunk
      float* red = reinterpret_cast<float*>(cs);
      __syncthreads();
      if (active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[rr * NBN + c * 8 + j] = csum[j];
      }
      __syncthreads();
      if (tid < NBN && n0 + tid < N) {
        float a = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) a += red[q * NBN + tid];
        ep.colpart[(long)(m0 / NBM) * N + n0 + tid] = a;
      }
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_narrow_kernel(const uint16_t* __restrict__ A, long lda,
                                                             const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                             int K, GemmEpi ep, int GROUP_M) {
  JM_DGUARD(blockDim.x == 512 && K % 64 == 0 && M > 0 && N > 0 && N % 8 == 0);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const int wr = wave >> 2, wc = wave & 3;
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // static young-half priority (as p4)
  int m0, n0, split;
  narrow_tile(M, N, GROUP_M, EPI == EPI_PARTIAL ? ep.splits : 1, m0, n0, split);
  int k_begin = 0;
  if (EPI == EPI_PARTIAL) {  // this split's K range, in units of 64
    const int ku = K / 64;
    const int ku0 = split * ku / ep.splits, ku1 = (split + 1) * ku / ep.splits;
    k_begin = ku0 * 64;
    K = (ku1 - ku0) * 64;
  }
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A + (long)m0 * lda + k_begin, (long)(M - m0) * lda * 2 - 2L * k_begin);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B + (long)n0 * ldb + k_begin, (long)(N - n0) * ldb * 2 - 2L * k_begin);
  // glds pieces of 8 rows x 128 B: A rows (wave + 8 p) * 8 + lane / 8 (p < 2), B rows (p < 3)
  uint32_t a_src[2], b_src[3];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int row = (wave + 8 * p) * 8 + (lane >> 3);
    a_src[p] = (uint32_t)((row * lda + ((lane & 7) ^ swz64(row)) * 8) * 2);
  }
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    const int row = (wave + 8 * p) * 8 + (lane >> 3);
    b_src[p] = (uint32_t)((row * ldb + ((lane & 7) ^ swz64(row)) * 8) * 2);
  }
  auto issue = [&](int t) {
    const uint32_t k0b = t * NKT * 2;
    uint16_t* la = smem + (t % N_RING) * N_STAGE;
    uint16_t* lb = la + N_AEL;
#pragma unroll
    for (int p = 0; p < 2; ++p) blds16(ra, a_src[p], k0b, la + (wave + 8 * p) * 8 * NKT);
#pragma unroll
    for (int p = 0; p < 3; ++p) blds16(rb, b_src[p], k0b, lb + (wave + 8 * p) * 8 * NKT);
  };
  const int ch0 = ((0 * 4 + g) ^ swz64(l16)) * 8, ch1 = ((1 * 4 + g) ^ swz64(l16)) * 8;
  const int a_row = (wr * 64 + l16) * NKT, b_row = N_AEL + (wc * 48 + l16) * NKT;
  f32x4_t acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = K / NKT;  // >= 1
  issue(0);
  if (nk > 1) issue(1);
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + 2 < nk) issue(t + 2);  // slot (t + 2) % 3 was read in step t - 1: every wave is past it
    const uint16_t* base = smem + (t % N_RING) * N_STAGE;
    bf16x8_t a[4][2], b[3][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk ? ch1 : ch0;
#pragma unroll
      for (int nt = 0; nt < 3; ++nt) b[nt][kk] = lds8(base + b_row + nt * 16 * NKT + ch);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) a[mt][kk] = lds8(base + a_row + mt * 16 * NKT + ch);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) acc[mt][nt] = mfma16(b[nt][kk], a[mt][kk], acc[mt][nt]);
    // 7 reads of k 0-31, then the 12 MFMAs of k 0-31 interleaved with the 7 reads of k 32-63
    __builtin_amdgcn_sched_group_barrier(0x100, 7, 0);
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 17, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (wave >= 4) __builtin_amdgcn_s_setprio(0);
  narrow_epilogue<EPI>(acc, ep, smem, M, N, m0, n0, split, wr, wc, l16, g);
}

// ------------------------------------------------------------------ tail split finish
// Sums the tail_S compact fp32 partials of the tail tiles and applies the launch's epilogue
// (same rounding points as epilogue_lds).  Block = 32 rows of one tail tile; thread = 4 rows x 8
// columns.  EPI_DGELU: the 32-row column sums go to colpart row nM + 8 * tile + row block
// (the caller zero-fills colpart and reduces all its rows).
template <int EPI>
__global__ __launch_bounds__(256) void tail_finish_kernel(GemmEpi ep, int M, int N, int GROUP_M) {
  __shared__ float red[8][BN];
  const int tg = blockIdx.x >> 3, rb = blockIdx.x & 7;
  int m0, n0;
  tile_coords(ep.t_begin + tg, M, N, GROUP_M, m0, n0);
  const int tid = threadIdx.x, c = tid & 31, rr = tid >> 5;
  const int n = n0 + c * 8;
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ep.bias && n < N) load8(ep.bias + n, bv);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = rb * 32 + rr + 8 * i;
    const int m = m0 + rl;
    if (m >= M || n >= N) continue;
    float v[8];
    load8(ep.tail + (long)tg * (BM * BN) + rl * BN + c * 8, v);
    for (int sp = 1; sp < ep.tail_S; ++sp) {
      float w[8];
      load8(ep.tail + ((long)sp * ep.t_count + tg) * (BM * BN) + rl * BN + c * 8, w);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += w[j];
    }
    uint16_t* o = ep.out + (long)m * ep.ldo + n;
    if (EPI == EPI_DGELU) {
      float hp[8], f[8];
      load8(ep.aux + (long)m * ep.ldo + n, hp);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f[j] = bf2f(f2bf(bf2f(f2bf(v[j])) * gelu_grad_f(hp[j])));
        csum[j] += f[j];
      }
      store8(o, f);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j] + bv[j]));  // the bf16 pre-activation
      if (EPI == EPI_GELU_ONLY) {
        float gq[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) gq[j] = gelu_tanh_f(v[j]);
        store8(o, gq);
      } else {
        store8(o, v);
      }
      if (EPI == EPI_GELU) {
        float gq[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) gq[j] = gelu_tanh_f(v[j]);
        store8(ep.out2 + (long)m * ep.ldo + n, gq);
      }
    }
  }
  if (EPI == EPI_DGELU && ep.colpart != nullptr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rr][c * 8 + j] = csum[j];
    __syncthreads();
    if (n0 + tid < N) {
      float a = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) a += red[q][tid];
      const int nM = (M + BM - 1) / BM;
      ep.colpart[(long)(nM + tg * 8 + rb) * N + n0 + tid] = a;
    }
  }
}


constexpr int GEMM_GROUP = 8;  // row tiles per column sweep (profiles/r2_gemm_group.txt: 8 best)
// Kernel-path override for the numerics tests only (jm_gemm_test_force); production launches
// choose by shape.  1: every launch on the 64-deep main loop (it otherwise runs at K % 128 == 64);
// 2: the 4-phase kernels at every M, no tail split, g_test_rows = forced tile height (0 = tile_rows).
int g_test_path = 0, g_test_rows = 0;
int g_num_cus = 0;

int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, dev);
    g_num_cus = prop.multiProcessorCount;
  }
  return g_num_cus;
}

template <int EPI, bool NTS>
void launch_nt64(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, const GemmEpi& ep,
                 int nwg, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt64_kernel<EPI, NTS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)GEMM_SMEM);
    attr = true;
  }
  gemm_nt64_kernel<EPI, NTS><<<nwg, 512, GEMM_SMEM, st>>>(A, lda, B, ldb, M, N, K, ep, GEMM_GROUP);
}

template <int EPI, int MTL>
void launch_p4(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, const GemmEpi& ep,
               int nwg, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_p4_kernel<EPI, MTL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)GEMM_SMEM);
    attr = true;
  }
  gemm_p4_kernel<EPI, MTL><<<nwg, 512, GEMM_SMEM, st>>>(A, lda, B, ldb, M, N, K, ep, GEMM_GROUP);
}

template <int EPI>
void launch_narrow(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, const GemmEpi& ep,
                   hipStream_t st) {
  static bool attr = false;
  constexpr size_t sm = (size_t)N_RING * N_STAGE * 2;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_narrow_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)sm);
    attr = true;
  }
  const int nwg = ((M + NBM - 1) / NBM) * ((N + NBN - 1) / NBN) * (EPI == EPI_PARTIAL ? ep.splits : 1);
  gemm_narrow_kernel<EPI><<<nwg, 512, sm, st>>>(A, lda, B, ldb, M, N, K, ep, GEMM_GROUP);
}

constexpr int NARROW_MAX_M = 4096;  // M below this: 128 x 192 tiles are a candidate

bool p4_ok(int K, int epi, int splits) {
  return g_test_path != 1 && K % 128 == 0 && (epi != EPI_PARTIAL || K / 128 >= splits);
}

// Relative cost per tile row of the short-row 4-phase tiles vs 256 rows (the same B panel feeds
// fewer MFMAs; measured per full wave, profiles/r3_gemm_tile_rows.txt)
// (160 rows: 1.20 -- ViT-B / finetune N = 768 GEMMs 5-6 % faster than 192 rows, the decoder's N = 512
// ones 2 % slower than 224: profiles/r5_gemm_tile160.txt)
float rows_cost(int tr) { return tr == 256 ? 1.f : (tr == 224 ? 1.05f : (tr == 192 ? 1.10f : 1.20f)); }

// Cost per output element of the 128 x 192 narrow tile relative to the 4-phase 256-row tile: its
// smaller tile re-reads operands 1.5-1.7x as often per FLOP (MFMA busy 35 vs 43-57 %, r4_gemm_pmc)
constexpr float NARROW_COST = 1.45f;

// M < NARROW_MAX_M: the narrow tiles unless a 4-phase launch fills the chip's waves better --
// waves x tile outputs x per-output cost.  The jumbo MLP at a 2048-row micro-batch: N = 12288
// runs 1.9 waves of 224-row tiles (16-20 % faster than 4 waves of narrow tiles), N = 3072 one
// full wave of narrow tiles (a 224-row launch would leave half the chip idle); at 512 rows every
// jumbo GEMM stays narrow (profiles/r4z_jumbo_routing.txt).  Split-K (EPI_PARTIAL) keeps the
// narrow tiles: the jumbo MLP's K = 12288 GEMMs run 4 splits of 128 x 192 tiles instead of 10 of
// 256 x 256 -- the GEMM alone is ~4 us slower (r3e_summary_vitl_b512_fused_reductions.txt) but the
// fp32 partials shrink 2.5x (profiles/r3_narrow_splitk.txt: ViT-L step -0.41 ms in-process).
bool narrow(int M, int N, int K, int epi) {
  if (g_test_path != 0 || M >= NARROW_MAX_M || N % 8) return false;
  if (epi == EPI_PARTIAL || epi == EPI_TAIL || !p4_ok(K, epi, 1)) return true;
  const int ncu = num_cus();
  const long tn = (long)((M + NBM - 1) / NBM) * ((N + NBN - 1) / NBN);
  const float c_narrow = (float)((tn + ncu - 1) / ncu) * NBM * NBN * NARROW_COST;
  const int nN = (N + BN - 1) / BN;
  for (int tr : {256, 224, 192}) {
    const long t = (long)((M + tr - 1) / tr) * nN;
    if ((float)((t + ncu - 1) / ncu) * tr * BN * rows_cost(tr) < c_narrow) return false;
  }
  return true;
}

int tail_plan_256(int M, int N, int K, int epi, int* tail_r);

// Tile height of a 4-phase launch: the candidate whose launch spans the fewest tile rows per CU,
// waves x rows x rows_cost (a last wave that fills part of the chip costs a full wave; 256-row
// launches may split a tail of at most a quarter wave instead, counted as 0.8 wave: the split
// tail and its finish kernel lost to 224 / 192-row tiles on every measured shape).  Split-K,
// tail-split and 64-deep launches and operands of >= 2 GB (the short tiles' unused a1 rows load
// from offset 2^31, which must be out of range) keep 256.
int tile_rows(int M, int N, int K, int epi, long lda) {
  if (narrow(M, N, K, epi) || !p4_ok(K, epi, 1) || epi == EPI_PARTIAL || epi == EPI_TAIL) return BM;
  if ((long)M * lda * 2 >= (1L << 31) - (1L << 20)) return BM;
  if (g_test_rows) return g_test_rows;
  const int ncu = num_cus(), nN = (N + BN - 1) / BN;
  int r = 0;
  const int t256 = ((M + BM - 1) / BM) * nN;
  float best_c = tail_plan_256(M, N, K, epi, &r) ? (t256 / ncu + 0.8f) * BM : (float)((t256 + ncu - 1) / ncu) * BM;
  int best = BM;
  for (int tr : {224, 192, 160}) {
    const int t = ((M + tr - 1) / tr) * nN;
    const float c = (float)((t + ncu - 1) / ncu) * tr * rows_cost(tr);
    if (c < best_c) best_c = c, best = tr;
  }
  return best;
}

// narrow tiles for M < 4096; K in 128-deep units (split-K: per split) -> p4 (256 / 224 / 192-row
// tiles, tile_rows), else the 64-deep kernel (nontemporal epilogue stores)
template <int EPI>
void launch_epi(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, const GemmEpi& ep,
                int nwg, hipStream_t st) {
  if constexpr (EPI != EPI_TAIL) {
    if (narrow(M, N, K, EPI) && ep.t_count == 0) return launch_narrow<EPI>(A, lda, B, ldb, M, N, K, ep, st);
  }
  if (p4_ok(K, EPI, ep.splits)) {
    const int tr = ep.t_count > 0 ? BM : tile_rows(M, N, K, EPI, lda);
    if constexpr (EPI != EPI_PARTIAL && EPI != EPI_TAIL) {
      const int nw = ((M + tr - 1) / tr) * ((N + BN - 1) / BN);
      if (tr == 224) return launch_p4<EPI, 3>(A, lda, B, ldb, M, N, K, ep, nw, st);
      if (tr == 192) return launch_p4<EPI, 2>(A, lda, B, ldb, M, N, K, ep, nw, st);
      if (tr == 160) return launch_p4<EPI, 1>(A, lda, B, ldb, M, N, K, ep, nw, st);
    }
    return launch_p4<EPI, 4>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  }
  return launch_nt64<EPI, true>(A, lda, B, ldb, M, N, K, ep, nwg, st);
}

template <int EPI>
void launch_tail(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, const GemmEpi& ep,
                 int tiles, hipStream_t st) {
  const int r = ep.t_count;  // tail tiles
  GemmEpi em = ep;
  em.t_begin = 0;
  em.t_count = tiles - r;
  launch_epi<EPI>(A, lda, B, ldb, M, N, K, em, tiles - r, st);
  GemmEpi et = ep;
  et.t_begin = tiles - r;
  launch_nt64<EPI_TAIL, false>(A, lda, B, ldb, M, N, K, et, r * ep.tail_S, st);
  tail_finish_kernel<EPI><<<r * 8, 256, 0, st>>>(et, M, N, GEMM_GROUP);
}

}  // namespace

// numerics tests: path 0 = by shape, 1 = 64-deep main loop everywhere, 2 = 4-phase kernels at
// every M without tail split (rows 256 / 224 / 192 forced, 0 = tile_rows)
void jm_gemm_test_force(int path, int rows) {
  g_test_path = (path == 1 || path == 2) ? path : 0;
  g_test_rows = (g_test_path == 2 && (rows == 224 || rows == 192 || rows == 160 || rows == 256)) ? rows : 0;
}

// output tiles of an NT launch (the narrow kernel's 128 x 192 or the 4-phase 256 / 224 / 192 x 256)
int jm_gemm_nt_tiles(int M, int N, int K, int epi, long lda) {
  if (narrow(M, N, K, epi)) return ((M + NBM - 1) / NBM) * ((N + NBN - 1) / NBN);
  const int tr = tile_rows(M, N, K, epi, lda);
  return ((M + tr - 1) / tr) * ((N + BN - 1) / BN);
}

// rows of the EPI_DGELU / EPI_DMUL column-partial buffer (one per row tile, before tail rows)
int jm_gemm_nt_colpart_rows(int M, int N, int K, int epi, long lda) {
  if (narrow(M, N, K, epi)) return (M + NBM - 1) / NBM;
  const int tr = tile_rows(M, N, K, epi, lda);
  return (M + tr - 1) / tr;
}

// Tail split plan for an NT launch: the last wave of output tiles (tiles % CUs of them) fills only
// part of the chip; when it is at most a quarter wave, those tiles run split-K S ways (compact fp32
// partials, *ws_floats) and a finish kernel applies the epilogue.  Returns S (0 = no tail split);
// *tail_r = number of tail tiles.
// ViT-B FF2 fwd 127 -> 109 us (profiles/r2_gemm_tail_p4.txt).
namespace {
int tail_plan_256(int M, int N, int K, int epi, int* tail_r) {
  *tail_r = 0;
  if (g_test_path != 0) return 0;
  if (!(epi == EPI_STORE || epi == EPI_GELU || epi == EPI_DGELU || epi == EPI_GELU_ONLY) || N % 8 || K % 128) return 0;
  if (narrow(M, N, K, epi)) return 0;
  const int ncu = num_cus();
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles < ncu) return 0;
  const int r = tiles % ncu;
  // (half a wave of tail tiles split 2 ways lost: ViT-L Wo 201 -> 224 us, step +5 ms, gpurun r4tl)
  if (r == 0 || r > ncu / 4) return 0;
  int S = ncu / r;
  // every split keeps >= 8 64-deep K steps (r1: splits of 1-2 steps lost to the partial round trip,
  // profiles/r1_gemm_tail_split.txt)
  if (S > K / 512) S = K / 512;
  if (S > 8) S = 8;
  if (S < 2) return 0;
  *tail_r = r;
  return S;
}
}  // namespace

int jm_gemm_nt_tail_plan(int M, int N, int K, int epi, long lda, int* tail_r, long* ws_floats) {
  *tail_r = 0;
  *ws_floats = 0;
  if (tile_rows(M, N, K, epi, lda) != BM) return 0;  // short-row tiles fill the last wave instead
  const int S = tail_plan_256(M, N, K, epi, tail_r);
  *ws_floats = (long)S * *tail_r * BM * BN;
  return S;
}

// returns 0 on success, <0 on unsupported shape
int jm_gemm_nt(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, int epi,
               const GemmEpi& ep, hipStream_t st) {
  if (K % 64 || N % 4 || M <= 0 || N <= 0) return -1;
  if ((long)M * lda * 2 >= (1L << 32) || (long)N * ldb * 2 >= (1L << 32)) return -2;
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN) * (epi == EPI_PARTIAL ? ep.splits : 1);
  if (epi == EPI_PARTIAL && (ep.splits < 1 || (K / 64) < ep.splits)) return -4;
  if (ep.tail != nullptr && ep.tail_S >= 2 && ep.t_count > 0) {  // tail split (jm_gemm_nt_tail_plan)
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (epi == EPI_STORE) launch_tail<EPI_STORE>(A, lda, B, ldb, M, N, K, ep, tiles, st);
    else if (epi == EPI_GELU) launch_tail<EPI_GELU>(A, lda, B, ldb, M, N, K, ep, tiles, st);
    else if (epi == EPI_DGELU) launch_tail<EPI_DGELU>(A, lda, B, ldb, M, N, K, ep, tiles, st);
    else if (epi == EPI_GELU_ONLY) launch_tail<EPI_GELU_ONLY>(A, lda, B, ldb, M, N, K, ep, tiles, st);
    else return -3;
    return 0;
  }
  if (epi == EPI_PARTIAL)
    launch_epi<EPI_PARTIAL>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else if (epi == EPI_STORE)
    launch_epi<EPI_STORE>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else if (epi == EPI_GELU)
    launch_epi<EPI_GELU>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else if (epi == EPI_GELU_ONLY)
    launch_epi<EPI_GELU_ONLY>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else if (epi == EPI_DGELU && N % 8 == 0)
    launch_epi<EPI_DGELU>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else if (epi == EPI_GELU_D)
    launch_epi<EPI_GELU_D>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else if (epi == EPI_DMUL && N % 8 == 0)
    launch_epi<EPI_DMUL>(A, lda, B, ldb, M, N, K, ep, nwg, st);
  else
    return -3;
  return 0;
}

JM_DEBUG_EXPORT(gemm)
