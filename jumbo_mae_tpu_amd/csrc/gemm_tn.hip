// Weight-gradient MFMA GEMM for gfx950:  G[N][K] += sum_m A[m][n] * B[m][k]
// (A = dY [M, N], B = X [M, K], both bf16 row-major; G fp32 = the flat gradient of a Dense
// kernel stored out x in).  Both operands are M-major ("TN"): the reduction runs down the rows.
//
// The outputs are small (0.25-38 M elements) and the reduction long (25k-100k rows), so the M
// range is split over S workgroups per 256 x 256 output tile, S chosen on the host so that
// tiles x S fills whole waves of the 256 CUs; the S fp32 partial tiles are summed (+= into G)
// by jm_splitk_reduce_add.  With S = 1 the epilogue accumulates into G directly.
//
// Per workgroup: 8 waves (2 x 4), each a 128 (n) x 64 (k) sub-tile = 8 x 4 MFMA 16x16x32 tiles.
// 32 rows of M per step are staged with buffer_load ... lds into a 4-stage ring of [32][256] bf16
// images (512 B rows) for each operand; the MFMA operands need 8 consecutive M per lane, i.e.
// COLUMNS of those images, which ds_read_b64_tr_b16 delivers (two reads of 4 rows each).  The
// images' 16-byte chunks are XOR-swizzled by tswz(row) so the 32 lanes of a transposing read
// (8 rows x 32 B) cover all 64 banks.  Same mid-step barrier pipeline as gemm.hip.
#include <type_traits>

#include "common.h"
#include "jm_api.h"

namespace {

constexpr int TN_ = 256, TK_ = 256, BS = 32, NST = 4, NTH = 512;
constexpr int STAGE = (TN_ + TK_) * BS;  // elements per ring stage

typedef __attribute__((address_space(3))) void lds_void_t;

JM_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const uint16_t* base, long bytes) {
  const int n = bytes >= 0xffffffffL ? -1 : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, n, 0x00020000);
}

JM_DEVICE void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint16_t* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(l), 16, voff, soff, 0, 0);
}

JM_DEVICE f32x4_t mfma16(bf16x8_t a, bf16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16 as inline asm: through the builtin, hipcc cannot tell these LDS reads from
// the in-flight LDS-DMA writes and drains vmcnt(0) before each one (the whole prefetch ring).
// The lgkmcnt waits for the results are therefore explicit (wait_lds) and fenced with
// sched_barrier so no MFMA is hoisted above them.
JM_DEVICE s16x4_t tr4(const uint16_t* p) {
  s16x4_t r;
  const uint32_t a = (uint32_t)(size_t)((const __attribute__((address_space(3))) uint16_t*)p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// tr4 of (addr ^ X) + OFF: the XOR in the same asm block, so no per-block address stays live
template <int X, int OFF>
JM_DEVICE s16x4_t tr4x(uint32_t a) {
  s16x4_t r;
  if constexpr (X == 0) {
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  } else {
    uint32_t tmp;
    asm volatile("v_xor_b32 %1, %3, %2\n\tds_read_b64_tr_b16 %0, %1 offset:%4"
                 : "=v"(r), "=&v"(tmp) : "v"(a), "i"(X), "i"(OFF));
  }
  return r;
}

template <int N, int I = 0, typename F>
JM_DEVICE void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

JM_DEVICE void wait_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

JM_DEVICE bf16x8_t cat44(s16x4_t lo, s16x4_t hi) {
  s16x8_t s;
  s[0] = lo[0]; s[1] = lo[1]; s[2] = lo[2]; s[3] = lo[3];
  s[4] = hi[0]; s[5] = hi[1]; s[6] = hi[2]; s[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, s);
}

// both transposing reads of one fragment (rows +0 and +4: OFF and OFF + 1024) from (addr ^ X):
// one v_xor per fragment instead of one per read
template <int X, int OFF>
JM_DEVICE bf16x8_t tr8x(uint32_t a) {
  s16x4_t lo, hi;
  if constexpr (X == 0) {
    asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
                 : "=&v"(lo), "=v"(hi) : "v"(a), "i"(OFF), "i"(OFF + 1024));
  } else {
    uint32_t tmp;
    asm volatile("v_xor_b32 %2, %4, %3\n\tds_read_b64_tr_b16 %0, %2 offset:%5\n\tds_read_b64_tr_b16 %1, %2 offset:%6"
                 : "=&v"(lo), "=&v"(hi), "=&v"(tmp) : "v"(a), "i"(X), "i"(OFF), "i"(OFF + 1024));
  }
  return cat44(lo, hi);
}

// chunk XOR (in 16-byte units, even so 32-byte pairs stay together): rows {0-3, 8-11} and
// {4-7, 12-15} -- the two row sets of one transposing read -- land on 8 distinct 32-byte slots
JM_DEVICE int tswz(int row) { return ((row & 3) | (((row >> 3) & 1) << 2)) << 1; }

// element offset of (row, col) in a [32][256] stage image
JM_DEVICE int toff(int row, int col) { return row * 256 + ((((col >> 3) ^ tswz(row)) & 31) << 3) + (col & 7); }

struct TFrags {
  bf16x8_t b[4], a[8];
};

}  // namespace

// Segmented M (the batched shared-jumbo-MLP weight gradient): the reduction rows are the
// concatenation of ``n`` separately allocated [rows, lda] / [rows, ldb] blocks (one per layer),
// read in place instead of being copied into one tensor first.
// A grouped segmented launch (jm_gemm_tn_group_seg) keeps problem p's blocks at entries 32 p + i.
struct TnSegs {
  const uint16_t* a[64];
  const uint16_t* b[64];
  int rows;  // rows per block, multiple of the 32-row step
  int n;
};

namespace {

// ACC = 1: G += tile (S == 1), 0: store the fp32 partial tile of split s into slice s.  (Split 0
// adding straight into G measured slower -- the read-modify-write exposes a load latency in the
// epilogue, profiles/r1_ab_tn_acc0.txt -- and so did float-atomic split reduction,
// profiles/r2_tn_atomic.txt; both removed.)
template <int ACC, bool SEG = false>
__global__ __launch_bounds__(NTH, 1) void gemm_tn_kernel(const uint16_t* __restrict__ A, long lda,
                                                         const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                         int K, int steps_per_split, float* __restrict__ out,
                                                         long ldo, long split_stride, TnSegs segs = {}) {
  JM_DGUARD(blockDim.x == NTH && steps_per_split >= 1 && M > 0);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const int wr = wave >> 2, wc = wave & 3;

  // ---- block -> (split, tile): split-major so concurrently running blocks share M rows
  const int nK = K / TK_;
  const int tiles = (N / TN_) * nK;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int split = wg / tiles, tile = wg - split * tiles;
  const int n0 = (tile / nK) * TN_, k0 = (tile % nK) * TK_;
  const int m_begin = split * steps_per_split * BS;
  const int rows = min(M - m_begin, steps_per_split * BS);  // > 0 (host guarantees)
  int nk = (rows + BS - 1) / BS;
  nk += nk & 1;  // even: the pipeline runs in pairs; rows past the split read zeros
  if (nk < 2) nk = 2;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(SEG ? segs.a[0] : A + (long)m_begin * lda + n0, SEG ? 0 : (long)rows * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(SEG ? segs.b[0] : B + (long)m_begin * ldb + k0, SEG ? 0 : (long)rows * ldb * 2);
  // staging: each wave-instruction moves 2 rows x 512 B; 16 per operand and stage -> 2 rounds
  uint32_t a_src[2], b_src[2];
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int row = rr * 16 + wave * 2 + (lane >> 5);
    const int c = (lane & 31) ^ tswz(row);
    a_src[rr] = (uint32_t)((row * lda + c * 8) * 2);
    b_src[rr] = (uint32_t)((row * ldb + c * 8) * 2);
  }
  auto issue = [&](int t) {
    uint16_t* la = smem + (t % NST) * STAGE;
    uint16_t* lb = la + BS * TN_;
    if constexpr (SEG) {  // this step's 32 rows lie in one block; past the split: empty range (zeros)
      const int row = m_begin + t * BS;
      const int sg = min(row / segs.rows, segs.n - 1);
      const int loc = row - sg * segs.rows;
      const int left = row < m_begin + rows ? min(segs.rows - loc, m_begin + rows - row) : 0;
      const __amdgpu_buffer_rsrc_t sra = make_rsrc(segs.a[sg] + (long)loc * lda + n0, (long)left * lda * 2);
      const __amdgpu_buffer_rsrc_t srb = make_rsrc(segs.b[sg] + (long)loc * ldb + k0, (long)left * ldb * 2);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        blds16(sra, a_src[rr], 0, la + (rr * 16 + wave * 2) * TN_);
        blds16(srb, b_src[rr], 0, lb + (rr * 16 + wave * 2) * TK_);
      }
    } else {
      const uint32_t sa = (uint32_t)(t * BS * lda * 2), sb = (uint32_t)(t * BS * ldb * 2);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        blds16(ra, a_src[rr], sa, la + (rr * 16 + wave * 2) * TN_);
        blds16(rb, b_src[rr], sb, lb + (rr * 16 + wave * 2) * TK_);
      }
    }
  };
  // transposing fragment reads: rows 8g + l16/4 (+4), columns base + 4 (l16 & 3)
  const int r1 = 8 * g + (l16 >> 2);
  const int cl = 4 * (l16 & 3);
  // fragment i of a step: i < 4 -> b[i] (X columns), else a[i - 4] (dY columns)
  auto read_one = [&](int t, TFrags& f, int i) {
    const uint16_t* la = smem + (t % NST) * STAGE;
    const uint16_t* lb = la + BS * TN_;
    if (i < 4) {
      const int col = wc * 64 + i * 16 + cl;
      f.b[i] = cat44(tr4(lb + toff(r1, col)), tr4(lb + toff(r1 + 4, col)));
    } else {
      const int col = wr * 128 + (i - 4) * 16 + cl;
      f.a[i - 4] = cat44(tr4(la + toff(r1, col)), tr4(la + toff(r1 + 4, col)));
    }
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto wait_bar = [&](auto outstanding_stages) {  // 4 loads per stage per thread
    constexpr int W = decltype(outstanding_stages)::value * 4;
    if constexpr (W == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if constexpr (W == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if constexpr (W == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  auto step = [&](auto kind, int t, TFrags& cur, TFrags& nxt) {
    constexpr int KIND = decltype(kind)::value;
    wait_lds();  // cur's transposing reads (issued during the previous step) have landed
    if constexpr (KIND == 3) issue(t + 3);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma16(cur.b[nt], cur.a[mt], acc[mt][nt]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (KIND > 0) wait_bar(std::integral_constant<int, KIND - 1>{});
    __builtin_amdgcn_sched_barrier(0);
    // second half: one fragment of the next step (2 transposing reads) per MFMA
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (KIND > 0) {
        if (i < 12) read_one(t + 1, nxt, i);
      }
      const int mt = 4 + i / 4, nt = i % 4;
      acc[mt][nt] = mfma16(cur.b[nt], cur.a[mt], acc[mt][nt]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using K3 = std::integral_constant<int, 3>;
  using K2 = std::integral_constant<int, 2>;
  using K1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;

  issue(0);
  issue(1);
  if (nk > 2) {
    issue(2);
    wait_bar(std::integral_constant<int, 2>{});
  } else {
    wait_bar(std::integral_constant<int, 1>{});
  }
  __builtin_amdgcn_sched_barrier(0);
  TFrags f0, f1;
#pragma unroll
  for (int i = 0; i < 12; ++i) read_one(0, f0, i);
  int t = 0;
  for (; t + 4 < nk; t += 2) {
    step(K3{}, t, f0, f1);
    step(K3{}, t + 1, f1, f0);
  }
  if (nk - t == 4) {
    step(K3{}, t, f0, f1);
    step(K2{}, t + 1, f1, f0);
    t += 2;
  }
  step(K1{}, t, f0, f1);
  step(K0{}, t + 1, f1, f0);

  // ---- epilogue: acc[mt][nt][i] = G[n0 + wr*128 + mt*16 + l16][k0 + wc*64 + nt*16 + 4g + i]
  float* dst = ACC ? out : out + (long)split * split_stride;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int n = n0 + wr * 128 + mt * 16 + l16;
    float* row = dst + (long)n * ldo + k0 + wc * 64 + 4 * g;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
      if (ACC) {
        float o[4];
        load4(row + nt * 16, o);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += o[i];
      }
      store4(row + nt * 16, v);
    }
  }
}

// ------------------------------------------------------------------ 4-phase variant (default)
// The NT kernel's 4-phase counted-vmcnt pipeline (gemm.hip gemm_p4_kernel) on the TN layout:
// 64-row (M) K-tiles cut into half-tile slots of 64 rows x 128 columns (256 B rows, 16 KB):
// a0 / a1 = the dY columns of the waves' upper / lower 64-row output halves (wr*128 + mh*64 +
// [0,64) for both wr), b0 / b1 = the X columns of the waves' left / right 32-column halves (wc*64
// + nh*32 + [0,32) for all wc).  8 slots = 2 K-tiles (128 KB); 4 phases per K-tile, one 64 x 32
// quadrant (16 MFMAs) each, in the order (0,0) (0,1) (1,1) (1,0); fragments one phase ahead;
// each phase starts with [vmcnt(N) lgkmcnt(0) s_barrier] and issues one slot of the tile after
// next (q1 a0, q2 b1, q3 a1, q4 b0).  Fragments are COLUMNS of the slot images (8 consecutive M
// per lane): two ds_read_b64_tr_b16 each.  16-byte chunks XOR-swizzled by tswz(row) (bits 1-3):
// the 8 rows of a transposing read's 32-lane half then cover 8 distinct 32-byte bank slots, and
// the swizzle only permutes a fragment's 4 (A) / 2 (B) column blocks, so each lane keeps one
// address per block (+ immediates for the slot, the k offsets and the second 4 rows: no VALU in the
// loop).  Waves 4-7 at static priority 1.
constexpr int SLOT4 = 64 * 128;  // elements per slot

// GRP: the grid covers the tiles of every problem of ``grp`` (same M); each workgroup picks its
// problem's operands, shape and output from the tile index (workgroup-uniform)
template <int ACC, bool SEG, bool GRP = false>
__global__ __launch_bounds__(NTH, 1) void gemm_tn4_kernel(const uint16_t* __restrict__ A, long lda,
                                                          const uint16_t* __restrict__ B, long ldb, int M, int N,
                                                          int K, int steps_per_split, float* __restrict__ out,
                                                          long ldo, long split_stride, TnSegs segs = {},
                                                          TnGroup grp = {}) {
  JM_DGUARD(blockDim.x == NTH && steps_per_split >= 4 && steps_per_split % 4 == 0 && M > 0);
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int l16 = lane & 15, g = lane >> 4;
  const int wr = wave >> 2, wc = wave & 3;
  if (__builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);

  int nK = K / TK_;
  const int tiles = GRP ? grp.tile0[grp.n] : (N / TN_) * nK;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int split = wg / tiles;
  int tile = wg - split * tiles;
  int soff = 0;  // GRP && SEG: this problem's entries in segs
  if constexpr (GRP) {
    int p = 0;
    while (p + 1 < grp.n && tile >= grp.tile0[p + 1]) ++p;
    tile -= grp.tile0[p];
    soff = 32 * p;
    A = grp.a[p];
    B = grp.b[p];
    lda = grp.lda[p];
    ldb = grp.ldb[p];
    N = grp.N[p];
    K = grp.K[p];
    out = grp.out[p];
    ldo = K;
    split_stride = (long)N * K;
    nK = K / TK_;
  }
  const int n0 = (tile / nK) * TN_, k0 = (tile % nK) * TK_;
  const int m_begin = split * steps_per_split * BS;
  const int rows = min(M - m_begin, steps_per_split * BS);  // > 0 (host guarantees)
  int nk = (rows + 63) / 64;
  nk += nk & 1;  // even (pairs of K-tiles); rows past the split read zeros

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(SEG ? segs.a[soff] : A + (long)m_begin * lda + n0, SEG ? 0 : (long)rows * lda * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(SEG ? segs.b[soff] : B + (long)m_begin * ldb + k0, SEG ? 0 : (long)rows * ldb * 2);
  // glds pieces: 4 rows x 256 B; slot rows pr = (2 wave + rr) * 4 + (lane >> 4); LDS chunk lane & 15
  // holds logical chunk c = (lane & 15) ^ tswz(pr) -> column of the half's segment
  uint32_t a_src[2][2], b_src[2][2];  // [half][rr] byte offsets
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int pr = (2 * wave + rr) * 4 + (lane >> 4);
    const int c = (lane & 15) ^ tswz(pr);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a_src[h][rr] = (uint32_t)((pr * lda + (c >> 3) * 128 + h * 64 + (c & 7) * 8) * 2);
      b_src[h][rr] = (uint32_t)((pr * ldb + (c >> 2) * 64 + h * 32 + (c & 3) * 8) * 2);
    }
  }
  auto issue = [&](int t, auto slot) {
    constexpr int S = decltype(slot)::value;
    uint16_t* l = smem + ((t & 1) * 4 + S) * SLOT4 + (2 * wave) * 4 * 128;
    if constexpr (SEG) {  // this K-tile's 64 rows lie in one block (segs.rows % 64 == 0)
      const int row = m_begin + t * 64;
      const int sg = min(row / segs.rows, segs.n - 1);
      const int loc = row - sg * segs.rows;
      const int left = row < m_begin + rows ? min(segs.rows - loc, m_begin + rows - row) : 0;
      if constexpr (S < 2) {
        const __amdgpu_buffer_rsrc_t sra = make_rsrc(segs.a[soff + sg] + (long)loc * lda + n0, (long)left * lda * 2);
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) blds16(sra, a_src[S][rr], 0, l + rr * 4 * 128);
      } else {
        const __amdgpu_buffer_rsrc_t srb = make_rsrc(segs.b[soff + sg] + (long)loc * ldb + k0, (long)left * ldb * 2);
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) blds16(srb, b_src[S - 2][rr], 0, l + rr * 4 * 128);
      }
    } else {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        if constexpr (S < 2) blds16(ra, a_src[S][rr], (uint32_t)(t * 64 * lda * 2), l + rr * 4 * 128);
        else blds16(rb, b_src[S - 2][rr], (uint32_t)(t * 64 * ldb * 2), l + rr * 4 * 128);
      }
    }
  };
  // transposing fragment reads: lane 4q + p of a 16-lane group -> slot row 8g + q (+4), columns
  // 4p..4p+3 of the fragment's 16-column block; the block's swizzled chunk differs per lane only
  // through bits 1-2 of the chunk index (A: the 4 blocks mt, B: bit 1 = nt), i.e. address bits 5-6
  // Byte address of block 0 per operand and slot set; block j (A: mt, B: nt) is at
  // addr ^ (j << 5) (the swizzle only permutes address bits 5-6); the slot within the set, the
  // k step and the second 4 rows are immediates (<= 58 KB).
  const int qrow = 8 * g + (l16 >> 2), pp = l16 & 3;
  const int sw = tswz(qrow);  // == tswz(qrow + 4 + 32 kk): rows differ in bits 2 and 5 only
  const uint32_t lds0 = (uint32_t)(size_t)((const __attribute__((address_space(3))) uint16_t*)smem);
  const uint32_t a_lo = 2 * (qrow * 128 + (((wr * 8 + (pp >> 1)) ^ sw) << 3) + (pp & 1) * 4);
  const uint32_t b_lo = 2 * (qrow * 128 + (((wc * 4 + (pp >> 1)) ^ sw) << 3) + (pp & 1) * 4);
  // one address VGPR per (slot set, column block): the blocks' swizzled addresses differ in bits
  // 5-6 only (addr ^ (j << 5)), precomputed so the fragment reads need no v_xor (12 VGPRs instead
  // of 4).  The loop's issue slots are the bound: per 16x16x32 MFMA gap (16 cycles, 8 of them the
  // MFMA's own issue) it already carries 1.5 transposing reads, and the v_xor per read (round 5)
  // pushed the gap past 16 cycles -- 5-8 % per weight-gradient GEMM (profiles/r6f_tn_xor_free.txt).
  // (The segmented variant spills two address dwords around its loop for this; PRE = false would
  // keep one address per set and one v_xor per fragment.)
  constexpr bool PRE = true;
  constexpr int NA = PRE ? 4 : 1, NB = PRE ? 2 : 1;
  uint32_t a_addr[2][NA], b_addr[2][NB];
#pragma unroll
  for (int st = 0; st < 2; ++st) {
#pragma unroll
    for (int j = 0; j < NA; ++j) a_addr[st][j] = (lds0 + st * 4 * SLOT4 * 2 + a_lo) ^ (uint32_t)(j << 5);
#pragma unroll
    for (int j = 0; j < NB; ++j) b_addr[st][j] = (lds0 + st * 4 * SLOT4 * 2 + b_lo) ^ (uint32_t)(j << 5);
  }
  typedef bf16x8_t AF[4][2];
  typedef bf16x8_t BF[2][2];
  // fragment i of a half: A (mt, kk) = (i % 4, i / 4), B (nt, kk) = (i % 2, i / 2); slot-in-set SL
  auto read_a1 = [&](int t, auto sl, AF& f, auto ic) {
    constexpr int SL = decltype(sl)::value, I = decltype(ic)::value;
    constexpr int OFF = SL * SLOT4 * 2 + (I / 4) * 32 * 256;
    if constexpr (PRE) f[I % 4][I / 4] = tr8x<0, OFF>(a_addr[t & 1][I % 4]);
    else f[I % 4][I / 4] = tr8x<(I % 4) << 5, OFF>(a_addr[t & 1][0]);
  };
  auto read_b1 = [&](int t, auto sl, BF& f, auto ic) {
    constexpr int SL = decltype(sl)::value, I = decltype(ic)::value;
    constexpr int OFF = SL * SLOT4 * 2 + (I / 2) * 32 * 256;
    if constexpr (PRE) f[I % 2][I / 2] = tr8x<0, OFF>(b_addr[t & 1][I % 2]);
    else f[I % 2][I / 2] = tr8x<(I % 2) << 5, OFF>(b_addr[t & 1][0]);
  };
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // one phase: the quadrant's 16 MFMAs (kk-major), fragment read r of the next phase issued just
  // before MFMA r (r < NR), each pair fenced (inline-asm reads are invisible to the scheduler's
  // instruction groups)
  auto phase = [&](auto mh, auto nh, const AF& a, const BF& b, auto nreads, auto&& rd) {
    constexpr int MH = decltype(mh)::value, NH = decltype(nh)::value, NR = decltype(nreads)::value;
    static_for<16>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i < NR) rd(ic);
      constexpr int kk = i / 8, mt = (i % 8) / 2, nt = i % 2;
      acc[MH * 4 + mt][NH * 2 + nt] = mfma16(b[nt][kk], a[mt][kk], acc[MH * 4 + mt][NH * 2 + nt]);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  // the transposing reads are inline asm (hipcc would drain the LDS-DMA ring before builtin ones),
  // so the waits for their results are explicit: lgkmcnt(0) + barrier at every phase start, where
  // the previous phase's reads are exactly the ones this phase's MFMAs consume
  auto sync = [&](auto n) {
    constexpr int V = decltype(n)::value;
    if constexpr (V == 12) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (V == 10) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (V == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (V == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (V == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (V == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I6 = std::integral_constant<int, 6>;
  using I8 = std::integral_constant<int, 8>;
  using I10 = std::integral_constant<int, 10>;
  using I12 = std::integral_constant<int, 12>;
  using IN = std::integral_constant<int, -1>;

  AF ax, ay;
  BF bp, bq;
  auto ktile = [&](auto kind, int t, BF& b0, BF& b1) {
    constexpr int KIND = decltype(kind)::value;
    // q1 (0,0): read b1(t)
    sync(std::conditional_t<KIND == 0, I4, I12>{});
    if constexpr (KIND == 2) issue(t + 2, I0{});
    phase(I0{}, I0{}, ax, b0, I4{}, [&](auto i) { read_b1(t, I3{}, b1, i); });
    // q2 (0,1): read a1(t)
    sync(std::conditional_t<KIND == 0, I2, std::conditional_t<KIND == 1, I10, I12>>{});
    if constexpr (KIND == 2) issue(t + 2, I3{});
    phase(I0{}, I1{}, ax, b1, I8{}, [&](auto i) { read_a1(t, I1{}, ay, i); });
    // q3 (1,1): no reads
    sync(IN{});
    if constexpr (KIND == 2) issue(t + 2, I1{});
    phase(I1{}, I1{}, ay, b1, I0{}, [&](auto) {});
    // q4 (1,0): read a0(t+1), b0(t+1) (into b1, free after q3)
    if constexpr (KIND > 0) {
      sync(std::conditional_t<KIND == 1, I0, I6>{});
      if constexpr (KIND == 2) issue(t + 2, I2{});
      phase(I1{}, I0{}, ay, b0, I12{}, [&](auto i) {
        constexpr int I = decltype(i)::value;
        if constexpr (I < 8) read_a1(t + 1, I0{}, ax, i);
        else read_b1(t + 1, I2{}, b1, std::integral_constant<int, I - 8>{});
      });
    } else {
      phase(I1{}, I0{}, ay, b0, I0{}, [&](auto) {});
    }
  };
  using K2 = std::integral_constant<int, 2>;
  using K1 = std::integral_constant<int, 1>;
  using K0 = std::integral_constant<int, 0>;

  issue(0, I0{});
  issue(0, I3{});
  issue(0, I1{});
  issue(0, I2{});
  issue(1, I0{});
  issue(1, I3{});
  issue(1, I1{});
  sync(I6{});
  issue(1, I2{});
  static_for<8>([&](auto i) { read_a1(0, I0{}, ax, i); });
  static_for<4>([&](auto i) { read_b1(0, I2{}, bp, i); });
  int t = 0;
  for (; t + 4 <= nk; t += 2) {
    ktile(K2{}, t, bp, bq);
    ktile(K2{}, t + 1, bq, bp);
  }
  ktile(K1{}, t, bp, bq);
  ktile(K0{}, t + 1, bq, bp);

  // ---- epilogue: acc[mt][nt][i] = G[n0 + wr*128 + mt*16 + l16][k0 + wc*64 + nt*16 + 4g + i]
  float* dst = ACC ? out : out + (long)split * split_stride;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int n = n0 + wr * 128 + mt * 16 + l16;
    float* row = dst + (long)n * ldo + k0 + wc * 64 + 4 * g;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
      if (ACC) {
        float o[4];
        load4(row + nt * 16, o);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += o[i];
      }
      store4(row + nt * 16, v);
    }
  }
}

}  // namespace

size_t jm_gemm_tn_smem() { return (size_t)NST * STAGE * sizeof(uint16_t); }

// Split of the M range: returns steps (of 32 rows) per split; *S_out = number of splits.
// Picks the split count that minimises an estimate of (waves of 256 CUs) x (steps per split +
// epilogue) + the fp32 partial-tile traffic of the reduction (weight A/B: profiles/r2_tn_plan_scale.txt).
namespace {
int tn_plan(int M, int tiles, long NK, int* S_out) {
  const int steps = (M + BS - 1) / BS;
  const int unit = 4;  // steps per split: whole 128-row units of the 4-phase kernel
  double best = 1e30;
  int best_sps = (steps + unit - 1) / unit * unit, best_S = 1;
  for (int S = 1; S <= 128; ++S) {
    int sps = (steps + S - 1) / S;
    sps = (sps + unit - 1) / unit * unit;
    if (sps < 4 && S > 1) break;
    const int s_eff = (steps + sps - 1) / sps;
    const long wgs = (long)tiles * s_eff;
    const long waves = (wgs + 255) / 256;
    const double t_steps = (double)waves * (sps + 12);                       // ~1 us per step
    const double t_red = s_eff > 1 ? (double)s_eff * NK * 8.0 / 5.0e12 * 1e6 : 0.0;  // us
    const double est = t_steps + t_red;
    if (est < best) {
      best = est;
      best_sps = sps;
      best_S = s_eff;
    }
  }
  *S_out = best_S;
  return best_sps;
}
}  // namespace

int jm_gemm_tn_plan(int M, int N, int K, int* S_out) { return tn_plan(M, (N / TN_) * (K / TK_), (long)N * K, S_out); }

// split plan of a grouped launch: the problems' tiles and output elements together
int jm_gemm_tn_group_plan(const TnGroup& grp, int M, int* S_out) {
  long nk = 0;
  int tiles = 0;
  for (int p = 0; p < grp.n; ++p) {
    nk += (long)grp.N[p] * grp.K[p];
    tiles += (grp.N[p] / TN_) * (grp.K[p] / TK_);
  }
  return tn_plan(M, tiles, nk, S_out);
}

namespace {
template <typename KERN>
void set_smem_once(KERN k, bool& done) {
  if (!done) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)jm_gemm_tn_smem());
    done = true;
  }
}

// the 4-phase kernel (whole 128-row units, 64-row segments) or the r1 32-row-step kernel
// returns 0 (the caller reduces the S partial slices into G when S > 1), < 0 on error
// store (S == 1): G = the product (the split-0 store kernel into G instead of the accumulating one)
template <bool SEG>
int launch_tn(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, int sps, int S,
              float* G, long ldo, float* partial, const TnSegs& segs, bool p4, hipStream_t st, bool store = false) {
  const int tiles = (N / TN_) * (K / TK_);
  const size_t sm = jm_gemm_tn_smem();
  if (S > 1 && partial == nullptr) return -3;
  if (S == 1 && store) {
    if (p4) {
      static bool a = false;
      set_smem_once(gemm_tn4_kernel<0, SEG>, a);
      gemm_tn4_kernel<0, SEG><<<tiles, NTH, sm, st>>>(A, lda, B, ldb, M, N, K, sps, G, ldo, 0, segs);
    } else {
      static bool a = false;
      set_smem_once(gemm_tn_kernel<0, SEG>, a);
      gemm_tn_kernel<0, SEG><<<tiles, NTH, sm, st>>>(A, lda, B, ldb, M, N, K, sps, G, ldo, 0, segs);
    }
    return 0;
  }
  if (p4) {
    if (S == 1) {
      static bool a = false;
      set_smem_once(gemm_tn4_kernel<1, SEG>, a);
      gemm_tn4_kernel<1, SEG><<<tiles, NTH, sm, st>>>(A, lda, B, ldb, M, N, K, sps, G, ldo, 0, segs);
    } else {
      static bool a = false;
      set_smem_once(gemm_tn4_kernel<0, SEG>, a);
      gemm_tn4_kernel<0, SEG><<<tiles * S, NTH, sm, st>>>(A, lda, B, ldb, M, N, K, sps, partial, K, (long)N * K,
                                                          segs);
    }
  } else if (S == 1) {
    static bool a = false;
    set_smem_once(gemm_tn_kernel<1, SEG>, a);
    gemm_tn_kernel<1, SEG><<<tiles, NTH, sm, st>>>(A, lda, B, ldb, M, N, K, sps, G, ldo, 0, segs);
  } else {
    static bool a = false;
    set_smem_once(gemm_tn_kernel<0, SEG>, a);
    gemm_tn_kernel<0, SEG><<<tiles * S, NTH, sm, st>>>(A, lda, B, ldb, M, N, K, sps, partial, K, (long)N * K, segs);
  }
  return 0;
}
}  // namespace



// G[N][K] (ldo) += A[M][N]^T . B[M][K]; partial: [S][N][K] fp32 workspace when S > 1 (else null);
// the caller reduces the S slices into G (jm_splitk_reduce_add).  Measured and removed: float-atomic
// split reduction (profiles/r2_tn_atomic.txt), split 0 into G (r1_ab_tn_acc0.txt), the last-arriving
// split adding the other slices in the kernel (r3e_summary_vitl_b512_fused_reductions.txt).
int jm_gemm_tn(const uint16_t* A, long lda, const uint16_t* B, long ldb, int M, int N, int K, int sps, int S,
               float* G, long ldo, float* partial, hipStream_t st, int store) {
  if (N % TN_ || K % TK_ || M <= 0) return -1;
  if ((long)M * lda * 2 >= (1L << 32) || (long)M * ldb * 2 >= (1L << 32)) return -2;
  return launch_tn<false>(A, lda, B, ldb, M, N, K, sps, S, G, ldo, partial, TnSegs{}, sps % 4 == 0, st, store);
}

// Segmented-M variant of jm_gemm_tn: A / B rows come from segs (n blocks of segs.rows rows).
int jm_gemm_tn_seg(const TnSegs& segs, long lda, long ldb, int N, int K, int sps, int S, float* G, long ldo,
                   float* partial, hipStream_t st, int store) {
  if (N % TN_ || K % TK_ || segs.n < 1 || segs.n > 32 || segs.rows % BS) return -1;
  if ((long)segs.rows * lda * 2 >= (1L << 32) || (long)segs.rows * ldb * 2 >= (1L << 32)) return -2;
  const int M = segs.rows * segs.n;
  return launch_tn<true>(nullptr, lda, nullptr, ldb, M, N, K, sps, S, G, ldo, partial, segs,
                         sps % 4 == 0 && segs.rows % 64 == 0, st, store);
}

// Grouped launch of up to 4 TN problems over the same M rows (e.g. the FF1 and FF2 weight
// gradients of a layer): one grid of sum(tiles) x S workgroups instead of two half-filled ones,
// so each problem needs half the splits -- half the fp32 partial slices written and reduced.
// S > 1: grp.out[p] = the [S][N_p K_p] partial workspace (the caller reduces into G_p); S == 1:
// grp.out[p] = G_p, accumulated in place.
int jm_gemm_tn_group(TnGroup grp, int M, int sps, int S, hipStream_t st, int store) {
  if (grp.n < 1 || grp.n > 4 || M <= 0 || sps % 4 || sps < 4 || S < 1) return -1;
  grp.tile0[0] = 0;
  for (int p = 0; p < grp.n; ++p) {
    if (grp.N[p] % TN_ || grp.K[p] % TK_ || grp.out[p] == nullptr) return -1;
    if ((long)M * grp.lda[p] * 2 >= (1L << 32) || (long)M * grp.ldb[p] * 2 >= (1L << 32)) return -2;
    grp.tile0[p + 1] = grp.tile0[p] + (grp.N[p] / TN_) * (grp.K[p] / TK_);
  }
  const size_t sm = jm_gemm_tn_smem();
  const int wgs = grp.tile0[grp.n] * S;
  if (S == 1 && !store) {
    static bool a = false;
    set_smem_once(gemm_tn4_kernel<1, false, true>, a);
    gemm_tn4_kernel<1, false, true><<<wgs, NTH, sm, st>>>(nullptr, 0, nullptr, 0, M, 0, 0, sps, nullptr, 0, 0,
                                                          TnSegs{}, grp);
  } else {
    static bool a = false;
    set_smem_once(gemm_tn4_kernel<0, false, true>, a);
    gemm_tn4_kernel<0, false, true><<<wgs, NTH, sm, st>>>(nullptr, 0, nullptr, 0, M, 0, 0, sps, nullptr, 0, 0,
                                                          TnSegs{}, grp);
  }
  return 0;
}

// Grouped + segmented (the batched jumbo-MLP weight gradients W1 and W2 of all layers in one
// grid): problem p's per-layer blocks at segs.a / segs.b[32 p + i], one M split (S == 1, the
// gradients accumulated in place) when the problems' tiles fill the chip, else partial slices.
int jm_gemm_tn_group_seg(TnGroup grp, const TnSegs& segs, int sps, int S, hipStream_t st, int store) {
  const int M = segs.rows * segs.n;
  if (grp.n < 1 || grp.n > 2 || segs.n < 1 || segs.n > 32 || segs.rows % 64 || sps % 4 || sps < 4 || S < 1)
    return -1;
  grp.tile0[0] = 0;
  for (int p = 0; p < grp.n; ++p) {
    if (grp.N[p] % TN_ || grp.K[p] % TK_ || grp.out[p] == nullptr) return -1;
    if ((long)segs.rows * grp.lda[p] * 2 >= (1L << 32) || (long)segs.rows * grp.ldb[p] * 2 >= (1L << 32)) return -2;
    grp.tile0[p + 1] = grp.tile0[p] + (grp.N[p] / TN_) * (grp.K[p] / TK_);
  }
  const size_t sm = jm_gemm_tn_smem();
  const int wgs = grp.tile0[grp.n] * S;
  if (S == 1 && !store) {
    static bool a = false;
    set_smem_once(gemm_tn4_kernel<1, true, true>, a);
    gemm_tn4_kernel<1, true, true><<<wgs, NTH, sm, st>>>(nullptr, 0, nullptr, 0, M, 0, 0, sps, nullptr, 0, 0, segs,
                                                         grp);
  } else {
    static bool a = false;
    set_smem_once(gemm_tn4_kernel<0, true, true>, a);
    gemm_tn4_kernel<0, true, true><<<wgs, NTH, sm, st>>>(nullptr, 0, nullptr, 0, M, 0, 0, sps, nullptr, 0, 0, segs,
                                                         grp);
  }
  return 0;
}

JM_DEBUG_EXPORT(gemm_tn)
