// Split-K weight gradients of the encoder layer on an LDS-DMA ring with
// producer / consumer waves (gfx950).  Replaces the autograd weight and bias
// gradients of the three encoder projections (models/model.py:773-775 Q/K/V,
// :787-788 the MLP; train_CLIP.py:158 backward):
//   part[z][a][b] = sum_{m in split z} A[m][a] B[m][b],  bias_part[z][a] = sum_m A[m][a]
// with the tokens m as the MFMA k axis, every product as three bf16 MFMAs
// (ghm_split.h).
//
// Workgroup = one 128 x 128 output tile of one token split, 8 waves:
//   waves 0-3 (producers, one per SIMD): issue the LDS-DMA fills of the step
//     KT * D tokens ahead (global_load_lds_dwordx4, no register staging and no
//     per-row address arithmetic in the consumers), convert the f32 operands of
//     the next step into bf16 hi / lo images (optionally through the LayerNorm
//     of the token), mask tokens past the split, and sum the bias of A;
//   waves 4-7 (consumers, one per SIMD beside a producer): only read operand
//     fragments with the hardware transpose (ds_read_b64_tr_b16) and issue MFMAs,
//     2 x 2 tiles of 32 x 32 per wave.
// One s_barrier per KT-token step publishes the next step's images and frees the
// slots the step just consumed.  Operand formats:
//   WG_F32   f32 [M][ld], DMA'd raw into a ring of D slots, converted by the producers
//   WG_LN    the same through LayerNorm: (x - mean) rstd gamma + beta, the per-token
//            (mean, rstd) DMA'd beside the rows with a system-scope policy (the rule
//            for cross-kernel statistics, DESIGN.md section 4 "Determinism")
//   WG_SPLIT pre-split bf16 planes (hi at the pointer, lo `plane` elements on), written
//            by the producing kernel (k_mlp_bwd_rc_x3 with split outputs) with the
//            columns of each 32-group in perm32 order; DMA'd straight into a ring of
//            D + 1 image slots (no conversion), the permutation undone in the epilogue.
// LDS images are [KT tokens][128 columns] bf16 per plane (256-B rows), 16-B chunk ch
// of row r at ch ^ sw(r), sw(r) = ((r & 3) << 2) | ((r >> 2) & 3): the transposed
// fragment reads (4 token rows x 32 columns per 32-lane half) and the converters'
// ds_write_b128 (8 chunks of one row per 8-lane group) are both conflict-free
// (cdna_hip_programming.md T10 "(b) plain 256-byte rows").  Raw f32 slots are
// [KT][128] f32 (512-B rows), chunk ch of row r at ch ^ (r & 1), so a converter's
// 16-lane ds_read_b128 groups (two token rows) hit disjoint bank halves.
#include <cstdlib>

#include "ghm_common.h"
#include "ghm_split.h"
#include "ghm_launch.h"

namespace {

constexpr int WG_F32 = 0, WG_LN = 1, WG_SPLIT = 2;

__device__ __forceinline__ constexpr int img_sw(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// byte offset of 16-B chunk ch of row r in a [KT][128] bf16 plane
__device__ __forceinline__ constexpr int img_off(int r, int ch) { return r * 256 + 16 * (ch ^ img_sw(r)); }
// byte offset of 16-B chunk ch of row r in a [KT][128] f32 raw slot
__device__ __forceinline__ constexpr int raw_off(int r, int ch) { return r * 512 + 16 * (ch ^ (r & 1)); }

// original column of image column x (0..127) of a WG_SPLIT operand: perm32 inside
// each 32-group (ghm_x3.hip perm32: k-slot 8g + i of the producer's 16x16x32
// accumulator holds unit 4g + i or 16 + 4g + i - 4)
__device__ __forceinline__ constexpr int split_col(int x) {
  const int q = x & 31;
  return (x & ~31) + ((q & 7) < 4 ? 4 * ((q >> 3) & 3) + (q & 3) : 16 + 4 * ((q >> 3) & 3) + (q & 3));
}

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
__device__ __forceinline__ bf16x4 ldtr4(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p));
}

__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <typename T>
__device__ __forceinline__ T* uniform_p(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return reinterpret_cast<T*>((static_cast<uint64_t>(hi) << 32) | lo);
}

// LDS-DMA of one step's operand by producer wave pw (0..3) with buffer loads: the
// per-lane byte offsets inside a step are fixed (computed once, init), the step
// moves only the SGPR descriptor's base (m0 rows on) and its record count (the
// rows left before M), so the DMAs of a step cost no vector address arithmetic and
// rows past M read as zeros (the buffer range check; the converters' token mask
// covers the LayerNorm operand, whose zero rows would become beta).
template <int FMT, int KT>
struct Filler {
  static constexpr int PW = KT / 8;  // 1-KB pieces per producer wave and step
  int voff[PW];                      // per-lane byte offset of each piece inside the step's rows
  int dst[PW];                       // LDS byte offset of each piece inside the slot
  int plane[PW];                     // SPLIT: hi (0) or lo (1) plane of each piece
  int soff;                          // LN: the lane's statistics dword inside the step's [KT][2] rows

  __device__ __forceinline__ void init(int ld_bytes, int col_bytes, int pw, int lane) {
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      if (FMT == WG_SPLIT) {  // per plane KT x 256 B = KT / 4 pieces of 4 rows
        constexpr int PP = KT / 4;
        const int piece = pw * PW + k, pp = piece % PP;
        const int r = 4 * pp + (lane >> 4);
        plane[k] = piece / PP;
        voff[k] = r * ld_bytes + col_bytes + 16 * ((lane & 15) ^ img_sw(r));
        dst[k] = plane[k] * (KT * 256) + 1024 * pp;
      } else {  // KT x 512 B = KT / 2 pieces of 2 rows
        const int pp = pw * PW + k;
        const int r = 2 * pp + (lane >> 5);
        plane[k] = 0;
        voff[k] = r * ld_bytes + col_bytes + 16 * ((lane & 31) ^ (r & 1));
        dst[k] = 1024 * pp;
      }
    }
    // LN: this wave's token statistics (8 B each) into its own 256-B region: entry
    // e = 4 it + r is token 16 it + 4 pw + r (the rows its items convert); dword lane
    // L < 2 NE is entry L >> 1, the other lanes re-read them
    constexpr int NE = 4 * (KT / 16);
    const int li = lane & (2 * NE - 1), e = li >> 1;
    soff = (16 * (e >> 2) + 4 * pw + (e & 3)) * 8 + 4 * (li & 1);
  }

  __device__ __forceinline__ void fill(const char* g, int ld_bytes, int64_t plane_bytes, int64_t m0, int64_t M,
                                       const char* stats, char* __restrict__ slot, int pw) const {
    const int64_t left = M - m0 > 0 ? M - m0 : 0;
    // descriptor inputs made provably wave-uniform (readfirstlane), so each DMA is one
    // instruction and not a waterfall loop (cdna_hip_programming.md T20)
    const int nrec = uniform_i(static_cast<int>(left * ld_bytes < 0x7fffffff ? left * ld_bytes : 0x7fffffff));
    char* base = uniform_p(const_cast<char*>(g + m0 * ld_bytes));
    const auto rs0 = __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), nrec, 0x00020000);
    const auto rs1 = __builtin_amdgcn_make_buffer_rsrc(uniform_p(base + plane_bytes), static_cast<short>(0), nrec,
                                                       0x00020000);
#pragma unroll
    for (int k = 0; k < PW; ++k) {
      void* d = uniform_p(slot + dst[k]);
      if (FMT == WG_SPLIT && plane[k])
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs1, (__attribute__((address_space(3))) void*)(d), 16, voff[k], 0,
                                                 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs0, (__attribute__((address_space(3))) void*)(d), 16, voff[k], 0,
                                                 0, 0);
    }
    if (FMT == WG_LN) {  // system scope (sc0 sc1): the rule for cross-kernel statistics
      const int srec = uniform_i(static_cast<int>(left * 8 < 0x7fffffff ? left * 8 : 0x7fffffff));
      const auto rss = __builtin_amdgcn_make_buffer_rsrc(uniform_p(const_cast<char*>(stats + m0 * 8)),
                                                         static_cast<short>(0), srec, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rss, (__attribute__((address_space(3))) void*)(uniform_p(slot + KT * 512 + 256 * pw)), 4, soff, 0, 0, 1 | 16);
    }
  }
};

// 8 f32 (two 16-B chunks of a raw row) -> bf16 hi / lo chunks of the image
__device__ __forceinline__ void split_store(const float* x, char* img_h, char* img_l, int off) {
  bf16x8 h, l;
  split8(x, h, l);
  *reinterpret_cast<bf16x8*>(img_h + off) = h;
  *reinterpret_cast<bf16x8*>(img_l + off) = l;
}

}  // namespace

// One producer iteration (Producer::iter): the fills of step `fs` (if do_fill) into fill_a / fill_b,
// then step ps's conversion (raw_a / raw_b -> img_a / img_b) and A's bias sums (if
// do_prod).  The buffers are __restrict__ parameters of one inlined function, so
// the waitcnt pass sees the DMA targets and the converter's LDS reads as disjoint
// and leaves the fills in flight (the producers wait for them explicitly, counted,
// before the barrier that publishes a step).
template <int AF, int BF, int KT>
struct Producer {
  // (a static member: as a free function template, hipcc's host pass rejected some
  // instantiations of the call with "substitution failure" and no reason given)
  static __device__ __forceinline__ void iter(
    bool do_fill, const Filler<AF, KT>& fa, const Filler<BF, KT>& fb, const char* A, int lda_b, int64_t a_plane_b,
    const char* B, int ldb_b, int64_t b_plane_b, const char* stats, int64_t fm0, int64_t M,
    char* __restrict__ fill_a, char* __restrict__ fill_b, bool do_prod, int nvalid, const char* __restrict__ raw_a,
    const char* __restrict__ raw_b, char* __restrict__ img_a, char* __restrict__ img_b, const float* gam,
    const float* bet, bool bias, float* bsum, int pw, int lane) {
  if (do_fill) {
    fa.fill(A, lda_b, a_plane_b, fm0, M, nullptr, fill_a, pw);
    fb.fill(B, ldb_b, b_plane_b, fm0, M, stats, fill_b, pw);
  }
  if (!do_prod) return;
  const int pc = lane & 15;
  // tokens past M arrive as zero rows (the DMA range check) and a split never ends
  // inside a step (tok_per_split % KT == 0), so only the last step of the last
  // split masks: the LayerNorm would turn a zero row into beta
  const bool partial = nvalid < KT;
#pragma unroll
  for (int it = 0; it < KT / 16; ++it) {
    const int t = 16 * it + 4 * pw + (lane >> 4);
    const bool ok = !partial || t < nvalid;
    if (AF != WG_SPLIT) {
      const float4 u = *reinterpret_cast<const float4*>(raw_a + raw_off(t, 2 * pc));
      const float4 v = *reinterpret_cast<const float4*>(raw_a + raw_off(t, 2 * pc + 1));
      float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
      if (bias) {
#pragma unroll
        for (int i = 0; i < 8; ++i) bsum[i] += x[i];  // (rows past M are zero)
      }
      split_store(x, img_a, img_a + KT * 256, img_off(t, pc));
    } else if (bias) {  // bias of a pre-split A: hi + lo of the valid tokens
      const bf16x8 h = *reinterpret_cast<const bf16x8*>(img_a + img_off(t, pc));
      const bf16x8 l = *reinterpret_cast<const bf16x8*>(img_a + KT * 256 + img_off(t, pc));
#pragma unroll
      for (int i = 0; i < 8; ++i) bsum[i] += static_cast<float>(h[i]) + static_cast<float>(l[i]);  // (zero past M)
    }
    if (BF != WG_SPLIT) {
      const float4 u = *reinterpret_cast<const float4*>(raw_b + raw_off(t, 2 * pc));
      const float4 v = *reinterpret_cast<const float4*>(raw_b + raw_off(t, 2 * pc + 1));
      float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
      if (BF == WG_LN) {  // this wave's statistics region: token t is entry 4 it + (lane >> 4)
        const float2 st = *reinterpret_cast<const float2*>(raw_b + KT * 512 + 256 * pw + 8 * (4 * it + (lane >> 4)));
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = (x[i] - st.x) * st.y * gam[i] + bet[i];
        if (partial) {
#pragma unroll
          for (int i = 0; i < 8; ++i) x[i] = ok ? x[i] : 0.f;
        }
      }
      split_store(x, img_b, img_b + KT * 256, img_off(t, pc));
    }
  }
}
};

// AF / BF: operand formats; D: DMA steps in flight (F32 / LN raw rings of D slots,
// WG_SPLIT image rings of D + 1); KT: tokens per step (16 or 32).
template <int AF, int BF, int D, int KT>
__global__ __launch_bounds__(512, 1) void k_wgrad_ring_x3(
    const char* __restrict__ A, int lda_b, int64_t a_plane_b, const char* __restrict__ B, int ldb_b,
    int64_t b_plane_b, const char* __restrict__ stats, const float* __restrict__ lnw,
    const float* __restrict__ lnb, float* __restrict__ part, float* __restrict__ bias_part, int64_t M,
    int tok_per_split, int Acols, int Bcols) {
  static_assert(AF != WG_LN, "the LayerNorm operand is B");
  static_assert(AF != WG_SPLIT || BF != WG_SPLIT, "one operand must be converted (it masks the split's tail)");
  static_assert(KT == 16 || KT == 32, "KT");
  static_assert(D >= 2 && D <= 6, "D (wait_fills covers up to D - 2 = 4 later steps)");
  constexpr int NKS = KT / 16;                       // 16-token MFMA k-steps per step
  constexpr int IMG = KT * 256 * 2;                  // hi + lo image bytes
  constexpr int RAW = KT * 512;                      // raw f32 slot
  constexpr int RAWA = AF == WG_SPLIT ? 0 : RAW;
  constexpr int RAWB = BF == WG_SPLIT ? 0 : RAW + (BF == WG_LN ? 1024 : 0);
  // ring slot counts: converted operands D raw + 2 images; split operands D + 1 images
  constexpr int A_RING = AF == WG_SPLIT ? (D + 1) * IMG : D * RAWA + 2 * IMG;
  constexpr int B_RING = BF == WG_SPLIT ? (D + 1) * IMG : D * RAWB + 2 * IMG;
  static_assert(A_RING + B_RING <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char lds[A_RING + B_RING];
  char* const a_base = lds;
  char* const b_base = lds + A_RING;
  // image of step s: split operand -> ring slot s % (D + 1); converted -> image s & 1
  auto a_img = [&](int s) -> char* {
    return AF == WG_SPLIT ? a_base + (s % (D + 1)) * IMG : a_base + D * RAWA + (s & 1) * IMG;
  };
  auto b_img = [&](int s) -> char* {
    return BF == WG_SPLIT ? b_base + (s % (D + 1)) * IMG : b_base + D * RAWB + (s & 1) * IMG;
  };
  // DMA target of step s: split operand -> its image slot; converted -> raw slot s % D
  auto a_dst = [&](int s) -> char* { return AF == WG_SPLIT ? a_img(s) : a_base + (s % D) * RAWA; };
  auto b_dst = [&](int s) -> char* { return BF == WG_SPLIT ? b_img(s) : b_base + (s % D) * RAWB; };

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool producer = wave < 4;
  // XCD-aware order (workgroup w runs on XCD w % 8): each XCD walks a contiguous run of
  // (tile, split) pairs, tiles fastest, so the tiles of one token range share its L2
  int lin = static_cast<int>(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
  {
    const int full = static_cast<int>(gridDim.x * gridDim.y * gridDim.z) / 8 * 8;
    if (lin < full) lin = (lin % 8) * (full / 8) + lin / 8;
  }
  const int tbx = lin % static_cast<int>(gridDim.x);
  const int tby = (lin / static_cast<int>(gridDim.x)) % static_cast<int>(gridDim.y);
  const int tbz = lin / static_cast<int>(gridDim.x * gridDim.y);
  const int a_blk = tbx * 128, b_blk = tby * 128;
  const int64_t m_begin = static_cast<int64_t>(tbz) * tok_per_split;
  const int64_t m_end = m_begin + tok_per_split < M ? m_begin + tok_per_split : M;
  const int nsteps = static_cast<int>((m_end - m_begin + KT - 1) / KT);
  const int a_colb = (AF == WG_SPLIT ? 2 : 4) * a_blk, b_colb = (BF == WG_SPLIT ? 2 : 4) * b_blk;

  // producer state: columns 8 pc .. 8 pc + 7 of B (gamma, beta) and of A (bias sums)
  const int pw = __builtin_amdgcn_readfirstlane(wave & 3), pc = lane & 15;
  float gam[8], bet[8], bsum[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    gam[i] = 1.f;
    bet[i] = 0.f;
    bsum[i] = 0.f;
  }
  if (BF == WG_LN && producer) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      gam[i] = lnw[b_blk + 8 * pc + i];
      bet[i] = lnb[b_blk + 8 * pc + i];
    }
  }
  const bool want_bias = bias_part != nullptr && tby == 0;
  Filler<AF, KT> fa;
  Filler<BF, KT> fb;
  fa.init(lda_b, a_colb, pw, lane);
  fb.init(ldb_b, b_colb, pw, lane);
  // LDS-DMA instructions per producer wave and step: KT / 8 per operand, + 1 statistics
  constexpr int NW = KT / 8 + KT / 8 + (BF == WG_LN ? 1 : 0);
  // wait until the fills of a step have landed with the fills of the n later steps
  // still in flight
  auto wait_fills = [&](int n) {
    if (n <= 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (n == 1)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NW) : "memory");
    else if (n == 2)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NW) : "memory");
    else if (n == 3)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NW) : "memory");
  };
  auto nvalid_of = [&](int s) {
    const int64_t left = m_end - (m_begin + static_cast<int64_t>(s) * KT);
    return static_cast<int>(left < KT ? left : KT);
  };

  // consumer state: wave cw = wave - 4 owns rows wa .. wa + 63 (A columns) and columns
  // wb .. wb + 63 (B columns) of the tile, as 2 x 2 accumulators of 32 x 32
  const int cw = wave & 3, wa = (cw >> 1) * 64, wb = (cw & 1) * 64;
  // transposed-read offsets: 16-lane group g reads rows k0 + 8 (g >> 1) + q (+ 4) of
  // the 16 columns c0 + 16 (g & 1) .. + 15, lane 4q + p supplying columns 4p .. 4p + 3;
  // lane i of the group receives column i, element e = row e (cdna_hip_programming.md T10)
  const int g4 = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  int offA[2][NKS][2], offB[2][NKS][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int rd = 0; rd < 2; ++rd) {
        const int r = 16 * ks + 8 * (g4 >> 1) + 4 * rd + q;
        const int ca = wa + 32 * i + 16 * (g4 & 1) + 4 * p, cb = wb + 32 * i + 16 * (g4 & 1) + 4 * p;
        offA[i][ks][rd] = img_off(r, ca >> 3) + 2 * (ca & 7);
        offB[i][ks][rd] = img_off(r, cb >> 3) + 2 * (cb & 7);
      }
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 2; ++k) acc[i][k] = zero16();

  // ---- one loop from s = -D: iteration s publishes step s + 1's fills and step s's
  // images, then the consumers compute step s while the producers fill step s + D
  // and convert step s + 1.  (One loop, so that every LDS-DMA and every producer LDS
  // access comes from the same inlined Producer::iter: fills from a separate prologue
  // carried no alias scope, and the waitcnt pass then drained vmcnt(0) before the
  // converters' image stores of every step.) ----
#pragma unroll 1
  for (int s = -D; s < nsteps; ++s) {
    const int fs = s + D, ps = s + 1;
    if (producer && ps >= 0 && ps < nsteps) {
      // step s + 1's fills have landed (steps s + 2 .. s + D - 1 stay in flight)
      wait_fills((fs - 1 < nsteps - 1 ? fs - 1 : nsteps - 1) - ps);
    }
    // publishes step s's images and step s + 1's fills; frees the slots of step s - 1
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (producer) {
      const int fsc = fs < nsteps ? fs : 0, psc = ps >= 0 && ps < nsteps ? ps : 0;
      Producer<AF, BF, KT>::iter(fs < nsteps, fa, fb, A, lda_b, a_plane_b, B, ldb_b, b_plane_b, stats,
                                m_begin + static_cast<int64_t>(fsc) * KT, M, a_dst(fsc), b_dst(fsc),
                                ps >= 0 && ps < nsteps, nvalid_of(psc), a_base + (psc % D) * RAWA,
                                b_base + (psc % D) * RAWB, a_img(psc), b_img(psc), gam, bet, want_bias, bsum, pw,
                                lane);
    } else if (s >= 0) {
      const char* ia = a_img(s);
      const char* ib = b_img(s);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bf16x4 a0 = ldtr4(ia + offA[i][ks][0]), a1 = ldtr4(ia + offA[i][ks][1]);
          const bf16x4 a2 = ldtr4(ia + KT * 256 + offA[i][ks][0]), a3 = ldtr4(ia + KT * 256 + offA[i][ks][1]);
          const bf16x4 b0 = ldtr4(ib + offB[i][ks][0]), b1 = ldtr4(ib + offB[i][ks][1]);
          const bf16x4 b2 = ldtr4(ib + KT * 256 + offB[i][ks][0]), b3 = ldtr4(ib + KT * 256 + offB[i][ks][1]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ah[i][e] = a0[e]; ah[i][4 + e] = a1[e];
            al[i][e] = a2[e]; al[i][4 + e] = a3[e];
            bh[i][e] = b0[e]; bh[i][4 + e] = b1[e];
            bl[i][e] = b2[e]; bl[i][4 + e] = b3[e];
          }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int k = 0; k < 2; ++k) acc[i][k] = mfma_x3(ah[i], al[i], bh[k], bl[k], acc[i][k]);
      }
    }
  }

  // ---- epilogue: the consumers' partial tile; the producers' bias partial ----
  if (!producer) {
    float* pz = part + static_cast<int64_t>(tbz) * Acols * Bcols;
    const int h = lane >> 5, j = lane & 31;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int x = wa + 32 * i + acc_row(r, h);
        const int ra = a_blk + (AF == WG_SPLIT ? split_col(x) : x);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int y = wb + 32 * k + j;
          pz[static_cast<int64_t>(ra) * Bcols + b_blk + (BF == WG_SPLIT ? split_col(y) : y)] = acc[i][k][r];
        }
      }
    }
  }
  if (want_bias) {  // fixed-order sum of the producers' 16 token lanes per column
    __syncthreads();  // the ring is idle: reuse it
    float* red = reinterpret_cast<float*>(lds);  // [16 token lanes][128]
    if (producer) {
      const int tl = 4 * pw + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) red[tl * 128 + 8 * pc + i] = bsum[i];
    }
    __syncthreads();
    if (threadIdx.x < 128) {
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sm += red[k * 128 + threadIdx.x];
      const int x = threadIdx.x;
      bias_part[static_cast<int64_t>(tbz) * Acols + a_blk + (AF == WG_SPLIT ? split_col(x) : x)] = sm;
    }
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
// LDS bytes of a configuration, and the deepest ring <= D that fits the 160 KiB
constexpr int ring_lds(int AF, int BF, int D, int KT) {
  return (AF == WG_SPLIT ? (D + 1) * KT * 512 : D * KT * 512 + 2 * KT * 512) +
         (BF == WG_SPLIT ? (D + 1) * KT * 512 : D * (KT * 512 + (BF == WG_LN ? 1024 : 0)) + 2 * KT * 512);
}
constexpr int fit_d(int AF, int BF, int D, int KT) {
  return D <= 2 || ring_lds(AF, BF, D, KT) <= 160 * 1024 ? D : fit_d(AF, BF, D - 1, KT);
}

template <int AF, int BF, int D0, int KT, int D = fit_d(AF, BF, D0, KT)>
static void wgrad_ring_launch(dim3 grid, hipStream_t s, const void* A, int lda, int64_t a_plane, const void* B,
                              int ldb, int64_t b_plane, const float* stats, const float* lnw, const float* lnb,
                              float* part, float* bias_part, int64_t M, int tps, int Acols, int Bcols) {
  const int ea = AF == WG_SPLIT ? 2 : 4, eb = BF == WG_SPLIT ? 2 : 4;
  hipLaunchKernelGGL((k_wgrad_ring_x3<AF, BF, D, KT>), grid, dim3(512), 0, s, static_cast<const char*>(A), lda * ea,
                     a_plane * ea, static_cast<const char*>(B), ldb * eb, b_plane * eb,
                     reinterpret_cast<const char*>(stats), lnw, lnb, part, bias_part, M, tps, Acols, Bcols);
}

extern "C" int ghm_wgrad_ring_x3(const void* A, int lda, int A_cols, int a_fmt, int64_t a_plane, const void* B,
                                 int ldb, int B_cols, int b_fmt, int64_t b_plane, const float* stats,
                                 const float* ln_w, const float* ln_b, float* part, float* bias_part, int64_t M,
                                 int tok_per_split, void* stream) {
  GHM_CHECK(A && B && part, "null pointer");
  GHM_CHECK(A_cols > 0 && B_cols > 0 && A_cols % 128 == 0 && B_cols % 128 == 0, "A_cols / B_cols % 128");
  GHM_CHECK(lda >= A_cols && ldb >= B_cols && M >= 1, "shape");
  GHM_CHECK(tok_per_split > 0 && tok_per_split % 32 == 0, "tok_per_split must be a positive multiple of 32");
  GHM_CHECK((a_fmt == 0 || a_fmt == 2) && (b_fmt >= 0 && b_fmt <= 2), "formats (A: 0 f32, 2 split; B: 0, 1 ln, 2)");
  GHM_CHECK(!(a_fmt == 2 && b_fmt == 2), "one operand must be f32 (it masks the split tails)");
  GHM_CHECK(b_fmt != 1 || (stats && ln_w && ln_b), "layernorm mode needs stats / ln_w / ln_b");
  GHM_CHECK(a_fmt != 2 || a_plane >= static_cast<int64_t>(M) * lda, "A lo plane overlaps the hi plane");
  GHM_CHECK(b_fmt != 2 || b_plane >= static_cast<int64_t>(M) * ldb, "B lo plane overlaps the hi plane");
  GHM_CHECK((reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(B) & 15) == 0 &&
                (lda * (a_fmt == 2 ? 2 : 4)) % 16 == 0 && (ldb * (b_fmt == 2 ? 2 : 4)) % 16 == 0,
            "operands and their rows must be 16-byte aligned");
  const int64_t nsplit = (M + tok_per_split - 1) / tok_per_split;
  GHM_CHECK(nsplit <= 65535, "too many splits");
  const dim3 grid(A_cols / 128, B_cols / 128, static_cast<unsigned>(nsplit));
  hipStream_t s = ghm_stream(stream);
  // (tokens per step, steps in flight): $GHM_WGRAD_RING_CFG = 0 the default per pairing,
  // 1 (32, 3 or the deepest ring that fits), 2 (16, 4), 3 (16, 6) -- read once per
  // process (A/B runs)
  static const int cfg = [] {
    const char* e = std::getenv("GHM_WGRAD_RING_CFG");
    return e ? std::atoi(e) : 0;
  }();
  const int c = cfg;
#define GHM_RING_CASES(AFV, BFV, DEF)                                                                             \
  {                                                                                                              \
    const int k = c ? c : (DEF);                                                                                 \
    if (k == 1)                                                                                                  \
      wgrad_ring_launch<AFV, BFV, 3, 32>(grid, s, A, lda, a_plane, B, ldb, b_plane, stats, ln_w, ln_b, part,      \
                                         bias_part, M, tok_per_split, A_cols, B_cols);                           \
    else if (k == 2)                                                                                             \
      wgrad_ring_launch<AFV, BFV, 4, 16>(grid, s, A, lda, a_plane, B, ldb, b_plane, stats, ln_w, ln_b, part,      \
                                         bias_part, M, tok_per_split, A_cols, B_cols);                           \
    else                                                                                                         \
      wgrad_ring_launch<AFV, BFV, 6, 16>(grid, s, A, lda, a_plane, B, ldb, b_plane, stats, ln_w, ln_b, part,      \
                                         bias_part, M, tok_per_split, A_cols, B_cols);                           \
  }
  if (a_fmt == 0 && b_fmt == 2)  // dW2 = dY^T G
    GHM_RING_CASES(WG_F32, WG_SPLIT, 1)
  else if (a_fmt == 2 && b_fmt == 1)  // dW1 = dU^T LN2(Hmid)
    GHM_RING_CASES(WG_SPLIT, WG_LN, 1)
  else if (a_fmt == 0 && b_fmt == 1)  // dWq|k|v = dqkv^T LN1(H)
    GHM_RING_CASES(WG_F32, WG_LN, 2)
  else if (a_fmt == 2 && b_fmt == 0)
    GHM_RING_CASES(WG_SPLIT, WG_F32, 2)
  else
    GHM_RING_CASES(WG_F32, WG_F32, 2)
#undef GHM_RING_CASES
  return ghm_launch_status();
}
