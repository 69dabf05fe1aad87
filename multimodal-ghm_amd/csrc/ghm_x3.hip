// Split-bf16 ("x3") token-parallel kernels of the GHM CLIP encoder step (gfx950).
//
// Same data flow, buffers and outputs as the exact-f32 kernels of ghm_fwd.hip /
// ghm_bwd.hip, with every product evaluated as three bf16 MFMAs
// (ghm_split.h).  Weights enter through a per-layer "pack" of pre-split bf16
// planes in the layouts the kernels read (written once per step by
// ghm_split_weights), so the LDS staging of a weight tile is a plain 16-byte
// copy.  Activations are split in registers where they become MFMA operands.
// Reference semantics: src/ghmclip/models/model.py:772-788 (LN1 + Q/K/V,
// LN2 + MLP) and their autograd backward (train_CLIP.py:158).
#include <cstdlib>
#include <cstring>

#include "ghm_common.h"
#include "ghm_ln.h"
#include "ghm_split.h"
#include "ghm_launch.h"

// Timing ablations of k_ln_mlp_fwd_x3b<., false> (experiment builds only; results
// are wrong when set): 1 no weight refill, 2 no GELU, 3 no up-projection MFMAs,
// 4 no down-projection MFMAs, 5 no refill and no per-chunk barrier.
#ifndef GHM_ABL
#define GHM_ABL 0
#endif
#if GHM_ABL != 0 && !defined(GHM_ABLATION_BUILD)
#error "GHM_ABL timing ablations give wrong results: only with -DGHM_ABLATION_BUILD (tools/, never the product library)"
#endif

// 1: k_qkv_bwd_x3 reads the forward's LN1 statistics (system-scope load); 0 (the
// product): it recomputes them from H, one more read of H (+0.85 % of the step,
// r4_ab8).  The recompute stays the default until the wrong-statistics mechanism
// beside k_wgrad_x3 is known (DESIGN.md section 4 "Determinism").
#ifndef GHM_QKV_STATS_LOAD
#define GHM_QKV_STATS_LOAD 0
#endif
#ifndef GHM_WGRAD_FAST
#define GHM_WGRAD_FAST 1  // 0: the run-time-stride weight gradients only (k_wgrad_x3 LDA / LDB = 0)
#endif
// waves per workgroup of the split-K weight gradient (k_wgrad_x3)
#ifndef GHM_WGRAD_WAVES
#define GHM_WGRAD_WAVES 4
#endif
// ---------------------------------------------------------------------------
// Weight pack (bf16 elements per layer; each region = hi plane then lo plane)
// ---------------------------------------------------------------------------
constexpr int PK_QKV = 3 * GHM_D * GHM_D;  // 49152 elements per plane
constexpr int PK_W = GHM_F * GHM_D;        // 65536
constexpr int PK_QKV_N = 0;                // [384][128]: row 128*mat + o, col d   = W_mat[o][d]
constexpr int PK_QKV_T = 2 * PK_QKV;       // [128][384]: row d, col 128*mat + o   = W_mat[o][d]
constexpr int PK_W1_N = 4 * PK_QKV;        // [512][128]: W1[f][d]
constexpr int PK_W1_T = PK_W1_N + 2 * PK_W;  // [128][512]: row d, col q           = W1[perm(q)][d]
constexpr int PK_W2_P = PK_W1_T + 2 * PK_W;  // [128][512]: row o, col q           = W2[o][perm(q)]
constexpr int PK_W2_T = PK_W2_P + 2 * PK_W;  // [512][128]: row f, col o           = W2[o][f]
constexpr int PK_W1_T32 = PK_W2_T + 2 * PK_W;   // [128][512]: row d, col q          = W1[perm32(q)][d]
constexpr int PK_W2_P32 = PK_W1_T32 + 2 * PK_W;  // [128][512]: row o, col q          = W2[o][perm32(q)]
constexpr int PK_ELEMS = PK_W2_P32 + 2 * PK_W;   // 983040
static_assert(PK_ELEMS == GHM_SPLIT_PACK_ELEMS, "pack layout mismatch with include/ghm_hip.h");
// pack3: the third split planes (lo2) of the x6 kernels' weight images, in the pack's layouts
constexpr int PK3_W1_N = 0;                   // [512][128] as PK_W1_N
constexpr int PK3_W2_P32 = PK_W;              // [128][512] as PK_W2_P32
constexpr int PK3_QKV_N = 2 * PK_W;           // [384][128] as PK_QKV_N
constexpr int PK3_ELEMS = 2 * PK_W + PK_QKV;  // 180224
static_assert(PK3_ELEMS == GHM_SPLIT3_PACK_ELEMS, "pack3 layout mismatch with include/ghm_hip.h");

// column permutation inside each 16-group for operands met by an accumulator
// tile (ghm_split.h): position q holds original column perm_col(q)
__device__ __forceinline__ constexpr int perm_col(int q) {
  return (q & ~15) + (q & 3) + 8 * ((q >> 2) & 1) + 4 * ((q >> 3) & 1);
}

// the same for 16x16x32 accumulator operands (ghm_split.h, 16-token tiles):
// k-slot 8g + i of a 32-group holds unit 4g + i (i < 4) or 16 + 4g + i - 4
__device__ __forceinline__ constexpr int perm32(int q) {
  return (q & ~31) + ((q & 7) < 4 ? 4 * ((q >> 3) & 3) + (q & 3) : 16 + 4 * ((q >> 3) & 3) + (q & 3));
}

struct SplitJobs {
  ghm_split_job job[GHM_SPLIT_MAX_JOBS];
};

// inverse of perm32: the k-slot holding unit f
__device__ __forceinline__ constexpr int inv_perm32(int f) {
  return (f & ~31) + ((f >> 3) & 1) * 16 + ((f >> 2) & 1) * 8 + ((f >> 4) & 1) * 4 + (f & 3);
}

// One workgroup per (layer, 64 x 64 tile of one weight matrix): the tile is read
// once, coalesced, into LDS, and written (split) into every pack region that
// holds it, 8 consecutive output columns (16 B per plane) per thread-store.
// Tiles 0-11: Wq / Wk / Wv (2 x 2 each), 12-27: W1 [512][128] (8 x 2), 28-43: W2
// [128][512] (2 x 8).  (The round-1 kernel gathered the transposed layouts with
// one 4-B load per element, 512 B apart: 11 us per tower, latency-bound.)
constexpr int SPLIT_TILES = 44;
__global__ __launch_bounds__(256) void k_split_weights(SplitJobs J) {
  __shared__ float tile[64][65];
  const ghm_split_job& jb = J.job[blockIdx.y];
  const int tix = blockIdx.x, t = threadIdx.x;
  int kind, m = 0, r0, c0, ld;  // kind 0: Q/K/V (m), 1: W1, 2: W2
  const float* W;
  if (tix < 12) {
    kind = 0; m = tix >> 2; r0 = 64 * ((tix & 3) >> 1); c0 = 64 * (tix & 1); ld = GHM_D;
    W = m == 0 ? jb.Wq : (m == 1 ? jb.Wk : jb.Wv);
  } else if (tix < 28) {
    kind = 1; r0 = 64 * ((tix - 12) >> 1); c0 = 64 * ((tix - 12) & 1); ld = GHM_D; W = jb.W1;
  } else {
    kind = 2; r0 = 64 * ((tix - 28) >> 3); c0 = 64 * ((tix - 28) & 7); ld = GHM_F; W = jb.W2;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i4 = t + 256 * k, row = i4 >> 4, col = 4 * (i4 & 15);
    const float4 v = *reinterpret_cast<const float4*>(W + static_cast<int64_t>(r0 + row) * ld + c0 + col);
    tile[row][col] = v.x; tile[row][col + 1] = v.y; tile[row][col + 2] = v.z; tile[row][col + 3] = v.w;
  }
  __syncthreads();
  __bf16* pk = reinterpret_cast<__bf16*>(jb.pack);
  // out(r, q) of a 64 x 64 output block: transposed layouts read tile[src][r],
  // the others tile[r][src], src = the permuted index of q inside the tile
  auto emit = [&](int base, int n, int ld_out, int orow0, int ocol0, bool trans, int perm) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int g = t + 256 * k, r = g >> 3, q0 = 8 * (g & 7);
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int q = q0 + e;
        const int src = perm == 1 ? perm_col(q) : (perm == 2 ? perm32(q) : q);
        v[e] = trans ? tile[src][r] : tile[r][src];
      }
      bf16x8 hi, lo;
      split8(v, hi, lo);
      const int64_t o = base + static_cast<int64_t>(orow0 + r) * ld_out + ocol0 + q0;
      *reinterpret_cast<bf16x8*>(pk + o) = hi;
      *reinterpret_cast<bf16x8*>(pk + o + n) = lo;
    }
  };
  if (kind == 0) {  // [384][128] row 128 m + o, col d; [128][384] row d, col 128 m + o
    emit(PK_QKV_N, PK_QKV, GHM_D, 128 * m + r0, c0, false, 0);
    emit(PK_QKV_T, PK_QKV, 3 * GHM_D, c0, 128 * m + r0, true, 0);
  } else if (kind == 1) {  // W1[f][d]: N; T / T32: row d, col q = W1[perm(q)][d]
    emit(PK_W1_N, PK_W, GHM_D, r0, c0, false, 0);
    emit(PK_W1_T, PK_W, GHM_F, c0, r0, true, 1);
    emit(PK_W1_T32, PK_W, GHM_F, c0, r0, true, 2);
  } else {  // W2[o][f]: P / P32: row o, col q = W2[o][perm(q)]; T: row f, col o
    emit(PK_W2_P, PK_W, GHM_F, r0, c0, false, 1);
    emit(PK_W2_T, PK_W, GHM_D, c0, r0, true, 0);
    emit(PK_W2_P32, PK_W, GHM_F, r0, c0, false, 2);
  }
}

// LN a token row (row layout) and split it into the 8 k-step fragments
__device__ __forceinline__ void ln_row_split(const float* __restrict__ row, const float* __restrict__ lnw,
                                             const float* __restrict__ lnb, int h, float eps, bool active,
                                             bf16x8* xh, bf16x8* xl, float& mean, float& rstd) {
  float x[64];
  if (active) {
    ln_row(row, lnw, lnb, h, eps, x, mean, rstd);
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) x[k] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) split8(x + 8 * t, xh[t], xl[t]);
}

__device__ __forceinline__ void ln_row_split3(const float* __restrict__ row, const float* __restrict__ lnw,
                                              const float* __restrict__ lnb, int h, float eps, bool active,
                                              bf16x8* x0, bf16x8* x1, bf16x8* x2, float& mean, float& rstd) {
  float x[64];
  if (active) {
    ln_row(row, lnw, lnb, h, eps, x, mean, rstd);
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) x[k] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) split3_8(x + 8 * t, x0[t], x1[t], x2[t]);
}

// load a row-layout token vector (64 floats at p) and split it
__device__ __forceinline__ void load_split64(const float* __restrict__ p, bool active, bf16x8* xh, bf16x8* xl) {
  float x[64];
  if (active) {
    load64(p, x);
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) x[k] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) split8(x + 8 * t, xh[t], xl[t]);
}

// ---------------------------------------------------------------------------
// LDS-DMA (global_load_lds_dwordx4) weight tiles: one wave-instruction writes
// 64 x 16 B lane-linearly, so images are unpadded and XOR-swizzled on 16-byte
// chunks; the swizzle goes on each lane's SOURCE address and again on the read
// (conflict-free ds_read_b128):
//   R32  [32 rows][128] (256-B rows):  chunk c of row r at c ^ (r & 15)
//   R128 [128 rows][32] (64-B rows):   chunk c of row r at c ^ s((r >> 2) & 3), s = {0, 2, 3, 1}
//                                      (with s = identity the 16x16x32 operand reads were
//                                      2-way bank conflicted in every ds_read_b128 lane group)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void glds16(const __bf16* src, __bf16* lds_base) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                   (__attribute__((address_space(3))) void*)(lds_base), 16, 0, 0);
}
constexpr int PLANE = 32 * GHM_D;  // bf16 elements of one tile plane (8 KB)
__device__ __forceinline__ int r32_off(int row, int lc) { return row * 128 + 8 * (lc ^ (row & 15)); }
__device__ __forceinline__ int r128_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int r128_off(int row, int lc) { return row * 32 + 8 * (lc ^ r128_swz(row)); }

// ---------------------------------------------------------------------------
// 16-token-per-wave variant of LN2 + MLP (v_mfma_f32_16x16x32_bf16).
// Lane l = (token t = l & 15, group g = l >> 4); a wave owns 16 tokens, a
// 512-thread workgroup 128.  The token row enters as the B operand in 4 k-steps
// of 32 features (lane holds features 32s + 8g + i); accumulators hold 4
// consecutive features 4g + r of a 16-row tile, and a 32-unit hidden chunk
// (two tiles) is the B operand of the down-projection with the perm32 k order
// (weights pre-permuted in the pack).  Weight tiles arrive by LDS-DMA (one
// instruction per wave per plane); the barrier waits only for them (counted
// vmcnt), every lane stores to a real row (lanes past M recompute row M-1), so
// each wave has exactly 4 stores in flight per chunk.
// ---------------------------------------------------------------------------
// NW waves fill a plane: wave b issues the instructions of row groups b, b+NW, ...
template <int NW>
__device__ __forceinline__ void fill_r32_w8(const __bf16* g, int ldg, int lo_off, __bf16* ih, __bf16* il) {
  const int L = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < (8 + NW - 1) / NW; ++k) {
    const int b = (threadIdx.x >> 6) + NW * k;
    if (8 % NW == 0 || b < 8) {
      const int row = 4 * b + (L >> 4), lc = (L & 15) ^ (row & 15);
      const __bf16* src = g + row * ldg + 8 * lc;
      glds16(src, ih + 512 * b);
      glds16(src + lo_off, il + 512 * b);
    }
  }
}
template <int NW>
__device__ __forceinline__ void fill_r128_w8(const __bf16* g, int ldg, int lo_off, __bf16* ih, __bf16* il) {
  const int L = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < (8 + NW - 1) / NW; ++k) {
    const int b = (threadIdx.x >> 6) + NW * k;
    if (8 % NW == 0 || b < 8) {
      const int row = 16 * b + (L >> 2), lc = (L & 3) ^ r128_swz(row);
      const __bf16* src = g + row * ldg + 8 * lc;
      glds16(src, ih + 512 * b);
      glds16(src + lo_off, il + 512 * b);
    }
  }
}

// one plane (the x6 kernels' third, lo2, plane) with fill_r32_w8 / fill_r128_w8's swizzles
template <int NW>
__device__ __forceinline__ void fill_r32_1(const __bf16* g, int ldg, __bf16* ih) {
  const int L = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < (8 + NW - 1) / NW; ++k) {
    const int b = (threadIdx.x >> 6) + NW * k;
    if (8 % NW == 0 || b < 8) {
      const int row = 4 * b + (L >> 4), lc = (L & 15) ^ (row & 15);
      glds16(g + row * ldg + 8 * lc, ih + 512 * b);
    }
  }
}
template <int NW>
__device__ __forceinline__ void fill_r128_1(const __bf16* g, int ldg, __bf16* ih) {
  const int L = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < (8 + NW - 1) / NW; ++k) {
    const int b = (threadIdx.x >> 6) + NW * k;
    if (8 % NW == 0 || b < 8) {
      const int row = 16 * b + (L >> 2), lc = (L & 3) ^ r128_swz(row);
      glds16(g + row * ldg + 8 * lc, ih + 512 * b);
    }
  }
}

// ---------------------------------------------------------------------------
// LN1 + Q/K/V projections                                       (model.py:772-775)
// Wave = 32 tokens (v_mfma_f32_32x32x16_bf16, the LN'd token row split into 8
// k-steps in registers); workgroup = 4 waves.  The 12 weight tiles (32 rows of
// [Wq; Wk; Wv] x 128) arrive by LDS-DMA from the pre-split pack into a
// double-buffered R32 ring (16-B chunk c of row r at c ^ (r & 15): the operand
// reads, row j and chunk 8h + t per lane, are conflict-free).  Round 2 staged
// the tiles through registers; the compiler sank those loads below the MFMAs
// to their LDS stores and waited for them at once (the L2 latency exposed in
// every tile).  Each tile's outputs are stored one tile later, so the
// barrier's vmcnt(0) that retires the next fill never waits for fresh stores.
// ---------------------------------------------------------------------------
// Y^T tile (32 rows x 32 tokens) = A[32][128] . X^T, A from an R32 image pair
__device__ __forceinline__ f32x16 proj_x3_r32(const __bf16* ih, const __bf16* il, int row, int h,
                                              const bf16x8* xh, const bf16x8* xl, f32x16 acc) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int o = r32_off(row, 8 * h + t);
    acc = mfma_x3(ldsb8(ih + o), ldsb8(il + o), xh[t], xl[t], acc);
  }
  return acc;
}

// One weight tile of a 4-wave token-parallel projection: LDS-DMA fill of the
// next tile (global rows at g, pitch ldg, lo plane at +PK_QKV) into ring
// buffer nb, then the product from the current buffer cb.  cb / nb are
// __restrict__ parameters of one inlined function, so the waitcnt pass knows
// the DMA target and the operand reads are disjoint (k_mlp_bwd_rc_x3).
__device__ __forceinline__ f32x16 qkv_tile_x3(const __bf16* __restrict__ cb, __bf16* __restrict__ nb,
                                              const __bf16* g, int ldg, int row, int h, bool active,
                                              const bf16x8* xh, const bf16x8* xl, f32x16 acc) {
  fill_r32_w8<4>(g, ldg, PK_QKV, nb, nb + PLANE);
  if (active) acc = proj_x3_r32(cb, cb + PLANE, row, h, xh, xl, acc);
  return acc;
}

// xs (optional): the split LN1 rows also leave as bf16 (hi, lo) planes [M][128]
// (lo plane M * 128 elements on) for the dWq|k|v weight gradient (k_wgrad_x3 MODE 3)
// tpg: weight tiles per workgroup (12 / tpg workgroups per token block, blockIdx.x =
// token block * (12 / tpg) + group): for token counts too small to fill the chip
// (the CDM's 10.5 K tokens: 82 token blocks on 256 CUs) each group recomputes the
// LayerNorm and writes its own 32-column tiles; group 0 writes the statistics
__global__ __launch_bounds__(256, 2) void k_ln_qkv_fwd_x3(
    const float* __restrict__ H, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const __bf16* pack, float* __restrict__ qkv, float2* __restrict__ stats, int64_t M,
    float eps, __bf16* __restrict__ xs, int tpg) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[4 * PLANE];  // 2 buffers x (hi, lo)
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int ngrp = 12 / tpg, grp = static_cast<int>(blockIdx.x) % ngrp;
  const int b0 = grp * tpg, b1 = b0 + tpg;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x / ngrp) * 4 + (threadIdx.x >> 6)) * 32;
  const bool active = m0 < M;
  const int64_t m = m0 + j;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W = pack + PK_QKV_N;
  fill_r32_w8<4>(W + b0 * 32 * GHM_D, GHM_D, PK_QKV, lds, lds + PLANE);  // tile b0, in flight over the LayerNorm
  bf16x8 xh[8], xl[8];
  {
    float mean = 0.f, rstd = 0.f;
    ln_row_split(H + mc * GHM_D, lnw, lnb, h, eps, active, xh, xl, mean, rstd);
    if (active && h == 0 && valid && grp == 0) stats[m] = make_float2(mean, rstd);
    if (xs && active && valid && grp == 0) {  // features 64 h + 8 t .. + 7: 8 chunks per plane
      __bf16* xr = xs + m * GHM_D + 64 * h;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        *reinterpret_cast<bf16x8*>(xr + 8 * t) = xh[t];
        *reinterpret_cast<bf16x8*>(xr + M * GHM_D + 8 * t) = xl[t];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  f32x16 prev = zero16();
  float* orow = qkv + m * (3 * GHM_D);
#pragma unroll 1
  for (int b = b0; b < b1; ++b) {  // tile b = rows 32b..32b+31 of [Wq; Wk; Wv]
    const int cur = (b - b0) & 1;
    if (b > b0 && active && valid) {  // tile b - 1's outputs
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st4(orow + 32 * (b - 1) + quad_off(q, h), prev[4 * q], prev[4 * q + 1], prev[4 * q + 2], prev[4 * q + 3]);
    }
    const int bn = b + 1 < b1 ? b + 1 : b1 - 1;  // branch-free: the last tile refills itself
    prev = qkv_tile_x3(lds + 2 * PLANE * cur, lds + 2 * PLANE * (cur ^ 1), W + bn * 32 * GHM_D, GHM_D, j, h,
                       active, xh, xl, zero16());
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (active && valid) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      st4(orow + 32 * (b1 - 1) + quad_off(q, h), prev[4 * q], prev[4 * q + 1], prev[4 * q + 2], prev[4 * q + 3]);
  }
}

// weight tiles per workgroup of the LN1 + QKV forwards: all 12 when the token blocks
// alone give every CU a workgroup; else split over 2, 3 or 4 groups of tiles
static int qkv_tiles_per_group(int64_t M) {
  const char* e = getenv("GHM_QKV_TPG");  // A/B knob: 12, 6, 4 or 3
  if (e) {
    const int t = atoi(e);
    if (t == 12 || t == 6 || t == 4 || t == 3) return t;
  }
  const int64_t nb = ghm_token_blocks(M);
  return nb >= 256 ? 12 : nb >= 128 ? 6 : nb >= 86 ? 4 : 3;
}

// qkv_tile_x3 on three planes (cb / nb __restrict__ for the same reason)
__device__ __forceinline__ f32x16 qkv_tile_x6(const __bf16* __restrict__ cb, __bf16* __restrict__ nb,
                                              const __bf16* g, const __bf16* gc, int row, int h, bool active,
                                              const bf16x8* x0, const bf16x8* x1, const bf16x8* x2) {
  fill_r32_w8<4>(g, GHM_D, PK_QKV, nb, nb + PLANE);
  fill_r32_1<4>(gc, GHM_D, nb + 2 * PLANE);
  f32x16 acc = zero16();
  if (active) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int o = r32_off(row, 8 * h + t);
      acc = mfma_x6(ldsb8(cb + o), ldsb8(cb + PLANE + o), ldsb8(cb + 2 * PLANE + o), x0[t], x1[t], x2[t], acc);
    }
  }
  return acc;
}

// LN1 + Q/K/V on three-way split operands (the "f32fwd" precision's qkv6 stage):
// k_ln_qkv_fwd_x3 with six bf16 MFMAs per product (mfma_x6) and the weights' third
// plane from pack3 (PK3_QKV_N); the ring holds three planes per buffer (48 KB).
__global__ __launch_bounds__(256, 2) void k_ln_qkv_fwd_x6(
    const float* __restrict__ H, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const __bf16* pack, const __bf16* pack3, float* __restrict__ qkv, float2* __restrict__ stats, int64_t M,
    float eps, int tpg) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[6 * PLANE];  // 2 buffers x (hi, lo, lo2)
  const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int ngrp = 12 / tpg, grp = static_cast<int>(blockIdx.x) % ngrp;  // (k_ln_qkv_fwd_x3)
  const int b0 = grp * tpg, b1 = b0 + tpg;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x / ngrp) * 4 + (threadIdx.x >> 6)) * 32;
  const bool active = m0 < M;
  const int64_t m = m0 + j;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W = pack + PK_QKV_N;
  const __bf16* Wc = pack3 + PK3_QKV_N;
  fill_r32_w8<4>(W + b0 * 32 * GHM_D, GHM_D, PK_QKV, lds, lds + PLANE);  // tile b0, in flight over the LayerNorm
  fill_r32_1<4>(Wc + b0 * 32 * GHM_D, GHM_D, lds + 2 * PLANE);
  bf16x8 x0[8], x1[8], x2[8];
  {
    float mean = 0.f, rstd = 0.f;
    ln_row_split3(H + mc * GHM_D, lnw, lnb, h, eps, active, x0, x1, x2, mean, rstd);
    if (active && h == 0 && valid && grp == 0) stats[m] = make_float2(mean, rstd);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  f32x16 prev = zero16();
  float* orow = qkv + m * (3 * GHM_D);
#pragma unroll 1
  for (int b = b0; b < b1; ++b) {  // tile b = rows 32b..32b+31 of [Wq; Wk; Wv]
    const int cur = (b - b0) & 1;
    if (b > b0 && active && valid) {  // tile b - 1's outputs
#pragma unroll
      for (int q = 0; q < 4; ++q)
        st4(orow + 32 * (b - 1) + quad_off(q, h), prev[4 * q], prev[4 * q + 1], prev[4 * q + 2], prev[4 * q + 3]);
    }
    const int bn = b + 1 < b1 ? b + 1 : b1 - 1;  // branch-free: the last tile refills itself
    prev = qkv_tile_x6(lds + 3 * PLANE * cur, lds + 3 * PLANE * (cur ^ 1), W + bn * 32 * GHM_D,
                       Wc + bn * 32 * GHM_D, j, h, active, x0, x1, x2);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (active && valid) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      st4(orow + 32 * (b1 - 1) + quad_off(q, h), prev[4 * q], prev[4 * q + 1], prev[4 * q + 2], prev[4 * q + 3]);
  }
}

// pick element 4g + r of a wave-uniform 16-float group (scalar registers)
__device__ __forceinline__ float pick16(const float4* b4, int g, int r) {
  const float v0 = (&b4[0].x)[r], v1 = (&b4[1].x)[r], v2 = (&b4[2].x)[r], v3 = (&b4[3].x)[r];
  return g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
}

// NW = waves per workgroup (8: 128 tokens; 4: 64 tokens, for token counts too
// small to fill 256 CUs with 128-token workgroups).  Measured: a 7-wave /
// 112-token variant (463 workgroups instead of 405) runs 96.6 us vs 79.1 us at
// the CLIP's 51,840 tokens.  Only H_out (and the LN statistics) leave the chip:
// the backward recomputes U (k_mlp_bwd_rc_x3), 2 x [M,128] of HBM traffic
// instead of 2 x [M,128] + 2 x [M,512] with G and GELU'(U) saved.
// xs (optional): the split LN2 rows also leave as bf16 (hi, lo) planes [M][128] (lo
// plane M * 128 elements on) for the dW1 weight gradient (k_wgrad_x3 MODE 3)
template <int NW>
__global__ __launch_bounds__(64 * NW, 2) void k_ln_mlp_fwd_x3b(
    const float* __restrict__ Hmid, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const __bf16* pack, const float* __restrict__ b1, const float* __restrict__ b2,
    float* __restrict__ Hout, float2* __restrict__ stats, int64_t M, float eps, __bf16* __restrict__ xs) {
  // ONE __shared__ object: [W1 hi|lo][W2 hi|lo] x 2 buffers, then b1 (f32).  The
  // chunk's b1 values are read at the top of the iteration, before its LDS-DMA
  // fills: any LDS read issued after them gets an s_waitcnt vmcnt(0) on the new
  // fills (the compiler cannot prove it disjoint from the DMA target; a separate
  // __shared__ object for b1 made it wait before EVERY ring read instead).
  __shared__ __attribute__((aligned(16))) __bf16 lds[8 * PLANE + 2 * GHM_F];
  float* sb1 = reinterpret_cast<float*>(lds + 8 * PLANE);
  auto s1h = [&](int buf) { return lds + 4 * PLANE * buf; };
  auto s1l = [&](int buf) { return lds + 4 * PLANE * buf + PLANE; };
  auto s2h = [&](int buf) { return lds + 4 * PLANE * buf + 2 * PLANE; };
  auto s2l = [&](int buf) { return lds + 4 * PLANE * buf + 3 * PLANE; };
  constexpr int NC = GHM_F / 32;
  const int lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int64_t m = (static_cast<int64_t>(blockIdx.x) * NW + (threadIdx.x >> 6)) * 16 + t;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W1 = pack + PK_W1_N;
  const __bf16* W2 = pack + PK_W2_P32;
  fill_r32_w8<NW>(W1, GHM_D, PK_W, s1h(0), s1l(0));
  fill_r128_w8<NW>(W2, GHM_F, PK_W, s2h(0), s2l(0));
  if (threadIdx.x < GHM_F / 4)  // b1 -> LDS: each lane reads its 4 hidden units as one float4
    reinterpret_cast<float4*>(sb1)[threadIdx.x] = reinterpret_cast<const float4*>(b1)[threadIdx.x];
  // LN2 of the token row, lane holds features 32s + 8g + i
  bf16x8 xh[4], xl[4];
  {
    const float* row = Hmid + mc * GHM_D;
    float x[32];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const float4 a = *reinterpret_cast<const float4*>(row + 32 * s2 + 8 * g);
      const float4 b = *reinterpret_cast<const float4*>(row + 32 * s2 + 8 * g + 4);
      x[8 * s2 + 0] = a.x; x[8 * s2 + 1] = a.y; x[8 * s2 + 2] = a.z; x[8 * s2 + 3] = a.w;
      x[8 * s2 + 4] = b.x; x[8 * s2 + 5] = b.y; x[8 * s2 + 6] = b.z; x[8 * s2 + 7] = b.w;
    }
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) sm += x[k];
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    const float mean = sm * (1.f / 128.f);
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const float d = x[k] - mean;
      v += d * d;
    }
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const float rstd = 1.f / sqrtf(v * (1.f / 128.f) + eps);
    if (g == 0 && valid) stats[m] = make_float2(mean, rstd);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int f = 32 * s2 + 8 * g + i;
        x[8 * s2 + i] = (x[8 * s2 + i] - mean) * rstd * lnw[f] + lnb[f];
      }
      split8(x + 8 * s2, xh[s2], xl[s2]);
    }
    if (xs && valid) {  // features 32 s2 + 8 g .. + 7: 4 chunks per plane
      __bf16* xr = xs + m * GHM_D + 8 * g;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        *reinterpret_cast<bf16x8*>(xr + 32 * s2) = xh[s2];
        *reinterpret_cast<bf16x8*>(xr + M * GHM_D + 32 * s2) = xl[s2];
      }
    }
  }
  // the residual and b2 seed the accumulators (H = Hmid + b2 + sum_c W2[:, c] G_c):
  // the rows were just read (L1 / L2-hot), so the epilogue needs no second read of
  // Hmid, which the 16 chunks' traffic had evicted from the L2 (an extra 26 MB
  // per launch, profiles/r3_v10_traffic.txt)
  f32x4 y[8];
  __builtin_amdgcn_sched_barrier(0);  // (after the LN block: its 32 row values are dead by now)
  {
    const float* hr = Hmid + mc * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * j + 4 * g;
      const float4 hv = *reinterpret_cast<const float4*>(hr + f);
      const float4 bv = *reinterpret_cast<const float4*>(b2 + f);
      y[j][0] = hv.x + bv.x;
      y[j][1] = hv.y + bv.y;
      y[j][2] = hv.z + bv.z;
      y[j][3] = hv.w + bv.w;
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const int cur = c & 1;
    float4 bb[2];  // b1 of hidden units 32c + 16jt + 4g + r
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) bb[jt] = lds4(sb1 + 32 * c + 16 * jt + 4 * g);
    issue_fence();
#if GHM_ABL != 1 && GHM_ABL != 5
    {  // branch-free: the last iteration refills chunk NC-1 into the idle buffer
      const int cn = c + 1 < NC ? c + 1 : NC - 1;
      fill_r32_w8<NW>(W1 + cn * 32 * GHM_D, GHM_D, PK_W, s1h(cur ^ 1), s1l(cur ^ 1));
      fill_r128_w8<NW>(W2 + cn * 32, GHM_F, PK_W, s2h(cur ^ 1), s2l(cur ^ 1));
    }
#endif
    f32x4 u[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      u[jt] = zero4();
#pragma unroll
      for (int s2 = 0; s2 < 4 * (GHM_ABL != 3); ++s2) {
        const int o = r32_off(16 * jt + t, 4 * s2 + g);
        u[jt] = mfma16_x3(ldsb8(s1h(cur) + o), ldsb8(s1l(cur) + o), xh[s2], xl[s2], u[jt]);
      }
    }
    float gv[8], dg[8];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {  // + b1
      gv[4 * jt + 0] = u[jt][0] + bb[jt].x;
      gv[4 * jt + 1] = u[jt][1] + bb[jt].y;
      gv[4 * jt + 2] = u[jt][2] + bb[jt].z;
      gv[4 * jt + 3] = u[jt][3] + bb[jt].w;
    }
#pragma unroll
    for (int r = 0; r < 8 * (GHM_ABL != 2); ++r) gelu_fast(gv[r], gv[r], dg[r]);
    bf16x8 gh, gl;
    split8(gv, gh, gl);
#pragma unroll
    for (int j = 0; j < 8 * (GHM_ABL != 4); ++j) {
      const int o = r128_off(16 * j + t, g);
      y[j] = mfma16_x3(ldsb8(s2h(cur) + o), ldsb8(s2l(cur) + o), gh, gl, y[j]);
    }
    // retire this iteration's LDS-DMA fills.  vmcnt(0) rather than the round-2
    // vmcnt(4) that skipped the stores issued after the fills: that count is
    // right only if loads, LDS-DMA and stores retire in issue order (as
    // MI355X_MICROARCH.md states), which LLVM's own waitcnt insertion does not
    // assume for mixed pending loads and stores; the wait that holds under both
    // models measured no slower (4.38 / 4.41 vs 4.38 / 4.39 ms/step,
    // profiles/r3_probe.txt; DESIGN.md §4 "Determinism").
    if (GHM_ABL != 5)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (valid) {
    float* orow = Hout + m * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) st4(orow + 16 * j + 4 * g, y[j][0], y[j][1], y[j][2], y[j][3]);
  }
}

// ---------------------------------------------------------------------------
// LN2 + MLP forward on three-way split operands (the "f32fwd" precision's MLP stage
// as `mlp6`): the k_ln_mlp_fwd_x3b schedule with every product as six bf16 MFMAs
// (mfma16_x6, ~2^-24 relative: the exact-f32 kernel's level, on the bf16 pipe)
// instead of three, and the exact GELU of the f32 kernel.  The weights' third
// planes come from pack3 ([W1 n | W2 p32] lo2 planes in the pack's layouts, written
// by ghm_split3_weights); the LDS ring holds six planes per buffer (96 KB
// double-buffered): one 8-wave workgroup per CU.
// ---------------------------------------------------------------------------
// SAVE: also store G = GELU(U) and Dg = GELU'(U) [M][512] (f32, natural columns) for
// an exact-f32 backward (ghm_mlp_bwd; precision "f32x6")
template <int NW, bool SAVE>
__global__ __launch_bounds__(64 * NW, 1) void k_ln_mlp_fwd_x6(
    const float* __restrict__ Hmid, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const __bf16* pack, const __bf16* pack3, const float* __restrict__ b1, const float* __restrict__ b2,
    float* __restrict__ Hout, float2* __restrict__ stats, int64_t M, float eps, float* __restrict__ G,
    float* __restrict__ Dg) {
  // ONE __shared__ object (see k_ln_mlp_fwd_x3b): [W1 hi|lo|lo2][W2 hi|lo|lo2] x 2, b1
  __shared__ __attribute__((aligned(16))) __bf16 lds[12 * PLANE + 2 * GHM_F];
  float* sb1 = reinterpret_cast<float*>(lds + 12 * PLANE);
  auto s1 = [&](int buf, int q) { return lds + 6 * PLANE * buf + q * PLANE; };
  auto s2 = [&](int buf, int q) { return lds + 6 * PLANE * buf + (3 + q) * PLANE; };
  constexpr int NC = GHM_F / 32;
  const int lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int64_t m = (static_cast<int64_t>(blockIdx.x) * NW + (threadIdx.x >> 6)) * 16 + t;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W1 = pack + PK_W1_N;
  const __bf16* W2 = pack + PK_W2_P32;
  const __bf16* W1c = pack3;         // W1 lo2, [512][128]
  const __bf16* W2c = pack3 + PK_W;  // W2 lo2, [128][512] perm32 columns
  fill_r32_w8<NW>(W1, GHM_D, PK_W, s1(0, 0), s1(0, 1));
  fill_r32_1<NW>(W1c, GHM_D, s1(0, 2));
  fill_r128_w8<NW>(W2, GHM_F, PK_W, s2(0, 0), s2(0, 1));
  fill_r128_1<NW>(W2c, GHM_F, s2(0, 2));
  if (threadIdx.x < GHM_F / 4)
    reinterpret_cast<float4*>(sb1)[threadIdx.x] = reinterpret_cast<const float4*>(b1)[threadIdx.x];
  // LN2 of the token row, lane holds features 32s + 8g + i, split three ways
  bf16x8 x0[4], x1[4], x2[4];
  {
    const float* row = Hmid + mc * GHM_D;
    float x[32];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const float4 a = *reinterpret_cast<const float4*>(row + 32 * s2 + 8 * g);
      const float4 b = *reinterpret_cast<const float4*>(row + 32 * s2 + 8 * g + 4);
      x[8 * s2 + 0] = a.x; x[8 * s2 + 1] = a.y; x[8 * s2 + 2] = a.z; x[8 * s2 + 3] = a.w;
      x[8 * s2 + 4] = b.x; x[8 * s2 + 5] = b.y; x[8 * s2 + 6] = b.z; x[8 * s2 + 7] = b.w;
    }
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) sm += x[k];
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    const float mean = sm * (1.f / 128.f);
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const float d = x[k] - mean;
      v += d * d;
    }
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const float rstd = 1.f / sqrtf(v * (1.f / 128.f) + eps);
    if (g == 0 && valid) stats[m] = make_float2(mean, rstd);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int f = 32 * s2 + 8 * g + i;
        x[8 * s2 + i] = (x[8 * s2 + i] - mean) * rstd * lnw[f] + lnb[f];
      }
      split3_8(x + 8 * s2, x0[s2], x1[s2], x2[s2]);
    }
  }
  // the MLP's own sum from zero; the residual and b2 are added once at the end
  f32x4 y[8];
  __builtin_amdgcn_sched_barrier(0);  // (after the LN block, as k_ln_mlp_fwd_x3b)
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = zero4();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const int cur = c & 1;
    float4 bb[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) bb[jt] = lds4(sb1 + 32 * c + 16 * jt + 4 * g);
    issue_fence();
    {  // branch-free: the last iteration refills chunk NC-1 into the idle buffer
      const int cn = c + 1 < NC ? c + 1 : NC - 1;
      fill_r32_w8<NW>(W1 + cn * 32 * GHM_D, GHM_D, PK_W, s1(cur ^ 1, 0), s1(cur ^ 1, 1));
      fill_r32_1<NW>(W1c + cn * 32 * GHM_D, GHM_D, s1(cur ^ 1, 2));
      fill_r128_w8<NW>(W2 + cn * 32, GHM_F, PK_W, s2(cur ^ 1, 0), s2(cur ^ 1, 1));
      fill_r128_1<NW>(W2c + cn * 32, GHM_F, s2(cur ^ 1, 2));
    }
    // the products chain into accumulators that start from zero (u per chunk, y over
    // all chunks): an MFMA adding small products into a much larger accumulator drops
    // their low bits, so y is not seeded with the residual as in k_ln_mlp_fwd_x3b
    // (measured against float64: residual-seeded 8.3e-6 -- the split-bf16 kernel's
    // 1.1e-5 level; zero-started six-product groups added on the VALU 2.0e-6; chained
    // from zero with the residual added at the end 8.0e-7, the f32 kernel 1.05e-6)
    f32x4 u[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      u[jt] = zero4();
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int o = r32_off(16 * jt + t, 4 * s2 + g);
        u[jt] = mfma16_x6(ldsb8(s1(cur, 0) + o), ldsb8(s1(cur, 1) + o), ldsb8(s1(cur, 2) + o), x0[s2], x1[s2],
                          x2[s2], u[jt]);
      }
    }
    float gv[8];
    if constexpr (SAVE) {  // gv[4 jt + r] is unit 32c + 16 jt + 4g + r of token m
      float dv[8];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        const float bs[4] = {bb[jt].x, bb[jt].y, bb[jt].z, bb[jt].w};
#pragma unroll
        for (int r = 0; r < 4; ++r) gelu_and_grad(u[jt][r] + bs[r], gv[4 * jt + r], dv[4 * jt + r]);
      }
      if (valid) {
        float* grow = G + m * GHM_F + 32 * c + 4 * g;
        float* drow = Dg + m * GHM_F + 32 * c + 4 * g;
        st4(grow, gv[0], gv[1], gv[2], gv[3]);
        st4(grow + 16, gv[4], gv[5], gv[6], gv[7]);
        st4(drow, dv[0], dv[1], dv[2], dv[3]);
        st4(drow + 16, dv[4], dv[5], dv[6], dv[7]);
      }
    } else {
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        gv[4 * jt + 0] = gelu_f(u[jt][0] + bb[jt].x);
        gv[4 * jt + 1] = gelu_f(u[jt][1] + bb[jt].y);
        gv[4 * jt + 2] = gelu_f(u[jt][2] + bb[jt].z);
        gv[4 * jt + 3] = gelu_f(u[jt][3] + bb[jt].w);
      }
    }
    bf16x8 g0, g1, g2;
    split3_8(gv, g0, g1, g2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = r128_off(16 * j + t, g);
      y[j] = mfma16_x6(ldsb8(s2(cur, 0) + o), ldsb8(s2(cur, 1) + o), ldsb8(s2(cur, 2) + o), g0, g1, g2, y[j]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (valid) {
    float* orow = Hout + m * GHM_D;
    {  // the residual and b2 added once, on the VALU, to the MLP's own sum
      const float* hr = Hmid + m * GHM_D;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 16 * j + 4 * g;
        const float4 hv = *reinterpret_cast<const float4*>(hr + f);
        const float4 bv = *reinterpret_cast<const float4*>(b2 + f);
        y[j][0] = hv.x + (y[j][0] + bv.x);
        y[j][1] = hv.y + (y[j][1] + bv.y);
        y[j][2] = hv.z + (y[j][2] + bv.z);
        y[j][3] = hv.w + (y[j][3] + bv.w);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) st4(orow + 16 * j + 4 * g, y[j][0], y[j][1], y[j][2], y[j][3]);
  }
}

// The lo2 planes of pack3 (the third split planes of the x6 kernels' weight images):
// [0, PK_W): W1 in the pack's W1_N layout (row f, col d); [PK_W, 2 PK_W): W2 in its
// W2_P32 layout (row o, col q = W2[o][perm32(q)]).  One thread per element of each.
__device__ __forceinline__ __bf16 lo2_of(float v) {
  const __bf16 a = static_cast<__bf16>(v);
  const float r = v - static_cast<float>(a);
  const __bf16 b = static_cast<__bf16>(r);
  return static_cast<__bf16>(r - static_cast<float>(b));
}
// blocks [0, PK_W / 256): W1 and W2 element i; [PK_W / 256, + PK_QKV / 256): the
// [Wq; Wk; Wv] image element i (row 128 mat + o, col d = W_mat[o][d])
__global__ __launch_bounds__(256) void k_split3_weights(SplitJobs J) {
  const ghm_split_job& jb = J.job[blockIdx.y];
  __bf16* out = static_cast<__bf16*>(jb.pack);
  if (blockIdx.x < PK_W / 256) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    out[PK3_W1_N + i] = lo2_of(jb.W1[i]);
    out[PK3_W2_P32 + i] = lo2_of(jb.W2[(i >> 9) * GHM_F + perm32(i & 511)]);
  } else {
    const int i = (blockIdx.x - PK_W / 256) * 256 + threadIdx.x, r = i >> 7, mat = r >> 7;
    const float* W = mat == 0 ? jb.Wq : (mat == 1 ? jb.Wk : jb.Wv);
    out[PK3_QKV_N + i] = lo2_of(W[(r & 127) * GHM_D + (i & 127)]);
  }
}

// ---------------------------------------------------------------------------
// Wave-specialised LN2 + MLP forward (8 waves, 128 tokens per workgroup).
// The same products as k_ln_mlp_fwd_x3b, scheduled so that the two waves a
// SIMD holds (waves w and w + 4 of a workgroup sit on one SIMD) are in opposite
// phases: an M phase (the chunk's down-projection Y += W2(c-1) G(c-1) and the
// next up-projection U(c) = W1(c) X: 48 MFMAs, 32 operand reads) and a V phase
// (G(c) = GELU(U(c) + b1) and its split: VALU only).  Waves 0-3 run
// M(p), V(p), M(p+1), ... and waves 4-7 the same one interval later; the
// intervals are separated by s_barrier, so the compiler cannot merge the two
// phases of one wave (the software-pipelined x3b variants of rounds 3-4 lost
// because the scheduler re-clustered the MFMAs).  Ring: interval pair p (2p,
// 2p+1) reads slot p & 1 = {W1(p), W2(p-1)}; the fills of pair p + 1 are issued
// at the start of interval 2p into the other slot, which pair p - 1 released
// at the barrier ending interval 2p - 1, and retired at the barrier ending
// interval 2p + 1: the same 64 KB double buffer as x3b.
// ---------------------------------------------------------------------------
struct WsState {
  f32x4 u[2];
  bf16x8 gh, gl;
};

// M phase on ring slot cb (W1 hi|lo, W2 hi|lo): Y += W2 G (DOWN) and U = W1 X (UP)
template <bool DOWN, bool UP>
__device__ __forceinline__ void ws_mphase(const __bf16* __restrict__ cb, const bf16x8* xh, const bf16x8* xl,
                                          f32x4* y, WsState& st, int t, int g) {
  __builtin_amdgcn_iglp_opt(0);  // interleave the operand reads with the MFMAs
  if (DOWN) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = r128_off(16 * j + t, g);
      y[j] = mfma16_x3(ldsb8(cb + 2 * PLANE + o), ldsb8(cb + 3 * PLANE + o), st.gh, st.gl, y[j]);
    }
  }
  if (UP) {
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      st.u[jt] = zero4();
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int o = r32_off(16 * jt + t, 4 * s2 + g);
        st.u[jt] = mfma16_x3(ldsb8(cb + o), ldsb8(cb + PLANE + o), xh[s2], xl[s2], st.u[jt]);
      }
    }
  }
}

// The same with every operand read issued before the first MFMA (64 VGPRs per
// product): the scheduler otherwise keeps one read ahead and waits lgkmcnt(0)
// every 3 MFMAs; here the waits count down (lgkmcnt(N)) while the MFMAs run.
// For the 256-VGPR build (one workgroup per CU) only.
template <bool DOWN, bool UP>
__device__ __forceinline__ void ws_mphase_deep(const __bf16* __restrict__ cb, const bf16x8* xh, const bf16x8* xl,
                                               f32x4* y, WsState& st, int t, int g) {
  bf16x8 dh[8], dl[8], uh[8], ul[8];
  if (DOWN) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = r128_off(16 * j + t, g);
      dh[j] = ldsb8(cb + 2 * PLANE + o);
      dl[j] = ldsb8(cb + 3 * PLANE + o);
    }
  }
  if (UP) {
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int o = r32_off(16 * jt + t, 4 * s2 + g);
        uh[4 * jt + s2] = ldsb8(cb + o);
        ul[4 * jt + s2] = ldsb8(cb + PLANE + o);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (DOWN) {
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = mfma16_x3(dh[j], dl[j], st.gh, st.gl, y[j]);
  }
  if (UP) {
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      st.u[jt] = zero4();
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
        st.u[jt] = mfma16_x3(uh[4 * jt + s2], ul[4 * jt + s2], xh[s2], xl[s2], st.u[jt]);
    }
  }
}

// V phase: G = GELU(U + b1) -> (gh, gl)
__device__ __forceinline__ void ws_vphase(const float4* bb, WsState& st) {
  float gv[8], dg[8];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    gv[4 * jt + 0] = st.u[jt][0] + bb[jt].x;
    gv[4 * jt + 1] = st.u[jt][1] + bb[jt].y;
    gv[4 * jt + 2] = st.u[jt][2] + bb[jt].z;
    gv[4 * jt + 3] = st.u[jt][3] + bb[jt].w;
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) gelu_fast(gv[r], gv[r], dg[r]);
  split8(gv, st.gh, st.gl);
}

// the interval barriers are scheduling barriers too: without sched_barrier the
// machine scheduler moved the (memory-free) GELU VALU and the last MFMAs of a
// phase across the asm s_barrier into the next interval
__device__ __forceinline__ void ws_bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void ws_bar_fills() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// fills of pair p + 1 = {W1(p + 1), W2(p)} into ring slot nb
template <int NW>
__device__ __forceinline__ void ws_fill(__bf16* nb, const __bf16* W1, const __bf16* W2, int p) {
  constexpr int NC = GHM_F / 32;
  if (p + 1 < NC) fill_r32_w8<NW>(W1 + (p + 1) * 32 * GHM_D, GHM_D, PK_W, nb, nb + PLANE);
  fill_r128_w8<NW>(W2 + p * 32, GHM_F, PK_W, nb + 2 * PLANE, nb + 3 * PLANE);
}

// one interval pair 0 < p < NC, straight-line per group: fills of pair p + 1,
// then A: M(p) | V(p), B: V(p-1) | M(p).  cb / nb: __restrict__ parameters of one
// inlined function (alias scopes: no vmcnt wait for the fresh fills before the
// operand reads)
template <bool DEEP, bool DOWN, bool UP>
__device__ __forceinline__ void ws_m(const __bf16* __restrict__ cb, const bf16x8* xh, const bf16x8* xl, f32x4* y,
                                     WsState& st, int t, int g) {
  if (DEEP)
    ws_mphase_deep<DOWN, UP>(cb, xh, xl, y, st, t, g);
  else
    ws_mphase<DOWN, UP>(cb, xh, xl, y, st, t, g);
}

template <int NW, bool GRP_A, bool DEEP = false>
__device__ __forceinline__ void ws_pair(const __bf16* __restrict__ cb, __bf16* __restrict__ nb, int p,
                                        const __bf16* W1, const __bf16* W2, const float4* bb, const bf16x8* xh,
                                        const bf16x8* xl, f32x4* y, WsState& st, int t, int g) {
  ws_fill<NW>(nb, W1, W2, p);
  if (GRP_A) {
    ws_m<DEEP, true, true>(cb, xh, xl, y, st, t, g);
    ws_bar();
    ws_vphase(bb, st);
  } else {
    ws_vphase(bb, st);
    ws_bar();
    ws_m<DEEP, true, true>(cb, xh, xl, y, st, t, g);
  }
  ws_bar_fills();
}

// a group's whole chunk loop: pair 0 (U(0) only), pairs 1 .. NC-1, pair NC (Y(NC-1) only)
template <int NW, bool GRP_A, bool DEEP = false>
__device__ __forceinline__ void ws_loop(__bf16* lds, const __bf16* W1, const __bf16* W2, const float* sb1,
                                        const bf16x8* xh, const bf16x8* xl, f32x4* y, int t, int g) {
  constexpr int NC = GHM_F / 32;
  WsState st;
  float4 bb[2];
  auto read_b1 = [&](int q) {  // b1 of chunk q, read before the pair's fills (see k_ln_mlp_fwd_x3b)
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) bb[jt] = lds4(sb1 + 32 * q + 16 * jt + 4 * g);
    issue_fence();
  };
  // pair 0: slot 0 = {W1(0)}
  if (GRP_A) read_b1(0);
  ws_fill<NW>(lds + 4 * PLANE, W1, W2, 0);
  if (GRP_A) {
    ws_m<DEEP, false, true>(lds, xh, xl, y, st, t, g);
    ws_bar();
    ws_vphase(bb, st);
  } else {
    ws_bar();
    ws_m<DEEP, false, true>(lds, xh, xl, y, st, t, g);
  }
  ws_bar_fills();
#pragma unroll 1
  for (int p = 1; p < NC; ++p) {
    const int cur = p & 1;
    read_b1(GRP_A ? p : p - 1);
    ws_pair<NW, GRP_A, DEEP>(lds + 4 * PLANE * cur, lds + 4 * PLANE * (cur ^ 1), p, W1, W2, bb, xh, xl, y, st, t, g);
  }
  // pair NC: slot NC & 1 = {W2(NC-1)}
  const __bf16* cb = lds + 4 * PLANE * (NC & 1);
  if (GRP_A) {
    ws_m<DEEP, true, false>(cb, xh, xl, y, st, t, g);
    ws_bar();
  } else {
    read_b1(NC - 1);
    ws_vphase(bb, st);
    ws_bar();
    ws_m<DEEP, true, false>(cb, xh, xl, y, st, t, g);
  }
  ws_bar();
}

// 4 waves per SIMD (HIP's second bound: minimum waves per EU), i.e. two
// workgroups per CU as x3b; at the bound 2 the compiler spent 153 VGPRs (one
// workgroup per CU)
template <int NW, int MINW = 4>
__global__ __launch_bounds__(64 * NW, MINW) void k_ln_mlp_fwd_x3w(
    const float* __restrict__ Hmid, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const __bf16* pack, const float* __restrict__ b1, const float* __restrict__ b2,
    float* __restrict__ Hout, float2* __restrict__ stats, int64_t M, float eps) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[8 * PLANE + 2 * GHM_F];
  float* sb1 = reinterpret_cast<float*>(lds + 8 * PLANE);
  const int lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const bool grpA = wave < NW / 2;
  const int64_t m = (static_cast<int64_t>(blockIdx.x) * NW + (threadIdx.x >> 6)) * 16 + t;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W1 = pack + PK_W1_N;
  const __bf16* W2 = pack + PK_W2_P32;
  fill_r32_w8<NW>(W1, GHM_D, PK_W, lds, lds + PLANE);  // pair 0 = {W1(0)} into slot 0
  if (threadIdx.x < GHM_F / 4)
    reinterpret_cast<float4*>(sb1)[threadIdx.x] = reinterpret_cast<const float4*>(b1)[threadIdx.x];
  bf16x8 xh[4], xl[4];
  {  // LN2 of the token row (as k_ln_mlp_fwd_x3b), lane holds features 32s + 8g + i
    const float* row = Hmid + mc * GHM_D;
    float x[32];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const float4 a = *reinterpret_cast<const float4*>(row + 32 * s2 + 8 * g);
      const float4 b = *reinterpret_cast<const float4*>(row + 32 * s2 + 8 * g + 4);
      x[8 * s2 + 0] = a.x; x[8 * s2 + 1] = a.y; x[8 * s2 + 2] = a.z; x[8 * s2 + 3] = a.w;
      x[8 * s2 + 4] = b.x; x[8 * s2 + 5] = b.y; x[8 * s2 + 6] = b.z; x[8 * s2 + 7] = b.w;
    }
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) sm += x[k];
    sm += __shfl_xor(sm, 16, 64);
    sm += __shfl_xor(sm, 32, 64);
    const float mean = sm * (1.f / 128.f);
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const float d = x[k] - mean;
      v += d * d;
    }
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    const float rstd = 1.f / sqrtf(v * (1.f / 128.f) + eps);
    if (g == 0 && valid) stats[m] = make_float2(mean, rstd);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int f = 32 * s2 + 8 * g + i;
        x[8 * s2 + i] = (x[8 * s2 + i] - mean) * rstd * lnw[f] + lnb[f];
      }
      split8(x + 8 * s2, xh[s2], xl[s2]);
    }
  }
  f32x4 y[8];  // seeded with the residual and b2 (as x3b)
  __builtin_amdgcn_sched_barrier(0);
  {
    const float* hr = Hmid + mc * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * j + 4 * g;
      const float4 hv = *reinterpret_cast<const float4*>(hr + f);
      const float4 bv = *reinterpret_cast<const float4*>(b2 + f);
      y[j][0] = hv.x + bv.x;
      y[j][1] = hv.y + bv.y;
      y[j][2] = hv.z + bv.z;
      y[j][3] = hv.w + bv.w;
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grpA)
    ws_loop<NW, true, MINW == 2>(lds, W1, W2, sb1, xh, xl, y, t, g);
  else
    ws_loop<NW, false, MINW == 2>(lds, W1, W2, sb1, xh, xl, y, t, g);
  if (valid) {
    float* orow = Hout + m * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) st4(orow + 16 * j + 4 * g, y[j][0], y[j][1], y[j][2], y[j][3]);
  }
}

// ---------------------------------------------------------------------------
// MLP + LN2 backward with the up-projection recomputed       (model.py:784-788)
// 16 tokens per wave, 8 waves (128 tokens) per workgroup, weight tiles by
// LDS-DMA as in k_ln_mlp_fwd_x3b.  The forward saved only Hmid and the LN2
// statistics; per 32-unit hidden chunk c:
//   U^T   = W1[c] LN2(Hmid)^T + b1       (recomputed, 2 tiles x 4 k-steps)
//   dG^T  = W2^T[c] dY^T                 (2 tiles x 4 k-steps over the 128 outputs)
//   G = GELU(U), dU = dG * GELU'(U)      -> HBM (inputs of dW2 and dW1)
//   dX2^T += W1^T[:, c] dU^T             (8 tiles, one k-step of 32 hidden units)
// then LN2 backward + residual: dHmid = dY + LN2'(dX2), and the workgroup's
// (sum dX2 * xhat, sum dX2) partials of the LN2 weight / bias gradients.
// Every lane runs a real row (lanes past M recompute row M-1 and store the same
// bytes), so each wave has exactly 4 stores in flight per chunk.
// ---------------------------------------------------------------------------
// Butterfly reduce-scatter of 32 values over the 16 lanes t = lane & 15 of a
// lane group: lane t returns the 16-lane sums of values 2t (.x) and 2t + 1 (.y).
__device__ __forceinline__ float2 reduce_scatter32_t16(float* v, int t) {
#pragma unroll
  for (int lvl = 0; lvl < 4; ++lvl) {
    const int m = 8 >> lvl;         // lane-bit of this level
    const int half = 16 >> lvl;     // live values 32 >> lvl
    const bool upper = (t & m) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float lo = v[i], hi = v[i + half];
      const float send = upper ? lo : hi;
      const float keep = upper ? hi : lo;
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
  return make_float2(v[0], v[1]);
}

// W1 chunk image shared by row reads and transposed reads: [32 rows][128]
// (256-B rows), 16-B chunk c of row r at c ^ 2(r & 7).  Row reads (16x16x32
// operand: lane t -> row 16 jt + t, chunk 4 s2 + g) hit 16 distinct chunks per
// ds_read_b128 lane group; a transposed read's 32-lane half (rows of one
// aligned 8-row block x the two chunks of 16 columns) hits all 64 banks once.
__device__ __forceinline__ int r32t_off(int row, int lc) { return row * 128 + 8 * (lc ^ (2 * (row & 7))); }
template <int NW>
__device__ __forceinline__ void fill_r32t_w8(const __bf16* g, int ldg, int lo_off, __bf16* ih, __bf16* il) {
  const int L = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < (8 + NW - 1) / NW; ++k) {
    const int b = (threadIdx.x >> 6) + NW * k;
    if (8 % NW == 0 || b < 8) {
      const int row = 4 * b + (L >> 4), lc = (L & 15) ^ (2 * (row & 7));
      const __bf16* src = g + row * ldg + 8 * lc;
      glds16(src, ih + 512 * b);
      glds16(src + lo_off, il + 512 * b);
    }
  }
}
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 ldtr(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(p));
}
// element offset of lane (g, q, p)'s transposed-read address for dX2 tile j:
// row 4 g + q, columns 16 j + 4 p .. + 3 (the second read: row + 16, same
// swizzle since (row + 16) & 7 == row & 7)
__device__ __forceinline__ int w1t_tr_off(int j, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, row = 4 * g + q;
  return row * 128 + 8 * ((2 * j + (p >> 1)) ^ (2 * (row & 7))) + 4 * (p & 1);
}
__device__ __forceinline__ bf16x8 tr_pair(const __bf16* p) {
  const bf16x4 a = ldtr(p), b = ldtr(p + 16 * 128);
  bf16x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  return v;
}
// G (for dW2) and dU (for dW1) of one hidden chunk: 4 stores per wave
__device__ __forceinline__ void store_g_du(const float* gv, const float* du, float* grow, float* drow) {
  st4(grow, gv[0], gv[1], gv[2], gv[3]);
  st4(grow + 16, gv[4], gv[5], gv[6], gv[7]);
  st4(drow, du[0], du[1], du[2], du[3]);
  st4(drow + 16, du[4], du[5], du[6], du[7]);
}

// Pieces of one 32-unit hidden chunk of k_mlp_bwd_rc_x3 (operands from ring
// buffer cb = [W1 hi | W1 lo | W2^T hi | W2^T lo]):
//   rc_ud:  U = W1[c] LN2(Hmid)^T + b1 (recomputed), dG = W2^T[c] dY^T,
//           G = GELU(U), dU = dG GELU'(U) -> HBM; returns dU split (dh, dl)
//   rc_dx2: dX2^T += W1^T[:, c] dU^T
// SPLITOUT: G and dU leave as pre-split bf16 planes (the weight gradients'
// WG_SPLIT operands, ghm_wgrad.hip): grow / drow point at the lane's 8 k-slots
// 32c + 8g .. + 7 of the hi plane (perm32 column order, one 16-B store per plane),
// the lo plane `plane` elements on; else f32 [M][512] rows at 32c + 4g
template <int SPLITOUT>
__device__ __forceinline__ void rc_ud(const __bf16* cb, const float4* bb, const bf16x8* xh, const bf16x8* xl,
                                      const bf16x8* yh, const bf16x8* yl, void* grow, void* drow, int64_t plane,
                                      int t, int g, bf16x8& dh, bf16x8& dl) {
  const __bf16* w1h = cb;
  const __bf16* w1l = cb + PLANE;
  const __bf16* w2h = cb + 2 * PLANE;
  const __bf16* w2l = cb + 3 * PLANE;
  f32x4 u[2], dg[2];
  float gv[8], du[8];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    u[jt] = zero4();
    dg[jt] = zero4();
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int o1 = r32t_off(16 * jt + t, 4 * s2 + g), o = r32_off(16 * jt + t, 4 * s2 + g);
      u[jt] = mfma16_x3(ldsb8(w1h + o1), ldsb8(w1l + o1), xh[s2], xl[s2], u[jt]);
      dg[jt] = mfma16_x3(ldsb8(w2h + o), ldsb8(w2l + o), yh[s2], yl[s2], dg[jt]);
    }
  }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {  // + b1, GELU, GELU'
    const float bs[4] = {bb[jt].x, bb[jt].y, bb[jt].z, bb[jt].w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float gd;
      gelu_fast(u[jt][r] + bs[r], gv[4 * jt + r], gd);
      du[4 * jt + r] = dg[jt][r] * gd;
    }
  }
  split8(du, dh, dl);
  if (SPLITOUT == 2) {
    // G as bf16 (hi, lo) planes [M][512] in natural column order (the dW2 weight
    // gradient's pre-split B operand, ghm_wgrad_x3p); dU stays f32.  grow points at
    // units 32c + 4g of the hi plane: gv[4 jt + r] is unit 32c + 16 jt + 4g + r
    bf16x8 gh, gl;
    split8(gv, gh, gl);
    __bf16* gp = static_cast<__bf16*>(grow);
    bf16x4 a, b;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = gh[4 * jt + r];
        b[r] = gl[4 * jt + r];
      }
      *reinterpret_cast<bf16x4*>(gp + 16 * jt) = a;
      *reinterpret_cast<bf16x4*>(gp + 16 * jt + plane) = b;
    }
    float* drw = static_cast<float*>(drow);
    st4(drw, du[0], du[1], du[2], du[3]);
    st4(drw + 16, du[4], du[5], du[6], du[7]);
  } else if (SPLITOUT) {
    bf16x8 gh, gl;
    split8(gv, gh, gl);
    __bf16* gp = static_cast<__bf16*>(grow);
    __bf16* dp = static_cast<__bf16*>(drow);
    *reinterpret_cast<bf16x8*>(gp) = gh;
    *reinterpret_cast<bf16x8*>(gp + plane) = gl;
    *reinterpret_cast<bf16x8*>(dp) = dh;
    *reinterpret_cast<bf16x8*>(dp + plane) = dl;
  } else {
    store_g_du(gv, du, static_cast<float*>(grow), static_cast<float*>(drow));
  }
}

// dX2^T tile j: A[d = 16 j + t][k-slot 8 g + i] = W1[unit perm32(8 g + i)][d],
// i.e. rows 4 g .. 4 g + 3 and 16 + 4 g .. 16 + 4 g + 3 of the W1 chunk at
// column 16 j + t: two transposed reads per plane
__device__ __forceinline__ void rc_dx2(const __bf16* cb, bf16x8 dh, bf16x8 dl, f32x4* dx, int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int o = w1t_tr_off(j, lane);
    dx[j] = mfma16_x3(tr_pair(cb + o), tr_pair(cb + PLANE + o), dh, dl, dx[j]);
  }
}

// One chunk iteration: LDS-DMA fills of the next chunk into ring buffer `nb`,
// then the products of chunk c from `cb`.  The buffers are __restrict__
// parameters of one inlined function, so every access carries alias-scope
// metadata that tells the waitcnt pass the DMA target and the operand reads are
// disjoint (without it the compiler waited vmcnt(0) for the just-issued fills
// before the first transposed read of the W1 image).  Tried and slower: waves
// 4-7 one dX2 behind on a 3-buffer ring, so the two waves of a SIMD sit in
// opposite MFMA / GELU phases (isolated 119 -> 124 us, step +1 %,
// profiles/r3_ab5).
template <int NW, int SPLITOUT>
__device__ __forceinline__ void mlp_bwd_rc_iter(const __bf16* __restrict__ cb, __bf16* __restrict__ nb,
                                                const __bf16* W1n, const __bf16* W2Tn, const float4* bb,
                                                const bf16x8* xh, const bf16x8* xl, const bf16x8* yh,
                                                const bf16x8* yl, f32x4* dx, void* grow, void* drow, int64_t plane,
                                                int t, int g, int lane) {
  fill_r32t_w8<NW>(W1n, GHM_D, PK_W, nb, nb + PLANE);
  fill_r32_w8<NW>(W2Tn, GHM_D, PK_W, nb + 2 * PLANE, nb + 3 * PLANE);
  bf16x8 dh, dl;
  // scheduling hint 0 (interleave the DS reads with the MFMAs): isolated 121.7 ->
  // 115.7 us, 186 instead of 226 VGPRs, step -1.2 % (profiles/r3_ab14; the same
  // hint in the MLP forward made the step slower)
  __builtin_amdgcn_iglp_opt(0);
  rc_ud<SPLITOUT>(cb, bb, xh, xl, yh, yl, grow, drow, plane, t, g, dh, dl);
  // the dX2 products as a scheduling region of their own, under the same hint:
  // isolated 116.1 -> 113.1 us, step unchanged (4.12 / 4.12 ms, r3_sr / r3_ab20)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_iglp_opt(0);
  rc_dx2(cb, dh, dl, dx, lane);
}

// STAMP (bench.py's in-graph timing only, ghm_mlp_bwd_rc_x3_stamped; 1 and 2 are
// two identical twins, so that a rocprofv3 trace tells bench.py's two
// measurements apart): thread 0
// of each workgroup writes the 100 MHz constant clock (s_memrealtime) at its
// start and after its last store to stamps[2 blockIdx.x + {0, 1}]; the launch
// spans min(start) .. max(end).  Nothing else differs.
// SPLITOUT: 0 G / dU f32 (the default), 1 both as perm32 bf16 planes (the ring
// weight gradients), 2 G as natural-order bf16 planes, dU f32 (ghm_wgrad_x3p dW2)
template <int NW, int STAMP = 0, int SPLITOUT = 0>
__global__ __launch_bounds__(64 * NW, 2) void k_mlp_bwd_rc_x3(
    const float* __restrict__ dHout, const float* __restrict__ Hmid, const float2* __restrict__ stats,
    const float* __restrict__ lnw, const float* __restrict__ lnb, const __bf16* pack, const float* __restrict__ b1,
    float* __restrict__ Gout, float* __restrict__ dU, float* __restrict__ dHmid, float* __restrict__ part_ln,
    int64_t M, uint64_t* __restrict__ stamps = nullptr) {
  uint64_t t_start = 0;
  if (STAMP) t_start = __builtin_amdgcn_s_memrealtime();
  constexpr int NC = GHM_F / 32;
  // [W1 hi|lo][W2^T hi|lo] x 2 buffers (64 KB: two workgroups per CU); the LN
  // partial buffer aliases it after the loop.  The W1 chunk serves both the U
  // recompute (row reads) and, through ds_read_b64_tr_b16, the dX2 product's
  // W1^T operand (round 1 staged a third, transposed W1^T image: 96 KB, one
  // workgroup per CU).
  __shared__ __attribute__((aligned(16))) __bf16 lds[8 * PLANE + 2 * GHM_F];
  float* sb1 = reinterpret_cast<float*>(lds + 8 * PLANE);  // read before the fills: see k_ln_mlp_fwd_x3b
  auto sw1h = [&](int b) { return lds + 4 * PLANE * b; };
  auto sw1l = [&](int b) { return lds + 4 * PLANE * b + PLANE; };
  auto sw2h = [&](int b) { return lds + 4 * PLANE * b + 2 * PLANE; };
  auto sw2l = [&](int b) { return lds + 4 * PLANE * b + 3 * PLANE; };
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int64_t m = (static_cast<int64_t>(blockIdx.x) * NW + wave) * 16 + t;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W1 = pack + PK_W1_N;    // [512 f][128 d]
  const __bf16* W2T = pack + PK_W2_T;   // [512 f][128 o]
  fill_r32t_w8<NW>(W1, GHM_D, PK_W, sw1h(0), sw1l(0));
  fill_r32_w8<NW>(W2T, GHM_D, PK_W, sw2h(0), sw2l(0));
  if (threadIdx.x < GHM_F / 4)
    reinterpret_cast<float4*>(sb1)[threadIdx.x] = reinterpret_cast<const float4*>(b1)[threadIdx.x];
  // B operands: LN2(Hmid) and dY of the token, lane holds features 32 s2 + 8 g + i
  bf16x8 xh[4], xl[4], yh[4], yl[4];
  const float2 st = ld_stats_sys(stats, mc);
  {
    const float* row = Hmid + mc * GHM_D;
    const float* dyr = dHout + mc * GHM_D;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int f0 = 32 * s2 + 8 * g;
      const float4 a = *reinterpret_cast<const float4*>(row + f0);
      const float4 b = *reinterpret_cast<const float4*>(row + f0 + 4);
      const float4 ga = *reinterpret_cast<const float4*>(lnw + f0);
      const float4 gb = *reinterpret_cast<const float4*>(lnw + f0 + 4);
      const float4 ba = *reinterpret_cast<const float4*>(lnb + f0);
      const float4 bb = *reinterpret_cast<const float4*>(lnb + f0 + 4);
      float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const float gw[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
      const float bw[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = (x[i] - st.x) * st.y * gw[i] + bw[i];
      split8(x, xh[s2], xl[s2]);
      const float4 c = *reinterpret_cast<const float4*>(dyr + f0);
      const float4 d = *reinterpret_cast<const float4*>(dyr + f0 + 4);
      const float y[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
      split8(y, yh[s2], yl[s2]);
    }
  }
  f32x4 dx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dx[j] = zero4();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const int cur = c & 1;
    float4 bb[2];  // b1 of hidden units 32c + 16jt + 4g + r
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) bb[jt] = lds4(sb1 + 32 * c + 16 * jt + 4 * g);
    issue_fence();
    const int cn = c + 1 < NC ? c + 1 : NC - 1;  // branch-free: the last iteration refills chunk NC-1
    void* grow = SPLITOUT == 1 ? static_cast<void*>(reinterpret_cast<__bf16*>(Gout) + mc * GHM_F + 32 * c + 8 * g)
                 : SPLITOUT == 2 ? static_cast<void*>(reinterpret_cast<__bf16*>(Gout) + mc * GHM_F + 32 * c + 4 * g)
                                 : static_cast<void*>(Gout + mc * GHM_F + 32 * c + 4 * g);
    void* drow = SPLITOUT == 1 ? static_cast<void*>(reinterpret_cast<__bf16*>(dU) + mc * GHM_F + 32 * c + 8 * g)
                               : static_cast<void*>(dU + mc * GHM_F + 32 * c + 4 * g);
    mlp_bwd_rc_iter<NW, SPLITOUT>(lds + 4 * PLANE * cur, lds + 4 * PLANE * (cur ^ 1), W1 + cn * 32 * GHM_D,
                                  W2T + cn * 32 * GHM_D, bb, xh, xl, yh, yl, dx, grow, drow, M * GHM_F, t, g, lane);
    // retire this iteration's LDS-DMA fills: vmcnt(0), also covering the G / dU
    // stores issued after them (see k_ln_mlp_fwd_x3b).  Storing them one chunk
    // later instead, so this wait would not cover fresh stores, measured slower
    // (isolated 119 -> 130 us, profiles/r3_ab2).
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // LN2 backward: lane holds dX2 of features d = 16 j + 4 g + r
  const float mean = st.x, rstd = st.y;
  float xhat[32], dyg[32];
  float s1 = 0.f, s2 = 0.f;
  {
    const float* row = Hmid + mc * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * j + 4 * g;
      const float4 xv = *reinterpret_cast<const float4*>(row + f);
      const float4 gv = *reinterpret_cast<const float4*>(lnw + f);
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float xh_ = (xs[r] - mean) * rstd;
        xhat[4 * j + r] = xh_;
        const float v = dx[j][r] * gs[r];
        dyg[4 * j + r] = v;
        s1 += v;
        s2 += v * xh_;
      }
    }
  }
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float m1 = s1 * (1.f / GHM_D), m2 = s2 * (1.f / GHM_D);
  {
    const float* dres = dHout + mc * GHM_D;
    float* orow = dHmid + mc * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * j + 4 * g;
      const float4 rv = *reinterpret_cast<const float4*>(dres + f);
      const float rs[4] = {rv.x, rv.y, rv.z, rv.w};
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = rs[r] + rstd * (dyg[4 * j + r] - m1 - xhat[4 * j + r] * m2);
      st4(orow + f, o[0], o[1], o[2], o[3]);
    }
  }
  // LN2 weight / bias partials of the workgroup: per wave a reduce-scatter over
  // its 16 tokens (lane t ends with features of value slots 2t, 2t + 1), then
  // the 8 waves in a fixed order
  float vg[32], vb[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const float d = valid ? dx[k >> 2][k & 3] : 0.f;
    vb[k] = d;
    vg[k] = d * xhat[k];
  }
  const float2 rg = reduce_scatter32_t16(vg, t);
  const float2 rb = reduce_scatter32_t16(vb, t);
  float* red = reinterpret_cast<float*>(lds);  // [2][NW][128]; the ring is idle after the last barrier
  {
    const int k0 = 2 * t;  // value slot k = 4 j + r -> feature 16 j + 4 g + r
    const int f0 = 16 * (k0 >> 2) + 4 * g + (k0 & 3);
    red[wave * GHM_D + f0] = rg.x;
    red[wave * GHM_D + f0 + 1] = rg.y;
    red[NW * GHM_D + wave * GHM_D + f0] = rb.x;
    red[NW * GHM_D + wave * GHM_D + f0 + 1] = rb.y;
  }
  __syncthreads();
  if (threadIdx.x < 2 * GHM_D) {
    const int q = threadIdx.x >> 7, f = threadIdx.x & 127;
    const float* rr = red + q * NW * GHM_D + f;
    float sum;
    if (NW == 8)
      sum = ((rr[0] + rr[GHM_D]) + (rr[2 * GHM_D] + rr[3 * GHM_D])) +
            ((rr[4 * GHM_D] + rr[5 * GHM_D]) + (rr[6 * GHM_D] + rr[7 * GHM_D]));
    else
      sum = (rr[0] + rr[GHM_D]) + (rr[2 * GHM_D] + rr[3 * GHM_D]);
    part_ln[static_cast<int64_t>(blockIdx.x) * 2 * GHM_D + q * GHM_D + f] = sum;
  }
  if (STAMP) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
      stamps[2 * blockIdx.x] = t_start;
      stamps[2 * blockIdx.x + 1] = t_end;
    }
  }
}

#ifdef GHM_FUSED_DW_PROTO
#ifndef GHM_ABLATION_BUILD
#error "GHM_FUSED_DW_PROTO is a timing prototype: only with -DGHM_ABLATION_BUILD (tools/, never the product library)"
#endif
// ---------------------------------------------------------------------------
// TIMING PROTOTYPE (review item 2; results are not the weight gradients): the MLP
// backward at 64 tokens per workgroup with dW2 / dW1 accumulated inside it per
// hidden chunk, instead of writing G / dU for k_wgrad_x3.  Everything the fused
// design must do is here at its real size: the dY and LN2(Hmid) token images
// staged once into LDS (bf16 hi / lo, [64 tokens][128]: 64 KB), per chunk the
// G_c / dU_c images written (16 KB) and a barrier, 48 more MFMAs per wave per chunk
// whose tokens-on-k operands come from those images through ds_read_b64_tr_b16,
// and the per-chunk partials (dW2_c + dW1_c: 2 x 128 x 32 f32 = 32 KB per
// workgroup and chunk) stored for a fixed-order reduction over the workgroups.
// The operand indexing inside the images is schematic (conflict-free offsets of
// the right instruction count); the U / dG / dU / dX2 / LN2 work is the product's.
// LDS: 66 KB ring + 80 KB images = 146 KB: one workgroup (4 waves) per CU.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void rc_ud_vals(const __bf16* cb, const float4* bb, const bf16x8* xh, const bf16x8* xl,
                                           const bf16x8* yh, const bf16x8* yl, int t, int g, float* gv, float* du) {
  const __bf16* w1h = cb;
  const __bf16* w1l = cb + PLANE;
  const __bf16* w2h = cb + 2 * PLANE;
  const __bf16* w2l = cb + 3 * PLANE;
  f32x4 u[2], dg[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    u[jt] = zero4();
    dg[jt] = zero4();
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int o1 = r32t_off(16 * jt + t, 4 * s2 + g), o = r32_off(16 * jt + t, 4 * s2 + g);
      u[jt] = mfma16_x3(ldsb8(w1h + o1), ldsb8(w1l + o1), xh[s2], xl[s2], u[jt]);
      dg[jt] = mfma16_x3(ldsb8(w2h + o), ldsb8(w2l + o), yh[s2], yl[s2], dg[jt]);
    }
  }
#pragma unroll
  for (int jt = 0; jt < 2; ++jt) {
    const float bs[4] = {bb[jt].x, bb[jt].y, bb[jt].z, bb[jt].w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float gd;
      gelu_fast(u[jt][r] + bs[r], gv[4 * jt + r], gd);
      du[4 * jt + r] = dg[jt][r] * gd;
    }
  }
}

__device__ __forceinline__ bf16x8 proto_tr(const __bf16* img, int off) {
  typedef __attribute__((address_space(3))) bf16x4 lds4_t;
  const bf16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds4_t*)(img + off));
  const bf16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds4_t*)(img + off + 16 * 64));
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    r[i] = a[i];
    r[4 + i] = b[i];
  }
  return r;
}

__global__ __launch_bounds__(256, 1) void k_mlp_bwd_fused_proto(
    const float* __restrict__ dHout, const float* __restrict__ Hmid, const float2* __restrict__ stats,
    const float* __restrict__ lnw, const float* __restrict__ lnb, const __bf16* pack, const float* __restrict__ b1,
    float* __restrict__ part_w, float* __restrict__ dHmid, float* __restrict__ part_ln, int64_t M) {
  constexpr int NW = 4, NC = GHM_F / 32;
  __shared__ __attribute__((aligned(16))) __bf16 lds[8 * PLANE + 2 * GHM_F];
  // token images: dY hi|lo, X2 hi|lo [64][128] (4 x 16 KB), G_c hi|lo, dU_c hi|lo [64][32] (4 x 4 KB)
  __shared__ __attribute__((aligned(16))) __bf16 img[4 * 64 * 128 + 4 * 64 * 32];
  float* sb1 = reinterpret_cast<float*>(lds + 8 * PLANE);
  auto sw1h = [&](int b) { return lds + 4 * PLANE * b; };
  auto sw1l = [&](int b) { return lds + 4 * PLANE * b + PLANE; };
  auto sw2h = [&](int b) { return lds + 4 * PLANE * b + 2 * PLANE; };
  auto sw2l = [&](int b) { return lds + 4 * PLANE * b + 3 * PLANE; };
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int tok = 16 * wave + t;
  const int64_t m = (static_cast<int64_t>(blockIdx.x) * NW + wave) * 16 + t;
  const bool valid = m < M;
  const int64_t mc = valid ? m : M - 1;
  const __bf16* W1 = pack + PK_W1_N;
  const __bf16* W2T = pack + PK_W2_T;
  fill_r32t_w8<NW>(W1, GHM_D, PK_W, sw1h(0), sw1l(0));
  fill_r32_w8<NW>(W2T, GHM_D, PK_W, sw2h(0), sw2l(0));
  if (threadIdx.x < GHM_F / 4)
    reinterpret_cast<float4*>(sb1)[threadIdx.x] = reinterpret_cast<const float4*>(b1)[threadIdx.x];
  bf16x8 xh[4], xl[4], yh[4], yl[4];
  const float2 st = ld_stats_sys(stats, mc);
  {
    const float* row = Hmid + mc * GHM_D;
    const float* dyr = dHout + mc * GHM_D;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int f0 = 32 * s2 + 8 * g;
      const float4 a = *reinterpret_cast<const float4*>(row + f0);
      const float4 b = *reinterpret_cast<const float4*>(row + f0 + 4);
      const float4 ga = *reinterpret_cast<const float4*>(lnw + f0);
      const float4 gb = *reinterpret_cast<const float4*>(lnw + f0 + 4);
      const float4 ba = *reinterpret_cast<const float4*>(lnb + f0);
      const float4 bb = *reinterpret_cast<const float4*>(lnb + f0 + 4);
      float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      const float gw[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
      const float bw[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = (x[i] - st.x) * st.y * gw[i] + bw[i];
      split8(x, xh[s2], xl[s2]);
      const float4 c = *reinterpret_cast<const float4*>(dyr + f0);
      const float4 d = *reinterpret_cast<const float4*>(dyr + f0 + 4);
      const float y[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
      split8(y, yh[s2], yl[s2]);
      // the token images of dY and X2 (once)
      const int o = tok * 128 + 8 * ((4 * s2 + g) ^ (tok & 15));
      *reinterpret_cast<bf16x8*>(img + o) = yh[s2];
      *reinterpret_cast<bf16x8*>(img + 64 * 128 + o) = yl[s2];
      *reinterpret_cast<bf16x8*>(img + 2 * 64 * 128 + o) = xh[s2];
      *reinterpret_cast<bf16x8*>(img + 3 * 64 * 128 + o) = xl[s2];
    }
  }
  __bf16* gimg = img + 4 * 64 * 128;
  f32x4 dx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dx[j] = zero4();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
  for (int c = 0; c < NC; ++c) {
    const int cur = c & 1;
    float4 bb[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) bb[jt] = lds4(sb1 + 32 * c + 16 * jt + 4 * g);
    issue_fence();
    const int cn = c + 1 < NC ? c + 1 : NC - 1;
    fill_r32t_w8<NW>(W1 + cn * 32 * GHM_D, GHM_D, PK_W, sw1h(cur ^ 1), sw1l(cur ^ 1));
    fill_r32_w8<NW>(W2T + cn * 32 * GHM_D, GHM_D, PK_W, sw2h(cur ^ 1), sw2l(cur ^ 1));
    float gv[8], du[8];
    rc_ud_vals(lds + 4 * PLANE * cur, bb, xh, xl, yh, yl, t, g, gv, du);
    bf16x8 gh, gl, dh, dl;
    split8(gv, gh, gl);
    split8(du, dh, dl);
    rc_dx2(lds + 4 * PLANE * cur, dh, dl, dx, lane);
    // G_c / dU_c token images [64][32], then every wave's quarter of dW2_c / dW1_c
    const int go = tok * 32 + 8 * (g ^ (tok & 3));
    *reinterpret_cast<bf16x8*>(gimg + go) = gh;
    *reinterpret_cast<bf16x8*>(gimg + 64 * 32 + go) = gl;
    *reinterpret_cast<bf16x8*>(gimg + 2 * 64 * 32 + go) = dh;
    *reinterpret_cast<bf16x8*>(gimg + 3 * 64 * 32 + go) = dl;
    __syncthreads();
    f32x4 w2a[4], w1a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w2a[q] = w1a[q] = zero4();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {  // 64 tokens = 2 k-steps of 32
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // dW2_c rows 32 wave + 16 (q >> 1) (features o), cols 16 (q & 1) (units): A = dY^T, B = G_c
        const int ao = (32 * ks + 4 * (lane >> 4)) * 128 + 32 * wave + 16 * (q >> 1) + (lane & 15);
        const int bo = (32 * ks + 4 * (lane >> 4)) * 32 + 16 * (q & 1) + (lane & 15);
        w2a[q] = mfma16_x3(proto_tr(img, ao), proto_tr(img + 64 * 128, ao), proto_tr(gimg, bo),
                           proto_tr(gimg + 64 * 32, bo), w2a[q]);
        // dW1_c rows 16 (q >> 1) (units), cols 32 wave + 16 (q & 1) (inputs): A = dU_c^T, B = X2
        const int ao1 = (32 * ks + 4 * (lane >> 4)) * 32 + 16 * (q >> 1) + (lane & 15);
        const int bo1 = (32 * ks + 4 * (lane >> 4)) * 128 + 32 * wave + 16 * (q & 1) + (lane & 15);
        w1a[q] = mfma16_x3(proto_tr(gimg + 2 * 64 * 32, ao1), proto_tr(gimg + 3 * 64 * 32, ao1),
                           proto_tr(img + 2 * 64 * 128, bo1), proto_tr(img + 3 * 64 * 128, bo1), w1a[q]);
      }
    }
    // this workgroup's chunk partials: [blk][c][wave][lane][32]
    float* pp = part_w + ((static_cast<int64_t>(blockIdx.x) * NC + c) * NW + wave) * 64 * 32 + lane * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      st4(pp + 4 * q, w2a[q][0], w2a[q][1], w2a[q][2], w2a[q][3]);
      st4(pp + 16 + 4 * q, w1a[q][0], w1a[q][1], w1a[q][2], w1a[q][3]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // LN2 backward (as k_mlp_bwd_rc_x3)
  const float mean = st.x, rstd = st.y;
  float xhat[32], dyg[32];
  float s1 = 0.f, s2 = 0.f;
  {
    const float* row = Hmid + mc * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * j + 4 * g;
      const float4 xv = *reinterpret_cast<const float4*>(row + f);
      const float4 gv = *reinterpret_cast<const float4*>(lnw + f);
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w}, gs[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float xh_ = (xs[r] - mean) * rstd;
        xhat[4 * j + r] = xh_;
        const float v = dx[j][r] * gs[r];
        dyg[4 * j + r] = v;
        s1 += v;
        s2 += v * xh_;
      }
    }
  }
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  const float m1 = s1 * (1.f / GHM_D), m2 = s2 * (1.f / GHM_D);
  {
    const float* dres = dHout + mc * GHM_D;
    float* orow = dHmid + mc * GHM_D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * j + 4 * g;
      const float4 rv = *reinterpret_cast<const float4*>(dres + f);
      const float rs[4] = {rv.x, rv.y, rv.z, rv.w};
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = rs[r] + rstd * (dyg[4 * j + r] - m1 - xhat[4 * j + r] * m2);
      st4(orow + f, o[0], o[1], o[2], o[3]);
    }
  }
  float vg[32], vb[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const float d = valid ? dx[k >> 2][k & 3] : 0.f;
    vb[k] = d;
    vg[k] = d * xhat[k];
  }
  const float2 rg = reduce_scatter32_t16(vg, t);
  const float2 rb = reduce_scatter32_t16(vb, t);
  float* red = reinterpret_cast<float*>(lds);
  {
    const int k0 = 2 * t;
    const int f0 = 16 * (k0 >> 2) + 4 * g + (k0 & 3);
    red[wave * GHM_D + f0] = rg.x;
    red[wave * GHM_D + f0 + 1] = rg.y;
    red[NW * GHM_D + wave * GHM_D + f0] = rb.x;
    red[NW * GHM_D + wave * GHM_D + f0 + 1] = rb.y;
  }
  __syncthreads();
  if (threadIdx.x < 2 * GHM_D) {
    const int q = threadIdx.x >> 7, f = threadIdx.x & 127;
    const float* rr = red + q * NW * GHM_D + f;
    part_ln[static_cast<int64_t>(blockIdx.x) * 2 * GHM_D + q * GHM_D + f] =
        (rr[0] + rr[GHM_D]) + (rr[2 * GHM_D] + rr[3 * GHM_D]);
  }
}

extern "C" int ghm_mlp_bwd_fused_proto(const float* dH_out, const float* H_mid, const float* stats,
                                       const float* ln_w, const float* ln_b, const void* pack, const float* b1,
                                       float* part_w, float* dH_mid, float* part_ln, int64_t M, void* stream) {
  GHM_CHECK(dH_out && H_mid && stats && ln_w && ln_b && pack && b1 && part_w && dH_mid && part_ln, "null pointer");
  hipLaunchKernelGGL(k_mlp_bwd_fused_proto, dim3(static_cast<unsigned>((M + 63) / 64)), dim3(256), 0,
                     ghm_stream(stream), dH_out, H_mid, reinterpret_cast<const float2*>(stats), ln_w, ln_b,
                     reinterpret_cast<const __bf16*>(pack), b1, part_w, dH_mid, part_ln, M);
  return ghm_launch_status();
}
#endif  // GHM_FUSED_DW_PROTO

// ---------------------------------------------------------------------------
// QKV + LN1 backward                                          (model.py:772-775)
//   dX1^T = Wq^T dQ^T + Wk^T dK^T + Wv^T dV^T, then LN1 backward + residual.
// ---------------------------------------------------------------------------
// LN1 statistics, STATS: 0 recomputed from H (the product path); diagnostic
// variants (ghm_qkv_bwd_x3_probe, tools/race_probe.py; DESIGN.md §4
// "Determinism"): 1 a plain vector load of the forward's [M][2] buffer (the
// round-2 load whose 16-token groups came back wrong beside k_wgrad_x3), 2 the
// same load at agent scope through a buffer descriptor (sc0 sc1), 3 at agent
// scope as a global load (ld_stats, sc1), 4 the plain load AND the recompute:
// the product uses the recomputed pair and every lane with h == 0 writes
// (loaded mean, loaded rstd, recomputed mean, recomputed rstd) to dbg[m];
// 5 as 1 (the plain load, used) and dbg[m] = (used mean, used rstd, 0, 0);
// 6 as 1 with no per-token store: thread 0 writes the workgroup's placement
// (XCC_ID, HW_ID register bits, blockIdx) to dbg[blockIdx.x] after the product,
// so the host can place every wrong row group on an XCD and infer the pair the
// row used from the output itself (tools/race_probe.py qkv_xcc).  Mode 4 writes
// the same placement record to dbg[M + blockIdx.x].
template <int STATS>
__global__ __launch_bounds__(256, 2) void k_qkv_bwd_x3(
    const float* __restrict__ dqkv, const float* __restrict__ H, const float* __restrict__ lnw,
    const __bf16* pack, const float* __restrict__ dHmid, float* __restrict__ dH,
    float* __restrict__ part_ln, int64_t M, float eps, const float2* __restrict__ stats,
    float4* __restrict__ dbg) {
  // weight tiles of W^T ([128 d][384], 32 d-rows x 128 columns) by LDS-DMA into
  // a double-buffered R32 ring, as k_ln_qkv_fwd_x3
  __shared__ __attribute__((aligned(16))) __bf16 lds[4 * PLANE];
  __shared__ float red[2 * 4 * GHM_D];
  __shared__ __attribute__((aligned(16))) float gam[GHM_D];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t m0 = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * 32;
  const bool active = m0 < M;
  const __bf16* W = pack + PK_QKV_T;  // [128 d][384]
  fill_r32_w8<4>(W, 3 * GHM_D, PK_QKV, lds, lds + PLANE);  // tile 0, in flight over the prologue
  for (int i = threadIdx.x; i < 2 * 4 * GHM_D; i += 256) red[i] = 0.f;
  if (threadIdx.x < GHM_D) gam[threadIdx.x] = lnw[threadIdx.x];
  const int64_t m = m0 + j;
  const bool valid = active && m < M;
  const int64_t mc = m < M ? m : M - 1;
  // STATS 0 recomputes the statistics exactly as the forward computed them
  // (ln_row's layout, ln_stats64: bit-identical to the saved values)
  float2 lnst;
  if (STATS == 0 || STATS == 4) {
    float x[64];
    load64(H + mc * GHM_D + 64 * h, x);
    ln_stats64(x, eps, lnst.x, lnst.y);
  } else if (STATS == 1 || STATS == 5 || STATS == 6) {
    lnst = stats[mc];
  } else if (STATS == 2) {
    lnst = ld_stats_sys(stats, mc);
  } else {
    lnst = ld_stats(stats + mc);
  }
  float2 loaded = make_float2(0.f, 0.f);
  if (STATS == 4) loaded = stats[mc];  // issued here, used only after the main loop (as STATS 1 used it)
  f32x16 dx[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) dx[it] = zero16();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll 1
  for (int mat = 0; mat < 3; ++mat) {
    bf16x8 gh[8], gl[8];
    load_split64(dqkv + mc * (3 * GHM_D) + mat * GHM_D + 64 * h, active, gh, gl);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int b = mat * 4 + it, cur = b & 1;
      const int nb = b + 1 < 12 ? b + 1 : 11;  // tile nb: rows 32*(nb&3).., columns 128*(nb>>2)..
      dx[it] = qkv_tile_x3(lds + 2 * PLANE * cur, lds + 2 * PLANE * (cur ^ 1),
                           W + (nb & 3) * 32 * (3 * GHM_D) + (nb >> 2) * GHM_D, 3 * GHM_D, j, h, active, gh, gl,
                           dx[it]);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  if (STATS == 4 && valid && h == 0) dbg[m] = make_float4(loaded.x, loaded.y, lnst.x, lnst.y);
  if (STATS == 5 && valid && h == 0) dbg[m] = make_float4(lnst.x, lnst.y, 0.f, 0.f);
  if (active)
    ln_bwd_acc(dx, H + mc * GHM_D, lnst, gam, dHmid + mc * GHM_D, dH + mc * GHM_D, valid, h, j,
               red + wave * GHM_D, red + 4 * GHM_D + wave * GHM_D);
  __syncthreads();
  ln_partial_store(red, part_ln + static_cast<int64_t>(blockIdx.x) * 2 * GHM_D);
  if ((STATS == 4 || STATS == 6) && threadIdx.x == 0) {
    // s_getreg immediates: id | offset << 6 | (size - 1) << 11; HW_REG_XCC_ID = 20
    // (bits 3:0 the XCD), HW_REG_HW_ID = 4 (wave, SIMD, CU, SE fields)
    const int xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
    const int hwid = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    dbg[(STATS == 4 ? M : 0) + blockIdx.x] = make_float4(__int_as_float(xcc), __int_as_float(hwid), __int_as_float(static_cast<int>(blockIdx.x)), 0.f);
  }
}

// ---------------------------------------------------------------------------
// Split-K weight gradient, split-bf16                 (nn.Linear weight/bias grads)
//   part[z][a][b] = sum_{m in chunk z} A[m][a] op(B)[m][b],  op = id | LayerNorm
// Tokens are the MFMA k dimension.  Per 32-token step each thread loads ONE
// column of A and of op(B) for 16 tokens (dword loads, coalesced across the
// wave), splits them and writes [column][token] bf16 images (64-B rows, 16-B
// chunks XOR-swizzled by row so the operand reads are conflict-free), so a
// lane's 8-token operand fragment is one ds_read_b128.  Workgroup = 128 x 128
// output tile, NWV = 4 waves as 2 x 2 of 64 x 64, or NWV = 8 waves as 2 x 4 of
// 64 x 32 (each thread then stages 8 tokens of its column: two waves per SIMD,
// so one wave's staging VALU runs beside its partner's MFMAs).
// ---------------------------------------------------------------------------
// 16-B chunk ch of image row r at ch ^ s(r), s(r) = bit 2 of r | (bit 1 ^ bit 3) << 1:
// the operand reads (ds_read_b128, rows 32n + j) stay conflict-free and the
// staging stores (ds_write_b128, 8 consecutive rows per LDS cycle, 32 banks)
// become so (s(r) = (r >> 2) & 3 left them 2-way: SQ_LDS_BANK_CONFLICT 1.66 M
// per dW2 launch).
__device__ __forceinline__ int wg_swz(int row) { return ((row >> 2) & 1) | ((((row >> 1) ^ (row >> 3)) & 1) << 1); }
__device__ __forceinline__ int wg_img(int row, int ch) { return row * 32 + 8 * (ch ^ wg_swz(row)); }

// LDA / LDB: the operands' row strides when known at compile time (the encoder's
// three products), 0 = the run-time lda / ldb.  A step whose 32 tokens are all
// valid (every step but a split's last) then loads with constant row offsets
// (folded into the loads' immediate offsets) and skips the token clamps and mask.
// MODE 3 (round 6): B arrives pre-split -- the bf16 (hi, lo) planes [M][ldb] of
// LN(x) that the forward kernel wrote beside its own split (k_ln_qkv_fwd_x3 /
// k_ln_mlp_fwd_x3b `xs`), the lo plane bplane elements after the hi plane.  A
// thread stages two columns x 8 tokens of B from dword loads (one per row: the
// column pair's hi or lo halves) and repacks them with v_perm into the same
// [column][token] chunks: no LayerNorm transform, no statistics, no split.
template <int MODE, int NWV = 4, int LDA = 0, int LDB = 0>
__global__ __launch_bounds__(64 * NWV, 8 / NWV) void k_wgrad_x3(const float* __restrict__ A, int lda,
                                                     const float* __restrict__ Bs, int ldb,
                                                     const float2* __restrict__ stats,
                                                     const float* __restrict__ lnw,
                                                     const float* __restrict__ lnb,
                                                     float* __restrict__ part,
                                                     float* __restrict__ bias_part, int64_t M,
                                                     int tok_per_split, int Acols, int Bcols, int64_t bplane) {
  static_assert(MODE != 3 || NWV == 4, "pre-split B: 4 waves (a wave stages 8 tokens of 128 columns)");
  constexpr int KT = 32, IMG = 128 * 32;
  __shared__ __attribute__((aligned(16))) __bf16 sAh[2][IMG];
  __shared__ __attribute__((aligned(16))) __bf16 sAl[2][IMG];
  __shared__ __attribute__((aligned(16))) __bf16 sBh[2][IMG];
  __shared__ __attribute__((aligned(16))) __bf16 sBl[2][IMG];
  constexpr int NB = NWV == 8 ? 1 : 2;    // 32-column b blocks per wave
  constexpr int NBW = 4 / NB;              // waves along b
  constexpr int TPT = 64 / NWV;            // tokens per thread and step (16 or 8)
  static_assert(NWV == 4 || NWV == 8, "4 or 8 waves");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int wa = (wave / NBW) * 64, wb = (wave % NBW) * 32 * NB;
  // XCD-aware order (linear id w runs on XCD w % 8): each XCD walks a contiguous
  // run of (tile, split) pairs, tiles fastest, so the tiles of one token range
  // read their shared operand through the same L2
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
  int64_t m_end = m_begin + tok_per_split;
  if (m_end > M) m_end = M;
  const int nsteps = static_cast<int>((m_end - m_begin + KT - 1) / KT);
  // staging role: column c of the tile, tokens TPT*th .. TPT*th + TPT - 1 of the step.
  // th is wave-uniform: readfirstlane makes every row index and row pointer
  // scalar, so a load is one global_load_dword (SGPR row base + the lane's
  // column offset) with no per-lane 64-bit address arithmetic or clamping.
  const int c = threadIdx.x & 127, th = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
  float gam = 1.f, bet = 0.f;
  if (MODE == 2) {
    gam = lnw[b_blk + c];
    bet = lnb[b_blk + c];
  }
  // Raw prefetch registers: the token mask and (MODE 2) the LayerNorm transform
  // are applied in store(), so the loads stay in flight across the compute.
  // (Round 1 applied the transform at load time; the ISA then waited for every
  // prefetch load before the step's MFMAs -- no latency hiding: 59 us vs 41 us
  // for MODE 0.)  The per-token statistics travel with the slot: lane l loads
  // row l's pair, store() broadcasts them with v_readlane (scalar loads there
  // serialised four K$-miss round trips per step: MODE 2 ran 2.4 us/step vs
  // 1.65 for MODE 0).
  // Two register slots: the loads of step st + 2 are issued while step st is
  // computed and step st + 1's loads (issued one step earlier) are consumed, so
  // each load has two compute phases to land (one phase, ~0.4 us of MFMAs, is
  // well under the loaded HBM latency).
  struct Slot {
    float va[TPT], vb[TPT];
    uint32_t ph[8], pl[8];  // MODE 3: rows 8 tg .. 8 tg + 7 of the column pair, hi / lo planes
    float2 st;  // MODE 2: LayerNorm statistics of the slot's row (lane & (TPT - 1))
    int nvalid;
  };
  Slot S0, S1;
  float bsum = 0.f;
  const int ca = a_blk + c, cb = b_blk + c;
  // Buffer loads: SGPR descriptor + SGPR row offset (soffset) + the lane's
  // column offset (voffset), one instruction per row and no VGPR address
  // arithmetic.  The host checks that both operands fit a 31-bit byte range.
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), static_cast<short>(0),
                                                     0x7fffffff, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Bs), static_cast<short>(0),
                                                     0x7fffffff, 0x00020000);
  const int voa = 4 * ca, vob = 4 * cb;
  // MODE 3: thread (c2, tg) stages columns b_blk + 2 c2, + 1 of tokens 8 tg .. 8 tg + 7
  const int c2 = threadIdx.x & 63, tg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rsBh = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Bs), static_cast<short>(0), 0x7fffffff,
                                                      0x00020000);
  const auto rsBl = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(reinterpret_cast<const __bf16*>(Bs) + (MODE == 3 ? bplane : 0)), static_cast<short>(0),
      0x7fffffff, 0x00020000);
  const int vop = 2 * (b_blk + 2 * c2);  // byte offset of the column pair in a bf16 row
  auto load_p = [&](Slot& S, int step) {
    // rows past the split re-read its last row (finite values; their A rows are zeroed)
    const int64_t r0 = m_begin + static_cast<int64_t>(step) * KT + 8 * tg;  // uniform
    const int64_t rl = m_end - 1;
    if (LDB > 0 && r0 + 7 <= rl) {
      const int sb = __builtin_amdgcn_readfirstlane(static_cast<int>(r0 * LDB * 2));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        S.ph[i] = __builtin_amdgcn_raw_buffer_load_b32(rsBh, vop + i * LDB * 2, sb, 0);
        S.pl[i] = __builtin_amdgcn_raw_buffer_load_b32(rsBl, vop + i * LDB * 2, sb, 0);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t r = r0 + i <= rl ? r0 + i : rl;
      const int sb = __builtin_amdgcn_readfirstlane(static_cast<int>(r * ldb * 2));
      S.ph[i] = __builtin_amdgcn_raw_buffer_load_b32(rsBh, vop, sb, 0);
      S.pl[i] = __builtin_amdgcn_raw_buffer_load_b32(rsBl, vop, sb, 0);
    }
  };
  auto load = [&](Slot& S, int step) {
    const int64_t mb = m_begin + static_cast<int64_t>(step) * KT + TPT * th;  // uniform
    const int64_t left = m_end - mb;
    S.nvalid = left < 0 ? 0 : (left > TPT ? TPT : static_cast<int>(left));
    if constexpr (MODE == 3) load_p(S, step);
    if (LDA > 0 && LDB > 0 && __builtin_amdgcn_readfirstlane(S.nvalid) == TPT) {
      if (MODE == 2) S.st = ld_stats_sys(stats, mb + (lane & (TPT - 1)));
      const int sa = __builtin_amdgcn_readfirstlane(static_cast<int>(mb * LDA * 4));
      const int sb = MODE == 3 ? 0 : __builtin_amdgcn_readfirstlane(static_cast<int>(mb * LDB * 4));
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        S.va[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsA, voa + i * LDA * 4, sa, 0));
        if constexpr (MODE != 3)
          S.vb[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsB, vob + i * LDB * 4, sb, 0));
      }
      issue_fence();
      return;
    }
    // rows past m_end re-read the last valid row (masked in store())
    const int64_t r0 = S.nvalid ? mb : m_begin;
    const int nv = __builtin_amdgcn_readfirstlane(S.nvalid > 0 ? S.nvalid : 1);
    if (MODE == 2) {  // one vector load: lane l holds row (l & (TPT - 1))'s (mean, rstd)
      const int li = lane & (TPT - 1);
      S.st = ld_stats_sys(stats, r0 + (li < nv ? li : nv - 1));
    }
    const int sa = __builtin_amdgcn_readfirstlane(static_cast<int>(r0 * lda * 4));
    const int sb = MODE == 3 ? 0 : __builtin_amdgcn_readfirstlane(static_cast<int>(r0 * ldb * 4));
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int ri = i < nv ? i : nv - 1;  // uniform
      S.va[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsA, voa, sa + ri * lda * 4, 0));
      if constexpr (MODE != 3)
        S.vb[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsB, vob, sb + ri * ldb * 4, 0));
    }
    issue_fence();
  };
  auto store = [&](Slot& S, int buf) {
    if (MODE == 2) {  // row i's statistics broadcast from lane i (v_readlane)
      const int mx = __float_as_int(S.st.x), rx = __float_as_int(S.st.y);
#pragma unroll
      for (int i = 0; i < TPT; ++i) {
        const float mean = __int_as_float(__builtin_amdgcn_readlane(mx, i));
        const float rstd = __int_as_float(__builtin_amdgcn_readlane(rx, i));
        S.vb[i] = (S.vb[i] - mean) * rstd * gam + bet;
      }
    }
    if (LDA == 0 || LDB == 0 || __builtin_amdgcn_readfirstlane(S.nvalid) < TPT) {
#pragma unroll
      for (int i = 0; i < TPT; ++i)
        if (i >= S.nvalid) S.va[i] = 0.f;
    }
#pragma unroll
    for (int half = 0; half < TPT / 8; ++half) {
      bf16x8 ah, al, bh, bl;
      split8(S.va + 8 * half, ah, al);
      const int off = wg_img(c, (TPT / 8) * th + half);
      *reinterpret_cast<bf16x8*>(sAh[buf] + off) = ah;
      *reinterpret_cast<bf16x8*>(sAl[buf] + off) = al;
      if constexpr (MODE != 3) {
        split8(S.vb + 8 * half, bh, bl);
        *reinterpret_cast<bf16x8*>(sBh[buf] + off) = bh;
        *reinterpret_cast<bf16x8*>(sBl[buf] + off) = bl;
      }
    }
    if constexpr (MODE == 3) {
      // dword i = (column 2 c2, column 2 c2 + 1) of token 8 tg + i: the even column's
      // 8 tokens are the low halves, the odd column's the high halves
      uint4 eh, oh, el, ol;
      uint32_t* e_h = &eh.x; uint32_t* o_h = &oh.x; uint32_t* e_l = &el.x; uint32_t* o_l = &ol.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        e_h[k] = __builtin_amdgcn_perm(S.ph[2 * k + 1], S.ph[2 * k], 0x05040100u);
        o_h[k] = __builtin_amdgcn_perm(S.ph[2 * k + 1], S.ph[2 * k], 0x07060302u);
        e_l[k] = __builtin_amdgcn_perm(S.pl[2 * k + 1], S.pl[2 * k], 0x05040100u);
        o_l[k] = __builtin_amdgcn_perm(S.pl[2 * k + 1], S.pl[2 * k], 0x07060302u);
      }
      const int oe = wg_img(2 * c2, tg), oo = wg_img(2 * c2 + 1, tg);
      *reinterpret_cast<uint4*>(sBh[buf] + oe) = eh;
      *reinterpret_cast<uint4*>(sBh[buf] + oo) = oh;
      *reinterpret_cast<uint4*>(sBl[buf] + oe) = el;
      *reinterpret_cast<uint4*>(sBl[buf] + oo) = ol;
    }
#pragma unroll
    for (int i = 0; i < TPT; ++i) bsum += S.va[i];
  };
  f32x16 acc[2][NB];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < NB; ++k) acc[i][k] = zero16();
  auto compute = [&](int cur) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[2], al[2], bh[NB], bl[NB];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int oa = wg_img(wa + 32 * i + j, 2 * s + h);
        ah[i] = ldsb8(sAh[cur] + oa);
        al[i] = ldsb8(sAl[cur] + oa);
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int ob = wg_img(wb + 32 * k + j, 2 * s + h);
        bh[k] = ldsb8(sBh[cur] + ob);
        bl[k] = ldsb8(sBl[cur] + ob);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < NB; ++k) acc[i][k] = mfma_x3(ah[i], al[i], bh[k], bl[k], acc[i][k]);
    }
  };
  // The loads are unconditional (past the last step they re-read it, L2-hot)
  // so the vmcnt bookkeeping is static: a store waits only for its own slot.
  const int last = nsteps - 1;
  load(S0, 0);
  store(S0, 0);
  load(S1, 1 < last ? 1 : last);
  __syncthreads();
#pragma unroll 1
  for (int st = 0; st < nsteps; st += 2) {
    // LDS buffer 0 holds step st; S1 holds step st + 1 (in flight)
    load(S0, st + 2 < last ? st + 2 : last);
    compute(0);
    if (st + 1 < nsteps) store(S1, 1);
    __syncthreads();
    if (st + 1 >= nsteps) break;
    // LDS buffer 1 holds step st + 1; S0 holds step st + 2 (in flight)
    load(S1, st + 3 < last ? st + 3 : last);
    compute(1);
    if (st + 2 < nsteps) store(S0, 0);
    __syncthreads();
  }
  float* pz = part + static_cast<int64_t>(tbz) * Acols * Bcols;
  const int a_base = a_blk + wa, b_base = b_blk + wb;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t ra = a_base + acc_row(r, h);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < NB; ++k) pz[(ra + 32 * i) * Bcols + b_base + 32 * k + j] = acc[i][k][r];
  }
  if (bias_part && tby == 0) {
    float* red = reinterpret_cast<float*>(&sAh[0][0]);  // the ring is idle after the last barrier
    red[th * 128 + c] = bsum;
    __syncthreads();
    if (th == 0)
      bias_part[static_cast<int64_t>(tbz) * Acols + a_blk + c] =
          NWV == 8 ? (red[c] + red[128 + c]) + (red[256 + c] + red[384 + c]) : red[c] + red[128 + c];
  }
}

// ---------------------------------------------------------------------------
// Attention, split-bf16                                         (model.py:778-782)
// Same decomposition as the f32 kernels (workgroup = sequence; forward and the
// dQ kernel: wave = query block with the query on the lane; dK/dV kernel: wave
// = key block with the key on the lane).  Operands that are read along the
// feature axis use [row][h][32] half images read with ds_read_b128; operands
// that are read along the token axis (V^T, K^T, dO^T, Q^T) use [token][32]
// column-block images read with ds_read_b64_tr_b16, the hardware transpose:
// one 8-token fragment = two transposed reads of 4 rows.
// ---------------------------------------------------------------------------
constexpr int AT_PAD = 96;         // padded sequence length of the P / dS layouts
constexpr int AH_PITCH = 64 + 8;   // [row][h][32] half image row (bf16): 144 B, b128 reads conflict-free

// 8-row transposed fragment from a [row][32] image (pitch 32 bf16 = 64 B: the
// 2 x 4 rows x 32 B a 32-lane half reads fall on 64 distinct banks).  Lane l of
// group g = l >> 4 receives column 16(g & 1) + (l & 15) of rows r0, r0 + 1,
// r0 + 2, r0 + 3 (first read) and rows r1 .. r1 + 3 (second read).
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* img, int r0, int r1, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = 16 * (g & 1) + 4 * p;
  const bf16x4 a = ldtr(img + (r0 + q) * 32 + col);
  const bf16x4 b = ldtr(img + (r1 + q) * 32 + col);
  bf16x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  return v;
}

// The fused backward's dS images ([query][32] per key block, 64-B rows) are
// written by ds_write_b64 with one query row per lane: 16 consecutive rows at the
// same column all land on banks {0, 1} or {16, 17} of the 32 a store spreads over
// (8-way: 1.29 M SQ_LDS_BANK_CONFLICT cycles per launch).  The 8-B chunk c of row
// r sits at c ^ ((r >> 1) & 7): 16 consecutive rows then cover all 32 banks once,
// and a transposed read (4 whole rows per 32-lane half) still covers 256
// contiguous bytes.
__device__ __forceinline__ int ds_img_off(int row, int chunk) { return row * 32 + 4 * (chunk ^ ((row >> 1) & 7)); }
__device__ __forceinline__ bf16x8 tr_frag_ds(const __bf16* img, int r0, int r1, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int c = 4 * (g & 1) + p;
  const bf16x4 a = ldtr(img + ds_img_off(r0 + q, c));
  const bf16x4 b = ldtr(img + ds_img_off(r1 + q, c));
  bf16x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  return v;
}

// Staging is split into a global->register half (*_load) and a register->LDS
// half (*_store) so a kernel can issue the next operand's loads before the
// barrier and MFMAs of the current one: plain loads stay in flight across
// __syncthreads() (no LDS-DMA is outstanding in these kernels), and each
// sequence's chain of dependent HBM round trips shrinks to about two.
constexpr int HALF_NIT = 8;  // float4 per thread: TP rows x 16 float4 over NKT * 64 threads
constexpr int COLS_NIT = 4;  // float4 per thread: TP rows x 8 float4 over NKT * 64 threads

// the feature half c of a [T][384]-strided operand (columns col0 + 64hh + 32c +
// 0..31, hh = 0,1), rows >= T clamped; stored as a split [row][hh][32] image
template <int NKT>
__device__ __forceinline__ void half_load(const float* __restrict__ seq, int T, int c, int col0, float4* v) {
  constexpr int NT = NKT * 64;
#pragma unroll
  for (int k = 0; k < HALF_NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    const int row = idx >> 4, hh = (idx >> 3) & 1, q4 = idx & 7;
    const int rc = row < T ? row : T - 1;
    v[k] = *reinterpret_cast<const float4*>(seq + static_cast<int64_t>(rc) * (3 * GHM_D) + col0 + 64 * hh +
                                            32 * c + 4 * q4);
  }
}
template <int NKT>
__device__ __forceinline__ void half_store(const float4* v, __bf16* ih, __bf16* il) {
  constexpr int NT = NKT * 64;
#pragma unroll
  for (int k = 0; k < HALF_NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    const int row = idx >> 4, hh = (idx >> 3) & 1, q4 = idx & 7;
    bf16x4 a, b;
    split4(v[k], a, b);
    stb4(ih + row * AH_PITCH + 32 * hh + 4 * q4, a);
    stb4(il + row * AH_PITCH + 32 * hh + 4 * q4, b);
  }
}

// columns col .. col+31 of rows 0..TP-1 (row pitch ld floats), rows >= T
// clamped; stored as a split [row][32] image for transposed reads
template <int NKT>
__device__ __forceinline__ void cols_load(const float* __restrict__ base, int ld, int T, int col, float4* v) {
  constexpr int NT = NKT * 64;
#pragma unroll
  for (int k = 0; k < COLS_NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    const int row = idx >> 3, q4 = idx & 7;
    const int rc = row < T ? row : T - 1;
    v[k] = *reinterpret_cast<const float4*>(base + static_cast<int64_t>(rc) * ld + col + 4 * q4);
  }
}
template <int NKT>
__device__ __forceinline__ void cols_store(const float4* v, __bf16* ih, __bf16* il) {
  constexpr int NT = NKT * 64;
#pragma unroll
  for (int k = 0; k < COLS_NIT; ++k) {
    const int idx = threadIdx.x + NT * k;
    bf16x4 a, b;
    split4(v[k], a, b);
    stb4(ih + idx * 4, a);  // row * 32 + 4 * q4 == 4 * idx
    stb4(il + idx * 4, b);
  }
}

// S^T tiles (keys on rows, this wave's queries on lanes) += X_half . Y^T where
// X rows come from a [row][h][32] half image (feature half c) and Y is the
// lane's row-layout token split into 8 k-steps (k-steps 4c .. 4c+3 used)
template <int NKT>
__device__ __forceinline__ void rows_dot_half(const __bf16* ih, const __bf16* il, const bf16x8* yh,
                                              const bf16x8* yl, int c, int j, int h, f32x16* acc) {
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int off = (32 * kt + j) * AH_PITCH + 32 * h;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
      acc[kt] = mfma_x3(ldsb8(ih + off + 8 * tt), ldsb8(il + off + 8 * tt), yh[4 * c + tt], yl[4 * c + tt], acc[kt]);
  }
}

// Attention activation (model.py:121-130, applied at :781): ACT_SOFTMAX, or the
// elementwise ACT_RELU / ACT_GELU of the scaled scores (no normalisation; keys
// past T contribute 0).  The backward needs act'(s): relu' = [P > 0]; for gelu
// the forward stores GELU'(s) beside P (Pd, same layout).
// (ACT_SOFTMAX / ACT_RELU / ACT_GELU: ghm_common.h)

template <int NKT, int ACT = ACT_SOFTMAX>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_fwd_x3(const float* __restrict__ qkv,
                                                             const float* __restrict__ H,
                                                             float* __restrict__ Hmid,
                                                             float* __restrict__ P, int T,
                                                             float scale_div, float* __restrict__ Pd = nullptr) {
  constexpr int TP = NKT * 32;
  __shared__ __attribute__((aligned(16))) __bf16 sh[TP * AH_PITCH];
  __shared__ __attribute__((aligned(16))) __bf16 sl[TP * AH_PITCH];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * (3 * GHM_D);
  const int q = 32 * w + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  float4 kst[HALF_NIT];
  half_load<NKT>(seq, T, 0, GHM_D, kst);  // K, feature half 0 (same round trip as Q)
  bf16x8 qh[8], ql[8];
  load_split64(seq + static_cast<int64_t>(qc) * (3 * GHM_D) + 64 * h, true, qh, ql);  // Q[q][64h + 8t + i]
  f32x16 s[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) s[kt] = zero16();
  half_store<NKT>(kst, sh, sl);
  half_load<NKT>(seq, T, 1, GHM_D, kst);  // K half 1 in flight across the first half's MFMAs
  __syncthreads();
  rows_dot_half<NKT>(sh, sl, qh, ql, 0, j, h, s);
  __syncthreads();
  half_store<NKT>(kst, sh, sl);
  float4 vst[COLS_NIT];
  cols_load<NKT>(seq, 3 * GHM_D, T, 2 * GHM_D, vst);  // V column block 0 in flight across softmax
  __syncthreads();
  rows_dot_half<NKT>(sh, sl, qh, ql, 1, j, h, s);
  // scores scaled by one reciprocal and exponentiated as exp2 of a base-2
  // argument: two VALU ops per score instead of an IEEE divide and a libm expf
  // (each ~10); both within 2 ulp, far below the split products' 2^-16
  const float inv_scale = 1.f / scale_div, l2e = 1.4426950408889634f;
  float inv = 0.f;
  if (ACT == ACT_SOFTMAX) {
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + acc_row(r, h);
        const float v = key < T ? s[kt][r] * inv_scale : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = fmaxf(mx, xhalf(mx));
    const float mx2 = mx * l2e;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(fmaf(s[kt][r], l2e, -mx2));
        s[kt][r] = e;
        sum += e;
      }
    }
    sum += xhalf(sum);
    inv = qv ? 1.f / sum : 0.f;
  } else {  // elementwise activation of the scaled score; act' for the backward (gelu)
    inv = qv ? 1.f : 0.f;
    float* drow = ACT == ACT_GELU ? Pd + (static_cast<int64_t>(blockIdx.x) * AT_PAD + q) * AT_PAD : nullptr;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      float dv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + acc_row(r, h);
        const float x = s[kt][r] * inv_scale;
        float a, d;
        if (ACT == ACT_RELU) {
          a = fmaxf(x, 0.f);
          d = 0.f;
        } else {
          gelu_fast(x, a, d);
        }
        const bool ok = key < T && qv;
        s[kt][r] = ok ? a : 0.f;
        dv[r] = ok ? d : 0.f;
      }
      if (ACT == ACT_GELU) {
#pragma unroll
        for (int qd = 0; qd < 4; ++qd)
          st4(drow + 32 * kt + quad_off(qd, h), dv[4 * qd], dv[4 * qd + 1], dv[4 * qd + 2], dv[4 * qd + 3]);
      }
    }
  }
  float* prow = P + (static_cast<int64_t>(blockIdx.x) * AT_PAD + q) * AT_PAD;
  bf16x8 ph[2 * NKT], pl[2 * NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kt][r] *= inv;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      st4(prow + 32 * kt + quad_off(qd, h), s[kt][4 * qd], s[kt][4 * qd + 1], s[kt][4 * qd + 2], s[kt][4 * qd + 3]);
    float pv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) pv[r] = s[kt][r];
    split_acc(pv, 0, ph[2 * kt], pl[2 * kt]);
    split_acc(pv, 1, ph[2 * kt + 1], pl[2 * kt + 1]);
  }
  // O^T[d][q] = sum_key V[key][d] P[q][key]: V column block [key][32] in LDS,
  // A fragment of k-step (kt, s) = keys 32kt + 16s + 4h + 0..3 and + 8
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    __syncthreads();  // the previous phase's LDS reads are done
    cols_store<NKT>(vst, sh, sl);
    if (dt < 3) cols_load<NKT>(seq, 3 * GHM_D, T, 2 * GHM_D + 32 * (dt + 1), vst);
    const int64_t row = (base + qc) * GHM_D + 32 * dt;
    float4 hv[4];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) hv[qd] = *reinterpret_cast<const float4*>(H + row + quad_off(qd, h));
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int r0 = 32 * kt + 16 * ss + 4 * h;
        acc = mfma_x3(tr_frag(sh, r0, r0 + 8, lane), tr_frag(sl, r0, r0 + 8, lane), ph[2 * kt + ss],
                      pl[2 * kt + ss], acc);
      }
    }
    if (qv) {
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(Hmid + row + quad_off(qd, h), hv[qd].x + acc[4 * qd], hv[qd].y + acc[4 * qd + 1],
            hv[qd].z + acc[4 * qd + 2], hv[qd].w + acc[4 * qd + 3]);
    }
  }
}

// dP^T = V dO^T, dS = P (dP - rowsum(P dP)) / c (stored, dense/padded), dQ^T = K^T dS^T
template <int NKT>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_bwd_q_x3(const float* __restrict__ qkv,
                                                               const float* __restrict__ P,
                                                               const float* __restrict__ dHmid,
                                                               float* __restrict__ dS_out,
                                                               float* __restrict__ dqkv, int T,
                                                               float scale_div) {
  constexpr int TP = NKT * 32;
  __shared__ __attribute__((aligned(16))) __bf16 sh[TP * AH_PITCH];
  __shared__ __attribute__((aligned(16))) __bf16 sl[TP * AH_PITCH];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * (3 * GHM_D);
  const int q = 32 * w + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  const float* prow = P + (static_cast<int64_t>(blockIdx.x) * AT_PAD + q) * AT_PAD;
  f32x16 dp[NKT];
  float4 kc[COLS_NIT];
  {
    float4 vst[HALF_NIT];
    half_load<NKT>(seq, T, 0, 2 * GHM_D, vst);  // V, feature half 0 (same round trip as dO)
    bf16x8 oh[8], ol[8];
    load_split64(dHmid + (base + qc) * GHM_D + 64 * h, true, oh, ol);  // dO[q][64h + 8t + i]
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) dp[kt] = zero16();
    half_store<NKT>(vst, sh, sl);
    half_load<NKT>(seq, T, 1, 2 * GHM_D, vst);  // V half 1 in flight across the first half's MFMAs
    __syncthreads();
    rows_dot_half<NKT>(sh, sl, oh, ol, 0, j, h, dp);
    __syncthreads();
    half_store<NKT>(vst, sh, sl);
    cols_load<NKT>(seq, 3 * GHM_D, T, GHM_D, kc);  // K column block 0 in flight across dS
    __syncthreads();
    rows_dot_half<NKT>(sh, sl, oh, ol, 1, j, h, dp);
  }
  const float inv_scale = 1.f / scale_div;
  float delta = 0.f;
  f32x16 p[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      const float4 pv = *reinterpret_cast<const float4*>(prow + 32 * kt + quad_off(qd, h));
      p[kt][4 * qd + 0] = qv ? pv.x : 0.f;
      p[kt][4 * qd + 1] = qv ? pv.y : 0.f;
      p[kt][4 * qd + 2] = qv ? pv.z : 0.f;
      p[kt][4 * qd + 3] = qv ? pv.w : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) delta += p[kt][r] * dp[kt][r];
  }
  delta += xhalf(delta);
  float* srow = dS_out + (static_cast<int64_t>(blockIdx.x) * AT_PAD + q) * AT_PAD;
  bf16x8 dh[2 * NKT], dl[2 * NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    float dv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) dv[r] = (p[kt][r] * (dp[kt][r] - delta)) * inv_scale;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      st4(srow + 32 * kt + quad_off(qd, h), dv[4 * qd], dv[4 * qd + 1], dv[4 * qd + 2], dv[4 * qd + 3]);
    split_acc(dv, 0, dh[2 * kt], dl[2 * kt]);
    split_acc(dv, 1, dh[2 * kt + 1], dl[2 * kt + 1]);
  }
  // dQ^T[d][q] = sum_key K[key][d] dS[q][key], K column block [key][32] in LDS
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    __syncthreads();  // the previous phase's LDS reads are done
    cols_store<NKT>(kc, sh, sl);
    if (dt < 3) cols_load<NKT>(seq, 3 * GHM_D, T, GHM_D + 32 * (dt + 1), kc);
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int r0 = 32 * kt + 16 * ss + 4 * h;
        acc = mfma_x3(tr_frag(sh, r0, r0 + 8, lane), tr_frag(sl, r0, r0 + 8, lane), dh[2 * kt + ss],
                      dl[2 * kt + ss], acc);
      }
    }
    if (qv) {
      float* o = dqkv + (base + q) * (3 * GHM_D) + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(o + quad_off(qd, h), acc[4 * qd], acc[4 * qd + 1], acc[4 * qd + 2], acc[4 * qd + 3]);
    }
  }
}

// dV^T = dO^T P and dK^T = Q^T dS, summing over queries; wave = key block, the
// key on the lane.  P / dS columns of the lane's key are read from HBM (rows >=
// T are 0) and split once; dO^T / Q^T fragments come from [query][32] column
// blocks through transposed reads.
template <int NKT>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_bwd_kv_x3(const float* __restrict__ qkv,
                                                                const float* __restrict__ P,
                                                                const float* __restrict__ dS,
                                                                const float* __restrict__ dHmid,
                                                                float* __restrict__ dqkv, int T) {
  constexpr int TP = NKT * 32, KS = TP / 16;  // k-steps over queries
  __shared__ __attribute__((aligned(16))) __bf16 soh[TP * 32];
  __shared__ __attribute__((aligned(16))) __bf16 sol[TP * 32];
  __shared__ __attribute__((aligned(16))) __bf16 sqh[TP * 32];
  __shared__ __attribute__((aligned(16))) __bf16 sql[TP * 32];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const int key = 32 * w + j;
  const bool kv = key < T;
  const float* dO = dHmid + base * GHM_D;
  const float* sq = qkv + base * (3 * GHM_D);
  // column block 0 of dO^T and Q^T: issued first, in flight while P / dS are split
  float4 ost[COLS_NIT], qst[COLS_NIT];
  cols_load<NKT>(dO, GHM_D, T, 0, ost);
  cols_load<NKT>(sq, 3 * GHM_D, T, 0, qst);
  // B fragments: P[16s + 8h + i][key] and dS[...][key], i = 0..7
  const float* pc = P + static_cast<int64_t>(blockIdx.x) * AT_PAD * AT_PAD + key;
  const float* sc = dS + static_cast<int64_t>(blockIdx.x) * AT_PAD * AT_PAD + key;
  bf16x8 pbh[KS], pbl[KS], sbh[KS], sbl[KS];
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    float pv[8], sv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int qq = 16 * st + 8 * h + i;
      pv[i] = pc[qq * AT_PAD];
      sv[i] = sc[qq * AT_PAD];
    }
    split8(pv, pbh[st], pbl[st]);
    split8(sv, sbh[st], sbl[st]);
  }
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    if (dt) __syncthreads();  // the previous phase's LDS reads are done
    cols_store<NKT>(ost, soh, sol);
    cols_store<NKT>(qst, sqh, sql);
    if (dt < 3) {
      cols_load<NKT>(dO, GHM_D, T, 32 * (dt + 1), ost);
      cols_load<NKT>(sq, 3 * GHM_D, T, 32 * (dt + 1), qst);
    }
    __syncthreads();
    f32x16 aV = zero16(), aK = zero16();
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int r0 = 16 * st + 8 * h;
      aV = mfma_x3(tr_frag(soh, r0, r0 + 4, lane), tr_frag(sol, r0, r0 + 4, lane), pbh[st], pbl[st], aV);
      aK = mfma_x3(tr_frag(sqh, r0, r0 + 4, lane), tr_frag(sql, r0, r0 + 4, lane), sbh[st], sbl[st], aK);
    }
    if (kv) {
      float* o = dqkv + (base + key) * (3 * GHM_D) + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        st4(o + 2 * GHM_D + quad_off(qd, h), aV[4 * qd], aV[4 * qd + 1], aV[4 * qd + 2], aV[4 * qd + 3]);
        st4(o + GHM_D + quad_off(qd, h), aK[4 * qd], aK[4 * qd + 1], aK[4 * qd + 2], aK[4 * qd + 3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Fused attention backward, one workgroup per sequence        (model.py:778-782)
// Phase A (as k_attn_bwd_q_x3): dP^T = V dO^T, delta, dS = P (dP - delta) / c,
//   with the queries on the lanes; P and dS go to LDS as split bf16 [query][32]
//   images per 32-key block (never to HBM).
// Phase B: dQ^T = K^T dS^T (K column blocks by transposed reads, dS from
//   registers).
// Phase C (as k_attn_bwd_kv_x3): wave w = key block w, the key on the lane;
//   dV^T = dO^T P and dK^T = Q^T dS over the queries, the P / dS B fragments
//   read from the LDS images through ds_read_b64_tr_b16.
// Against the two-kernel form it drops the dS round trip through HBM (36 + 36
// KB per sequence); P's columns (phase C) are read again, L2-warm from phase A.
// LDS (64.5 KB at T <= 96: two workgroups per CU): the dS images (2 planes x TP
// x TP bf16) + one operand-staging region (V half images, then K, then dO / Q
// column blocks).
// ---------------------------------------------------------------------------
template <int NKT, int ACT = ACT_SOFTMAX>
__global__ __launch_bounds__(NKT * 64, 2) void k_attn_bwd_x3f(const float* __restrict__ qkv,
                                                             const float* __restrict__ P,
                                                             const float* __restrict__ dHmid,
                                                             float* __restrict__ dqkv, int T,
                                                             float scale_div,
                                                             const float* __restrict__ Pd = nullptr) {
  constexpr int TP = NKT * 32, KS = TP / 16;
  constexpr int IMG = TP * TP;  // one [query][32] image per key block, NKT blocks: TP * 32 * NKT elements
  constexpr int STG = TP * AH_PITCH > 2 * TP * 32 ? TP * AH_PITCH : 2 * TP * 32;
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * IMG + 2 * STG];
  __bf16* sim_h = lds;            // dS hi [kt][query][32]
  __bf16* sim_l = lds + IMG;      // dS lo
  __bf16* sh = lds + 2 * IMG;     // staging hi (V / K images; dO^T + Q^T column blocks in phase C)
  __bf16* sl = sh + STG;          // staging lo
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * T;
  const float* seq = qkv + base * (3 * GHM_D);
  const int q = 32 * w + j;
  const bool qv = q < T;
  const int qc = qv ? q : T - 1;
  const float* prow = P + (static_cast<int64_t>(blockIdx.x) * AT_PAD + q) * AT_PAD;
  // ---- phase A: dP^T, dS ----
  f32x16 dp[NKT];
  float4 kc[COLS_NIT];
  {
    float4 vst[HALF_NIT];
    half_load<NKT>(seq, T, 0, 2 * GHM_D, vst);
    bf16x8 oh[8], ol[8];
    load_split64(dHmid + (base + qc) * GHM_D + 64 * h, true, oh, ol);
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) dp[kt] = zero16();
    half_store<NKT>(vst, sh, sl);
    half_load<NKT>(seq, T, 1, 2 * GHM_D, vst);
    __syncthreads();
    rows_dot_half<NKT>(sh, sl, oh, ol, 0, j, h, dp);
    __syncthreads();
    half_store<NKT>(vst, sh, sl);
    cols_load<NKT>(seq, 3 * GHM_D, T, GHM_D, kc);  // K column block 0 in flight across dS
    __syncthreads();
    rows_dot_half<NKT>(sh, sl, oh, ol, 1, j, h, dp);
  }
  const float inv_scale = 1.f / scale_div;
  float delta = 0.f;
  f32x16 p[NKT];  // softmax / relu: P; gelu: GELU'(s) (the factor dS needs)
  const float* arow = ACT == ACT_GELU ? Pd + (prow - P) : prow;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      const float4 pv = *reinterpret_cast<const float4*>(arow + 32 * kt + quad_off(qd, h));
      p[kt][4 * qd + 0] = qv ? pv.x : 0.f;
      p[kt][4 * qd + 1] = qv ? pv.y : 0.f;
      p[kt][4 * qd + 2] = qv ? pv.z : 0.f;
      p[kt][4 * qd + 3] = qv ? pv.w : 0.f;
    }
    if (ACT == ACT_SOFTMAX) {
#pragma unroll
      for (int r = 0; r < 16; ++r) delta += p[kt][r] * dp[kt][r];
    }
  }
  if (ACT == ACT_SOFTMAX) delta += xhalf(delta);
  bf16x8 dh[2 * NKT], dl[2 * NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    float dv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (ACT == ACT_SOFTMAX)
        dv[r] = (p[kt][r] * (dp[kt][r] - delta)) * inv_scale;
      else if (ACT == ACT_RELU)
        dv[r] = (p[kt][r] > 0.f ? dp[kt][r] : 0.f) * inv_scale;
      else
        dv[r] = (p[kt][r] * dp[kt][r]) * inv_scale;
    }
    // dS of this key block into the [query][32] images (row = this lane's query;
    // 8-B chunk quad_off / 4 = 2 qd + h, swizzled: ds_img_off)
    __bf16* dsh = sim_h + kt * TP * 32;
    __bf16* dsl = sim_l + kt * TP * 32;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      bf16x4 a, b;
      split4(make_float4(dv[4 * qd], dv[4 * qd + 1], dv[4 * qd + 2], dv[4 * qd + 3]), a, b);
      stb4(dsh + ds_img_off(q, 2 * qd + h), a);
      stb4(dsl + ds_img_off(q, 2 * qd + h), b);
    }
    split_acc(dv, 0, dh[2 * kt], dl[2 * kt]);
    split_acc(dv, 1, dh[2 * kt + 1], dl[2 * kt + 1]);
  }
  // phase C's P B fragments, P[16 st + 8 h + i][key] of this wave's key block
  // (rows >= T are 0): issued now, in flight across phase B
  const int key = 32 * w + j;
  const bool kv = key < T;
  float pcol[KS][8];
  {
    const float* pc = P + static_cast<int64_t>(blockIdx.x) * AT_PAD * AT_PAD + key;
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
      for (int i = 0; i < 8; ++i) pcol[st][i] = pc[(16 * st + 8 * h + i) * AT_PAD];
  }
  // ---- phase B: dQ^T[d][q] = sum_key K[key][d] dS[q][key] ----
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    __syncthreads();  // the previous phase's LDS reads are done
    cols_store<NKT>(kc, sh, sl);
    if (dt < 3) cols_load<NKT>(seq, 3 * GHM_D, T, GHM_D + 32 * (dt + 1), kc);
    __syncthreads();
    f32x16 acc = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        const int r0 = 32 * kt + 16 * ss + 4 * h;
        acc = mfma_x3(tr_frag(sh, r0, r0 + 8, lane), tr_frag(sl, r0, r0 + 8, lane), dh[2 * kt + ss],
                      dl[2 * kt + ss], acc);
      }
    }
    if (qv) {
      float* o = dqkv + (base + q) * (3 * GHM_D) + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        st4(o + quad_off(qd, h), acc[4 * qd], acc[4 * qd + 1], acc[4 * qd + 2], acc[4 * qd + 3]);
    }
  }
  // ---- phase C: dV^T = dO^T P, dK^T = Q^T dS; wave w = keys 32w .. 32w + 31 ----
  const float* dO = dHmid + base * GHM_D;
  __bf16* soh = sh;
  __bf16* sqh = sh + TP * 32;
  __bf16* sol = sl;
  __bf16* sql = sl + TP * 32;
  float4 ost[COLS_NIT], qst[COLS_NIT];
  cols_load<NKT>(dO, GHM_D, T, 0, ost);
  cols_load<NKT>(seq, 3 * GHM_D, T, 0, qst);
  __syncthreads();  // the P / dS images are complete; phase B's staging reads are done
  bf16x8 pbh[KS], pbl[KS], sbh[KS], sbl[KS];
  {
    const __bf16* sih = sim_h + w * TP * 32;
    const __bf16* sil = sim_l + w * TP * 32;
#pragma unroll
    for (int st = 0; st < KS; ++st) {  // B fragment: rows (queries) 16 st + 8 h .. + 7, column = the lane's key
      const int r0 = 16 * st + 8 * h;
      split8(pcol[st], pbh[st], pbl[st]);
      sbh[st] = tr_frag_ds(sih, r0, r0 + 4, lane);
      sbl[st] = tr_frag_ds(sil, r0, r0 + 4, lane);
    }
  }
#pragma unroll 1
  for (int dt = 0; dt < 4; ++dt) {
    if (dt) __syncthreads();  // the previous block's LDS reads are done
    cols_store<NKT>(ost, soh, sol);
    cols_store<NKT>(qst, sqh, sql);
    if (dt < 3) {
      cols_load<NKT>(dO, GHM_D, T, 32 * (dt + 1), ost);
      cols_load<NKT>(seq, 3 * GHM_D, T, 32 * (dt + 1), qst);
    }
    __syncthreads();
    f32x16 aV = zero16(), aK = zero16();
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int r0 = 16 * st + 8 * h;
      aV = mfma_x3(tr_frag(soh, r0, r0 + 4, lane), tr_frag(sol, r0, r0 + 4, lane), pbh[st], pbl[st], aV);
      aK = mfma_x3(tr_frag(sqh, r0, r0 + 4, lane), tr_frag(sql, r0, r0 + 4, lane), sbh[st], sbl[st], aK);
    }
    if (kv) {
      float* o = dqkv + (base + key) * (3 * GHM_D) + 32 * dt;
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        st4(o + 2 * GHM_D + quad_off(qd, h), aV[4 * qd], aV[4 * qd + 1], aV[4 * qd + 2], aV[4 * qd + 3]);
        st4(o + GHM_D + quad_off(qd, h), aK[4 * qd], aK[4 * qd + 1], aK[4 * qd + 2], aK[4 * qd + 3]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// C-ABI launchers
// ---------------------------------------------------------------------------
extern "C" int ghm_split_weights(const ghm_split_job* jobs, int n_jobs, void* stream) {
  GHM_CHECK(jobs && n_jobs >= 1 && n_jobs <= GHM_SPLIT_MAX_JOBS, "jobs");
  SplitJobs J;
  for (int i = 0; i < n_jobs; ++i) {
    const ghm_split_job& jb = jobs[i];
    GHM_CHECK(jb.Wq && jb.Wk && jb.Wv && jb.W1 && jb.W2 && jb.pack, "null pointer in job");
    GHM_CHECK((reinterpret_cast<uintptr_t>(jb.pack) & 15) == 0, "pack must be 16-byte aligned");
    GHM_CHECK(((reinterpret_cast<uintptr_t>(jb.Wq) | reinterpret_cast<uintptr_t>(jb.Wk) |
                reinterpret_cast<uintptr_t>(jb.Wv) | reinterpret_cast<uintptr_t>(jb.W1) |
                reinterpret_cast<uintptr_t>(jb.W2)) & 15) == 0, "weights must be 16-byte aligned");
    J.job[i] = jb;
  }
  hipLaunchKernelGGL(k_split_weights, dim3(SPLIT_TILES, static_cast<unsigned>(n_jobs)), dim3(256), 0,
                     ghm_stream(stream), J);
  return ghm_launch_status();
}

extern "C" int ghm_ln_qkv_fwd_x3(const float* H, const float* ln_w, const float* ln_b, const void* pack,
                                 float* qkv, float* stats, int64_t M, int D, float eps, void* stream) {
  GHM_CHECK(H && ln_w && ln_b && pack && qkv && stats, "null pointer");
  GHM_CHECK(D == GHM_D && M >= 1, "shape");
  const int tpg = qkv_tiles_per_group(M);
  hipLaunchKernelGGL(k_ln_qkv_fwd_x3, dim3(static_cast<unsigned>(ghm_token_blocks(M) * (12 / tpg))), dim3(256), 0,
                     ghm_stream(stream), H, ln_w, ln_b, reinterpret_cast<const __bf16*>(pack), qkv,
                     reinterpret_cast<float2*>(stats), M, eps, nullptr, tpg);
  return ghm_launch_status();
}

extern "C" int ghm_ln_qkv_fwd_x3s(const float* H, const float* ln_w, const float* ln_b, const void* pack, float* qkv,
                                  float* stats, void* xs, int64_t M, int D, float eps, void* stream) {
  GHM_CHECK(H && ln_w && ln_b && pack && qkv && stats && xs, "null pointer");
  GHM_CHECK(D == GHM_D && M >= 1, "shape");
  GHM_CHECK((reinterpret_cast<uintptr_t>(xs) & 15) == 0, "16-byte aligned xs");
  const int tpg = qkv_tiles_per_group(M);
  hipLaunchKernelGGL(k_ln_qkv_fwd_x3, dim3(static_cast<unsigned>(ghm_token_blocks(M) * (12 / tpg))), dim3(256), 0,
                     ghm_stream(stream), H, ln_w, ln_b, reinterpret_cast<const __bf16*>(pack), qkv,
                     reinterpret_cast<float2*>(stats), M, eps, static_cast<__bf16*>(xs), tpg);
  return ghm_launch_status();
}

static int rc_waves(int64_t M) { return (M + 127) / 128 >= 256 ? 8 : 4; }
extern "C" int64_t ghm_mlp_bwd_rc_x3_blocks(int64_t M) {
  const int64_t tok = 16 * rc_waves(M);
  return (M + tok - 1) / tok;
}

template <int NW, int STAMP, int SPLITOUT>
static void mlp_bwd_rc_launch(unsigned nblk, hipStream_t s, const float* dH_out, const float* H_mid,
                              const float* stats, const float* ln_w, const float* ln_b, const void* pack,
                              const float* b1, void* G, void* dU, float* dH_mid, float* part_ln, int64_t M,
                              uint64_t* stamps) {
  hipLaunchKernelGGL((k_mlp_bwd_rc_x3<NW, STAMP, SPLITOUT>), dim3(nblk), dim3(64 * NW), 0, s, dH_out, H_mid,
                     reinterpret_cast<const float2*>(stats), ln_w, ln_b, reinterpret_cast<const __bf16*>(pack), b1,
                     static_cast<float*>(G), static_cast<float*>(dU), dH_mid, part_ln, M, stamps);
}
template <int STAMP>
static void mlp_bwd_rc_dispatch(int64_t M, int split_out, hipStream_t s, const float* dH_out, const float* H_mid,
                                const float* stats, const float* ln_w, const float* ln_b, const void* pack,
                                const float* b1, void* G, void* dU, float* dH_mid, float* part_ln,
                                uint64_t* stamps) {
  const unsigned nblk = static_cast<unsigned>(ghm_mlp_bwd_rc_x3_blocks(M));
  if (rc_waves(M) == 8) {
    if (split_out == 1)
      mlp_bwd_rc_launch<8, STAMP, 1>(nblk, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, M, stamps);
    else if (split_out == 2)
      mlp_bwd_rc_launch<8, STAMP, 2>(nblk, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, M, stamps);
    else
      mlp_bwd_rc_launch<8, STAMP, 0>(nblk, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, M, stamps);
  } else {
    if (split_out == 1)
      mlp_bwd_rc_launch<4, STAMP, 1>(nblk, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, M, stamps);
    else if (split_out == 2)
      mlp_bwd_rc_launch<4, STAMP, 2>(nblk, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, M, stamps);
    else
      mlp_bwd_rc_launch<4, STAMP, 0>(nblk, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, M, stamps);
  }
}

extern "C" int ghm_mlp_bwd_rc_x3(const float* dH_out, const float* H_mid, const float* stats, const float* ln_w,
                                 const float* ln_b, const void* pack, const float* b1, void* G, void* dU,
                                 float* dH_mid, float* part_ln, int64_t M, int D, int F, int split_out,
                                 void* stream) {
  GHM_CHECK(dH_out && H_mid && stats && ln_w && ln_b && pack && b1 && G && dU && dH_mid && part_ln, "null pointer");
  GHM_CHECK(M < (int64_t(1) << 28), "stats byte offsets must fit 31 bits (M < 2^28 tokens)");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  GHM_CHECK(split_out >= 0 && split_out <= 2, "split_out (0 f32, 1 perm32 planes, 2 natural G planes + f32 dU)");
  GHM_CHECK(dH_mid != dH_out, "dH_mid must not alias dH_out (it is the residual input)");
  mlp_bwd_rc_dispatch<0>(M, split_out, ghm_stream(stream), dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid,
                         part_ln, nullptr);
  return ghm_launch_status();
}

// bench.py's in-graph timing of the dominant kernel: the same launch with
// per-workgroup clock stamps (2 x ghm_mlp_bwd_rc_x3_blocks(M) uint64).
extern "C" int ghm_mlp_bwd_rc_x3_stamped(const float* dH_out, const float* H_mid, const float* stats,
                                         const float* ln_w, const float* ln_b, const void* pack, const float* b1,
                                         void* G, void* dU, float* dH_mid, float* part_ln, int64_t M, int D, int F,
                                         int split_out, uint64_t* stamps, int twin, void* stream) {
  GHM_CHECK(dH_out && H_mid && stats && ln_w && ln_b && pack && b1 && G && dU && dH_mid && part_ln && stamps,
            "null pointer");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  GHM_CHECK(M < (int64_t(1) << 28), "stats byte offsets must fit 31 bits (M < 2^28 tokens)");
  GHM_CHECK(split_out >= 0 && split_out <= 2, "split_out (0 f32, 1 perm32 planes, 2 natural G planes + f32 dU)");
  GHM_CHECK(dH_mid != dH_out, "dH_mid must not alias dH_out (it is the residual input)");
  GHM_CHECK(twin == 1 || twin == 2, "twin must be 1 or 2");
  hipStream_t s = ghm_stream(stream);
  if (twin == 1)
    mlp_bwd_rc_dispatch<1>(M, split_out, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, stamps);
  else
    mlp_bwd_rc_dispatch<2>(M, split_out, s, dH_out, H_mid, stats, ln_w, ln_b, pack, b1, G, dU, dH_mid, part_ln, stamps);
  return ghm_launch_status();
}

extern "C" int ghm_qkv_bwd_x3(const float* dqkv, const float* H, const float* stats, const float* ln_w,
                              const void* pack, const float* dH_mid, float* dH, float* part_ln, int64_t M, int D,
                              float eps, void* stream) {
  GHM_CHECK(dqkv && H && ln_w && pack && dH_mid && dH && part_ln, "null pointer");
  GHM_CHECK(D == GHM_D && M >= 1, "shape");
#if GHM_QKV_STATS_LOAD
  // the forward's statistics by a system-scope load, as every other reader of
  // cross-kernel statistics (DESIGN.md §4 "Determinism"): one read of H fewer,
  // 47.6 -> 44.7 us isolated, step 4.155 -> 4.120 ms (r4_ab8)
  GHM_CHECK(stats && M * 8 < (int64_t(1) << 31), "stats");
  hipLaunchKernelGGL(k_qkv_bwd_x3<2>, dim3(static_cast<unsigned>(ghm_token_blocks(M))), dim3(256), 0,
                     ghm_stream(stream), dqkv, H, ln_w, reinterpret_cast<const __bf16*>(pack), dH_mid, dH, part_ln,
                     M, eps, reinterpret_cast<const float2*>(stats), nullptr);
#else
  (void)stats;  // the statistics are recomputed (DESIGN.md §4 "Determinism")
  hipLaunchKernelGGL(k_qkv_bwd_x3<0>, dim3(static_cast<unsigned>(ghm_token_blocks(M))), dim3(256), 0,
                     ghm_stream(stream), dqkv, H, ln_w, reinterpret_cast<const __bf16*>(pack), dH_mid, dH, part_ln,
                     M, eps, nullptr, nullptr);
#endif
  return ghm_launch_status();
}

extern "C" int ghm_qkv_bwd_x3_probe(const float* dqkv, const float* H, const float* stats, const float* ln_w,
                                    const void* pack, const float* dH_mid, float* dH, float* part_ln, float* dbg,
                                    int64_t M, int D, float eps, int mode, void* stream) {
  GHM_CHECK(dqkv && H && stats && ln_w && pack && dH_mid && dH && part_ln, "null pointer");
  GHM_CHECK(D == GHM_D && M >= 1 && mode >= 1 && mode <= 6, "shape / mode (1..6)");
  GHM_CHECK(mode < 4 || dbg, "modes 4 to 6 need dbg [M + blocks][4]");
  GHM_CHECK(M * 8 < (int64_t(1) << 31), "stats must fit a 31-bit byte range");
  const dim3 g(static_cast<unsigned>(ghm_token_blocks(M)));
  const __bf16* pk = reinterpret_cast<const __bf16*>(pack);
  const float2* st = reinterpret_cast<const float2*>(stats);
  float4* d4 = reinterpret_cast<float4*>(dbg);
  hipStream_t s = ghm_stream(stream);
  if (mode == 1)
    hipLaunchKernelGGL(k_qkv_bwd_x3<1>, g, dim3(256), 0, s, dqkv, H, ln_w, pk, dH_mid, dH, part_ln, M, eps, st, d4);
  else if (mode == 2)
    hipLaunchKernelGGL(k_qkv_bwd_x3<2>, g, dim3(256), 0, s, dqkv, H, ln_w, pk, dH_mid, dH, part_ln, M, eps, st, d4);
  else if (mode == 3)
    hipLaunchKernelGGL(k_qkv_bwd_x3<3>, g, dim3(256), 0, s, dqkv, H, ln_w, pk, dH_mid, dH, part_ln, M, eps, st, d4);
  else if (mode == 4)
    hipLaunchKernelGGL(k_qkv_bwd_x3<4>, g, dim3(256), 0, s, dqkv, H, ln_w, pk, dH_mid, dH, part_ln, M, eps, st, d4);
  else if (mode == 5)
    hipLaunchKernelGGL(k_qkv_bwd_x3<5>, g, dim3(256), 0, s, dqkv, H, ln_w, pk, dH_mid, dH, part_ln, M, eps, st, d4);
  else
    hipLaunchKernelGGL(k_qkv_bwd_x3<6>, g, dim3(256), 0, s, dqkv, H, ln_w, pk, dH_mid, dH, part_ln, M, eps, st, d4);
  return ghm_launch_status();
}

static int wgrad_x3_launch(const float* A, int lda, int A_cols, const float* B, int ldb, int B_cols, int b_mode,
                           const float* stats, const float* ln_w, const float* ln_b, float* part, float* bias_part,
                           int64_t M, int tok_per_split, int64_t bplane, void* stream);

extern "C" int ghm_wgrad_x3(const float* A, int lda, int A_cols, const float* B, int ldb, int B_cols, int b_mode,
                            const float* stats, const float* ln_w, const float* ln_b, float* part, float* bias_part,
                            int64_t M, int tok_per_split, void* stream) {
  GHM_CHECK(b_mode == 0 || b_mode == 2, "b_mode (split path: 0 plain, 2 layernorm; 3: ghm_wgrad_x3p)");
  return wgrad_x3_launch(A, lda, A_cols, B, ldb, B_cols, b_mode, stats, ln_w, ln_b, part, bias_part, M, tok_per_split,
                         0, stream);
}

extern "C" int ghm_wgrad_x3p(const float* A, int lda, int A_cols, const void* Bp, int ldb, int B_cols, int64_t bplane,
                             float* part, float* bias_part, int64_t M, int tok_per_split, void* stream) {
  GHM_CHECK(Bp && bplane >= M * ldb, "pre-split B: hi plane [M][ldb] bf16, lo plane bplane elements on");
  GHM_CHECK((reinterpret_cast<uintptr_t>(Bp) & 3) == 0 && ldb % 2 == 0, "4-byte aligned bf16 column pairs");
  GHM_CHECK(M * ldb * 2 + 2 * bplane < (int64_t(1) << 31), "planes must fit a 31-bit byte range");
  return wgrad_x3_launch(A, lda, A_cols, static_cast<const float*>(Bp), ldb, B_cols, 3, nullptr, nullptr, nullptr,
                         part, bias_part, M, tok_per_split, bplane, stream);
}

static int wgrad_x3_launch(const float* A, int lda, int A_cols, const float* B, int ldb, int B_cols, int b_mode,
                           const float* stats, const float* ln_w, const float* ln_b, float* part, float* bias_part,
                           int64_t M, int tok_per_split, int64_t bplane, void* stream) {
  GHM_CHECK(A && B && part, "null pointer");
  GHM_CHECK(A_cols > 0 && B_cols > 0 && A_cols % 128 == 0 && B_cols % 128 == 0, "A_cols/B_cols % 128");
  GHM_CHECK(lda >= A_cols && ldb >= B_cols && M >= 1, "shape");
  GHM_CHECK(tok_per_split > 0 && tok_per_split % 32 == 0, "tok_per_split must be a positive multiple of 32");
  GHM_CHECK(M * lda * 4 < (int64_t(1) << 31) && M * ldb * 4 < (int64_t(1) << 31),
            "operands must fit a 31-bit byte range (buffer-load row offsets)");
  GHM_CHECK(b_mode != 2 || (stats && ln_w && ln_b), "layernorm mode needs stats/ln_w/ln_b");
  const int64_t nsplit = (M + tok_per_split - 1) / tok_per_split;
  GHM_CHECK(nsplit <= 65535, "too many splits");
  dim3 grid(A_cols / 128, B_cols / 128, static_cast<unsigned>(nsplit));
  hipStream_t s = ghm_stream(stream);
  const float2* st = reinterpret_cast<const float2*>(stats);
  if (b_mode == 3) {  // pre-split B (LN1 / LN2 outputs of the forward, or G), 4 waves
    if (GHM_WGRAD_FAST && lda == GHM_D && ldb == GHM_F)  // dW2 (G from the MLP backward, split_out 2)
      hipLaunchKernelGGL((k_wgrad_x3<3, 4, GHM_D, GHM_F>), grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part,
                         bias_part, M, tok_per_split, A_cols, B_cols, bplane);
    else if (GHM_WGRAD_FAST && lda == GHM_F && ldb == GHM_D)  // dW1
      hipLaunchKernelGGL((k_wgrad_x3<3, 4, GHM_F, GHM_D>), grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part,
                         bias_part, M, tok_per_split, A_cols, B_cols, bplane);
    else if (GHM_WGRAD_FAST && lda == 3 * GHM_D && ldb == GHM_D)  // dWq|k|v
      hipLaunchKernelGGL((k_wgrad_x3<3, 4, 3 * GHM_D, GHM_D>), grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b,
                         part, bias_part, M, tok_per_split, A_cols, B_cols, bplane);
    else
      hipLaunchKernelGGL(k_wgrad_x3<3>, grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part, M,
                         tok_per_split, A_cols, B_cols, bplane);
  } else if (GHM_WGRAD_WAVES == 8) {
    if (b_mode == 0)
      hipLaunchKernelGGL((k_wgrad_x3<0, 8>), grid, dim3(512), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part,
                         M, tok_per_split, A_cols, B_cols, 0);
    else
      hipLaunchKernelGGL((k_wgrad_x3<2, 8>), grid, dim3(512), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part,
                         M, tok_per_split, A_cols, B_cols, 0);
  } else if (GHM_WGRAD_FAST && b_mode == 0 && lda == GHM_D && ldb == GHM_F) {  // dW2
    hipLaunchKernelGGL((k_wgrad_x3<0, 4, GHM_D, GHM_F>), grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part,
                       bias_part, M, tok_per_split, A_cols, B_cols, 0);
  } else if (GHM_WGRAD_FAST && b_mode == 2 && lda == GHM_F && ldb == GHM_D) {  // dW1
    hipLaunchKernelGGL((k_wgrad_x3<2, 4, GHM_F, GHM_D>), grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part,
                       bias_part, M, tok_per_split, A_cols, B_cols, 0);
  } else if (GHM_WGRAD_FAST && b_mode == 2 && lda == 3 * GHM_D && ldb == GHM_D) {  // dWq|k|v
    hipLaunchKernelGGL((k_wgrad_x3<2, 4, 3 * GHM_D, GHM_D>), grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b,
                       part, bias_part, M, tok_per_split, A_cols, B_cols, 0);
  } else if (b_mode == 0) {
    hipLaunchKernelGGL(k_wgrad_x3<0>, grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part, M,
                       tok_per_split, A_cols, B_cols, 0);
  } else {
    hipLaunchKernelGGL(k_wgrad_x3<2>, grid, dim3(256), 0, s, A, lda, B, ldb, st, ln_w, ln_b, part, bias_part, M,
                       tok_per_split, A_cols, B_cols, 0);
  }
  return ghm_launch_status();
}

extern "C" int ghm_attn_fwd_x3(const float* qkv, const float* H, float* H_mid, float* P, int64_t n_seq, int T,
                               int D, float scale_div, void* stream) {
  GHM_CHECK(qkv && H && H_mid && P, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  const unsigned g = static_cast<unsigned>(n_seq);
  hipStream_t s = ghm_stream(stream);
  if (T <= 32)
    hipLaunchKernelGGL(k_attn_fwd_x3<1>, dim3(g), dim3(64), 0, s, qkv, H, H_mid, P, T, scale_div);
  else if (T <= 64)
    hipLaunchKernelGGL(k_attn_fwd_x3<2>, dim3(g), dim3(128), 0, s, qkv, H, H_mid, P, T, scale_div);
  else
    hipLaunchKernelGGL(k_attn_fwd_x3<3>, dim3(g), dim3(192), 0, s, qkv, H, H_mid, P, T, scale_div);
  return ghm_launch_status();
}

// attention with an elementwise activation (model.py:121-130): act 0 softmax
// (= ghm_attn_fwd_x3), 1 relu, 2 gelu (Pd: GELU'(s) [n_seq][96][96], required)
template <int ACT>
static void attn_fwd_x3_launch(const float* qkv, const float* H, float* H_mid, float* P, float* Pd, int64_t n_seq,
                               int T, float scale_div, hipStream_t s) {
  const unsigned g = static_cast<unsigned>(n_seq);
  if (T <= 32)
    hipLaunchKernelGGL((k_attn_fwd_x3<1, ACT>), dim3(g), dim3(64), 0, s, qkv, H, H_mid, P, T, scale_div, Pd);
  else if (T <= 64)
    hipLaunchKernelGGL((k_attn_fwd_x3<2, ACT>), dim3(g), dim3(128), 0, s, qkv, H, H_mid, P, T, scale_div, Pd);
  else
    hipLaunchKernelGGL((k_attn_fwd_x3<3, ACT>), dim3(g), dim3(192), 0, s, qkv, H, H_mid, P, T, scale_div, Pd);
}
extern "C" int ghm_attn_fwd_x3_act(const float* qkv, const float* H, float* H_mid, float* P, float* Pd,
                                   int64_t n_seq, int T, int D, float scale_div, int act, void* stream) {
  GHM_CHECK(qkv && H && H_mid && P, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  GHM_CHECK(act >= 0 && act <= 2, "act must be 0 (softmax), 1 (relu) or 2 (gelu)");
  GHM_CHECK(act != 2 || Pd, "gelu attention needs Pd");
  hipStream_t s = ghm_stream(stream);
  if (act == 0)
    attn_fwd_x3_launch<ACT_SOFTMAX>(qkv, H, H_mid, P, Pd, n_seq, T, scale_div, s);
  else if (act == 1)
    attn_fwd_x3_launch<ACT_RELU>(qkv, H, H_mid, P, Pd, n_seq, T, scale_div, s);
  else
    attn_fwd_x3_launch<ACT_GELU>(qkv, H, H_mid, P, Pd, n_seq, T, scale_div, s);
  return ghm_launch_status();
}

template <int ACT>
static void attn_bwd_x3_launch(const float* qkv, const float* P, const float* Pd, const float* dH_mid, float* dqkv,
                               int64_t n_seq, int T, float scale_div, hipStream_t s) {
  const unsigned g = static_cast<unsigned>(n_seq);
  if (T <= 32)
    hipLaunchKernelGGL((k_attn_bwd_x3f<1, ACT>), dim3(g), dim3(64), 0, s, qkv, P, dH_mid, dqkv, T, scale_div, Pd);
  else if (T <= 64)
    hipLaunchKernelGGL((k_attn_bwd_x3f<2, ACT>), dim3(g), dim3(128), 0, s, qkv, P, dH_mid, dqkv, T, scale_div, Pd);
  else
    hipLaunchKernelGGL((k_attn_bwd_x3f<3, ACT>), dim3(g), dim3(192), 0, s, qkv, P, dH_mid, dqkv, T, scale_div, Pd);
}
extern "C" int ghm_attn_bwd_x3_act(const float* qkv, const float* P, const float* Pd, const float* dH_mid,
                                   float* dqkv, int64_t n_seq, int T, int D, float scale_div, int act,
                                   void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dqkv, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  GHM_CHECK(act >= 0 && act <= 2, "act must be 0 (softmax), 1 (relu) or 2 (gelu)");
  GHM_CHECK(act != 2 || Pd, "gelu attention needs Pd");
  hipStream_t s = ghm_stream(stream);
  if (act == 0)
    attn_bwd_x3_launch<ACT_SOFTMAX>(qkv, P, Pd, dH_mid, dqkv, n_seq, T, scale_div, s);
  else if (act == 1)
    attn_bwd_x3_launch<ACT_RELU>(qkv, P, Pd, dH_mid, dqkv, n_seq, T, scale_div, s);
  else
    attn_bwd_x3_launch<ACT_GELU>(qkv, P, Pd, dH_mid, dqkv, n_seq, T, scale_div, s);
  return ghm_launch_status();
}

// $GHM_ATTN_BWD = "split" selects the two-kernel attention backward (A/B and
// validation); default fused.  Read once per process.
static bool ghm_attn_bwd_fused() {
  static const bool fused = [] {
    const char* e = std::getenv("GHM_ATTN_BWD");
    return !(e && std::strcmp(e, "split") == 0);
  }();
  return fused;
}

extern "C" int ghm_attn_bwd_x3(const float* qkv, const float* P, const float* dH_mid, float* dS, float* dqkv,
                               int64_t n_seq, int T, int D, float scale_div, void* stream) {
  GHM_CHECK(qkv && P && dH_mid && dS && dqkv, "null pointer");
  GHM_CHECK(D == GHM_D && T >= 1 && T <= GHM_MAXT && n_seq >= 1, "shape (T <= 96, D == 128)");
  const unsigned g = static_cast<unsigned>(n_seq);
  hipStream_t s = ghm_stream(stream);
  if (ghm_attn_bwd_fused()) {  // one kernel, P / dS through LDS (dS is not written)
    if (T <= 32)
      hipLaunchKernelGGL(k_attn_bwd_x3f<1>, dim3(g), dim3(64), 0, s, qkv, P, dH_mid, dqkv, T, scale_div);
    else if (T <= 64)
      hipLaunchKernelGGL(k_attn_bwd_x3f<2>, dim3(g), dim3(128), 0, s, qkv, P, dH_mid, dqkv, T, scale_div);
    else
      hipLaunchKernelGGL(k_attn_bwd_x3f<3>, dim3(g), dim3(192), 0, s, qkv, P, dH_mid, dqkv, T, scale_div);
    return ghm_launch_status();
  }
  if (T <= 32) {
    hipLaunchKernelGGL(k_attn_bwd_q_x3<1>, dim3(g), dim3(64), 0, s, qkv, P, dH_mid, dS, dqkv, T, scale_div);
    hipLaunchKernelGGL(k_attn_bwd_kv_x3<1>, dim3(g), dim3(64), 0, s, qkv, P, dS, dH_mid, dqkv, T);
  } else if (T <= 64) {
    hipLaunchKernelGGL(k_attn_bwd_q_x3<2>, dim3(g), dim3(128), 0, s, qkv, P, dH_mid, dS, dqkv, T, scale_div);
    hipLaunchKernelGGL(k_attn_bwd_kv_x3<2>, dim3(g), dim3(128), 0, s, qkv, P, dS, dH_mid, dqkv, T);
  } else {
    hipLaunchKernelGGL(k_attn_bwd_q_x3<3>, dim3(g), dim3(192), 0, s, qkv, P, dH_mid, dS, dqkv, T, scale_div);
    hipLaunchKernelGGL(k_attn_bwd_kv_x3<3>, dim3(g), dim3(192), 0, s, qkv, P, dS, dH_mid, dqkv, T);
  }
  return ghm_launch_status();
}

extern "C" int ghm_ln_mlp_fwd_x3b(const float* H_mid, const float* ln_w, const float* ln_b, const void* pack,
                                  const float* b1, const float* b2, float* H_out, float* stats, int64_t M, int D,
                                  int F, float eps, void* stream) {
  GHM_CHECK(H_mid && ln_w && ln_b && pack && b1 && b2 && H_out && stats, "null pointer");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  const __bf16* pk = reinterpret_cast<const __bf16*>(pack);
  float2* st = reinterpret_cast<float2*>(stats);
  hipStream_t s = ghm_stream(stream);
  const bool big = (M + 127) / 128 >= 256;  // enough 128-token workgroups to give every CU one
  const dim3 g8(static_cast<unsigned>((M + 127) / 128)), g4(static_cast<unsigned>((M + 63) / 64));
  // GHM_MLP_FWD_WS=1: the wave-specialised schedule (k_ln_mlp_fwd_x3w); read per
  // call (a graph captures the choice made at capture time)
  const char* ws_env = std::getenv("GHM_MLP_FWD_WS");
  // 1: 8 waves (two workgroups per CU), 2: 16 waves (one), 3: 8 waves at up to 256 VGPRs (one)
  const int ws = ws_env ? std::atoi(ws_env) : 0;
  if (big && ws == 4)  // the plain schedule at 16 waves / 256 tokens: half the weight streaming per token
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3b<16>, dim3(static_cast<unsigned>((M + 255) / 256)), dim3(1024), 0, s, H_mid,
                       ln_w, ln_b, pk, b1, b2, H_out, st, M, eps, nullptr);
  else if (big && ws == 3)  // 8 waves at <= 256 VGPRs: one workgroup per CU, deeper operand prefetch
    hipLaunchKernelGGL((k_ln_mlp_fwd_x3w<8, 2>), g8, dim3(512), 0, s, H_mid, ln_w, ln_b, pk, b1, b2, H_out, st, M, eps);
  else if (big && ws == 2)
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3w<16>, dim3(static_cast<unsigned>((M + 255) / 256)), dim3(1024), 0, s, H_mid,
                       ln_w, ln_b, pk, b1, b2, H_out, st, M, eps);
  else if (big && ws)
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3w<8>, g8, dim3(512), 0, s, H_mid, ln_w, ln_b, pk, b1, b2, H_out, st, M, eps);
  else if (big)
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3b<8>, g8, dim3(512), 0, s, H_mid, ln_w, ln_b, pk, b1, b2, H_out, st, M, eps,
                       nullptr);
  else
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3b<4>, g4, dim3(256), 0, s, H_mid, ln_w, ln_b, pk, b1, b2, H_out, st, M, eps,
                       nullptr);
  return ghm_launch_status();
}

extern "C" int ghm_split3_weights(const ghm_split_job* jobs, int n_jobs, void* stream) {
  GHM_CHECK(jobs && n_jobs >= 1 && n_jobs <= GHM_SPLIT_MAX_JOBS, "jobs");
  SplitJobs J;
  for (int i = 0; i < n_jobs; ++i) {
    GHM_CHECK(jobs[i].Wq && jobs[i].Wk && jobs[i].Wv && jobs[i].W1 && jobs[i].W2 && jobs[i].pack,
              "null pointer in job");
    GHM_CHECK((reinterpret_cast<uintptr_t>(jobs[i].pack) & 15) == 0, "pack3 must be 16-byte aligned");
    J.job[i] = jobs[i];
  }
  hipLaunchKernelGGL(k_split3_weights, dim3((PK_W + PK_QKV) / 256, static_cast<unsigned>(n_jobs)), dim3(256), 0,
                     ghm_stream(stream), J);
  return ghm_launch_status();
}

extern "C" int ghm_ln_qkv_fwd_x6(const float* H, const float* ln_w, const float* ln_b, const void* pack,
                                 const void* pack3, float* qkv, float* stats, int64_t M, int D, float eps,
                                 void* stream) {
  GHM_CHECK(H && ln_w && ln_b && pack && pack3 && qkv && stats, "null pointer");
  GHM_CHECK(D == GHM_D && M >= 1, "shape");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(pack) | reinterpret_cast<uintptr_t>(pack3)) & 15) == 0,
            "16-byte aligned packs");
  const int tpg = qkv_tiles_per_group(M);
  hipLaunchKernelGGL(k_ln_qkv_fwd_x6, dim3(static_cast<unsigned>(ghm_token_blocks(M) * (12 / tpg))), dim3(256), 0,
                     ghm_stream(stream), H, ln_w, ln_b, reinterpret_cast<const __bf16*>(pack),
                     reinterpret_cast<const __bf16*>(pack3), qkv, reinterpret_cast<float2*>(stats), M, eps, tpg);
  return ghm_launch_status();
}

extern "C" int ghm_ln_mlp_fwd_x6(const float* H_mid, const float* ln_w, const float* ln_b, const void* pack,
                                 const void* pack3, const float* b1, const float* b2, float* H_out, float* stats,
                                 float* G, float* Dg, int64_t M, int D, int F, float eps, void* stream) {
  GHM_CHECK(H_mid && ln_w && ln_b && pack && pack3 && b1 && b2 && H_out && stats, "null pointer");
  GHM_CHECK((G != nullptr) == (Dg != nullptr), "G and Dg: both saved or neither");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(pack) | reinterpret_cast<uintptr_t>(pack3) |
              reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(Dg)) & 15) == 0,
            "16-byte aligned packs and G / Dg");
  const dim3 grid(static_cast<unsigned>((M + 127) / 128));
  const __bf16* pk = reinterpret_cast<const __bf16*>(pack);
  const __bf16* pk3 = reinterpret_cast<const __bf16*>(pack3);
  float2* st = reinterpret_cast<float2*>(stats);
  if (G)
    hipLaunchKernelGGL((k_ln_mlp_fwd_x6<8, true>), grid, dim3(512), 0, ghm_stream(stream), H_mid, ln_w, ln_b, pk, pk3,
                       b1, b2, H_out, st, M, eps, G, Dg);
  else
    hipLaunchKernelGGL((k_ln_mlp_fwd_x6<8, false>), grid, dim3(512), 0, ghm_stream(stream), H_mid, ln_w, ln_b, pk,
                       pk3, b1, b2, H_out, st, M, eps, nullptr, nullptr);
  return ghm_launch_status();
}

extern "C" int ghm_ln_mlp_fwd_x3bs(const float* H_mid, const float* ln_w, const float* ln_b, const void* pack,
                                   const float* b1, const float* b2, float* H_out, float* stats, void* xs, int64_t M,
                                   int D, int F, float eps, void* stream) {
  GHM_CHECK(H_mid && ln_w && ln_b && pack && b1 && b2 && H_out && stats && xs, "null pointer");
  GHM_CHECK(D == GHM_D && F == GHM_F && M >= 1, "shape (D == 128, F == 512)");
  GHM_CHECK((reinterpret_cast<uintptr_t>(xs) & 15) == 0, "16-byte aligned xs");
  const __bf16* pk = reinterpret_cast<const __bf16*>(pack);
  float2* st = reinterpret_cast<float2*>(stats);
  hipStream_t s = ghm_stream(stream);
  __bf16* x = static_cast<__bf16*>(xs);
  if ((M + 127) / 128 >= 256)
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3b<8>, dim3(static_cast<unsigned>((M + 127) / 128)), dim3(512), 0, s, H_mid,
                       ln_w, ln_b, pk, b1, b2, H_out, st, M, eps, x);
  else
    hipLaunchKernelGGL(k_ln_mlp_fwd_x3b<4>, dim3(static_cast<unsigned>((M + 63) / 64)), dim3(256), 0, s, H_mid,
                       ln_w, ln_b, pk, b1, b2, H_out, st, M, eps, x);
  return ghm_launch_status();
}
