// Split-bf16 (x3) tiled GEMM for the VLM projections (gfx950).
//
// C[m][n] = sum_k A(m, k) B(k, n) on v_mfma_f32_32x32x16_bf16 with every f32
// operand split into (hi, lo) bf16 parts while it is staged into LDS
// (ghm_split.h: hi·hi + hi·lo + lo·hi, f32 accumulate).  One template covers the
// three shapes of a Linear layer's training step:
//   forward   Y  = X W^T    A = X [M][K]        (TA = 0)  B(k,n) = W[n][k] (TB = 1)
//   data grad dX = dY W     A = dY [M][K]       (TA = 0)  B(k,n) = W[k][n] (TB = 0)
//   wgrad     dW = dY^T X   A(m,k) = dY[k][m]   (TA = 1)  B(k,n) = X[k][n] (TB = 0),
//             split over k (tokens) into f32 partial slabs summed in a fixed
//             order by k_gemm_reduce (deterministic, no atomics).
// B may be up to three separate tensors stacked along its storage rows (the
// VLM's separate W_q, W_k, W_v: one launch for the fused QKV product and its
// data gradient); the reduce writes the wgrad rows back into up to three
// destinations the same way.
//
// Tiling: 256 threads = 4 waves in a 2 x 2 grid, workgroup tile BM x 128
// (BM = 128 for N >= 768, else 64), K tile 32.  LDS images are [row][k] bf16 with a 40-element
// pitch (80 B), so each lane reads its 8-element MFMA fragment with one 16-byte
// load.  Operands whose storage is k-contiguous are staged row by row (8 lanes
// per 128-B row segment); operands whose storage is [k][outer] are loaded as
// 4 (or 2) consecutive k rows x 4 columns per thread and transposed in
// registers before the split store.  The next K tile's global loads are issued
// before the current tile's MFMAs.  Loads are buffer loads (round 5): per-thread
// byte offsets fixed for the whole K loop, a tile moves only the SGPR descriptor,
// whose record count makes rows past M / past a split's last token read as zeros
// (no per-tile 64-bit address arithmetic, row clamps or zeroing selects); for the
// weight gradients the next tile's split store is interleaved into the current
// tile's MFMAs (sched_group_barrier).
//
// The MFMA computes C^T tiles (B image rows as its A operand) so each lane owns
// one output row and 4 consecutive columns per register quad: the epilogue reads
// bias / R and writes C with 16-byte accesses (scalar-dword epilogues were
// store-issue bound: ~1.4 TB/s).  LDS is double-buffered, one barrier per K tile.
// Epilogues:
//   EPI_STORE   C = acc
//   EPI_GELU    u = acc + bias[n]; C = GELU(u), C2 = GELU'(u)   (MLP up, fused)
//   EPI_RESID   C = acc + bias[n] + R[m][n]                     (MLP down + residual)
//   EPI_MUL     C = acc * R[m][n]                               (dG * GELU'(U))
//   EPI_SLAB    slab[z][m][n] = acc                             (split-k wgrad)
//               C2[z][m] = sum over the split's k of A(m, k)      (ta = 1, C2 set: bias grad)
#include "ghm_launch.h"
#include "ghm_split.h"

namespace {

constexpr int GB_N = 128;   // workgroup tile columns
constexpr int GB_K = 32;    // K tile
constexpr int GP = 40;      // LDS pitch (bf16) of a [row][k] image

enum { EPI_STORE = 0, EPI_GELU = 1, EPI_RESID = 2, EPI_MUL = 3, EPI_SLAB = 4 };

struct GemmArgs {
  const float* A;
  int64_t lda;
  const float* B[3];
  int64_t ldb, b_chunk;   // B storage rows per tensor (0: one tensor)
  float* C;
  int64_t ldc;
  float* C2;
  const float* bias;
  const float* R;
  int64_t ldr;
  int64_t M, N, K, k_per_split;
  const __bf16* Bp;  // V bit 2: B pre-split, hi image [N][K] (pitch ldb), lo image bplane elements on
  int64_t bplane;
};

// k-contiguous tile: rows r0..r0+ROWS-1 (rows >= nrows read row nrows-1: their
// outputs are never stored), k0..k0+31 (K % 32 == 0 on this path).  Loads are
// unconditional and their data is consumed only by the split store: a guard or
// select on the loaded value forces a vmcnt wait right after the load, which
// serialises every prefetch.
// Row of a k-contiguous tile staged by element idx (8 lanes per row): within each
// 16-row group a half-wave takes rows 4 apart (0, 4, 8, 12 | 2, 6, 10, 14, and the
// odd rows in the next wave), whose 20-dword pitch offsets land in the 4 disjoint
// 16-bank windows of the LDS: conflict-free stores (plain idx >> 3 put rows 0-3
// of a half-wave on overlapping windows).  ROWS % 16 == 0.
__device__ __forceinline__ int kc_row(int idx) {
  const int w8 = idx >> 6, q = (idx >> 3) & 7;
  return 16 * (w8 >> 1) + 4 * (q & 3) + 2 * (q >> 2) + (w8 & 1);
}

template <int ROWS>
__device__ __forceinline__ void load_kc(float4* v, const float* __restrict__ base, int64_t ld, int64_t r0,
                                        int64_t nrows, int64_t k0) {
  constexpr int N = ROWS * 8 / 256;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int row = kc_row(idx), k4 = idx & 7;
    const int64_t r = r0 + row;
    const int64_t rc = r < nrows ? r : nrows - 1;
    v[i] = *reinterpret_cast<const float4*>(base + rc * ld + k0 + 4 * k4);
  }
}
template <int ROWS>
__device__ __forceinline__ void store_kc(const float4* v, __bf16* hi, __bf16* lo) {
  constexpr int N = ROWS * 8 / 256;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int idx = threadIdx.x + 256 * i;
    const int row = kc_row(idx), k4 = idx & 7;
    bf16x4 a, b;
    split4(v[i], a, b);
    stb4(hi + row * GP + 4 * k4, a);
    stb4(lo + row * GP + 4 * k4, b);
  }
}

// [k][outer] tile: k rows k0..k0+31, outer columns c0..c0+COLS-1; thread = (k group
// of RPT rows, 4 columns), k groups fastest across the lanes: the transposed LDS
// stores of a wave then spread over the k offsets of a row (distinct banks) rather
// than over 4-row groups whose 2 GP-dword stride maps onto 4 banks (PMC r4_m3: 10-17
// conflict cycles per LDS instruction in the ta = 1 / tb = 0 GEMMs); each global
// load still covers whole 128-B row segments.  Rows >= kend read a clamped row; with ZERO the store
// writes zeros for them (the split-k token tail: one operand zeroed suffices).
template <int COLS>
__device__ __forceinline__ void load_oc(float4* v, const float* __restrict__ base, int64_t ld, int64_t k0,
                                        int64_t kend, int64_t c0) {
  constexpr int RPT = COLS / 32, KG = 32 / RPT;
  const int kg = threadIdx.x % KG, c4 = threadIdx.x / KG;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int64_t k = k0 + RPT * kg + i;
    const int64_t kc = k < kend ? k : kend - 1;  // kend >= 1; an empty split (k0 >= kend) reads row kend - 1
    v[i] = *reinterpret_cast<const float4*>(base + kc * ld + c0 + 4 * c4);
  }
}
template <int COLS, bool ZERO>
__device__ __forceinline__ void store_oc(const float4* v, __bf16* hi, __bf16* lo, int64_t k0, int64_t kend) {
  constexpr int RPT = COLS / 32, KG = 32 / RPT;
  const int kg = threadIdx.x % KG, c4 = threadIdx.x / KG;  // k groups fastest: see load_oc
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    __bf16 h[RPT], l[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      float x = c == 0 ? v[i].x : (c == 1 ? v[i].y : (c == 2 ? v[i].z : v[i].w));
      if constexpr (ZERO) x = (k0 + RPT * kg + i < kend) ? x : 0.f;
      split1(x, h[i], l[i]);
    }
    const int off = (4 * c4 + c) * GP + RPT * kg;
    if constexpr (RPT == 4) {
      bf16x4 a, b;
      a[0] = h[0]; a[1] = h[1]; a[2] = h[2]; a[3] = h[3];
      b[0] = l[0]; b[1] = l[1]; b[2] = l[2]; b[3] = l[3];
      stb4(hi + off, a);
      stb4(lo + off, b);
    } else {
      typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
      bf16x2 a, b;
      a[0] = h[0]; a[1] = h[1];
      b[0] = l[0]; b[1] = l[1];
      *reinterpret_cast<bf16x2*>(hi + off) = a;
      *reinterpret_cast<bf16x2*>(lo + off) = b;
    }
  }
}

// Buffer-load staging (BUF): each thread's byte offsets inside a K tile are
// fixed (computed once, the same row / column mapping as load_kc / load_oc); a
// tile moves only the SGPR descriptor's base, and its record count ends the
// operand at the last valid row, so rows past M (k-contiguous A), past the
// split's last token (the [k][outer] operands) or past the end of K read as
// zeros in hardware: no per-tile 64-bit address arithmetic, row clamps or
// zeroing selects on the VALU.
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t rs, int voff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, int64_t bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  const int n = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes > 0 ? bytes : 0));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo),
                                           static_cast<short>(0), n, 0x00020000);
}
// a thread's byte offsets: k-contiguous tile (row kc_row(idx), 4 floats at k4)
template <int ROWS>
__device__ __forceinline__ void voff_kc(int* vo, int64_t ld) {
#pragma unroll
  for (int i = 0; i < ROWS * 8 / 256; ++i) {
    const int idx = threadIdx.x + 256 * i;
    vo[i] = static_cast<int>((kc_row(idx) * ld + 4 * (idx & 7)) * 4);
  }
}
// [k][outer] tile: rows RPT kg + i, columns 4 c4 (load_oc's mapping)
template <int COLS>
__device__ __forceinline__ void voff_oc(int* vo, int64_t ld) {
  constexpr int RPT = COLS / 32, KG = 32 / RPT;
  const int kg = threadIdx.x % KG, c4 = threadIdx.x / KG;
#pragma unroll
  for (int i = 0; i < RPT; ++i) vo[i] = static_cast<int>(((RPT * kg + i) * ld + 4 * c4) * 4);
}

// exact-f32 variant (F32): [row][k] f32 images with a 36-float pitch, staged
// without a split; lane (r, h) of a v_mfma_f32_32x32x2f32 takes k = 16 h + kk at
// step kk (both operands alike), so a lane's 16 operands are four 16-byte reads.
constexpr int GPF = 36;
template <int ROWS>
__device__ __forceinline__ void store_kc_f32(const float4* v, float* img) {
  constexpr int N = ROWS * 8 / 256;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int idx = threadIdx.x + 256 * i;
    *reinterpret_cast<float4*>(img + kc_row(idx) * GPF + 4 * (idx & 7)) = v[i];
  }
}
template <int COLS, bool ZERO>
__device__ __forceinline__ void store_oc_f32(const float4* v, float* img, int64_t k0, int64_t kend) {
  constexpr int RPT = COLS / 32, KG = 32 / RPT;
  const int kg = threadIdx.x % KG, c4 = threadIdx.x / KG;  // k groups fastest: see load_oc
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float x[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      x[i] = c == 0 ? v[i].x : (c == 1 ? v[i].y : (c == 2 ? v[i].z : v[i].w));
      if constexpr (ZERO) x[i] = (k0 + RPT * kg + i < kend) ? x[i] : 0.f;
    }
    float* dst = img + (4 * c4 + c) * GPF + RPT * kg;
    if constexpr (RPT == 4) *reinterpret_cast<float4*>(dst) = make_float4(x[0], x[1], x[2], x[3]);
    else *reinterpret_cast<float2*>(dst) = make_float2(x[0], x[1]);
  }
}

// F32 = true: the exact-f32 product (the VLM's precision "f32" mode) on the same
// tiling, prefetch schedule and epilogues; GELU then uses the erf form.
// V bit 0 (BUF): stage through buffer loads (bload4 / brsrc above) instead of
// pointer loads; bit 1 (IL, with BUF): the next tile's split store is issued in
// the same scheduling region as the current tile's MFMAs, interleaved with them
// by sched_group_barrier (a wave's staging VALU fills its own MFMA gaps); bit 2
// (BP, with BUF and TB): B arrives pre-split (g.Bp: bf16 hi / lo images [N][K],
// written once per step by ghm_split_pack), so its tiles are copied into LDS
// without a split -- the weights' split, which every workgroup of a column
// block repeated, is gone from the K loop
template <bool TA, bool TB, int EPI, int TM, bool F32, int V = 0, int BN = GB_N>
__global__ __launch_bounds__(256, (V & 8) ? 3 : 2) void k_gemm_x3(GemmArgs g) {
  constexpr bool BUF = (V & 1) != 0, IL = (V & 3) == 3, BP = (V & 4) != 0;
  // SB (V & 8): one LDS tile instead of two (a second barrier per K tile), so
  // three 128 x 128 workgroups fit a CU's LDS (TM = 2, split-bf16, not IL)
  constexpr bool SB = (V & 8) != 0;
  static_assert(!SB || (TM == 2 && !F32 && !IL), "single LDS tile: TM = 2, split-bf16, no interleave");
  constexpr int NBUF = SB ? 1 : 2;
  static_assert(!BP || (BUF && TB && !F32), "pre-split B: buffer loads, k-contiguous, split-bf16");
  // BN: workgroup tile columns, 128 or 64 (split-bf16 only: twice the workgroups
  // for the N = 256 products); a wave owns JN 32-column blocks
  static_assert(BN == GB_N || (BN == 64 && !F32), "64-column tiles: split-bf16");
  constexpr int JN = BN / 64;
  // pre-split B: BN rows x 32 bf16 = 4 16-byte chunks per row and plane, NBP per thread
  constexpr int NBP = BN / 64;
  constexpr int BM = 64 * TM;
  constexpr int NA = TA ? BM / 32 : BM * 8 / 256;   // float4 per thread, A tile
  constexpr int NB = TB ? BN * 8 / 256 : BN / 32;
  // double-buffered images: [buf][row][k], split (hi, lo) bf16 or (F32) f32
  constexpr int SM_X3 = NBUF * 2 * (BM + BN) * GP * 2, SM_F32 = 2 * (BM + BN) * GPF * 4;
  __shared__ __attribute__((aligned(16))) char smem[F32 ? SM_F32 : SM_X3];
  __bf16(*ah)[BM * GP] = reinterpret_cast<__bf16(*)[BM * GP]>(smem);
  __bf16(*al)[BM * GP] = ah + NBUF;
  __bf16(*bh)[BN * GP] = reinterpret_cast<__bf16(*)[BN * GP]>(smem + NBUF * 2 * BM * GP * 2);
  __bf16(*bl)[BN * GP] = bh + NBUF;
  float(*af)[BM * GPF] = reinterpret_cast<float(*)[BM * GPF]>(smem);
  float(*bf)[BN * GPF] = reinterpret_cast<float(*)[BN * GPF]>(smem + 2 * BM * GPF * 4);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so
  // linear id w runs on XCD w % 8; remap so each XCD walks a contiguous run of
  // tiles (n fastest) and the n-tiles sharing an A row block (and, in split-k,
  // the tiles sharing a token range) hit the same L2
  int lin = static_cast<int>(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
  {
    const int full = static_cast<int>(gridDim.x * gridDim.y * gridDim.z) / 8 * 8;
    if (lin < full) lin = (lin % 8) * (full / 8) + lin / 8;
  }
  const int tbx = lin % static_cast<int>(gridDim.x);
  const int tby = (lin / static_cast<int>(gridDim.x)) % static_cast<int>(gridDim.y);
  const int tbz = lin / static_cast<int>(gridDim.x * gridDim.y);
  const int64_t n0 = static_cast<int64_t>(tbx) * BN;
  const int64_t m0 = static_cast<int64_t>(tby) * BM;
  const int64_t kb = static_cast<int64_t>(tbz) * g.k_per_split;
  const int64_t ke = kb + g.k_per_split < g.K ? kb + g.k_per_split : g.K;
  const int64_t klast = ke > kb ? kb + (ke - 1 - kb) / GB_K * GB_K : kb;  // start of the last K tile

  // B tile base: the stacked tensor holding storage row (TB ? n0 : k)
  auto bbase = [&](int64_t srow, int64_t& local) -> const float* {
    if (g.b_chunk <= 0) {
      local = srow;
      return g.B[0];
    }
    // at most three stacked tensors: compares, not a 64-bit division
    const int q = srow >= 2 * g.b_chunk ? 2 : (srow >= g.b_chunk ? 1 : 0);
    local = srow - q * g.b_chunk;
    return g.B[q];
  };

  int voa[BUF ? NA : 1], vob[BUF ? NB : 1];
  if constexpr (BUF) {
    if constexpr (TA) voff_oc<BM>(voa, g.lda);
    else voff_kc<BM>(voa, g.lda);
    if constexpr (BP) {
      // BN rows x 32 bf16 = 4 16-byte chunks per row and plane: chunk idx & 3 of
      // row idx >> 2, idx = thread + 256 i (i < NBP)
#pragma unroll
      for (int i = 0; i < NBP; ++i) {
        const int idx = threadIdx.x + 256 * i;
        vob[i] = static_cast<int>(((idx >> 2) * g.ldb + 8 * (idx & 3)) * 2);
      }
    } else if constexpr (TB) {
      voff_kc<BN>(vob, g.ldb);
    } else {
      voff_oc<BN>(vob, g.ldb);
    }
  }
  auto load = [&](float4* va, float4* vb, int64_t k0) {
    if constexpr (BUF) {
      // the tile's rows from its first: k0 on for [k][outer], m0 / n0 on for
      // k-contiguous.  A tile at or past ke (the prefetch past the last one) gets
      // no records at all: its k-contiguous rows would otherwise run past the end
      // of the operand's last row.
      const int64_t krows = ke - k0 < GB_K ? ke - k0 : GB_K;
      const bool live = k0 < ke;
      if constexpr (TA) {
        const auto rs = brsrc(g.A + k0 * g.lda + m0, krows * g.lda * 4);
#pragma unroll
        for (int i = 0; i < NA; ++i) va[i] = bload4(rs, voa[i]);
      } else {
        const int64_t mrows = g.M - m0 < BM ? g.M - m0 : BM;
        const auto rs = brsrc(g.A + m0 * g.lda + k0, live ? mrows * g.lda * 4 : 0);
#pragma unroll
        for (int i = 0; i < NA; ++i) va[i] = bload4(rs, voa[i]);
      }
      if constexpr (BP) {
        // vb[0 .. NBP-1]: the hi chunks, vb[NBP ..]: the lo chunks (raw bf16 bits)
        const __bf16* b = g.Bp + n0 * g.ldb + k0;
        const auto rh = brsrc(b, live ? BN * g.ldb * 2 : 0);
        const auto rl = brsrc(b + g.bplane, live ? BN * g.ldb * 2 : 0);
#pragma unroll
        for (int i = 0; i < NBP; ++i) {
          vb[i] = bload4(rh, vob[i]);
          vb[NBP + i] = bload4(rl, vob[i]);
        }
      } else if constexpr (TB) {
        int64_t ln;
        const float* b = bbase(n0, ln);
        const auto rs = brsrc(b + ln * g.ldb + k0, live ? BN * g.ldb * 4 : 0);
#pragma unroll
        for (int i = 0; i < NB; ++i) vb[i] = bload4(rs, vob[i]);
      } else {
        int64_t lk;
        const float* b = bbase(k0, lk);
        const auto rs = brsrc(b + lk * g.ldb + n0, krows * g.ldb * 4);
#pragma unroll
        for (int i = 0; i < NB; ++i) vb[i] = bload4(rs, vob[i]);
      }
      return;
    }
    if constexpr (TA) load_oc<BM>(va, g.A, g.lda, k0, ke, m0);
    else load_kc<BM>(va, g.A, g.lda, m0, g.M, k0);
    if constexpr (TB) {
      int64_t ln;
      const float* b = bbase(n0, ln);
      load_kc<BN>(vb, b + ln * g.ldb, g.ldb, 0, BN, k0);
    } else {
      int64_t lk;
      const float* b = bbase(k0, lk);
      load_oc<BN>(vb, b + (lk - k0) * g.ldb, g.ldb, k0, ke, n0);
    }
  };
  // split-k wgrad with C2 set: per-thread row sums of A (the bias gradient, sum
  // over tokens of dY) accumulated from the staged registers, tile by tile in k order
  float4 rs = make_float4(0.f, 0.f, 0.f, 0.f);
  // k0: the K tile being stored (zeroes A's token tail in split-k)
  auto store = [&](const float4* va, const float4* vb, int buf, int64_t k0) {
    if constexpr (TA && EPI == EPI_SLAB) {
      if (g.C2) {
        const int kg = threadIdx.x % (32 / NA);  // load_oc's lane mapping
#pragma unroll
        for (int i = 0; i < NA; ++i)
          if (BUF || k0 + NA * kg + i < ke) {  // BUF: rows past the split read as zeros
            rs.x += va[i].x; rs.y += va[i].y; rs.z += va[i].z; rs.w += va[i].w;
          }
      }
    }
    if constexpr (F32) {
      if constexpr (TA) store_oc_f32<BM, !BUF>(va, af[buf], k0, ke);
      else store_kc_f32<BM>(va, af[buf]);
      if constexpr (TB) store_kc_f32<BN>(vb, bf[buf]);
      else store_oc_f32<BN, false>(vb, bf[buf], k0, ke);
      return;
    }
    if constexpr (TA) store_oc<BM, !BUF>(va, ah[buf], al[buf], k0, ke);
    else store_kc<BM>(va, ah[buf], al[buf]);
    if constexpr (BP) {
#pragma unroll
      for (int i = 0; i < NBP; ++i) {
        const int idx = threadIdx.x + 256 * i;
        const int off = (idx >> 2) * GP + 8 * (idx & 3);
        *reinterpret_cast<float4*>(bh[buf] + off) = vb[i];
        *reinterpret_cast<float4*>(bl[buf] + off) = vb[NBP + i];
      }
    } else if constexpr (TB) store_kc<BN>(vb, bh[buf], bl[buf]);
    else store_oc<BN, false>(vb, bh[buf], bl[buf], k0, ke);
  };

  // acc[i][j] = C^T tile: rows = 32 n (B image rows), lanes = 32 m (A image rows),
  // so each lane owns one output row m and 4 consecutive n per register quad
  f32x16 acc[TM][JN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = zero16();

  auto compute = [&](int buf) {
    if constexpr (F32) {
      float xa[TM][16], yb[JN][16];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(af[buf] + (32 * (TM * wm + i) + r) * GPF + 16 * h + 4 * q);
          xa[i][4 * q] = v.x; xa[i][4 * q + 1] = v.y; xa[i][4 * q + 2] = v.z; xa[i][4 * q + 3] = v.w;
        }
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(bf[buf] + (32 * (JN * wn + j) + r) * GPF + 16 * h + 4 * q);
          yb[j][4 * q] = v.x; yb[j][4 * q + 1] = v.y; yb[j][4 * q + 2] = v.z; yb[j][4 * q + 3] = v.w;
        }
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < JN; ++j) acc[i][j] = mfma32(yb[j][kk], xa[i][kk], acc[i][j]);
      return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 xh[TM], xl[TM], yh[JN], yl[JN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int off = (32 * (TM * wm + i) + r) * GP + 16 * s + 8 * h;
        xh[i] = ldsb8(ah[buf] + off);
        xl[i] = ldsb8(al[buf] + off);
      }
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        const int off = (32 * (JN * wn + j) + r) * GP + 16 * s + 8 * h;
        yh[j] = ldsb8(bh[buf] + off);
        yl[j] = ldsb8(bl[buf] + off);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) acc[i][j] = mfma_x3(yh[j], yl[j], xh[i], xl[i], acc[i][j]);
    }
  };

  // IL: one MFMA, then up to 6 VALU (the split of the next tile) and one LDS
  // write, repeated over the tile's MFMAs
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < TM * JN * 2 * 3; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
  };

  // two K tiles in flight in registers (sets p, q) ahead of the LDS tile being
  // multiplied: the global loads of a tile are issued two compute phases before
  // their split store, which keeps enough bytes in flight per CU to cover HBM
  // latency (one tile ahead left the streaming GEMMs latency-bound)
  if constexpr (TM == 2) {
    // 128 x 128 tiles: one K tile in flight (two would exceed 256 VGPRs)
    float4 pa[NA], pb[NB];
    load(pa, pb, kb);
    store(pa, pb, 0, kb);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += GB_K) {
      const bool more = k0 + GB_K < ke;
      // unconditional: no branch around the loads (BUF: a tile past ke reads zeros)
      load(pa, pb, more || BUF ? k0 + GB_K : k0);
      issue_fence();
      compute(buf);
      if constexpr (SB) {
        __syncthreads();  // every wave is done with the tile before it is overwritten
        if (more) store(pa, pb, 0, k0 + GB_K);
        __syncthreads();
        continue;
      }
      if constexpr (IL) {
        store(pa, pb, buf ^ 1, k0 + GB_K);  // past the end: zeros into a buffer nobody reads
        interleave();
      } else if (more) {
        store(pa, pb, buf ^ 1, k0 + GB_K);
      }
      __syncthreads();
      buf ^= 1;
    }
  } else {
    float4 pa[NA], pb[NB], qa[NA], qb[NB];
    // loads are unconditional (past the last tile they re-read it, unused): a load
    // under a branch made the wait-count pass drain every load at the next store
    auto kt = [&](int64_t k) { return BUF || k < ke ? k : klast; };  // BUF: past ke reads zeros
    load(pa, pb, kb);
    load(qa, qb, kt(kb + GB_K));
    issue_fence();
    store(pa, pb, 0, kb);
    __syncthreads();
    load(pa, pb, kt(kb + 2 * GB_K));
    issue_fence();
    for (int64_t k0 = kb; k0 < ke; k0 += 2 * GB_K) {
      // LDS[0] = tile k0; q = tile k0 + 32; p = tile k0 + 64 (in flight)
      compute(0);
      if constexpr (IL) {
        store(qa, qb, 1, k0 + GB_K);
        interleave();
      } else if (k0 + GB_K < ke) {
        store(qa, qb, 1, k0 + GB_K);
      }
      __syncthreads();
      load(qa, qb, kt(k0 + 3 * GB_K));
      issue_fence();
      if (k0 + GB_K >= ke) break;
      compute(1);
      if constexpr (IL) {
        store(pa, pb, 0, k0 + 2 * GB_K);
        interleave();
      } else if (k0 + 2 * GB_K < ke) {
        store(pa, pb, 0, k0 + 2 * GB_K);
      }
      __syncthreads();
      load(pa, pb, kt(k0 + 4 * GB_K));
      issue_fence();
    }
  }

  if constexpr (TA && EPI == EPI_SLAB) {
    // row-sum partial C2[z][m]: the 32 / NA k groups of a column quad combined in
    // group order through LDS, once per (m block, split)
    if (g.C2 && tbx == 0) {
      constexpr int C4 = BM / 4, G = 32 / NA;  // lane = c4 * G + k group
      float4* red = reinterpret_cast<float4*>(smem);
      __syncthreads();
      red[threadIdx.x] = rs;
      __syncthreads();
      if (threadIdx.x < C4) {
        float4 a = red[threadIdx.x * G];
#pragma unroll
        for (int q = 1; q < G; ++q) {
          const float4 v = red[threadIdx.x * G + q];
          a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
        const int64_t m = m0 + 4 * threadIdx.x;
        if (m < g.M) *reinterpret_cast<float4*>(g.C2 + static_cast<int64_t>(tbz) * g.M + m) = a;
      }
    }
  }

  // epilogue: lane row m = m0 + 32(TM wm + i) + r; register quad qd of acc[i][j] holds
  // n = n0 + 32(2 wn + j) + 8 qd + 4 h + 0..3 -> one 16-byte access per quad
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int64_t m = m0 + 32 * (TM * wm + i) + r;
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < JN; ++j) {
      const int64_t nb = n0 + 32 * (JN * wn + j);
      float4 rv[4], bv[4];
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int64_t n = nb + quad_off(qd, h);
        if constexpr (EPI == EPI_GELU || EPI == EPI_RESID) bv[qd] = *reinterpret_cast<const float4*>(g.bias + n);
        if constexpr (EPI == EPI_RESID || EPI == EPI_MUL)
          rv[qd] = *reinterpret_cast<const float4*>(g.R + m * g.ldr + n);
      }
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int64_t n = nb + quad_off(qd, h);
        float x[4] = {acc[i][j][4 * qd], acc[i][j][4 * qd + 1], acc[i][j][4 * qd + 2], acc[i][j][4 * qd + 3]};
        if constexpr (EPI == EPI_STORE) {
          st4(g.C + m * g.ldc + n, x[0], x[1], x[2], x[3]);
        } else if constexpr (EPI == EPI_GELU) {
          const float bb[4] = {bv[qd].x, bv[qd].y, bv[qd].z, bv[qd].w};
          float gg[4], dd[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if constexpr (F32) gelu_and_grad(x[t] + bb[t], gg[t], dd[t]);
            else gelu_fast(x[t] + bb[t], gg[t], dd[t]);
          }
          st4(g.C + m * g.ldc + n, gg[0], gg[1], gg[2], gg[3]);
          st4(g.C2 + m * g.ldc + n, dd[0], dd[1], dd[2], dd[3]);
        } else if constexpr (EPI == EPI_RESID) {
          st4(g.C + m * g.ldc + n, (x[0] + bv[qd].x) + rv[qd].x, (x[1] + bv[qd].y) + rv[qd].y,
              (x[2] + bv[qd].z) + rv[qd].z, (x[3] + bv[qd].w) + rv[qd].w);
        } else if constexpr (EPI == EPI_MUL) {
          st4(g.C + m * g.ldc + n, x[0] * rv[qd].x, x[1] * rv[qd].y, x[2] * rv[qd].z, x[3] * rv[qd].w);
        } else {
          st4(g.C + (static_cast<int64_t>(tbz) * g.M + m) * g.N + n, x[0], x[1], x[2], x[3]);
        }
      }
    }
  }
}

// s[0] + s[stride] + ... + s[(nsplit - 1) stride], added in z order, with the loads
// of 8 slabs in flight at once (one load per round trip, as the plain loop
// compiled, made the 16-slab reduce 16 serial HBM round trips: 6.2 -> 5.2 us,
// profiles/r5_red_ab.txt)
__device__ __forceinline__ float4 slab_sum(const float4* s, int nsplit, int64_t stride) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int z = 0; z < nsplit; z += 8) {
    // unconditional loads (past the last slab they re-read it, unused): a load
    // under a branch drains the wait count at the join
    float4 b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) b[u] = s[static_cast<int64_t>(z + u < nsplit ? z + u : nsplit - 1) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (z + u == 0) {
        a = b[0];  // the first slab as is (not 0 + s[0]: the sign of a zero stays)
      } else if (z + u < nsplit) {
        a.x += b[u].x; a.y += b[u].y; a.z += b[u].z; a.w += b[u].w;
      }
    }
  }
  return a;
}

// dst rows (stacked as B is): out = sum_z slab[z] in z order.  Workgroups past the
// slab's (nmain) sum the row-sum partials bslab[z][M] into bdst (bias gradient).
__global__ __launch_bounds__(256) void k_gemm_reduce(const float* __restrict__ slab, int nsplit, int64_t M, int64_t N,
                                                      float* d0, float* d1, float* d2, int64_t chunk,
                                                      const float* __restrict__ bslab, float* bdst, int64_t nmain) {
  if (static_cast<int64_t>(blockIdx.x) >= nmain) {
    const int64_t b4 = (static_cast<int64_t>(blockIdx.x) - nmain) * 256 + threadIdx.x;
    if (4 * b4 >= M) return;
    reinterpret_cast<float4*>(bdst)[b4] = slab_sum(reinterpret_cast<const float4*>(bslab) + b4, nsplit, M / 4);
    return;
  }
  const int64_t i4 = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t total = M * N;
  if (4 * i4 >= total) return;
  const float4 a = slab_sum(reinterpret_cast<const float4*>(slab) + i4, nsplit, total / 4);
  const int64_t m = (4 * i4) / N, n = (4 * i4) % N;
  float* d = d0;
  int64_t lm = m;
  if (chunk > 0) {
    const int64_t q = m / chunk;
    lm = m - q * chunk;
    d = q == 0 ? d0 : (q == 1 ? d1 : d2);
  }
  *reinterpret_cast<float4*>(d + lm * N + n) = a;
}

// Column sums out[n] = sum_m X[m][n] (bias and position-embedding gradients),
// deterministic: stage 1 sums a chunk of rows per workgroup (threads split into
// row groups when N/4 < 256, combined through LDS in group order), stage 2 sums
// the chunk partials in chunk order.
__global__ __launch_bounds__(256) void k_colsum_part(const float* __restrict__ X, int64_t M, int64_t N, int64_t R,
                                                     float* __restrict__ part) {
  __shared__ float4 red[256];
  const int64_t N4 = N / 4;
  const int CB = N4 < 256 ? static_cast<int>(N4) : 256;
  const int G = 256 / CB;
  const int t = threadIdx.x, grp = t / CB;
  const int64_t c4 = static_cast<int64_t>(blockIdx.x) * CB + t % CB;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * R;
  const int64_t r1 = r0 + R < M ? r0 + R : M;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (grp < G && c4 < N4) {
    for (int64_t row0 = r0 + grp; row0 < r1; row0 += 4 * G) {  // 4 loads in flight, summed in row order
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t row = row0 + u * G;
        v[u] = row < r1 ? *reinterpret_cast<const float4*>(X + row * N + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
  }
  red[t] = a;
  __syncthreads();
  if (grp == 0 && c4 < N4) {
    for (int q = 1; q < G; ++q) {
      const float4 v = red[t + q * CB];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    reinterpret_cast<float4*>(part + static_cast<int64_t>(blockIdx.y) * N)[c4] = a;
  }
}

// chunk partials summed per column: 64 float4 columns per workgroup (fewer when
// N/4 < 64), the chunks split over 256 / columns thread groups, groups combined in
// order through LDS
// Columns from float4 index split4 on go to out2 (its first n2 floats): the
// weighted sums' class totals ride in the same partial rows (ghm_wcolsum).
__global__ __launch_bounds__(256) void k_colsum_final(const float* __restrict__ part, int nchunk, int64_t N,
                                                      float* __restrict__ out, float* __restrict__ out2,
                                                      int64_t split4, int n2, int cbw) {
  __shared__ float4 red[256];
  const int64_t N4 = N / 4;
  const int CB = N4 < cbw ? static_cast<int>(N4) : cbw;
  const int G = 256 / CB;
  const int t = threadIdx.x, grp = t / CB;
  const int64_t c4 = static_cast<int64_t>(blockIdx.x) * CB + t % CB;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (grp < G && c4 < N4) {
    // 8 loads issued together per round (a dependent one-at-a-time chain was
    // latency-bound: ~18 us for 256 chunks)
    for (int z0 = grp; z0 < nchunk; z0 += 8 * G) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int z = z0 + u * G;
        v[u] = z < nchunk ? reinterpret_cast<const float4*>(part + static_cast<int64_t>(z) * N)[c4]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
  }
  red[t] = a;
  __syncthreads();
  if (grp == 0 && c4 < N4) {
    for (int q = 1; q < G; ++q) {
      const float4 v = red[t + q * CB];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (c4 < split4) {
      reinterpret_cast<float4*>(out)[c4] = a;
    } else if (out2) {
      const int j = static_cast<int>(4 * (c4 - split4));
      const float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (j + k < n2) out2[j + k] = v[k];
    }
  }
}

// Weighted column sums (the readout and token-embedding weight gradients,
// reference model.py _read_out / t_embedding through autograd):
//   out[c][n] = sum_m w(m, c) X[xrow(m)][n],   wsum[c] = sum_m w(m, c)
// w(m, c) = W[m][c] (dense, e.g. dlogits) or [tok[m] == c] (token ids: the one-hot
// product without the one-hot matrix); xrow(m) = (m / rps) * seq_rows + off + m % rps
// picks the text (or prefix) rows of each sequence.  Up to 16 classes per
// workgroup (blockIdx.y selects the class block); rows split over 256 / (N/4)
// thread groups combined in group order through LDS, chunk partials
// [chunk][C*N | wsum] summed in chunk order by k_colsum_final: deterministic.
template <bool TOK>
__global__ __launch_bounds__(256) void k_wcolsum_part(const float* __restrict__ W, const uint8_t* __restrict__ tok,
                                                      int C, const float* __restrict__ X, int64_t rps,
                                                      int64_t seq_rows, int64_t off, int64_t M, int64_t N, int64_t R,
                                                      int64_t ldp, float* __restrict__ part) {
  __shared__ float4 red[256];
  __shared__ float redw[64][16];  // up to 256 / (N/4) = 64 row groups
  const int N4 = static_cast<int>(N / 4);
  const int G = 256 / N4;
  const int t = threadIdx.x, grp = t / N4, c4 = t % N4;
  const int cb = static_cast<int>(blockIdx.y) * 16;
  const int nc = C - cb < 16 ? C - cb : 16;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int64_t r1 = r0 + R < M ? r0 + R : M;
  float4 acc[16];
  float ws[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    ws[c] = 0.f;
  }
  if (grp < G) {
    // U rows' loads in flight per round, accumulated in row order; the row map in
    // 32-bit arithmetic (rows < 2^31), skipped when it is the identity
    const bool ident = rps == seq_rows && off == 0;
    const uint32_t rps32 = static_cast<uint32_t>(rps), sr32 = static_cast<uint32_t>(seq_rows),
                   off32 = static_cast<uint32_t>(off);
    constexpr int U = TOK ? 8 : 4;  // rows in flight per round
    for (int64_t row0 = r0 + grp; row0 < r1; row0 += U * G) {
      // branch-free body: rows past the chunk re-read row0 with weight 0
      float4 x[U];
      int k[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = row0 + u * G;
        ok[u] = row < r1;
        const int64_t rr = ok[u] ? row : row0;
        const uint32_t r = static_cast<uint32_t>(rr);
        const int64_t xr = ident ? rr : static_cast<int64_t>((r / rps32) * sr32 + off32 + r % rps32);
        x[u] = *reinterpret_cast<const float4*>(X + xr * N + 4 * c4);
        if (TOK) {
          const int tv = static_cast<int>(tok[rr]);  // unconditional: a guarded load serialises the round
          k[u] = ok[u] ? tv - cb : -1;
        }
      }
      if (TOK) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int c = 0; c < 16; ++c) {
            if (c < nc) {  // uniform
              const bool hit = c == k[u];
              acc[c].x += hit ? x[u].x : 0.f;
              acc[c].y += hit ? x[u].y : 0.f;
              acc[c].z += hit ? x[u].z : 0.f;
              acc[c].w += hit ? x[u].w : 0.f;
            }
          }
        }
      } else {
        // every weight load issued before the first use (clamped columns, zeroed)
        float wv[U][16];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t rr = ok[u] ? row0 + u * G : row0;
#pragma unroll
          for (int c = 0; c < 16; ++c) wv[u][c] = W[rr * C + (cb + c < C ? cb + c : C - 1)];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
          for (int c = 0; c < 16; ++c)
            if (c < nc) {  // uniform
              const float w = ok[u] ? wv[u][c] : 0.f;
              acc[c].x += w * x[u].x; acc[c].y += w * x[u].y; acc[c].z += w * x[u].z; acc[c].w += w * x[u].w;
              ws[c] += w;
            }
        }
      }
    }
  }
  float* dst = part + static_cast<int64_t>(blockIdx.x) * ldp;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c < nc) {  // uniform over the workgroup
      red[t] = acc[c];
      __syncthreads();
      if (grp == 0) {
        float4 a = acc[c];
        for (int q = 1; q < G; ++q) {
          const float4 v = red[t + q * N4];
          a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
        reinterpret_cast<float4*>(dst + static_cast<int64_t>(cb + c) * N)[c4] = a;
      }
      __syncthreads();
    }
  }
  if (c4 == 0 && grp < G) {
#pragma unroll
    for (int c = 0; c < 16; ++c) redw[grp][c] = ws[c];
  }
  __syncthreads();
  if (t < nc) {
    float a = redw[0][t];
    for (int q = 1; q < G; ++q) a += redw[q][t];
    dst[static_cast<int64_t>(C) * N + cb + t] = a;
  }
}

// Small-C linear rows (the VLM readout, reference model.py _read_out):
//   Y[m][c] = b[c] + sum_d X[m][d] W[c][d]       (k_rows_linear, forward logits)
// W [C][D] staged in LDS; 16 lanes per row, lane l holding features 4l + 64j..;
// each class's 16 lane partials summed by a 4-step xor butterfly, lane c % 16
// keeps class c.  Fixed order per row: deterministic.
template <int D>
__global__ __launch_bounds__(256) void k_rows_linear(const float* __restrict__ X, const float* __restrict__ W,
                                                     const float* __restrict__ b, float* __restrict__ Y, int64_t M,
                                                     int C) {
  extern __shared__ float ws[];
  constexpr int NJ = D / 64;
  for (int i = threadIdx.x; i < C * D / 4; i += 256)
    reinterpret_cast<float4*>(ws)[i] = reinterpret_cast<const float4*>(W)[i];
  __syncthreads();
  const int l = threadIdx.x & 15;
  const int64_t m = static_cast<int64_t>(blockIdx.x) * 16 + (threadIdx.x >> 4);
  if (m >= M) return;
  float4 x[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) x[j] = *reinterpret_cast<const float4*>(X + m * D + 64 * j + 4 * l);
  float out[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int cq = 0; cq < 4; ++cq) {
    for (int ci = 0; ci < 16; ++ci) {
      const int c = 16 * cq + ci;
      if (c >= C) break;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float4 w = reinterpret_cast<const float4*>(ws + c * D + 64 * j)[l];
        s += x[j].x * w.x + x[j].y * w.y + x[j].z * w.z + x[j].w * w.w;
      }
      s += __shfl_xor(s, 8, 16);
      s += __shfl_xor(s, 4, 16);
      s += __shfl_xor(s, 2, 16);
      s += __shfl_xor(s, 1, 16);
      if (l == ci) out[cq] = s;
    }
  }
#pragma unroll
  for (int cq = 0; cq < 4; ++cq) {
    const int c = 16 * cq + l;
    if (c < C) Y[m * C + c] = out[cq] + b[c];
  }
}

// dX[m][d] = sum_c dZ[m][c] W[c][d]   (the readout's data gradient): one float4 of
// a row per thread, W [C][D] in LDS, classes summed in order.
template <int D>
__global__ __launch_bounds__(256) void k_rows_linear_t(const float* __restrict__ dZ, const float* __restrict__ W,
                                                       float* __restrict__ dX, int64_t M, int C) {
  extern __shared__ float ws[];
  constexpr int D4 = D / 4, RPB = 256 / D4;
  for (int i = threadIdx.x; i < C * D4; i += 256)
    reinterpret_cast<float4*>(ws)[i] = reinterpret_cast<const float4*>(W)[i];
  __syncthreads();
  const int q = threadIdx.x % D4;
  const int64_t m = static_cast<int64_t>(blockIdx.x) * RPB + threadIdx.x / D4;
  if (m >= M) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c = 0; c < C; ++c) {
    const float z = dZ[m * C + c];
    const float4 w = reinterpret_cast<const float4*>(ws + c * D)[q];
    a.x += z * w.x; a.y += z * w.y; a.z += z * w.z; a.w += z * w.w;
  }
  reinterpret_cast<float4*>(dX + m * D)[q] = a;
}

void colsum_plan(int64_t M, int64_t N, int64_t& colblocks, int64_t& nchunk, int64_t& R) {
  const int64_t N4 = N / 4;
  colblocks = N4 < 256 ? 1 : (N4 + 255) / 256;
  int64_t want = 256 / colblocks;
  if (want < 1) want = 1;
  const int64_t cap = (M + 7) / 8;
  nchunk = want < cap ? want : cap;
  if (nchunk < 1) nchunk = 1;
  R = (M + nchunk - 1) / nchunk;
  nchunk = (M + R - 1) / R;
}

template <bool TA, bool TB, int EPI, bool F32>
void launch_tm(const GemmArgs& g, int nsplit, hipStream_t s) {
  // measured (VLM shapes, M = 10,368): 128 x 128 tiles with one K tile in flight
  // are faster for N >= 768; 64 x 128 tiles with two K tiles in flight for N = 256
  // GHM_GEMM_TM2_MIN_N: A/B knob for that cut (read once)
  static const int64_t tm2_min = [] {
    const char* e = getenv("GHM_GEMM_TM2_MIN_N");
    return e ? static_cast<int64_t>(atoll(e)) : static_cast<int64_t>(768);
  }();
  // staging variant V: buffer loads (1), with the split stores interleaved into
  // the MFMAs (3, split-bf16 only) for the weight gradients (ta = 1), where it
  // measured 39.6 -> 37.6 us; the forward / data-gradient shapes ran slower with
  // it (profiles/r5_vlm_gemm_buf.txt).  GHM_GEMM_BUF = 0 / 1 / 3 forces one
  // variant for every shape (A/B knob, read per call).
  const char* be = getenv("GHM_GEMM_BUF");
  const int v = be ? atoi(be) : (TA ? 3 : 1);
  const unsigned gx = static_cast<unsigned>(g.N / GB_N);
  const dim3 g2(gx, static_cast<unsigned>((g.M + 127) / 128), nsplit), g1(gx, static_cast<unsigned>((g.M + 63) / 64), nsplit);
  const bool narrow_n = g.N % GB_N != 0 || (TB && g.b_chunk > 0 && g.b_chunk % GB_N != 0);
  if (g.N >= tm2_min && !narrow_n) {
    // split-bf16: one LDS tile and a second barrier per K tile (V = 9), so that
    // three workgroups share a CU (40 KB of LDS, 156-164 VGPRs) instead of two (80
    // KB): GELU forward 42.0 -> 36.5, dU product 47.4 -> 43.5, dW2 39.6 -> 37.2 us,
    // VLM step -1.3 % (profiles/r5_sb_ab.txt); the same for the 64 x 128 weight
    // gradients (30 KB, 154 VGPRs) was slower, 37.5 -> 39.2 us (r5_sb1_ab.txt).
    // GHM_GEMM_SB = 0 restores the double buffer (A/B knob, read per call).
    if constexpr (!F32) {
      const char* sb = getenv("GHM_GEMM_SB");
      if ((sb ? atoi(sb) == 1 : true) && v != 0) {
        hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 2, F32, 9>), g2, dim3(256), 0, s, g);
        return;
      }
    }
    if (v == 1) hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 2, F32, 1>), g2, dim3(256), 0, s, g);
    else if (v == 3) hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 2, F32, F32 ? 1 : 3>), g2, dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 2, F32>), g2, dim3(256), 0, s, g);
    return;
  }
  // 64 x 64 tiles (split-bf16, buffer staging) for the forward / data-gradient
  // products with N < tm2_min: twice the workgroups for the N = 256 shapes, which
  // ran 324 per launch; measured 43.4 -> 34.2 us (dY W2, VLM) and 39.4 -> 36.2 us
  // (X Wo^T + residual), while the weight gradients ran slower with them (38.4 ->
  // 44.8 us; profiles/r5_bn_ab.txt).  GHM_GEMM_BN = 64 / 128 forces one tile width
  // for every shape (A/B knob, read per call).
  const char* bne = getenv("GHM_GEMM_BN");
  // N or a stacked tb = 1 operand's chunk not a multiple of 128 (the generic-width
  // CLIP encoder, n_embd = 64: N = 64 / 192 products, csrc path of
  // models/gemm_encoder.py): only the 64-column tiles fit
  const bool narrow = g.N % GB_N != 0 || (TB && g.b_chunk > 0 && g.b_chunk % GB_N != 0);
  const bool bn64 = narrow || (bne ? atoi(bne) == 64 : !TA);
  if constexpr (!F32) {
    if (bn64 && (v == 1 || v == 3 || narrow)) {
      const dim3 g64(static_cast<unsigned>(g.N / 64), static_cast<unsigned>((g.M + 63) / 64), nsplit);
      if (v != 3) hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 1, F32, 1, 64>), g64, dim3(256), 0, s, g);
      else hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 1, F32, 3, 64>), g64, dim3(256), 0, s, g);
      return;
    }
  }
  if (v == 1) hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 1, F32, 1>), g1, dim3(256), 0, s, g);
  else if (v == 3) hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 1, F32, F32 ? 1 : 3>), g1, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((k_gemm_x3<TA, TB, EPI, 1, F32>), g1, dim3(256), 0, s, g);
}

// pre-split B (V = 5: buffer loads + BP), ta = 0: the VLM's weight products
template <int EPI>
void launch_bp(const GemmArgs& g, int nsplit, hipStream_t s) {
  const int64_t tm2_min = [] {
    const char* e = getenv("GHM_GEMM_TM2_MIN_N");
    return e ? static_cast<int64_t>(atoll(e)) : static_cast<int64_t>(768);
  }();
  const unsigned gx = static_cast<unsigned>(g.N / GB_N);
  if (g.N >= tm2_min) {
    // one LDS tile (V bit 3) as launch_tm's split-bf16 128 x 128 tiles: three
    // workgroups per CU (the double-buffered pre-split kernel ran the GELU forward
    // at 40.4 against 37.6 us without the pre-split, profiles/r6_vpack64); GHM_GEMM_SB
    // = 0 restores the double buffer
    const char* sb = getenv("GHM_GEMM_SB");
    const dim3 g2(gx, static_cast<unsigned>((g.M + 127) / 128), nsplit);
    if (sb ? atoi(sb) == 1 : true)
      hipLaunchKernelGGL((k_gemm_x3<false, true, EPI, 2, false, 13>), g2, dim3(256), 0, s, g);
    else
      hipLaunchKernelGGL((k_gemm_x3<false, true, EPI, 2, false, 5>), g2, dim3(256), 0, s, g);
    return;
  }
  // N < tm2_min: 64 x 64 tiles, as launch_tm's ta = 0 products (the pre-split path
  // at 64 x 128 ran the N = 256 products on half the workgroups: pack on 4.51 vs
  // off 4.44-4.45 ms per VLM step, profiles/r6_vpack_ab.txt); GHM_GEMM_BN = 128 keeps
  // the 128-column tiles
  const char* bne = getenv("GHM_GEMM_BN");
  if (bne && atoi(bne) == 128)
    hipLaunchKernelGGL((k_gemm_x3<false, true, EPI, 1, false, 5>),
                       dim3(gx, static_cast<unsigned>((g.M + 63) / 64), nsplit), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((k_gemm_x3<false, true, EPI, 1, false, 5, 64>),
                       dim3(static_cast<unsigned>(g.N / 64), static_cast<unsigned>((g.M + 63) / 64), nsplit),
                       dim3(256), 0, s, g);
}

// Weight pre-split for the pre-split-B GEMMs: job j (8 int64: src, src pitch,
// rows, cols, dst, dst pitch, lo-plane offset, transpose) writes the split of the
// f32 matrix src [rows][cols] into the bf16 hi image at dst (transpose: dst[c][r])
// and the lo image plane elements on; one workgroup per 64 x 64 tile, through
// LDS so the reads and the (transposed) writes are both row-contiguous.  The
// split is split1's, the one the GEMM's staging applies: bit-identical operands.
__global__ __launch_bounds__(256) void k_split_pack(const int64_t* __restrict__ jobs) {
  __shared__ float tile[64][65];
  const int64_t* jb = jobs + 8 * blockIdx.y;
  const float* src = reinterpret_cast<const float*>(jb[0]);
  const int64_t lds_ = jb[1], rows = jb[2], cols = jb[3];
  __bf16* dst = reinterpret_cast<__bf16*>(jb[4]);
  const int64_t ldd = jb[5], plane = jb[6];
  const bool tr = jb[7] != 0;
  const int64_t tcols = (cols + 63) / 64;
  if (static_cast<int64_t>(blockIdx.x) >= tcols * ((rows + 63) / 64)) return;
  const int64_t r0 = 64 * (blockIdx.x / tcols), c0 = 64 * (blockIdx.x % tcols);
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, c = i & 63;
    tile[r][c] = (r0 + r < rows && c0 + c < cols) ? src[(r0 + r) * lds_ + c0 + c] : 0.f;
  }
  __syncthreads();
  // output element (a, b) of the tile: row a, column b of the (transposed) image
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int a = i >> 6, b = i & 63;
    const int64_t orow = (tr ? c0 : r0) + a, ocol = (tr ? r0 : c0) + b;
    if (orow >= (tr ? cols : rows) || ocol >= (tr ? rows : cols)) continue;
    __bf16 h, l;
    split1(tr ? tile[b][a] : tile[a][b], h, l);
    dst[orow * ldd + ocol] = h;
    dst[orow * ldd + ocol + plane] = l;
  }
}

}  // namespace

extern "C" int64_t ghm_gemm_slab_elems(int64_t M, int64_t N, int nsplit) { return M * N * nsplit; }

static int gemm_launch(bool f32, int ta, int tb, int epi, const float* A, int64_t lda, const float* B0,
                       const float* B1, const float* B2, int64_t ldb, int64_t b_chunk, float* C, int64_t ldc,
                       float* C2, const float* bias, const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K,
                       int nsplit, void* stream) {
  GHM_CHECK(A && B0 && C, "null pointer");
  // N % 128 == 0, or (split-bf16: 64-column tiles) N % 64 == 0
  GHM_CHECK(M >= 1 && N >= 64 && N % (f32 ? GB_N : 64) == 0 && K >= 1 && nsplit >= 1 && nsplit <= 256,
            "shape (N % 128 == 0; split-bf16: N % 64 == 0)");
  GHM_CHECK(!(ta && tb), "TA and TB together are not a VLM shape");
  GHM_CHECK(epi >= EPI_STORE && epi <= EPI_SLAB, "epilogue");
  GHM_CHECK(nsplit == 1 || epi == EPI_SLAB, "split k needs the slab epilogue");
  GHM_CHECK(epi != EPI_GELU || (bias && C2), "GELU epilogue needs bias and C2");
  GHM_CHECK(!C2 || epi == EPI_GELU || (epi == EPI_SLAB && ta && M % 4 == 0), "C2: GELU' or the ta = 1 slab row sums");
  GHM_CHECK(epi != EPI_RESID || (bias && R), "residual epilogue needs bias and R");
  GHM_CHECK(epi != EPI_MUL || R, "product epilogue needs R");
  GHM_CHECK(lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 && ldr % 4 == 0, "row strides % 4 == 0");
  // buffer-load staging: a tile's byte offsets (up to 128 rows) fit 31 bits
  GHM_CHECK(lda < (1 << 20) && ldb < (1 << 20), "row strides < 2^20 floats");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(R) |
              reinterpret_cast<uintptr_t>(C2) | reinterpret_cast<uintptr_t>(bias)) & 15) == 0,
            "16-byte aligned operands");
  // k-contiguous operands are read as float4 along k
  // k-contiguous operands (A with ta = 0, B with tb = 1) and the stacked / [k][n]
  // weights are read in whole 32-deep K tiles; only the split-k wgrad has a tail
  GHM_CHECK(ta || K % 32 == 0, "K % 32 == 0 unless ta = 1");
  if (b_chunk > 0) {
    const int64_t rows = tb ? N : K;
    // a B tile never straddles two tensors: tb = 1 tiles are BN rows of n (128, or
    // 64 when the chunk is not a multiple of 128), tb = 0 tiles 32 rows of k
    GHM_CHECK(b_chunk % (f32 ? GB_N : 64) == 0 && rows <= 3 * b_chunk && B1 && (rows <= 2 * b_chunk || B2),
              "stacked B: chunk % 128 == 0 (split-bf16: % 64), at most 3 tensors");
  }
  GemmArgs g;
  g.A = A; g.lda = lda;
  g.B[0] = B0; g.B[1] = B1 ? B1 : B0; g.B[2] = B2 ? B2 : B0;
  g.ldb = ldb; g.b_chunk = b_chunk;
  g.C = C; g.ldc = ldc; g.C2 = C2; g.bias = bias; g.R = R; g.ldr = ldr;
  g.M = M; g.N = N; g.K = K;
  g.k_per_split = ((K + nsplit - 1) / nsplit + GB_K - 1) / GB_K * GB_K;
  // an empty split would stage (unused) A columns past K: only ta = 1 clamps them
  GHM_CHECK(ta || (nsplit - 1) * g.k_per_split < K, "ta = 0 split k: every split needs a K tile");
  hipStream_t s = ghm_stream(stream);
#define GHM_GEMM_CASE(TA_, TB_, E_)                                    \
  if (ta == TA_ && tb == TB_ && epi == E_) {                           \
    if (f32) launch_tm<TA_, TB_, E_, true>(g, nsplit, s);              \
    else launch_tm<TA_, TB_, E_, false>(g, nsplit, s);                 \
    return ghm_launch_status();                                        \
  }
  GHM_GEMM_CASE(0, 1, EPI_STORE)
  GHM_GEMM_CASE(0, 1, EPI_GELU)
  GHM_GEMM_CASE(0, 1, EPI_RESID)
  GHM_GEMM_CASE(0, 0, EPI_STORE)
  GHM_GEMM_CASE(0, 0, EPI_MUL)
  GHM_GEMM_CASE(0, 0, EPI_RESID)  // the f32 VLM's dX += dk Wk, dv Wv
  GHM_GEMM_CASE(0, 0, EPI_SLAB)  // split-k data gradient (VLM dX over K = 768 / 1024)
  GHM_GEMM_CASE(1, 0, EPI_SLAB)
  GHM_GEMM_CASE(1, 0, EPI_STORE)
#undef GHM_GEMM_CASE
  GHM_CHECK(false, "unsupported (ta, tb, epilogue) combination");
}

extern "C" int ghm_gemm_x3(int ta, int tb, int epi, const float* A, int64_t lda, const float* B0, const float* B1,
                           const float* B2, int64_t ldb, int64_t b_chunk, float* C, int64_t ldc, float* C2,
                           const float* bias, const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K, int nsplit,
                           void* stream) {
  return gemm_launch(false, ta, tb, epi, A, lda, B0, B1, B2, ldb, b_chunk, C, ldc, C2, bias, R, ldr, M, N, K, nsplit,
                     stream);
}

extern "C" int ghm_gemm_f32(int ta, int tb, int epi, const float* A, int64_t lda, const float* B0, const float* B1,
                            const float* B2, int64_t ldb, int64_t b_chunk, float* C, int64_t ldc, float* C2,
                            const float* bias, const float* R, int64_t ldr, int64_t M, int64_t N, int64_t K,
                            int nsplit, void* stream) {
  return gemm_launch(true, ta, tb, epi, A, lda, B0, B1, B2, ldb, b_chunk, C, ldc, C2, bias, R, ldr, M, N, K, nsplit,
                     stream);
}

extern "C" int ghm_gemm_x3p(int epi, const float* A, int64_t lda, const void* Bp, int64_t ldbp, int64_t bplane,
                            float* C, int64_t ldc, float* C2, const float* bias, const float* R, int64_t ldr, int64_t M,
                            int64_t N, int64_t K, int nsplit, void* stream) {
  GHM_CHECK(A && Bp && C, "null pointer");
  GHM_CHECK(M >= 1 && N >= GB_N && N % GB_N == 0 && K >= 32 && K % 32 == 0 && nsplit >= 1 && nsplit <= 256,
            "shape (N % 128 == 0, K % 32 == 0)");
  GHM_CHECK(epi >= EPI_STORE && epi <= EPI_SLAB, "epilogue");
  GHM_CHECK(nsplit == 1 || epi == EPI_SLAB, "split k needs the slab epilogue");
  GHM_CHECK(epi != EPI_GELU || (bias && C2), "GELU epilogue needs bias and C2");
  GHM_CHECK(epi != EPI_RESID || (bias && R), "residual epilogue needs bias and R");
  GHM_CHECK(epi != EPI_MUL || R, "product epilogue needs R");
  GHM_CHECK(!C2 || epi == EPI_GELU, "C2: GELU' only");
  GHM_CHECK(lda % 4 == 0 && ldc % 4 == 0 && ldr % 4 == 0 && ldbp % 8 == 0 && bplane % 8 == 0 && ldbp >= K,
            "row strides (pre-split images: pitch and plane % 8 bf16)");
  GHM_CHECK(lda < (1 << 20) && ldbp < (1 << 20), "row strides < 2^20");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(C) | reinterpret_cast<uintptr_t>(R) |
              reinterpret_cast<uintptr_t>(C2) | reinterpret_cast<uintptr_t>(bias) |
              reinterpret_cast<uintptr_t>(Bp)) & 15) == 0,
            "16-byte aligned operands");
  GemmArgs g{};
  g.A = A; g.lda = lda;
  g.B[0] = g.B[1] = g.B[2] = nullptr;
  g.ldb = ldbp; g.b_chunk = 0;
  g.C = C; g.ldc = ldc; g.C2 = C2; g.bias = bias; g.R = R; g.ldr = ldr;
  g.M = M; g.N = N; g.K = K;
  g.k_per_split = ((K + nsplit - 1) / nsplit + GB_K - 1) / GB_K * GB_K;
  GHM_CHECK((nsplit - 1) * g.k_per_split < K, "split k: every split needs a K tile");
  g.Bp = static_cast<const __bf16*>(Bp); g.bplane = bplane;
  hipStream_t s = ghm_stream(stream);
  switch (epi) {
    case EPI_STORE: launch_bp<EPI_STORE>(g, nsplit, s); break;
    case EPI_GELU: launch_bp<EPI_GELU>(g, nsplit, s); break;
    case EPI_RESID: launch_bp<EPI_RESID>(g, nsplit, s); break;
    case EPI_MUL: launch_bp<EPI_MUL>(g, nsplit, s); break;
    default: launch_bp<EPI_SLAB>(g, nsplit, s); break;
  }
  return ghm_launch_status();
}

extern "C" int ghm_split_pack(const int64_t* jobs, int n_jobs, int max_tiles, void* stream) {
  GHM_CHECK(jobs && n_jobs >= 1 && n_jobs <= 65535 && max_tiles >= 1, "jobs");
  hipLaunchKernelGGL(k_split_pack, dim3(static_cast<unsigned>(max_tiles), static_cast<unsigned>(n_jobs)), dim3(256), 0,
                     ghm_stream(stream), jobs);
  return ghm_launch_status();
}

extern "C" int ghm_gemm_reduce_bias(const float* slab, int nsplit, int64_t M, int64_t N, float* D0, float* D1,
                                    float* D2, int64_t chunk, const float* bslab, float* bdst, void* stream) {
  GHM_CHECK(slab && D0 && nsplit >= 1 && M >= 1 && N >= 4 && N % 4 == 0, "bad arguments");
  GHM_CHECK(chunk <= 0 || (M <= 3 * chunk && D1 && (M <= 2 * chunk || D2)), "stacked destination");
  GHM_CHECK(!bslab == !bdst && (!bslab || M % 4 == 0), "row sums: bslab and bdst together, M % 4 == 0");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(bslab) | reinterpret_cast<uintptr_t>(bdst)) & 15) == 0,
            "16-byte aligned row sums");
  const int64_t nmain = (M * N / 4 + 255) / 256, nb = bslab ? (M / 4 + 255) / 256 : 0;
  hipLaunchKernelGGL(k_gemm_reduce, dim3(static_cast<unsigned>(nmain + nb)), dim3(256), 0, ghm_stream(stream), slab,
                     nsplit, M, N, D0, D1, D2, chunk, bslab, bdst, nmain);
  return ghm_launch_status();
}

extern "C" int ghm_gemm_reduce(const float* slab, int nsplit, int64_t M, int64_t N, float* D0, float* D1, float* D2,
                               int64_t chunk, void* stream) {
  return ghm_gemm_reduce_bias(slab, nsplit, M, N, D0, D1, D2, chunk, nullptr, nullptr, stream);
}

extern "C" int64_t ghm_colsum_part_elems(int64_t M, int64_t N) {
  int64_t cb, nc, R;
  colsum_plan(M, N, cb, nc, R);
  return nc * N;
}

extern "C" int ghm_colsum(const float* X, int64_t M, int64_t N, float* out, float* part, void* stream) {
  GHM_CHECK(X && out && part && M >= 1 && N >= 4 && N % 4 == 0, "bad arguments (N % 4 == 0)");
  GHM_CHECK(N / 4 >= 256 || 256 % (N / 4) == 0, "N / 4 must divide 256 or be >= 256");
  GHM_CHECK(N / 4 >= 64 || 64 % (N / 4) == 0, "N / 4 must divide 64 or be >= 64");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(part)) &
             15) == 0, "16-byte aligned operands");
  int64_t cb, nc, R;
  colsum_plan(M, N, cb, nc, R);
  hipStream_t s = ghm_stream(stream);
  hipLaunchKernelGGL(k_colsum_part, dim3(static_cast<unsigned>(cb), static_cast<unsigned>(nc)), dim3(256), 0, s, X, M,
                     N, R, part);
  const int64_t CBf = N / 4 < 64 ? N / 4 : 64;
  hipLaunchKernelGGL(k_colsum_final, dim3(static_cast<unsigned>((N / 4 + CBf - 1) / CBf)), dim3(256), 0, s, part,
                     static_cast<int>(nc), N, out, nullptr, N / 4, 0, 64);
  return ghm_launch_status();
}

namespace {
// partial row: C*N weighted sums, then the C class totals padded to a float4
int64_t wcolsum_ldp(int64_t N, int C) { return static_cast<int64_t>(C) * N + 4 * ((C + 3) / 4); }

void wcolsum_plan(int64_t M, int64_t& nchunk, int64_t& R) {
  const int64_t cap = (M + 7) / 8;
  nchunk = cap < 512 ? cap : 512;
  if (nchunk < 1) nchunk = 1;
  R = (M + nchunk - 1) / nchunk;
  nchunk = (M + R - 1) / R;
}
}  // namespace

extern "C" int64_t ghm_wcolsum_part_elems(int64_t M, int64_t N, int C) {
  int64_t nc, R;
  wcolsum_plan(M, nc, R);
  return nc * wcolsum_ldp(N, C);
}

extern "C" int ghm_wcolsum(const float* W, const uint8_t* tok, int C, const float* X, int64_t rps, int64_t seq_rows,
                           int64_t off, int64_t M, int64_t N, float* out, float* wsum, float* part, void* stream) {
  GHM_CHECK((W || tok) && !(W && tok) && X && out && part, "exactly one of W / tok; X, out, part");
  GHM_CHECK(!(tok && wsum), "class totals (wsum) only with dense weights");
  GHM_CHECK(M < (int64_t(1) << 31) && ((M + rps - 1) / rps) * seq_rows < (int64_t(1) << 31), "rows < 2^31");
  GHM_CHECK(C >= 1 && C <= 64 && M >= 1 && rps >= 1 && seq_rows >= rps && off >= 0 && off + rps <= seq_rows,
            "shape (1 <= C <= 64, row map inside each sequence)");
  GHM_CHECK(N >= 4 && N <= 1024 && N % 4 == 0 && 256 % (N / 4) == 0, "N / 4 must divide 256");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(part)) &
             15) == 0, "16-byte aligned X, out, part");
  int64_t nc, R;
  wcolsum_plan(M, nc, R);
  const int64_t ldp = wcolsum_ldp(N, C);
  hipStream_t s = ghm_stream(stream);
  const dim3 grid(static_cast<unsigned>(nc), static_cast<unsigned>((C + 15) / 16));
  if (tok)
    hipLaunchKernelGGL(k_wcolsum_part<true>, grid, dim3(256), 0, s, W, tok, C, X, rps, seq_rows, off, M, N, R, ldp,
                       part);
  else
    hipLaunchKernelGGL(k_wcolsum_part<false>, grid, dim3(256), 0, s, W, tok, C, X, rps, seq_rows, off, M, N, R, ldp,
                       part);
  // 16 float4 columns x 16 chunk groups per workgroup: the partial rows are short
  // and many (64 columns per workgroup left ~6 workgroups on a latency chain)
  const int64_t L4 = ldp / 4;
  const int64_t CBf = L4 < 16 ? L4 : 16;
  hipLaunchKernelGGL(k_colsum_final, dim3(static_cast<unsigned>((L4 + CBf - 1) / CBf)), dim3(256), 0, s, part,
                     static_cast<int>(nc), ldp, out, wsum, static_cast<int64_t>(C) * N / 4, C, 16);
  return ghm_launch_status();
}

extern "C" int ghm_rows_linear(const float* X, const float* W, const float* b, float* Y, int64_t M, int D, int C,
                               void* stream) {
  GHM_CHECK(X && W && b && Y && M >= 1 && C >= 1 && C <= 64 && (D == 64 || D == 128 || D == 256) && C * D <= 16384,
            "shape");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W)) & 15) == 0, "16-byte aligned X, W");
  const dim3 grid(static_cast<unsigned>((M + 15) / 16));
  const size_t lds = static_cast<size_t>(C) * D * sizeof(float);
  hipStream_t s = ghm_stream(stream);
  if (D == 64)
    hipLaunchKernelGGL(k_rows_linear<64>, grid, dim3(256), lds, s, X, W, b, Y, M, C);
  else if (D == 128)
    hipLaunchKernelGGL(k_rows_linear<128>, grid, dim3(256), lds, s, X, W, b, Y, M, C);
  else
    hipLaunchKernelGGL(k_rows_linear<256>, grid, dim3(256), lds, s, X, W, b, Y, M, C);
  return ghm_launch_status();
}

extern "C" int ghm_rows_linear_t(const float* dZ, const float* W, float* dX, int64_t M, int D, int C, void* stream) {
  GHM_CHECK(dZ && W && dX && M >= 1 && C >= 1 && C <= 64 && (D == 64 || D == 128 || D == 256) && C * D <= 16384,
            "shape");
  GHM_CHECK(((reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(dX)) & 15) == 0, "16-byte aligned W, dX");
  const int64_t rpb = 256 / (D / 4);
  const dim3 grid(static_cast<unsigned>((M + rpb - 1) / rpb));
  const size_t lds = static_cast<size_t>(C) * D * sizeof(float);
  hipStream_t s = ghm_stream(stream);
  if (D == 64)
    hipLaunchKernelGGL(k_rows_linear_t<64>, grid, dim3(256), lds, s, dZ, W, dX, M, C);
  else if (D == 128)
    hipLaunchKernelGGL(k_rows_linear_t<128>, grid, dim3(256), lds, s, dZ, W, dX, M, C);
  else
    hipLaunchKernelGGL(k_rows_linear_t<256>, grid, dim3(256), lds, s, dZ, W, dX, M, C);
  return ghm_launch_status();
}
