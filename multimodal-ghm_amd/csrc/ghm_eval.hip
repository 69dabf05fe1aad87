// Zero-shot-classification evaluation: the all-pairs similarity contraction
// (figures/eval-zsc-risk.py:107-118).
//
// The reference materialises exp(I Tᵀ) for all N x N (image, text) pairs and
// then, per class c and support size n, averages the columns of the first n
// text samples whose first leaf is c:
//     logit[r][c](n) = log( mean_{k < n} exp(<I_r, T_{idx_c[k]}>) ).
// Only 10 x n_max of the N columns are ever read, so this kernel contracts
// exactly those: workgroup = 128 image rows x one class; each wave owns 32
// image rows (the B operand: image row on the lane) and walks the class's
// prototypes 32 at a time as the A operand of v_mfma_f32_32x32x2_f32 (exact
// f32 products, K = the embedding width, zero-padded to even), so the 16
// accumulator registers of a lane are 16 prototypes of its row.  exp and the
// prefix sums at every requested n are fused; nothing N x N reaches HBM.
// Deterministic: fixed per-lane order, then one lane-pair exchange.
#include "ghm_common.h"
#include "ghm_launch.h"

namespace {

constexpr int ZSC_MAX_D = 16;
constexpr int ZSC_MAX_J = 8;

__global__ __launch_bounds__(256) void k_zsc_logits(const float* __restrict__ I, int64_t n_rows,
                                                    const float* __restrict__ Temb, int D,
                                                    const int32_t* __restrict__ idx, int n_proto,
                                                    const int32_t* __restrict__ n_list, int n_j,
                                                    float* __restrict__ logits, int n_class) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
  const int c = blockIdx.y;
  const int64_t row = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * 32 + j;
  const int64_t rc = row < n_rows ? row : n_rows - 1;
  const int ksteps = (D + 1) / 2;
  // B fragments: I[row][2s + h], zero past D
  float b[ZSC_MAX_D / 2];
#pragma unroll
  for (int s = 0; s < ZSC_MAX_D / 2; ++s) {
    const int k = 2 * s + h;
    b[s] = (s < ksteps && k < D) ? I[rc * D + k] : 0.f;
  }
  int nl[ZSC_MAX_J];
  float acc_n[ZSC_MAX_J];
#pragma unroll
  for (int q = 0; q < ZSC_MAX_J; ++q) {
    nl[q] = q < n_j ? n_list[q] : 0;
    acc_n[q] = 0.f;
  }
  const int32_t* ci = idx + static_cast<int64_t>(c) * n_proto;
  for (int p0 = 0; p0 < n_proto; p0 += 32) {
    // A fragments: T[idx_c[p0 + j]][2s + h] (prototype p0 + j on row j of the tile)
    const int p = p0 + j;
    const int64_t t = p < n_proto ? ci[p] : ci[0];
    f32x16 acc = zero16();
#pragma unroll
    for (int s = 0; s < ZSC_MAX_D / 2; ++s) {
      if (s < ksteps) {
        const int k = 2 * s + h;
        const float a = k < D ? Temb[t * D + k] : 0.f;
        acc = mfma32(a, b[s], acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int pr = p0 + acc_row(r, h);  // prototype of register r (column = this lane's row)
      const float e = expf(acc[r]);
#pragma unroll
      for (int q = 0; q < ZSC_MAX_J; ++q) acc_n[q] += pr < nl[q] ? e : 0.f;
    }
  }
#pragma unroll
  for (int q = 0; q < ZSC_MAX_J; ++q) acc_n[q] += xhalf(acc_n[q]);
  if (h == 0 && row < n_rows) {
    for (int q = 0; q < n_j; ++q)
      logits[(static_cast<int64_t>(q) * n_rows + row) * n_class + c] = logf(acc_n[q] / static_cast<float>(nl[q]));
  }
}

}  // namespace

extern "C" int ghm_zsc_logits(const float* i_emb, int64_t n_rows, const float* t_emb, int D,
                              const int32_t* proto_idx, int n_class, int n_proto, const int32_t* n_list, int n_j,
                              float* logits, void* stream) {
  GHM_CHECK(i_emb && t_emb && proto_idx && n_list && logits, "null pointer");
  GHM_CHECK(n_rows >= 1 && D >= 1 && D <= ZSC_MAX_D, "shape (1 <= D <= 16)");
  GHM_CHECK(n_class >= 1 && n_class <= 65535 && n_proto >= 1, "n_class / n_proto");
  GHM_CHECK(n_j >= 1 && n_j <= ZSC_MAX_J, "n_j (1..8 support sizes)");
  const int64_t nblk = (n_rows + 127) / 128;
  GHM_CHECK(nblk <= 0x7fffffff, "too many rows");
  hipLaunchKernelGGL(k_zsc_logits, dim3(static_cast<unsigned>(nblk), static_cast<unsigned>(n_class)), dim3(256), 0,
                     ghm_stream(stream), i_emb, n_rows, t_emb, D, proto_idx, n_proto, n_list, n_j, logits, n_class);
  return ghm_launch_status();
}
