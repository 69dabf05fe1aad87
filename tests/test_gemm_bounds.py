"""Host model of the split-bf16 GEMM's buffer-load staging bounds (csrc/ghm_gemm.hip
k_gemm_x3, V bit 0): for every tile a workgroup loads -- including the prefetched
tiles past the end of its K range -- each 16-byte load whose offset is inside the
descriptor's record count must lie inside the operand's allocation (a load past
the record count reads zeros without touching memory).  Round 5's first version
gave the k-contiguous operands' past-the-end tiles a full record count, so the
last row's prefetch ran past the allocation (an illegal address in
test_gpu_vlm.py at exact-size buffers); this model counts 76,416 such loads for
that version and none for the fix.  Mirrors load()'s BUF branch, voff_kc / voff_oc
and kc_row."""
import pytest

GB_N, GB_K = 128, 32


def kc_row(idx):
    w8, q = idx >> 6, (idx >> 3) & 7
    return 16 * (w8 >> 1) + 4 * (q & 3) + 2 * (q >> 2) + (w8 & 1)


def _offs_kc(rows, ld):
    return [(kc_row(t + 256 * i) * ld + 4 * ((t + 256 * i) & 7)) * 4 for t in range(256) for i in range(rows * 8 // 256)]


def _offs_oc(cols, ld):
    rpt = cols // 32
    kgn = 32 // rpt
    return [((rpt * kg + i) * ld + 4 * c4) * 4 for kg in range(kgn) for c4 in range(256 // kgn) for i in range(rpt)]


def out_of_allocation(ta, tb, M, N, K, lda, ldb, nsplit, a_rows, b_rows, TM, fixed=True, BN=GB_N):
    BM = 64 * TM
    kps = ((K + nsplit - 1) // nsplit + GB_K - 1) // GB_K * GB_K
    oa = _offs_oc(BM, lda) if ta else _offs_kc(BM, lda)
    ob = _offs_kc(BN, ldb) if tb else _offs_oc(BN, ldb)
    bad = 0
    for z in range(nsplit):
        kb, ke = z * kps, min(z * kps + kps, K)
        for t in range(max(0, -(-(ke - kb) // GB_K)) + 3):  # the loop's tiles + prefetch past the end
            k0 = kb + t * GB_K
            krows, live = min(ke - k0, GB_K), (k0 < ke or not fixed)
            for m0 in range(0, M, BM):
                if ta:
                    base, nrec = k0 * lda + m0, max(0, krows) * lda * 4
                else:
                    base, nrec = m0 * lda + k0, min(M - m0, BM) * lda * 4 if live else 0
                bad += sum(o < nrec and base * 4 + o + 16 > a_rows * lda * 4 for o in oa)
            for n0 in range(0, N, BN):
                if tb:
                    base, nrec = n0 * ldb + k0, BN * ldb * 4 if live else 0
                else:
                    base, nrec = k0 * ldb + n0, max(0, krows) * ldb * 4
                bad += sum(o < nrec and base * 4 + o + 16 > b_rows * ldb * 4 for o in ob)
    return bad


@pytest.mark.parametrize("Mtok", [405, 2000])
@pytest.mark.parametrize("TM,BN", [(1, 128), (2, 128), (1, 64)])
def test_buffer_staging_stays_inside_the_operands(Mtok, TM, BN):
    d, F = 256, 1024
    for K, N in ((d, d), (d, 3 * d), (d, F), (F, d)):  # forward X W^T
        assert out_of_allocation(0, 1, Mtok, N, K, K, K, 1, Mtok, N, TM, BN=BN) == 0
    for K, N, ns in ((F, d, 1), (F, d, 3), (3 * d, d, 2), (d, F, 1)):  # data gradients dY W
        assert out_of_allocation(0, 0, Mtok, N, K, K, N, ns, Mtok, K, TM, BN=BN) == 0
    for m, n, ns in ((d, F, 7), (F, d, 16), (3 * d, d, 4)):  # weight gradients over the tokens
        assert out_of_allocation(1, 0, m, n, Mtok, m, n, ns, Mtok, Mtok, TM, BN=BN) == 0


def test_the_model_sees_the_first_versions_overrun():
    assert out_of_allocation(0, 1, 405, 256, 256, 256, 256, 1, 405, 256, 1, fixed=False) > 0
