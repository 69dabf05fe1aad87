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


def bp_out_of_image(M, N, K, ldbp, nsplit, TM, BN=GB_N):
    """Pre-split B (k_gemm_x3 V bit 2, ghm_gemm_x3p): per K tile BN / 64 16-byte
    loads per thread and plane at byte offsets ((idx >> 2) ldbp + 8 (idx & 3)) 2
    from the tile's base (n0 ldbp + k0) bf16, records BN ldbp 2 bytes when the tile
    is live; the hi plane is [N][ldbp] bf16 and the lo plane the next one.  Counts
    loads inside the records that leave their own plane (either end)."""
    kps = ((K + nsplit - 1) // nsplit + GB_K - 1) // GB_K * GB_K
    ob = [((idx >> 2) * ldbp + 8 * (idx & 3)) * 2 for idx in range(4 * BN)]
    plane = N * ldbp * 2
    bad = 0
    for z in range(nsplit):
        kb, ke = z * kps, min(z * kps + kps, K)
        for t in range(max(0, -(-(ke - kb) // GB_K)) + 3):
            k0 = kb + t * GB_K
            nrec = BN * ldbp * 2 if k0 < ke else 0
            for n0 in range(0, N, BN):
                base = (n0 * ldbp + k0) * 2
                bad += sum(o < nrec and (base + o < 0 or base + o + 16 > plane) for o in ob)
    return bad


@pytest.mark.parametrize("TM,BN", [(1, 128), (2, 128), (1, 64)])
def test_presplit_b_loads_stay_inside_their_plane(TM, BN):
    """Every ghm_gemm_x3p product of models/vlm.py (D = 128 / 256): forward W
    images (N = 3D / F / D), data-gradient W^T images, split-k data gradients;
    64 x 64 tiles (launch_bp below 768 columns) as well as the 128-column ones."""
    for d in (128, 256):
        F = 4 * d
        for N, K, ns in ((3 * d, d, 1), (F, d, 1), (d, F, 1), (F, d, 1), (d, F, 2), (d, 3 * d, 1), (d, 3 * d, 3)):
            assert bp_out_of_image(405, N, K, K, ns, TM, BN) == 0, (d, N, K, ns)


def split_pack_writes(L, D):
    """models/vlm.py VlmPlan._split_weights' job table against k_split_pack's
    writes: every (hi, lo) element a job writes lies inside its own image of the
    layer's wpack region, and no element is written twice (the three Q / K / V
    jobs tile the fused [3D][D] / [D][3D] images exactly)."""
    F = 4 * D
    sizes = {"qkv": 3 * D * D, "qkvT": 3 * D * D, "w1": F * D, "w1T": F * D, "w2": F * D, "w2T": F * D}
    pitch = {"qkv": D, "qkvT": 3 * D, "w1": D, "w1T": F, "w2": F, "w2T": D}
    off, o = {}, 0
    for l in range(L):
        for k, n in sizes.items():
            off[(l, k)] = o
            o += 2 * n
    total = o
    written = bytearray(total)
    for l in range(L):
        jobs = []
        for i in range(3):
            jobs.append((D, D, off[(l, "qkv")] + i * D * D, D, sizes["qkv"], 0, (l, "qkv")))
            jobs.append((D, D, off[(l, "qkvT")] + i * D, 3 * D, sizes["qkvT"], 1, (l, "qkvT")))
        for (rows, cols), k, kt in (((F, D), "w1", "w1T"), ((D, F), "w2", "w2T")):
            jobs.append((rows, cols, off[(l, k)], cols, sizes[k], 0, (l, k)))
            jobs.append((rows, cols, off[(l, kt)], rows, sizes[kt], 1, (l, kt)))
        for rows, cols, dst, ldd, plane, tr, img in jobs:
            assert ldd == pitch[img[1]]
            lo_img, hi_img = off[img], off[img] + 2 * sizes[img[1]]
            orows, ocols = (cols, rows) if tr else (rows, cols)
            for r in range(orows):
                for c in (0, ocols - 1) if r not in (0, orows - 1) else range(ocols):
                    for e in (dst + r * ldd + c, dst + r * ldd + c + plane):
                        assert lo_img <= e < hi_img, (img, r, c)
            for r in range(orows):
                for c in range(ocols):
                    for e in (dst + r * ldd + c, dst + r * ldd + c + plane):
                        assert not written[e], (img, r, c)
                        written[e] = 1
    return sum(written), total


def test_split_pack_jobs_tile_the_images_exactly():
    for D in (128, 256):
        n, total = split_pack_writes(2, D)
        assert n == total


@pytest.mark.parametrize("Mtok", [405, 2000])
def test_narrow_products_stay_inside_the_operands(Mtok):
    """The generic-width CLIP encoder (models/gemm_encoder.py, n_embd = 64): N = 64 /
    192 products run on 64-column tiles (N % 128 != 0), the rest as the VLM's."""
    d, F = 64, 256
    for K, N in ((d, 3 * d), (d, F), (F, d)):  # forward X W^T
        assert out_of_allocation(0, 1, Mtok, N, K, K, K, 1, Mtok, N, 1, BN=64 if N % 128 else 128) == 0
    for K, N in ((F, d), (3 * d, d), (d, F)):  # data gradients dY W
        assert out_of_allocation(0, 0, Mtok, N, K, K, N, 1, Mtok, K, 1, BN=64 if N % 128 else 128) == 0
    for m, n, ns in ((d, F, 128), (F, d, 64), (3 * d, d, 85)):  # weight gradients over the tokens
        ns = min(ns, max(1, Mtok // 256))
        assert out_of_allocation(1, 0, m, n, Mtok, m, n, ns, Mtok, Mtok, 1, BN=64 if n % 128 else 128) == 0
