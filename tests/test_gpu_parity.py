"""Parity of the HIP path (through the C ABI) against the CPU oracle and the reference's golden vectors.

Tolerances (north_star): LBP codes and histogram counts bit-exact; projections
and distances within 1e-4 relative of numpy float64 (projections norm-relative
per row; a distance may also carry an absolute 1e-6*||q|| term, the size of the
fp32 rounding of the features it is computed from); labels identical except
on near-ties, (d2-d1)/d1 <= 1e-4 between distinct gallery rows in the oracle.
"""
import os

import numpy as np
import pytest
import torch

import facerec_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    torch.cuda.set_device(0)
    from opencv_facerecognizer_amd import _lib
    _lib.device()


def _rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def _check_search(metric_name, Q, G, d_got, i_got, k, near_rel=1e-4):
    """Compare device top-k with the float64 oracle on the same (fp32-representable) inputs."""
    Dref = O.pairwise(metric_name, Q, G)
    order = np.argsort(Dref, axis=1, kind="stable")
    n_ties = 0
    for b in range(Q.shape[0]):
        kk = min(k, G.shape[0])
        ref_i = order[b, :kk]
        ref_d = Dref[b, ref_i]
        got_i = i_got[b, :kk]
        got_d = d_got[b, :kk]
        assert np.all(i_got[b, kk:] == -1)
        qn = np.linalg.norm(Q[b])
        tol = 1e-4 * np.abs(ref_d) + 1e-6 * max(qn, 1e-30)
        assert np.all(np.abs(got_d - ref_d) <= tol), (b, got_d, ref_d)
        # every returned row is really at the reported oracle distance
        np.testing.assert_allclose(Dref[b, got_i], got_d, rtol=1e-4, atol=1e-6 * max(qn, 1e-30))
        if not np.array_equal(got_i, ref_i):
            # allowed only where the oracle itself has near-ties at the differing ranks
            for j in np.nonzero(got_i != ref_i)[0]:
                a, c = Dref[b, got_i[j]], Dref[b, ref_i[j]]
                assert abs(a - c) <= near_rel * max(abs(c), 1e-300) + 1e-6 * qn, (b, j, a, c)
                n_ties += 1
    return n_ties


# ---------------------------------------------------------------------------
# search kernel (ofr_knn_f32) — Euclidean / Cosine
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("metric", ["EuclideanDistance", "CosineDistance"])
@pytest.mark.parametrize("B,N,d,k", [(1, 31, 3, 1), (7, 1000, 99, 5), (300, 5000, 3, 1), (257, 3000, 300, 16),
                                     (600, 20000, 64, 3), (5, 4, 10, 8)])
def test_knn_vs_oracle(metric, B, N, d, k):
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    r = _rng(B * 7 + N + d)
    G = r.normal(100, 40, (N, d)).astype(np.float32).astype(np.float64)
    Q = r.normal(100, 40, (B, d)).astype(np.float32).astype(np.float64)
    if N > 10:
        Q[0] = G[N // 2]           # exact match -> distance 0
        G[N - 1] = G[3]            # duplicate rows -> lowest index first
    mid = _lib.METRIC_EUCLIDEAN if metric == "EuclideanDistance" else _lib.METRIC_COSINE
    g = FloatGallery(G, mid)
    dd, ii = g.search(g.query_rows(Q), k)
    ties = _check_search(metric, Q, G, dd.cpu().numpy(), ii.cpu().numpy(), k)
    assert ties <= max(1, B // 100)


@pytest.mark.parametrize("B,N,d,k", [(1, 3000, 99, 1), (5, 257, 64, 8), (32, 20000, 200, 3), (33, 300, 3, 1),
                                     (300, 5000, 99, 5), (257, 3000, 300, 16), (600, 20000, 64, 3),
                                     (1000, 70000, 130, 1), (64, 10, 16, 3), (48, 17, 40, 5)])
@pytest.mark.parametrize("mode", ["auto", "q8", "q8x2", "fp32"])
def test_knn_euclidean_paths_vs_oracle(monkeypatch, mode, B, N, d, k):
    """Euclidean searches with k <= 8 take the certified tiers (ofr_knn_f6 -- the streaming kernel for
    B <= 32, the tile kernel above -- then ofr_knn_q8 with 1 and 2 slices) unless OFR_SEARCH=fp32;
    OFR_SEARCH=q8 / q8x2 start at the int8 tiers."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", mode)
    r = _rng(B * 11 + N + d)
    protos = r.normal(0, 30, (max(N // 10, 1), d))
    G = (protos[np.arange(N) % len(protos)] + r.normal(0, 5, (N, d))).astype(np.float32).astype(np.float64)
    Q = (protos[r.integers(0, len(protos), B)] + r.normal(0, 5, (B, d))).astype(np.float32).astype(np.float64)
    Q[0] = G[N // 2]
    G[N - 1] = G[3]
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    q8 = mode != "fp32" and k <= 8
    assert g.use_q8(B, k) == q8
    dd, ii = g.search(g.query_rows(Q), k)
    ties = _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), k)
    assert ties <= max(1, B // 100)
    if q8:
        assert g.last_fallbacks[0] <= B // 10     # well-separated data: nearly every query certifies


def test_knn_q8_certificate_forces_fallback(monkeypatch):
    """A gallery on a sphere around the queries: more than 16 rows lie within the quantized passes'
    error bounds of the k-th distance, so no query can be certified by any tier (fp6, int8 x1,
    int8 x2); all of them must be re-run on the fp32 path and still match the oracle (up to its
    own near-ties)."""
    from opencv_facerecognizer_amd._device import FloatGallery
    from opencv_facerecognizer_amd import _lib
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(99)
    c = r.normal(0, 50, 64)
    U = r.normal(0, 1, (2000, 64))
    G = (c + 100.0 * U / np.linalg.norm(U, axis=1, keepdims=True)).astype(np.float32).astype(np.float64)
    Q = (c + r.normal(0, 1e-6, (100, 64))).astype(np.float32).astype(np.float64)   # every row ~equidistant
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    dd, ii = g.search(g.query_rows(Q), 3)
    # every quantized tier that ran left queries uncertified (the fp32 pass resolved them)
    assert g.last_fallbacks[0] == 100 and min(g.last_fallbacks) > 0, g.last_fallbacks
    _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), 3)


def test_fallback_routing_is_only_a_choice(monkeypatch):
    """_route may send an fp6 failure past the f6x2 tier; with the skip disabled (every failure runs
    every tier) the results are identical, on crowded data where both routes are taken."""
    from opencv_facerecognizer_amd._device import FloatGallery
    from opencv_facerecognizer_amd import _lib
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(98)
    d, N, B = 96, 30000, 300
    protos = r.normal(0, 6, (300, d))
    G = (protos[np.arange(N) % 300] + r.normal(0, 4, (N, d))).astype(np.float32).astype(np.float64)
    Q = (protos[r.integers(0, 300, B)] + r.normal(0, 4, (B, d))).astype(np.float32).astype(np.float64)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    dd, ii = g.search(g.query_rows(Q), 1)
    routed = (g.last_fallbacks, dict(g.last_skipped))
    monkeypatch.setattr(FloatGallery, "ROUTE_SLACK", float("inf"))   # never skip
    d2, i2 = g.search(g.query_rows(Q), 1)
    assert g.last_skipped.get("f6x2", 0) == 0
    assert torch.equal(ii, i2) and torch.equal(dd, d2), routed
    _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), 1)


def test_knn_f6_sieve_overflow_falls_back(monkeypatch):
    """The fp6 sieve (B > 32) keeps the rows at or below a sampled threshold in a per-query bucket of
    32768 rows.  40,000 exact copies of one row all tie with the threshold, every bucket overflows:
    each query must come back uncertified from the fp6 tier and be resolved by the next tiers, with
    ties to the lowest index (the oracle's order)."""
    from opencv_facerecognizer_amd._device import FloatGallery
    from opencv_facerecognizer_amd import _lib
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(1234)
    d = 96
    x = r.normal(0, 20, d)
    G = np.concatenate([np.tile(x, (40000, 1)), r.normal(0, 20, (2000, d))]).astype(np.float32).astype(np.float64)
    Q = (x + r.normal(0, 0.5, (40, d))).astype(np.float32).astype(np.float64)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    dd, ii = g.search(g.query_rows(Q), 3)
    assert g.last_fallbacks[0] == 40
    assert (ii.cpu().numpy() == np.array([0, 1, 2])).all()
    # the kept-row counts of the fp6 pass: the duplicates overflowed every bucket; the count
    # saturates just past the cap (32768) however many tiles overflow, so it can never wrap
    qq = g.quantize_queries(g.query_rows(Q), tier="f6")
    g.search_q8_phase(1, g.query_rows(Q), qq, 3)
    cnt = g.sieve_counts(40).cpu().numpy()
    assert (cnt > 32768).all() and (cnt <= 32769 + len(G)).all(), cnt
    _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), 3)


def _e2m3_values():
    return np.array([m / 8 for m in range(8)] + [(1 + m / 8) * 2.0 ** (e - 1) for e in (1, 2, 3) for m in range(8)])


def _decode_f6_tiles(tiles, R, d):
    """Host decode of the f6 tiled layout (csrc/ofr_f6_tile.h) -> e2m3 values [R][nst*128]."""
    nst = -(-d // 128)
    P = -(-R // 256)
    t = tiles.reshape(P, nst, 4, 6144)                       # (panel, stage, 2j+h, sub-block)
    p0 = t[..., :4096].reshape(P, nst, 4, 256, 16)
    p1 = t[..., 4096:].reshape(P, nst, 4, 256, 8)
    # part1 row slots are swizzled: row r of sub-block 2j+h sits at slot r ^ 16h (ofr_f6_tile.h p1_slot)
    p1 = np.stack([p1[:, :, jh, np.arange(256) ^ (16 * (jh & 1))] for jh in range(4)], axis=2)
    grp = np.concatenate([p0, p1], axis=-1)                  # 24 bytes = 32 x 6 bits per row and group
    bits = np.unpackbits(grp, axis=-1, bitorder="little").reshape(P, nst, 4, 256, 32, 6)
    code = (bits * (1 << np.arange(6))).sum(-1)
    mag = _e2m3_values()[code & 31]
    val = np.where(code & 32, -mag, mag)                     # (P, nst, 4, 256, 32)
    val = val.transpose(0, 3, 1, 2, 4).reshape(P * 256, nst * 128)
    return val[:R]


def _block_scales_host(d, seed, spread):
    """Random column-block scales (E8M0 bytes, 4 per 128-feature stage; exponents 0 .. -spread, 127 past d)
    -> (device uint8 tensor or None, per-feature 2^e fp64 [d])."""
    if spread is None:
        return None, np.ones(d)
    nb, npad = -(-d // 32), 4 * -(-d // 128)
    e = -_rng(seed).integers(0, spread + 1, nb)
    e[0] = 0
    b = np.full(npad, 127, np.uint8)
    b[:nb] = 127 + e
    return torch.from_numpy(b).cuda(), np.repeat(2.0 ** e, 32)[:d]


@pytest.mark.parametrize("spread", [None, 8])
@pytest.mark.parametrize("R,d", [(1, 3), (300, 99), (513, 260), (256, 128), (40, 1000)])
def test_f6_quantize_rows_vs_host(R, d, spread):
    """ofr_f6_quantize_rows: every value is the nearest e2m3 value of x / (s 2^e) (ties either way), e the
    feature's column-block exponent (spread None: unit scales), s = max|x / 2^e| / 7.5 rounded up, padding is
    zero, and the stats are ||x~|| and ||x - x~|| of x~ = s 2^e v."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    r = _rng(R * 7 + d)
    X = r.normal(0, 3, (R, d)).astype(np.float32)
    X[0, : d // 2] = 0
    if R > 2:
        X[2] = 0                                                          # all-zero row
        X[1, 0] = 1e6                                                     # one huge feature
    bs, f = _block_scales_host(d, R + d, spread)
    X = (X * f).astype(np.float32)          # columns spread like the scales (a trained W's feature profile)
    ldx = d + 5
    Xd = torch.zeros((R, ldx), dtype=torch.float32, device="cuda")
    Xd[:, :d] = torch.from_numpy(X).cuda()
    nbytes = _lib.load().ofr_f6_tiles_bytes(R, d)
    T = torch.full((nbytes,), 0xAB, dtype=torch.uint8, device="cuda")
    sc = torch.empty(R, dtype=torch.float32, device="cuda")
    st = torch.empty((R, 3), dtype=torch.float64, device="cuda")
    call("ofr_f6_quantize_rows", stream(), ptr(Xd), R, d, ldx, ptr(T), nbytes, ptr(sc), ptr(st), None, None, ptr(bs))
    torch.cuda.synchronize()
    Vall = _decode_f6_tiles(T.cpu().numpy(), -(-R // 256) * 256, d)
    assert np.all(Vall[R:] == 0)                                          # tail rows of the last panel
    V = Vall[:R]
    s = sc.cpu().numpy().astype(np.float64)
    assert np.all(V[:, d:] == 0)
    Xn = X.astype(np.float64) / f                                         # exact power-of-two rescaling
    mx = np.abs(Xn).max(1)
    assert np.all(np.where(mx > 0, mx / s, 0) <= 7.5)
    assert np.all(np.where(mx > 0, s <= np.nextafter(np.float32(mx / 7.5), np.float32(np.inf)) * (1 + 1e-6), s == 1))
    grid = _e2m3_values()
    r_ = np.abs(Xn / s[:, None])
    err = np.abs(np.abs(V[:, :d]) - r_)
    best = np.abs(r_[..., None] - grid).min(-1)
    assert np.all(err <= best + 1e-12)                                    # nearest representable value
    assert np.all((np.sign(V[:, :d]) == np.sign(X)) | (V[:, :d] == 0))
    Xt = s[:, None] * f * V[:, :d]
    a = np.linalg.norm(Xt, axis=1)
    e = np.linalg.norm(X.astype(np.float64) - Xt, axis=1)
    got = st.cpu().numpy()
    np.testing.assert_allclose(got[:, 0], a, rtol=1e-11, atol=0)
    np.testing.assert_allclose(got[:, 1], e, rtol=1e-11, atol=0)
    assert np.all(got[:, 0] >= a) and np.all(got[:, 1] >= e)             # rounded up, never shrinks the bound
    assert np.all(got[:, 2] == 0)


@pytest.mark.parametrize("spread", [None, 8])
@pytest.mark.parametrize("R,d", [(1, 3), (300, 99), (513, 260), (40, 1000)])
def test_f6x2_quantize_rows_vs_host(R, d, spread):
    """ofr_f6x2_quantize_rows: the first slice is byte-identical to ofr_f6_quantize_rows (same scale), the
    second holds the nearest e2m3 value of 2^4 (x / 2^e / s - v1), and the stats are (s(|v1|' + |v2|'/16),
    |x - x~|, s |v2|'/16) of x~ = s 2^e (v1 + v2/16), |v|' = |2^e v| (e: column-block exponents)."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    r = _rng(R * 5 + d)
    X = r.normal(0, 3, (R, d)).astype(np.float32)
    if R > 2:
        X[2] = 0
        X[1, 0] = 1e6
    bs, f = _block_scales_host(d, R * 3 + d, spread)
    X = (X * f).astype(np.float32)          # columns spread like the scales (a trained W's feature profile)
    ldx = d + 3
    Xd = torch.zeros((R, ldx), dtype=torch.float32, device="cuda")
    Xd[:, :d] = torch.from_numpy(X).cuda()
    nbytes = _lib.load().ofr_f6_tiles_bytes(R, d)
    T1 = torch.full((nbytes,), 0xAB, dtype=torch.uint8, device="cuda")
    T2 = torch.full((nbytes,), 0xCD, dtype=torch.uint8, device="cuda")
    T0 = torch.full((nbytes,), 0x11, dtype=torch.uint8, device="cuda")
    sc, sc0 = (torch.empty(R, dtype=torch.float32, device="cuda") for _ in range(2))
    st, st0 = (torch.empty((R, 3), dtype=torch.float64, device="cuda") for _ in range(2))
    call("ofr_f6x2_quantize_rows", stream(), ptr(Xd), R, d, ldx, ptr(T1), ptr(T2), nbytes, ptr(sc), ptr(st), None,
         None, ptr(bs))
    call("ofr_f6_quantize_rows", stream(), ptr(Xd), R, d, ldx, ptr(T0), nbytes, ptr(sc0), ptr(st0), None, None, ptr(bs))
    torch.cuda.synchronize()
    assert torch.equal(T1, T0) and torch.equal(sc, sc0)
    P = -(-R // 256) * 256
    V1 = _decode_f6_tiles(T1.cpu().numpy(), P, d)
    V2 = _decode_f6_tiles(T2.cpu().numpy(), P, d)
    assert np.all(V2[R:] == 0) and np.all(V2[:R, d:] == 0)
    V1, V2 = V1[:R, :d], V2[:R, :d]
    s = sc.cpu().numpy().astype(np.float64)[:, None]
    u = 16.0 * (X.astype(np.float64) / f - s * V1) / s
    assert np.all(np.abs(u) <= 4.0 + 1e-9)
    grid = _e2m3_values()
    best = np.abs(np.abs(u)[..., None] - grid).min(-1)
    assert np.all(np.abs(np.abs(V2) - np.abs(u)) <= best + 1e-9)             # nearest (ties either way)
    assert np.all((np.sign(V2) == np.sign(u)) | (V2 == 0) | (np.abs(u) < 1e-9))
    Xt = s * f * (V1 + V2 / 16.0)
    got = st.cpu().numpy()
    a = s[:, 0] * (np.linalg.norm(f * V1, axis=1) + np.linalg.norm(f * V2, axis=1) / 16.0)
    e = np.linalg.norm(X.astype(np.float64) - Xt, axis=1)
    t = s[:, 0] * np.linalg.norm(f * V2, axis=1) / 16.0
    for j, ref in enumerate((a, e, t)):
        np.testing.assert_allclose(got[:, j], ref, rtol=1e-11, atol=0)
        assert np.all(got[:, j] >= ref)
    assert np.all(got[:, 0] >= np.linalg.norm(Xt, axis=1))
    # the second slice cuts the residual by more than 10x on Gaussian rows
    e1 = st0.cpu().numpy()[:, 1]
    ok = e1 > 0
    assert np.median(got[ok, 1] / e1[ok]) < 0.1


def test_f6_block_scales_from_sums():
    """ofr_f6_block_sumsq + ofr_f6_block_scales: sums of squares per 32-feature block (accumulated over
    calls), bytes 127 + rint(log2(rms_b / max rms)) clamped to [-63, 0], 127 for empty and padding blocks."""
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    d, R = 300, 777
    r = _rng(31)
    sig = np.repeat(2.0 ** -r.uniform(0, 12, -(-d // 32)), 32)[:d]
    sig[64:96] = 0                                                     # an empty block
    X = (r.normal(0, 1, (R, d)) * sig).astype(np.float32)
    ldx = 320
    Xd = torch.zeros((R, ldx), dtype=torch.float32, device="cuda")
    Xd[:, :d] = torch.from_numpy(X).cuda()
    sums = torch.zeros(-(-d // 32), dtype=torch.float64, device="cuda")
    call("ofr_f6_block_sumsq", stream(), ptr(Xd[:500]), 500, d, ldx, ptr(sums))
    call("ofr_f6_block_sumsq", stream(), ptr(Xd[500:]), R - 500, d, ldx, ptr(sums))
    bs = torch.full((4 * -(-d // 128),), 0, dtype=torch.uint8, device="cuda")
    call("ofr_f6_block_scales", stream(), ptr(sums), d, ptr(bs))
    torch.cuda.synchronize()
    X64 = X.astype(np.float64)
    ref = np.array([(X64[:, b * 32:(b + 1) * 32] ** 2).sum() for b in range(-(-d // 32))])
    np.testing.assert_allclose(sums.cpu().numpy(), ref, rtol=1e-12)
    e = np.where(ref > 0, np.clip(np.rint(0.5 * np.log2(np.where(ref > 0, ref, 1) / ref.max())), -63, 0), 0)
    want = np.full(bs.numel(), 127)
    want[:len(e)] = 127 + e
    assert np.array_equal(bs.cpu().numpy(), want)


@pytest.mark.parametrize("k", [1, 4])
def test_knn_f6x2_certifies_crowded_clusters(monkeypatch, k):
    """Clusters of 40 rows (sigma 0.5 around unit-variance centres, d = 128): the 16 candidates all lie
    in the query's cluster, within a fraction of the fp6 tier's bound of each other, so the fp6 tier
    certifies none; the two-slice tier (residual ~1/30 of fp6's) must certify them, with the oracle's
    neighbours.  The merge's deep continuation (round 6) would certify most of them at the fp6 tier
    already (test_deep_merge_certifies_crowded_clusters): off here, so the tier chain runs."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    monkeypatch.setenv("OFR_MERGE_DEEP", "0")
    r = _rng(3)
    d, K, per, B = 128, 200, 40, 300
    mu = r.normal(0, 1, (K, d))
    G = (mu[np.arange(K * per) % K] + r.normal(0, 0.5, (K * per, d))).astype(np.float32).astype(np.float64)
    Q = (mu[r.integers(0, K, B)] + r.normal(0, 0.5, (B, d))).astype(np.float32).astype(np.float64)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    dd, ii = g.search(g.query_rows(Q), k)
    fb = g.last_fallbacks
    assert fb[0] >= 0.9 * B and len(fb) >= 2 and fb[1] <= 0.02 * B, fb
    assert g.last_skipped.get("f6x2", 0) == 0
    _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), k)


@pytest.mark.parametrize("k", [1, 4])
def test_deep_merge_certifies_crowded_clusters(monkeypatch, k):
    """The merge's deep continuation (round 6, merge_kernel MergeArgs::deep): on the crowded clusters
    above, where the best 16 candidates never certify, the fp6 tier re-ranks each open query's bucket 16
    candidates at a time until its k-th exact distance clears the bound of every row it has not re-ranked.
    Most queries then certify at the first tier (k = 4 leaves 35 of 300 open on one box), and every answer
    equals the tier chain's (deep off) and the oracle's."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(3)
    d, K, per, B = 128, 200, 40, 300
    mu = r.normal(0, 1, (K, d))
    G = (mu[np.arange(K * per) % K] + r.normal(0, 0.5, (K * per, d))).astype(np.float32).astype(np.float64)
    Q = (mu[r.integers(0, K, B)] + r.normal(0, 0.5, (B, d))).astype(np.float32).astype(np.float64)
    res = {}
    for deep in ("1", "0"):   # "1": the default round cap (OFR_MERGE_DEEP unset)
        if deep == "1":
            monkeypatch.delenv("OFR_MERGE_DEEP", raising=False)
        else:
            monkeypatch.setenv("OFR_MERGE_DEEP", deep)
        g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
        dd, ii = g.search(g.query_rows(Q), k)
        res[deep] = (dd.cpu().numpy(), ii.cpu().numpy(), tuple(g.last_fallbacks))
    assert res["0"][2][0] >= 0.9 * B, res["0"][2]                       # without: the fp6 tier certifies few
    assert res["1"][2][0] <= 0.2 * B, res["1"][2]                       # with: most at the fp6 tier
    # the same rows; distances equal up to the fp64 summation order of the exact pass that ended each query
    # (the chain sends its last few queries to the fp32 pass, whose sum runs in another order)
    assert np.array_equal(res["1"][1], res["0"][1])
    np.testing.assert_allclose(res["1"][0], res["0"][0], rtol=1e-12, atol=0)
    _check_search("EuclideanDistance", Q, G, res["1"][0], res["1"][1], k)


@pytest.mark.parametrize("k", [1, 4])
def test_resieve_certifies_open_queries(monkeypatch, k):
    """The fp6 tier's second sieve pass (round 6, FloatGallery._resieve + ofr_knn_f6_set_thresholds): for the
    queries the deep merge leaves open (their buckets hold too few rows below the sample's threshold), a
    sieve pass keeping every row whose coarse score could beat the k-th exact distance, then the deep merge
    again.  On the crowded clusters: no more open queries than without it (usually none), the answers of the
    tier chain and of the oracle."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    monkeypatch.delenv("OFR_MERGE_DEEP", raising=False)
    r = _rng(3)
    d, K, per, B = 128, 200, 40, 300
    mu = r.normal(0, 1, (K, d))
    G = (mu[np.arange(K * per) % K] + r.normal(0, 0.5, (K * per, d))).astype(np.float32).astype(np.float64)
    Q = (mu[r.integers(0, K, B)] + r.normal(0, 0.5, (B, d))).astype(np.float32).astype(np.float64)
    res = {}
    for rs in ("1", "0"):
        monkeypatch.setenv("OFR_RESIEVE", rs)
        g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
        dd, ii = g.search(g.query_rows(Q), k)
        res[rs] = (dd.cpu().numpy(), ii.cpu().numpy(), tuple(g.last_fallbacks))
    print("open after fp6: resieve", res["1"][2], "without", res["0"][2])
    assert res["1"][2][0] <= res["0"][2][0], (res["1"][2], res["0"][2])
    assert np.array_equal(res["1"][1], res["0"][1])
    np.testing.assert_allclose(res["1"][0], res["0"][0], rtol=1e-12, atol=0)
    _check_search("EuclideanDistance", Q, G, res["1"][0], res["1"][1], k)


def test_resieve_small_open_set_padding(monkeypatch):
    """The second sieve pass on an open set smaller than the sieve's 33-query minimum (FloatGallery._resieve
    pads it with repeats of its first query): 48 queries on the crowded clusters, the deep merge off so that
    the fp6 tier leaves most of them open, then _resieve on the first 5 open rows only -- each certified
    answer equals the oracle's, and the padded rows change nothing outside those 5."""
    import torch
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery, open_rows
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(7)
    d, K, per, B, k = 128, 200, 40, 48, 1
    mu = r.normal(0, 1, (K, d))
    G = (mu[np.arange(K * per) % K] + r.normal(0, 0.5, (K * per, d))).astype(np.float32).astype(np.float64)
    Q = (mu[r.integers(0, K, B)] + r.normal(0, 0.5, (B, d))).astype(np.float32).astype(np.float64)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    Qd = g.query_rows(Q)
    monkeypatch.setenv("OFR_MERGE_DEEP", "0")
    qq = g.quantize_queries(Qd, tier="f6")
    out = g.search_q8_phase(3, Qd, qq, k)
    torch.cuda.synchronize()
    bad = open_rows(qq["cert"])
    assert int(bad.numel()) >= 5, int(bad.numel())
    rows = bad[:5]
    before_i = out[1].clone()
    monkeypatch.delenv("OFR_MERGE_DEEP", raising=False)
    still = g._resieve(Qd, rows, k, out, 0, qq)
    torch.cuda.synchronize()
    done = sorted(set(rows.cpu().tolist()) - set(still.cpu().tolist()))
    assert len(done) >= 4, (rows.cpu().tolist(), still.cpu().tolist())
    other = sorted(set(range(B)) - set(rows.cpu().tolist()))
    assert torch.equal(out[1][other], before_i[other])
    dd, ii = out[0].cpu().numpy()[done], out[1].cpu().numpy()[done]
    _check_search("EuclideanDistance", Q[done], G, dd, ii, k)


def test_knn_f6_tier_certifies_separated_data(monkeypatch):
    """f6 tier on well-separated identities (integer prototypes, +-1 noise, 10 rows per identity so
    that the 16 candidates reach past the query's own identity): the fp6 tier alone must certify
    every query and return the oracle's neighbours."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(5)
    N, B, d = 5000, 300, 200
    protos = r.integers(-7, 8, (N // 10, d)).astype(np.float64)
    G = protos[np.arange(N) % (N // 10)] + r.integers(-1, 2, (N, d))
    Q = protos[r.integers(0, N // 10, B)] + r.integers(-1, 2, (B, d))
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    dd, ii = g.search(g.query_rows(Q), 4)
    assert g.last_fallbacks[0] == 0
    _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), 4)


def test_knn_exact_duplicates_tie_to_lowest_index():
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    r = _rng(5)
    base = r.normal(0, 1, (40, 16)).astype(np.float32)
    G = np.concatenate([base, base, base]).astype(np.float64)     # every row appears 3 times
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    dd, ii = g.search(g.query_rows(base.astype(np.float64)), 3)
    ii = ii.cpu().numpy()
    assert np.array_equal(ii, np.stack([np.arange(40), np.arange(40) + 40, np.arange(40) + 80], 1))
    assert np.all(dd.cpu().numpy() == 0)


@pytest.mark.parametrize("mode", ["auto", "fp32"])
def test_gallery_append_in_place_vs_oracle(monkeypatch, mode):
    """FloatGallery.append (NearestNeighbor.update without a re-upload): rows appended in chunks that
    cross 256-row panels, with the fp6 / int8 tiers already built (extended in place) and across a
    storage growth (tiers dropped, rebuilt); every search matches the oracle on the full set."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", mode)
    r = _rng(77)
    d = 130
    protos = r.normal(0, 30, (900, d))
    G = (protos[np.arange(9000) % 900] + r.normal(0, 5, (9000, d))).astype(np.float32).astype(np.float64)
    Q = (protos[r.integers(0, 900, 300)] + r.normal(0, 5, (300, d))).astype(np.float32).astype(np.float64)
    g = FloatGallery(G[:1000], _lib.METRIC_EUCLIDEAN)
    n = 1000
    for step, m in enumerate([1, 255, 200, 2444, 5000]):   # steps 1-2 in place (capacity 1500), then growth
        if step == 1:
            g.search(g.query_rows(Q[:64]), 1)       # build the first tier before the next appends
            if mode == "auto":
                g._tier_gallery(1)                  # and the int8 tier
                g._tier_gallery("f6x2")             # and the two-slice fp6 tier
        g.append(G[n:n + m])
        n += m
        assert g.N == n and g.G.shape[0] == n
        for B, k in [(300, 1), (5, 3)]:
            dd, ii = g.search(g.query_rows(Q[:B]), k)
            _check_search("EuclideanDistance", Q[:B], G[:n], dd.cpu().numpy(), ii.cpu().numpy(), k)
        if mode == "auto":
            assert g.last_fallbacks[0] <= 30
        if mode == "auto" and g.q8 and "f6x2" in g.q8:   # extended in place == built from scratch
            fresh = FloatGallery.from_device_rows(g.G.clone(), d, _lib.METRIC_EUCLIDEAN, shift64=g.shift64)
            a_, b_ = g.q8["f6x2"], fresh._tier_gallery("f6x2")
            nb = _lib.load().ofr_f6_tiles_bytes(n, d)
            assert torch.equal(a_["Gs"][:nb], b_["Gs"][:nb]) and torch.equal(a_["Gs2"][:nb], b_["Gs2"][:nb])
            assert torch.equal(a_["stats"][:n], b_["stats"][:n]) and torch.equal(a_["gmax"], b_["gmax"])


def test_nearest_neighbor_update_extends_device_gallery():
    """NearestNeighbor.update (classifier.py:65-70) appends to the cached device gallery instead of
    rebuilding it; predictions equal the oracle's on the grown set; a new X list rebuilds."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    r = _rng(78)
    d = 40
    G = r.normal(0, 10, (700, d)).astype(np.float32).astype(np.float64)
    y = np.arange(700) % 70
    nn = NearestNeighbor(EuclideanDistance(), k=1)
    nn.compute([np.asmatrix(x.reshape(-1, 1)) for x in G[:500]], y[:500])
    Q = (G[r.integers(0, 700, 50)] + r.normal(0, 0.1, (50, d))).astype(np.float32).astype(np.float64)
    nn.predict_batch(list(Q))
    g0 = nn._gallery()
    for i in range(500, 700):
        nn.update(np.asmatrix(G[i].reshape(-1, 1)), y[i])
        if i % 50 == 0:
            nn.predict(Q[0])
    assert nn._gallery() is g0 and g0.N == 700
    dd, ii = nn.search(list(Q))
    _check_search("EuclideanDistance", Q, G, dd, ii, 1)
    labels = [p[0] for p in nn.predict_batch(list(Q))]
    assert labels == [int(y[i]) for i in ii[:, 0]]
    nn.compute(list(G[:10].reshape(10, d, 1)), y[:10])
    assert nn._gallery() is not g0 and nn._gallery().N == 10


def test_chi2_gallery_append_vs_oracle():
    from opencv_facerecognizer_amd._device import Chi2Gallery
    r = _rng(79)
    G = (r.random((700, 200)) ** 3).astype(np.float32).astype(np.float64)
    Q = (r.random((20, 200)) ** 3).astype(np.float32).astype(np.float64)
    g = Chi2Gallery(G[:300])
    g.append(G[300:301])
    g.append(G[301:700])
    assert g.N == 700
    dd, ii = g.search(g.query_rows(Q), 3)
    _check_search("ChiSquareDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), 3)


@pytest.mark.parametrize("B,N,d,k", [(300, 20000, 64, 1), (40, 9000, 130, 5), (5, 3000, 99, 3)])
def test_knn_cosine_certified_vs_oracle(monkeypatch, B, N, d, k):
    """CosineDistance with k <= 8 runs the certified Euclidean tiers on the unit rows (the Cosine
    ranking) and evaluates distance.py:77 in fp64 for the result; matches the oracle and the fp32
    path, including after an append (the unit-row twin grows with the gallery)."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(B + N + d)
    protos = r.normal(0, 1, (max(N // 10, 1), d))
    G = (protos[np.arange(N) % len(protos)] * r.uniform(0.5, 3, (N, 1)) + r.normal(0, 0.15, (N, d)))
    G = G.astype(np.float32).astype(np.float64)
    Q = (protos[r.integers(0, len(protos), B)] * 2 + r.normal(0, 0.15, (B, d))).astype(np.float32).astype(np.float64)
    g = FloatGallery(G[:N - 500], _lib.METRIC_COSINE)
    assert g.use_cos_cert(B, k)
    dd, ii = g.search(g.query_rows(Q), k)
    _check_search("CosineDistance", Q, G[:N - 500], dd.cpu().numpy(), ii.cpu().numpy(), k)
    assert g.last_fallbacks[0] <= max(1, B // 10)
    g.append(G[N - 500:])
    dd, ii = g.search(g.query_rows(Q), k)
    _check_search("CosineDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), k)
    monkeypatch.setenv("OFR_SEARCH", "fp32")
    d2, i2 = g.search(g.query_rows(Q), k)
    np.testing.assert_allclose(d2.cpu().numpy(), dd.cpu().numpy(), rtol=0, atol=1e-12)
    # a zero row makes the Cosine distance NaN: such galleries stay on the fp32 path
    Z = G[:100].copy()
    Z[7] = 0
    assert not FloatGallery(Z, _lib.METRIC_COSINE).use_cos_cert(40, 1)


def test_knn_golden_reference_predictions(golden):
    """NearestNeighbor.predict vs the reference's own outputs (tests/golden/dist_golden.npz)."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import ChiSquareDistance, CosineDistance, EuclideanDistance
    d = golden("dist_golden.npz")
    mets = {"EuclideanDistance": EuclideanDistance, "CosineDistance": CosineDistance,
            "ChiSquareDistance": ChiSquareDistance}
    for s in ("d3", "d99", "hist"):
        for mname, cls in mets.items():
            if f"{s}_{mname}_D" not in d.files:
                continue
            for k in (1, 3, 5):
                c = NearestNeighbor(dist_metric=cls(), k=k)
                c.compute([g.reshape(-1, 1) for g in d[s + "_G"]], d[s + "_y"])
                preds = c.predict_batch([q.reshape(-1, 1) for q in d[s + "_Q"]])
                for qi, p in enumerate(preds):
                    ref_l = d[f"{s}_{mname}_k{k}_labels"][qi]
                    ref_d = d[f"{s}_{mname}_k{k}_dists"][qi]
                    qn = np.linalg.norm(d[s + "_Q"][qi])
                    np.testing.assert_allclose(p[1]["distances"], ref_d, rtol=1e-4, atol=1e-6 * qn)
                    if not np.array_equal(p[1]["labels"], ref_l):
                        # exact duplicate gallery rows: the reference's quicksort order is unspecified
                        assert np.allclose(np.sort(p[1]["distances"]), np.sort(ref_d), rtol=1e-6)
                    assert p[0] == d[f"{s}_{mname}_k{k}_label"][qi] or len(set(ref_d)) < len(ref_d)
    # the single-pair metric call (distance.py:57-116) runs the same kernels
    for mname, cls in mets.items():
        s = "hist" if mname == "ChiSquareDistance" else "d99"
        D = d[f"{s}_{mname}_D"]
        assert cls()(d[s + "_G"][3], d[s + "_Q"][1]) == pytest.approx(D[1, 3], rel=1e-4, abs=1e-9)


# ---------------------------------------------------------------------------
# projection kernel (ofr_project_u8 / _f32)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("B,D,d", [(1, 4900, 3), (31, 4900, 3), (300, 10000, 99), (513, 777, 260), (5, 100, 70)])
def test_projection_vs_oracle(B, D, d):
    """ofr_project_u8_exact: exact int8-slice MFMA projection vs numpy float64 (feature.py:241-242)."""
    from opencv_facerecognizer_amd._device import Projection, f64_dev, u8_rows
    r = _rng(B + D + d)
    W = r.normal(0, 1.0 / np.sqrt(D), (D, d))
    X = r.integers(0, 256, (B, D), dtype=np.uint8)
    X[0] = 255
    P = Projection(W)
    ref = X.astype(np.float64) @ W
    Y64 = P.project(u8_rows(X), f64=True).cpu().numpy()
    # 4 int8 slices represent W to 2^-28 of each column maximum: ~1e-8, far below the 1e-4 bound
    err = np.abs(Y64 - ref).max(axis=1) / np.linalg.norm(ref, axis=1)
    assert err.max() < 1e-7, err.max()
    Y = P.project(u8_rows(X)).cpu().numpy()
    assert Y.shape[1] == max(32, -(-d // 32) * 32) and np.all(Y[:, d:] == 0)
    np.testing.assert_array_equal(Y[:, :d], Y64.astype(np.float32))   # rounded once from the exact value
    # with a shift, subtracted in fp64 before the rounding (PCA.project form, feature.py:114-116)
    mu = r.normal(128, 5, D)
    c = mu @ W
    Y2 = P.project(u8_rows(X), shift64=f64_dev(c), f64=True).cpu().numpy()
    ref2 = (X - mu) @ W
    err2 = np.abs(Y2 - ref2).max(axis=1) / np.linalg.norm(ref2, axis=1)
    assert err2.max() < 1e-7, err2.max()


@pytest.mark.parametrize("D,d", [(4900, 3), (10000, 130), (777, 45)])
def test_projection_small_batch_gemv_identical(D, d):
    """B <= 4 runs the split-K GEMV (project_gemv_kernel): results bit-identical to the same faces
    projected in a batch on the MFMA tile engine (same exact integers, same fp64 combination)."""
    from opencv_facerecognizer_amd._device import Projection, f64_dev, u8_rows
    r = _rng(D + d)
    W = r.normal(0, 1.0 / np.sqrt(D), (D, d))
    X = r.integers(0, 256, (40, D), dtype=np.uint8)
    P = Projection(W)
    c = f64_dev(r.normal(0, 3, d))
    big = P.project(u8_rows(X), shift64=c, f64=True).cpu().numpy()
    big32 = P.project(u8_rows(X), shift64=c).cpu().numpy()
    for B in (1, 2, 3, 4):
        for s in (0, 7, 36):
            small = P.project(u8_rows(X[s:s + B]), shift64=c, f64=True).cpu().numpy()
            np.testing.assert_array_equal(small, big[s:s + B])
            small32 = P.project(u8_rows(X[s:s + B]), shift64=c).cpu().numpy()
            np.testing.assert_array_equal(small32, big32[s:s + B])


@pytest.mark.parametrize("B,D,d", [(600, 10000, 130), (1000, 777, 450)])
def test_projection_tile_ranges_identical(B, D, d):
    """ofr_project_u8_exact_range: launches over a partition of the grid's tiles (the bench's merge_at
    "tail" runs the last round as its own launch) give ofr_project_u8_exact's output bit for bit; empty and
    out-of-range ranges; B <= 4 (the GEMV) has no tiles."""
    import torch
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import Projection, f64_dev, u8_rows
    r = _rng(B + D + d)
    W = r.normal(0, 1.0 / np.sqrt(D), (D, d))
    X = u8_rows(r.integers(0, 256, (B, D), dtype=np.uint8))
    P = Projection(W)
    c = f64_dev(r.normal(0, 3, d))
    want = P.project(X, shift64=c).cpu().numpy()
    want64 = P.project(X, shift64=c, f64=True).cpu().numpy()
    nt = P.tile_count(B)
    assert nt == -(-(-(-d // 64) * 256) // 384) * -(-B // 256)
    for cuts in ([0, nt], [0, nt // 2, nt], [0, 1, nt - 1, nt], [0, 0, nt]):
        got = torch.full(want.shape, float("nan"), dtype=torch.float32, device=X.device)
        got64 = torch.full((B, d), float("nan"), dtype=torch.float64, device=X.device)
        for t0, t1 in zip(cuts, cuts[1:]):
            P.project(X, shift64=c, out=got, tiles=(t0, t1))
            P.project(X, shift64=c, out=got64, tiles=(t0, t1))
        np.testing.assert_array_equal(got.cpu().numpy()[:, :d], want[:, :d])
        np.testing.assert_array_equal(got64.cpu().numpy(), want64)
    with pytest.raises(_lib.OfrError):
        P.project(X, shift64=c, tiles=(0, nt + 1))
    assert P.tile_count(3) == 0


def test_projection_fp32_weights_exact():
    """fp32 weights within 2^4 of their column maximum are represented exactly: the result equals the
    correctly rounded float64 dot product of the fp32 W."""
    import torch
    from opencv_facerecognizer_amd._device import Projection, u8_rows
    r = _rng(21)
    D, d, B = 2000, 40, 64
    W32 = (r.uniform(0.5, 1.0, (d, D)) * r.choice([-1.0, 1.0], (d, D))).astype(np.float32)
    X = r.integers(0, 256, (B, D), dtype=np.uint8)
    P = Projection(Wt_device=torch.from_numpy(W32).cuda(), D=D)
    Y = P.project(u8_rows(X), f64=True).cpu().numpy()
    ref = X.astype(np.float64) @ W32.T.astype(np.float64)   # exact in float64 here (small integers x 24-bit)
    np.testing.assert_array_equal(Y, ref)


def test_pickled_model_predict_matches_reference(golden):
    """Bundled individuals.pkl: predictions on the 31 bundled faces equal the reference's (golden)."""
    from ocvfacerec.facerec.serialization import load_model
    m = load_model(os.path.join(GOLDEN, "individuals.pkl"))
    f = golden("individuals_faces.npz")
    preds = m.predict_batch(list(f["X"]))
    labels = np.array([p[0] for p in preds])
    dists = np.array([p[1]["distances"][0] for p in preds])
    assert np.array_equal(labels, f["pkl_pred_labels"])
    np.testing.assert_allclose(dists, f["pkl_pred_dist"], rtol=1e-4)
    # single-face API (one face per call, as the recognizer loops use it)
    p0 = m.predict(f["X"][5])
    assert p0[0] == f["pkl_pred_labels"][5] and p0[1]["distances"][0] == pytest.approx(f["pkl_pred_dist"][5], rel=1e-4)
    q = m.feature.extract(f["X"][5])
    assert isinstance(q, np.matrix) and q.shape == (3, 1) and q.dtype == np.float64
    np.testing.assert_allclose(np.asarray(q).ravel(), O.fisherfaces_project(np.asarray(m.feature._eigenvectors),
                                                                            f["X"][5]).A.ravel(), rtol=1e-5)


# ---------------------------------------------------------------------------
# LBP + histograms (bit-exact)
# ---------------------------------------------------------------------------
def test_lbp_codes_bit_exact_vs_reference(golden):
    from ocvfacerec.facerec.lbp import ExtendedLBP
    g = golden("lbp_golden.npz")
    names = sorted(k[4:] for k in g.files if k.startswith("img_"))
    for nm in names:
        im = g["img_" + nm]
        for r, P in ((1, 8), (2, 8), (2, 16), (3, 4)):
            got = ExtendedLBP(radius=r, neighbors=P)(im)
            assert got.dtype == np.uint32
            assert np.array_equal(got, g[f"codes_{nm}_r{r}p{P}"]), (nm, r, P)


def test_spatial_histogram_bit_exact_vs_reference(golden):
    from ocvfacerec.facerec.feature import SpatialHistogram
    from ocvfacerec.facerec.lbp import ExtendedLBP
    g = golden("lbp_golden.npz")
    names = [k[4:] for k in g.files if k.startswith("img_") and f"hist_{k[4:]}_r1p8_g8" in g.files]
    imgs = [g["img_" + n] for n in names]
    h8 = SpatialHistogram(ExtendedLBP(1, 8), (8, 8)).compute(imgs, None)
    h45 = SpatialHistogram(ExtendedLBP(2, 8), (4, 5)).compute(imgs, None)
    for n, a, b in zip(names, h8, h45):
        assert np.array_equal(a, g[f"hist_{n}_r1p8_g8"]), n
        assert np.array_equal(b, g[f"hist_{n}_r2p8_g4x5"]), n


def test_lbp_hist_counts_batch_vs_oracle():
    from ocvfacerec.facerec.feature import SpatialHistogram
    from opencv_facerecognizer_amd._device import counts_numpy
    r = _rng(11)
    imgs = r.integers(0, 256, (200, 128, 128), dtype=np.uint8)
    imgs[:50] = (imgs[:50] // 64) * 64 + 100          # tie-heavy
    sh = SpatialHistogram()
    counts, cell, cb = sh.counts_device(imgs)
    c = counts_numpy(counts, cb).astype(np.int64)
    assert cell == 225 and cb == 1
    for i in range(0, 200, 13):
        ref, _ = O.spatial_histogram_counts(O.elbp(imgs[i]), 8, (8, 8))
        assert np.array_equal(c[i], ref), i


@pytest.mark.parametrize("shape,grid", [((70, 70), (7, 7)), ((61, 93), (5, 4)), ((130, 128), (8, 8)),
                                        ((130, 128), (2, 2))])
def test_lbp_hist_r1p8_ragged_vs_oracle(shape, grid):
    """The register-window ExtendedLBP(1, 8) histogram kernel on sizes whose cells leave code rows /
    columns uncovered and whose pixel counts are not multiples of 16 (unaligned image staging)."""
    from ocvfacerec.facerec.feature import SpatialHistogram
    from ocvfacerec.facerec.lbp import ExtendedLBP
    from opencv_facerecognizer_amd._device import counts_numpy
    r = _rng(12)
    imgs = r.integers(0, 256, (24,) + shape, dtype=np.uint8)
    imgs[:8] = (imgs[:8] // 128) * 128 + 60            # tie-heavy
    sh = SpatialHistogram(ExtendedLBP(1, 8), grid)
    counts, cell, cb = sh.counts_device(imgs)
    c = counts_numpy(counts, cb).astype(np.int64)
    for i in range(24):
        ref, _ = O.spatial_histogram_counts(O.elbp(imgs[i]), 8, grid)
        assert np.array_equal(c[i], ref), i


def test_lbp_hist_r1p8_smooth_faces_vs_oracle():
    """Smooth images with little noise: the fast r1p8 kernel's fp32 decisions meet many near-ties
    (flat and mirror-symmetric neighbourhoods, which take the wave through the fp64 sequence) and
    its integer tie thresholds of points 4 and 6 (b == C) on every centre value."""
    from ocvfacerec.facerec.feature import SpatialHistogram
    from opencv_facerecognizer_amd._device import counts_numpy
    r = _rng(13)
    protos = r.integers(0, 256, (6, 16, 16)).astype(np.float64)
    up = np.kron(protos, np.ones((8, 8)))
    imgs = np.clip(up[np.arange(36) % 6] + r.normal(0, 1.5, (36, 128, 128)), 0, 255).astype(np.uint8)
    imgs[30:] = np.arange(128, dtype=np.uint8)[None, :, None] * 2      # ramps: every centre value ties
    sh = SpatialHistogram()
    counts, cell, cb = sh.counts_device(imgs)
    c = counts_numpy(counts, cb).astype(np.int64)
    for i in range(36):
        ref, _ = O.spatial_histogram_counts(O.elbp(imgs[i]), 8, (8, 8))
        assert np.array_equal(c[i], ref), i


# ---------------------------------------------------------------------------
# chi-square search
# ---------------------------------------------------------------------------
def test_chi2_counts_search_vs_oracle():
    from ocvfacerec.facerec.feature import SpatialHistogram
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import Chi2Gallery, counts_numpy
    r = _rng(12)
    protos = r.integers(0, 256, (20, 16, 16)).astype(np.float64)
    up = np.kron(protos, np.ones((8, 8)))
    gal = np.clip(up[np.arange(300) % 20] + r.normal(0, 20, (300, 128, 128)), 0, 255).astype(np.uint8)
    qry = np.clip(up[np.arange(70) % 20] + r.normal(0, 20, (70, 128, 128)), 0, 255).astype(np.uint8)
    sh = SpatialHistogram()
    gc, cell, cb = sh.counts_device(gal)
    qc, _, _ = sh.counts_device(qry)
    n, nb = gc.shape[0], gc.shape[1] * gc.shape[2]
    g = Chi2Gallery(gc.reshape(n, nb), dtype=_lib.DT_U8, denom=float(cell), nbins=nb)
    dd, ii = g.search(qc.reshape(qc.shape[0], nb).contiguous(), 5)
    Gh = counts_numpy(gc, cb).reshape(n, nb).astype(np.float64) / cell
    Qh = counts_numpy(qc, cb).reshape(-1, nb).astype(np.float64) / cell
    _check_search("ChiSquareDistance", Qh, Gh, dd.cpu().numpy(), ii.cpu().numpy(), 5)
    assert g.last_fallbacks[0] <= len(qry) // 10     # separated identities: the fp32 pass certifies


def test_chi2_certificate_forces_exact_pass():
    """Near-identical gallery rows: the 8 candidates of the fp32 pass lie within its error bound of each
    other, so no query can be certified there; every query is re-run by the exact fp64 pass
    (ofr_chi2_knn_exact) and the result matches the oracle."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import Chi2Gallery
    r = _rng(14)
    G = np.full((600, 4096), 10)
    for i in range(600):                               # every row: 50 bins one count above the base
        G[i, r.choice(4096, 50, replace=False)] += 1
    Q = np.full((12, 4096), 10)                        # every query is the base: all 600 rows tie
    g = Chi2Gallery(torch.from_numpy(G.astype(np.uint8)).cuda(), dtype=_lib.DT_U8, denom=225.0, nbins=4096)
    dd, ii = g.search(torch.from_numpy(Q.astype(np.uint8)).cuda().contiguous(), 3)
    assert g.last_fallbacks[0] == 12, g.last_fallbacks
    _check_search("ChiSquareDistance", Q / 225.0, G / 225.0, dd.cpu().numpy(), ii.cpu().numpy(), 3)


@pytest.mark.parametrize("data", ["lbp", "wide"])
def test_chi2_mfma_pass_equals_valu_pass_and_oracle(monkeypatch, data):
    """uint8 counts take the low-rank MFMA coarse pass (ofr_chi2.hip, c2m): the exact fp64 re-rank and
    its absolute certificate must give the oracle's top-k (distance.py:112-116 over the whole gallery),
    the same as the VALU pass (OFR_CHI2_ENGINE=valu).  'lbp': spatial histograms of 128x128 faces
    (tile edges: 700 rows, 300 queries); 'wide': counts spread over 0..255 with shared bins (the table's
    whole range)."""
    from ocvfacerec.facerec.feature import SpatialHistogram
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import Chi2Gallery, counts_numpy
    r = _rng(15)
    if data == "lbp":
        protos = r.integers(0, 256, (30, 16, 16)).astype(np.float64)
        up = np.kron(protos, np.ones((8, 8)))
        gal = np.clip(up[np.arange(700) % 30] + r.normal(0, 20, (700, 128, 128)), 0, 255).astype(np.uint8)
        qry = np.clip(up[r.integers(0, 30, 300)] + r.normal(0, 20, (300, 128, 128)), 0, 255).astype(np.uint8)
        sh = SpatialHistogram()
        gc, cell, cb = sh.counts_device(gal)
        qc, _, _ = sh.counts_device(qry)
        G = counts_numpy(gc, cb).reshape(700, -1).astype(np.int64)
        Q = counts_numpy(qc, cb).reshape(300, -1).astype(np.int64)
        denom = float(cell)
    else:
        base = r.integers(0, 256, (40, 1024))
        G = np.clip(base[np.arange(600) % 40] + r.integers(-3, 4, (600, 1024)), 0, 255)
        Q = np.clip(base[r.integers(0, 40, 257)] + r.integers(-3, 4, (257, 1024)), 0, 255)
        denom = 255.0
    g = Chi2Gallery.from_counts(G.astype(np.uint8), 1, denom)
    Qd = torch.from_numpy(Q.astype(np.uint8)).cuda()
    monkeypatch.delenv("OFR_CHI2_ENGINE", raising=False)
    dm, im = g.search(Qd, 3)
    fb_m = g.last_fallbacks
    monkeypatch.setenv("OFR_CHI2_ENGINE", "valu")
    dv, iv = g.search(Qd, 3)
    assert torch.equal(im, iv) and torch.equal(dm, dv)
    assert fb_m[0] <= len(Q) // 10, fb_m            # separated identities: the MFMA pass certifies
    _check_search("ChiSquareDistance", Q / denom, G / denom, dm.cpu().numpy(), im.cpu().numpy(), 3)


def test_chi2_float_search_vs_oracle():
    from opencv_facerecognizer_amd._device import Chi2Gallery
    r = _rng(13)
    G = r.random((500, 300)) ** 3
    Q = r.random((40, 300)) ** 3
    G = G.astype(np.float32).astype(np.float64)
    Q = Q.astype(np.float32).astype(np.float64)
    g = Chi2Gallery(G)
    dd, ii = g.search(g.query_rows(Q), 4)
    _check_search("ChiSquareDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), 4)


# ---------------------------------------------------------------------------
# training (Fisherfaces.compute on the bundled faces)
# ---------------------------------------------------------------------------
def test_fisherfaces_compute_bundled(golden):
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import LDA, PCA, Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    f = golden("individuals_faces.npz")
    X, y = list(f["X"]), f["y"]
    # PCA: mean exact, eigenvalues and subspace match the reference SVD
    pca = PCA(len(y) - 4)
    pf = pca.compute(X, y)
    assert np.array_equal(np.asarray(pca.mean).ravel(), f["pca_mean"])
    np.testing.assert_allclose(pca.eigenvalues, f["pca_eigenvalues"], rtol=1e-6)
    U, Ur = np.asarray(pca.eigenvectors), f["pca_eigenvectors"]
    cos = np.abs(np.sum(U * Ur, 0))
    assert cos.min() > 1 - 1e-6, cos
    # PCA features equal the reference's up to column sign
    sgn = np.sign(np.sum(U * Ur, 0))
    pfa = np.stack([np.asarray(p).ravel() for p in pf]) * sgn
    np.testing.assert_allclose(pfa, f["pca_features"], rtol=0, atol=1e-6 * np.abs(f["pca_features"]).max())
    # LDA scatter matrices equal the oracle's (on the reference PCA features)
    Sw, Sb, _ = LDA.scatter(list(f["pca_features"]), y)
    _, Sw_ref, Sb_ref = O.lda_scatter(f["pca_features"].T, y)
    np.testing.assert_allclose(Sw, Sw_ref, rtol=0, atol=1e-10 * np.abs(Sw_ref).max())
    np.testing.assert_allclose(Sb, Sb_ref, rtol=0, atol=1e-10 * np.abs(Sb_ref).max())
    # full model: resubstitution labels equal the reference's
    m = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
    m.compute(X, list(y))
    W = np.asarray(m.feature.eigenvectors)
    assert W.shape == (4900, 3) and m.feature.num_components == 3
    labels = [p[0] for p in m.predict_batch(X)]
    assert np.array_equal(labels, f["resub_labels"])
    # gallery features are W^T x of the model's own W (feature.py:231-235)
    feats = np.stack([np.asarray(x).ravel() for x in m.classifier.X])
    ref = f["X"].reshape(31, -1).astype(np.float64) @ W
    assert (np.linalg.norm(feats - ref, axis=1) / np.linalg.norm(ref, axis=1)).max() < 1e-4


def test_fisherfaces_eigh_solver_matches_eig(golden, monkeypatch):
    """OFR_LDA_SOLVER=eigh (symmetric-definite LDA, feature.lda_eigen) trains the same model on the
    bundled faces: W columns equal the reference-eig W up to sign, same resubstitution labels."""
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    f = golden("individuals_faces.npz")
    X, y = list(f["X"]), list(f["y"])
    Ws = []
    for solver in ("eig", "eigh", "device"):
        monkeypatch.setenv("OFR_LDA_SOLVER", solver)
        m = PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1))
        m.compute(X, y)
        Ws.append(np.asarray(m.feature.eigenvectors))
        assert np.array_equal([p[0] for p in m.predict_batch(X)], f["resub_labels"])
    # On these 31 faces Sw (27 x 27, PCA(n - c) space) is numerically singular (its Cholesky fails
    # or passes at order 27 depending on the last bits of the PCA features), so only the dominant
    # Fisherface is determined by the data for any solver: the pencil solvers must give the same
    # labels and that column (well-posed pencils: test_sygv_device_matches_lapack, test_lda_solver).
    W0 = Ws[0]
    for W1, ncol in ((Ws[1], 1), (Ws[2], 1)):
        cos = np.abs(np.sum(W0 * W1, 0)) / (np.linalg.norm(W0, axis=0) * np.linalg.norm(W1, axis=0))
        assert cos[:ncol].min() > 1 - 1e-5, cos


def test_kfold_validation_matches_reference_loop():
    """KFoldCrossValidation (validation.py:202-258) of the trainer's model (Fisherfaces +
    NearestNeighbor, thetrainer.py:120-124): one device batch per fold gives the reference loop's
    counts (oracle: per-face predicts, same random.seed shuffle).  Synthetic 32x32 faces of 12
    identities: the bundled set's folds (16 training faces, 4 classes) make LDA ill-conditioned
    (W parity is judged on scatter matrices and well-posed labels there)."""
    import random
    from opencv_facerecognizer_amd.synthetic import IdentityBank
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.feature import Fisherfaces
    from ocvfacerec.facerec.model import PredictableModel
    from ocvfacerec.facerec.validation import KFoldCrossValidation
    ids = torch.arange(12 * 9, device="cuda") % 12
    imgs = IdentityBank(12, 32, 32, device="cuda").images(ids, seed=5).reshape(-1, 32, 32).cpu().numpy()
    X, y = list(imgs), ids.cpu().numpy()
    for k, seed in [(3, 1), (9, 7)]:
        random.seed(seed)
        v = KFoldCrossValidation(PredictableModel(Fisherfaces(), NearestNeighbor(EuclideanDistance(), k=1)), k=k)
        v.validate(X, y)
        r = v.validation_results[0]
        tp, fp, k_used = O.kfold_fisherfaces_faithful(X, y, k=k, seed=seed)
        assert v.k == k_used and (r.true_positives, r.false_positives) == (tp, fp), (r, tp, fp)
        assert tp >= 0.9 * (tp + fp)


def test_gemm_f64_vs_numpy():
    from opencv_facerecognizer_amd._device import f64_dev, gemm_f64
    r = _rng(3)
    for (M, N, K) in [(31, 31, 4900), (100, 7, 33), (130, 257, 64), (257, 129, 17), (1, 300, 5), (513, 64, 1000)]:
        A = r.normal(size=(M, K))
        Bm = r.normal(size=(K, N))
        ref = A @ Bm
        for ta in (False, True):
            for tb in (False, True):
                Ad = f64_dev(A.T.copy() if ta else A)
                Bd = f64_dev(Bm.T.copy() if tb else Bm)
                C = gemm_f64(Ad, Bd, transA=ta, transB=tb).cpu().numpy()
                np.testing.assert_allclose(C, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def test_topk_merge_kernel():
    from opencv_facerecognizer_amd._device import topk_merge
    r = _rng(4)
    B, P, kin, k = 50, 4, 5, 7
    d = r.random((B, P, kin))
    d[:, 1, 0] = d[:, 0, 0]                      # cross-list ties
    i = r.integers(0, 10**6, (B, P, kin))
    for b in range(B):                           # each list ascending by (distance, index), as the ranks emit them
        for p in range(P):
            o = np.lexsort((i[b, p], d[b, p]))
            d[b, p], i[b, p] = d[b, p][o], i[b, p][o]
    i[:, 2, 3:] = -1                             # short list
    d[:, 2, 3:] = np.inf
    od, oi = topk_merge(torch.from_numpy(d.reshape(B, -1)).cuda(), torch.from_numpy(i.reshape(B, -1)).cuda(), P, kin, k)
    od, oi = od.cpu().numpy(), oi.cpu().numpy()
    for b in range(B):
        cand = [(d[b, p, j], i[b, p, j]) for p in range(P) for j in range(kin) if i[b, p, j] >= 0]
        cand.sort()
        ref = cand[:k]
        assert [x[1] for x in ref] == list(oi[b, :len(ref)])
        assert np.array_equal([x[0] for x in ref], od[b, :len(ref)])


def test_knn_cosine_zero_query_takes_fp32_path(monkeypatch):
    """A zero query has no unit vector: every reference distance is NaN (distance.py:77).  It must
    not be answered by the certified unit-row twin (whose row for it would be -shift); it gets the
    fp32 path's answer, NaN distances ranked by index like any all-NaN row set."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    r = _rng(404)
    G = r.normal(50, 10, (3000, 40)).astype(np.float32).astype(np.float64)
    Q = r.normal(50, 10, (64, 40)).astype(np.float32).astype(np.float64)
    Q[5] = 0.0
    g = FloatGallery(G, _lib.METRIC_COSINE)
    assert g.use_cos_cert(64, 3)
    dd, ii = g.search(g.query_rows(Q), 3)
    dd, ii = dd.cpu().numpy(), ii.cpu().numpy()
    monkeypatch.setenv("OFR_SEARCH", "fp32")
    d32, i32 = g.search(g.query_rows(Q[5:6]), 3)
    assert np.array_equal(ii[5], i32.cpu().numpy()[0]) and np.isnan(dd[5]).all()
    keep = np.arange(64) != 5
    _check_search("CosineDistance", Q[keep], G, dd[keep], ii[keep], 3)


def _merge_certify_ref(lists, P, B, k):
    """numpy restatement of ofr_topk_merge_certify (the global certificate of parallel.certify_sharded)."""
    L = lists.reshape(P, B, 2 * k + 1)
    od, oi, cert = np.empty((B, k)), np.empty((B, k), np.int64), np.empty(B, np.int32)
    for b in range(B):
        d = L[:, b, :k].reshape(-1)
        i = L[:, b, k:2 * k].copy().view(np.int64).reshape(-1)
        ok = i >= 0
        o = np.lexsort((i[ok], d[ok]))[:k]
        dd, ii = np.full(k, np.inf), np.full(k, -1, np.int64)
        dd[:len(o)], ii[:len(o)] = d[ok][o], i[ok][o]
        bnd = L[:, b, 2 * k]
        minb = -np.inf if np.isnan(bnd).any() else bnd.min()
        od[b], oi[b] = dd, ii
        cert[b] = np.isposinf(minb) or dd[-1] ** 2 < minb
    return od, oi, cert


@pytest.mark.parametrize("B", [1, 1000, 4096, 70001])
def test_exchange_kernels_pack_kth_open_rows(B):
    """The sharded step's exchange kernels against numpy: ofr_topk_pack (one rank's [B][2k+1] block,
    NULL bound = +inf), ofr_kth_bound (k-th smallest of P ascending lists of k bounds, +inf rows) and
    ofr_open_rows (ascending indices of cert == 0, across the 1024-query chunks of its scan)."""
    from opencv_facerecognizer_amd import _device as D_
    r = _rng(37 + B)
    k, P = 3, 4
    d = np.sort(r.random((B, k)), axis=1)
    i = r.integers(-1, 10 ** 9, (B, k)).astype(np.int64)
    bnd = r.random(B)
    for bound in (None, bnd):
        out = D_.topk_pack(torch.from_numpy(d).cuda(), torch.from_numpy(i).cuda(),
                           None if bound is None else torch.from_numpy(bound).cuda()).cpu().numpy()
        assert np.array_equal(out[:, :k], d) and np.array_equal(out[:, k:2 * k].copy().view(np.int64), i)
        assert np.array_equal(out[:, 2 * k], np.full(B, np.inf) if bound is None else bound)
    allb = np.sort(r.random((P, B, k)) * 10, axis=2)
    allb[1, ::7] = np.inf                                  # a rank with no candidate for some queries
    ub = D_.kth_bound(torch.from_numpy(allb).cuda(), P, B, k).cpu().numpy()
    ref = np.sort(allb.transpose(1, 0, 2).reshape(B, P * k), axis=1)[:, k - 1]
    assert np.array_equal(ub, ref)
    cert = (r.random(B) < 0.7).astype(np.int32)
    rows = D_.open_rows(torch.from_numpy(cert).cuda()).cpu().numpy()
    assert np.array_equal(rows, np.nonzero(cert == 0)[0])
    assert D_.open_rows(torch.ones(B, dtype=torch.int32, device="cuda")).numel() == 0


def test_topk_merge_certify_kernel():
    """In-library global certificate (ofr_topk_merge_certify): P = 3 ranks' lists with ties across
    ranks, empty slots, and bounds -inf (an overflowed rank: never certifies), +inf, NaN, finite."""
    from opencv_facerecognizer_amd._lib import call, ptr, stream
    r = _rng(31)
    P, B, k = 3, 64, 4
    L = np.empty((P, B, 2 * k + 1))
    for p in range(P):
        d = np.sort(np.round(r.random((B, k)) * 8) / 4, axis=1)          # coarse values: ties across ranks
        idx = (np.arange(k)[None, :] + 1000 * p + 10 * np.arange(B)[:, None]).astype(np.int64)
        idx[r.random((B, k)) < 0.05] = -1
        d[idx < 0] = np.inf
        L[p, :, :k], L[p, :, k:2 * k] = d, idx.view(np.float64)
        L[p, :, 2 * k] = r.choice([-np.inf, np.inf, np.nan, 0.5, 3.0, 100.0], B)
    lt = torch.from_numpy(L.reshape(-1).copy()).cuda()
    od = torch.empty((B, k), dtype=torch.float64, device="cuda")
    oi = torch.empty((B, k), dtype=torch.int64, device="cuda")
    ce = torch.empty(B, dtype=torch.int32, device="cuda")
    call("ofr_topk_merge_certify", stream(), ptr(lt), P, B, k, ptr(od), ptr(oi), ptr(ce))
    rd, ri, rc = _merge_certify_ref(L, P, B, k)
    assert np.array_equal(oi.cpu().numpy(), ri) and np.array_equal(od.cpu().numpy(), rd)
    assert np.array_equal(ce.cpu().numpy(), rc)
    assert rc.min() == 0 and rc.max() == 1


@pytest.mark.parametrize("data", ["separated", "sphere", "crowded", "prefix"])
def test_knn_sharded_c_abi_one_device(monkeypatch, data):
    """ofr_comm_init_all + ofr_knn_sharded (single process, RCCL) on this box's one device: the fp6
    tier, the all-gather, the global certificate and the tier chain of uncertified queries (f6x2,
    int8 x2, exact fp32), against the oracle.  'sphere' (equidistant rows) leaves every query
    uncertified by every quantized tier, forcing the exact pass; 'crowded' (tight clusters) is
    certified by f6x2 after fp6 fails -- with the same per-tier counts as the single-process
    chain (FloatGallery.search).  The merge's deep continuation is off: the chain is what runs here."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    from opencv_facerecognizer_amd.parallel import DeviceComm
    monkeypatch.setenv("OFR_MERGE_DEEP", "0")
    r = _rng(41)
    if data == "separated":
        protos = r.normal(0, 30, (300, 96))
        G = (protos[np.arange(3000) % 300] + r.normal(0, 5, (3000, 96)))
        Q = (protos[r.integers(0, 300, 100)] + r.normal(0, 5, (100, 96)))
    elif data == "sphere":
        c = r.normal(0, 50, 64)
        U = r.normal(0, 1, (2000, 64))
        G = c + 100.0 * U / np.linalg.norm(U, axis=1, keepdims=True)
        Q = c + r.normal(0, 1e-6, (100, 64))
    elif data == "prefix":   # Fisherfaces-like: identity variance in the leading 64 features (round 6)
        from test_gpu_prefix import _lda_like
        G, Q = _lda_like(1000, 10, 1280, 300, seed=11)
    else:   # test_knn_f6x2_certifies_crowded_clusters' data
        r = _rng(3)
        mu = r.normal(0, 1, (200, 128))
        G = mu[np.arange(8000) % 200] + r.normal(0, 0.5, (8000, 128))
        Q = mu[r.integers(0, 200, 300)] + r.normal(0, 0.5, (300, 128))
    G = G.astype(np.float32).astype(np.float64)
    Q = Q.astype(np.float32).astype(np.float64)
    k = 3 if data != "crowded" else 1
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    with DeviceComm([0]) as comm:
        (dd, ii, cert), = comm.knn([g], [g.query_rows(Q)], k)
        counts = comm.last_tier_counts
        popen = comm.last_prefix_open
    _check_search("EuclideanDistance", Q, G, dd.cpu().numpy(), ii.cpu().numpy(), k)
    c = cert.cpu().numpy()
    if data == "prefix":
        # the prefix tier ran first (its own exchange and global certificate) and certified every query
        assert g.prefix_stages() >= 1 and popen == 0 and counts[0] == 0, (g.prefix_stages(), popen, counts)
        assert c.min() == 1
        # forced on isotropic rows: the prefix tier certifies nothing, the fp6 tier takes every query
        G2 = _rng(12).normal(0, 20, (4000, 1280)).astype(np.float32).astype(np.float64)
        Q2 = (G2[_rng(13).integers(0, 4000, 100)] + _rng(14).normal(0, 1, (100, 1280))).astype(np.float32).astype(np.float64)
        monkeypatch.setenv("OFR_F6_PREFIX", "1")
        g2 = FloatGallery(G2, _lib.METRIC_EUCLIDEAN)
        with DeviceComm([0]) as comm:
            (d2, i2, c2), = comm.knn([g2], [g2.query_rows(Q2)], k)
            assert comm.last_prefix_open == len(Q2) and comm.last_tier_counts[0] >= 0, (
                comm.last_prefix_open, comm.last_tier_counts)
        _check_search("EuclideanDistance", Q2, G2, d2.cpu().numpy(), i2.cpu().numpy(), k)
    elif data == "separated":
        assert c.min() == 1 and counts == [0, -1, -1, -1]
    elif data == "sphere":
        assert c.max() == 0 and counts[0] == len(Q) and counts[3] == counts[2] == counts[1] == len(Q), counts
    else:
        monkeypatch.setenv("OFR_SEARCH", "auto")
        g.search(g.query_rows(Q), k)                    # the single-process chain on the same gallery
        fb = list(g.last_fallbacks)
        assert counts[0] >= 0.9 * len(Q) and counts[1] <= 0.02 * len(Q), counts
        assert counts[:2] == fb[:2], (counts, fb)
        # cert 0 marks exactly the queries the exact pass resolved
        assert int((c == 0).sum()) == max(counts[3], 0), (counts, int((c == 0).sum()))


def _spd(r, n, extra=0.2):
    X = r.normal(0, 1, (int(n * (1 + extra)), n))
    return X.T @ X / X.shape[0] + 1e-3 * np.eye(n)


@pytest.mark.parametrize("n,m", [(300, 300), (300, 17), (1, 1), (257, 0)])
def test_eigh_device_matches_lapack(n, m):
    """ofr_eigh_f64 (rocSOLVER dsyevd): the m largest eigenpairs, descending, vs numpy eigh
    (the PCA eigensolve of training.eigh_desc; feature.py:94 svd)."""
    from opencv_facerecognizer_amd import _device
    r = _rng(51)
    A = _spd(r, n)
    lam, V = _device.eigh_desc_f64(torch.from_numpy(A).cuda(), m)
    l0, V0 = np.linalg.eigh(A)
    l0, V0 = l0[::-1][:m], V0[:, ::-1][:, :m]
    lam, V = lam.cpu().numpy(), V.cpu().numpy()
    assert lam.shape == (m,) and V.shape == (n, m)
    assert np.allclose(lam, l0, rtol=1e-10, atol=1e-12 * max(1.0, abs(l0).max(initial=0)))
    if m:
        cos = np.abs(np.sum(V * V0, 0))
        gap = np.minimum(np.abs(np.diff(np.r_[np.inf, l0])), np.abs(np.diff(np.r_[l0, -np.inf])))
        assert cos[gap > 1e-6 * abs(l0).max()].min() > 1 - 1e-8
        assert np.allclose(V.T @ V, np.eye(m), atol=1e-10)


@pytest.mark.parametrize("m", [40, 250])
def test_sygv_device_matches_lapack(m):
    """ofr_sygv_f64 (rocSOLVER dsygvd): Sb v = lambda Sw v, the m largest, unit columns, vs scipy
    eigh(Sb, Sw) and the reference's eig(inv(Sw) Sb) (feature.py:170) through lda_eigen."""
    import scipy.linalg
    from opencv_facerecognizer_amd import _device
    from opencv_facerecognizer_amd.facerec.feature import lda_eigen
    r = _rng(52)
    n = 250
    Sw = _spd(r, n)
    Y = r.normal(0, 1, (60, n))
    Sb = Y.T @ Y                                       # rank 60 like c - 1 classes
    lam, V = _device.sygv_desc_f64(torch.from_numpy(Sb).cuda(), torch.from_numpy(Sw).cuda(), m)
    lam, V = lam.cpu().numpy(), V.cpu().numpy()
    l0, V0 = scipy.linalg.eigh(Sb, Sw)
    l0, V0 = l0[::-1][:m], V0[:, ::-1][:, :m]
    scale = abs(l0).max()
    assert np.allclose(lam, l0, rtol=1e-9, atol=1e-11 * scale)
    assert np.allclose(np.linalg.norm(V, axis=0), 1.0, atol=1e-12)
    k = min(m, 59)                                     # the non-null part: distinct eigenvalues
    V0n = V0[:, :k] / np.linalg.norm(V0[:, :k], axis=0)
    assert np.abs(np.sum(V[:, :k] * V0n, 0)).min() > 1 - 1e-8
    # lda_eigen "device" against the reference's inv + eig
    le, Ve = lda_eigen(Sw, Sb, k, solver="eig")
    ld, Vd = lda_eigen(torch.from_numpy(Sw).cuda(), torch.from_numpy(Sb).cuda(), k, solver="device")
    assert np.allclose(ld, le, rtol=1e-8)
    assert np.abs(np.sum(Vd * Ve, 0)).min() > 1 - 1e-7


def test_sygv_device_not_positive_definite_falls_back():
    """An indefinite Sw: ofr_sygv_f64 reports OFR_E_NUMERIC and lda_eigen falls back to the
    reference's general eig with a warning (as the host pencil solver does)."""
    from opencv_facerecognizer_amd import _device, _lib
    from opencv_facerecognizer_amd.facerec.feature import lda_eigen
    r = _rng(53)
    n = 40
    N = r.normal(0, 0.01, (n, n))
    Sw = np.diag(np.r_[-1.0, np.linspace(1, 2, n - 1)]) + (N + N.T)   # invertible, not definite
    Sb = _spd(r, n)
    with pytest.raises(_lib.OfrError) as e:
        _device.sygv_desc_f64(torch.from_numpy(Sb).cuda(), torch.from_numpy(Sw).cuda(), 5)
    assert e.value.code == _lib.E_NUMERIC
    with pytest.warns(UserWarning, match="not positive definite"):
        lam, V = lda_eigen(Sw, Sb, 3, solver="device")
    le, Ve = lda_eigen(Sw, Sb, 3, solver="eig")
    assert np.array_equal(lam, le) and np.array_equal(V, Ve)


def test_model_reload_releases_device_memory(golden):
    """The ROS recognizer reloads the model on every restart (ocvf_recognizer_ros.py:251-256): the
    dropped model's device state (projection, gallery, quantized tiers, workspaces) must be freed,
    so repeated load -> predict -> drop cycles do not grow device memory."""
    import gc
    from ocvfacerec.facerec.classifier import NearestNeighbor
    from ocvfacerec.facerec.distance import EuclideanDistance
    from ocvfacerec.facerec.serialization import load_model
    f = golden("individuals_faces.npz")
    r = _rng(77)
    G = r.normal(0, 3, (20000, 64))
    Q = G[:300] + r.normal(0, 0.1, (300, 64))

    def cycle():
        m = load_model(os.path.join(GOLDEN, "individuals.pkl"))
        m.predict_batch(list(f["X"]))
        m.predict(f["X"][0])
        nn = NearestNeighbor(EuclideanDistance(), k=1)
        nn.compute(list(G), np.arange(len(G)))
        nn.predict_batch(Q)          # fp6 sieve tier: gallery tiles, workspaces
        nn.predict_batch(Q[:3])      # fp6 stream tier
        del m, nn
        gc.collect()
        torch.cuda.synchronize()

    cycle()
    base = torch.cuda.memory_allocated()
    for _ in range(4):
        cycle()
    assert torch.cuda.memory_allocated() <= base
