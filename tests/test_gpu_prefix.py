"""The prefix tier f6p (ofr_knn_f6p_sampled): the fp6 sieve on the first pstages
128-feature stages of the f6 tiles, certified by the projection bound d^2 >= |q_m - g_m|^2.

Reference: classifier.py:104-119 (the exact k nearest of the whole gallery, any features).  Fisherfaces
features come in eigenvalue order (feature.py:211-235, the LDA eigenvectors sorted by eigenvalue), so the
identity-separating variance sits in the leading columns; _lda_like makes such features: identity centres
in the first `lead` columns, within-identity noise in all of them.
Checked: the tier is chosen only for such galleries; its certified answers are the exact fp64 top-k
(numpy / torch fp64 over the fp32 rows) and equal the f6 tier's; the sieve keeps every row whose exact
prefix score of the device's own fp6 codes is below theta; forced onto isotropic data it hands its
failures to f6 and the results stay exact; the B <= 32 streaming pass and append.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    torch.cuda.set_device(0)


def _lda_like(n_id, per, d, B, lead=64, seed=0, spread=60.0, noise=3.0):
    r = np.random.default_rng(seed)
    C = np.zeros((n_id, d))
    C[:, :lead] = r.normal(0, spread, (n_id, lead))
    G = (np.repeat(C, per, axis=0) + r.normal(0, noise, (n_id * per, d))).astype(np.float32).astype(np.float64)
    ids = r.integers(0, n_id, B)
    Q = (C[ids] + r.normal(0, noise, (B, d))).astype(np.float32).astype(np.float64)
    return G, Q


def _exact_topk(g, Qd, k):
    Gt = g.G[:, :g.d].double()
    Qt = Qd[:, :g.d].double()
    D2 = (Qt * Qt).sum(1)[:, None] + (Gt * Gt).sum(1)[None, :] - 2.0 * Qt @ Gt.t()
    return torch.topk(D2, k, dim=1, largest=False).indices.cpu().numpy()


@pytest.mark.parametrize("k", [1, 5, 8])
def test_prefix_tier_certifies_exact_topk(k, monkeypatch):
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.delenv("OFR_F6_PREFIX", raising=False)
    G, Q = _lda_like(3000, 10, 1280, 512, seed=k)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    assert g.prefix_stages() == 1
    Qd = g.query_rows(Q)
    d_, i_ = g.search(Qd, k)
    torch.cuda.synchronize()
    assert g.last_start_tier == "f6p"
    assert g.last_fallbacks[0] == 0, g.last_fallbacks           # every query certified by the prefix
    got = i_.cpu().numpy()
    want = _exact_topk(g, Qd, k)
    assert np.array_equal(np.sort(got, 1), np.sort(want, 1))
    # the same answers as the full fp6 tier (distances: the same exact fp64 re-rank)
    monkeypatch.setenv("OFR_F6_PREFIX", "0")
    h = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    assert h.prefix_stages() == 0
    d2, i2 = h.search(h.query_rows(Q), k)
    torch.cuda.synchronize()
    assert h.last_start_tier == "f6"
    assert np.array_equal(got, i2.cpu().numpy())
    assert np.array_equal(d_.cpu().numpy(), d2.cpu().numpy())


def test_prefix_sieve_keeps_every_row_below_theta():
    """Bucket completeness of the prefix sieve pass: every row whose EXACT prefix coarse score (the
    device's fp6 codes of the first pstages stages, decoded; times the block scales; the prefix aux) is
    below theta by more than the fp32 accumulation bound is kept, none above it by more."""
    from test_gpu_sieve import _decode_panels, _e2m3_table, _key_float
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    G, Q = _lda_like(2500, 8, 1280, 300, seed=11)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    pst = g.prefix_stages()
    assert pst == 1
    Qd = g.query_rows(Q)
    qq = g.quantize_queries(Qd, tier="f6p")
    g.search_q8_phase(4 | 8, Qd, qq, 1)
    torch.cuda.synchronize()
    B, N, d = len(Q), g.N, g.d
    theta, count, keys, rows = g.sieve_state(B)
    cnt = count.cpu().numpy()
    assert np.all((cnt >= 1) & (cnt <= g.SIEVE_CAP)), cnt
    dev = Qd.device
    nst, m = -(-d // 128), 128 * pst
    table = _e2m3_table(dev)
    bs = g._block_scales()
    f = torch.pow(2.0, bs.double() - 127.0).repeat_interleave(32)[:d]
    Vq = _decode_panels(qq["Qs"], 0, -(-B // 256), nst, d, table)[:B, :m] * f[:m]
    gt = g._tier_gallery("f6p")              # its own compact tiles: pst stages per panel
    Vg = _decode_panels(gt["Gs"], 0, -(-N // 256), pst, d, table, pst)[:N, :m] * f[:m]
    gsc = gt["scale"][:N]
    assert torch.equal(gsc, torch.exp2(torch.round(torch.log2(gsc)))), "row scales must be powers of two"
    sq, gs = qq["scale"].double(), gt["scale"][:N].double()
    paux = gt["paux"][:N].double()
    # the prefix terms are |g_m|^2 of the stored rows
    assert torch.allclose(paux, g.G[:, :m].double().pow(2).sum(1), rtol=1e-6)
    dot = Vq @ Vg.t()
    t = 2.0 * sq[:, None] * gs[None, :]
    S = paux[None, :] - t * dot
    gamma = (2 * nst + 64) * 2.0 ** -23
    # the pass adds -paux inside the MFMA's fp32 accumulation: the certificate's 2^-14 paux
    band = (t * (gamma * (Vq.abs() @ Vg.abs().t()) + 2.0 ** -22 * dot.abs()) + 2.0 ** -14 * paux[None, :]
            + 2.0 ** -22 * S.abs())
    thf = torch.from_numpy(_key_float(theta.cpu().numpy())).to(dev)
    below = (S < thf[:, None] - band).cpu().numpy()
    above = (S > thf[:, None] + band).cpu().numpy()
    rows_h = rows.cpu().numpy()
    for b in range(B):
        kept = rows_h[b, :cnt[b]]
        assert len(np.unique(kept)) == len(kept), b
        assert np.setdiff1d(np.nonzero(below[b])[0], kept).size == 0, b
        assert np.intersect1d(np.nonzero(above[b])[0], kept).size == 0, b
    assert below.sum() >= B


def test_isotropic_gallery_has_no_prefix():
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    r = np.random.default_rng(4)
    g = FloatGallery(r.normal(0, 10, (5000, 1280)), _lib.METRIC_EUCLIDEAN)
    assert g.prefix_stages() == 0
    assert g.start_tier(512) == "f6"


def test_prefix_forced_on_isotropic_data_stays_exact(monkeypatch):
    """OFR_F6_PREFIX=1 on features without a leading block: the prefix bound is weak, queries fail the
    prefix certificate and go on to f6 (then f6x2 ...): the answers are still the exact top-k."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_F6_PREFIX", "1")
    r = np.random.default_rng(8)                 # no clusters: every row about equally far, the prefix
    G = r.normal(0, 10, (15000, 640))            # (1/5 of the features) bounds a fifth of each distance
    Q = r.normal(0, 10, (300, 640)).astype(np.float32).astype(np.float64)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    assert g.prefix_stages() == 1
    Qd = g.query_rows(Q)
    d_, i_ = g.search(Qd, 3)
    torch.cuda.synchronize()
    assert g.last_start_tier == "f6p"
    assert g.last_fallbacks[0] > len(Q) // 2, g.last_fallbacks
    assert np.array_equal(np.sort(i_.cpu().numpy(), 1), np.sort(_exact_topk(g, Qd, 3), 1))


@pytest.mark.parametrize("B", [1, 7, 32])
def test_prefix_small_batch_streaming_pass(B):
    """B <= 32: the fp6 streaming pass over the first pstages stages (stream_kernel_f6), premerge and
    merge with the prefix bound."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    G, Q = _lda_like(4000, 10, 1280, B, seed=100 + B)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    Qd = g.query_rows(Q)
    d_, i_ = g.search(Qd, 2)
    torch.cuda.synchronize()
    assert g.last_start_tier == "f6p" and g.last_fallbacks[0] == 0, g.last_fallbacks
    assert np.array_equal(np.sort(i_.cpu().numpy(), 1), np.sort(_exact_topk(g, Qd, 2), 1))


def test_prefix_tier_extended_by_append():
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    G, Q = _lda_like(1200, 10, 1280, 300, seed=5)
    g = FloatGallery(G[:7000], _lib.METRIC_EUCLIDEAN)
    g.append(G[7000:9000])
    g._tier_gallery("f6p")
    cap = g.capacity()
    g.append(G[9000:cap])                                     # in place: the prefix terms are extended
    assert g.q8 is not None and "f6p" in g.q8
    h = FloatGallery(G[:cap], _lib.METRIC_EUCLIDEAN, shift64=g.shift64)
    h.set_block_scales(g.block_sums())
    a, b = g._tier_gallery("f6p"), h._tier_gallery("f6p")
    assert torch.equal(a["paux"][:cap], b["paux"][:cap])
    assert torch.equal(a["spaux"], b["spaux"])
    Qd = g.query_rows(Q)
    d_, i_ = g.search(Qd, 4)
    torch.cuda.synchronize()
    assert g.last_start_tier == "f6p"
    assert np.array_equal(np.sort(i_.cpu().numpy(), 1), np.sort(_exact_topk(g, Qd, 4), 1))


@pytest.mark.parametrize("pst,B,n_id", [(1, 300, 2003), (2, 700, 1501), (2, 4096, 997)])
def test_persistent_prefix_pass_matches_per_tile_pass(monkeypatch, pst, B, n_id):
    """tile_kernel_f6p (persistent, pstages = 2) keeps exactly the rows, with exactly the keys, of
    tile_kernel_f6w on the same prefix (OFR_F6P_PERSIST=0): the same MFMAs in the same order and the same
    compares.  pstages = 1 runs prefix_pass_kernel<true> (round 6), whose MFMA adds -|g_m|^2 inside its fp32
    accumulation: its keys are within 2^-14 |g_m|^2 (the certificate's term) of f6w's, and a row kept by
    only one of the two passes lies within that band of theta.  The exact outputs (distances, indices,
    certificates) are equal either way.  Partial last gallery tile and query panel; B = 4096: 16 query
    panels per item."""
    from opencv_facerecognizer_amd import _lib
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_F6_PREFIX", str(pst))
    G, Q = _lda_like(n_id, 9, 1280, B, seed=pst * 7 + B)
    g = FloatGallery(G, _lib.METRIC_EUCLIDEAN)
    assert g.prefix_stages() == pst
    Qd = g.query_rows(Q)
    monkeypatch.setenv("OFR_F6P_PERSIST", "1")
    folded = pst == 1 and "folded" in _lib.load().ofr_f6p_sieve_kernel(1).decode()   # the default engine
    state, res = {}, {}
    for mode in ("1", "0"):
        monkeypatch.setenv("OFR_F6P_PERSIST", mode)
        qq = g.quantize_queries(Qd, tier="f6p")
        out = g.search_q8_phase(4 | 8 | 2, Qd, qq, 3)
        torch.cuda.synchronize()
        theta, count, keys, rows = g.sieve_state(B)
        count = count.cpu().numpy().copy()
        assert np.all((count >= 3) & (count <= g.SIEVE_CAP)), count
        pairs = []
        rows_h, keys_h = rows.cpu().numpy(), keys.cpu().numpy()
        for b in range(B):
            r = rows_h[b, :count[b]]
            kk = keys_h[b, :count[b]]
            o = np.argsort(r)
            pairs.append((r[o], kk[o]))
        state[mode] = (count, pairs)
        res[mode] = (out[0].cpu().numpy(), out[1].cpu().numpy(), qq["cert"].cpu().numpy().copy())
    if not folded:
        assert np.array_equal(state["1"][0], state["0"][0])
        for b in range(B):
            assert np.array_equal(state["1"][1][b][0], state["0"][1][b][0]), b
            assert np.array_equal(state["1"][1][b][1].view(np.uint32), state["0"][1][b][1].view(np.uint32)), b
    else:
        from test_gpu_sieve import _key_float
        paux = g._tier_gallery("f6p")["paux"][:g.N].double().cpu().numpy()
        th = _key_float(theta.cpu().numpy())
        n_diff = 0
        for b in range(B):
            (ra, ka), (rb, kb) = state["1"][1][b], state["0"][1][b]
            common, ia, ib = np.intersect1d(ra, rb, return_indices=True)
            tol = 2.0 ** -14 * paux[common] + 2.0 ** -14 * np.abs(kb[ib].astype(np.float64))   # + the key truncation
            assert np.all(np.abs(ka[ia].astype(np.float64) - kb[ib].astype(np.float64)) <= tol), b
            for r in np.setxor1d(ra, rb):   # kept by one pass only: at theta up to the band
                n_diff += 1
                k_any = ka[ra == r] if r in ra else kb[rb == r]
                assert abs(float(k_any[0]) - th[b]) <= 2.0 ** -14 * paux[r] + 2.0 ** -14 * abs(th[b]), (b, r)
        assert n_diff <= B, n_diff
    for j in range(3):
        assert np.array_equal(res["1"][j], res["0"][j])
    assert res["1"][2].all()
    assert np.array_equal(np.sort(res["1"][1], 1), np.sort(_exact_topk(g, Qd, 3), 1))
