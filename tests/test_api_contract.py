"""Reference API conventions that need no GPU (model.py:40-44, feature.py:269-270, reprs, pickled state),
and the loud failure of the compute path when no HIP device is visible (no CPU fallback)."""
import numpy as np
import pytest
import torch

from ocvfacerec.facerec.classifier import AbstractClassifier, NearestNeighbor
from ocvfacerec.facerec.distance import ChiSquareDistance, CosineDistance, EuclideanDistance
from ocvfacerec.facerec.feature import LDA, PCA, AbstractFeature, Fisherfaces, Identity, SpatialHistogram
from ocvfacerec.facerec.lbp import ExtendedLBP, LocalDescriptor
from ocvfacerec.facerec.model import PredictableModel
from ocvfacerec.facerec.operators import ChainOperator
from ocvfacerec.trainer.thetrainer import ExtendedPredictableModel, TheTrainer


def test_type_checks():
    with pytest.raises(TypeError, match="feature must be of type AbstractFeature"):
        PredictableModel(object(), NearestNeighbor())
    with pytest.raises(TypeError, match="classifier must be of type AbstractClassifier"):
        PredictableModel(Fisherfaces(), object())
    with pytest.raises(TypeError, match="LocalDescriptor"):
        SpatialHistogram(lbp_operator=object())
    with pytest.raises(Exception, match="FeatureOperator only works"):
        ChainOperator(PCA(), object())


def test_abstract_methods_raise():
    with pytest.raises(NotImplementedError):
        AbstractFeature().compute([], [])
    with pytest.raises(NotImplementedError):
        AbstractClassifier().predict(None)
    with pytest.raises(NotImplementedError):
        AbstractClassifier().update(None, None)
    with pytest.raises(NotImplementedError):
        LocalDescriptor(8)(np.zeros((3, 3)))


def test_reprs_and_defaults():
    assert repr(Fisherfaces()) == "Fisherfaces (num_components=0)"
    assert repr(PCA(5)) == "PCA (num_components=5)" and repr(LDA(2)) == "LDA (num_components=2)"
    assert repr(NearestNeighbor()) == "NearestNeighbor (k=1, dist_metric=EuclideanDistance)"
    assert repr(ExtendedLBP()) == "ExtendedLBP (neighbors=8, radius=1)"
    assert repr(SpatialHistogram()) == "SpatialHistogram (operator=ExtendedLBP (neighbors=8, radius=1), grid=(8, 8))"
    assert [m().name for m in (EuclideanDistance, CosineDistance, ChiSquareDistance)] == \
        ["EuclideanDistance", "CosineDistance", "ChiSquareDistance"]
    m = TheTrainer.get_model((70, 70), {0: "a"})
    assert isinstance(m, ExtendedPredictableModel) and isinstance(m.feature, Fisherfaces)
    assert m.classifier.k == 1 and isinstance(m.classifier.dist_metric, EuclideanDistance)
    assert Identity().extract(5) == 5


def test_classes_pickle_under_reference_paths():
    assert Fisherfaces.__module__ == "ocvfacerec.facerec.feature"
    assert NearestNeighbor.__module__ == "ocvfacerec.facerec.classifier"
    assert ExtendedPredictableModel.__module__ == "ocvfacerec.trainer.thetrainer"
    import ocvfacerec.facerec.feature as f
    import opencv_facerecognizer_amd.facerec.feature as g
    assert f is g


def test_nearest_neighbor_update_and_state():
    c = NearestNeighbor(k=3)
    c.update(np.ones((4, 1)), 2)
    assert len(c.X) == 1 and list(c.y) == [2]
    c.__dict__["_dev"] = object()
    assert "_dev" not in c.__getstate__()


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device failure mode")
def test_compute_path_fails_loudly_without_gpu():
    from opencv_facerecognizer_amd._lib import OfrError
    c = NearestNeighbor()
    c.compute([np.ones((3, 1)), np.zeros((3, 1))], [0, 1])
    with pytest.raises(OfrError, match="no HIP device"):
        c.predict(np.ones((3, 1)))
    with pytest.raises(OfrError, match="no HIP device"):
        ExtendedLBP()(np.zeros((5, 5), np.uint8))
    with pytest.raises(OfrError, match="no HIP device"):
        EuclideanDistance()(np.ones(3), np.zeros(3))


def test_vote_matches_reference_expression():
    """classifier.vote: the reference's bincount/dict/max (classifier.py:121-123) -- most frequent
    label, ties to the smallest -- computed with np.unique; same value and type, same errors."""
    import operator as op
    from ocvfacerec.facerec.classifier import vote

    def ref(sorted_y):
        hist = dict((key, val) for key, val in enumerate(np.bincount(sorted_y)) if val)
        return max(hist.items(), key=op.itemgetter(1))[0]

    r = np.random.default_rng(7)
    for _ in range(3000):
        y = r.integers(0, r.integers(1, 40), r.integers(1, 17))
        got = vote(y)
        assert got == ref(y) and type(got) is int
    with pytest.raises(ValueError):
        vote(np.array([], dtype=np.int64))
    with pytest.raises(ValueError):
        vote(np.array([2, -1]))


def test_shard_is_derived_state():
    """NearestNeighbor.shard / PredictableModel.shard (multi-GPU, tests/test_gpu_shard_api.py): a
    no-op outside torch.distributed, never pickled, and a loaded file cannot pre-seed it."""
    import pickle
    from opencv_facerecognizer_amd.facerec import _safepickle
    clf = NearestNeighbor(EuclideanDistance(), k=1)
    clf.compute([np.zeros(3), np.ones(3)], [0, 1])
    model = PredictableModel(Fisherfaces(), clf).shard()
    assert model.classifier is clf and clf._shard_info() is None      # world size 1: unsharded
    assert "_shard" not in clf.__getstate__()
    assert _safepickle._is_cache_key("_shard")
    clf2 = pickle.loads(pickle.dumps(clf))
    assert "_shard" not in clf2.__dict__ and clf2.k == 1


def test_certified_tier_paths():
    """The certified search chain (host logic, _device.FloatGallery): fp6 -> two-slice fp6 -> int8 x2
    -> fp32 for the default first tier; OFR_SEARCH=q8 / q8x2 start at the int8 tiers; sets of <= 32
    open queries go straight to the exact fp32 pass."""
    from opencv_facerecognizer_amd._device import SMALL_BATCH, FloatGallery
    assert FloatGallery.tier_path("f6") == ("f6", "f6x2", 2, "fp32")
    assert FloatGallery.tier_path(1) == (1, 2, "fp32")
    assert FloatGallery.tier_path(2) == (2, "fp32")
    g = FloatGallery.__new__(FloatGallery)
    assert g.next_tier("f6", SMALL_BATCH + 1) == "f6x2" and g.next_tier("f6x2", 4096) == 2
    assert g.next_tier("f6", SMALL_BATCH) == "fp32" and g.next_tier(2, 4096) == "fp32"
    for t in FloatGallery.TIER_CHAIN[:-1]:
        assert FloatGallery.tier_path(t)[-1] == "fp32"


def test_start_tier_policy_host_logic(monkeypatch):
    """FloatGallery.start_tier / note_failures without a device: skip a tier at >= SKIP_FAIL recent
    failures (never to fp32), small batches and OFR_ADAPTIVE_TIER=0 keep the first tier, the
    average of the last two batches decides, every REPROBE-th batch probes the first tier."""
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    monkeypatch.delenv("OFR_ADAPTIVE_TIER", raising=False)
    g = FloatGallery.__new__(FloatGallery)
    g.tier_failures, g._starts, g._pst = {}, 0, 0          # no prefix tier (isotropic features)
    assert g.start_tier(4096) == "f6"
    g.note_failures("f6", 4096, 4096)
    assert g.start_tier(4096) == "f6x2"
    assert g.start_tier(32) == "f6"                      # small batches: no statistics, no skipping
    g.note_failures("f6x2", 4096, 4000)
    assert g.start_tier(4096) == 2                        # f6x2 fails too: int8 x2
    g.note_failures(2, 4096, 4096)
    assert g.start_tier(4096) == 2                        # never skipped to the fp32 pass
    g.note_failures("f6", 4096, 0)                        # (1.0 + 0.0) / 2 < SKIP_FAIL
    g.tier_failures.pop("f6x2")
    assert g.start_tier(4096) == "f6"
    g.note_failures("f6", 100, 100)                       # batches below ADAPT_MIN_BATCH are not counted
    assert g.tier_failures["f6"] == 0.5
    g.tier_failures["f6"] = 1.0
    seen = [g.start_tier(4096) for _ in range(2 * FloatGallery.REPROBE)]
    assert seen.count("f6") == 2 and seen.count("f6x2") == 2 * FloatGallery.REPROBE - 2
    monkeypatch.setenv("OFR_ADAPTIVE_TIER", "0")
    assert g.start_tier(4096) == "f6"


def test_prefix_tier_start_and_skip_host_logic(monkeypatch):
    """With a prefix (FloatGallery.prefix_stages > 0) the chain starts at f6p, whose failures go on to
    f6 (no skip prediction: a prefix bound says nothing of f6's); a failing prefix is skipped."""
    from opencv_facerecognizer_amd._device import FloatGallery
    monkeypatch.setenv("OFR_SEARCH", "auto")
    monkeypatch.delenv("OFR_ADAPTIVE_TIER", raising=False)
    assert FloatGallery.tier_path("f6p") == ("f6p", "f6", "f6x2", 2, "fp32")
    g = FloatGallery.__new__(FloatGallery)
    g.tier_failures, g._starts, g._pst = {}, 0, 2
    assert g.start_tier(4096) == "f6p" and g.start_tier(8) == "f6p"
    g.note_failures("f6p", 4096, 4000)
    assert g.start_tier(4096) == "f6"
    monkeypatch.setenv("OFR_SEARCH", "q8")
    assert g.start_tier(4096) == 1                        # an explicit int8 start ignores the prefix


def _block_sums(ms, N, d):
    width = np.minimum(32, d - 32 * np.arange(len(ms)))
    return np.asarray(ms, np.float64) * N * width


def test_choose_prefix_host_logic(monkeypatch):
    """FloatGallery.choose_prefix: stages up to the last block whose mean square is >= PREFIX_RATIO x
    the median, if they are <= 1/PREFIX_MAX_FRAC of the stages and hold >= PREFIX_MIN_SHARE of the
    variance, shortened while PREFIX_SHORTEN of that share stays; OFR_F6_PREFIX forces a count or 0."""
    from opencv_facerecognizer_amd._device import FloatGallery as F
    monkeypatch.delenv("OFR_F6_PREFIX", raising=False)
    monkeypatch.delenv("OFR_SIEVE_SAMPLE", raising=False)
    d = 9999
    nb = -(-d // 32)
    # the trained W's profile (bench feature_profile): 6 blocks of rms 272 .. 54, the rest ~11.4
    rms = np.full(nb, 11.4)
    rms[:6] = [272, 218, 180, 137, 87, 54]
    # features 0..191 lead (2 stages), but the first stage holds 0.94 of their share -> 1 stage
    assert F.choose_prefix(_block_sums(rms ** 2, 1000, d), d, 1000) == 1
    late = rms.copy()
    late[4:8] = [200, 190, 180, 170]                       # the second stage as loud as the first: 2 stages
    assert F.choose_prefix(_block_sums(late ** 2, 1000, d), d, 1000) == 2
    assert F.choose_prefix(_block_sums(np.full(nb, 130.0), 1000, d), d, 1000) == 0   # isotropic
    spread = rms.copy()
    spread[300] = 500                                      # a leading block late: prefix too long
    assert F.choose_prefix(_block_sums(spread ** 2, 1000, d), d, 1000) == 0
    weak = np.full(nb, 11.4)
    weak[0] = 40                                           # one loud block, but < half of the variance
    assert F.choose_prefix(_block_sums(weak ** 2, 1000, d), d, 1000) == 0
    assert F.choose_prefix(_block_sums(rms ** 2, 1000, 400)[:13], 400, 1000) == 0   # 4 stages: too few
    monkeypatch.setenv("OFR_SIEVE_SAMPLE", "panels")       # the prefix tier has the row sample only
    assert F.choose_prefix(_block_sums(rms ** 2, 1000, d), d, 1000) == 0
    monkeypatch.delenv("OFR_SIEVE_SAMPLE")
    monkeypatch.setenv("OFR_F6_PREFIX", "3")
    assert F.choose_prefix(_block_sums(np.full(nb, 130.0), 1000, d), d, 1000) == 3
    monkeypatch.setenv("OFR_F6_PREFIX", "0")
    assert F.choose_prefix(_block_sums(rms ** 2, 1000, d), d, 1000) == 0


def test_results_batch_equals_per_row_reference_vote():
    """classifier.results (the batched classifier.py:113-129): the vectorised vote equals the
    reference's per-query vote (most frequent label, ties -> smallest), ragged rows keep the loop."""
    import numpy as np
    from opencv_facerecognizer_amd.facerec.classifier import results, vote
    r = np.random.default_rng(4)
    y = r.integers(0, 5, 300)
    for k in (1, 2, 3, 8, 16):
        i_all = r.integers(0, 300, (200, k))
        d_all = np.sort(r.random((200, k)), axis=1)
        out = results(d_all, i_all, y)
        for o, idx, dist in zip(out, i_all, d_all):
            ref = max(dict((key, val) for key, val in enumerate(np.bincount(y[idx])) if val).items(),
                      key=lambda kv: kv[1])[0]                      # classifier.py:121-123
            assert o[0] == ref == vote(y[idx])
            assert np.array_equal(o[1]["labels"], y[idx]) and np.array_equal(o[1]["distances"], dist)
    i_all = np.array([[3, -1], [5, 7]])
    out = results(np.ones((2, 2)), i_all, y)
    assert np.array_equal(out[0][1]["labels"], y[[3]]) and len(out[0][1]["distances"]) == 1
