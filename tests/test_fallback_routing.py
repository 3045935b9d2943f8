"""Host logic of the certified tier chain's routing (FloatGallery.fallback, _device.py): a query the
fp6 tier missed by need = d_k^2 - bound can only be certified by a tier whose dS is smaller by
more than need, so it skips the tiers without that room and every query is still answered by a
certifying tier or the exact fp32 pass.  The kernels are replaced by a model of the certificate
(no GPU): tier t certifies a row iff its fp6 miss m < dS_f6 - dS_t."""
import numpy as np
import torch

from opencv_facerecognizer_amd import _device

DS = {"f6": 1.0, 1: 0.5, 2: 0.01}
TAG = {1: 1000.0, 2: 2000.0, "fp32": 3000.0}


class _ModelGallery(_device.FloatGallery):
    """FloatGallery with the device stages replaced by the certificate model.  Query rows carry
    (row id, fp6 miss m) in their first two columns."""

    def __init__(self):      # no device state
        self.ran = []

    def _tier_dS(self, tier, stats):
        return torch.full((stats.shape[0],), DS[tier], dtype=torch.float64)

    def quantize_queries(self, Qd, out=None, tier="f6"):
        B = Qd.shape[0]
        return dict(Qs=Qd, stats=torch.ones((B, 3), dtype=torch.float64), tier=tier, B=B,
                    cert=torch.zeros(B, dtype=torch.int32), bound=torch.zeros(B, dtype=torch.float64))

    def search_q8_phase(self, phases, Qd, qq, k, index_base=0, out=None, workspace=None):
        tier = qq["tier"]
        self.ran.append((tier, Qd[:, 0].long().tolist()))
        m = Qd[:, 1].double()
        room = DS["f6"] - DS[tier]
        qq["cert"] = (m < room).int()
        d = torch.full((Qd.shape[0], k), 1.0, dtype=torch.float64)
        qq["bound"] = 1.0 - (m - room)                 # need at this tier = m - room
        i = (Qd[:, 0].long() + int(TAG[tier]))[:, None].repeat(1, k)
        return d, i

    def _search_f32(self, Qd, k, index_base=0):
        self.ran.append(("fp32", Qd[:, 0].long().tolist()))
        d = torch.full((Qd.shape[0], k), 1.0, dtype=torch.float64)
        i = (Qd[:, 0].long() + int(TAG["fp32"]))[:, None].repeat(1, k)
        return d, i


def _batch(ms):
    B = len(ms)
    Qd = torch.zeros((B, 32), dtype=torch.float32)
    Qd[:, 0] = torch.arange(B, dtype=torch.float32)
    Qd[:, 1] = torch.tensor(ms, dtype=torch.float32)
    m = torch.tensor(ms, dtype=torch.float64)
    qq = dict(tier="f6", cert=(m <= 0).int(), bound=1.0 - m, stats=torch.ones((B, 3), dtype=torch.float64))
    out = (torch.ones((B, 1), dtype=torch.float64), torch.arange(B, dtype=torch.int64)[:, None].clone())
    return Qd, qq, out


def test_routing_skips_tiers_without_room():
    # 40 rows per class (> SMALL_BATCH, so the int8 tiers are in play): certified by fp6 (m <= 0),
    # by int8 x1 (m < 0.45 = 0.9 of its room), by int8 x2 only (m in [0.45, 0.891)), by fp32 only
    ms = [0.0] * 40 + [0.2] * 40 + [0.7] * 40 + [5.0] * 40
    g = _ModelGallery()
    Qd, qq, out = _batch(ms)
    first = g.fallback(Qd, qq, 1, out)
    assert first == 120
    ran = {t: set(r) for t, r in g.ran}
    assert ran[1] == set(range(40, 80))                  # only the rows with room run int8 x1
    assert ran[2] == set(range(80, 120))                 # the rest of the hopeful rows skip to x2
    assert ran["fp32"] == set(range(120, 160))           # no quantized tier has room for these
    idx = out[1][:, 0].numpy()
    assert np.array_equal(idx[:40], np.arange(40))       # fp6 answers untouched
    assert np.array_equal(idx[40:80], np.arange(40, 80) + 1000)
    assert np.array_equal(idx[80:120], np.arange(80, 120) + 2000)
    assert np.array_equal(idx[120:], np.arange(120, 160) + 3000)
    assert g.last_fallbacks == (120, 80, 40)


def test_routing_hopeless_everywhere_goes_to_fp32():
    ms = [9.0] * 50
    g = _ModelGallery()
    Qd, qq, out = _batch(ms)
    g.fallback(Qd, qq, 1, out)
    assert [t for t, _ in g.ran] == ["fp32"]
    assert np.array_equal(out[1][:, 0].numpy(), np.arange(50) + 3000)
    assert g.last_fallbacks == (50, 50, 50)


def test_routing_overflow_bound_goes_to_fp32():
    """An overflowed sieve bucket reports bound -inf: need = +inf, no tier has room."""
    g = _ModelGallery()
    Qd, qq, out = _batch([0.2] * 40)
    qq["bound"][:5] = -float("inf")
    g.fallback(Qd, qq, 1, out)
    ran = {t: set(r) for t, r in g.ran}
    assert ran[1] == set(range(5, 40)) and ran["fp32"] == set(range(5))
