"""GPU: AtariPolicy.compute_vbn (policies/policy.py:31-34 on atari.py:36-51) on the device (fdr_atari_bn_refresh)
against the reference's own compute_vbn (G16: tests/golden/g16_atari_vbn.npz) and the oracle's restatement.

Train mode over the stacked buffer: each BatchNorm (2d(16), 2d(32), 1d(256)) normalises with its batch statistics and
folds them into its running stats (unbiased variance, momentum 0.1).  Tolerance: running stats <= 1e-5 relative,
plus an absolute floor of 1e-6 x the BN's scale for means that cancel to near zero (f32 conv sums of 256 / 2592
products, summed in another order than torch's CPU kernels)."""
import numpy as np
import pytest
import torch

from oracle import atari as oa

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _policy(A, flat, rm, rv):
    from policies import AtariPolicy
    pol = AtariPolicy((84, 84), A, seed=124, device=torch.device("cuda", 0))
    pol.set_trainable_flat(flat)
    bns = [m for m in pol.model if isinstance(m, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d))]
    o = 0
    for m in bns:
        n = m.num_features
        m.running_mean.copy_(torch.as_tensor(rm[o:o + n]))
        m.running_var.copy_(torch.as_tensor(rv[o:o + n]))
        o += n
    return pol, bns


def _check(pol, want_rm, want_rv, tag):
    bm, bv = pol.bn_stats()
    bm, bv = bm.cpu().numpy(), bv.cpu().numpy()
    for got, want, name in ((bm, want_rm, "rm"), (bv, want_rv, "rv")):
        for lo, hi in ((0, 16), (16, 48), (48, 304)):
            floor = 1e-6 * max(1.0, float(np.abs(want[lo:hi]).max()))
            np.testing.assert_allclose(got[lo:hi], want[lo:hi], rtol=RTOL, atol=floor,
                                       err_msg="%s %s [%d:%d]" % (tag, name, lo, hi))


def test_compute_vbn_matches_reference_golden(golden):
    """G16: one call (a) and a second call on the same buffer (a2); num_batches_tracked counts the calls; eval mode
    after; the eval-mode forward reads the refreshed statistics."""
    g = golden("g16_atari_vbn.npz")
    A, P = int(g["A"]), int(g["P"])
    flat = (np.random.RandomState(int(g["param_seed"])).randn(P) * float(g["param_scale"])).astype(np.float32)
    pol, bns = _policy(A, flat, g["rm"], g["rv"])
    frames = torch.as_tensor(g["frames"].astype(np.float32))
    for tag in ("a", "a2"):
        pol.compute_vbn(frames)
        torch.cuda.synchronize()
        assert not pol.training
        _check(pol, g[tag + "_rm"], g[tag + "_rv"], tag)
    assert all(int(m.num_batches_tracked) == 2 for m in bns)
    probs = pol.forward(frames).cpu().numpy()
    want, _ = oa.forward(oa.unflatten(flat, A), oa.split_bn(g["a2_rm"], g["a2_rv"]), g["frames"].astype(np.float32))
    np.testing.assert_allclose(probs, want.numpy(), rtol=1e-4, atol=1e-6)


def test_compute_vbn_matches_oracle_larger_buffer():
    """n = 37 frames (not a multiple of the fc kernel's 8-row blocks, fewer than the 64 statistic blocks), from a
    numpy array; vs oracle.atari.compute_vbn (pinned by G16 in tests/test_oracle_atari.py)."""
    A, n = 4, 37
    rs = np.random.RandomState(3)
    P = oa.num_params(A)
    flat = (0.03 * rs.randn(P)).astype(np.float32)
    rm = (rs.randn(304) * 5).astype(np.float32)
    rv = (1.0 + rs.rand(304) * 20).astype(np.float32)
    frames = rs.randint(0, 256, size=(n, 4, 84, 84)).astype(np.float32)
    pol, _ = _policy(A, flat, rm, rv)
    pol.compute_vbn(frames)
    want_rm, want_rv = oa.compute_vbn(oa.unflatten(flat, A), rm, rv, frames, 0.1)
    _check(pol, want_rm, want_rv, "n37")


def test_compute_vbn_rejects_a_single_frame():
    from fdr import engine
    A = 3
    pol, _ = _policy(A, np.zeros(oa.num_params(A), np.float32), np.zeros(304, np.float32), np.ones(304, np.float32))
    with pytest.raises(ValueError):
        pol.compute_vbn(np.zeros((1, 4, 84, 84), np.float32))
    bm, bv = pol.bn_stats()
    from fdr._lib import FDRError
    import ctypes
    d = pol.spec.desc(None, None)
    fr = torch.zeros(1, 4 * 84 * 84, device=bm.device)
    ws = torch.empty(1 << 22, dtype=torch.uint8, device=bm.device)
    with pytest.raises(FDRError, match="n >= 2"):
        engine.check(engine.lib.fdr_atari_bn_refresh(None, ctypes.byref(d), engine._p(pol.flat), 1, engine._p(fr), 0.1,
                                                     engine._p(bm), engine._p(bv), engine._p(ws), ws.numel(), None),
                     "fdr_atari_bn_refresh")
