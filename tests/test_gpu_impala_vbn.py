"""GPU: ImpalaPolicy.compute_vbn (policies/impala.py:12-16) on the device (fdr_impala_bn_refresh) against the
reference's own compute_vbn (G14: tests/golden/g14_impala_vbn.npz) and the oracle's restatement.

The reference's pass is train mode over the stacked buffer (B = n, T = 1): every BatchNorm normalises with its
batch statistics and folds them into its running stats, and the batch_first LSTM reads the n obs as ONE sequence
from the carried state (zeroed iff the first obs is done), leaving its end state.  Tolerance: running stats
<= 1e-5 relative (+ 1e-6 absolute for entries near zero); the LSTM state, which sits after 15 convs, the fc and the
recurrence (f32, summed in another order than torch's CPU kernels), <= 2e-5 absolute + 1e-4 relative."""
import numpy as np
import pytest
import torch

from oracle import impala as oi

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-5, 1e-6
STATE_RTOL, STATE_ATOL = 1e-4, 2e-5


def _policy(A, flat, rm, rv, h0, c0):
    from policies import ImpalaPolicy
    pol = ImpalaPolicy((64, 64, 3), A, seed=124)
    pol.set_trainable_flat(flat)
    o = 0
    for m in pol.model.bn_layers():
        n = m.num_features
        m.running_mean.copy_(torch.as_tensor(rm[o:o + n]))
        m.running_var.copy_(torch.as_tensor(rv[o:o + n]))
        o += n
    dev = pol.flat.device
    pol.state = (torch.as_tensor(h0).view(1, 256).to(dev), torch.as_tensor(c0).view(1, 256).to(dev))
    return pol


def _buffer(frames, rewards, dones):
    return [{"frame": torch.as_tensor(frames[i].astype(np.float32)).view(1, 1, 3, 64, 64),
             "reward": torch.as_tensor(rewards[i]).view(1, 1),
             "done": torch.as_tensor(bool(dones[i])).view(1, 1)} for i in range(len(frames))]


def _stats(pol):
    bns = pol.model.bn_layers()
    return (torch.cat([m.running_mean for m in bns]).cpu().numpy(), torch.cat([m.running_var for m in bns]).cpu().numpy(),
            pol.state[0].reshape(-1).cpu().numpy(), pol.state[1].reshape(-1).cpu().numpy())


def _check(got, g, tag):
    rm, rv, h, c = got
    for name, a in (("rm", rm), ("rv", rv)):
        np.testing.assert_allclose(a, g[tag + "_" + name], rtol=RTOL, atol=ATOL, err_msg="%s %s" % (tag, name))
    for name, a in (("h", h), ("c", c)):
        np.testing.assert_allclose(a, g[tag + "_" + name], rtol=STATE_RTOL, atol=STATE_ATOL, err_msg="%s %s" % (tag, name))


def test_compute_vbn_matches_reference_golden(golden):
    """G14 cases a (carried state), b (first obs done), a2 (two chained calls): every BN's running stats and the
    policy's LSTM state after the call; num_batches_tracked counts the calls; the policy is left in eval mode."""
    g = golden("g14_impala_vbn.npz")
    A, P = int(g["A"]), int(g["P"])
    tab = np.random.RandomState(int(g["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(g["param_offset"])
    flat = (tab[off:off + P] * np.float32(0.1)).astype(np.float32)
    for tag in ("a", "b"):
        pol = _policy(A, flat, g["rm"], g["rv"], g["h0"], g["c0"])
        buf = _buffer(g["frames"], g["rewards"], g[tag + "_dones"])
        pol.compute_vbn(buf)
        torch.cuda.synchronize()
        assert not pol.training
        _check(_stats(pol), g, tag)
        if tag == "a":
            pol.compute_vbn(np.asarray(buf, dtype=object))     # run_sequential.py:212 hands an object array
            _check(_stats(pol), g, "a2")
            assert all(int(m.num_batches_tracked) == 2 for m in pol.model.bn_layers())
    # the kernels read the refreshed stats: an eval-mode forward after compute_vbn uses them
    bm, bv = pol.bn_stats()
    np.testing.assert_allclose(bm.cpu().numpy(), g["b_rm"], rtol=RTOL, atol=ATOL)


def test_compute_vbn_matches_oracle_larger_buffer():
    """n = 70 obs (not a multiple of the kernels' 8-row / 64-block splits), random params at a larger scale (more
    ReLU zeros), a nonzero reward column and a carried state; vs oracle.compute_vbn (the restatement pinned by G14
    in tests/test_oracle_impala.py)."""
    A, n = 5, 70
    rs = np.random.RandomState(21)
    P = oi.num_params(A)
    flat = (0.15 * rs.randn(P)).astype(np.float32)
    nbn = oi.num_bn()
    rm = (0.1 * rs.randn(nbn)).astype(np.float32)
    rv = (1.0 + rs.rand(nbn)).astype(np.float32)
    frames = rs.randint(0, 256, size=(n, 3, 64, 64)).astype(np.uint8)
    rewards = rs.choice([-3.0, -1.0, 0.0, 0.5, 2.0], size=n).astype(np.float32)
    h0 = (0.3 * rs.randn(256)).astype(np.float32)
    c0 = (0.3 * rs.randn(256)).astype(np.float32)
    pol = _policy(A, flat, rm, rv, h0, c0)
    pol.compute_vbn(_buffer(frames, rewards, np.zeros(n, bool)))
    got = _stats(pol)
    want = oi.compute_vbn(oi.unflatten(flat, A), rm, rv, frames.astype(np.float32), rewards, False, h0, c0, 0.1)
    for a, b, name in zip(got, want, ("rm", "rv", "h", "c")):
        np.testing.assert_allclose(a, b, rtol=RTOL if name[0] == "r" else STATE_RTOL, atol=ATOL if name[0] == "r" else STATE_ATOL,
                                   err_msg=name)


def test_compute_vbn_rejects_a_single_obs():
    """torch's train-mode BatchNorm1d raises for one value per channel; the device call refuses n < 2."""
    from fdr import engine
    A = 4
    pol = _policy(A, np.zeros(oi.num_params(A), np.float32), np.zeros(oi.num_bn(), np.float32),
                  np.ones(oi.num_bn(), np.float32), np.zeros(256, np.float32), np.zeros(256, np.float32))
    with pytest.raises(ValueError):
        pol.compute_vbn(_buffer(np.zeros((1, 3, 64, 64), np.uint8), np.zeros(1, np.float32), np.zeros(1, bool)))
    bm, bv = pol.bn_stats()
    fr = torch.zeros(1, 3, 64, 64, device=bm.device)
    from fdr._lib import FDRError
    with pytest.raises(FDRError, match="n >= 2"):
        d = pol.spec.desc(None, None)
        import ctypes
        ws = torch.empty(1 << 20, dtype=torch.uint8, device=bm.device)
        engine.check(engine.lib.fdr_impala_bn_refresh(None, ctypes.byref(d), engine._p(pol.flat), 1, engine._p(fr), None,
                                                      0, None, None, 0.1, engine._p(bm), engine._p(bv), engine._p(ws),
                                                      ws.numel(), None), "fdr_impala_bn_refresh")
