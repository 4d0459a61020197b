"""The fused learner (fdr_fd_grad_fused: weights + gradient + in-launch chunk combine; the fused DSGD) against
the per-stage kernels it replaces and the oracle.  Tolerances: g rel-L2 1e-12 against the staged kernels (same
f64 arithmetic, summation order of the chunk combine identical), 1e-5 against the oracle (f32 sdot norms in the
reference); theta 1e-7 abs; centred ranks exact."""
import numpy as np
import pytest
import torch

from oracle import learner as olearn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fdr import engine
    return engine


def _case(n_dirs, P, seed=21, mean=1.0, ties=False):
    rs = np.random.RandomState(seed)
    table = rs.randn(max(1 << 22, P + 4096)).astype(np.float32)
    idx_dirs = rs.randint(0, table.size - P, size=n_dirs).astype(np.int64)
    idx = np.repeat(idx_dirs, 2)
    sign = np.tile(np.array([1, -1], np.int8), n_dirs)
    rew = rs.randn(2 * n_dirs) * 3 + mean
    if ties:
        rew = np.round(rew)
    s32 = np.float32(0.02)
    n2 = np.array([float(np.dot((table[i:i + P] * s32).astype(np.float64), (table[i:i + P] * s32).astype(np.float64)))
                   for i in idx])
    d = {k: torch.as_tensor(v, device="cuda") for k, v in
         dict(table=table, idx_dirs=idx_dirs, idx=idx, sign=sign, rew=rew, n2=n2).items()}
    return table, idx, sign, rew, d


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.mark.parametrize("n_dirs,P", [(2048, 6092), (512, 6092), (16, 5197), (64, 300_000)])
def test_fused_zscore_matches_staged_kernels_and_oracle(eng, n_dirs, P):
    table, idx, sign, rew, d = _case(n_dirs, P)
    coef = eng.fd_weights(d["rew"], 0.25, 0, d["sign"], d["n2"], 2, 0.02)
    g_staged = eng.fd_grad(d["table"], d["idx_dirs"], coef, P).cpu().numpy()
    outs = [eng.fd_grad_fused(d["table"], d["idx"], d["rew"], 0.25, 0, d["sign"], d["n2"], 2, 0.02, P).cpu().numpy()
            for _ in range(3)]   # repeated calls: the in-launch counters are left zero every time
    for g in outs:
        np.testing.assert_array_equal(g, outs[0])
    assert _rel(outs[0], g_staged) <= 1e-12
    if P <= 6092:
        g_ref, _ = olearn.fd_gradient(table, P, idx, sign, rew, 0.25, 0.02)
        assert _rel(outs[0], g_ref) <= 1e-5


def test_fused_sharded_slices_sum_to_unsharded(eng):
    """fdr_fd_grad_fused(lane_lo > 0) per rank slice (3 ranks) sums to the unsharded gradient."""
    from fdr import dist as fdist
    n_dirs, P = 512, 6092
    _, _, _, _, d = _case(n_dirs, P, seed=4)
    g_full = eng.fd_grad_fused(d["table"], d["idx"], d["rew"], 0.0, 0, d["sign"], d["n2"], 2, 0.02, P).cpu().numpy()
    g_sum = np.zeros(P)
    for r in range(3):
        lo, hi = fdist.lane_range(n_dirs, 2, 3, r)
        g_sum += eng.fd_grad_fused(d["table"], d["idx"][lo:hi].contiguous(), d["rew"], 0.0, lo,
                                   d["sign"][lo:hi].contiguous(), d["n2"][lo:hi].contiguous(), 2, 0.02, P).cpu().numpy()
    assert _rel(g_sum, g_full) <= 1e-12


@pytest.mark.parametrize("ties", [False, True])
def test_centred_rank_weights_and_gradient(eng, ties):
    n_dirs, P = 300, 4874
    table, idx, sign, rew, d = _case(n_dirs, P, seed=8, ties=ties)
    w = eng.rank_weights(d["rew"], 0, rew.size).cpu().numpy()
    np.testing.assert_array_equal(w, olearn.centred_ranks(rew))
    w_part = eng.rank_weights(d["rew"], 100, 50).cpu().numpy()
    np.testing.assert_array_equal(w_part, olearn.centred_ranks(rew)[100:150])
    g = eng.fd_grad_fused(d["table"], d["idx"], d["rew"], 0.0, 0, d["sign"], d["n2"], 2, 0.02, P,
                          mode="centred_rank").cpu().numpy()
    g_ref = olearn.fd_gradient_weights(table, P, idx, sign, olearn.centred_ranks(rew), 0.02)
    assert _rel(g, g_ref) <= 1e-5


@pytest.mark.parametrize("world,P,near_constant", [(1, 6092, False), (2, 6092, False), (3, 6092, False),
                                                   (2, 6092, True), (3, 200_000, False), (2, 200_000, True)])
def test_moments_one_collective_equals_zscore_path(eng, world, P, near_constant):
    """Per-rank moments [A | B | n_local | r' slots] summed (the all-reduce) -> DSGD from moments == the z-score
    gradient + DSGD (fused one-workgroup DSGD for P <= 65536, stats + multi-block path above).  near_constant:
    returns 500 +- 1e-12 (|m| / sd ~ 1e13), where a one-pass variance is rounding noise -- the slots give the
    two-pass statistics of standardize_arr, and the pair-shifted coefficients keep A free of cancellation."""
    from fdr import dist as fdist
    n_dirs = 512 if P <= 6092 else 64
    table, idx, sign, rew, d = _case(n_dirs, P, seed=6, mean=40.0)
    if near_constant:
        rew = 500.0 + np.random.RandomState(9).choice([-1e-12, 1e-12], rew.size)
        d["rew"] = torch.as_tensor(rew, device="cuda")
    theta0 = torch.as_tensor(np.random.RandomState(1).randn(P).astype(np.float32) * 0.1, device="cuda")
    g_z = eng.fd_grad_fused(d["table"], d["idx"], d["rew"], 0.5, 0, d["sign"], d["n2"], 2, 0.02, P)
    th_z = theta0.clone()
    out_z = eng.dsgd_step_ex(th_z, g_z, False, 0.01, 0.6).cpu().numpy()
    mom = torch.zeros(2 * P + 1 + rew.size, dtype=torch.float64, device="cuda")
    for r in range(world):
        lo, hi = fdist.lane_range(n_dirs, 2, world, r)
        mom += eng.fd_grad_fused(d["table"], d["idx"][lo:hi].contiguous(), d["rew"][lo:hi].contiguous(),
                                 0.5, lo, d["sign"][lo:hi].contiguous(), d["n2"][lo:hi].contiguous(), 2, 0.02, P,
                                 mode="moments", n_all=rew.size)
    assert mom[2 * P].item() == rew.size
    np.testing.assert_array_equal(mom[2 * P + 1:].cpu().numpy(), rew - 0.5)
    th_m = theta0.clone()
    g_m = torch.empty(P, dtype=torch.float64, device="cuda")
    out_m = eng.dsgd_step_ex(th_m, mom, True, 0.01, 0.6, g_out=g_m).cpu().numpy()
    assert _rel(g_m.cpu().numpy(), g_z.cpu().numpy()) <= (1e-12 if not near_constant else 1e-9)
    np.testing.assert_allclose(th_m.cpu().numpy(), th_z.cpu().numpy(), rtol=0, atol=1e-7)
    np.testing.assert_allclose(out_m, out_z, rtol=1e-6)
    if near_constant and P <= 6092:
        g_ref, _ = olearn.fd_gradient(table, P, idx, sign, rew, 0.5, 0.02)
        assert _rel(g_m.cpu().numpy(), g_ref) <= 1e-5


def test_fused_workspace_counters_rezeroed_when_prefix_grows(eng):
    """a fused call at small P leaves only ITS ticket-counter prefix at zero and writes slabs behind it;
    a later call at a larger P (more column blocks, n_chunks > 1) reusing the workspace must find its longer
    counter prefix zero, or a column block's owner never fires and g keeps stale values."""
    big_dirs, big_P = 2048, 40_000           # 157 column blocks -> 768 B counter prefix, 6 row chunks
    _, _, _, _, d = _case(big_dirs, big_P, seed=31)
    _, _, _, _, ds = _case(64, 6092, seed=30)  # 24 column blocks -> 256 B prefix; gsq / DSGD partials behind it
    coef = eng.fd_weights(d["rew"], 0.0, 0, d["sign"], d["n2"], 2, 0.02)
    g_staged = eng.fd_grad(d["table"], d["idx"][::2].contiguous(), coef, big_P).cpu().numpy()

    def big():
        return eng.fd_grad_fused(d["table"], d["idx"], d["rew"], 0.0, 0, d["sign"], d["n2"], 2, 0.02,
                                 big_P).cpu().numpy()

    assert _rel(big(), g_staged) <= 1e-12     # sizes the shared workspace for the big call
    theta = torch.zeros(6092, dtype=torch.float32, device="cuda")
    eng.fd_step(ds["table"], ds["idx"], ds["rew"], 0.0, ds["sign"], ds["n2"], 2, 0.02, theta, 0.01, 1.0)
    torch.cuda.synchronize()                  # the small step wrote its gsq / partials into bytes 256..704
    assert _rel(big(), g_staged) <= 1e-12


@pytest.mark.parametrize("P", [6092, 200_000])
def test_fused_dsgd_matches_staged_and_oracle(eng, P):
    rs = np.random.RandomState(P)
    theta = rs.randn(P).astype(np.float32) * 0.1
    g = rs.randn(P)
    t1 = torch.as_tensor(theta, device="cuda")
    out = eng.dsgd_step_ex(t1, torch.as_tensor(g, device="cuda"), False, 0.01, 0.23).cpu().numpy()
    ref, upd = olearn.dsgd_step(theta, g, 0.01)
    np.testing.assert_allclose(t1.cpu().numpy(), ref, rtol=0, atol=1e-6)
    assert abs(out[0] - upd) <= 1e-5 * upd


@pytest.mark.parametrize("mode", ["zscore", "centred_rank"])
def test_fd_step_matches_staged(eng, mode):
    """fdr_fd_step (weights + gradient in one launch, DSGD + history copy in a second) == fdr_fd_grad_fused +
    fdr_dsgd_step; repeated calls (the in-launch tickets are left zero); theta within 1e-7, norms equal."""
    n_dirs, P = 2048, 6092
    _, _, _, _, d = _case(n_dirs, P, seed=12)
    theta0 = torch.as_tensor(np.random.RandomState(2).randn(P).astype(np.float32) * 0.1, device="cuda")
    th_a, th_b = theta0.clone(), theta0.clone()
    for _ in range(3):
        g = eng.fd_grad_fused(d["table"], d["idx"], d["rew"], 0.3, 0, d["sign"], d["n2"], 2, 0.02, P, mode=mode)
        out_a = eng.dsgd_step_ex(th_a, g, False, 0.01, 0.5).cpu().numpy()
        g_b = torch.empty(P, dtype=torch.float64, device="cuda")
        hist = torch.zeros(P, dtype=torch.float32, device="cuda")
        out_b = eng.fd_step(d["table"], d["idx"], d["rew"], 0.3, d["sign"], d["n2"], 2, 0.02, th_b, 0.01, 0.5,
                            mode=mode, g=g_b, theta_hist=hist).cpu().numpy()
        np.testing.assert_array_equal(g_b.cpu().numpy(), g.cpu().numpy())
        np.testing.assert_array_equal(hist.cpu().numpy(), th_b.cpu().numpy())
        np.testing.assert_allclose(th_b.cpu().numpy(), th_a.cpu().numpy(), rtol=0, atol=1e-7)
        np.testing.assert_allclose(out_b, out_a, rtol=1e-6)
