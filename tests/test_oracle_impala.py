"""CPU: the ImpalaCNN restatement (oracle/impala.py) pinned to the reference's own outputs (G3-impala)
and the synthetic frame env's definition; the ABI's Impala layout queries (no GPU needed)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import impala as oi


@pytest.fixture(scope="module")
def g8(golden):
    return golden("g8_impala.npz")


@pytest.fixture(scope="module")
def net(g8):
    A, P = int(g8["A"]), int(g8["P"])
    table = np.random.RandomState(int(g8["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(g8["param_offset"])
    flat = (table[off:off + P] * np.float32(0.1)).astype(np.float32)
    return oi.unflatten(flat, A), oi.split_bn(g8["rm"], g8["rv"])


def test_layout_is_the_reference_parameter_order(g8):
    A = int(g8["A"])
    assert oi.num_params(A) == int(g8["P"])
    assert [str(tuple(s)) for _, s in oi.layout(A)] == list(g8["param_shapes"])
    assert oi.num_bn() == len(g8["rm"])


def test_forward_matches_reference_sequences(g8, net):
    """policies/impala.py forward, B=1 sequences with a done reset in the middle of the 2nd."""
    p, bn = net
    for q in range(g8["frames"].shape[0]):
        h, c = torch.zeros(1, 256), torch.zeros(1, 256)
        for t in range(g8["frames"].shape[1]):
            nd = [0.0 if g8["dones"][q, t] else 1.0]
            probs, h, c, feat, _ = oi.forward(p, bn, g8["frames"][q, t][None].astype(np.float32),
                                              g8["rewards"][q, t:t + 1], h, c, notdone=nd)
            np.testing.assert_allclose(feat.numpy()[0], g8["feat"][q, t], atol=1e-6)
            np.testing.assert_allclose(h.numpy()[0], g8["h"][q, t], atol=1e-6)
            np.testing.assert_allclose(c.numpy()[0], g8["c"][q, t], atol=1e-6)
            np.testing.assert_allclose(probs.numpy()[0], g8["probs"][q, t], atol=1e-7)


def test_entropy_pass_is_a_sequence_from_the_final_state(g8, net):
    """worker/agent.py:66 -> ImpalaPolicy.get_entropy: the batch of visited obs is one LSTM sequence
    (batch_first) starting at the end-of-episode state -- not T independent steps."""
    p, bn = net
    for q in range(g8["frames"].shape[0]):
        h, c = torch.zeros(1, 256), torch.zeros(1, 256)
        cis = []
        for t in range(g8["frames"].shape[1]):
            nd = [0.0 if g8["dones"][q, t] else 1.0]
            _, h, c, _, ci = oi.forward(p, bn, g8["frames"][q, t][None].astype(np.float32),
                                        g8["rewards"][q, t:t + 1], h, c, notdone=nd)
            cis.append(ci)
        for t in range(len(cis)):
            pe, h, c = oi.lstm_head(p, bn, cis[t], h, c)
            np.testing.assert_allclose(pe.numpy()[0], g8["ent_probs"][q, t], atol=1e-7)


def test_synthetic_frames_and_rewards():
    f0 = oi.frames(3, [0, 1, 2], 0)
    assert f0.shape == (3, 3, 64, 64) and f0.dtype == np.uint8
    assert not np.array_equal(f0[0], f0[1])
    assert np.array_equal(oi.frames(3, [1], 0)[0], f0[1])          # per-env, order-free
    assert not np.array_equal(oi.frames(3, [0], 1)[0], f0[0])       # changes with t
    assert abs(f0.astype(np.float64).mean() - 127.5) < 3.0
    tg = oi.targets(3, np.arange(1000), 5, 6)
    assert set(np.unique(tg)) == set(range(6))
    r = oi.rewards(3, np.arange(1000), 5, tg, 6)
    assert np.all(r == 1.0)
    r = oi.rewards(3, np.arange(1000), 5, (tg + 1) % 6, 6)
    assert np.all(r == -1.0)


def test_abi_impala_layout_queries():
    from fdr import _lib
    assert _lib.lib.fdr_impala_num_params(6) == oi.num_params(6)
    assert _lib.lib.fdr_impala_num_params(15) == oi.num_params(15)
    assert _lib.lib.fdr_impala_num_params(0) == -1
    assert _lib.lib.fdr_impala_num_bn_stats() == oi.num_bn()
    d = _lib.ImpalaDesc(6, 4, 1000, 1, 0, oi.num_params(6), None, None, 0)
    nb = _lib.lib.fdr_impala_workspace_bytes(ctypes.byref(d), 1024)
    assert nb > 1024 * oi.num_params(6) * 4                       # the theta' packs at least
    d16 = _lib.ImpalaDesc(6, 4, 1000, 1, 0, oi.num_params(6), None, None, 1)
    assert _lib.lib.fdr_impala_workspace_bytes(ctypes.byref(d16), 1024) > nb + 1024 * oi.num_params(6) * 2 * 0.9
    bad = _lib.ImpalaDesc(6, 3, 10, 0, 0, oi.num_params(6), None, None, 0)   # E = 3 unsupported
    ld = _lib.LanesDesc(1, 0, None, 0, None, None, 0.0, None, 0)
    rc = _lib.lib.fdr_impala_rollout(None, ctypes.byref(bad), ctypes.byref(ld), 1, 0, 0, 1, 1, 1, None, None,
                                     None, 1, 1 << 40, None)
    assert rc == _lib.FDR_ERR_UNSUPPORTED


def test_strategy_sequence_matches_reference_entropy_pass(g8):
    """oracle.strategy (get_strategy's one-sequence form) == the reference's stacked-obs pass (G8 ent_probs)."""
    A, P = int(g8["A"]), int(g8["P"])
    tab = np.random.RandomState(int(g8["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(g8["param_offset"])
    p = oi.unflatten((tab[off:off + P] * np.float32(0.1)).astype(np.float32), A)
    bn = oi.split_bn(g8["rm"], g8["rv"])
    for q in range(g8["frames"].shape[0]):
        h, c = torch.zeros(1, oi.HID), torch.zeros(1, oi.HID)
        for t in range(g8["frames"].shape[1]):
            _, h, c, _, _ = oi.forward(p, bn, g8["frames"][q, t:t + 1].astype(np.float32), g8["rewards"][q, t:t + 1],
                                       h, c, notdone=[0.0 if g8["dones"][q, t] else 1.0])
        pr, _, _ = oi.strategy(p, bn, g8["frames"][q].astype(np.float32), g8["rewards"][q], h, c)
        np.testing.assert_allclose(pr, g8["ent_probs"][q], atol=1e-6)


def test_compute_vbn_matches_reference(golden):
    """oracle.compute_vbn == the reference's ImpalaPolicy.compute_vbn (G14): every BN's running stats and the
    carried LSTM state after a train-mode pass of the VBN buffer, for a carried state (a), a first-obs done (b)
    and two chained calls (a2)."""
    g = golden("g14_impala_vbn.npz")
    A, P = int(g["A"]), int(g["P"])
    tab = np.random.RandomState(int(g["table_seed"])).randn(2 ** 22).astype(np.float32)
    off = int(g["param_offset"])
    p = oi.unflatten((tab[off:off + P] * np.float32(0.1)).astype(np.float32), A)
    fr = g["frames"].astype(np.float32)
    mom = float(g["momentum"])
    runs = {}
    for tag in ("a", "b"):
        runs[tag] = oi.compute_vbn(p, g["rm"], g["rv"], fr, g["rewards"], bool(g[tag + "_dones"][0]), g["h0"], g["c0"], mom)
    rm, rv, h, c = runs["a"]
    runs["a2"] = oi.compute_vbn(p, rm, rv, fr, g["rewards"], False, h, c, mom)
    for tag, (rm, rv, h, c) in runs.items():
        np.testing.assert_allclose(rm, g[tag + "_rm"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rv, g[tag + "_rv"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(h, g[tag + "_h"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(c, g[tag + "_c"], rtol=1e-5, atol=1e-6)
    assert not np.allclose(runs["a"][2], runs["b"][2])   # the carried state matters
