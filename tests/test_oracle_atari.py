"""CPU: the AtariPolicy restatement (oracle/atari.py) pinned to the reference (G11, policies/atari.py)."""
import hashlib

import numpy as np
import pytest

from oracle import atari as oa


@pytest.fixture(scope="module")
def g11(golden):
    return golden("g11_atari.npz")


def test_layout_and_init_match_reference(g11):
    A = int(g11["A"])
    assert oa.num_params(A) == int(g11["P"])
    assert [str(tuple(s)) for _, s in oa.layout(A)] == list(g11["param_shapes"])
    theta = oa.init_theta(A, 124)
    assert hashlib.sha256(np.ascontiguousarray(theta).tobytes()).hexdigest() == str(g11["init_sha"])
    np.testing.assert_array_equal(theta[:64], g11["init_head"])


def test_forward_matches_reference(g11):
    A = int(g11["A"])
    p = oa.unflatten(oa.init_theta(A, 124), A)
    bn = oa.split_bn(g11["rm"], g11["rv"])
    probs, feat = oa.forward(p, bn, g11["frames"].astype(np.float32))
    np.testing.assert_allclose(feat.numpy(), g11["feat"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(probs.numpy(), g11["probs"], rtol=1e-6, atol=1e-7)


def test_synthetic_stacked_frames():
    f = oa.frames(3, [0, 1], 0)
    assert f.shape == (2, 4, 84, 84) and f.dtype == np.uint8
    assert not np.array_equal(f[0], f[1])
    assert np.array_equal(oa.frames(3, [1], 0)[0], f[1])


def test_compute_vbn_matches_reference(golden):
    """oracle.atari.compute_vbn == the reference's AtariPolicy.compute_vbn (G16): every BN's running stats after one
    train-mode pass of the VBN buffer and after a second (chained) pass."""
    g = golden("g16_atari_vbn.npz")
    A, P = int(g["A"]), int(g["P"])
    assert P == oa.num_params(A)
    flat = (np.random.RandomState(int(g["param_seed"])).randn(P) * float(g["param_scale"])).astype(np.float32)
    p = oa.unflatten(flat, A)
    rm, rv = g["rm"], g["rv"]
    for tag in ("a", "a2"):
        rm, rv = oa.compute_vbn(p, rm, rv, g["frames"].astype(np.float32), float(g["momentum"]))
        np.testing.assert_allclose(rm, g[tag + "_rm"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(rv, g[tag + "_rv"], rtol=1e-5, atol=1e-6)
