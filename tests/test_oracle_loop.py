"""Pose-graph + loop-closure oracle (oracle/numpy_loop.py) against
independent definitions: SE(3) exp/log round trips, the edge Jacobians against central
differences, Gauss-Newton recovering an exactly-measured graph, gauge fixing, and the
signature vote on constructed descriptor sets."""

from __future__ import annotations

import numpy as np
import pytest

from oracle import numpy_loop as L


def _random_graph(rng, N, loops, noise_meas=0.0, noise_init=0.01):
    gt = [np.eye(4)]
    for _ in range(1, N):
        gt.append(gt[-1] @ L.se3_exp(np.r_[rng.normal(0, 0.1, 3), rng.normal(0, 0.05, 3)]))
    gt = np.array(gt)
    edges = [(i, i + 1) for i in range(N - 1)] + list(loops)
    Z = np.array([L.inv_se3(gt[i]) @ gt[j] @ L.se3_exp(np.r_[rng.normal(0, noise_meas, 3), rng.normal(0, noise_meas, 3)])
                  for i, j in edges])
    T0 = [np.eye(4)]
    for k in range(N - 1):
        T0.append(T0[-1] @ Z[k] @ L.se3_exp(np.r_[rng.normal(0, noise_init, 3), rng.normal(0, noise_init, 3)]))
    info = np.array([L.loop_information(0.01, 0.005)] * len(edges))
    return gt, np.array(T0), np.array(edges), Z, info


def test_se3_exp_log_round_trip():
    rng = np.random.default_rng(1)
    for scale in (1e-9, 1e-4, 0.3, 0.8):   # |phi| < pi
        for _ in range(20):
            xi = rng.normal(0, scale, 6)
            assert np.abs(L.se3_log(L.se3_exp(xi)) - xi).max() < 1e-12 * np.abs(xi).max()
    T = L.se3_exp(np.r_[0.1, -0.2, 0.3, 0.2, -0.1, 0.05])
    assert np.abs(T[:3, :3] @ T[:3, :3].T - np.eye(3)).max() < 1e-15


def test_adjoint_identity():
    rng = np.random.default_rng(2)
    T = L.se3_exp(rng.normal(0, 0.5, 6))
    d = rng.normal(0, 1e-3, 6)
    lhs = T @ L.se3_exp(d) @ L.inv_se3(T)
    rhs = L.se3_exp(L.adjoint(T) @ d)
    assert np.abs(lhs - rhs).max() < 1e-12


def test_edge_jacobians_match_central_differences():
    rng = np.random.default_rng(3)
    Ti, Tj = L.se3_exp(rng.normal(0, 0.5, 6)), L.se3_exp(rng.normal(0, 0.5, 6))
    Z = L.inv_se3(Ti) @ Tj @ L.se3_exp(rng.normal(0, 1e-3, 6))   # small residual
    e, Ji, Jj = L.edge_terms(Ti, Tj, Z)
    h = 1e-6
    for which, J in ((0, Ji), (1, Jj)):
        num = np.zeros((6, 6))
        for a in range(6):
            d = np.zeros(6)
            d[a] = h
            if which == 0:
                num[:, a] = (L.edge_terms(Ti @ L.se3_exp(d), Tj, Z)[0] - L.edge_terms(Ti @ L.se3_exp(-d), Tj, Z)[0]) / (2 * h)
            else:
                num[:, a] = (L.edge_terms(Ti, Tj @ L.se3_exp(d), Z)[0] - L.edge_terms(Ti, Tj @ L.se3_exp(-d), Z)[0]) / (2 * h)
        # Jr^-1 ~ I + ad/2 is second-order accurate in the residual
        assert np.abs(num - J).max() < 1e-5


def test_gauss_newton_recovers_exact_graph_and_fixes_the_gauge():
    rng = np.random.default_rng(4)
    gt, T0, edges, Z, info = _random_graph(rng, 25, [(0, 24), (5, 17)], noise_meas=0.0, noise_init=0.02)
    res = L.optimize(T0, edges, Z, info, 8)
    assert res["cost"] < 1e-16
    assert np.abs(res["T"] - gt).max() < 1e-9
    np.testing.assert_array_equal(res["T"][0], T0[0])


def test_loop_edge_pulls_drift_back():
    rng = np.random.default_rng(5)
    gt, T0, edges, Z, info = _random_graph(rng, 40, [(0, 39)], noise_meas=0.002, noise_init=0.0)
    # odometry-only initial guess has drifted; the loop edge reduces the end-point error
    chain = [np.eye(4)]
    for k in range(39):
        chain.append(chain[-1] @ Z[k])
    chain = np.array(chain)
    res = L.optimize(chain, edges, Z, info, 8)
    before = np.linalg.norm(chain[-1][:3, 3] - gt[-1][:3, 3])
    after = np.linalg.norm(res["T"][-1][:3, 3] - gt[-1][:3, 3])
    assert after < before
    assert res["steps"][-1] < 1e-9


def test_signature_votes():
    rng = np.random.default_rng(6)
    a = rng.integers(0, 2**32, size=(300, 8), dtype=np.uint32)
    b = rng.integers(0, 2**32, size=(300, 8), dtype=np.uint32)
    assert L.vote(a, a, 256, 64, 80) == 256         # every descriptor finds itself (distance 0)
    assert L.vote(a, b, 256, 64, 80) == 0           # random 256-bit strings sit ~128 bits apart
    flip = a.copy()
    flip[:, 0] ^= np.uint32(0xF)                    # 4 bits off: still the best, well under the ratio
    assert L.vote(flip, a, 256, 64, 80) == 256
    assert L.vote(a[:0], a, 256, 64, 80) == 0 and L.vote(a, a[:1], 256, 64, 80) == 1
    assert L.best_candidate(np.array([3, 9, 9, 2]), 4, 5) == 1 and L.best_candidate(np.array([3, 4]), 2, 5) == -1


@pytest.mark.parametrize("n", [1, 2])
def test_tiny_graphs(n):
    T = np.array([np.eye(4)] * n)
    edges = np.array([(0, 1)]) if n == 2 else np.zeros((0, 2), dtype=int)
    Z = np.array([L.se3_exp(np.r_[0.1, 0, 0, 0, 0, 0.1])]) if n == 2 else np.zeros((0, 4, 4))
    info = np.array([np.eye(6)] * len(edges))
    res = L.optimize(T, edges, Z, info, 3)
    if n == 2:
        assert np.abs(res["T"][1] - Z[0]).max() < 1e-12
