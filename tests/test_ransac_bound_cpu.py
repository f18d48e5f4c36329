"""The bounded RANSAC scoring of k_ransac (csrc/k_pose.hip) modelled on the CPU: whatever order the
waves take their poses in, dropping a pose once (count + unscanned + 1) << 12 | tag falls below the
block's best key, the grouped pre-tests on a wave's own outlier list and the "list good enough"
rule leave the winning key equal to the exhaustive one (oracle/numpy_slam.py estimate_pose: argmax
of the counts, first maximum = lowest pose index).  The GPU kernel itself is checked against the
oracle in tests/test_gpu_parity.py; this pins the argument on many random inlier patterns (shared
outliers, ties, invalid poses) that a handful of rendered frames cannot cover."""

from __future__ import annotations

import numpy as np
import pytest

WAVES, GROUP, CHUNK, UNROLL = 4, 8, 64, 4


def exhaustive_key(inl: np.ndarray, valid: np.ndarray) -> int:
    best = 0
    for p in range(inl.shape[0]):
        tag = 4095 - p
        key = ((int(inl[p].sum()) + 1) << 12 | tag) if valid[p] else tag
        best = max(best, key)
    return best


def bounded_key(inl: np.ndarray, valid: np.ndarray, order_seed: int) -> int:
    """The kernel's per-wave loop, the waves interleaved one pose-step at a time in a random order
    (the hardware's interleaving is arbitrary; every one must give the same key)."""
    n_pose, n = inl.shape
    rng = np.random.default_rng(order_seed)
    best = 0
    state = []
    for w in range(WAVES):
        groups = [list(range(g0, min(n_pose, g0 + WAVES * GROUP), WAVES)) for g0 in range(w, n_pose, WAVES * GROUP)]
        state.append({"groups": groups, "my_key": 0, "my_out": [], "done": False})

    def run_group(st, group):
        nonlocal best
        g0 = group[0]
        bnd0 = best
        if (((n + 1) << 12) | (4095 - g0)) < bnd0:
            st["done"] = True
            return
        live = []
        for pk in group:
            if not valid[pk]:
                best = max(best, 4095 - pk)
                continue
            if st["my_key"]:
                miss = sum(1 for i in st["my_out"][:GROUP] if not inl[pk, i])
                if (((n - miss + 1) << 12) | (4095 - pk)) < bnd0:
                    continue
            live.append(pk)
        for pi in live:
            tag = 4095 - pi
            bnd = best   # snapshot per pose
            if (((n + 1) << 12) | tag) < bnd:
                st["done"] = True
                return
            list_ok = (st["my_key"] >> 12) + 2 >= (bnd >> 12)
            cnt, misses, dropped = 0, [], False
            for c0 in range(0, n, CHUNK * UNROLL):
                seg = inl[pi, c0:c0 + CHUNK * UNROLL]
                cnt += int(seg.sum())
                misses += [c0 + int(i) for i in np.nonzero(~seg)[0]]
                rest = max(0, n - (c0 + CHUNK * UNROLL))
                if list_ok and (((cnt + rest + 1) << 12) | tag) < bnd:
                    dropped = True
                    break
            if not dropped:
                key = ((cnt + 1) << 12) | tag
                best = max(best, key)
                if key > st["my_key"]:
                    st["my_key"], st["my_out"] = key, misses[:64]

    pending = [w for w in range(WAVES) if state[w]["groups"]]
    while pending:
        w = int(rng.choice(pending))
        st = state[w]
        run_group(st, st["groups"].pop(0))
        if st["done"] or not st["groups"]:
            pending.remove(w)
    return best


def random_case(rng, n_pose: int, n: int, outlier_rate: float):
    """Correct poses share the scene's outliers (plus a few near-threshold flips of their own);
    wrong roots match little; some poses have no solution."""
    outl = rng.random(n) < outlier_rate
    inl = np.zeros((n_pose, n), bool)
    good = rng.random(n_pose) < 0.4
    for p in range(n_pose):
        if good[p]:
            row = ~outl
            flips = rng.random(n) < 0.003
            inl[p] = row ^ flips
        else:
            inl[p] = rng.random(n) < rng.uniform(0.0, 0.2)
    valid = rng.random(n_pose) < 0.6
    return inl, valid


@pytest.mark.parametrize("outlier_rate", [0.0, 0.002, 0.05, 0.35])
def test_bounded_key_equals_exhaustive(outlier_rate):
    rng = np.random.default_rng(int(outlier_rate * 1000) + 7)
    for trial in range(12):
        n_pose = int(rng.choice([32, 128, 512]))
        n = int(rng.integers(6, 700))
        inl, valid = random_case(rng, n_pose, n, outlier_rate)
        want = exhaustive_key(inl, valid)
        for order_seed in range(3):
            assert bounded_key(inl, valid, order_seed) == want, (trial, order_seed)


def test_ties_resolve_to_the_lowest_pose_index():
    rng = np.random.default_rng(3)
    n = 300
    row = rng.random(n) < 0.9
    inl = np.tile(row, (64, 1))          # every pose has the same inlier set
    valid = np.ones(64, bool)
    valid[:5] = False
    want = exhaustive_key(inl, valid)
    assert 4095 - (want & 4095) == 5
    for order_seed in range(5):
        assert bounded_key(inl, valid, order_seed) == want


def test_no_valid_pose():
    inl = np.zeros((16, 50), bool)
    valid = np.zeros(16, bool)
    assert bounded_key(inl, valid, 0) == exhaustive_key(inl, valid) == 4095
