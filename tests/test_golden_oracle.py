"""The oracle reproduces its committed golden digests (tests/golden/make_oracle_golden.py)."""

import json
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).parent / "golden"))
from make_oracle_golden import N, record  # noqa: E402

from helpers import scenario  # noqa: E402

GOLD = json.loads((Path(__file__).parent / "golden" / "oracle_digest.json").read_text())


@pytest.mark.parametrize("key,kwargs", [("seed0", dict(seed=0, n=N)), ("seed0_distorted", dict(seed=0, n=2, distorted=True))])
def test_oracle_matches_golden(key, kwargs):
    got = record(scenario(**kwargs))
    want = GOLD[key]
    assert got["frames"] == want["frames"], "synthetic renderer drifted"
    for i, (g, w) in enumerate(zip(got["per_frame"], want["per_frame"])):
        for k, v in w.items():
            if k == "T":
                np.testing.assert_allclose(np.array(g[k]), np.array(v), rtol=0, atol=1e-12, err_msg=f"frame {i} {k}")
            else:
                assert g[k] == v, f"frame {i}: {k}"
