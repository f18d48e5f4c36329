"""Constant tables: product derivation == independent oracle derivation == generated header."""

import importlib.util
from pathlib import Path

import numpy as np

from oracle import numpy_slam as O
from thor_slam_amd import features as F

ROOT = Path(__file__).resolve().parents[1]


def test_brief_pattern_matches_oracle():
    np.testing.assert_array_equal(F.brief_pattern(), O.make_brief_pattern())
    np.testing.assert_array_equal(F.rotated_brief_table(), O.BRIEF_TABLE)


def test_pattern_geometry():
    pat = F.brief_pattern()
    assert pat.shape == (256, 4) and np.abs(pat).max() <= 13
    assert not np.any((pat[:, 0] == pat[:, 2]) & (pat[:, 1] == pat[:, 3]))
    tab = F.rotated_brief_table()
    assert np.abs(tab).max() <= 18  # stays inside the 19-px edge margin
    np.testing.assert_array_equal(tab[0], pat)  # bin 0 is the unrotated pattern


def test_wedges_and_disc():
    np.testing.assert_array_equal(F.wedge_table(), O.WEDGES)
    disc = F.orient_disc()
    np.testing.assert_array_equal(disc, O.DISC.astype(np.int32))
    umax = F.orient_half_widths()
    for dy in range(16):
        assert (disc[disc[:, 1] == dy][:, 0].max()) == umax[dy]


def test_generated_header_is_current():
    spec = importlib.util.spec_from_file_location("gen_tables", ROOT / "tools" / "gen_tables.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    header = (ROOT / "thor-slam_amd" / "csrc" / "tslam_tables.h").read_text()
    assert header == mod.render(), "run tools/gen_tables.py"
