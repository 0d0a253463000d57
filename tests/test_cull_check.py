"""The footprint-vs-block tests are conservative: neither the blends' edge form (hlgs_math.h foot_touches) nor
the key scatter's band form (splat_bands / row_quad_mask, whose masks travel in the tile-list entries) rejects a
block holding a pixel with alpha >= 1/255 (brute force in float64 over random splats; tools/cull_check.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import cull_check  # noqa: E402


def test_footprint_block_tests_are_conservative():
    r = cull_check.run(N=60000, seed=3)
    assert r["true"] > 10000
    assert r["foot_missed"] == 0 and r["band_missed"] == 0, r
    assert r["band_test"] <= 1.01 * r["foot_test"], r  # and hardly looser


def test_sub_block_band_test_is_conservative():
    """The blend backward's 4x4 sub-block lists (sub_block_mask) come from the band form with 4-row bands."""
    r = cull_check.run(N=60000, seed=5, size=4)
    assert r["true"] > 3000
    assert r["band_missed"] == 0, r
    assert r["band_test"] <= 1.03 * r["true"] + 200, r  # close to exact
