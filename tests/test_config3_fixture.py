"""CPU: the config-3 golden fixture (tests/golden/gen_config3_fixture.py) is consistent -- the
packed labels unpack to the stored shape and class counts, and the pack / unpack pair is exact."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from gen_config3_fixture import SHAPE, pack_labels, unpack_labels  # noqa: E402


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(0)
    lab = rng.integers(0, 4, size=(1, 7, 5, 3), dtype=np.uint8)
    assert np.array_equal(unpack_labels(pack_labels(lab), lab.shape), lab)


def test_config3_fixture_consistent():
    fx = np.load(os.path.join(HERE, "golden", "config3_fixture.npz"))
    shape = tuple(int(v) for v in fx["c3_labels_shape"])
    assert shape == (SHAPE[0],) + tuple(SHAPE[2:])
    assert tuple(int(v) for v in fx["c3__shape"]) == (SHAPE[0], 4) + tuple(SHAPE[2:])
    lab = unpack_labels(fx["c3_labels_packed"], shape)
    assert np.array_equal(np.bincount(lab.reshape(-1), minlength=4), fx["c3_label_counts"])
