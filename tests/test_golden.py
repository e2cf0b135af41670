"""The CPU restatement reproduces its frozen regression vectors (tests/golden/,
written by tests/golden/make_golden.py) bit for bit."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden  # noqa: E402


@pytest.mark.parametrize("name", sorted(make_golden.CASES))
def test_oracle_matches_golden(name):
    g = np.load(os.path.join(HERE, "golden", f"{name}.npz"))
    got = make_golden.compute(make_golden.CASES[name])
    for k in g.files:
        assert np.array_equal(np.asarray(got[k]), g[k]), k
