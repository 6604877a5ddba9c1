"""The wide-row canonical top-k helper the real-shape GPU tests check against equals
the oracle's canonical_topk (score desc, index asc), ties and -1e10 masks included."""
import numpy as np

import rsx_oracle as O
from helpers import canonical_topk_fast


def test_canonical_topk_fast_equals_oracle():
    rng = np.random.default_rng(0)
    for scores in (rng.integers(-3, 4, size=(40, 700)).astype(np.float32),   # heavy ties
                   rng.standard_normal((40, 700)).astype(np.float32)):
        scores[3, 10:] = -1e10   # a user with all but 10 items masked
        scores[5, :] = -1e10
        v1, i1 = O.canonical_topk(scores, 50)
        v2, i2 = canonical_topk_fast(scores, 50)
        assert np.array_equal(i1, i2) and np.array_equal(v1, v2)
