"""cqgpu_route_major (host code, no device): the repartitioned join's routing mode
from the ranks' summed ON-key counts per value class (NULL, number, string, date).
value_compare calls any two non-NULL keys of different classes equal
(reference csv_reader.c:126-129, the join's compare at evaluator_joins.c:53-55), so
replication is needed exactly when the left side holds a class x and the right side a
class y != x; the class most keys hold then routes by key."""
import numpy as np

import cq_amd


def _want(l, r):
    if not any(x != y and l[x] and r[y] for x in (1, 2, 3) for y in (1, 2, 3)):
        return 0
    best = 1
    for k in (2, 3):
        if l[k] + r[k] > l[best] + r[best]:
            best = k
    return best


def test_route_major_rule():
    rng = np.random.default_rng(3)
    for _ in range(3000):
        l = [int(x) for x in rng.integers(0, 4, 4) * (rng.random(4) < 0.5)]
        r = [int(x) for x in rng.integers(0, 4, 4) * (rng.random(4) < 0.5)]
        assert cq_amd.route_major(l, r) == _want(l, r), (l, r)


def test_route_major_cases():
    assert cq_amd.route_major([5, 9, 0, 0], [7, 3, 0, 0]) == 0            # numbers only (NULLs match NULLs)
    assert cq_amd.route_major([0, 0, 4, 0], [0, 0, 9, 0]) == 0            # strings only
    assert cq_amd.route_major([0, 10, 0, 0], [0, 0, 1, 0]) == 1           # numbers x one string: replicate
    assert cq_amd.route_major([0, 1, 30, 0], [0, 2, 0, 0]) == 2           # strings the majority
    assert cq_amd.route_major([0, 0, 0, 4], [0, 0, 0, 5]) == 0            # dates only
    assert cq_amd.route_major([0, 2, 2, 0], [0, 0, 0, 0]) == 0            # an empty right side
