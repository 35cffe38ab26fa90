"""Golden vectors from the reference's own tests.

reference pkg/dealer/rater_test.go:9-401 and allocate_test.go:16-230 — their expected
values are still valid specs for the non-load path even though those files no longer
compile against the reference HEAD.
"""
import hashlib

import pytest

from nanogpu import _native as N

B = N.Options(N.Policy.BINPACK, compat=True)
S = N.Options(N.Policy.SPREAD, compat=True)
F = N.Options(N.Policy.FIRSTFIT, compat=True)


def dev(frees, total=100):
    return [{"pct_free": f, "pct_total": total} for f in frees]


def dem(ps):
    return [(p, 0) for p in ps]


@pytest.mark.parametrize("a,b,sa,sb", [([30, 50], [20, 40], 58, 68)])
def test_binpack_rate(a, b, sa, sb):
    # rater_test.go:9-37: the busier node (second) is preferred
    assert N.rate(dev(a), dem([1]), B) == sa
    assert N.rate(dev(b), dem([1]), B) == sb
    assert sb > sa


@pytest.mark.parametrize("a,b,sa,sb", [
    ([30, 50], [20, 40], 6, 4),
    ([90], [50, 40], 8, 7),
    ([100], [50, 50], 109, 8),
    ([100], [100, 50], 109, 113),
])
def test_spread_rate(a, b, sa, sb):
    # rater_test.go:39-131
    assert N.rate(dev(a), dem([1]), S) == sa
    assert N.rate(dev(b), dem([1]), S) == sb


def test_spread_rate_empty_8gpu_is_872():
    assert N.rate(dev([100] * 8), dem([1]), S) == 872


def test_binpack_truncation():
    # 58/200*100 = 28.999... truncates to 28 (Appendix B.3); minus G=2
    assert N.rate(dev([42, 100]), dem([1]), B) == 28 - 2


@pytest.mark.parametrize("frees,demand,want", [
    ([100, 100], [20, 40], [0, 0]),
    ([20, 100], [20, 40], [0, 1]),
    ([10, 100], [20, 40], [1, 1]),
    ([100, 100], [0, 40, 40], [-1, 0, 0]),
    ([10, 50], [20, 40], None),
])
def test_binpack_choose(frees, demand, want):
    rc, plan, _ = N.choose(dev(frees), dem(demand), B)
    if want is None:
        assert rc == N.ERR_NO_FIT
    else:
        assert rc == N.OK and [p[0] for p in plan] == want


@pytest.mark.parametrize("frees,demand,want", [
    ([100, 100], [20, 40], [0, 1]),
    ([20, 100], [20, 40], [1, 1]),
    ([10, 100], [20, 40], [1, 1]),
    ([100, 100], [0, 40, 40], [-1, 0, 1]),
    ([10, 50], [20, 40], None),
])
def test_spread_choose(frees, demand, want):
    rc, plan, _ = N.choose(dev(frees), dem(demand), S)
    if want is None:
        assert rc == N.ERR_NO_FIT
    else:
        assert rc == N.OK and [p[0] for p in plan] == want


@pytest.mark.parametrize("frees,demand,ok", [
    ([100, 100], [50, 50], True),
    ([100], [50, 50], True),
    ([100], [50, 60], False),
    ([100, 100], [100, 10], True),
])
def test_first_fit(frees, demand, ok):
    # allocate_test.go:160-190 (SampleRater)
    rc, plan, score = N.choose(dev(frees), dem(demand), F)
    assert (rc == N.OK) == ok
    if ok:
        assert score == 100


def test_sort_order():
    # allocate_test.go:213-230: free [80,100,30,50] sorts to indices [2,3,0,1]
    assert N.go116_sort_perm([80, 100, 30, 50]) == [2, 3, 0, 1]


def test_go116_unstable_tiebreak_picks_gpu1():
    # Appendix B.2 worked example: a stable sort would pick GPU 0, Go 1.16 picks GPU 1.
    rc, plan, _ = N.choose(dev([50, 50, 50, 50, 50, 50, 10, 50]), dem([40]), B)
    assert rc == N.OK and plan == [[1]]


def test_zero_gpu_node_is_unfit_not_a_crash():
    # D6: the reference divides by len(gpus) == 0 and panics.
    rc, plan, _ = N.choose([], dem([10]), B)
    assert rc == N.ERR_NO_DEVICES


def test_demand_hash_matches_reference_format():
    from nanogpu.state.cluster import demand_hash_compat

    assert demand_hash_compat([(20, 0), (40, 0)]) == hashlib.sha256(b"(20)(40)").hexdigest()[:8]


def test_apply_release_roundtrip_and_rollback():
    devs = dev([100, 100])
    rc, after = N.apply(devs, dem([30, 50]), [[0], [1]])
    assert rc == N.OK and [d["pct_free"] for d in after] == [70, 50]
    rc, back = N.apply(after, dem([30, 50]), [[0], [1]], release=True)
    assert [d["pct_free"] for d in back] == [100, 100]
    # D5: a misfit in the second container restores exactly the first one's debit
    rc, same = N.apply(dev([100, 20]), dem([30, 50]), [[0], [1]])
    assert rc == N.ERR_PLAN_NO_LONGER_FITS
    assert [d["pct_free"] for d in same] == [100, 20]
