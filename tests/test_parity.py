"""Property tests: native compat mode == reference oracle, bit for bit.

The oracle (nanogpu/sim/oracle.py) is an independent Python executable spec of the
reference algorithm; the C++ compat path must agree on every
placement, every score and every Go 1.16 sort permutation, including n > 12 where
Go switches from shell+insertion sort to introsort.
"""
from hypothesis import given, settings
from hypothesis import strategies as st

from nanogpu import _native as N
from nanogpu.sim import oracle as O

frees = st.lists(st.integers(min_value=0, max_value=100), min_size=1, max_size=16)
demands = st.lists(st.sampled_from([0, 5, 10, 20, 25, 30, 40, 50, 60, 75, 100]), min_size=1, max_size=6)


@settings(max_examples=400, deadline=None)
@given(st.lists(st.integers(min_value=-5, max_value=120), min_size=0, max_size=80))
def test_go116_sort_permutation(keys):
    data = list(enumerate(keys))
    O.go116_sort(data, key=lambda x: x[1])
    assert N.go116_sort_perm(keys) == [i for i, _ in data]


@settings(max_examples=400, deadline=None)
@given(frees, demands, st.sampled_from(["binpack", "spread"]))
def test_choose_matches_oracle(fs, ds, policy):
    spread = policy == "spread"
    opts = N.Options(N.Policy.SPREAD if spread else N.Policy.BINPACK, compat=True)
    want = O.choose([O.G(f) for f in fs], ds, spread)
    rc, plan, score = N.choose([{"pct_free": f} for f in fs], [(d, 0) for d in ds], opts)
    if want is None:
        assert rc == N.ERR_NO_FIT
    else:
        assert rc == N.OK
        assert [p[0] for p in plan] == want
        ref_score = O.rate_spread([O.G(f) for f in fs]) if spread else O.rate_binpack([O.G(f) for f in fs])
        assert score == ref_score


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(min_value=0, max_value=100), min_size=13, max_size=64),
       st.lists(st.sampled_from([10, 20, 30, 50]), min_size=1, max_size=4))
def test_choose_matches_oracle_many_devices(fs, ds):
    # CPX nodes have 64 devices: exercises Go's introsort path (n > 12)
    for policy, spread in ((N.Policy.BINPACK, False), (N.Policy.SPREAD, True)):
        want = O.choose([O.G(f) for f in fs], ds, spread)
        rc, plan, _ = N.choose([{"pct_free": f} for f in fs], [(d, 0) for d in ds], N.Options(policy, compat=True))
        assert (want is None) == (rc != N.OK)
        if want is not None:
            assert [p[0] for p in plan] == want


@settings(max_examples=200, deadline=None)
@given(frees, demands)
def test_first_fit_matches_oracle(fs, ds):
    want = O.first_fit([O.G(f) for f in fs], ds)
    rc, plan, _ = N.choose([{"pct_free": f} for f in fs], [(d, 0) for d in ds],
                           N.Options(N.Policy.FIRSTFIT, compat=True))
    assert (want is None) == (rc != N.OK)
    if want is not None:
        assert [p[0] for p in plan] == want


@settings(max_examples=150, deadline=None)
@given(st.lists(st.integers(min_value=0, max_value=100), min_size=1, max_size=8),
       st.lists(st.integers(min_value=0, max_value=2), min_size=8, max_size=8),
       st.lists(st.sampled_from([10, 20, 40]), min_size=1, max_size=3))
def test_load_aware_ordering_matches_oracle(fs, loads, ds):
    # RemainLoad enters the sort key as free + 50*RemainLoad (allocate.go:247)
    devs = [{"pct_free": f, "remain_load": loads[i]} for i, f in enumerate(fs)]
    for policy, spread in ((N.Policy.BINPACK, False), (N.Policy.SPREAD, True)):
        want = O.choose([O.G(f, 100, loads[i]) for i, f in enumerate(fs)], ds, spread)
        rc, plan, _ = N.choose(devs, [(d, 0) for d in ds], N.Options(policy, compat=True, load_aware=True))
        assert (want is None) == (rc != N.OK)
        if want is not None:
            assert [p[0] for p in plan] == want
