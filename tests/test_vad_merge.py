"""Host side of merge_chunks (vad.py:264-311) without a device: the timeline of the region
arrays (Annotation.get_timeline: the sorted set of segments) and the greedy chunk merge by
binary search, both against the reference's per-region loop as restated in the oracle."""
import numpy as np

from oracle import oracle


def _regions(rng, n, gaps=True):
    """A single VAD column's regions: increasing starts, non-decreasing ends, some sharing
    an endpoint with the next one (min-cut splits) and some with tiny gaps."""
    d = rng.choice([0.017, 0.5, 3.0, 12.0, 29.9], size=n, p=[0.3, 0.3, 0.2, 0.15, 0.05]) * rng.uniform(0.5, 1, n)
    g = np.where(rng.random(n) < 0.4, 0.0, rng.exponential(0.8, n)) if gaps else np.zeros(n)
    s = np.empty(n)
    e = np.empty(n)
    t = rng.uniform(0, 2)
    for i in range(n):
        s[i] = t
        e[i] = t + d[i]
        t = e[i] + g[i]
    return s, e


def test_greedy_chunks_arrays_matches_loop():
    from whisperx_amd.vad import _greedy_chunks_arrays

    rng = np.random.default_rng(0)
    for trial in range(60):
        n = int(rng.integers(1, 3000))
        s, e = _regions(rng, n, gaps=trial % 3 != 0)
        for chunk in (30.0, 10.0, 2.5, 0.25):
            want = oracle.merge_chunks_regions(list(zip(s.tolist(), e.tolist())), chunk)
            got = _greedy_chunks_arrays(s, e, chunk)
            assert got == want, (trial, chunk)


def test_greedy_chunks_arrays_edges():
    from whisperx_amd.vad import _greedy_chunks_arrays

    def ref(s, e, c):
        return oracle.merge_chunks_regions(list(zip(s, e)), c)

    cases = [
        ([0.0], [1.0], 30.0),
        ([0.0, 1.0], [1.0, 31.0], 30.0),  # end - start exactly at chunk_size (not >): no flush
        ([0.0, 1.0], [1.0, 30.000000001], 30.0),
        ([0.1, 0.2, 0.3], [40.0, 80.0, 120.0], 30.0),  # every region longer than a chunk
        ([-5.0, 1.0], [40.0, 41.0], 30.0),  # negative start: the reference flushes an empty chunk first
        ([0.1 * k for k in range(100)], [0.1 * k + 0.1 for k in range(100)], 0.3),  # fp-rounding boundaries
    ]
    for s, e, c in cases:
        assert _greedy_chunks_arrays(np.array(s), np.array(e), c) == ref(s, e, c), (s, e, c)


def test_greedy_chunks_arrays_unsorted_ends_fall_back():
    from whisperx_amd.vad import _greedy_chunks_arrays

    s = np.array([0.0, 1.0, 2.0, 3.0])
    e = np.array([50.0, 2.0, 45.0, 4.0])  # ends not monotone (two overlapping columns)
    assert _greedy_chunks_arrays(s, e, 30.0) == oracle.merge_chunks_regions(list(zip(s, e)), 30.0)


def test_timeline_is_sorted_set_of_all_columns():
    from whisperx_amd.vad import _timeline

    rng = np.random.default_rng(1)
    a = _regions(rng, 500)
    b = _regions(rng, 300)
    # a third column repeating some of the first one's regions
    c = (a[0][::7].copy(), a[1][::7].copy())
    s, e = _timeline([a, b, c])
    want = sorted(set(zip(a[0].tolist(), a[1].tolist())) | set(zip(b[0].tolist(), b[1].tolist())))
    assert list(zip(s.tolist(), e.tolist())) == want
    s1, e1 = _timeline([a])
    assert np.array_equal(s1, a[0]) and np.array_equal(e1, a[1])
    s0, e0 = _timeline([(np.zeros(0), np.zeros(0))])
    assert len(s0) == 0 and len(e0) == 0
