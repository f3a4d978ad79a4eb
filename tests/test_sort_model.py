"""CPU check of the algorithm behind the pair stage's workgroup-parallel
std::sort (k_match.hip block_gnu_sort): a level-synchronous introsort whose
Hoare partitions are expressed through left/right stop ranks, followed by a
stable sort inside each final range. This Python model of the same rules must
reproduce libstdc++'s std::sort permutation (oracle_sort_dmatch) exactly,
ties included; the GPU kernel itself is checked by
test_gpu_parity.py::test_good_match_sort_is_std_sort."""
import numpy as np
import pytest

import oracle_lib as O


def _median_to_first(k, v, res, x, y, z):
    def sw(i, j):
        k[i], k[j] = k[j], k[i]
        v[i], v[j] = v[j], v[i]
    ax, ay, az = k[x], k[y], k[z]
    if ax < ay:
        sw(res, y) if ay < az else (sw(res, z) if ax < az else sw(res, x))
    elif ax < az:
        sw(res, x)
    elif ay < az:
        sw(res, z)
    else:
        sw(res, y)


def parallel_introsort_model(keys):
    k, v, n = list(keys), list(range(len(keys))), len(keys)
    cuts = {0}
    ranges = [(0, n, 2 * (n.bit_length() - 1))] if n > 16 else []
    while ranges:
        nxt = []
        for f, l, d in ranges:
            assert d > 0, "depth limit (heap sort path) not modelled"
            _median_to_first(k, v, f, f + 1, f + (l - f) // 2, l - 1)
            pk = k[f]
            L = [j for j in range(f + 1, l) if k[j] >= pk]       # left stops, original order
            R = [j for j in range(l - 1, f, -1) if k[j] <= pk]   # right stops
            ks = 0
            while ks < min(len(L), len(R)) and L[ks] < R[ks]:
                ks += 1
            for i in range(ks):
                a, b = L[i], R[i]
                k[a], k[b] = k[b], k[a]
                v[a], v[b] = v[b], v[a]
            cut = min(([L[ks]] if ks < len(L) else []) + ([R[ks - 1]] if ks else []))
            cuts.add(cut)
            nxt += [(a, b, d - 1) for a, b in ((f, cut), (cut, l)) if b - a > 16]
        ranges = sorted(nxt)
    bounds = sorted(cuts) + [n]
    for a, b in zip(bounds[:-1], bounds[1:]):
        seg = sorted(range(a, b), key=lambda i: k[i])  # stable
        k[a:b], v[a:b] = [k[i] for i in seg], [v[i] for i in seg]
    return v


@pytest.mark.parametrize("seed", range(12))
def test_model_matches_std_sort(seed):
    rng = np.random.default_rng(seed)
    for _ in range(4):
        n = int(rng.integers(1, 1500))
        d = rng.integers(0, int(rng.integers(1, 300)), n).astype(np.float32)
        if seed % 3 == 0:
            t = n // 3
            d[:t] = np.sort(d[:t])
            d[t:2 * t] = np.sort(d[t:2 * t])[::-1]
        m = np.zeros(n, O.DMATCH_DTYPE)
        m["queryIdx"] = np.arange(n)
        m["distance"] = d
        O.lib().oracle_sort_dmatch(O.ptr(m), n)
        assert list(m["queryIdx"]) == parallel_introsort_model(d.tolist())
