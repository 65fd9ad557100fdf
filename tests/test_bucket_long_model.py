"""CPU model of the long-list bucket sort (binning.hip bucket_sort_long), checked against a plain sort.

The kernel keeps a long tile list (more keys than its workgroup holds in registers) in memory and sorts it in
windows of whole bins: one read for the key range, one for the bin counts, then per window of at most NMAX
keys a read that scatters the window's keys into LDS through an atomic on each bin's start.  The atomic leaves
start[b] at the next bin's start, so after a window's scatter bin b spans [start[b - 1], start[b]); a key's rank
in its bin is its count of smaller keys there.  This model follows the same arithmetic (the bins, the window
cut at a straddling bin, the first bin past a window, the moving starts) with the atomics' order shuffled, so
the window bookkeeping is checked on many lists without a GPU; the GPU tests run the kernel itself
(tests/test_gpu_options.py sort_prefix=0 on the long-list cases, tests/test_gpu_fullsize.py at 5M@4K in
whole-list mode, profiles/r06/r7x)."""
import random

import pytest

K_BIN_SHIFT = 1
K_SKEW = 48


def bucket_sort_long_model(keys, nmax=2048, nbmax=2048, threads=256, rng=None, lim=None):
    """Returns the sorted list -- in prefix mode (lim) (its first `sorted` entries, sorted) -- or None where the
    kernel reports failure (skew, or one bin over the buffer)."""
    rng = rng or random.Random(0)
    n = len(keys)
    mn, mx = min(keys), max(keys)
    lg = 0
    while (1 << lg) < (n >> K_BIN_SHIFT) and (1 << lg) < nbmax:
        lg += 1
    span = mx - mn
    bits = span.bit_length() if span else 0
    sh = bits - lg if bits > lg else 0
    nb = (span >> sh) + 1
    per = (nb + threads - 1) // threads
    start = [0] * (per * threads + 2)
    for k in keys:
        start[(k - mn) >> sh] += 1
    if sum(v * v for v in start[:nb]) > K_SKEW * n:
        return None
    at = 0
    for b in range(per * threads):
        v = start[b]
        start[b] = at
        at += v
    start[nb] = n
    out = [None] * n
    bw0 = w0 = 0
    lim = n if lim is None else lim
    while w0 < n and w0 < lim:
        cut = w0 + nmax
        w1 = cut if cut < n else n
        if cut < n:
            for b in range(bw0, nb):
                if start[b] < cut < start[b + 1]:
                    w1 = min(w1, start[b])
        if w1 <= w0:
            return None
        bw1 = min([b for b in range(bw0, nb) if start[b] >= w1], default=nb)
        buf = [None] * nmax
        order = list(range(n))
        rng.shuffle(order)  # the atomics' arrival order is arbitrary
        for i in order:
            k = keys[i]
            b = (k - mn) >> sh
            if bw0 <= b < bw1:
                buf[start[b] - w0] = k
                start[b] += 1
        for j in range(w1 - w0):
            kj = buf[j]
            b = (kj - mn) >> sh
            st = (start[b - 1] if b else 0) - w0
            en = start[b] - w0
            c = sum(1 for q in range(st, en) if buf[q] < kj)
            out[w0 + st + c] = kj
        w0, bw0 = w1, bw1
    return out if lim >= n else (out[:w0], w0)


@pytest.mark.parametrize("seed", range(6))
def test_bucket_sort_long_model_sorts(seed):
    rng = random.Random(seed)
    sorted_ok = 0
    for _ in range(12):
        n = rng.choice([4097, 5000, 8191, 12000])
        spread = rng.choice([1 << 12, 1 << 24, 1 << 36])
        base = rng.randint(0, 1 << 30)
        # keys as K3 forms them: depth bits above, the Gaussian index below (unique keys)
        keys = [((base + rng.randint(0, spread)) << 20) | i for i in range(n)]
        rng.shuffle(keys)
        out = bucket_sort_long_model(keys, rng=rng)
        if out is None:
            continue
        assert out == sorted(keys)
        sorted_ok += 1
    assert sorted_ok > 0


@pytest.mark.parametrize("lim", [1024, 3000])
def test_bucket_sort_long_model_prefix(lim):
    """Prefix mode (the reachable-prefix sort): the windows stop once they cover lim keys; what they wrote is the
    smallest `sorted` keys in order, sorted >= lim."""
    rng = random.Random(lim)
    for _ in range(8):
        n = rng.choice([5000, 9000, 20000])
        keys = [((rng.randint(0, 1 << 24)) << 20) | i for i in range(n)]
        rng.shuffle(keys)
        res = bucket_sort_long_model(keys, rng=rng, lim=lim)
        if res is None:
            continue
        head, m = res
        assert lim <= m <= n
        assert head == sorted(keys)[:m]


def test_bucket_sort_long_model_reports_skew():
    # every key in a sliver of the range but one: one bin holds nearly all keys -> the kernel falls back
    keys = [(1000 << 20) | i for i in range(6000)] + [((1 << 40) << 20) | 6000]
    assert bucket_sort_long_model(keys) is None
