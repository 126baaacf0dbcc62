"""summary_ref.py — CPU restatement of Mamba's posterior summaries (TEST INFRASTRUCTURE ONLY).

Imported by tests/ as the checker of the device summaries (mamba.jl_amd/summary.py +
summary.hip); never by the product.  Restates, on an n x p x m draw array:

  summarystats(c; etype=:bm)   src/output/stats.jl:85-94
      f(x) = [mean(x), std(x), sem(x), mcse(vec(x), :bm)],  x = c.value[:, j, :] (n x m)
      ESS  = min((SD ./ MCSE).^2, size(c.value, 1))
  mcse_bm(x; size=100)         src/output/mcse.jl:10-19
      m = div(length(x), size) (>= 2 else ArgumentError); mbar_i = mean(x[i*size + (1:size)]);
      sem(mbar)
  quantile(c; q)               src/output/stats.jl:73-80 -> Julia 0.5 Base.quantile!
      (not vendored; recalled): index = 1 + (lv-1) q, lo = floor, hi = ceil, sorted v,
      r = v[lo] where index == lo else (1-h) v[lo] + h v[hi], h = index - lo
  StatsBase 0.7 (not vendored): std = sqrt(sum((x - mean)^2) / (N - 1)), sem = std / sqrt(N).

vec(x) is column-major: chain 1's n draws, then chain 2's, ... (Julia `vec`).  Sums use
math.fsum (exactly rounded), so the device results are compared with a stated relative
tolerance, not bit for bit (reduction order is a design choice on both sides).
"""
import math

import numpy as np


def _fmean(v):
    return math.fsum(v) / len(v)


def _fstd(v):
    mu = _fmean(v)
    return math.sqrt(math.fsum((x - mu) ** 2 for x in v) / (len(v) - 1))


def mcse_bm(x, size=100):
    x = list(map(float, x))
    n = len(x)
    m = n // size
    if m < 2:
        raise ValueError(f"iterations are < {2 * size} and batch size is > {n // 2}")
    mbar = [_fmean(x[i * size:(i + 1) * size]) for i in range(m)]
    return _fstd(mbar) / math.sqrt(m)


def summarystats(value, batch_size=100):
    """value: n x p x m -> p x [Mean, SD, Naive SE, MCSE, ESS]."""
    value = np.asarray(value, dtype=np.float64)
    n, p, _ = value.shape
    out = np.empty((p, 5))
    for j in range(p):
        v = value[:, j, :].ravel(order="F")  # vec(x): chains concatenated
        sd = _fstd(v)
        out[j] = [_fmean(v), sd, sd / math.sqrt(v.size), mcse_bm(v, batch_size), 0.0]
        out[j, 4] = min((out[j, 1] / out[j, 3]) ** 2, n)
    return out


def quantile(value, q=(0.025, 0.25, 0.5, 0.75, 0.975)):
    value = np.asarray(value, dtype=np.float64)
    n, p, _ = value.shape
    out = np.empty((p, len(q)))
    for j in range(p):
        v = np.sort(value[:, j, :].ravel())
        lv = v.size
        for t, qq in enumerate(q):
            index = 1.0 + (lv - 1) * qq
            lo, hi = int(math.floor(index)), int(math.ceil(index))
            h = index - lo
            out[j, t] = v[lo - 1] if index == lo else (1.0 - h) * v[lo - 1] + h * v[hi - 1]
    return out


def chain_partials(value, kg, bs, shift):
    """Per-chain partials in the layout of mmb_chain_summary (a direct restatement of the
    kernel's contract, used to test the host pooling logic without a GPU)."""
    value = np.asarray(value, dtype=np.float64)
    n, p, K = value.shape
    out = np.zeros((K, p, 10))
    for k in range(K):
        t0 = int(kg[k]) * n
        for j in range(p):
            x = value[:, j, k] - shift[j]
            o = out[k, j]
            o[0], o[1] = x.sum(), (x * x).sum()
            i = 0
            while i < n:
                b = (t0 + i) // bs
                end = min(n, (b + 1) * bs - t0)  # first index past this batch inside the chain
                seg = x[i:end]
                starts = (t0 + i) % bs == 0
                closes = (t0 + end) % bs == 0
                if starts and closes:
                    d = seg.sum() / bs
                    o[2] += d
                    o[3] += d * d
                    o[4] += 1
                elif not starts:
                    o[5], o[6] = seg.sum(), seg.size      # head (or whole chain inside one batch)
                else:
                    o[7], o[8] = seg.sum(), seg.size      # tail
                i = end
    return out
