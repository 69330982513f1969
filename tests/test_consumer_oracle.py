"""CPU: the server-side consumer restatements in oracle/psf_port.c (SURVEY.md
§8(f) f4) against independent Python restatements of the reference code.

No reference test or fixture covers ParallelOrderedMatch or FTRLEntry
(parallel_ordered_match_test.cc reads key files that are not in the tree,
src/test/parallel_ordered_match_test.cc:15-16), and their headers need the
protobuf / glog / Eigen the image lacks, so these two restatements are pinned
only against each other: parity for this row is "unpinned" by the reference.
"""
import numpy as np
import pytest


def match_py(sk, sv, dk, dv, k, op):
    """parallel_ordered_match.h:14-34, line by line, in Python."""
    if len(dk) == 0 or len(sk) == 0:
        return 0
    s = int(np.searchsorted(sk, dk[0], side="left"))
    d, n = 0, 0
    while d < len(dk) and s < len(sk):
        if sk[s] < dk[d]:
            s += 1
        else:
            if not (dk[d] < sk[s]):
                for i in range(k):
                    a, b = dv[d * k + i], sv[s * k + i]
                    dv[d * k + i] = [b, a + b, a - b, a * b, a / b if b != 0 else a / b][op]
                s += 1
                n += k
            d += 1
    return n


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("op", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_ordered_match_port_vs_python(port, k, op, dtype):
    rng = np.random.default_rng(op * 10 + k)
    dk = np.unique(rng.integers(0, 5000, 900).astype(np.uint64))
    sk = np.sort(rng.integers(0, 5000, 700).astype(np.uint64))  # with repeated keys
    sv = (rng.standard_normal(sk.size * k) + 3).astype(dtype)
    dv0 = (rng.standard_normal(dk.size * k) + 3).astype(dtype)
    a, b = dv0.copy(), dv0.copy()
    with np.errstate(all="ignore"):
        n1 = port.ordered_match(sk, sv, dk, a, k, op)
        n2 = match_py(sk, sv, dk, b, k, op)
    assert n1 == n2
    assert a.tobytes() == b.tobytes()


def test_ordered_match_edge_cases(port):
    e = np.zeros(0, np.uint64)
    v = np.zeros(0, np.float32)
    assert port.ordered_match(e, v, np.arange(3, dtype=np.uint64), np.zeros(3, np.float32)) == 0
    assert port.ordered_match(np.arange(3, dtype=np.uint64), np.ones(3, np.float32), e, v) == 0
    # repeated dst keys pair with repeated src keys in order
    dk = np.array([2, 2, 2, 5], np.uint64)
    sk = np.array([2, 2, 5, 5], np.uint64)
    dv = np.zeros(4, np.float32)
    assert port.ordered_match(sk, np.array([1, 2, 3, 4], np.float32), dk, dv, 1, 1) == 3
    assert dv.tolist() == [1, 2, 0, 3]


def ftrl_py(state, keys, grads, decay, alpha, beta, l1, l2):
    """async_sgd.h:137-151 + learning_rate.h:15-22 + penalty.h:51-56 in numpy
    float32 scalars (each operation rounded to float, as g++ on x86-64 does)."""
    f = np.float32
    for key, g in zip(keys.tolist(), grads.astype(np.float32)):
        w, z, sn = state.get(key, (f(0), f(0), f(0)))
        w_old = w
        sn_new = f(np.sqrt(f(sn * sn + g * g)))
        sigma = f(f(sn_new - sn) / alpha)
        z = f(z + f(g - f(sigma * w)))
        sn = sn_new
        eta = f(alpha / f(sn + beta)) if decay else alpha
        zz = f(-z * eta)
        leta = f(l1 * eta)
        if zz <= leta and zz >= -leta:
            w = f(0)
        else:
            den = f(f(1) + f(l2 * eta))
            w = f(f(zz - leta) / den) if zz > 0 else f(f(zz + leta) / den)
        state[key] = (w, z, sn)
        state["nnz"] = state.get("nnz", 0) + (-1 if (w == 0 and w_old != 0) else (1 if (w != 0 and w_old == 0) else 0))


@pytest.mark.parametrize("decay,l1,l2", [(1, 0.0, 0.0), (1, 1.0, 0.5), (0, 0.2, 0.0)])
def test_ftrl_port_vs_python(port, decay, l1, l2):
    import oracle
    f = np.float32
    alpha, beta = f(0.05), f(1.0)
    m = oracle.FtrlModel(port, 2 if decay else 1, alpha, beta, l1, l2)
    st = {}
    rng = np.random.default_rng(7)
    for step in range(6):
        keys = np.unique(rng.integers(0, 400, 250).astype(np.uint64))
        g = (rng.standard_normal(keys.size) * 3).astype(np.float32)
        assert m.push(keys, g) == 0
        ftrl_py(st, keys, g, decay, alpha, beta, f(l1), f(l2))
    keys = np.array(sorted(k for k in st if k != "nnz"), np.uint64)
    want = np.array([st[k][0] for k in keys.tolist()], np.float32)
    assert m.pull(keys).tobytes() == want.tobytes()
    assert m.nnz.value == st["nnz"]
    assert (m.pull(keys) != 0).sum() == m.nnz.value
