"""CPU check of the int8 scan's lower bound (knn_kernels.hip rows_to_i8_kernel /
prep_queries_i8_kernel, DESIGN.md §3 "The int8 scan"), restated in numpy f64:

    x^ = rint(x * 127 / max|x_i|), s_x = f32(max|x_i| / 127), x~ = s_x x^, e_x = x - x~
    |x.q - s_x s_q (x^.q^)| <= |e_x||q| + |x~||e_q|

so LB = exact(x, q) - 2(|e_x||q| + |x~||e_q|) (l2), - (..) (dot), - (..)/(|x||q|)
(cosine) never exceeds the exact distance the reference ranks by
(lance_manager.rs:393-451: squared L2, 1 - x.q, 1 - cos).  Distributions where
per-row scaling is worst: heavy tails, one dominant coordinate, near-constant
rows, tiny and huge norms.  (The GPU tests check the kernel end to end against
the f64 oracle; this pins the algebra and the exact-integer claim.)"""
import numpy as np
import pytest


def quant(A):
    m = np.abs(A).max(1)
    s = (m / np.float32(127.0)).astype(np.float32).astype(np.float64)
    inv = np.where(m > 0, np.float32(127.0) / np.where(m > 0, m, 1), 0).astype(np.float32)
    q = np.clip(np.rint((A * inv[:, None]).astype(np.float32)), -127, 127)
    return q, s


def bounds(X, Q, metric):
    Xh, sx = quant(X)
    Qh, sq = quant(Q)
    X64, Q64 = X.astype(np.float64), Q.astype(np.float64)
    ex = np.linalg.norm(X64 - sx[:, None] * Xh, axis=1)
    xt = np.linalg.norm(sx[:, None] * Xh, axis=1)
    eq = np.linalg.norm(Q64 - sq[:, None] * Qh, axis=1)
    xn, qn = np.linalg.norm(X64, axis=1), np.linalg.norm(Q64, axis=1)
    S_int = Qh @ Xh.T                       # exact integers (|.| < 2^24 checked below)
    assert np.abs(S_int).max() < 2 ** 24
    approx = S_int * sq[:, None] * sx[None, :]
    eps = qn[:, None] * ex[None, :] + eq[:, None] * xt[None, :]
    dot = Q64 @ X64.T
    if metric == "l2":
        exact = (xn ** 2)[None, :] + (qn ** 2)[:, None] - 2 * dot
        lb = (xn ** 2)[None, :] + (qn ** 2)[:, None] - 2 * approx - 2 * eps
    elif metric == "dot":
        exact = 1 - dot
        lb = 1 - approx - eps
    else:
        den = qn[:, None] * xn[None, :]
        exact = 1 - dot / den
        lb = 1 - (approx + eps) / den
    return lb, exact


def datasets(rng, d):
    yield "gauss", rng.standard_normal((400, d)).astype(np.float32)
    yield "heavy", rng.standard_cauchy((400, d)).clip(-1e4, 1e4).astype(np.float32)
    spike = rng.standard_normal((400, d)).astype(np.float32) * 1e-3
    spike[np.arange(400), rng.integers(0, d, 400)] = 50.0
    yield "spike", spike
    yield "near_const", (3.0 + 1e-4 * rng.standard_normal((400, d))).astype(np.float32)
    yield "tiny", (1e-20 * rng.standard_normal((400, d))).astype(np.float32)
    yield "huge", (1e15 * rng.standard_normal((400, d))).astype(np.float32)
    yield "sparse_int", rng.integers(-3, 4, (400, d)).astype(np.float32)


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("d", [128, 768, 1024])
def test_i8_bound_is_rigorous(metric, d):
    rng = np.random.default_rng(d)
    for name, X in datasets(rng, d):
        Q = np.concatenate([X[:50] + 0.01 * rng.standard_normal((50, d)).astype(np.float32),
                            rng.standard_normal((30, d)).astype(np.float32) * np.abs(X).max()])
        lb, exact = bounds(X, Q, metric)
        scale = np.abs(exact).max() + 1e-300
        # rigorous in exact arithmetic; the kernel's slack covers its f32 evaluation
        assert (lb <= exact + 1e-9 * scale).all(), (name, metric, float((lb - exact).max() / scale))


def test_i8_bound_tightness_gaussian():
    # the reason the selection refines k + 96 / k + 192 candidates:
    # the slack is ~0.3 of the distance spread for N(0,1) rows at d = 768
    rng = np.random.default_rng(0)
    X = rng.standard_normal((20_000, 768)).astype(np.float32)
    Q = rng.standard_normal((16, 768)).astype(np.float32)
    lb, exact = bounds(X, Q, "l2")
    slack = exact - lb
    assert 0.1 < np.median(slack) / exact.std() < 0.6
    dk = np.sort(exact, 1)[:, 9]
    below = (lb <= dk[:, None]).sum(1)
    assert below.max() < 96
