"""CPU restatement of the int8 scan's bound and of scan8's integer screen
(knn_kernels.hip tiles_to_i8_kernel / prep_queries_i8_kernel, scan8_kernels.hip
s8_row_part / s8_query_part), in numpy f64 with the kernels' f32
roundings:

    rows: v = x (l2, dot) or x/|x| (cosine); one scale per 256-row tile
          s_T = f32(max over the tile of max|v_i| / 127), x^ = rint(v / s_T), x~ = s_T x^
    queries: one scale for the batch, s_Q likewise
    |v.q - s_T s_Q (x^.q^)| <= |e_x||q| + |x~||e_q|

so LB = alpha + C + xn B + ux A + s s_T S never exceeds the exact distance the
reference ranks by (lance_manager.rs:393-451: squared L2, 1 - x.q, 1 - cos), and
the integer screen acc = s - Bi >= Gi passes every (row, query) with LB <= tau
(Bi, Gi rounded down from the tile's maxima).  Distributions where common
scales are worst: heavy tails, one dominant coordinate, near-constant rows,
tiny and huge norms, small integers.  (The GPU tests check the kernels end to end
against the f64 oracle; this pins the algebra, the exact-integer claim and the
screen's rounding margins.)"""
import numpy as np
import pytest

U = 2.0 ** -23
UP = 1.0 + 4.0 * U
BIG, LIVE_MAX, GLO = 1 << 30, 1 << 29, -(1 << 29) - (1 << 25)
f32 = np.float32


def fma32(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f32)


def quant_tiles(X, metric, tile=256):
    """tiles_to_i8_kernel: -> int rows, per-row (alpha, xn, ux, sc) f32, per-tile (s_T, max xn, max ux)"""
    X64 = X.astype(np.float64)
    xn = np.linalg.norm(X64, axis=1)
    V = X64 / np.where(xn > 0, xn, 1)[:, None] if metric == "cosine" else X64
    n = len(X)
    Xh = np.zeros_like(V)
    aux = np.zeros((n, 4), f32)
    tst = []
    for t0 in range(0, n, tile):
        sl = slice(t0, min(n, t0 + tile))
        rmax = np.abs(X[sl]).max(1).astype(np.float64)
        if metric == "cosine":
            rmax = np.where(xn[sl] > 0, (rmax / np.where(xn[sl] > 0, xn[sl], 1)).astype(f32), 0)
        M = f32(rmax.max())
        sT = f32(M / f32(127.0))
        inv = 127.0 / float(M) if M > 0 else 0.0
        q = np.clip(np.rint(V[sl] * inv), -127, 127)
        Xh[sl] = q
        xt = float(sT) * q
        e = V[sl] - xt
        ex = np.linalg.norm(e, axis=1) * UP + (2.0 ** -40 if metric == "cosine" else 0.0)
        ut = np.linalg.norm(xt, axis=1) * UP
        al = (xn[sl] ** 2).astype(f32) if metric == "l2" else np.zeros(len(q), f32)
        if metric == "cosine":
            al = np.where(xn[sl] > 0, al, np.nan).astype(f32)
        aux[sl] = np.stack([al, ex.astype(f32), ut.astype(f32), np.full(len(q), sT)], 1)
        tst.append((sT, aux[sl, 1].max(), aux[sl, 2].max()))
    return Xh, aux, np.array(tst, f32)


def quant_queries(Q, metric, max_alpha, max_x):
    """query_absmax_kernel + prep_queries_i8_kernel: -> int queries, per-query (S, A, B, C) f32"""
    Q64 = Q.astype(np.float64)
    qn = np.linalg.norm(Q64, axis=1)
    qn32 = qn.astype(f32).astype(np.float64)
    V = Q64 / np.where(qn32 > 0, qn32, 1)[:, None] if metric == "cosine" else Q64
    m = np.abs(Q).max(1).astype(np.float64)
    if metric == "cosine":
        m = np.where(qn > 0, (m / np.where(qn > 0, qn, 1)).astype(f32), 0)
    M = f32(m.max())
    sq = f32(M / f32(127.0))
    inv = 127.0 / float(M) if M > 0 else 0.0
    Qh = np.clip(np.rint(V * inv), -127, 127)
    e2 = ((V - float(sq) * Qh) ** 2).sum(1)
    s2 = (Q64 ** 2).sum(1)
    qnu = np.sqrt(s2) * UP
    equ = np.sqrt(e2) * UP + ((2.0 ** -20) * (1 + np.sqrt(e2)) if metric == "cosine" else 0.0)
    if metric == "l2":
        slack = 16 * U * (max_alpha + s2 + 4 * max_x * (qnu + equ)) + 1e-30
        qa = np.stack([np.full(len(Q), -2 * sq), -2 * equ, -2 * qnu, s2 - slack], 1)
    elif metric == "dot":
        slack = 16 * U * (1 + 4 * max_x * (qnu + equ)) + 1e-30
        qa = np.stack([np.full(len(Q), -sq), -equ, -qnu, 1 - slack], 1)
    else:
        vn = 1 + 2.0 ** -20
        slack = 16 * U * (2 + 4 * max_x * (vn + equ)) + 1e-30
        qa = np.stack([np.full(len(Q), -sq), -equ, np.full(len(Q), -vn * UP), 1 - slack], 1)
    return Qh, qa.astype(f32)


def row_part(alpha, W):
    """s8_row_part"""
    with np.errstate(invalid="ignore", over="ignore"):
        b = (alpha * W).astype(f32)
        b = (fma32(-np.abs(b), f32(2.0 ** -20), b) - f32(1)).astype(f32)
        b = np.where(np.isnan(b), 0, np.minimum(np.maximum(b, 0), LIVE_MAX))
    out = b.astype(np.int64)
    return np.where(alpha < np.inf, out, BIG)


def query_part(qa, tq, ts, W):
    """s8_query_part"""
    with np.errstate(invalid="ignore", over="ignore"):
        cmt = (qa[:, 3] - tq).astype(f32)
        g = (fma32(ts[1], qa[:, 2], fma32(ts[2], qa[:, 1], cmt)) * W).astype(f32)
        E = ((np.abs(qa[:, 3]) + np.abs(tq) + ts[1] * np.abs(qa[:, 2]) + ts[2] * np.abs(qa[:, 1])) * W
             * f32(2.0 ** -20) + f32(1)).astype(f32)
        g = (g - E).astype(f32)
        gi = np.floor(np.clip(np.where(np.isfinite(g), g, 0), GLO, BIG)).astype(np.int64)
    gi = np.where(np.isfinite(g), gi, GLO)
    return np.where(np.isnan(cmt) | (cmt == np.inf), BIG, gi)


def bounds(X, Q, metric, tile=256):
    Xh, aux, tst = quant_tiles(X, metric, tile)
    max_alpha = float(np.nanmax(np.abs(aux[:, 0])))
    max_x = float(np.nanmax(np.maximum(aux[:, 1], aux[:, 2])))
    Qh, qa = quant_queries(Q, metric, max_alpha, max_x)
    S = Qh @ Xh.T
    assert np.abs(S).max() < 2 ** 24            # exact in f32 and in the i32 accumulators
    X64, Q64 = X.astype(np.float64), Q.astype(np.float64)
    dot = Q64 @ X64.T
    xn, qn = np.linalg.norm(X64, axis=1), np.linalg.norm(Q64, axis=1)
    if metric == "l2":
        exact = (xn ** 2)[None, :] + (qn ** 2)[:, None] - 2 * dot
    elif metric == "dot":
        exact = 1 - dot
    else:
        exact = 1 - dot / (qn[:, None] * xn[None, :])
    a = aux.astype(np.float64)
    q = qa.astype(np.float64)
    lb = a[None, :, 0] + q[:, None, 3] + a[None, :, 1] * q[:, None, 2] + a[None, :, 2] * q[:, None, 1] \
        + S * a[None, :, 3] * q[:, None, 0]
    return lb, exact, S, aux, tst, qa


def datasets(rng, d, n=512):
    yield "gauss", rng.standard_normal((n, d)).astype(f32)
    yield "heavy", rng.standard_cauchy((n, d)).clip(-1e4, 1e4).astype(f32)
    spike = rng.standard_normal((n, d)).astype(f32) * 1e-3
    spike[np.arange(n), rng.integers(0, d, n)] = 50.0
    yield "spike", spike
    yield "near_const", (3.0 + 1e-4 * rng.standard_normal((n, d))).astype(f32)
    yield "tiny", (1e-20 * rng.standard_normal((n, d))).astype(f32)
    yield "huge", (1e15 * rng.standard_normal((n, d))).astype(f32)
    yield "sparse_int", rng.integers(-3, 4, (n, d)).astype(f32)
    mixed = rng.standard_normal((n, d)).astype(f32)
    mixed[: n // 2] *= 100.0  # two norm scales in one tile: the common scale's worst case
    yield "mixed_norms", mixed


def queries(rng, X, d):
    return np.concatenate([X[:40] + 0.01 * rng.standard_normal((40, d)).astype(f32),
                           rng.standard_normal((24, d)).astype(f32) * np.abs(X).max()])


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("d", [128, 768, 1024])
def test_i8_bound_is_rigorous(metric, d):
    rng = np.random.default_rng(d)
    for name, X in datasets(rng, d):
        Q = queries(rng, X, d)
        lb, exact, *_ = bounds(X, Q, metric)
        scale = np.abs(exact).max() + 1e-300
        ok = np.isnan(lb) | (lb <= exact + 1e-9 * scale)
        assert ok.all(), (name, metric, float(np.nanmax((lb - exact) / scale)))


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
@pytest.mark.parametrize("d", [512, 768, 1024])
def test_scan8_screen_passes_every_bound_below_tau(metric, d):
    """acc = s - Bi >= Gi for every (row, query) with LB <= tau, per tile, at taus
    that put the cut inside the bound distribution, at +inf and at NaN / -inf."""
    rng = np.random.default_rng(7 + d)
    for name, X in datasets(rng, d):
        Q = queries(rng, X, d)
        lb, exact, S, aux, tst, qa = bounds(X, Q, metric)
        Sabs = f32(np.max(-qa[:, 0]))
        fin = np.isfinite(lb)
        for pct in (0.1, 1.0, 10.0):
            tau = np.array([np.percentile(r[np.isfinite(r)], pct) if np.isfinite(r).any() else np.inf
                            for r in lb], f32)
            for t in range(len(tst)):
                sl = slice(256 * t, 256 * t + 256)
                sT = tst[t][0]
                with np.errstate(divide="ignore", over="ignore"):
                    W = f32(1) / f32(Sabs * sT) if (Sabs > 0 and sT > 0) else f32(0)
                bi = row_part(aux[sl, 0], W)
                gi = query_part(qa, tau, tst[t], W)
                acc = S[:, sl].astype(np.int64) - bi[None, :]
                passed = acc >= gi[:, None]
                must = fin[:, sl] & (lb[:, sl] <= tau[:, None])
                assert (passed | ~must).all(), (name, metric, pct, t)
        # tau = +inf passes every live row; a NaN tau or -inf passes nothing
        for tq, want in ((np.inf, True), (np.nan, False), (-np.inf, False)):
            W = f32(1) / f32(Sabs * tst[0][0]) if (Sabs > 0 and tst[0][0] > 0) else f32(0)
            gi = query_part(qa[:1], np.array([tq], f32), tst[0], W)
            bi = row_part(aux[:256, 0], W)
            acc = S[:1, :256].astype(np.int64) - bi[None, :]
            live = np.isfinite(aux[:256, 0])
            assert ((acc >= gi[:, None])[0][live] == want).all(), (name, metric, tq)


def test_scan8_screen_rejects_dead_rows():
    # a tombstone (alpha = +inf) never passes, whatever tau: acc <= 2^24 - BIG < GLO
    aux0 = np.array([np.inf, np.nan], f32)
    bi = row_part(aux0, f32(3.0))
    assert (bi == BIG).all()
    assert (2 ** 24 - BIG) < GLO


def test_i8_bound_tightness_gaussian():
    # the reason the selection refines k + 96 / k + 192 candidates:
    # the slack is a fraction of the distance spread for N(0,1) rows at d = 768
    rng = np.random.default_rng(0)
    X = rng.standard_normal((4096, 768)).astype(f32)
    Q = rng.standard_normal((16, 768)).astype(f32)
    lb, exact, *_ = bounds(X, Q, "l2")
    gap = exact - lb
    spread = exact.std(1).mean()
    assert (gap >= 0).all()
    assert 0.05 < gap.mean() / spread < 1.0, gap.mean() / spread
