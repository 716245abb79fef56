"""CPU checks of the filtered-search predicate evaluator of the HIP library
(``lance_hip_predicate_mask``: Arrow C Data Interface import + Lance-SQL
predicate, ``duckdb-lancedb_amd/csrc/meta.cpp``) against ``oracle/predicate.py``
— no device needed.  Pinned by the reference's filter goldens
(``test/sql/lance_optimizer_filter.test:23-99``, predicates as
``src/lance_optimizer.cpp:204-344`` writes them) and by random predicates over
every supported column type with NULLs."""
import numpy as np
import pyarrow as pa
import pytest

import lance_hip
from oracle import predicate as P
from tests.golden_runner import eval_predicate, load_sql_goldens


def _mask(batch, labels, live, pred):
    return lance_hip.LanceHipPredicateMask(batch, labels, live, pred)


def test_filter_goldens_masks():
    case = next(c for c in load_sql_goldens() if c["name"] == "filter_pushdown")
    n = len(case["ids"])
    batch = lance_hip.arrow_rows(np.array(case["rows"], np.float32),
                                 [("lang", case["lang"], pa.string()), ("score", case["score"], pa.int32())])
    labels = np.arange(n)
    live = np.ones(n, np.uint8)
    for q in case["queries"]:
        if q["where"] is None:
            continue
        got = _mask(batch, labels, live, q["where"])
        exp = [eval_predicate(q["where"], lang, sc) for lang, sc in zip(case["lang"], case["score"])]
        assert got.tolist() == exp, q


def _table(rng, n):
    def nulls(vals, p=0.15):
        return [None if rng.random() < p else v for v in vals]

    words = ["en", "fr", "es", "it's", "", "de", "EN", "zz"]
    cols = {
        "i32": nulls(rng.integers(-50, 50, n).tolist()),
        "i64": nulls((rng.integers(-3, 3, n) * 10**12).tolist()),
        "f32": nulls([float(np.float32(x)) for x in rng.normal(0, 10, n)]),
        "f64": nulls(rng.normal(0, 10, n).tolist()),
        "flag": nulls(rng.random(n).astype(bool).tolist()),
        "lang": nulls([words[i] for i in rng.integers(0, len(words), n)]),
    }
    types = {"i32": pa.int32(), "i64": pa.int64(), "f32": pa.float32(), "f64": pa.float64(), "flag": pa.bool_(),
             "lang": pa.string()}
    return cols, types


def _lit(rng, col):
    if col in ("i32", "label"):
        return str(int(rng.integers(-60, 60)))
    if col == "i64":
        return str(int(rng.integers(-3, 3)) * 10**12)
    if col in ("f32", "f64"):
        return repr(round(float(rng.normal(0, 10)), 3))
    if col == "flag":
        return "true" if rng.random() < 0.5 else "false"
    w = ["en", "fr", "es", "it''s", "", "de", "EN", "zz", "e"][int(rng.integers(0, 9))]
    return f"'{w}'"


def _atom(rng):
    col = ["i32", "i64", "f32", "f64", "flag", "lang", "label"][int(rng.integers(0, 7))]
    r = rng.random()
    if r < 0.5:
        op = ["=", "!=", "<", "<=", ">", ">="][int(rng.integers(0, 6))]
        if col == "flag":
            op = ["=", "!="][int(rng.integers(0, 2))]
        a, b = col, _lit(rng, col)
        return f"{b} {op} {a}" if rng.random() < 0.2 else f"{a} {op} {b}"
    if r < 0.65:
        return f"{col} IS {'NOT ' if rng.random() < 0.5 else ''}NULL"
    if r < 0.85:
        vals = [_lit(rng, col) for _ in range(int(rng.integers(1, 4)))]
        if rng.random() < 0.2:
            vals.append("NULL")
        return f"{col} {'NOT ' if rng.random() < 0.3 else ''}IN ({', '.join(vals)})"
    if col in ("flag",):
        return "flag"
    lo, hi = sorted([_lit(rng, col), _lit(rng, col)]) if col != "lang" else (_lit(rng, col), _lit(rng, col))
    return f"{col} {'NOT ' if rng.random() < 0.2 else ''}BETWEEN {lo} AND {hi}"


def _pred(rng, depth=0):
    r = rng.random()
    if depth >= 2 or r < 0.4:
        return _atom(rng)
    if r < 0.6:
        return f"NOT ({_pred(rng, depth + 1)})"
    if r < 0.8:
        return f"{_pred(rng, depth + 1)} AND {_pred(rng, depth + 1)}"
    return f"({_pred(rng, depth + 1)}) OR ({_pred(rng, depth + 1)})"


def test_random_predicates_match_oracle():
    rng = np.random.default_rng(7)
    n = 600
    cols, types = _table(rng, n)
    X = rng.standard_normal((n, 4)).astype(np.float32)
    batch = lance_hip.arrow_rows(X, [(k, cols[k], types[k]) for k in cols])
    labels = np.arange(n, dtype=np.int64) * 2 + 3
    live = (rng.random(n) > 0.1).astype(np.uint8)
    checked = 0
    for _ in range(400):
        pred = _pred(rng)
        exp = P.mask(pred, cols, labels, live)
        got = _mask(batch, labels, live, pred)
        assert got.tolist() == exp, pred
        checked += 1
    assert checked == 400


def test_scalar_index_path_matches_oracle():
    # every column through the sorted-permutation scalar index
    # (lance_detached_create_scalar_index): identical masks
    rng = np.random.default_rng(9)
    n = 700
    cols, types = _table(rng, n)
    X = rng.standard_normal((n, 4)).astype(np.float32)
    batch = lance_hip.arrow_rows(X, [(k, cols[k], types[k]) for k in cols])
    labels = np.arange(n, dtype=np.int64)
    live = (rng.random(n) > 0.1).astype(np.uint8)
    for _ in range(300):
        pred = _pred(rng)
        exp = P.mask(pred, cols, labels, live)
        got = lance_hip.LanceHipPredicateMask(batch, labels, live, pred, indexed_columns=list(cols))
        assert got.tolist() == exp, pred


def test_literal_forms_and_offsets():
    # sliced struct arrays (non-zero Arrow offsets), large_string, quoted names,
    # keyword case, constant-only predicates
    n = 50
    X = np.zeros((n, 2), np.float32)
    names = [f"n{i % 7}" for i in range(n)]
    batch = lance_hip.arrow_rows(X, [("name", pa.array(names, pa.large_string()), None),
                                     ("v", list(range(n)), pa.int16())]).slice(10, 30)
    labels = np.arange(30)
    live = np.ones(30, np.uint8)
    cols = {"name": names[10:40], "v": list(range(10, 40))}
    for pred in ["name = 'n3'", "\"name\" in ('n1','n2')", "v between 12 and 20", "v not between 12 and 20",
                 "1 = 1", "NULL = 1", "true", "label >= 5 and v < 30", "v <> 15", "name >= 'n5' or v = 39",
                 "v = 12.0", "v < 12.5", "-3 < v"]:
        assert _mask(batch, labels, live, pred).tolist() == P.mask(pred, cols, labels, live), pred


@pytest.mark.parametrize("bad", ["nosuchcol = 1", "lang = ", "lang = 'x", "(lang = 'a'", "lang === 'a'",
                                 "lang = 1", "score = 'a'"])
def test_errors(bad):
    batch = lance_hip.arrow_rows(np.zeros((3, 2), np.float32), [("lang", ["a", "b", None], pa.string()),
                                                                 ("score", [1, 2, 3], pa.int32())])
    with pytest.raises(lance_hip.IOException):
        _mask(batch, np.arange(3), np.ones(3, np.uint8), bad)
