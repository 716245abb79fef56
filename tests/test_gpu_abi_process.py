"""GPU: the drop-in driven the way a DuckDB process loads it.

``tests/cpp/abi_caller.cpp`` is a C++ program that re-declares the reference's
``extern "C"`` backend symbols (``rust_ffi.cpp:7-42``), restates the
``rust_ffi.cpp`` wrappers and the hot-path subset of ``lance_index.cpp``
(Append / Delete / Search with its label -> row id map, CHECKPOINT + restart),
links ``liblancedb_hip.so`` and never loads torch.  It therefore runs the
library on the HIP runtime the library links (``/opt/rocm``'s
``libamdhip64.so.7``, what ``CMakeLists.txt:117-121``'s link swap gives
DuckDB), not on torch's bundled copy that every in-process test uses.

Each test writes a command script (and binary inputs), runs the program as its
own process, and checks its output against the reference's goldens
(``tests/golden/sql_goldens.json``) or the f64 oracle (the checker only).
"""
import json
import math
import os
import subprocess

import numpy as np
import pytest

from oracle import flat_knn
from tests.golden_runner import check_expect, check_filter_result, gen, hnsw_rows, load_seeded, load_sql_goldens, seeded_inputs

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RTOL = 1e-4
ATOL = 1e-5


@pytest.fixture(scope="module")
def caller(tmp_path_factory, hip):
    src = os.path.join(ROOT, "tests", "cpp", "abi_caller.cpp")
    exe = str(tmp_path_factory.mktemp("abi") / "abi_caller")
    libdir = os.path.dirname(hip.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", src, "-o", exe, f"-L{libdir}", "-llancedb_hip",
                    f"-Wl,-rpath,{libdir}"], check=True, timeout=120)
    return exe


def run(exe, tmp_path, lines, timeout=240, devices=None, tie=None):
    """devices: LANCE_HIP_DEVICES for the process (e.g. "0,0": every handle it
    creates or opens is row-sharded over two stores on device 0, shards.cpp);
    tie: LANCE_HIP_TIE (the final order's tie rule; unset = label_desc)."""
    script = tmp_path / "script.txt"
    script.write_text("\n".join(lines) + "\n")
    env = dict(os.environ)
    env.pop("LANCE_HIP_DEVICES", None)
    env.pop("LANCE_HIP_TIE", None)
    if devices:
        env["LANCE_HIP_DEVICES"] = devices
    if tie:
        env["LANCE_HIP_TIE"] = tie
    r = subprocess.run([exe, "gpu", str(script)], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout.splitlines()
    assert out and out[-1] == "done", r.stdout + r.stderr
    errs = [l for l in out if l.startswith("error")]
    return out[:-1], errs


def fl(a):
    return " ".join(repr(float(x)) for x in np.asarray(a, np.float32).reshape(-1))


def parse_res(line):
    t = line.split()
    assert t[0] == "res", line
    n = int(t[1])
    return [(int(t[2 + 2 * i]), float(t[3 + 2 * i])) for i in range(n)]


def test_process_maps_opt_rocm_runtime_and_no_torch(caller, tmp_path):
    out, errs = run(caller, tmp_path, ["index 3 l2 - vectors", "append 1 0 1 0 0",
                                       "search 1 3 1 0 0", "maps"])
    assert not errs, errs
    maps = [l.split(None, 1)[1] for l in out if l.startswith("maps ")]
    hip_rt = {m for m in maps if "libamdhip64" in m}
    assert len(hip_rt) == 1, maps
    rt = hip_rt.pop()
    assert rt.startswith("/opt/rocm"), rt            # the runtime the .so links, not torch's bundled copy
    assert "torch" not in rt and "site-packages" not in rt, rt
    assert "torch 0" in out, out
    assert parse_res(out[0]) == [(0, 0.0)]


# ---------------------------------------------------------------------------
# the reference's SQL goldens through the C++ LanceIndex restatement
# ---------------------------------------------------------------------------
INDEX_CASES = [c for c in load_sql_goldens() if "steps" in c and not c["name"].startswith("rust_")]


@pytest.mark.parametrize("devices", [None, "0,0"], ids=["one_store", "two_shards"])
@pytest.mark.parametrize("case", INDEX_CASES, ids=[c["name"] for c in INDEX_CASES])
def test_sql_goldens_in_torch_free_process(caller, tmp_path, case, devices):
    lines = [f"index {case['dim']} l2 {tmp_path / 'db.lance' / case['name']} vectors"]
    checks = []
    for st in case["steps"]:
        op = st["op"]
        if op == "append":
            rows = np.array(st["rows"], np.float32)
            lines.append(f"append {len(rows)} {' '.join(map(str, st['row_ids']))} {fl(rows)}")
        elif op == "append_hnsw_rows":
            rows = hnsw_rows(st["n"])
            lines.append(f"append {len(rows)} {' '.join(map(str, range(st['n'])))} {fl(rows)}")
        elif op == "create_hnsw":
            lines.append(f"hnsw {st['m']} {st['ef']}")
        elif op == "delete":
            lines.append(f"delete {len(st['row_ids'])} {' '.join(map(str, st['row_ids']))}")
        elif op == "restart":
            lines.append("restart")
        elif op in ("search", "count_search"):
            q = np.array(st["q"], np.float32)
            lines.append(f"search {st['k']} {len(q)} {fl(q)}")
            checks.append(st)
        else:
            raise ValueError(op)
    out, errs = run(caller, tmp_path, lines, devices=devices)
    assert not errs, errs
    res = [parse_res(l) for l in out if l.startswith("res")]
    assert len(res) == len(checks)
    for st, r in zip(checks, res):
        where = st.get("ref", case["ref"])
        if "expect" in st:
            check_expect(r, st["expect"], where)
        if "expect_ids" in st:
            assert [x for x, _ in r] == st["expect_ids"], (where, r)
        if "expect_count" in st:
            assert len(r) == st["expect_count"], (where, r)
        if "expect_count_gt" in st:
            assert len(r) > st["expect_count_gt"], (where, r)


@pytest.mark.parametrize("tie", [None, "label_asc"], ids=["tie_default", "tie_asc"])
@pytest.mark.parametrize("devices", [None, "0,0"], ids=["one_store", "two_shards"])
def test_filter_goldens_through_arrow_in_torch_free_process(caller, tmp_path, devices, tie):
    # lance_optimizer_filter.test:9-99: CREATE INDEX .. USING LANCE (embedding, lang, score), rows handed over
    # through the Arrow C Data Interface, each WHERE pushed down as a Lance predicate.  Default tie rule
    # (label_desc): every answer verbatim, including :36-44's tie (ids 3 and 4 at d = 2.0 -> 4)
    case = next(c for c in load_sql_goldens() if c["name"] == "filter_pushdown")
    rows = np.array(case["rows"], np.float32)
    lines = [f"index 3 l2 {tmp_path / 'docs'} docs_idx cols",
             f"append_cols {len(rows)} {' '.join(map(str, range(len(rows))))} {fl(rows)} "
             f"{' '.join(case['lang'])} {' '.join(map(str, case['score']))}"]
    for query in case["queries"]:
        lines.append(f"search {query['k']} 3 1 0 0" + (f" | {query['where']}" if query["where"] else ""))
    lines.append("restart")  # the metadata columns persist with the table log
    for query in case["queries"]:
        lines.append(f"search {query['k']} 3 1 0 0" + (f" | {query['where']}" if query["where"] else ""))
    out, errs = run(caller, tmp_path, lines, devices=devices, tie=tie)
    assert not errs, errs
    res = [parse_res(l) for l in out if l.startswith("res")]
    assert len(res) == 2 * len(case["queries"])
    for i, r in enumerate(res):
        check_filter_result(case["queries"][i % len(case["queries"])], [case["ids"][rid] for rid, _ in r],
                            tie or "label_desc")
    if tie is None:  # the reference's tie golden, verbatim
        q = next(i for i, x in enumerate(case["queries"]) if x["where"] == "score > 20")
        assert [case["ids"][rid] for rid, _ in res[q]] == [5, 4]


def test_rust_label_goldens_in_torch_free_process(caller, tmp_path):
    # lance_manager.rs:779-867 through the raw C-ABI
    p, p2, p3 = tmp_path / "t.lance", tmp_path / "e.lance", tmp_path / "tbl.lance"
    lines = [f"raw_create a 3 {p} vectors"] + [f"raw_add a 3 {i} 0 0" for i in range(5)] + [
        "raw_delete a 1", "raw_delete a 2", "raw_free a", f"raw_open a {p} vectors", "raw_add a 3 99 0 0",
        "raw_free a",
        f"raw_create e 2 {p2} vectors", "raw_free e", f"raw_open e {p2} vectors", "raw_add e 2 1 2", "raw_free e",
        f"raw_create x 2 {p3} idx_a", f"raw_create y 2 {p3} idx_b", "raw_add x 2 1 0", "raw_add x 2 2 0",
        "raw_add y 2 10 0", "raw_count x", "raw_count y", "raw_free x", "raw_free y",
        f"raw_open x {p3} idx_a", f"raw_open y {p3} idx_b", "raw_count x", "raw_count y"]
    out, errs = run(caller, tmp_path, lines)
    assert not errs, errs
    labels = [int(l.split()[1]) for l in out if l.startswith("label")]
    counts = [int(l.split()[1]) for l in out if l.startswith("count")]
    assert labels[:5] == [0, 1, 2, 3, 4]          # :786-790
    assert labels[5] >= 5                          # :796-803
    assert labels[6] == 0                          # empty reopen (:806-818)
    assert counts == [2, 1, 2, 1]                  # two tables in one dataset (:843-867)


# ---------------------------------------------------------------------------
# seeded fixtures and the f64 oracle through the C++ caller
# ---------------------------------------------------------------------------
def read_out(path, nq, k):
    b = open(path, "rb").read()
    L = np.frombuffer(b[:nq * k * 8], np.int64).reshape(nq, k)
    D = np.frombuffer(b[nq * k * 8:nq * k * 12], np.float32).reshape(nq, k)
    C = np.frombuffer(b[nq * k * 12:nq * k * 12 + nq * 4], np.int32)
    return L, D, C


def check(L, D, C, el, ed, ec=None):
    if ec is not None:
        np.testing.assert_array_equal(C, ec)
    for i in range(el.shape[0]):
        n = int(C[i])
        np.testing.assert_array_equal(L[i, :n], el[i, :n], err_msg=f"query {i}")
        np.testing.assert_allclose(D[i, :n], ed[i, :n], rtol=RTOL, atol=ATOL, err_msg=f"query {i}")


@pytest.mark.parametrize("metric", ["l2", "dot", "cosine"])
def test_knn_small_fixture_in_torch_free_process(caller, tmp_path, metric):
    z = np.load(os.path.join(ROOT, "tests", "golden", "knn_small.npz"))
    X, Q, live = z["X"], z["Q"], z["live"]
    k = z["l2_labels"].shape[1]
    X.tofile(tmp_path / "x.bin")
    Q.tofile(tmp_path / "q.bin")
    dead = np.nonzero(~live)[0].astype(np.int64)
    dead.tofile(tmp_path / "del.bin")
    lines = [f"bulk {X.shape[1]} {metric} {tmp_path / 'x.bin'} {len(X)} 2048",
             f"bulk_delete {tmp_path / 'del.bin'} {len(dead)}",
             f"bulk_search {tmp_path / 'q.bin'} {len(Q)} {k} {tmp_path / 'pc.bin'} percall",
             f"bulk_search {tmp_path / 'q.bin'} {len(Q)} {k} {tmp_path / 'b.bin'} batch",
             # the predicate form (lance_index.cpp:452-453) on the implicit label column
             f"bulk_search {tmp_path / 'q.bin'} {len(Q)} {k} {tmp_path / 'pp.bin'} percall | label >= 500",
             f"bulk_search {tmp_path / 'q.bin'} {len(Q)} {k} {tmp_path / 'pb.bin'} batch | label < 300 OR label >= 700",
             "count"]
    out, errs = run(caller, tmp_path, lines)
    assert not errs, errs
    assert f"count {int(live.sum())}" in out
    el, ed = z[f"{metric}_labels"], z[f"{metric}_dists"]
    for f in ("pc.bin", "b.bin"):
        L, D, C = read_out(tmp_path / f, len(Q), k)
        check(L, D, C, el, ed)
    labels = np.arange(len(X))
    for f, sel in (("pp.bin", labels >= 500), ("pb.bin", (labels < 300) | (labels >= 700))):
        el2, ed2, ec2 = flat_knn.flat_search_batch(X, labels, live & sel, Q, k, metric=metric)
        L, D, C = read_out(tmp_path / f, len(Q), k)
        check(L, D, C, el2, ed2, ec2)


@pytest.mark.parametrize("name", ["c1_10k_d128", "n100k_d768_l2"])
def test_seeded_fixture_in_torch_free_process(caller, tmp_path, name):
    # c1_10k_d128: configs[0] (lance_search() flat L2, 10k x 128, k = 10) one query per call;
    # n100k_d768_l2: past the dense path (threshold sample + int8 append scan + refine), batched and per call
    spec = next(s for s in load_seeded() if s["name"] == name)
    X, Q, exp = seeded_inputs(spec)
    k = spec["k"]
    X.tofile(tmp_path / "x.bin")
    Q.tofile(tmp_path / "q.bin")
    lines = [f"bulk {spec['d']} {spec['metric']} {tmp_path / 'x.bin'} {spec['n']} 2048",
             f"bulk_search {tmp_path / 'q.bin'} {spec['nq']} {k} {tmp_path / 'pc.bin'} percall",
             f"bulk_search {tmp_path / 'q.bin'} {spec['nq']} {k} {tmp_path / 'b.bin'} batch"]
    out, errs = run(caller, tmp_path, lines, timeout=600)
    assert not errs, errs
    for f in ("pc.bin", "b.bin"):
        L, D, C = read_out(tmp_path / f, spec["nq"], k)
        check(L, D, C, exp["labels"], exp["dists"], exp["counts"])


@pytest.mark.parametrize("devices", [None, "0,0"], ids=["one_store", "two_shards"])
def test_deletes_and_appends_in_torch_free_process(caller, tmp_path, devices):
    # 90k x 128 rows in DuckDB's 2048-row Sink chunks, a third deleted, then searched per call and batched;
    # two_shards: the process sets LANCE_HIP_DEVICES, the handle row-shards the chunks over two stores
    rng = np.random.default_rng(77)
    n, d, nq, k = 90_000, 128, 24, 10
    X = gen(31, n, d)
    Q = gen(32, nq, d)
    dead = np.sort(rng.choice(n, n // 3, replace=False)).astype(np.int64)
    live = np.ones(n, bool)
    live[dead] = False
    X.tofile(tmp_path / "x.bin")
    Q.tofile(tmp_path / "q.bin")
    dead.tofile(tmp_path / "del.bin")
    lines = [f"bulk {d} l2 {tmp_path / 'x.bin'} {n} 2048", f"bulk_delete {tmp_path / 'del.bin'} {len(dead)}",
             f"bulk_search {tmp_path / 'q.bin'} {nq} {k} {tmp_path / 'pc.bin'} percall",
             f"bulk_search {tmp_path / 'q.bin'} {nq} {k} {tmp_path / 'b.bin'} batch", "count"]
    out, errs = run(caller, tmp_path, lines, timeout=600, devices=devices)
    assert not errs, errs
    assert f"count {int(live.sum())}" in out
    el, ed, ec = flat_knn.flat_search_batch(X, np.arange(n), live, Q, k)
    for f in ("pc.bin", "b.bin"):
        L, D, C = read_out(tmp_path / f, nq, k)
        check(L, D, C, el, ed, ec)
