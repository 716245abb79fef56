"""CPU: the C-ABI library loads, exports every symbol include/lancedb_hip.h
declares, and keeps ffi.rs's error conventions on paths that touch no GPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import lance_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lancedb_hip.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lance_\w+)\s*\(", src)))


def test_header_declares_reference_ffi_symbols():
    # the 19 extern "C" declarations of /root/reference/src/rust_ffi.cpp:9-41
    ref = ["lance_create_detached", "lance_create_detached_from_arrow", "lance_open_detached", "lance_free_detached",
           "lance_detached_has_extra_columns", "lance_detached_dimension", "lance_detached_add",
           "lance_detached_add_batch", "lance_detached_add_batch_arrow", "lance_detached_merge",
           "lance_detached_search", "lance_detached_count", "lance_detached_delete", "lance_detached_delete_batch",
           "lance_detached_create_index", "lance_detached_create_hnsw_index", "lance_detached_compact",
           "lance_detached_get_vector", "lance_detached_get_all_vectors"]
    syms = header_symbols()
    for s in ref:
        assert s in syms, s


def test_library_exports_every_header_symbol():
    L = lance_hip.lib()
    for s in header_symbols():
        assert hasattr(L, s), f"{s} declared in lancedb_hip.h but not exported"
    out = subprocess.run(["nm", "-D", "--defined-only", lance_hip.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (lance_\w+)", out))
    for s in header_symbols():
        assert s in exported, s


def test_python_binding_covers_header():
    assert set(header_symbols()) <= set(lance_hip.EXPORTED_SYMBOLS)


def test_version_string():
    assert "gfx950" in lance_hip.version()


def _null_call(name, *args):
    L = lance_hip.lib()
    e = ctypes.create_string_buffer(2048)
    r = getattr(L, name)(None, *args, e, 2048)
    return r, e.value.decode()


def test_null_handle_errors_match_ffi_rs():
    # ffi.rs:156-159 etc: "null handle" + -1
    q = np.zeros(3, np.float32)
    lab = np.zeros(4, np.int64)
    dist = np.zeros(4, np.float32)
    assert _null_call("lance_detached_add", q.ctypes.data, 3) == (-1, "null handle")
    assert _null_call("lance_detached_add_batch", q.ctypes.data, 1, 3, lab.ctypes.data) == (-1, "null handle")
    assert _null_call("lance_detached_search", q.ctypes.data, 3, 4, 20, 1, lab.ctypes.data,
                      dist.ctypes.data) == (-1, "null handle")
    assert _null_call("lance_detached_count") == (-1, "null handle")
    assert _null_call("lance_detached_delete", 1) == (-1, "null handle")
    assert _null_call("lance_detached_delete_batch", lab.ctypes.data, 1) == (-1, "null handle")
    assert _null_call("lance_detached_create_index", 4, 2) == (-1, "null handle")
    assert _null_call("lance_detached_create_hnsw_index", 4, 2) == (-1, "null handle")
    assert _null_call("lance_detached_compact") == (-1, "null handle")
    assert _null_call("lance_detached_get_vector", 0, dist.ctypes.data, 4) == (-1, "null handle")
    L = lance_hip.lib()
    assert L.lance_detached_dimension(None) == 0
    assert L.lance_detached_has_extra_columns(None) == 0
    L.lance_free_detached(None)  # null-safe (ffi.rs:137-142)


def test_wrappers_raise_ioexception_like_rust_ffi_cpp():
    with pytest.raises(lance_hip.IOException, match="^Lance count: null handle"):
        lance_hip.LanceDetachedCount(None)
    with pytest.raises(lance_hip.IOException, match="^Lance search: null handle"):
        lance_hip.LanceDetachedSearch(None, np.zeros(3, np.float32), 3, 1)


def test_error_buffer_truncation():
    # ffi.rs:15-24: message truncated to err_buf_len-1 and NUL terminated
    L = lance_hip.lib()
    e = ctypes.create_string_buffer(b"\xff" * 6, 6)
    r = L.lance_detached_count(None, e, 5)
    assert r == -1
    assert e.raw[:5] == b"null\x00"


def test_arrow_paths_report_unsupported():
    L = lance_hip.lib()
    e = ctypes.create_string_buffer(2048)
    assert L.lance_create_detached_from_arrow(b"/tmp/x", None, b"l2", b"t", e, 2048) is None
    assert e.value == b"null arrow schema"


@pytest.mark.skipif(lance_hip.device_count() > 0, reason="a HIP device is present")
def test_create_without_gpu_fails_cleanly():
    with pytest.raises(lance_hip.IOException, match="no HIP device"):
        lance_hip.LanceCreateDetached("", 3, "l2", "vectors")


def test_cpp_caller_links_against_library(tmp_path):
    """A C++ caller with the reference's extern "C" declarations (rust_ffi.cpp:7-42)
    compiles, links against liblancedb_hip.so and runs (no GPU needed)."""
    src = os.path.join(ROOT, "tests", "cpp", "abi_caller.cpp")
    exe = str(tmp_path / "abi_caller")
    libdir = os.path.dirname(lance_hip.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", src, "-o", exe, f"-L{libdir}", "-llancedb_hip",
                    f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")


def test_one_hip_runtime_per_process():
    """lance_hip.lib() maps torch's bundled HIP runtime, never a second copy:
    two libamdhip64 / libhsa-runtime64 in one process leave the one initialised
    second without a device (GPU suite: 'No HIP GPUs are available')."""
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r)\n"
            "import lance_hip; lance_hip.lib()\n"
            "import torch\n"
            "m = open('/proc/self/maps').read().splitlines()\n"
            "print(len({l.split()[-1] for l in m if 'libamdhip64' in l}))\n") % (os.path.join(ROOT, "duckdb-lancedb_amd"),)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "1", out.stdout
