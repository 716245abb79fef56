"""The MFMA operand write-after-read guard, checked on the built code objects
(CPU only: disassembly, no GPU).

hipcc may allocate a VALU result onto an A / B register of an MFMA that is
still reading it (round 2: a wrong accumulator block in ~1 % of cosine
searches).  tools/check_mfma_war.py walks every kernel of every gfx950 code
object in duckdb-lancedb_amd/lib/*.o and reports a VALU write into a live A / B
register after the MFMAs that end a run (the tile-final MFMAs, where
mfma_operand_guard() sits in scan8_kernel, scan_kernel and the IVF kernels).
A new register allocation that reintroduces the hazard fails this test."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJS = sorted(glob.glob(os.path.join(ROOT, "duckdb-lancedb_amd", "lib", "*.o")))
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.mark.skipif(not OBJS or not os.path.exists(os.path.join(LLVM, "llvm-objdump")),
                    reason="needs the built objects (make) and the ROCm LLVM tools")
def test_no_valu_write_into_a_live_mfma_operand():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_mfma_war.py"), *OBJS],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    # every object with MFMAs was really disassembled
    kernels_with_mfma = [ln for ln in r.stdout.splitlines() if "MFMAs," in ln]
    assert any(ln.startswith("scan8_kernels.o") for ln in kernels_with_mfma), r.stdout
    assert any(ln.startswith("knn_kernels.o") for ln in kernels_with_mfma), r.stdout
