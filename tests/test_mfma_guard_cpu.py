"""The MFMA operand write-after-read guard, checked on the built code objects
(CPU only: disassembly, no GPU).

hipcc may allocate a VALU result onto an A / B register of an MFMA that is
still reading it (round 2: a wrong accumulator block in ~1 % of cosine
searches).  tools/check_mfma_war.py walks every kernel of every gfx950 code
object in duckdb-lancedb_amd/lib/*.o and reports a VALU write into a live A / B
register after the MFMAs that end a run (the tile-final MFMAs, where
mfma_operand_guard() sits in scan8_kernel, scan_kernel and the IVF kernels).
Loads (VMEM / DS) writing a live A / B register are modelled at their minimum
return latency (tools/check_mfma_war.py LOAD_MIN_LATENCY).  A new register
allocation that reintroduces the hazard fails this test.

The release build carries no scan8 timing ablation: every scan8_kernel
instantiation in the code object has ABL = 0 and the ld = 768 default geometry
<12, 4, 2> (the wrong-result variants exist only in LHIP_ABLATION_BUILD builds)."""
import re
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
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_mfma_war.py"), "--list", *OBJS],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    # every object with MFMAs was really disassembled
    kernels_with_mfma = [ln for ln in r.stdout.splitlines() if "MFMAs," in ln]
    assert any(ln.startswith("scan8_kernels.o") for ln in kernels_with_mfma), r.stdout
    assert any(ln.startswith("knn_kernels.o") for ln in kernels_with_mfma), r.stdout
    assert any(ln.startswith("ivf_kernels.o") for ln in kernels_with_mfma), r.stdout
    # release scan8 instantiations: ABL = 0 only, ld = 768 only the default geometry
    s8 = set(re.findall(r"scan8_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", r.stdout))
    assert s8, r.stdout[-2000:]
    assert all(abl == "0" for (_, _, _, abl) in s8), sorted(s8)
    assert {(d, rb) for (ks, d, rb, _) in s8 if ks == "12"} == {("4", "2")}, sorted(s8)


def _kernel_metadata(obj):
    """{kernel symbol: (private_segment_fixed_size, vgpr_count)} of an object's gfx950 code object."""
    import tempfile

    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        fb, co = os.path.join(tmp, "fb.bin"), os.path.join(tmp, "co.elf")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", obj], check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"],
                       check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    name = None
    for ln in notes.splitlines():
        ln = ln.strip()
        if ln.startswith(".name:"):
            name = ln.split(":", 1)[1].strip()
        elif ln.startswith(".private_segment_fixed_size:") and name:
            out.setdefault(name, [0, 0])[0] = int(ln.split(":", 1)[1])
        elif ln.startswith(".vgpr_count:") and name:
            out.setdefault(name, [0, 0])[1] = int(ln.split(":", 1)[1])
    return out


@pytest.mark.skipif(not OBJS or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                    reason="needs the built objects (make) and the ROCm LLVM tools")
def test_hot_kernels_do_not_spill():
    """The hot kernels keep every value in registers: a scratch spill in
    pool_refine's final mode cost 69 -> 104 us per C2 batch (round 4), and the
    m = 96 PQ fast scan reloaded 88 B of spilled lane state at every item start
    (round 5), so a register-allocation change that spills fails here, before
    the GPU.  Covered: scan8 (C2 / north_star / C3), pool_refine (f32), the
    PQ fast scans (C5) and the IVF_FLAT bound scan (C4); round 6: the C5 step's
    fused kernels (coarse bounds / select, per-query tables, invert + item
    layout, run select)."""
    meta = {}
    for obj in OBJS:
        if os.path.basename(obj) in ("knn_kernels.o", "scan8_kernels.o", "ivf_kernels.o", "coarse_kernels.o"):
            meta.update(_kernel_metadata(obj))
    step = ("coarse_bounds_kernel", "coarse_select_kernel", "pq_lut_fused_kernel", "invert_fused_kernel",
            "pq_run_select_kernel")
    hot = [k for k in meta if ("pool_refine_kernel" in k and "Ef" in k) or "scan8_kernel" in k
           or "pq_fast_scan_bank_kernel" in k or "flat_list_lb_kernel" in k or any(s in k for s in step)]
    assert all(any(s in k for k in hot) for s in step), hot
    assert len(hot) >= 10, sorted(meta)[:20]
    assert sum("pq_fast_scan_bank_kernel" in k for k in hot) == 3, hot  # m = 32, 64, 96
    assert sum("flat_list_lb_kernel" in k for k in hot) == 3, hot       # l2, dot, cosine
    spills = {k: v for k, v in meta.items() if k in hot and v[0] != 0}
    assert not spills, spills


@pytest.mark.skipif(not OBJS or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                    reason="needs the built objects (make) and the ROCm LLVM tools")
def test_release_objects_carry_no_scan8_ablations():
    """The timing ablations of scan8_kernel (ABL != 0: no screen / no appends,
    wrong results by design) are not instantiated in a release build: every
    scan8_kernel<KS, D, RB, ABL, TM> of the built object has ABL == 0."""
    import re

    meta = {}
    for obj in OBJS:
        if os.path.basename(obj) == "scan8_kernels.o":
            meta.update(_kernel_metadata(obj))
    names = [k for k in meta if "scan8_kernel" in k]
    assert names, sorted(meta)[:10]
    for k in names:
        m = re.search(r"scan8_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E", k)
        assert m, k
        assert int(m.group(4)) == 0, k
