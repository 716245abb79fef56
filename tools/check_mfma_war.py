#!/usr/bin/env python3
"""Disassembly check of the MFMA operand write-after-read hazard (DESIGN.md §3,
device_common.h mfma_operand_guard).

hipcc (ROCm 7.2, gfx950) may allocate a VALU result onto an A / B source VGPR of
an MFMA that is still executing; the MFMA then reads the new value (round 2: one
wrong 32x32 accumulator block in ~1 % of cosine searches).  This script pulls
the gfx950 code object out of each built object file, walks every kernel, and
for every v_mfma_* estimates the cycles until it has finished reading its
operands (its issue time + its cycle count + a margin, the wave's own later
instructions counted at their issue cost, s_nop N as N + 1 wait states, a later
MFMA as the end of the window since the matrix pipe runs them in order); any
VALU instruction inside that window writing one of its A / B registers is
reported.  Exit status 1 when something is found.

Loads that write a register (VMEM global_/buffer_/flat_ and DS ds_read*) are
checked too: such a write lands when the data returns, at the earliest the
load's minimum return latency after its issue (LOAD_MIN_LATENCY: an LDS read
returns in >= ~50 cycles on an idle CU, a vector-memory load in >= ~120 even on
an L1 hit, MI355X_MICROARCH.md constants; the model takes 32 and 64); a load
whose return could land inside the MFMA's operand window is reported like a
VALU write.  (A load refilling an A / B register right after the MFMAs that
read it, as scan8_kernel's register ring and the IVF bound scan do, returns
long after the operands were read: not a hazard under this model.)

Default mode checks the MFMAs that END a run (no further MFMA in the next RUN_GAP
instructions: the tile-final MFMAs before an epilogue, where round 2 saw the
failure and where mfma_operand_guard() sits).  --strict checks every MFMA: that
flags hundreds of VALU writes one or two instructions after an MFMA inside
k-loops (e.g. scan_kernel<.,.,i8>'s address updates into a just-used B
register) in kernels whose outputs are bit-exact across the whole GPU suite, so
A / B are read at issue there; the strict count is reported for reference.

usage: tools/check_mfma_war.py [--strict] [--list] [objects...]   (default: duckdb-lancedb_amd/lib/*.o)
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MARGIN = 16
RUN_GAP = 24
# earliest return of a register-writing load after its issue (cycles; conservative)
LOAD_MIN_LATENCY = {"ds_": 32, "global_": 64, "buffer_": 64, "flat_": 32, "scratch_": 64}


def load_latency(mn):
    """Minimum return latency of a load that writes its first operand, else None."""
    for pre, lat in LOAD_MIN_LATENCY.items():
        if mn.startswith(pre) and ("load" in mn or "read" in mn or ("atomic" in mn and "rtn" in mn)):
            return lat
    return None


def mfma_cycles(op):
    m = re.search(r"_(\d+)x(\d+)x(\d+)", op)
    if not m:
        return 64
    M, N, K = map(int, m.groups())
    if op.endswith("_f32") and ("x2_f32" in op or "x4_f32" in op or "x1_f32" in op or "x4f32" in op):
        return 64 if M == 32 else 32  # f32-input forms: 32x32x2 64, 16x16x4 32
    return 32 if M == 32 else 16      # bf16 / fp8 / i8 double-K forms on gfx950


def regs(tok):
    """'v[54:57]' -> {('v',54..57)}; 'v12' -> {('v',12)}; a-registers likewise."""
    tok = tok.strip().rstrip(",")
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.fullmatch(r"([va])(\d+)", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def code_object(obj, tmp):
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "co.elf")
    for f in (fb, co):
        if os.path.exists(f):
            os.remove(f)
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fb}", obj], check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}", f"--output={co}"],
                   check=True, capture_output=True)
    if not os.path.exists(co) or os.path.getsize(co) == 0:
        raise subprocess.CalledProcessError(1, "clang-offload-bundler")
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout


def parse(disasm):
    """-> {kernel: [(mnemonic, operand list)]}"""
    funcs, cur = {}, None
    for line in disasm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is None:
            continue
        line = line.split("//")[0].strip()
        if not line or line.endswith(":"):
            continue
        parts = line.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        cur.append((parts[0], ops))
    return funcs


def issue_cost(mn, ops):
    if mn == "s_nop":
        return int(ops[0], 0) + 1 if ops else 1
    return 4


def check(funcs, strict=False):
    bad = []
    n_mfma = 0
    for name, ins in funcs.items():
        for i, (mn, ops) in enumerate(ins):
            if not mn.startswith("v_mfma"):
                continue
            n_mfma += 1
            if not strict and any(x[0].startswith("v_mfma") for x in ins[i + 1:i + 1 + RUN_GAP]):
                continue  # not the last MFMA of its run
            src = set()
            for o in ops[1:3]:  # A, B
                src |= regs(o)
            window = mfma_cycles(mn) + MARGIN
            t = 8  # the MFMA itself holds vector issue
            for j in range(i + 1, len(ins)):
                mn2, ops2 = ins[j]
                if mn2.startswith("v_mfma") or mn2.startswith("s_endpgm") or mn2.startswith("s_setpc"):
                    break
                if mn2.startswith("v_") and ops2:
                    hit = regs(ops2[0]) & src
                    if hit:
                        bad.append((name, i, mn, j, mn2, ops2[0], t))
                lat = load_latency(mn2)
                if lat is not None and ops2 and t + lat < window and regs(ops2[0]) & src:
                    bad.append((name, i, mn, j, mn2, ops2[0], t + lat))
                t += issue_cost(mn2, ops2)
                if t >= window:
                    break
    return bad, n_mfma


def main():
    args = sys.argv[1:]
    strict = "--strict" in args
    args = [a for a in args if a not in ("--strict", "--list")]
    objs = args or sorted(glob.glob(os.path.join(ROOT, "duckdb-lancedb_amd", "lib", "*.o")))
    total_bad, total = 0, 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            try:
                dis = code_object(obj, tmp)
            except subprocess.CalledProcessError:
                continue  # host-only object
            funcs = parse(dis)
            bad, n = check(funcs, strict)
            total += n
            if "--list" in sys.argv:
                for name in sorted(funcs):
                    print(f"kernel {os.path.basename(obj)} {name}")
            if n == 0:
                continue
            print(f"{os.path.basename(obj)}: {n} MFMAs, {len(bad)} VALU writes into a live MFMA operand")
            for (name, i, mn, j, mn2, dst, t) in bad[:int(os.environ.get("SHOW", "20"))]:
                print(f"  {name[:70]}: #{i} {mn} ... #{j} {mn2} {dst} at ~{t} cycles")
            total_bad += len(bad)
    print(f"checked {total} MFMAs ({'every MFMA' if strict else 'run-final MFMAs'}): {total_bad} hazards")
    return 1 if total_bad else 0


if __name__ == "__main__":
    sys.exit(main())
