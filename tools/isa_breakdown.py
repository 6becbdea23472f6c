#!/usr/bin/env python3
"""Static ISA breakdown of a traversal kernel's main loop (profiles/r04_isa_*.txt).

Disassembles the gfx950 code object of an object file built by the Makefile
(build/dev/mtsg.o), finds the kernel, splits it into basic blocks, finds the
outermost loop (the backward branch with the widest span) and prints, per
block inside it, the instruction classes and a label from the block's
characteristic instructions (fetch, triangle test, IEEE division, stack push /
pop, refill, hit write, ...).  The per-iteration figures are bounds: a wave
executes a block when any of its lanes needs it, so the executed count lies
between the shortest path through the loop and the sum of all its blocks; the
SQ counters (tools/gpu_sq.sh) give the measured average.

  python3 tools/isa_breakdown.py build/dev/mtsg.o 'k_trace_sILb0ELi16ELb0ELb0E' > profiles/r04_isa_flat.txt
"""
import re
import subprocess
import sys
import tempfile
import os
from collections import Counter, OrderedDict

LLVM = "/opt/rocm/lib/llvm/bin"


def disassemble(obj):
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        co = os.path.join(d, "dev.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], text=True)


def kernel_lines(text, pat):
    out, on = [], False
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            on = re.search(pat, m.group(2)) is not None
            if on:
                out = []
            continue
        if on:
            m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", line)
            if m:
                out.append((int(m.group(3), 16), m.group(1), m.group(2)))
    return out


def iclass(op):
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_rd"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store")):
        return "vmem_wr"
    if op.startswith(("global_atomic", "buffer_atomic")):
        return "atomic"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def label(ins):
    ops = [o for _, o, _ in ins]
    tags = []
    nld = sum(o.startswith("global_load_dwordx4") for o in ops)
    if nld >= 4:
        tags.append("fetch: node pair + grandchild pair + 48-B TriAccel")
    elif nld:
        tags.append(f"{nld} x 16-B load")
    if "v_div_scale_f32" in ops:
        tags.append("IEEE division (triangle / rectangle test)")
    if any(o.startswith("ds_write") for o in ops):
        tags.append("stack push")
    if any(o.startswith("ds_read") for o in ops):
        tags.append("stack pop")
    if any(o.startswith("global_atomic_add") for o in ops):
        tags.append("work-list refill / tie list")
    if any(o.startswith("global_atomic_or") for o in ops):
        tags.append("error word")
    if any(o.startswith("global_store") for o in ops):
        tags.append("hit / miss record write")
    if "v_mbcnt_lo_u32_b32" in ops and not tags:
        tags.append("lane index")
    return "; ".join(tags)


def blocks(ins):
    """basic blocks: split after branches and at branch targets"""
    targets = set()
    for addr, op, args in ins:
        if op.startswith(("s_cbranch", "s_branch")):
            m = re.match(r"(-?\d+)", args)
            if m:
                k = int(m.group(1))
                if k >= 32768:
                    k -= 65536
                targets.add(addr + 4 + 4 * k)
    bl, cur = [], []
    for it in ins:
        if it[0] in targets and cur:
            bl.append(cur)
            cur = []
        cur.append(it)
        if it[1].startswith(("s_cbranch", "s_branch", "s_endpgm")):
            bl.append(cur)
            cur = []
    if cur:
        bl.append(cur)
    return bl


def main():
    obj, pat = sys.argv[1], sys.argv[2]
    ins = kernel_lines(disassemble(obj), pat)
    if not ins:
        sys.exit(f"kernel matching {pat!r} not found")
    base = ins[0][0]
    # the main loop: the backward branch spanning the most code
    best = None
    for addr, op, args in ins:
        if op.startswith(("s_cbranch", "s_branch")):
            m = re.match(r"(-?\d+)", args)
            if not m:
                continue
            k = int(m.group(1))
            if k >= 32768:
                k -= 65536
            tgt = addr + 4 + 4 * k
            if tgt < addr and (best is None or addr - tgt > best[1] - best[0]):
                best = (tgt, addr)
    lo, hi = best
    bl = blocks(ins)
    loop = [b for b in bl if lo <= b[0][0] <= hi]
    total = Counter()
    print(f"kernel /{pat}/: {len(ins)} instructions; main loop 0x{lo - base:x}-0x{hi - base:x} "
          f"({sum(len(b) for b in loop)} instructions in {len(loop)} basic blocks)")
    print(f"{'offset':>8} {'n':>4} {'valu':>5} {'salu':>5} {'vmem':>5} {'lds':>4} {'wait':>5} {'br':>3}  label")
    for b in loop:
        c = Counter(iclass(o) for _, o, _ in b)
        total += c
        vm = c["vmem_rd"] + c["vmem_wr"] + c["atomic"]
        print(f"{b[0][0] - base:8x} {len(b):4d} {c['valu']:5d} {c['salu']:5d} {vm:5d} {c['lds']:4d} {c['waitcnt']:5d} "
              f"{c['branch']:3d}  {label(b)}")
    print("loop totals by class:", dict(total))
    ops = Counter(o for b in loop for _, o, _ in b if iclass(o) == "valu")
    print("most frequent VALU opcodes in the loop:")
    for o, k in ops.most_common(25):
        print(f"  {o:28s} {k}")


if __name__ == "__main__":
    main()
