#!/usr/bin/env python3
"""Instruction mix of a kernel's hottest loop in the built library (static count, one trip of the loop body).

  python tools/isa_mix.py 'rollout_pair_kernelILi17ELi6ELb0ELi0E'   [--so path] [--dump]

Finds the function whose mangled name contains the pattern, takes the step loop (hot_loop: the smallest region closed
by a backward branch that holds the most packed-FMA / MFMA / DPP-FMA work -- the unrolled step loop) and counts its instructions by class: packed f32 FMA, other VALU, transcendental, DPP,
permlane, LDS, global, scalar, waits.  Per-step numbers: divide by the unroll (5 steps for 6 action dims).
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_hazards as ih  # noqa: E402

TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_sqrt_f32", "v_rsq_f32", "v_sin_f32", "v_cos_f32")


def disasm(so):
    cos = ih.code_objects(so)
    out = []
    for co in cos:
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(co)
        try:
            out.append(subprocess.run([os.path.join(ih.LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", f.name],
                                      capture_output=True, text=True, check=True).stdout)
        finally:
            os.unlink(f.name)
    return "\n".join(out)


def classify(line):
    mn = line.split()[0]
    if mn.startswith("v_pk_fma_f32"):
        return "v_pk_fma_f32"
    if mn.startswith(TRANS):
        return "transcendental"
    if mn.startswith("v_") and ("row_" in line or "quad_perm" in line or "row_newbcast" in line):
        return "valu_dpp"
    if mn.startswith("v_permlane"):
        return "permlane"
    if mn.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "readlane"
    if mn.startswith("v_pk_"):
        return "valu_pk_other"
    if mn.startswith(("v_fma_f32", "v_fmac_f32")):
        return "v_fma_f32"
    if mn.startswith("v_") and "f64" in mn:
        return "valu_f64"
    if mn.startswith("v_"):
        return "valu_other"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if mn.startswith("s_waitcnt"):
        return "s_waitcnt"
    if mn.startswith("s_nop"):
        return "s_nop"
    if mn.startswith("s_"):
        return "salu/branch"
    return "other"


def hot_loop(insns, lines):
    """The step loop: among regions closed by a backward branch, the one holding the most packed / MFMA / DPP compute,
    the smallest such (regions that merely wrap out-of-line blocks -- the compiler places the prologue's conditional
    loads after the function body and branches back -- hold the same compute plus unrelated code)."""
    def work(a, b):
        return sum(1 for x in insns[a:b + 1] if lines[x.addr].startswith(("v_pk_fma", "v_mfma", "v_fmac_f32_dpp")))
    cands = []
    for k, ins in enumerate(insns):
        if ins.target is not None and ins.target <= ins.addr:
            lo = next(i for i, x in enumerate(insns) if x.addr == ins.target)
            cands.append((lo, k))
    return max(cands, key=lambda r: (work(*r), -(r[1] - r[0])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern")
    ap.add_argument("--so", default=ih.DEFAULT_SO)
    ap.add_argument("--dump", action="store_true")
    args = ap.parse_args()
    text = disasm(args.so)
    funcs = ih.functions(text)
    names = [n for n in funcs if args.pattern in n]
    if not names:
        sys.exit("no function matches %r" % args.pattern)
    name = names[0]
    insns = funcs[name]
    # raw lines of that function for the mnemonic text (modifiers included)
    lines, on = {}, False
    for line in text.splitlines():
        m = ih._FUNC.match(line)
        if m:
            on = m.group(2) == name
            continue
        if on:
            mm = ih._INSN.match(line)
            if mm:
                lines[int(mm.group(3), 16)] = line.split("//")[0].strip()
    lo, hi = hot_loop(insns, lines)
    body = [lines[x.addr] for x in insns[lo:hi + 1]]
    cnt = collections.Counter(classify(b) for b in body)
    print("%s\nloop body: %d instructions (0x%x..0x%x)" % (name, len(body), insns[lo].addr, insns[hi].addr))
    for k, v in cnt.most_common():
        print("  %-16s %5d" % (k, v))
    if args.dump:
        print("\n".join(body))


if __name__ == "__main__":
    main()
