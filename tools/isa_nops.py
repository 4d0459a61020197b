#!/usr/bin/env python3
"""Per-pad hazard table of a kernel's hot loop: for every `s_nop` the compiler placed in the shipped code object, the
instruction it delays, the producer it waits for, and the gfx950 wait-state rule that forces it.

  python tools/isa_nops.py 'rollout_pair_kernelILi17ELi6ELb0ELi0E' [--so path] [--steps 5] [--list]

The consumer is the first instruction after the pad; its producer is the nearest earlier instruction (linear order in
the loop, pads and s_waitcnt counted as wait states) that writes a register the consumer reads.  Rules (CDNA3/4
"manually inserted wait states", the ones LLVM's GCNHazardRecognizer enforces for gfx940+):
  trans->VALU      a transcendental (v_exp / v_rcp / v_log / v_sqrt / v_rsq / v_sin / v_cos) result read by a
                   non-transcendental VALU op: 1 wait state
  VALU->DPP        a VALU-written VGPR read by a DPP op: 2
  VALU->permlane   a VALU-written VGPR read by v_permlane{16,32}_swap: 2
  VALU sgpr->VALU  an SGPR / VCC written by a VALU op (v_cmp_*_e64, v_readlane, carry-out) read by a VALU op: 2
  VALU->readlane   a VALU-written VGPR read by v_readlane / v_readfirstlane: 1
  pk/DPP fwd       the compiler also pads 1 state after a packed-f32 (v_pk_fma / v_pk_add / v_pk_mul) or a DPP result
                   that the next instruction reads (gfx950 forwarding; LLVM inserts it, no ISA table entry is cited)
A pad longer than its rule needs, or with no producer in reach, is reported as such (scheduling slack).
"""
import argparse
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_mix  # noqa: E402
import isa_hazards as ih  # noqa: E402

TRANS = isa_mix.TRANS
_REG = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]|\b(vcc)\b")


def reg_set(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(6):
            out |= {("s", 106), ("s", 107)}      # vcc_lo / vcc_hi
        elif m.group(1):
            out.add((m.group(1), int(m.group(2))))
        else:
            out |= {(m.group(3), r) for r in range(int(m.group(4)), int(m.group(5)) + 1)}
    return out


def split(line):
    mn, _, rest = line.partition(" ")
    ops = rest.split(" ")[0] if False else rest
    # operands end at the first modifier keyword
    core = re.split(r"\s(?:op_sel|op_sel_hi|row_|quad_perm|bank_mask|row_mask|bound_ctrl|offset|neg_lo|neg_hi|clamp|"
                    r"offen|idxen|sc0|sc1|nt|glc|slc)", " " + rest)[0]
    parts = [p.strip() for p in core.split(",") if p.strip()]
    return mn, parts


def dst_src(line):
    mn, parts = split(line)
    if not parts:
        return mn, set(), set()
    if mn.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch")):
        return mn, set(), set()
    if mn.startswith(("ds_write", "global_store", "buffer_store", "flat_store", "ds_bpermute")) and \
            not mn.startswith("ds_bpermute"):
        return mn, set(), reg_set(",".join(parts))
    if mn.startswith("v_cmp") and not mn.endswith("_e64"):     # VOPC: implicit vcc destination
        return mn, {("s", 106), ("s", 107)}, reg_set(",".join(parts))
    dst = reg_set(parts[0])
    src = reg_set(",".join(parts[1:]))
    if mn.startswith(("v_cndmask_b32_e32", "v_addc", "v_subb", "v_subrev_co", "v_add_co_ci")) and "_e64" not in mn:
        src |= {("s", 106), ("s", 107)}
    if mn.startswith(("v_fmac", "v_mac")) or ("_dpp" in mn and mn.startswith(("v_fmac", "v_mac"))):
        src |= dst                                   # accumulate: the destination is read too
    return mn, dst, src


def rule(prod, cons, regs, src0=None):
    sg = any(k == "s" for k, _ in regs)
    if prod.startswith(TRANS) and cons.startswith("v_") and not cons.startswith(TRANS):
        return "trans->VALU", 1
    if "_dpp" in cons and src0 is not None and regs & src0:
        return "VALU->DPP", 2
    if cons.startswith("v_permlane"):
        return "VALU->permlane", 2
    if sg and prod.startswith("v_") and cons.startswith("v_"):
        return "VALU sgpr->VALU", 2
    if cons.startswith(("v_readlane", "v_readfirstlane")):
        return "VALU->readlane", 1
    if prod.startswith(("v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32")) and cons.startswith("v_"):
        return "pk-f32 fwd->VALU", 1
    if "_dpp" in prod and cons.startswith("v_"):
        return "DPP fwd->VALU", 1
    return None, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern")
    ap.add_argument("--so", default=ih.DEFAULT_SO)
    ap.add_argument("--steps", type=int, default=5, help="steps in the unrolled loop body (per-step numbers)")
    ap.add_argument("--list", action="store_true")
    args = ap.parse_args()
    text = isa_mix.disasm(args.so)
    funcs = ih.functions(text)
    name = next(n for n in funcs if args.pattern in n)
    insns = funcs[name]
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
    lo, hi = isa_mix.hot_loop(insns, lines)
    body = [lines[x.addr] for x in insns[lo:hi + 1]]
    table = collections.Counter()
    slack = collections.Counter()
    rows = []
    for i, line in enumerate(body):
        if not line.startswith("s_nop"):
            continue
        n_pad = int(line.split()[1], 0) + 1
        # consumer: the next non-nop instruction
        j = i + 1
        while j < len(body) and body[j].startswith("s_nop"):
            j += 1
        cons, _, csrc = dst_src(body[j])
        # producer: walk back, counting wait states (every instruction 1, s_nop N: N + 1)
        ws, k, found = 0, i - 1, None
        ws_total = n_pad + sum(int(body[q].split()[1], 0) + 1 for q in range(i + 1, j))
        while k >= 0 and ws < 8:
            pm, pdst, _ = dst_src(body[k])
            hit = pdst & csrc
            if hit and pm.startswith("v_"):
                found = (pm, hit, ws)
                break
            ws += int(body[k].split()[1], 0) + 1 if body[k].startswith("s_nop") else 1
            k -= 1
        if found is None:
            key = ("slack: no VALU producer within 8 states", "")
            table[key] += n_pad
            rows.append((i, line, body[j], "-", "slack"))
            continue
        pm, hit, dist = found
        _, cparts = split(body[j])
        src0 = reg_set(cparts[1]) if len(cparts) > 1 else set()
        r, need = rule(pm, cons, hit, src0)
        have = dist + ws_total
        if r is None:
            r = "other %s->%s" % (pm, cons)
        table[(r, "")] += n_pad
        if have > need:
            slack[r] += min(n_pad, have - need)
        rows.append((i, line, body[j], pm, "%s (needs %d, has %d)" % (r, need, have)))
    total = sum(table.values())
    print("%s: %d s_nop wait states in the %d-step loop body = %.1f per step" % (name, total, args.steps,
                                                                               total / args.steps))
    print("%-44s %8s %9s  %s" % ("rule", "states", "per step", "of which slack"))
    for (r, extra), v in table.most_common():
        lab = r if not extra else "%s (%s)" % (r, extra)
        print("%-44s %8d %9.1f  %d" % (lab, v, v / args.steps, slack.get(r, 0)))
    if args.list:
        for i, pad, cons, prod, why in rows:
            print("%5d  %-10s %-60s <- %-22s %s" % (i, pad, cons[:60], prod, why))


if __name__ == "__main__":
    main()
