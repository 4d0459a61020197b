"""Instruction mix of the innermost loop of a kernel that contains a marker instruction (hipcc -S listing).

    python tools/step_loop.py /tmp/fdr_rollout.s rollout_pair_kernelILi17ELi6ELb0ELi0 row_half_mirror [8] [--dump]

(the optional count = marker lines per step, to report the unroll factor)

Unlike loop_stats.py (largest loop), this isolates the per-step body: the innermost backward-branch region
with the most marker lines (the unrolled main body).  Prints VALU / trans / DPP / DS / SALU / s_nop counts and the v_mov breakdown.
"""
import re
import sys
from collections import Counter


def body_of(path, pat):
    s = open(path).read()
    m = re.search(r"^(_Z\w*%s\w*):" % re.escape(pat), s, re.M)
    end = s.index(".Lfunc_end", m.start())
    return m.group(1), [l.strip() for l in s[m.start():end].splitlines() if l.strip()]


def loops(body):
    labels = {}
    for i, l in enumerate(body):
        mm = re.match(r"^(\.LBB\S+):", l)
        if mm:
            labels[mm.group(1)] = i
    for i, l in enumerate(body):
        mm = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            yield labels[mm.group(1)], i


def main(path, pat, marker, dump=False):
    name, body = body_of(path, pat)
    cand = [(sum(marker in body[j] for j in range(a, b)), a, b) for a, b in loops(body)]
    top = max(n for n, _, _ in cand)  # the unrolled main body, not a remainder loop
    _, a, b = min((c for c in cand if c[0] == top), key=lambda c: c[2] - c[1])
    steps = top // int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4].isdigit() else 1
    ins = [x for x in body[a:b + 1] if not x.startswith((".", ";")) and not x.endswith(":")]
    c = Counter(x.split()[0] for x in ins)
    valu = [x for x in ins if x.startswith("v_")]
    trans = sum(1 for x in valu if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32", x))
    dpp = sum(1 for x in valu if "_dpp" in x.split()[0] or "row_" in x or "quad_perm" in x)
    movs = Counter()
    for x in valu:
        if x.startswith("v_mov_b32_e32"):
            src = x.split(",")[1].strip()
            movs["const" if src[0] not in "vs" else src[0] + "gpr"] += 1
    print("%s: step loop %d instrs: VALU %d (trans %d, dpp %d), DS %d, SALU %d, s_nop %d (sum of waits %d), "
          "waitcnt %d" % (name[:50], len(ins), len(valu), trans, dpp,
                          sum(v for k, v in c.items() if k.startswith("ds_")),
                          sum(v for k, v in c.items() if k.startswith("s_") and k not in ("s_nop", "s_waitcnt")),
                          c.get("s_nop", 0), sum(int(x.split()[1]) + 1 for x in ins if x.startswith("s_nop")),
                          c.get("s_waitcnt", 0)))
    print("   v_mov_b32:", dict(movs), " steps in body:", steps)
    for k, v in c.most_common(30):
        print("   %-28s %d" % (k, v))
    if dump:
        print("\n".join(body[a:b + 1]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], "--dump" in sys.argv)
