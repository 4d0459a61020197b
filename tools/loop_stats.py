"""Instruction mix of the innermost hot loop of a kernel in a hipcc -S listing.

    python tools/loop_stats.py /tmp/fdr_rollout.s rollout_kernelILi17ELi6ELb0ELi0
"""
import re
import sys
from collections import Counter


def main(path, pat):
    s = open(path).read()
    m = re.search(r"^(_Z\w*%s\w*):" % re.escape(pat), s, re.M)
    start = m.start()
    end = s.index(".Lfunc_end", start)
    body = s[start:end].splitlines()
    labels = {}
    for i, l in enumerate(body):
        mm = re.match(r"^(\.LBB\S+):", l)
        if mm:
            labels[mm.group(1)] = i
    best = None
    for i, l in enumerate(body):
        mm = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            a = labels[mm.group(1)]
            ins = [x.strip() for x in body[a:i + 1] if x.strip() and not x.strip().startswith((".", ";"))
                   and not x.strip().endswith(":")]
            if best is None or len(ins) > len(best[2]):
                best = (a, i, ins)
    a, b, ins = best
    c = Counter(x.split()[0] for x in ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print("%s: largest loop %d instrs (VALU %d, DS %d, SALU %d, scratch %d, s_nop %d)" % (
        m.group(1)[:60], len(ins), valu, sum(v for k, v in c.items() if k.startswith("ds_")),
        sum(v for k, v in c.items() if k.startswith("s_") and k != "s_nop"),
        sum(v for k, v in c.items() if "scratch" in k or k.startswith("buffer_")), c.get("s_nop", 0)))
    for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
        print("   %-28s %d" % (k, v))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
