"""Dump the innermost loop (smallest backward-branch region containing v_pk_fma_f32 / MFMA) of a kernel
in a hipcc -S listing, with its instruction mix.

    python tools/loop_dump.py /tmp/fdr_rollout.s rollout_pair_kernelILi17ELi6ELb0ELi0E [out.s]
"""
import re
import sys
from collections import Counter


def main(path, pat, out=None, key="v_pk_fma_f32"):
    s = open(path).read()
    m = re.search(r"^(_Z\w*%s\w*):" % re.escape(pat), s, re.M)
    body = s[m.start():s.index(".Lfunc_end", m.start())].splitlines()
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
            seg = body[a:i + 1]
            if any(key in x for x in seg) and (best is None or len(seg) < len(best)):
                best = seg
    ins = [x.strip() for x in best if x.strip() and not x.strip().startswith((".", ";")) and not x.strip().endswith(":")]
    c = Counter(x.split()[0] for x in ins)
    print("%d instrs, VALU %d" % (len(ins), sum(v for k, v in c.items() if k.startswith("v_"))))
    for k, v in c.most_common(40):
        print("   %-28s %d" % (k, v))
    if out:
        open(out, "w").write("\n".join(x for x in best if not x.strip().startswith((";", ".loc", ".file"))))


if __name__ == "__main__":
    main(*sys.argv[1:])
