"""Static check of the shipped gfx950 code for the DPP / permlane read-after-VALU-write hazards.

LLVM's hazard recognizer does not look inside inline asm, and the rollout kernels issue their DPP
reduce-scatters and permlane swaps from asm blocks whose first instructions read registers that the
previous statement's VALU instructions wrote.  The CDNA rules checked here:
  * a VALU write of a VGPR, then a DPP instruction reading it as src0: 2 wait states;
  * a VALU write of a VGPR, then v_permlane{16,32}_swap reading it: 2 wait states;
  * a VALU write of EXEC (v_cmpx), then a DPP instruction: 5 wait states.
Every instruction issued in between is one wait state, `s_nop N` is N + 1.  The search walks back
over every control-flow predecessor (fall-through and branch sources), so a DPP at a loop head is
checked against the loop's back edge too.

Usage: python tools/isa_hazards.py [libfdr.so]   (exit 1 and a listing on any violation)
Test: tests/test_isa_hazards.py runs it on the in-tree library.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_SO = os.path.join(ROOT, "dfd-starter_amd", "fdr", "libfdr.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_INSN = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):[^<]*(?:<(.+)\+0x([0-9a-f]+)>)?\s*$")
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")
_UNCOND = ("s_branch", "s_endpgm", "s_setpc_b64", "s_trap")


def code_objects(so_path):
    """The gfx950 ELF code objects bundled in the library's .hip_fatbin section."""
    hdr = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-S", "-W", so_path], capture_output=True, text=True,
                         check=True).stdout
    off = size = None
    for line in hdr.splitlines():
        if ".hip_fatbin" in line:
            f = line.split()
            i = f.index("PROGBITS")
            off, size = int(f[i + 2], 16), int(f[i + 3], 16)
    if off is None:
        raise RuntimeError("%s has no .hip_fatbin section" % so_path)
    with open(so_path, "rb") as fh:
        fh.seek(off)
        sec = fh.read(size)
    cos, pos = [], 0
    while True:
        p = sec.find(MAGIC, pos)
        if p < 0:
            return cos
        (n,) = struct.unpack_from("<Q", sec, p + 24)
        q = p + 32
        for _ in range(n):
            eo, es, ts = struct.unpack_from("<QQQ", sec, q)
            q += 24
            triple = sec[q:q + ts].decode()
            q += ts
            if "gfx950" in triple and es:
                cos.append(sec[p + eo:p + eo + es])
        pos = p + 1


def regs(op):
    """VGPR numbers named by one operand ('v5', 'v[4:5]'), else empty."""
    m = _VREG.match(op.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def operands(text):
    # operands up to the first modifier (quad_perm:..., row_mask:..., op_sel..., offset:...)
    out = []
    for tok in text.split(","):
        tok = tok.strip()
        if not tok:
            continue
        out.append(tok.split()[0])
    return out


class Insn:
    __slots__ = ("addr", "mn", "ops", "target")

    def __init__(self, addr, mn, ops, target):
        self.addr, self.mn, self.ops, self.target = addr, mn, ops, target

    @property
    def valu_vgpr_writes(self):
        if not self.mn.startswith("v_") or self.mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp", "v_mfma")):
            return set()
        return regs(self.ops[0]) if self.ops else set()

    @property
    def writes_exec(self):
        return self.mn.startswith("v_cmpx")

    @property
    def wait_states(self):
        if self.mn == "s_nop":
            return int(self.ops[0], 0) + 1
        return 1


def functions(asm_text):
    funcs, cur, base = {}, None, 0
    for line in asm_text.splitlines():
        m = _FUNC.match(line)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        mn, rest, addr, tfun, toff = m.groups()
        is_branch = mn.startswith("s_cbranch") or mn == "s_branch"
        target = base + int(toff, 16) if (toff and tfun == cur and is_branch) else None
        funcs[cur].append(Insn(int(addr, 16), mn, operands(rest), target))
    return funcs


def hazards(func_name, insns):
    """(reader address, reader text, writer address, wait states seen) for every violation in one function."""
    index = {ins.addr: k for k, ins in enumerate(insns)}
    preds = [[] for _ in insns]
    for k, ins in enumerate(insns):
        if k + 1 < len(insns) and ins.mn not in _UNCOND:
            preds[k + 1].append(k)
        if ins.target is not None and ins.target in index:
            preds[index[ins.target]].append(k)
    bad = []
    for k, ins in enumerate(insns):
        dpp = "_dpp" in ins.mn
        perm = ins.mn.startswith(("v_permlane16_swap", "v_permlane32_swap"))
        if not (dpp or perm):
            continue
        if dpp:
            srcs = regs(ins.ops[1]) if len(ins.ops) > 1 else set()
        else:
            srcs = regs(ins.ops[0]) | (regs(ins.ops[1]) if len(ins.ops) > 1 else set())
        # depth-first over predecessors: (index, wait states between it and the reader)
        stack, seen = [(p, 0) for p in preds[k]], set()
        while stack:
            j, ws = stack.pop()
            if (j, ws) in seen:
                continue
            seen.add((j, ws))
            w = insns[j]
            if ws < 2 and srcs & w.valu_vgpr_writes:
                bad.append((ins.addr, "%s %s" % (ins.mn, ",".join(ins.ops)), w.addr, ws, w.mn))
            if dpp and ws < 5 and w.writes_exec:
                bad.append((ins.addr, "%s (EXEC)" % ins.mn, w.addr, ws, w.mn))
            nws = ws + w.wait_states
            if nws < 5:
                stack.extend((p, nws) for p in preds[j])
    return bad


def check(so_path=DEFAULT_SO):
    """{function: [violations]} over every kernel in the library, and the number of DPP/permlane reads checked."""
    out, n_checked = {}, 0
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(so_path)):
            path = os.path.join(td, "co%d.elf" % i)
            with open(path, "wb") as fh:
                fh.write(co)
            asm = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", path],
                                 capture_output=True, text=True, check=True).stdout
            for name, insns in functions(asm).items():
                n_checked += sum(1 for x in insns if "_dpp" in x.mn or x.mn.startswith("v_permlane"))
                bad = hazards(name, insns)
                if bad:
                    out[name] = bad
    return out, n_checked


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_SO
    bad, n = check(so)
    print("checked %d DPP / permlane reads in %s" % (n, so))
    for name, items in sorted(bad.items()):
        print(name)
        for reader, text, writer, ws, wmn in items[:20]:
            print("   %x %s  <- %s at %x, %d wait states" % (reader, text, wmn, writer, ws))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
