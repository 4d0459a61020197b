"""The C-ABI's struct layouts and prototypes, not just its symbol names.

* Every `typedef struct` of include/fdr.h is compiled into a small C program (gcc, against the header itself)
  that prints sizeof / offsetof / field sizes; the ctypes Structures of dfd-starter_amd/fdr/_lib.py and the
  stubs shown in INTEGRATION.md must match it field by field.
* Every prototype's argument list and return type are parsed from the header and compared, argument by argument,
  with the argtypes / restype that fdr/_lib.py installs.
Any field or argument drift between the header and a binding fails here, without a GPU.
"""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "fdr.h")
CTYPES_OF = {"fdr_policy_desc": "PolicyDesc", "fdr_env_desc": "EnvDesc", "fdr_lanes_desc": "LanesDesc",
             "fdr_rollout_extras": "RolloutExtras", "fdr_impala_desc": "ImpalaDesc", "fdr_atari_desc": "AtariDesc"}


def _header_text():
    src = open(HEADER).read() + "\n" + open(os.path.join(os.path.dirname(HEADER), "fdr_diag.h")).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))


def header_structs():
    """{struct name: [field, ...]} in declaration order."""
    out = {}
    for name, body in re.findall(r"typedef struct (\w+) \{(.*?)\}\s*\w+\s*;", _header_text(), flags=re.S):
        fields = []
        for stmt in body.split(";"):
            stmt = " ".join(stmt.split())
            if not stmt:
                continue
            m = re.match(r"^(?:const\s+)?\w+\s*\**\s*(.*)$", stmt)
            for decl in m.group(1).split(","):
                fields.append(decl.strip().lstrip("*").strip())
        out[name] = fields
    return out


def _kind(c_type):
    c_type = " ".join(c_type.replace("const", " ").split())
    if "*" in c_type or c_type in ("fdr_stream",):
        return "P"
    return {"int": "i32", "int32_t": "i32", "int64_t": "i64", "uint64_t": "u64", "float": "f32",
            "double": "f64"}[c_type]


def _arg_type(arg):
    m = re.match(r"^(.*?[\s\*])(\w+)$", arg.strip())  # "const float* x" -> "const float*"; "int32_t" stays
    return m.group(1) if m and m.group(1).strip() not in ("", "const") else arg.strip()


def header_prototypes():
    """{function: (return kind, [argument kinds])}."""
    out = {}
    for ret, name, args in re.findall(r"([\w\s\*]+?)\s*\b(fdr_\w+)\s*\(([^)]*)\)\s*;", _header_text()):
        args = args.strip()
        kinds = [] if args in ("", "void") else [_kind(_arg_type(a)) for a in args.split(",")]
        out[name] = (_kind(ret.strip()), kinds)
    return out


def _ctype_kind(t):
    if t is None:
        return None
    if t in (ctypes.c_void_p, ctypes.c_char_p) or (isinstance(t, type) and issubclass(t, ctypes._Pointer)):
        return "P"
    for k, v in ((ctypes.c_int32, "i32"), (ctypes.c_int64, "i64"), (ctypes.c_uint64, "u64"), (ctypes.c_float, "f32"),
                 (ctypes.c_double, "f64")):
        if t is k:
            return v
    raise AssertionError("unmapped ctypes type %r" % (t,))


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    structs = header_structs()
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "fdr.h"', "int main(void) {"]
    for s, fields in structs.items():
        lines.append('  printf("%s %%zu\\n", sizeof(%s));' % (s, s))
        for f in fields:
            lines.append('  printf("%s.%s %%zu %%zu\\n", offsetof(%s, %s), sizeof(((%s*)0)->%s));' % (s, f, s, f, s, f))
    lines += ["  return 0;", "}"]
    d = tmp_path_factory.mktemp("abi")
    src, exe = d / "abi_layout.c", d / "abi_layout"
    src.write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    layout = {}
    for line in out.splitlines():
        key, *vals = line.split()
        layout[key] = tuple(int(v) for v in vals)
    return structs, layout


def _check_structure(cls, s, fields, layout):
    names = [f[0] for f in cls._fields_]
    assert names == fields, "%s fields %s != header %s" % (cls.__name__, names, fields)
    assert ctypes.sizeof(cls) == layout[s][0], "%s: sizeof %d != C %d" % (cls.__name__, ctypes.sizeof(cls), layout[s][0])
    for f in fields:
        off, size = layout["%s.%s" % (s, f)]
        desc = getattr(cls, f)
        assert (desc.offset, desc.size) == (off, size), "%s.%s: ctypes (%d, %d) != C (%d, %d)" % (
            cls.__name__, f, desc.offset, desc.size, off, size)


def test_every_header_struct_has_a_ctypes_mirror(c_layout):
    structs, _ = c_layout
    assert set(structs) == set(CTYPES_OF), sorted(structs)


def test_ctypes_structures_match_the_c_layout(c_layout):
    from fdr import _lib
    structs, layout = c_layout
    for s, fields in structs.items():
        _check_structure(getattr(_lib, CTYPES_OF[s]), s, fields, layout)


def test_integration_stubs_match_the_c_layout(c_layout):
    """The ctypes stubs a maintainer copies from INTEGRATION.md are the header's layouts too."""
    structs, layout = c_layout
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"^class (\w+)\(ctypes\.Structure\):\n((?:    .*\n|\s*\n)+?)(?=\S)", text, flags=re.M)
    assert blocks, "no ctypes stubs found in INTEGRATION.md"
    by_ctypes = {v: k for k, v in CTYPES_OF.items()}
    for cls_name, body in blocks:
        ns = {"ctypes": ctypes}
        exec("class %s(ctypes.Structure):\n%s" % (cls_name, body), ns)
        s = by_ctypes[cls_name]
        _check_structure(ns[cls_name], s, structs[s], layout)


def test_prototypes_match_argtypes():
    from fdr import _lib
    protos = header_prototypes()
    assert set(protos) == set(_lib.EXPORTS)
    for name, (ret, args) in protos.items():
        fn = getattr(_lib.lib, name)
        got = [_ctype_kind(t) for t in fn.argtypes]
        assert got == args, "%s: argtypes %s != header %s" % (name, got, args)
        assert _ctype_kind(fn.restype) == ret, "%s: restype %s != header %s" % (name, fn.restype, ret)


def test_parser_sees_known_shapes():
    protos = header_prototypes()
    assert protos["fdr_version"] == ("P", [])
    assert protos["fdr_fd_grad_fused_out_len"] == ("i64", ["i32", "i64", "i32"])
    assert protos["fdr_rollout"][1][:6] == ["P", "P", "P", "P", "i32", "u64"]
    assert header_structs()["fdr_env_desc"][-4:] == ["map_w", "map_h", "done_threshold", "done_dim"]
