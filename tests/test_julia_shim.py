"""Static checks of the Julia binding julia/HIPBackend.jl (no Julia on this
image, so it cannot be run here):

* every ccall names an entry point declared in include/pa_hip.h and passes
  as many argument types as the C prototype has parameters;
* every helper the module calls (dev_*, mark_*, sync_*, _*) is defined in it;
* the names it imports from PartitionedArrays exist in the reference
  (src/*.jl), when the reference checkout is present."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = open(os.path.join(ROOT, "julia", "HIPBackend.jl")).read()
HDR = open(os.path.join(ROOT, "include", "pa_hip.h")).read()


def _strip_comments(src):
    out = []
    for line in src.splitlines():
        i = line.find("#")
        out.append(line if i < 0 else line[:i])
    return "\n".join(out)


CODE = _strip_comments(JL)


def _c_prototypes():
    hdr = re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(?:int|const char\*)\s+(pa_\w+)\s*\(([^)]*)\)\s*;", hdr, flags=re.S):
        params = m.group(2).strip()
        protos[m.group(1)] = 0 if params in ("", "void") else len(params.split(","))
    return protos


def _balanced(s, i):
    """s[i] == '(' → index after its matching ')'"""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def _split_top(s):
    parts, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts]


def _ccalls():
    out = []
    for m in re.finditer(r"ccall\(", CODE):
        start = m.end() - 1
        end = _balanced(CODE, start)
        args = _split_top(CODE[start + 1:end - 1])
        name = re.match(r"\(:(\w+),\s*libpa\)", args[0]).group(1)
        types = args[2]
        assert types.startswith("(") and types.endswith(")"), (name, types)
        tlist = _split_top(types[1:-1])
        out.append((name, len(tlist), len(args) - 3))
    return out


def test_ccalls_match_the_c_abi():
    protos = _c_prototypes()
    calls = _ccalls()
    assert len(calls) >= 25
    for name, ntypes, nargs in calls:
        assert name in protos, f"{name} is not declared in include/pa_hip.h"
        assert ntypes == protos[name], f"{name}: {ntypes} argument types, the C prototype has {protos[name]}"
        assert nargs == ntypes, f"{name}: {nargs} arguments for {ntypes} types"
    # the hot path and the coherence layer reach the library
    used = {c[0] for c in calls}
    for must in ("pa_spmv_all", "pa_exchange_all", "pa_mat_exchange_all", "pa_dot_all", "pa_norm2_all",
                 "pa_cg_solve_all", "pa_vec_upload", "pa_vec_download", "pa_mat_get_values", "pa_mat_set_values",
                 "pa_vec_axpby", "pa_vec_copy", "pa_vec_fill", "pa_ctx_create_shared"):
        assert must in used, must


def _defined():
    names = set(re.findall(r"^\s*function\s+(?:[\w.]+\.)?([\w!]+)\s*[({]", CODE, flags=re.M))
    names |= set(re.findall(r"^\s*(?:[\w.]+\.)?([\w!]+)\s*\([^=\n]*\)\s*(?:where\s*\{[^}]*\}\s*)?=", CODE, flags=re.M))
    names |= set(re.findall(r"^\s*(?:mutable\s+)?struct\s+(\w+)", CODE, flags=re.M))
    names |= set(re.findall(r"^\s*const\s+(\w+)", CODE, flags=re.M))
    return names


def test_every_helper_is_defined():
    defined = _defined()
    called = set(re.findall(r"(?<![\w.:])((?:dev_|mark_|sync_|_)[\w!]*)\s*\(", CODE))
    called |= set(re.findall(r"foreach\(((?:mark_|sync_)[\w!]*)", CODE))
    missing = sorted(c for c in called if c not in defined)
    assert not missing, f"called but not defined in julia/HIPBackend.jl: {missing}"
    for h in ("dev_vec", "dev_idx", "dev_xchg", "dev_mat", "dev_mat_xchg", "mark_device_newer!",
              "mark_host_newer!", "sync_host!", "dev_vec_nocopy"):
        assert h in defined, h
    # the AbstractPData contract (Interfaces.jl:50-124) for HIPData
    for sig in (r"Base\.size\(a::HIPData\)", r"get_backend\(a::HIPData\)", r"function Base\.iterate\(a::HIPData\)",
                r"function Base\.iterate\(a::HIPData, state::HIPData\)", r"function map_parts\(task, args::HIPData\.\.\.\)",
                r"i_am_main\(::HIPData\)", r"get_part\(a::HIPData, part::Integer\)", r"gather!\(rcv::HIPData",
                r"gather_all!\(rcv::HIPData", r"function scatter\(snd::HIPData\)", r"function async_exchange!\(data_rcv::HIPData"):
        assert re.search(sig, CODE), sig


def test_reference_names_exist():
    ref = "/root/reference/src"
    if not os.path.isdir(ref):
        pytest.skip("reference checkout absent")
    src = "\n".join(open(os.path.join(ref, f)).read() for f in os.listdir(ref) if f.endswith(".jl"))
    imp = re.search(r"import PartitionedArrays:(.*?)\n\n", CODE, flags=re.S).group(1)
    names = [n.strip() for n in imp.replace("\n", " ").split(",") if n.strip()]
    for n in names:
        assert re.search(r"(?<![\w!])" + re.escape(n) + r"(?![\w!])", src), f"PartitionedArrays has no {n}"
    for n in set(re.findall(r"PartitionedArrays\.(\w+)", CODE)):
        assert re.search(r"\b" + re.escape(n) + r"\b", src), f"PartitionedArrays has no {n}"
