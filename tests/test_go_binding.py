"""The Go side of the drop-in boundary (go/pkg/..., no Go toolchain here to compile it): every
function include/placement.h declares is bound in the cgo package and called with the header's
arity; the adapters call the engine through it and keep the reference's entry-point signatures."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "placement.h")
GO = os.path.join(ROOT, "go", "pkg")
HIP_GO = os.path.join(GO, "placement", "hip", "hip.go")
COSCHED_GO = os.path.join(GO, "runtime.v2", "framework", "plugins", "coscheduling", "engine.go")
V1_GO = os.path.join(GO, "controller.v1", "common", "engine.go")


def strip_c_comments(text):
    return re.sub(r"/\*.*?\*/", "", re.sub(r"//[^\n]*", "", text, flags=0), flags=re.S)


def split_top(args: str):
    """Split an argument list on top-level commas."""
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def header_arity():
    text = strip_c_comments(open(HEADER).read())
    decls = {}
    for m in re.finditer(r"\b(pe_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
        name, params = m.group(1), m.group(2).strip()
        if name == "pe_allgather_fn":
            continue
        decls[name] = 0 if params in ("", "void") else len(split_top(params))
    return decls


def go_calls(path):
    text = open(path).read()
    calls = {}
    for m in re.finditer(r"\bC\.(pe_[a-z0-9_]+)\(", text):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        args = text[m.end():i - 1].strip()
        calls.setdefault(m.group(1), set()).add(0 if not args else len(split_top(args)))
    return calls


def test_header_parses():
    decls = header_arity()
    assert len(decls) >= 30
    assert decls["pe_pg_min_resources"] == 13 and decls["pe_abi_version"] == 0


def test_every_header_function_is_bound_with_its_arity():
    decls = header_arity()
    calls = go_calls(HIP_GO)
    missing = sorted(set(decls) - set(calls))
    assert not missing, f"not bound in hip.go: {missing}"
    for name, arities in calls.items():
        assert name in decls, f"hip.go calls {name}, which placement.h does not declare"
        assert arities == {decls[name]}, f"{name}: header arity {decls[name]}, Go calls {arities}"


def test_cgo_preamble_and_package():
    text = open(HIP_GO).read()
    assert re.search(r"^package hip$", text, flags=re.M)
    assert '#include "placement.h"' in text and 'import "C"' in text
    # the Go side pins slices only for the call: no C pointer into Go memory is stored
    assert "runtime.SetFinalizer" in text


@pytest.mark.parametrize("path,needles", [
    (COSCHED_GO, ["package coscheduling", "func NewWithEngine(", "func flattenInfo(", "func unflatten(",
                  "PGMinResources(hip.ModeV2", "needsCreateOrUpdate(oldPG, newPG", "SetControllerReference",
                  "c.CoScheduling.Build(ctx, obj, info, trainJob)", "framework.ComponentBuilderPlugin"]),
    (V1_GO, ["package common", "func flattenV1(", "func CalcPGMinResourcesEngine(", "PGMinResources(hip.ModeV1",
             "c.Resources.Limits", "CalcPGMinResources(minMember, replicas, pcGetFunc)", "pc.Value"]),
])
def test_adapters(path, needles):
    text = open(path).read()
    for n in needles:
        assert n in text, (os.path.basename(path), n)


def test_go_files_are_balanced():
    """No compiler here: at least braces, brackets and parentheses balance in every Go file."""
    for dirpath, _, files in os.walk(GO):
        for f in files:
            if not f.endswith(".go"):
                continue
            text = open(os.path.join(dirpath, f)).read()
            text = re.sub(r'"(\\.|[^"\\])*"', '""', text)               # strings
            text = re.sub(r"`[^`]*`", "``", text)
            text = re.sub(r"'(\\.|[^'\\])'", "''", text)
            text = re.sub(r"//[^\n]*", "", text)
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            for o, c in ("()", "[]", "{}"):
                assert text.count(o) == text.count(c), (f, o)
