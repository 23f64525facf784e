"""The cgo shim integration/shock-server/node/file/index/gpurecord.go, checked without a Go
toolchain (none exists here or on the GPU box):

(a) every C.shockidx_* / C.SHOCKIDX_* it names is declared in include/shockidx.h, and every call
    passes as many arguments as the prototype takes;
(b) none of its package-level identifiers collides with an import name or a package-level
    identifier of the reference's package index (tests/golden/ref_index_pkg.json, extracted from
    /root/reference by tests/golden/make_ref_index_pkg.py), and none of its import names is
    declared in that package (Go: no identifier in both the file and the package block);
(c) Go's own compile errors a text check can see: imports before declarations, one cgo preamble
    directly above import "C", every import used, balanced brackets;
(d) what it uses from package index, conf and logger exists there;
(e) INTEGRATION.md quotes the file verbatim.
"""
import json
import os
import re

import golapi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "shock-server", "node", "file", "index", "gpurecord.go")
HDR = os.path.join(ROOT, "include", "shockidx.h")
REFPKG = os.path.join(ROOT, "tests", "golden", "ref_index_pkg.json")
CGO_BUILTINS = {"CString", "GoString", "GoStringN", "GoBytes", "CBytes", "free", "malloc", "int", "uint64_t",
                "int64_t", "char", "size_t", "uint32_t", "int32_t"}  # stdlib.h (free, malloc) and C scalar types


def _src():
    return open(SHIM, encoding="utf-8").read()


def _header():
    h = golapi.strip(open(HDR, encoding="utf-8").read())
    protos = {}
    for m in re.finditer(r"\b([A-Za-z_][A-Za-z_0-9 \*]*?)\b(shockidx_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", h, re.S):
        args = m.group(3).strip()
        protos[m.group(2)] = 0 if args in ("", "void") else args.count(",") + 1
    consts = set(re.findall(r"\b(SHOCKIDX_[A-Z0-9_]+)\s*=", h)) | set(re.findall(r"#define\s+(SHOCKIDX_[A-Z0-9_]+)", h))
    types = set(re.findall(r"typedef\s+struct\s+\w+\s*\{[^}]*\}\s*(shockidx_\w+)\s*;", h, re.S))
    types |= set(re.findall(r"typedef\s+struct\s+\w+\s+(shockidx_\w+)\s*;", h))
    return protos, consts, types


def _calls(src):
    """(name, argument count) of every C.shockidx_* call (top-level commas of the argument list)."""
    s = golapi.strip(src)
    out = []
    for m in re.finditer(r"\bC\.(shockidx_[a-z0-9_]+)\s*\(", s):
        i, depth, commas, nonempty = m.end(), 1, 0, False
        while depth:
            c = s[i]
            if c in "([{":
                depth += 1
            elif c in ")]}":
                depth -= 1
            elif c == "," and depth == 1:
                commas += 1
            if depth and not c.isspace():
                nonempty = True
            i += 1
        out.append((m.group(1), commas + 1 if nonempty else 0))
    return out


def test_c_symbols_declared_in_header():
    protos, consts, types = _header()
    s = golapi.strip(_src())
    used = set(re.findall(r"\bC\.([A-Za-z_][A-Za-z_0-9]*)", s))
    assert used, "the shim calls nothing through cgo"
    for name in sorted(used):
        if name in CGO_BUILTINS:
            continue
        assert name in protos or name in consts or name in types, f"C.{name} is not declared in include/shockidx.h"
    calls = _calls(_src())
    assert calls
    for name, n in calls:
        assert protos[name] == n, f"C.{name}: {n} arguments, the prototype takes {protos[name]}"


def test_no_identifier_in_both_file_and_package_block():
    ref = json.load(open(REFPKG))
    ref_imports = set().union(*map(set, ref["index_imports"].values()))
    ref_decls = set(ref["index_toplevel"])
    src = _src()
    mine = golapi.toplevel(src)
    assert {"NewGPURecordIndexer", "NewGPULineIndexer", "NewGPUChunkRecordIndexer", "gpuMulti", "gpuIndexer"} <= mine
    clash_imports = sorted(mine & ref_imports)
    assert not clash_imports, f"declared here, imported by another file of package index: {clash_imports}"
    clash_decls = sorted(mine & ref_decls)
    assert not clash_decls, f"already declared in package index: {clash_decls}"
    my_imports = set(golapi.imports(src)) - {"C"}
    assert not (my_imports & ref_decls), sorted(my_imports & ref_decls)
    assert not (my_imports & mine), sorted(my_imports & mine)


def test_the_old_markdown_shim_would_have_failed():
    """The round-3 shim declared `var multi` in package index; the check above must catch that."""
    ref = json.load(open(REFPKG))
    ref_imports = set().union(*map(set, ref["index_imports"].values()))
    bad = "package index\n\nvar multi struct {\n\tg int\n}\n"
    assert golapi.toplevel(bad) & ref_imports == {"multi"}


def test_go_file_structure():
    src = _src()
    s = golapi.strip(src)
    assert golapi.balanced(src)
    assert golapi.strip(src, keep_strings=True).count('import "C"') == 1
    pre = golapi.cgo_preamble(src)
    assert '#include "shockidx.h"' in pre and "#include <stdlib.h>" in pre
    # imports come before every declaration
    first_decl = re.search(r"^(func|type|var|const)\b", s, re.M).start()
    last_import = max(m.end() for m in re.finditer(r"^import\b[^\n]*(\((.*?)^\))?", s, re.M | re.S))
    assert last_import < first_decl, "an import after a declaration"
    # every imported package is used (an unused import is a compile error)
    for name in golapi.imports(src):
        if name in ("C", "_"):
            continue
        assert re.search(rf"\b{name}\.[A-Za-z_]", s), f"import {name} unused"
    assert re.match(r"\s*package index\b", s)


def test_uses_exist_in_reference_packages():
    ref = json.load(open(REFPKG))
    s = golapi.strip(_src())
    for name in ("Indexers", "Indexer", "NewRecordIndexer", "NewLineIndexer", "NewChunkRecordIndexer"):
        assert re.search(rf"\b{name}\b", s) and name in ref["index_toplevel"], name
    for name in set(re.findall(r"\bconf\.([A-Za-z_]\w*)", s)):
        assert name in ref["conf_toplevel"], f"conf.{name}"
    for name in set(re.findall(r"\blogger\.([A-Za-z_]\w*)", s)):
        assert name in ref["logger_toplevel"], f"logger.{name}"
    # registered under the reference's keys (index.go:21-28)
    lit = golapi.strip(_src(), keep_strings=True)
    assert re.search(r'Indexers\["record"\]\s*=\s*NewGPURecordIndexer', lit)
    assert re.search(r'Indexers\["line"\]\s*=\s*NewGPULineIndexer', lit)
    assert re.search(r'Indexers\["chunkrecord"\]\s*=\s*NewGPUChunkRecordIndexer', lit)


def test_init_makes_no_hip_call():
    """the GPU runtime starts lazily -- init() only registers constructors, and the
    first HIP call (the device count) happens in gpuInit, run once by the first Create."""
    s = golapi.strip(_src())
    body = s[s.index("func init()"):]
    assert "C." not in body[:body.index("\n}")]
    gi = s[s.index("func gpuInit()"):]
    assert "C.shockidx_device_count()" in gi[:gi.index("\n}")]


def test_multi_group_requires_rccl():
    s = golapi.strip(_src())
    assert re.search(r"C\.shockidx_multi_rccl\(g\)\s*==\s*0", s)
    body = s[s.index("func initGPUMulti"):]
    body = body[:body.index("\nfunc ")]
    i = body.index("shockidx_multi_rccl")
    assert "shockidx_multi_destroy" in body[i:] and body.index("gpuMulti.g = g") > i


def test_integration_md_quotes_the_file():
    md = open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8").read()
    m = re.search(r"<!-- gpurecord.go begin -->\n```go\n(.*?)```\n<!-- gpurecord.go end -->", md, re.S)
    assert m, "INTEGRATION.md does not quote gpurecord.go"
    assert m.group(1) == _src()
