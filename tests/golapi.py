"""A small lexer / top-level scanner for Go source, enough to check the cgo shim
(integration/shock-server/node/file/index/gpurecord.go) without a Go toolchain (none exists in this
image or on the GPU box).  Used by tests/test_go_shim.py and by
tests/golden/make_ref_index_pkg.py, which records the reference package's identifiers as a fixture.

It does not parse Go; it strips comments and literals, tracks bracket depth and reads the
top-level declarations the Go spec puts in the package block (func / type / var / const, including
grouped declarations) and the file block (imports)."""
import re

_IDENT = re.compile(r"[A-Za-z_][A-Za-z_0-9]*")


def strip(src: str, keep_strings: bool = False) -> str:
    """Comments removed (newlines kept); string / rune literals blanked unless keep_strings."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append("\n" * src.count("\n", i, j))
            i = j
        elif c in "\"'`":
            j = i + 1
            while j < n and src[j] != c:
                if c != "`" and src[j] == "\\":
                    j += 1
                j += 1
            lit = src[i:j + 1]
            out.append(lit if keep_strings else c + " " * (len(lit) - 2) + c)
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def imports(src: str) -> dict:
    """{name in the file block: import path} (alias, else the path's last element)."""
    s = strip(src, keep_strings=True)
    res = {}
    spec = re.compile(r'^\s*(?:([A-Za-z_][A-Za-z_0-9]*|\.)\s+)?"([^"]+)"\s*$')
    for m in re.finditer(r"^import\s*\((.*?)^\)", s, re.S | re.M):
        for line in m.group(1).splitlines():
            mm = spec.match(line)
            if mm:
                res[mm.group(1) or mm.group(2).rsplit("/", 1)[-1]] = mm.group(2)
    for m in re.finditer(r'^import\s+(?:([A-Za-z_][A-Za-z_0-9]*)\s+)?"([^"]+)"', s, re.M):
        res[m.group(1) or m.group(2).rsplit("/", 1)[-1]] = m.group(2)
    return res


def toplevel(src: str) -> set:
    """Identifiers declared in the package block (methods excluded, init excluded)."""
    s = strip(src)
    names, depth, i = set(), 0, 0
    lines = s.splitlines()
    group = None  # "var" / "const" / "type" while inside a grouped declaration
    for line in lines:
        t = line.strip()
        if depth == 0 and group is None:
            m = re.match(r"^func\s+([A-Za-z_][A-Za-z_0-9]*)", t)
            if m and m.group(1) != "init":
                names.add(m.group(1))
            m = re.match(r"^(var|const|type)\s*\(\s*$", t)
            if m:
                group = m.group(1)
            else:
                m = re.match(r"^(var|const|type)\s+(.*)$", t)
                if m:
                    lhs = m.group(2).split("=")[0]
                    if m.group(1) == "type":
                        names.add(_IDENT.match(lhs.strip()).group(0))
                    else:
                        for part in lhs.split(","):
                            mm = _IDENT.match(part.strip())
                            if mm:
                                names.add(mm.group(0))
        elif group is not None and depth == 1:
            if t == ")":
                group = None
            elif t:
                lhs = t.split("=")[0]
                if group == "type":
                    names.add(_IDENT.match(lhs).group(0))
                else:
                    for part in lhs.split(","):
                        mm = _IDENT.match(part.strip())
                        if mm:
                            names.add(mm.group(0))
        for c in line:
            if c in "({[":
                depth += 1
            elif c in ")}]":
                depth -= 1
        if group is not None and depth == 0:
            group = None
    return names


def balanced(src: str) -> bool:
    s = strip(src)
    stack = []
    pairs = {")": "(", "}": "{", "]": "["}
    for c in s:
        if c in "({[":
            stack.append(c)
        elif c in ")}]":
            if not stack or stack.pop() != pairs[c]:
                return False
    return not stack


def cgo_preamble(src: str) -> str:
    """The comment immediately before `import "C"` (cgo's preamble)."""
    m = re.search(r"/\*(.*?)\*/\s*\nimport \"C\"", src, re.S)
    return m.group(1) if m else ""
