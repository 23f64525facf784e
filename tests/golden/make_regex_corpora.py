"""Extracts the reference's labelled regex corpora into tests/golden/regex_corpora.json.

The reference's only expectations on this path are the `valid` / `invalid` string lists of
  shock-server/node/file/format/fastq/fastq_test.go:19-72   (fastq.Regex, fastq.go:22)
  shock-server/node/file/format/fasta/fasta_test.go:19-169  (fasta.Regex, fasta.go:22)
whose TestRegex prints Regex.MatchString(s) for every entry (the labels say what the authors
expected).  This script copies those string literals -- data, not code -- as hex, with their
label, into a JSON fixture.  Go raw string literals (backquotes) hold their bytes verbatim
except that carriage returns are discarded (Go spec, "String literals"); the two files use
only raw literals.

Run in the build container (the GPU box has no /root/reference):
    python tests/golden/make_regex_corpora.py
"""
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/shock-server/node/file/format"
SOURCES = {"fastq": os.path.join(REF, "fastq", "fastq_test.go"),
           "fasta": os.path.join(REF, "fasta", "fasta_test.go")}


def raw_strings(src: str, var: str):
    """The backquoted literals of `var <var> = []string{ ... }` in order, with their line."""
    m = re.search(r"var\s+" + var + r"\s*=\s*\[\]string\{", src)
    if not m:
        raise SystemExit(f"no `var {var}` in source")
    i, out = m.end(), []
    while True:
        while src[i] in " \t\n,":
            i += 1
        if src[i] == "}":
            return out
        if src[i] != "`":
            raise SystemExit(f"unexpected {src[i]!r} in {var} at offset {i}")
        j = src.index("`", i + 1)
        line = src.count("\n", 0, i) + 1
        out.append((line, src[i + 1:j].replace("\r", "")))
        i = j + 1


def main():
    entries = []
    for regex, path in SOURCES.items():
        src = open(path, encoding="utf-8").read()
        for label in ("valid", "invalid"):
            for k, (line, s) in enumerate(raw_strings(src, label)):
                entries.append({"id": f"{regex}_{label}_{k}", "regex": regex, "label": label,
                                "source": f"shock-server/node/file/format/{regex}/{regex}_test.go:{line}",
                                "text_hex": s.encode("utf-8").hex()})
    out = os.path.join(HERE, "regex_corpora.json")
    with open(out, "w") as f:
        json.dump({"generated_by": "tests/golden/make_regex_corpora.py", "entries": entries}, f, indent=1)
    print(f"wrote {len(entries)} entries to {out}")


if __name__ == "__main__":
    main()
