"""Record, as a fixture, the identifiers of the reference's Go package `index`
(shock-server/node/file/index/*.go) and of the two packages the cgo shim imports from the server
(conf, logger): the file-block import names of every file and the package-block declarations.
tests/test_go_shim.py checks integration/shock-server/node/file/index/gpurecord.go against them
(the Go spec forbids an identifier declared in both the file and the package block, and a name
the shim uses from the package or from conf / logger must exist).

Run in the build container (the reference is not on the GPU box):
    python tests/golden/make_ref_index_pkg.py
"""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import golapi  # noqa: E402

REF = "/root/reference/shock-server"


def package(path):
    files = sorted(f for f in glob.glob(os.path.join(path, "*.go")) if not f.endswith("_test.go"))
    per_file, decls = {}, set()
    for f in files:
        src = open(f, encoding="utf-8").read()
        per_file[os.path.relpath(f, REF)] = sorted(golapi.imports(src))
        decls |= golapi.toplevel(src)
    return per_file, sorted(decls)


def main():
    imps, decls = package(os.path.join(REF, "node/file/index"))
    _, conf = package(os.path.join(REF, "conf"))
    _, logger = package(os.path.join(REF, "logger"))
    out = {
        "source": "MG-RAST/Shock shock-server (snapshot under /root/reference), extracted by tests/golapi.py",
        "index_imports": imps,
        "index_toplevel": decls,
        "conf_toplevel": conf,
        "logger_toplevel": logger,
    }
    with open(os.path.join(HERE, "ref_index_pkg.json"), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()
