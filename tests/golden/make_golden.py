"""Regenerates tests/golden/expected/ from the pure-Python restatement (oracle/pyref.py).

Inputs: tests/golden/fixtures/* (data files copied verbatim from the reference's own
test/testdata/) and the known-answer vectors in tests/golden/kats.json (SURVEY.md
Appendix B plus edge cases added here, each with the expected answer written by hand from
the Go source -- the KAT expectations are NOT generated, they pin the restatement).

Outputs, per fixture and mode (auto | fasta | fastq | sam | line):
  expected/<fixture>.<mode>.idx   the index file bytes (LE u64 offset, u64 length)
  expected/manifest.json          count, error message (hex), sha256 of the .idx

Run:  python tests/golden/make_golden.py   (only needed when fixtures change)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyref  # noqa: E402

MODES = ("auto", "fasta", "fastq", "sam", "line")


def run(data, mode):
    if mode == "line":
        return pyref.line_index(data)
    return pyref.record_index(data, None if mode == "auto" else mode)


def main():
    fx_dir = os.path.join(HERE, "fixtures")
    out_dir = os.path.join(HERE, "expected")
    os.makedirs(out_dir, exist_ok=True)
    manifest = {}
    for name in sorted(os.listdir(fx_dir)):
        data = open(os.path.join(fx_dir, name), "rb").read()
        entry = {"size": len(data), "sha256": hashlib.sha256(data).hexdigest(),
                 "detect": pyref.detect_all(data), "modes": {}}
        for mode in MODES:
            rows, err = run(data, mode)
            idx = pyref.rows_to_idx(rows)
            with open(os.path.join(out_dir, f"{name}.{mode}.idx"), "wb") as f:
                f.write(idx)
            entry["modes"][mode] = {"count": len(rows), "err_hex": err.hex() if err is not None else None,
                                    "idx_sha256": hashlib.sha256(idx).hexdigest()}
        manifest[name] = entry
    with open(os.path.join(out_dir, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(f"wrote {len(manifest)} fixtures")


if __name__ == "__main__":
    main()
