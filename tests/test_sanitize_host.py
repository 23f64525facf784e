"""CPU: the host side of the C ABI and the C oracle under ASan + UBSan (tools/sanitize.sh).

The C-ABI layer is rebuilt with host-only sanitizers (libshockidx_san.so; device code is
unchanged -- GPU sanitizers are not used on this pool) and the oracle with clang's
-fsanitize=address,undefined; a child pytest loads both with the sanitizer runtime preloaded
and runs the CPU tests that call into them.  Any ASan / UBSan report aborts the child."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_sanitizers():
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), "-x",
                        "--ignore=tests/test_sanitize_host.py",
                        "tests/test_abi.py", "tests/test_oracle_part.py", "tests/test_oracle_filter.py",
                        "tests/test_oracle_subset.py", "tests/test_oracle_chunk.py", "tests/test_oracle_regex.py"],
                       cwd=ROOT, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error:" not in tail, tail
