#!/bin/bash
# the whole -m gpu suite (as the driver runs it) + smoke
set -o pipefail
export TMPDIR=/tmp
O=$(pwd)/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/full_pytest.log 2>&1 || { tail -40 $O/full_pytest.log; exit 1; }
tail -2 $O/full_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
