#!/bin/bash
# Round-4 GPU session t: the whole GPU suite + smoke on the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
