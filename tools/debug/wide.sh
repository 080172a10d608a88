set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_join_sort_window.py tests/test_pipeline.py -m gpu -k "table or widened" > gpurun_out/wide_tests.log 2>&1 || { tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -3 gpurun_out/wide_tests.log
timeout -k 10 400 python tools/bench_configs.py --only shapes > gpurun_out/shapes_wide.jsonl 2> gpurun_out/shapes_wide.err || { tail -5 gpurun_out/shapes_wide.err; exit 1; }
cut -c1-330 gpurun_out/shapes_wide.jsonl
