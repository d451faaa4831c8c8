# GPU check after a kernel change: all -m gpu tests, replay A/B (auto vs
# forced variants, digests must agree), per-row device timings
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/d3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/d3/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/d3/gpu_tests.log; exit 1; }
tail -2 gpurun_out/d3/gpu_tests.log
rm -rf gpurun_out/replay_ab
QUICK=1 SPWS="${SPWS:-64}" bash tools/replay_ab.sh
timeout -k 10 300 python tools/row_costs.py > gpurun_out/d3/row_costs.log 2>&1 || { echo ROWS_FAILED; tail gpurun_out/d3/row_costs.log; exit 1; }
