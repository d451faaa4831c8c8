# GPU: a pytest selection (-k expression in $1), then the pipeline breakdown ($PIPES)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/quick
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${1:+-k "$1"} > gpurun_out/quick/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 gpurun_out/quick/gpu_tests.log; exit 1; }
tail -1 gpurun_out/quick/gpu_tests.log
bash tools/pipeline_profile.sh
