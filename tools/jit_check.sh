# GPU tests of the fused programs (both evaluations) and the strategy
# pipelines, then the per-kernel pipeline breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/jit
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/jit/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 gpurun_out/jit/gpu_tests.log; exit 1; }
tail -1 gpurun_out/jit/gpu_tests.log
bash tools/pipeline_profile.sh
