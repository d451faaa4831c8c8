# GPU: rolling/strategy parity tests, order-statistic A/B, pipeline breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rank
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/rank/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 gpurun_out/rank/gpu_tests.log; exit 1; }
tail -1 gpurun_out/rank/gpu_tests.log
bash tools/rank_ab.sh || exit 1
bash tools/pipeline_profile.sh
