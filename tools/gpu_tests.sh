# GPU: a pytest selection only. Usage: bash tools/gpu_tests.sh "<-k expr>" [files...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
K=$1; shift
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/t/gpu_tests.log 2>&1
rc=$?
tail -60 gpurun_out/t/gpu_tests.log | grep -E "Error|error|assert|FAILED|passed|failed" | head -60
exit $rc
