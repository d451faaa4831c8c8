# GPU: store/accumulator parity tests + the tick profile + the bench's store leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sc
timeout -k 10 600 python -u -m pytest tests/test_store_gpu.py tests/test_regime_scoring_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sc/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "Error|error|assert|FAILED" gpurun_out/sc/tests.log | head -30; tail -5 gpurun_out/sc/tests.log; exit 1; }
tail -1 gpurun_out/sc/tests.log
timeout -k 10 300 python tools/store_profile.py > gpurun_out/sc/prof.txt 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/sc/prof.txt; exit 1; }
head -30 gpurun_out/sc/prof.txt
timeout -k 10 300 python -c "
import sys, json, types; sys.argv=['bench.py']; import bench, torch
a = bench.parse(); a.store_ticks = 400
print(json.dumps(bench.bench_store(a, torch.device('cuda'))))" > gpurun_out/sc/store_leg.json 2>&1 || { echo LEG_FAILED; tail gpurun_out/sc/store_leg.json; exit 1; }
tail -1 gpurun_out/sc/store_leg.json
