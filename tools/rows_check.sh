# GPU: parity tests of the given files, then the bench's rows leg (no CPU timings)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rc
timeout -k 10 600 python -u -m pytest ${@:-tests/test_beta_corr.py} -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/rc/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "^E |FAILED" gpurun_out/rc/tests.log | head -30; tail -3 gpurun_out/rc/tests.log; exit 1; }
tail -1 gpurun_out/rc/tests.log
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py', '--no-cpu-baseline']; import bench, torch
a = bench.parse()
r = bench.bench_rows(a, torch.device('cuda'))
for k, v in r.items():
    print(k, v if isinstance(v, str) else (round(v['ms'], 3), round(v['frac'], 3)))" > gpurun_out/rc/rows.txt 2>&1 || { echo ROWS_FAILED; tail gpurun_out/rc/rows.txt; exit 1; }
cat gpurun_out/rc/rows.txt
