# tile rank A/B: rolling parity on the default library, then tools/rank_ab.py
# (tile implementation) for the default and a variant library
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rk2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rolling_impls_gpu.py tests/test_strategies_gpu.py -m gpu > gpurun_out/rk2/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/rk2/tests.log; exit 1; }
tail -1 gpurun_out/rk2/tests.log
for rep in 1 2; do
  BQ_RANK_IMPL=${IMPL:-tile} timeout -k 10 300 python3 tools/rank_ab.py > gpurun_out/rk2/new_$rep.jsonl || exit 1
  BQ_LIB_PATH=$PWD/$BQ_AB_LIB BQ_RANK_IMPL=${IMPL:-tile} timeout -k 10 300 python3 tools/rank_ab.py > gpurun_out/rk2/old_$rep.jsonl || exit 1
done
python3 - <<'PY'
import json
for rep in (1, 2):
    new=[json.loads(l) for l in open(f'gpurun_out/rk2/new_{rep}.jsonl')]; old=[json.loads(l) for l in open(f'gpurun_out/rk2/old_{rep}.jsonl')]
    for a,b in zip(new,old):
        if a['S'] == 12500: print(rep, a['w'], a['stat'], a['q'], 'new', round(a['ms'],4), 'old', round(b['ms'],4), 'same' if a['digest']==b['digest'] else 'DIFF')
PY
