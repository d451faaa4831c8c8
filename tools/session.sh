# One GPU session: parity tests (recording the fused-program manifest), the
# manifest tool, the default bench line. Usage: bash tools/session.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r2}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
K=${2:+-k "$2"}
BQ_FUSED_MANIFEST=$O/manifest_tests.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $K > $O/gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u tools/fused_manifest.py $O/manifest_tool.jsonl > $O/manifest.log 2>&1 || { echo MANIFEST_FAILED; tail -20 $O/manifest.log; exit 1; }
tail -1 $O/manifest.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAILED; tail -20 $O/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$O/bench.json')); print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'], d.get('shard'), d.get('tick'), d.get('store',{}).get('p99_ms'), d.get('cpu_baseline'))"
echo SESSION_DONE
