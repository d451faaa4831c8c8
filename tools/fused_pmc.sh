# PMC counters of the fused interpreter on the tools/fused_bench.py programs
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 python3 $R/tools/fused_bench.py > $R/gpurun_out/fused_bench.jsonl || { echo FB_FAILED; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/fused_pmc -o p1 -- python3 $R/tools/fused_bench.py > /dev/null 2>&1 || { echo PMC_FAILED; exit 1; }
echo FUSED_PMC_DONE
