# SQ counter passes over `python tools/call_prof.py $CALL $S $T`, summed per dispatch of kernels matching $KERN
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
O=$R/gpurun_out/kern_pmc_$CALL
rm -rf $O; mkdir -p $O
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/tools/${PROG:-call_prof.py} $CALL $S $T > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for p in ("p1", "p2"):
    f = glob.glob("$O/%s/**/*counter_collection.csv" % p, recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "$KERN" in r["Kernel_Name"]:
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print("%-24s %.4g  (%d dispatches)" % (k, sum(v.values()) / len(v), len(v)))
PY
