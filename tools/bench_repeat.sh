# headline leg only, N times on one box (box-to-box / run-to-run spread)
cd $GRAFT_REPO_ROOT
for i in $(seq ${1:-3}); do
  timeout -k 10 120 python bench.py --no-rows --no-tick --no-cpu-baseline --no-breadth --steps 30 > gpurun_out/bench_rep_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_rep_$i.json'));r=d['roofline'];print('rep $i', round(r['kernel_ms'],4), round(r['frac'],4))"
done
