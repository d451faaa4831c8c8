cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tail
for s in 11520 12288 12500 13056; do
  timeout -k 10 120 python bench.py --symbols $s --no-rows --no-tick --no-cpu-baseline --no-breadth --steps 20 > gpurun_out/tail/s$s.json 2>gpurun_out/tail/s$s.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tail/s$s.json'));r=d['roofline'];print($s, r['kernel_ms'], $s/r['kernel_ms'], r['frac'])"
done
