import os, sys, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from binquant_amd import engine
from binquant_amd.synth import device_panel
p = device_panel(12500, 2000, seed=3); v = p["volume"]
def t(fn):
    fn(); torch.cuda.synchronize()
    a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    a.record(); [fn() for _ in range(3)]; b.record(); torch.cuda.synchronize(); return a.elapsed_time(b)/3
print(os.environ.get("BQ_RANK_SEG_MULT"), "med19 %.3f q80 %.3f q48 %.3f max6 %.3f" % (t(lambda: engine.rolling(v,19,"median",shift=2)), t(lambda: engine.rolling(v,80,"quantile",q=0.92,min_periods=20)), t(lambda: engine.rolling(v,48,"quantile",q=0.8,shift=1)), t(lambda: engine.rolling(v,6,"max",shift=1))))
