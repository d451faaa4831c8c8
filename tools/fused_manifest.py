"""Record the fused-program manifest (binquant_amd/fused_manifest.json) on a
GPU: runs every strategy / signal pipeline at the live (1000 x 400) and bench
(12 500 x 2 000) shapes plus the smoke stage with BQ_FUSED_MANIFEST set, so
that __graft_entry__.build() can compile all of them ahead of a deploy.
Usage (GPU box): python tools/fused_manifest.py <out.jsonl>"""
import os
import sys

out = sys.argv[1]
if os.path.exists(out):
    os.remove(out)
os.environ["BQ_FUSED_MANIFEST"] = out
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from binquant_amd import fused as F  # noqa: E402
from binquant_amd import engine, signals, strategies  # noqa: E402
from binquant_amd.synth import device_panel  # noqa: E402

for S, T in ((8, 600), (1000, 400), (12_500, 2_000)):
    p = device_panel(S, T, seed=1)
    o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
    qv = v * c
    strategies.activity_burst_features(o, h, l, c, v, qv)
    strategies.activity_burst_features(o, h, l, c, v, None)
    strategies.pump_score_features(o, h, l, c, v, c[0])
    strategies.failed_spike_features(o, h, l, c, v, qv)
    signals.wilder_rsi(c)
    signals.adx(h, l, c)
    signals.zscore(c)
    signals.trend_score(c)
    signals.top_gainer_features(o, h, l, c, v, qv)
    signals.mean_reversion_features(o, h, l, c, v, engine.enrich(o, h, l, c, v, columns=("ATR",))["ATR"])
    C, O = F.inp(c), F.inp(o)
    F.run({"body": (C - O).abs() / (O + 1e-6), "up": C > F.shift(C, 1)})   # __graft_entry__.smoke's stage
    torch.cuda.synchronize()
    del p, o, h, l, c, v, qv
    torch.cuda.empty_cache()
n = sum(1 for _ in open(out))
print(f"manifest: {n} program structures -> {out}; {F.native_stats()}")
