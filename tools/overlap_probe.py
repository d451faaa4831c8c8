"""Does an HBM-bound pass overlap a VALU-bound order statistic on MI355X?
Times, at 12.5k x 2k: the burst pass alone, the two w = 19 slide medians
alone, both serially on one stream, both on two streams; then the whole a17
row once on the full panel against its two row halves on two streams (the
halves' outputs stay separate: the probe measures the overlap, not a drop-in).

    PYTHONPATH=. python tools/overlap_probe.py
"""
import torch

from binquant_amd import engine, strategies
from binquant_amd.engine import Roll as R
from binquant_amd.synth import device_panel

S, T = 12_500, 2_000
p = device_panel(S, T, seed=99)
o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
qv = v * c
bp = strategies.BurstParams()
bw = max(bp.lookback_window, 2)


def meds(vv, qq):
    return engine.rolling_many(R(vv, bw - 1, "median", min_periods=bw - 1, shift=2),
                               R(qq, bw - 1, "median", min_periods=bw - 1, shift=2))


med = meds(v, qv)
fA = lambda: engine.burst_features(o, h, l, c, v, qv, med[0], med[1], bp)   # noqa: E731
fB = lambda: meds(v, qv)   # noqa: E731
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def both_streams(f1, f2):
    def run():
        cur = torch.cuda.current_stream()
        e = torch.cuda.Event()
        e.record(cur)
        sA.wait_event(e)
        sB.wait_event(e)
        with torch.cuda.stream(sA):
            f1()
        with torch.cuda.stream(sB):
            f2()
        ea, eb = torch.cuda.Event(), torch.cuda.Event()
        ea.record(sA)
        eb.record(sB)
        cur.wait_event(ea)
        cur.wait_event(eb)
    return run


halves = [slice(0, S // 2), slice(S // 2, S)]
hp = [tuple(x[hs].contiguous() for x in (o, h, l, c, v, qv)) for hs in halves]
g = [lambda a=a: strategies.activity_burst_features(*a) for a in hp]
whole = lambda: strategies.activity_burst_features(o, h, l, c, v, qv)   # noqa: E731

for rnd in range(2):
    ta, tb = timed(fA), timed(fB)
    ts = timed(lambda: (fA(), fB()))
    tc = timed(both_streams(fA, fB))
    tw = timed(whole)
    th = timed(lambda: (g[0](), g[1]()))
    t2 = timed(both_streams(g[0], g[1]))
    print(f"round {rnd}: burst pass {ta:.3f} ms, medians {tb:.3f}, serial {ts:.3f}, two streams {tc:.3f}; "
          f"a17 whole {tw:.3f}, halves serial {th:.3f}, halves on two streams {t2:.3f}", flush=True)
