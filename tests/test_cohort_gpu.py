"""One message cohort on the device (binquant_amd.cohort.process_cohort:
ContextEvaluator.process_data, producers/context_evaluator.py:347-512, for a
whole 15-minute cohort): the cohort's outputs equal the stage calls made one
by one, the 1h resample with a fixed bin count equals the read-back one, and
the whole cohort captured as one hipGraph replays bit for bit on new inputs
(no host synchronisation inside, no stale buffers)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(S, T, seed):
    from binquant_amd.synth import numpy_panel

    p5 = numpy_panel(S, T, seed0=seed, edges=True)
    p15 = numpy_panel(S, T, seed0=seed + 1000, edges=True)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    ts = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)
    ins = [d(p5[k]) for k in ("open", "high", "low", "close", "volume")]
    ins += [d(p15[k]) for k in ("open", "high", "low", "close", "volume")]
    ins += [d(np.broadcast_to(ts, (S, T))), d(ts), d(p15["close"][0])]
    return ins


def test_cohort_equals_stage_calls(cuda):
    from binquant_amd import engine, signals, strategies
    from binquant_amd.cohort import RESAMPLE_AGG, process_cohort

    S, T = 48, 400
    ins = _inputs(S, T, 5)
    o5, h5, l5, c5, v5, o15, h15, l15, c15, v15, ts15, bts, bc = ins
    out = process_cohort(*ins)
    for k, v in engine.enrich(o15, h15, l15, c15, v15).items():
        np.testing.assert_array_equal(out[f"e15.{k}"].cpu().numpy(), v.cpu().numpy(), err_msg=k)
    _, res, nb = engine.resample(ts15, {"open": o15, "high": h15, "low": l15, "close": c15, "volume": v15},
                                 RESAMPLE_AGG, 3_600_000)
    assert torch.equal(out["h1.bins"], nb)
    B = int(nb.max())
    for k, v in res.items():
        np.testing.assert_array_equal(out[f"h1.{k}"][:, :B].cpu().numpy(), v.cpu().numpy(), err_msg=k)
    lead = signals.gradual_gainer_leadership(ts15, c15, bts, bc)
    for k, v in lead.items():
        assert torch.equal(out[f"lead.{k}"], v), k
    spike = strategies.failed_spike_features(o15, h15, l15, c15, v15, v15 * c15, exact=True)
    for k, v in spike.items():
        np.testing.assert_array_equal(out[f"spike.{k}"].cpu().numpy(), v.cpu().numpy(), err_msg=k)
    part, last = engine.context_partials(h15, l15, c15, max_bars=400, last=True)
    assert torch.equal(out["context.partial"], part)


def test_cohort_graph_replays_bit_exact(cuda):
    from binquant_amd.cohort import process_cohort
    from binquant_amd.graphs import CapturedPipeline

    S, T = 64, 400
    a, b = _inputs(S, T, 11), _inputs(S, T, 12)
    g = CapturedPipeline(process_cohort, *a)
    got = g(*b)
    want = process_cohort(*b)
    torch.cuda.synchronize()
    assert set(got) == set(want)
    for k in want:
        x, y = got[k].cpu().numpy(), want[k].cpu().numpy()
        if k.startswith("h1."):   # bins past a row's count are unwritten
            n = int(want["h1.bins"].max())
            x, y = x[..., :n] if x.ndim == 2 else x, y[..., :n] if y.ndim == 2 else y
        np.testing.assert_array_equal(x, y, err_msg=k)


def test_cohort_branches_equal_one_stream(cuda, monkeypatch):
    """The four concurrent branches (side streams forked from and joined to
    the caller's stream) give the one-stream outputs bit for bit, eager and
    as a replayed graph, and the caller's stream sees finished outputs."""
    from binquant_amd import cohort
    from binquant_amd.graphs import CapturedPipeline

    S, T = 96, 400
    a, b = _inputs(S, T, 21), _inputs(S, T, 22)
    monkeypatch.setattr(cohort, "_COHORT_STREAMS", False)
    one = {k: v.clone() for k, v in cohort.process_cohort(*b).items()}
    monkeypatch.setattr(cohort, "_COHORT_STREAMS", True)
    many = cohort.process_cohort(*b)
    monkeypatch.setattr(cohort, "_COHORT_STREAMS", "capture")   # the default: branches inside the capture only
    g = CapturedPipeline(cohort.process_cohort, *a)
    rep = g(*b)
    torch.cuda.synchronize()
    assert list(many) == list(one)
    n = int(one["h1.bins"].max())
    for k in one:
        for name, got in (("eager", many[k]), ("graph", rep[k])):
            x, y = got.cpu().numpy(), one[k].cpu().numpy()
            if k.startswith("h1.") and x.ndim == 2:
                x, y = x[:, :n], y[:, :n]
            np.testing.assert_array_equal(x, y, err_msg=f"{name} {k}")


def test_cohort_h1_gap_keeps_newest_bins_and_btc_change(cuda):
    """pandas' 1h resample emits every empty hour of a gap, so a
    15m frame with a multi-hour gap has more bins than T15 // 4 + 2. The
    cohort keeps each row's NEWEST bins (bq_resample_tail): h1.bins - 1 is
    the latest hour, h1.dropped counts the oldest bins left out, and the kept
    bins equal the tail of the full read-back resample. Also the a12 BTC
    change with a missing close at t - 96 (pandas' pad fill)."""
    from binquant_amd import engine
    from binquant_amd.cohort import RESAMPLE_AGG, process_cohort
    from oracle import indicators_ref as ref

    S, T = 16, 400
    ins = _inputs(S, T, 31)
    ts = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)
    ts = np.broadcast_to(ts, (S, T)).copy()
    ts[::2, 200:] += 3_600_000 * np.arange(1, S // 2 + 1)[:, None] * 5   # gaps of 5, 10, ... hours
    ins[10] = torch.from_numpy(ts).cuda()
    btc = ins[12].cpu().numpy().copy()
    btc[-97] = np.nan
    btc[-1] = np.nan
    ins[12] = torch.from_numpy(btc).cuda()
    out = process_cohort(*ins)
    B1 = T // 4 + 2
    _, res, nb = engine.resample(ins[10], {k: ins[5 + i] for i, k in enumerate(("open", "high", "low", "close", "volume"))},
                                 RESAMPLE_AGG, 3_600_000)
    nb = nb.cpu().numpy()
    assert nb.max() > B1
    bins = out["h1.bins"].cpu().numpy()
    drop = out["h1.dropped"].cpu().numpy()
    np.testing.assert_array_equal(bins, np.minimum(nb, B1))
    np.testing.assert_array_equal(drop, np.maximum(nb - B1, 0))
    for k, v in res.items():
        full = v.cpu().numpy()
        got = out[f"h1.{k}"].cpu().numpy()
        for s in range(S):
            np.testing.assert_array_equal(got[s, : bins[s]], full[s, drop[s] : nb[s]], err_msg=f"{k}[{s}]")
    want = ref.pct_change_pad(btc, 96)[-1] * 100
    got = float(out["btc.change_24h"].cpu().numpy()[0])
    assert got == want, (got, want)
