"""Generate golden vectors from the REAL reference (carkod/binquant) modules.

Run in the build container only (the reference does not exist on the GPU box):

    python tests/golden/make_golden.py            # writes tests/golden/*.npz|json

The reference targets Python 3.11 and imports packages absent from this
offline image (pybinbot, pandera, dotenv). A throw-away shim directory supplies
NAMES ONLY for those imports — enums, a permissive model base class, a
``__class_getitem__`` for pandera's DataFrame type and ``datetime.UTC`` — and
no arithmetic (round_numbers is only used by outputs we do not take). The
reference modules are imported in place from /root/reference by a child
process; nothing of the reference is copied into this repository. Only the
numeric inputs/outputs below are written.

Fixtures:
  market_features.npz   LiveMarketContextAccumulator._compute_symbol_features
                        (market_regime/live_market_context_accumulator.py:244-297)
  market_context.json   refresh_context_for_timestamp + annotate_context
                        (:72-84, :95-242; regime_transitions.py:25-232)
  rsi_helpers.npz       MeanReversionFade._rsi (strategies/mean_reversion_fade.py:88-109),
                        BBExtremeReversion._compute_rsi (strategies/coinrule/bb_extreme_reversion.py:134-150)
  activity_burst.npz    ActivityBurstPump.compute_indicators (strategies/activity_burst_pump.py:51-158)
  liquidation_sweep.npz LiquidationSweepPump.compute_pump_score (strategies/liquidation_sweep_pump.py:195-269)
  failed_spike.npz      FailedSpikeFade.detect (strategies/failed_spike_fade.py:258-544)
  signal_helpers.npz    a20 helpers: MeanReversionFade._rsi/_trend_score,
                        RangeBbRsiMeanReversion._compute_adx/_compute_zscore,
                        TopGainerEarlyMomentum._features on every prefix
  beta_corr.npz         ContextEvaluator.dynamic_btc_beta_corr (producers/context_evaluator.py:154-194)
                        on every prefix (last-row value), BTC pct_change(96) (:427-430).
                        round_numbers is stubbed to identity: values are unrounded.
  ohlcv_pins.npz        the frames of the reference's own make_ohlcv_df(n=50, oversold=...)
                        (tests/test_coinrule_price_tracker.py:148-189) behind its
                        Indicators.mfi pins (:226-248) and the docstring's RSI < 30 /
                        MACD < 0 claim for the oversold frame
  inf_windows.npz       the burst / pump / spike frames of 6 x 700 candles whose rolling
                        windows meet +-inf (long zero-volume halts, zero closes), every
                        column at every candle (pandas' window ops skip infinities)
  leadership.npz        GradualGainerRetest._leadership_allows on every prefix frame
                        (strategies/gradual_gainer_retest.py:131-196): the reference
                        test's make_frames + a 20 x 360 panel with BTC gaps
  strategy_panel.npz    64 symbols x 1100 candles (tests/golden/panel_gen.py, inputs
                        regenerated from seeds, digest stored) through the real
                        ActivityBurstPump.compute_indicators, LiquidationSweepPump
                        .compute_pump_score, FailedSpikeFade.detect,
                        _compute_symbol_features (400-bar store window) and the a20
                        helpers; outputs recorded at 48 sampled positions per symbol
                        (panel_gen.sample_positions: last rows, tile boundary, random)

  headline_twins.npz    per-candle pins of the headline enrich columns from the reference's
                        own twins, on every prefix of 4 frames (random walk across a
                        1024-candle tile, a 1e-3-priced walk, constant runs, NaN gaps):
                        LiveMarketContextAccumulator._compute_symbol_features (ema20, ema50,
                        atr_pct = rolling-14 TR mean / close, bb_width = ddof-0 rolling-20
                        (upper - lower) / |mid|, trend_score; :256-272),
                        BBExtremeReversion._compute_rsi (SMA RSI, windows 14 and 6;
                        bb_extreme_reversion.py:134-150) and MeanReversionFade._trend_score
                        with its EMA windows set to 9 / 21 — the expression of
                        price_tracker.py:204-205 and inverse_price_tracker.py:157-158 —
                        and at its own 20 / 50 (mean_reversion_fade.py:150-155)

  store_gaps.json       a second scripted store feed (the store_sequence.json format) whose
                        candles miss their high and / or low — None, non-numeric strings,
                        NaN — which MarketStateStore keeps (it drops only a missing close,
                        market_state_store.py:84): _compute_symbol_features' skip-NaN true
                        range and min_periods=1 windows over such histories

Usage: python tests/golden/make_golden.py [--only pins,panel,leadership,inf,btc_change,twins,store_gaps]
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import textwrap
from pathlib import Path

HERE = Path(__file__).resolve().parent
REFERENCE = Path("/root/reference")

SHIM_FILES = {
    "sitecustomize.py": """
        import datetime as _d
        if not hasattr(_d, "UTC"):
            _d.UTC = _d.timezone.utc
    """,
    "pybinbot/__init__.py": """
        import enum

        class ExchangeId(str, enum.Enum):
            BINANCE = "binance"
            KUCOIN = "kucoin"

        class MarketType(str, enum.Enum):
            SPOT = "SPOT"
            FUTURES = "FUTURES"

        class Position(str, enum.Enum):
            long = "long"
            short = "short"

        class _Interval(str, enum.Enum):
            one_minute = "1m"
            five_minutes = "5m"
            fifteen_minutes = "15m"
            one_hour = "1h"
            FIVE_MINUTES = "5min"
            FIFTEEN_MINUTES = "15min"

            def get_ms(self):
                return {"1m": 60_000, "5m": 300_000, "15m": 900_000, "1h": 3_600_000,
                        "5min": 300_000, "15min": 900_000}[self.value]

        BinanceKlineIntervals = _Interval
        KucoinKlineIntervals = _Interval

        def round_numbers(value, decimals=6):
            return value

        class _Model:
            def __init__(self, *args, **kwargs):
                for k, v in kwargs.items():
                    setattr(self, k, v)

            def __class_getitem__(cls, item):
                return cls

        def __getattr__(name):
            return type(name, (_Model,), {})
    """,
    "pandera/__init__.py": "",
    "pandera/typing/__init__.py": """
        import pandas as pd

        class DataFrame(pd.DataFrame):
            def __class_getitem__(cls, item):
                return pd.DataFrame
    """,
    "dotenv/__init__.py": """
        def load_dotenv(*args, **kwargs):
            return False
    """,
    # python-telegram-bot (imported by consumers.telegram_consumer): names only
    "telegram/__init__.py": """
        class _Any:
            def __init__(self, *a, **k):
                pass

            def __getattr__(self, n):
                return _Any()

            def __call__(self, *a, **k):
                return _Any()

        def __getattr__(name):
            return type(name, (_Any,), {})
    """,
    "telegram/constants.py": "from telegram import __getattr__  # noqa\n",
    "telegram/error.py": "from telegram import __getattr__  # noqa\n",
    "telegram/helpers.py": "from telegram import __getattr__  # noqa\n",
}


def write_shim(root: Path) -> None:
    for rel, body in SHIM_FILES.items():
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(textwrap.dedent(body))


# ---------------------------------------------------------------------------
# child process: runs with PYTHONPATH=<shim>:/root/reference
# ---------------------------------------------------------------------------
def child(out_dir: Path, only: set[str] | None = None) -> None:
    if only:
        if "pins" in only:
            ohlcv_pins(out_dir)
        if "panel" in only:
            strategy_panel(out_dir)
        if "leadership" in only:
            leadership(out_dir)
        if "inf" in only:
            inf_windows(out_dir)
        if "btc_change" in only:
            btc_change(out_dir)
        if "twins" in only:
            headline_twins(out_dir)
        if "store_gaps" in only:
            store_gaps(out_dir)
        return
    import numpy as np
    import pandas as pd
    from types import SimpleNamespace

    from market_regime.live_market_context_accumulator import LiveMarketContextAccumulator
    from market_regime.market_state_store import MarketStateStore

    rng = np.random.default_rng(20261015)

    def walk(n, scale=100.0, vol=0.004, seed=None):
        r = np.random.default_rng(seed).normal(0, vol, n)
        c = scale * np.exp(np.cumsum(r))
        o = np.r_[c[0], c[:-1]]
        h = np.maximum(o, c) * (1 + np.random.default_rng(seed + 1).uniform(0, 0.003, n))
        l = np.minimum(o, c) * (1 - np.random.default_rng(seed + 2).uniform(0, 0.003, n))
        v = np.random.default_rng(seed + 3).lognormal(3, 1, n)
        return o, h, l, c, v

    # ---- 1. per-symbol market features ----------------------------------------
    cases = []
    for i, n in enumerate([1, 2, 3, 5, 14, 15, 19, 20, 21, 49, 50, 51, 120, 200, 400]):
        o, h, l, c, v = walk(n, scale=10 ** rng.uniform(-3, 4), seed=100 + i)
        cases.append((f"walk{n}", h, l, c))
    c = np.full(60, 0.3)
    cases.append(("const0.3", c * 1.0, c * 1.0, c))
    c = np.r_[np.linspace(1, 2, 30), np.full(30, 2.7)]
    cases.append(("ramp_then_flat", c * 1.01, c * 0.99, c))
    c = np.r_[np.linspace(5, 1, 30), np.zeros(3)]
    cases.append(("to_zero", c + 0.1, np.maximum(c - 0.1, 0), c))
    feats_cols = ["close", "return_pct", "ema20", "ema50", "above_ema20", "above_ema50",
                  "trend_score", "atr_pct", "bb_width"]
    arrays = {}
    names = []
    for name, h, l, c in cases:
        df = pd.DataFrame({"timestamp": np.arange(len(c)) * 60_000, "open": c, "high": h, "low": l,
                           "close": c, "volume": 1.0})
        f = LiveMarketContextAccumulator._compute_symbol_features("SYMUSDT", df)
        arrays[f"{name}__high"] = h
        arrays[f"{name}__low"] = l
        arrays[f"{name}__close"] = c
        if f is None:
            arrays[f"{name}__features"] = np.full(len(feats_cols), np.nan)
            arrays[f"{name}__none"] = np.array(True)
        else:
            arrays[f"{name}__features"] = np.array([float(getattr(f, k)) for k in feats_cols])
            arrays[f"{name}__none"] = np.array(False)
        names.append(name)
    arrays["names"] = np.array(names)
    arrays["feature_columns"] = np.array(feats_cols)
    np.savez(out_dir / "market_features.npz", **arrays)

    # ---- 2. cross-symbol context + regime annotation -----------------------------
    def context_dict(ctx):
        if ctx is None:
            return None
        d = ctx.model_dump()
        d["symbol_features"] = {k: v for k, v in sorted(d["symbol_features"].items())}
        d["metadata"] = {k: v for k, v in d["metadata"].items() if k != "fresh_symbols"}
        return d

    scenarios = {}
    # (a) 40 symbols seeded at 100+i closing at 103+i, BTC first
    store = MarketStateStore(max_bars_per_symbol=400)
    acc = LiveMarketContextAccumulator(store, btc_symbol="BTCUSDT")
    syms = ["BTCUSDT"] + [f"ALT{i}USDT" for i in range(1, 40)]
    panel = {}
    for i, s in enumerate(syms):
        base = 100.0 + i
        rows = [dict(timestamp=1_000, open=base * 0.99, high=base * 1.01, low=base * 0.98, close=base, volume=1000.0),
                dict(timestamp=2_000, open=(base + 3) * 0.99, high=(base + 3) * 1.01, low=(base + 3) * 0.98,
                     close=base + 3, volume=1000.0)]
        panel[s] = rows
        for r in rows:
            store.update(s, r)
    ctx = acc.refresh_context_for_timestamp(2_000)
    scenarios["trend_up_40"] = dict(panel=panel, timestamps=[2_000], contexts=[context_dict(ctx)], max_bars=400,
                                    btc="BTCUSDT", symbols=syms)

    # (b) 64 random-walk symbols x 260 bars; contexts at the last 6 timestamps
    #     (transitions between consecutive contexts), history cap 200.
    for label, drift in (("random_64", 0.0), ("selloff_64", -0.004)):
        store = MarketStateStore(max_bars_per_symbol=200)
        acc = LiveMarketContextAccumulator(store, btc_symbol="BTCUSDT")
        syms = ["BTCUSDT"] + [f"S{i:02d}USDT" for i in range(1, 64)]
        T = 260
        panel = {}
        ts_list = [60_000 * (t + 1) for t in range(T)]
        for j, s in enumerate(syms):
            r = np.random.default_rng(500 + j).normal(drift, 0.006, T)
            c = (10 ** np.random.default_rng(900 + j).uniform(-2, 3)) * np.exp(np.cumsum(r))
            o = np.r_[c[0], c[:-1]]
            h = np.maximum(o, c) * 1.002
            l = np.minimum(o, c) * 0.998
            rows = [dict(timestamp=ts_list[t], open=float(o[t]), high=float(h[t]), low=float(l[t]),
                         close=float(c[t]), volume=1.0) for t in range(T)]
            panel[s] = rows
        for t in range(T - 6):
            for s in syms:
                store.update(s, panel[s][t])
        contexts = []
        for t in range(T - 6, T):
            for s in syms:
                store.update(s, panel[s][t])
            contexts.append(context_dict(acc.refresh_context_for_timestamp(ts_list[t])))
        scenarios[label] = dict(panel=panel, timestamps=ts_list[T - 6:], contexts=contexts, max_bars=200,
                                btc="BTCUSDT", symbols=syms)
    # panels as [S, T] arrays (npz); contexts as JSON
    arrays = {}
    meta = {}
    for label, sc in scenarios.items():
        syms_ = sc["symbols"]
        for f in ("timestamp", "open", "high", "low", "close", "volume"):
            arrays[f"{label}__{f}"] = np.array([[r[f] for r in sc["panel"][s]] for s in syms_], dtype=np.float64)
        meta[label] = {k: v for k, v in sc.items() if k != "panel"}
    np.savez_compressed(out_dir / "market_context_panels.npz", **arrays)
    with open(out_dir / "market_context.json", "w") as f:
        json.dump(meta, f, separators=(",", ":"))

    # ---- 3. RSI helpers -------------------------------------------------------------
    from strategies.coinrule.bb_extreme_reversion import BBExtremeReversion
    from strategies.mean_reversion_fade import MeanReversionFade

    rsi = {}
    series = {
        "walk": walk(300, seed=7)[3],
        "rally": 100.0 + np.arange(60, dtype=float),
        "flat": np.full(40, 5.0),
        "selloff": 100.0 - 0.5 * np.arange(60, dtype=float),
    }
    for k, c in series.items():
        rsi[f"{k}__close"] = c
        rsi[f"{k}__wilder"] = MeanReversionFade._rsi(pd.Series(c)).to_numpy()
        last = []
        for n in range(1, len(c) + 1):
            v = BBExtremeReversion._compute_rsi(pd.Series(c[:n]), 14)
            last.append(np.nan if v is None else v)
        rsi[f"{k}__sma_rsi_last"] = np.array(last)
    np.savez(out_dir / "rsi_helpers.npz", **rsi)

    # ---- 4. activity burst features ------------------------------------------------
    from strategies.activity_burst_pump import ActivityBurstPump

    ctx_ns = SimpleNamespace(config=SimpleNamespace(env="test"), symbol="TESTUSDT", kucoin_symbol="TEST-USDT",
                             exchange=None, binbot_api=None, telegram_consumer=None, market_type=None,
                             at_consumer=None, _breadth_cross_tolerance=0.05, _autotrade_stress_threshold=0.35,
                             current_symbol_data=None, price_precision=8, qty_precision=8)
    abp = ActivityBurstPump(ctx_ns)
    out = {}
    for k, (with_quote, seed) in {"with_quote": (True, 31), "no_quote": (False, 32)}.items():
        o, h, l, c, v = walk(400, seed=seed)
        v = v.copy()
        spikes = np.random.default_rng(seed).choice(np.arange(30, 400), 12, replace=False)
        v[spikes] *= 8
        c = c.copy()
        c[spikes] *= 1.03
        h = np.maximum(h, c)
        df = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v})
        if with_quote:
            df["quote_asset_volume"] = v * c
        res = abp.compute_indicators(df)
        for col in res.columns:
            out[f"{k}__{col}"] = res[col].to_numpy(dtype=float)
    np.savez(out_dir / "activity_burst.npz", **out)

    # ---- 5. liquidation sweep pump score ------------------------------------------
    from strategies.liquidation_sweep_pump import LiquidationSweepPump

    lsp = object.__new__(LiquidationSweepPump)
    out = {}
    o, h, l, c, v = walk(400, seed=41)
    t = np.arange(400, dtype=np.int64) * 900_000
    df = pd.DataFrame({"open_time": t, "open": o, "high": h, "low": l, "close": c, "volume": v})
    bo, bh, bl, bc, bv = walk(400, scale=60000.0, seed=42)
    keep = np.ones(400, bool)
    keep[[50, 51, 52, 200]] = False   # missing BTC candles -> NaN gaps after the left merge
    dfb = pd.DataFrame({"open_time": t[keep], "close": bc[keep]})
    res = lsp.compute_pump_score(df, dfb)
    for col in res.columns:
        out[col] = res[col].to_numpy(dtype=float)
    out["btc_open_time"] = t[keep]
    out["btc_close"] = bc[keep]
    np.savez(out_dir / "liquidation_sweep.npz", **out)
    # ---- 6. BTC beta / correlation (producers/context_evaluator.py:154-194) ----
    from producers.context_evaluator import ContextEvaluator

    out = {}
    for k, (n, seed, rho) in {"corr_pos": (420, 61, 0.7), "corr_neg": (300, 62, -0.4), "short": (45, 63, 0.5)}.items():
        rb = np.random.default_rng(seed).normal(0, 0.004, n)
        ra = rho * rb + np.sqrt(1 - rho**2) * np.random.default_rng(seed + 1).normal(0, 0.006, n)
        btc = 60000.0 * np.exp(np.cumsum(rb))
        alt = 3.0 * np.exp(np.cumsum(ra))
        if k == "corr_pos":
            alt[200:260] = alt[200]   # flat stretch: constant returns window
        out[f"{k}__close"] = alt
        out[f"{k}__btc"] = btc
        betas, corrs = [], []
        for m in range(2, n + 1):
            ns = SimpleNamespace(df_15m=pd.DataFrame({"close": alt[:m]}), df_btc_15m=pd.DataFrame({"close": btc[:m]}))
            b, c = ContextEvaluator.dynamic_btc_beta_corr(ns, window=50)
            betas.append(b)
            corrs.append(c)
        out[f"{k}__beta_last"] = np.array([np.nan] + betas)
        out[f"{k}__corr_last"] = np.array([np.nan] + corrs)
        # BTC 24h change (:427-430): pct_change(periods=96) * 100, last value
        out[f"{k}__btc_change_96"] = (pd.Series(btc).pct_change(periods=96) * 100).to_numpy()
    np.savez(out_dir / "beta_corr.npz", **out)

    # ---- 7. FailedSpikeFade.detect (strategies/failed_spike_fade.py:258-544) ------
    from strategies.failed_spike_fade import FailedSpikeFade

    out = {}
    for k, (n, seed) in {"fsf_a": (400, 71), "fsf_b": (400, 72), "fsf_c": (150, 73)}.items():
        o, h, l, c, v = walk(n, seed=seed, vol=0.006)
        c = c.copy()
        v = v.copy()
        rng2 = np.random.default_rng(seed)
        for j in rng2.choice(np.arange(25, n - 2), 10, replace=False):   # volume + price spikes
            v[j] *= rng2.uniform(3, 8)
            c[j] *= 1 + rng2.choice([-1, 1]) * rng2.uniform(0.02, 0.06)
        o = np.r_[c[0], c[:-1]]
        h = np.maximum(np.maximum(o, c), h)
        l = np.minimum(np.minimum(o, c), l)
        df = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v, "quote_asset_volume": v * c})
        ns = SimpleNamespace(symbol="TESTUSDT", market_type=None, df_15m=df, telegram_consumer=None,
                             at_consumer=None, current_symbol_data=None, price_precision=8,
                             market_breadth_data=None, strategy_cooldowns={}, strategy_states={})
        fsf = FailedSpikeFade(ns)
        res = fsf.detect()
        for col in res.columns:
            out[f"{k}__{col}"] = res[col].to_numpy(dtype=float)
        out[f"{k}__calibrated"] = np.array([fsf.volume_cluster_min_ratio, fsf.price_break_base_threshold])
    np.savez(out_dir / "failed_spike.npz", **out)

    # ---- 8. inline signal helpers --------------------------------
    #   MeanReversionFade._rsi / _trend_score (strategies/mean_reversion_fade.py:88-155),
    #   RangeBbRsiMeanReversion._compute_adx / _compute_zscore
    #   (strategies/range_bb_rsi_mean_reversion.py:101-138),
    #   TopGainerEarlyMomentum._features (strategies/top_gainer_early_momentum.py:92-160),
    #   evaluated on every prefix df.iloc[:k] (they read the last row only).
    from strategies.mean_reversion_fade import MeanReversionFade
    from strategies.range_bb_rsi_mean_reversion import RangeBbRsiMeanReversion
    from strategies.top_gainer_early_momentum import TopGainerEarlyMomentum

    out = {}
    tg_keys = ["close", "open", "high", "low", "volume", "quote_volume", "previous_high", "return_1h", "return_2h",
               "return_6h", "extension_return", "extension_window_bars", "extension_cap", "candle_return",
               "volume_ratio", "quote_volume_ratio", "range_position", "upper_wick_fraction", "ema20", "ema50", "atr"]
    statuses = []
    for k, (n, seed, quote) in {"sig_a": (260, 81, True), "sig_b": (180, 82, False), "sig_c": (130, 83, True)}.items():
        o, h, l, c, v = walk(n, seed=seed, vol=0.008)
        c = c.copy()
        if k == "sig_a":
            c[60:80] = c[59] * np.cumprod(np.full(20, 1.01))   # monotonic rally: RSI -> 100
            c[120:150] = c[119]                                # flat: RSI neutral 50, std 0
        o = np.r_[c[0], c[:-1]]
        h = np.maximum(np.maximum(o, c), h)
        l = np.minimum(np.minimum(o, c), l)
        if k == "sig_a":
            h[120:150] = l[120:150] = c[120:150]
        df = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v,
                           "open_time": 1_700_000_000_000 + 900_000 * np.arange(n)})
        if quote:
            df["quote_asset_volume"] = v * c
        for col in df.columns:
            out[f"{k}__{col}"] = df[col].to_numpy(dtype=float)
        out[f"{k}__rsi"] = MeanReversionFade._rsi(df["close"]).to_numpy(dtype=float)
        out[f"{k}__trend_score"] = np.array([MeanReversionFade._trend_score(df["close"].iloc[:j])
                                             for j in range(1, n + 1)])
        out[f"{k}__adx"] = np.array([RangeBbRsiMeanReversion._compute_adx(df.iloc[:j], 14)
                                     for j in range(1, n + 1)])
        out[f"{k}__zscore"] = np.array([RangeBbRsiMeanReversion._compute_zscore(df.iloc[:j], 20)
                                        for j in range(1, n + 1)])
        tg = np.full((n, len(tg_keys)), np.nan)
        st = []
        for j in range(1, n + 1):
            vals, status = TopGainerEarlyMomentum._features(df.iloc[:j])
            st.append(status)
            if vals is not None:
                tg[j - 1] = [vals[key] for key in tg_keys]
        out[f"{k}__topgainer"] = tg
        statuses.append(st)
        out[f"{k}__topgainer_status"] = np.array(st)
    out["topgainer_keys"] = np.array(tg_keys)
    np.savez(out_dir / "signal_helpers.npz", **out)

    # ---- 9. MarketStateStore + accumulator under a scripted feed ---------------------
    store_sequence(out_dir, context_dict)
    # ---- 10. candidate scoring and portfolio selection ------------------------------
    scoring_and_selection(out_dir)
    # ---- 11. the reference's own pybinbot-boundary frames --------------------------
    ohlcv_pins(out_dir)
    # ---- 12. panel-size fixtures ------------------------------------------------------
    strategy_panel(out_dir)
    print("golden fixtures written to", out_dir)


def ohlcv_pins(out_dir: Path) -> None:
    """The frames of make_ohlcv_df (reference tests/test_coinrule_price_tracker.py:148-189),
    imported from the reference test module itself."""
    import importlib.util

    import numpy as np

    spec = importlib.util.spec_from_file_location("ref_test_price_tracker",
                                                  REFERENCE / "tests" / "test_coinrule_price_tracker.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    for case, oversold in (("oversold", True), ("uptrend", False)):
        df = mod.make_ohlcv_df(n=50, oversold=oversold)
        for col in ("open", "high", "low", "close", "volume", "close_time"):
            out[f"{case}__{col}"] = df[col].to_numpy(dtype=float)
    np.savez(out_dir / "ohlcv_pins.npz", **out)


def strategy_panel(out_dir: Path) -> None:
    """64 x 1100 panel through the reference's per-symbol functions."""
    from types import SimpleNamespace

    import numpy as np
    import pandas as pd

    sys.path.insert(0, str(HERE))
    import panel_gen

    from market_regime.live_market_context_accumulator import LiveMarketContextAccumulator
    from strategies.activity_burst_pump import ActivityBurstPump
    from strategies.failed_spike_fade import FailedSpikeFade
    from strategies.liquidation_sweep_pump import LiquidationSweepPump
    from strategies.mean_reversion_fade import MeanReversionFade
    from strategies.range_bb_rsi_mean_reversion import RangeBbRsiMeanReversion
    from strategies.top_gainer_early_momentum import TopGainerEarlyMomentum

    S, T = 64, 1100
    P = panel_gen.strategy_panel(S, T)
    keep, btc = panel_gen.btc_series(T)
    idx = panel_gen.sample_positions(S, T)
    out = {"digest": np.array(panel_gen.digest(P)), "positions": idx, "btc_keep": keep}
    open_time = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)
    dfb = pd.DataFrame({"open_time": open_time[keep], "close": btc[keep]})

    ctx_ns = SimpleNamespace(config=SimpleNamespace(env="test"), symbol="TESTUSDT", kucoin_symbol="TEST-USDT",
                             exchange=None, binbot_api=None, telegram_consumer=None, market_type=None,
                             at_consumer=None, _breadth_cross_tolerance=0.05, _autotrade_stress_threshold=0.35,
                             current_symbol_data=None, price_precision=8, qty_precision=8)
    abp = ActivityBurstPump(ctx_ns)
    lsp = object.__new__(LiquidationSweepPump)
    rec: dict[str, list] = {}

    def put(name, s, series):
        a = np.asarray(series, dtype=float)
        rec.setdefault(name, [None] * S)[s] = a[idx[s]]

    tg_keys = ["close", "previous_high", "return_1h", "return_2h", "return_6h", "extension_return",
               "extension_window_bars", "extension_cap", "candle_return", "volume_ratio", "quote_volume_ratio",
               "range_position", "upper_wick_fraction", "ema20", "ema50", "atr"]
    feat_cols = ["close", "return_pct", "ema20", "ema50", "above_ema20", "above_ema50", "trend_score", "atr_pct",
                 "bb_width"]
    calib = np.zeros((S, 2))
    for s in range(S):
        o, h, l, c, v, qv = (P[f][s] for f in panel_gen.FIELDS)
        df = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v})
        if s % 2 == 0:   # with and without quote_asset_volume (activity_burst_pump.py:69-133)
            df["quote_asset_volume"] = qv
        for col, ser in abp.compute_indicators(df.copy()).items():
            if col not in df.columns:
                put(f"abp__{col}", s, ser)
        dfl = pd.DataFrame({"open_time": open_time, "open": o, "high": h, "low": l, "close": c, "volume": v})
        for col, ser in lsp.compute_pump_score(dfl, dfb).items():
            if col not in dfl.columns:
                put(f"lsp__{col}", s, ser)
        dff = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v, "quote_asset_volume": qv})
        ns = SimpleNamespace(symbol="TESTUSDT", market_type=None, df_15m=dff, telegram_consumer=None,
                             at_consumer=None, current_symbol_data=None, price_precision=8,
                             market_breadth_data=None, strategy_cooldowns={}, strategy_states={})
        fsf = FailedSpikeFade(ns)
        for col, ser in fsf.detect().items():
            if col not in dff.columns:
                put(f"fsf__{col}", s, ser)
        calib[s] = [fsf.volume_cluster_min_ratio, fsf.price_break_base_threshold]
        put("a20__rsi", s, MeanReversionFade._rsi(pd.Series(c)))
        trend, adx, z, feats = [], [], [], []
        tg = np.full((idx.shape[1], len(tg_keys)), np.nan)
        st = []
        dft = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v,
                            "open_time": open_time, "quote_asset_volume": qv})
        for j, t in enumerate(idx[s]):
            trend.append(MeanReversionFade._trend_score(dft["close"].iloc[: t + 1]))
            adx.append(RangeBbRsiMeanReversion._compute_adx(dft.iloc[: t + 1], 14))
            z.append(RangeBbRsiMeanReversion._compute_zscore(dft.iloc[: t + 1], 20))
            vals, status = TopGainerEarlyMomentum._features(dft.iloc[: t + 1])
            st.append(status)
            if vals is not None:
                tg[j] = [vals[k] for k in tg_keys]
            lo = max(0, t - 400 + 1)   # MarketStateStore(400) history at candle t
            dfm = pd.DataFrame({"timestamp": open_time[lo : t + 1], "open": o[lo : t + 1], "high": h[lo : t + 1],
                                "low": l[lo : t + 1], "close": c[lo : t + 1], "volume": v[lo : t + 1]})
            f = LiveMarketContextAccumulator._compute_symbol_features("SYMUSDT", dfm)
            feats.append(np.full(len(feat_cols), np.nan) if f is None
                         else [float(getattr(f, k)) for k in feat_cols])
        rec.setdefault("a20__trend_score", [None] * S)[s] = np.array(trend, dtype=float)
        rec.setdefault("a20__adx", [None] * S)[s] = np.array(adx, dtype=float)
        rec.setdefault("a20__zscore", [None] * S)[s] = np.array(z, dtype=float)
        rec.setdefault("tg__values", [None] * S)[s] = tg
        rec.setdefault("tg__status", [None] * S)[s] = np.array(st)
        rec.setdefault("features", [None] * S)[s] = np.array(feats, dtype=float)
    for k, rows in rec.items():
        out[k] = np.stack(rows)
    out["fsf_calibrated"] = calib
    out["tg_keys"] = np.array(tg_keys)
    out["feature_columns"] = np.array(feat_cols)
    np.savez_compressed(out_dir / "strategy_panel.npz", **out)


def inf_windows(out_dir: Path) -> None:
    """inf_windows.npz: the three strategy frames on 6 symbols x 700 candles
    built so that their rolling windows meet +-inf — halts of 30-60 zero-volume
    bars (relative_volume = v / 0 = inf once the volume mean's window is all
    zero, then inside the 48-bar score / volume quantiles), zero closes (the
    pct changes after them are inf, inside the spike pass's sums and the
    quantile of |pct change|) — every output column at every candle:
      lsp__*  LiquidationSweepPump.compute_pump_score (liquidation_sweep_pump.py:195-269)
      abp__*  ActivityBurstPump.compute_indicators (activity_burst_pump.py:51-158)
      fsf__*  FailedSpikeFade.detect (failed_spike_fade.py:258-544)
    Inputs are stored beside them (open / high / low / close / volume / qv)."""
    from types import SimpleNamespace

    import numpy as np
    import pandas as pd

    from strategies.activity_burst_pump import ActivityBurstPump
    from strategies.failed_spike_fade import FailedSpikeFade
    from strategies.liquidation_sweep_pump import LiquidationSweepPump

    S, T = 6, 700
    g = np.random.default_rng(2024)
    P = {k: np.zeros((S, T)) for k in ("open", "high", "low", "close", "volume", "qv")}
    for s in range(S):
        c = 10.0 * (s + 1) * np.exp(np.cumsum(g.normal(0.0, 0.006, T)))
        v = g.lognormal(3.0, 1.0, T)
        o = np.r_[c[0], c[:-1]]
        h = np.maximum(o, c) * (1.0 + g.uniform(0.0, 0.003, T))
        l = np.minimum(o, c) * (1.0 - g.uniform(0.0, 0.003, T))
        for a, n in ((120 + 40 * s, 30 + 6 * s), (420, 45)):   # halts: flat bars, no volume
            c[a : a + n] = c[a]
            o[a : a + n] = h[a : a + n] = l[a : a + n] = c[a]
            v[a : a + n] = 0.0
        if s % 2 == 0:   # a zero close (and bar) -> inf pct changes after it
            z = 300 + 10 * s
            o[z] = h[z] = l[z] = c[z] = 0.0
        P["open"][s], P["high"][s], P["low"][s], P["close"][s], P["volume"][s] = o, h, l, c, v
        P["qv"][s] = v * c
    out = {k: v for k, v in P.items()}
    open_time = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)
    bc = 60000.0 * np.exp(np.cumsum(g.normal(0.0, 0.004, T)))
    out["btc_close"] = bc
    dfb = pd.DataFrame({"open_time": open_time, "close": bc})
    ctx_ns = SimpleNamespace(config=SimpleNamespace(env="test"), symbol="TESTUSDT", kucoin_symbol="TEST-USDT",
                             exchange=None, binbot_api=None, telegram_consumer=None, market_type=None,
                             at_consumer=None, _breadth_cross_tolerance=0.05, _autotrade_stress_threshold=0.35,
                             current_symbol_data=None, price_precision=8, qty_precision=8)
    abp = ActivityBurstPump(ctx_ns)
    lsp = object.__new__(LiquidationSweepPump)
    rec: dict[str, list] = {}
    for s in range(S):
        o, h, l, c, v, qv = (P[k][s] for k in ("open", "high", "low", "close", "volume", "qv"))
        df = pd.DataFrame({"open": o, "high": h, "low": l, "close": c, "volume": v, "quote_asset_volume": qv})
        for col, ser in abp.compute_indicators(df.copy()).items():
            if col not in df.columns:
                rec.setdefault(f"abp__{col}", [None] * S)[s] = np.asarray(ser, dtype=float)
        dfl = pd.DataFrame({"open_time": open_time, "open": o, "high": h, "low": l, "close": c, "volume": v})
        for col, ser in lsp.compute_pump_score(dfl, dfb).items():
            if col not in dfl.columns:
                rec.setdefault(f"lsp__{col}", [None] * S)[s] = np.asarray(ser, dtype=float)
        ns = SimpleNamespace(symbol="TESTUSDT", market_type=None, df_15m=df.copy(), telegram_consumer=None,
                             at_consumer=None, current_symbol_data=None, price_precision=8,
                             market_breadth_data=None, strategy_cooldowns={}, strategy_states={})
        fsf = FailedSpikeFade(ns)
        for col, ser in fsf.detect().items():
            if col not in df.columns:
                rec.setdefault(f"fsf__{col}", [None] * S)[s] = np.asarray(ser, dtype=float)
    for k, rows in rec.items():
        out[k] = np.stack(rows)
    np.savez_compressed(out_dir / "inf_windows.npz", **out)


def leadership(out_dir: Path) -> None:
    """leadership.npz: GradualGainerRetest._leadership_allows (and the
    _relative_strengths it starts from; strategies/gradual_gainer_retest.py:131-196)
    on every prefix frame df.iloc[:t + 1] of
      ref_*   the frames of the reference's own test
              (tests/test_gradual_gainer_retest.py make_frames, imported from it);
      pan_*   20 symbols x 360 candles of 15-minute random walks against a BTC
              frame with missing candles, a duplicated timestamp (the dict keeps
              the last row) and a zero close; symbols with zero / negative
              closes, a late-listed symbol, steady gainers.
    Outputs: leader (bool), rs_2h, rs_6h per (symbol, t) as the method returns
    them (False, 0.0, 0.0 when strengths are None or history is short)."""
    import importlib.util

    import numpy as np
    import pandas as pd

    from strategies.gradual_gainer_retest import GradualGainerRetest

    spec = importlib.util.spec_from_file_location("ref_test_ggr", REFERENCE / "tests" / "test_gradual_gainer_retest.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}

    def run(name, times, closes, btc_t, btc_c):
        S, T = closes.shape
        lead = np.zeros((S, T), dtype=bool)
        r2 = np.zeros((S, T))
        r6 = np.zeros((S, T))
        btc_df = pd.DataFrame({"open_time": btc_t, "close": btc_c})
        for s in range(S):
            df = pd.DataFrame({"open_time": times[s], "close": closes[s]})
            for t in range(T):
                a, b, c = GradualGainerRetest._leadership_allows(df.iloc[: t + 1], btc_df)
                lead[s, t], r2[s, t], r6[s, t] = bool(a), float(b), float(c)
        out.update({f"{name}__open_time": times, f"{name}__close": closes, f"{name}__btc_time": btc_t,
                    f"{name}__btc_close": btc_c, f"{name}__leader": lead, f"{name}__rs_2h": r2,
                    f"{name}__rs_6h": r6})

    sym, btc = mod.make_frames()
    run("ref", sym["open_time"].to_numpy(np.int64)[None], sym["close"].to_numpy(float)[None],
        btc["open_time"].to_numpy(np.int64), btc["close"].to_numpy(float))

    rng = np.random.default_rng(20261017)
    S, T = 20, 360
    t0 = 1_800_000_000_000
    times = np.broadcast_to(t0 + 900_000 * np.arange(T, dtype=np.int64), (S, T)).copy()
    drift = np.where(np.arange(S) % 4 == 0, 0.004, 0.0)[:, None]
    closes = 50.0 * np.exp(np.cumsum(rng.normal(0.0, 0.006, (S, T)) + drift, axis=1))
    closes[3, 200] = 0.0
    closes[5, 150:153] = -1.0
    times[7] = t0 + 900_000 * (np.arange(T, dtype=np.int64) + 40)   # late listing: its frame starts 40 bars later
    keep = rng.random(T) > 0.03
    keep[:30] = True
    bt = t0 + 900_000 * np.arange(T + 40, dtype=np.int64)
    bc = 30_000.0 * np.exp(np.cumsum(rng.normal(0.0, 0.004, T + 40)))
    keep = np.concatenate([keep, np.ones(40, dtype=bool)])
    bt, bc = bt[keep], bc[keep]
    j = 120   # a duplicated timestamp: the later row wins in the reference's dict
    bt = np.insert(bt, j + 1, bt[j])
    bc = np.insert(bc, j + 1, bc[j] * 1.01)
    bc[250] = 0.0
    run("pan", times, closes, bt, bc)
    np.savez_compressed(out_dir / "leadership.npz", **out)


def scoring_and_selection(out_dir: Path) -> None:
    """context_scoring.json: RuleBasedMarketContextModel.evaluate
    (market_regime/context_scoring.py:13-114) + SignalContextScorer
    (market_regime/signal_context_scorer.py:15-55) and
    score_signal_candidate_with_context's emit gate on random contexts and
    candidates (LONG/SHORT, in/out of the snapshot, local_features overrides,
    no context, zero confidence).
    portfolio.json: LiquidationSweepPortfolioSelector
    (strategies/liquidation_sweep_pump.py:38-87) and
    GradualGainerPortfolioSelector (strategies/gradual_gainer_retest.py:33-70)
    driven with asyncio on random submission streams (late candidates, ties,
    re-submissions of a symbol); records submit() results and the dispatch order."""
    import asyncio

    import numpy as np

    from market_regime.models import LiveMarketContext, SymbolMarketFeatures
    from market_regime.score_signal_candidate_with_context import score_signal_candidate_with_context
    from market_regime.signal_context_scorer import SignalContextScorer
    from strategies.gradual_gainer_retest import GradualGainerCandidate, GradualGainerPortfolioSelector
    from strategies.liquidation_sweep_pump import LiquidationSweepCandidate, LiquidationSweepPortfolioSelector

    rng = np.random.default_rng(4242)
    syms = [f"C{i:02d}USDT" for i in range(30)]
    cases = []
    for k in range(40):
        feats = {}
        for s in syms[: int(rng.integers(0, 30))]:
            feats[s] = SymbolMarketFeatures(
                symbol=s, timestamp=1000, close=1.0, return_pct=float(rng.normal(0, 0.02)), ema20=1.0, ema50=1.0,
                above_ema20=bool(rng.random() < 0.5), above_ema50=bool(rng.random() < 0.5),
                trend_score=float(rng.normal(0, 0.03)), relative_strength_vs_btc=float(rng.normal(0, 0.03)),
                atr_pct=0.01, bb_width=0.05)
        ctx = None
        if k % 9 != 0:
            ctx = LiveMarketContext(
                timestamp=1000 + k, fresh_count=40, total_tracked_symbols=50, coverage_ratio=0.8, btc_symbol="BTCUSDT",
                btc_present=True, confidence=float(0.0 if k % 13 == 0 else rng.uniform(0.2, 1.0)),
                is_provisional=False, advancers=20, decliners=20, advancers_ratio=0.5, decliners_ratio=0.5,
                advancers_decliners_ratio=1.0, average_return=0.0, average_relative_strength_vs_btc=0.0,
                pct_above_ema20=0.5, pct_above_ema50=0.5, average_trend_score=0.0, average_atr_pct=0.01,
                average_bb_width=0.05, btc_return=0.0, btc_trend_score=0.0,
                btc_regime_score=float(rng.uniform(-1, 1)), market_stress_score=float(rng.uniform(0, 1)),
                long_tailwind=float(rng.uniform(-1, 1)), short_tailwind=float(rng.uniform(-1, 1)),
                symbol_features=feats)
        weights = dict(context_weight=float(rng.uniform(0, 1.5)), risk_weight=float(rng.uniform(0, 1)),
                       support_weight=float(rng.uniform(0, 1)))
        scorer = SignalContextScorer(**weights)
        cands = []
        for j in range(12):
            sym = syms[int(rng.integers(0, 30))]
            direction = ["LONG", "SHORT", " long ", "short"][int(rng.integers(0, 4))]
            local = {}   # SignalContextEvaluation rejects None (models.py)
            if rng.random() < 0.4:
                if rng.random() < 0.7:
                    local["relative_strength_vs_btc"] = float(rng.normal(0, 0.05))
                if rng.random() < 0.7:
                    local["trend_score"] = float(rng.normal(0, 0.05))
            score = float(rng.uniform(-1, 2))
            thr = None if rng.random() < 0.3 else float(rng.uniform(0, 1.5))
            ev = score_signal_candidate_with_context(sym, direction, score, ctx, scorer, local_features=local,
                                                     emit_threshold=thr)
            cs = ev.context_score
            cands.append(dict(symbol=sym, direction=direction, local_score=score, local_features=local,
                              emit_threshold=thr, adjusted_score=ev.adjusted_score, emit=ev.emit,
                              score={k2: getattr(cs, k2) for k2 in (
                                  "direction", "confidence", "breadth_score", "btc_alignment_score",
                                  "cross_asset_confirmation", "followthrough_score", "adverse_excursion_risk",
                                  "override_strength", "supportiveness_score")}))
        cases.append(dict(weights=weights, context=None if ctx is None else dict(
            confidence=ctx.confidence, long_tailwind=ctx.long_tailwind, short_tailwind=ctx.short_tailwind,
            btc_regime_score=ctx.btc_regime_score, market_stress_score=ctx.market_stress_score, timestamp=ctx.timestamp,
            symbol_features={s: dict(relative_strength_vs_btc=f.relative_strength_vs_btc, trend_score=f.trend_score)
                             for s, f in feats.items()}), candidates=cands))
    with open(out_dir / "context_scoring.json", "w") as f:
        json.dump(cases, f, separators=(",", ":"))

    async def drive(selector_cls, cand_cls, stream):
        sel = selector_cls()
        dispatched, accepted = [], []
        for i, (t, s, sc) in enumerate(stream):
            async def disp(i=i):
                dispatched.append(i)
            accepted.append(await sel.submit(cand_cls(candle_open_time=t, symbol=s, rank_score=sc, dispatch=disp)))
        await sel.flush()
        return accepted, dispatched

    runs = {}
    for name, sel_cls, cand_cls, step in (("liquidation", LiquidationSweepPortfolioSelector, LiquidationSweepCandidate,
                                           900_000),
                                          ("gradual", GradualGainerPortfolioSelector, GradualGainerCandidate, 900_000)):
        streams = []
        for k in range(6):
            n = int(rng.integers(20, 400))
            base = 1_760_000_000_000
            t = base + step * np.cumsum(rng.integers(0, 2, n) * (rng.random(n) < 0.3))
            late = rng.random(n) < 0.1
            t = np.where(late, t - step * rng.integers(1, 4, n), t)
            st = [(int(t[i]), syms[int(rng.integers(0, 12))],
                   float(np.round(rng.normal(0, 1), 1 if k % 2 else 6))) for i in range(n)]
            acc, disp = asyncio.run(drive(sel_cls, cand_cls, st))
            streams.append(dict(stream=st, accepted=acc, dispatched=disp))
        runs[name] = streams
    with open(out_dir / "portfolio.json", "w") as f:
        json.dump(runs, f, separators=(",", ":"))


def store_sequence(out_dir: Path, context_dict) -> None:
    """store_sequence.json: a scripted feed (REST history syncs with shuffled,
    duplicated, NaN and string rows; live ticks with skipped symbols, late
    corrections and out-of-order candles) replayed through the reference's
    MarketStateStore.update (market_regime/market_state_store.py:19-31) and
    LiveMarketContextAccumulator.on_closed_candle / refresh_context_for_timestamp
    (live_market_context_accumulator.py:38-84). Records every context, the
    final histories, last-closed timestamps and fresh sets."""
    import numpy as np

    from market_regime.live_market_context_accumulator import LiveMarketContextAccumulator
    from market_regime.market_state_store import MarketStateStore

    rng = np.random.default_rng(777)
    M = 30
    step = 900_000
    t0 = 1_760_000_400_000
    syms = ["BTCUSDT"] + [f"A{i:02d}USDT" for i in range(1, 50)]
    scale = {s: float(10 ** rng.uniform(-2, 3)) for s in syms}
    price = {s: scale[s] for s in syms}

    def candle(s, k, jitter=0.0):
        p = price[s] * float(np.exp(rng.normal(0.0004, 0.006)))
        price[s] = p
        o = p * float(np.exp(rng.normal(0, 0.002)))
        return dict(timestamp=t0 + k * step, open=o, high=max(o, p) * (1 + float(rng.uniform(0, 0.003))),
                    low=min(o, p) * (1 - float(rng.uniform(0, 0.003))), close=p * (1 + jitter),
                    volume=float(rng.lognormal(3, 1)))

    store = MarketStateStore(max_bars_per_symbol=M)
    acc = LiveMarketContextAccumulator(store, btc_symbol="BTCUSDT")
    ops, contexts = [], []
    # phase 1: REST history sync, one frame per symbol
    for s in syms:
        rows = [candle(s, k) for k in range(45)]
        for k in rng.choice(45, 3, replace=False):      # later copies of a timestamp win
            r = dict(rows[k])
            r["close"] = r["close"] * 1.01
            rows.append(r)
        for k in rng.choice(len(rows), 2, replace=False):   # rows without a close are dropped
            rows[k] = dict(rows[k], close=None)
        order = rng.permutation(len(rows))
        rows = [rows[i] for i in order]
        for r in rows[:5]:                               # wire-style strings
            r.update({f: (str(v) if v is not None else v) for f, v in r.items() if f != "timestamp"})
        if s == "A07USDT":                               # open/high/low/volume omitted
            rows = [dict(timestamp=r["timestamp"], close=r["close"]) for r in rows]
        ops.append(dict(op="update", symbol=s, rows=rows))
        store.update(s, pd_frame(rows))
    # phase 2: live ticks
    for k in range(45, 53):
        ts = t0 + k * step
        active = [s for s in syms if rng.random() > 0.12 or s == "BTCUSDT"]
        for i in rng.permutation(len(active)):
            s = active[i]
            c = candle(s, k)
            ops.append(dict(op="on_closed_candle", symbol=s, rows=[c]))
            ctx = context_dict(acc.on_closed_candle(s, c))
            if ctx is not None:   # per-symbol rows are kept for the refresh contexts only
                ctx.pop("symbol_features")
            contexts.append(ctx)
        if k == 48:   # late corrections of the current candle
            for s in active[:5]:
                c = dict(candle(s, k), close=price[s] * 0.97)
                ops.append(dict(op="update", symbol=s, rows=[c]))
                store.update(s, c)
        if k == 50:   # out-of-order older candles (replace inside the ring)
            for s in active[5:8]:
                c = candle(s, k - 5)
                ops.append(dict(op="update", symbol=s, rows=[c]))
                store.update(s, c)
        ops.append(dict(op="refresh", ts=ts))
        contexts.append(context_dict(acc.refresh_context_for_timestamp(ts)))
    final = {
        "histories": {s: store.get_symbol_history(s).to_dict(orient="list") for s in syms},
        "last_closed": {s: store.get_last_closed_timestamp(s) for s in syms},
        "fresh": {str(t0 + k * step): sorted(store.get_fresh_symbols(t0 + k * step)) for k in range(40, 53)},
        "tracked": store.get_tracked_symbols(),
        "latest_context_ts": (acc.get_latest_context().timestamp if acc.get_latest_context() else None),
    }
    with open(out_dir / "store_sequence.json", "w") as f:
        json.dump(dict(max_bars=M, btc="BTCUSDT", ops=ops, contexts=contexts, final=final), f,
                  separators=(",", ":"), default=float)


def store_gaps(out_dir: Path) -> None:
    """store_gaps.json: MarketStateStore + LiveMarketContextAccumulator under a
    feed whose candles miss high / low (kept by the store: only a missing
    close is dropped) — the features' true range is a skip-NaN max and its
    rolling(14, min_periods=1) mean skips missing values
    (live_market_context_accumulator.py:256-268)."""
    import numpy as np

    from market_regime.live_market_context_accumulator import LiveMarketContextAccumulator
    from market_regime.market_state_store import MarketStateStore

    def context_dict(ctx):
        if ctx is None:
            return None
        d = ctx.model_dump()
        d["symbol_features"] = {k: v for k, v in sorted(d["symbol_features"].items())}
        d["metadata"] = {k: v for k, v in d["metadata"].items() if k != "fresh_symbols"}
        return d

    rng = np.random.default_rng(4242)
    M = 40
    step = 900_000
    t0 = 1_760_100_000_000
    syms = ["BTCUSDT"] + [f"G{i:02d}USDT" for i in range(1, 50)]
    price = {s: float(10 ** rng.uniform(-2, 3)) for s in syms}
    missing = [None, "n/a", float("nan"), ""]

    def candle(s, k):
        p = price[s] * float(np.exp(rng.normal(0.0003, 0.007)))
        price[s] = p
        o = p * float(np.exp(rng.normal(0, 0.002)))
        c = dict(timestamp=t0 + k * step, open=o, high=max(o, p) * (1 + float(rng.uniform(0, 0.003))),
                 low=min(o, p) * (1 - float(rng.uniform(0, 0.003))), close=p, volume=float(rng.lognormal(3, 1)))
        r = rng.random()
        if r < 0.12:
            c["high"] = missing[int(rng.integers(0, 4))]
        elif r < 0.24:
            c["low"] = missing[int(rng.integers(0, 4))]
        elif r < 0.30:
            c["high"] = c["low"] = missing[int(rng.integers(0, 4))]
        return c

    store = MarketStateStore(max_bars_per_symbol=M)
    acc = LiveMarketContextAccumulator(store, btc_symbol="BTCUSDT")
    ops, contexts = [], []
    for s in syms:
        rows = [candle(s, k) for k in range(50)]
        if s == "G05USDT":   # a stretch where every candle misses both
            for r in rows[20:36]:
                r["high"] = r["low"] = None
        ops.append(dict(op="update", symbol=s, rows=rows))
        store.update(s, pd_frame(rows))
    for k in range(50, 58):
        ts = t0 + k * step
        for i in rng.permutation(len(syms)):
            s = syms[i]
            c = candle(s, k)
            ops.append(dict(op="on_closed_candle", symbol=s, rows=[c]))
            ctx = context_dict(acc.on_closed_candle(s, c))
            if ctx is not None:   # per-symbol rows are kept for the refresh contexts only
                ctx.pop("symbol_features")
            contexts.append(ctx)
        ops.append(dict(op="refresh", ts=ts))
        contexts.append(context_dict(acc.refresh_context_for_timestamp(ts)))
    final = {
        "histories": {s: store.get_symbol_history(s).to_dict(orient="list") for s in syms},
        "last_closed": {s: store.get_last_closed_timestamp(s) for s in syms},
        "fresh": {str(t0 + k * step): sorted(store.get_fresh_symbols(t0 + k * step)) for k in range(45, 58)},
        "tracked": store.get_tracked_symbols(),
        "latest_context_ts": (acc.get_latest_context().timestamp if acc.get_latest_context() else None),
    }
    with open(out_dir / "store_gaps.json", "w") as f:
        json.dump(dict(max_bars=M, btc="BTCUSDT", ops=ops, contexts=contexts, final=final), f,
                  separators=(",", ":"), default=float)
    print("store_gaps.json", len(ops), "ops,", sum(c is not None for c in contexts), "contexts")


def btc_change(out_dir: Path) -> None:
    """a12: the BTC 24h change exactly as ContextEvaluator.process_data forms
    it (producers/context_evaluator.py:427-430) —
    df_btc_15m["close"].pct_change(periods=96) * 100, read at [-1:] — on BTC
    closes with missing values (pandas 2.3.3's default fill_method='pad'
    forward-fills them first): NaN at the last row, at t - 96, runs across
    both, leading NaNs reaching past t - 96, short frames, a zero close.
    Writes btc_change.npz: <case>__close, <case>__pct (the whole series) and
    <case>__last (the value process_data keeps)."""
    import warnings

    import numpy as np
    import pandas as pd

    rng = np.random.default_rng(20261018)

    def walk(n):
        return 30000.0 * np.exp(np.cumsum(rng.normal(0, 0.004, n)))

    cases = {}
    c = walk(400)
    cases["clean"] = c.copy()
    x = c.copy(); x[-1] = np.nan
    cases["nan_last"] = x
    x = c.copy(); x[-97] = np.nan
    cases["nan_t96"] = x
    x = c.copy(); x[-100:-95] = np.nan; x[-3:] = np.nan
    cases["nan_runs_both"] = x
    x = c.copy(); x[:310] = np.nan
    cases["leading_past_t96"] = x
    x = c.copy(); x[:303] = np.nan
    cases["leading_to_t96"] = x
    x = c.copy(); x[rng.choice(400, 60, replace=False)] = np.nan
    cases["scattered"] = x
    x = c[:97].copy(); x[0] = np.nan
    cases["short97_nan_first"] = x
    cases["short97"] = c[:97].copy()
    cases["short96"] = c[:96].copy()
    x = c.copy(); x[-97] = 0.0
    cases["zero_t96"] = x
    x = c.copy(); x[-98] = np.nan; x[-97] = np.nan; x[-150] = np.nan
    cases["nan_t96_t97"] = x
    out = {}
    for name, close in cases.items():
        df_btc_15m = pd.DataFrame({"close": close})
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", FutureWarning)   # pandas 2.3.3's pad-fill deprecation notice
            df_pct_change = df_btc_15m["close"].pct_change(periods=96) * 100
        last = df_pct_change[-1:].iloc[0] if not df_pct_change.empty else 0.0
        out[f"{name}__close"] = close
        out[f"{name}__pct"] = df_pct_change.to_numpy()
        out[f"{name}__last"] = np.float64(last)
    np.savez_compressed(out_dir / "btc_change.npz", **out)
    print("btc_change.npz", len(cases), "cases, pandas", pd.__version__)


def headline_twins(out_dir: Path) -> None:
    """Per-candle values of the reference's in-repo twins of the headline
    enrich columns (pybinbot itself is absent), each real function called on
    every prefix df.iloc[:k] (they read the last row). See the module
    docstring; tests/test_twins_gpu.py runs bq_enrich with the matching
    IndicatorParams against them."""
    import numpy as np
    import pandas as pd

    from market_regime.live_market_context_accumulator import LiveMarketContextAccumulator
    from strategies.coinrule.bb_extreme_reversion import BBExtremeReversion
    from strategies.mean_reversion_fade import MeanReversionFade

    class TrendScore921(MeanReversionFade):   # price_tracker.py:204-205's spans through the real method
        EMA_FAST_WINDOW = 9
        EMA_SLOW_WINDOW = 21

    rng = np.random.default_rng(20261019)

    def walk(n, scale, vol):
        c = scale * np.exp(np.cumsum(rng.normal(0, vol, n)))
        o = np.r_[c[0], c[:-1]]
        h = np.maximum(o, c) * (1 + rng.uniform(0, 0.003, n))
        l = np.minimum(o, c) * (1 - rng.uniform(0, 0.003, n))
        return o, h, l, c, rng.lognormal(3, 1, n)

    frames = {}
    frames["walk"] = walk(1100, 100.0, 0.004)
    frames["tiny"] = walk(400, 1e-3, 0.01)
    o, h, l, c, v = walk(600, 25.0, 0.006)
    for a, b in ((100, 140), (300, 330), (500, 505)):   # constant runs: flat candles
        c[a:b] = c[a - 1]
        o[a:b] = h[a:b] = l[a:b] = c[a - 1]
    frames["runs"] = (o, h, l, c, v)
    o, h, l, c, v = walk(600, 3.0, 0.005)
    for a, b in ((50, 51), (200, 203), (450, 451), (451, 452)):   # missing candles (close, high, low)
        c[a:b] = h[a:b] = l[a:b] = np.nan
    frames["gaps"] = (o, h, l, c, v)
    feat_cols = ["ema20", "ema50", "atr_pct", "bb_width", "trend_score", "return_pct"]
    out = {}
    for name, (o, h, l, c, v) in frames.items():
        n = len(c)
        df = pd.DataFrame({"timestamp": 1_700_000_000_000 + 300_000 * np.arange(n), "open": o, "high": h,
                           "low": l, "close": c, "volume": v})
        for col in ("open", "high", "low", "close", "volume"):
            out[f"{name}__{col}"] = df[col].to_numpy(dtype=float)
        feats = np.full((n, len(feat_cols)), np.nan)
        for k in range(2, n + 1):
            f = LiveMarketContextAccumulator._compute_symbol_features("SYMUSDT", df.iloc[:k])
            if f is not None:
                feats[k - 1] = [float(getattr(f, col)) for col in feat_cols]
        out[f"{name}__features"] = feats
        for w in (14, 6):
            r = np.full(n, np.nan)
            for k in range(1, n + 1):
                val = BBExtremeReversion._compute_rsi(df["close"].iloc[:k], w)
                if val is not None:
                    r[k - 1] = val
            out[f"{name}__sma_rsi{w}"] = r
        out[f"{name}__trend_9_21"] = np.array([TrendScore921._trend_score(df["close"].iloc[:k])
                                               for k in range(1, n + 1)])
        out[f"{name}__trend_20_50"] = np.array([MeanReversionFade._trend_score(df["close"].iloc[:k])
                                                for k in range(1, n + 1)])
    out["names"] = np.array(list(frames))
    out["feature_columns"] = np.array(feat_cols)
    np.savez_compressed(out_dir / "headline_twins.npz", **out)
    print("headline_twins.npz", list(frames), "pandas", pd.__version__)


def pd_frame(rows):
    import pandas as pd

    return pd.DataFrame(rows)


def main() -> None:
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(Path(sys.argv[2]), set(sys.argv[3].split(",")) if len(sys.argv) > 3 and sys.argv[3] else None)
        return
    only = ""
    if len(sys.argv) > 2 and sys.argv[1] == "--only":
        only = sys.argv[2]
    if not REFERENCE.exists():
        sys.exit("make_golden.py runs only where /root/reference is mounted")
    with tempfile.TemporaryDirectory(prefix="bq_shim_") as tmp:
        shim = Path(tmp)
        write_shim(shim)
        env = dict(os.environ)
        env["PYTHONPATH"] = f"{shim}:{REFERENCE}"
        env["PYTHONDONTWRITEBYTECODE"] = "1"
        env["ENV"] = "ci"
        env["PYTHONHASHSEED"] = "0"   # the accumulator iterates symbol sets: fixed order, stable last bits
        subprocess.run([sys.executable, __file__, "--child", str(HERE), only], check=True, env=env, cwd=tmp)


if __name__ == "__main__":
    main()
