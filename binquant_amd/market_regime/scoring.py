"""Regime annotation and candidate scoring on the device.

* ``micro_regime`` — RegimeTransitionDetector._annotate_symbol_regime
  (market_regime/regime_transitions.py:162-232) for a whole fresh-symbol set
  in one launch (bq_micro_regime), bit-exact with the Python floats.
* ``score_candidates`` — the strategies' shared seam
  score_signal_candidate_with_context (market_regime/score_signal_candidate_with_context.py)
  = RuleBasedMarketContextModel.evaluate (context_scoring.py:13-114) +
  SignalContextScorer.adjust_score (signal_context_scorer.py:15-28) + the
  emit gate, for a batch of candidates against one context (bq_context_score).
  The symbol lookup of LiveMarketContext.get_symbol_features (models.py:157-168,
  exact then canonical match) and the local_features overrides
  (context_scoring.py:116-124) are resolved on the host into two columns.
"""

from __future__ import annotations

import ctypes
from collections.abc import Mapping, Sequence

import numpy as np
import torch

from .. import _lib, engine
from .._lib import MICRO_REGIMES, MICRO_TRANSITIONS, SCORE_FIELDS

_REG_CODE = {r: i for i, r in enumerate(MICRO_REGIMES)}


def _f64(x, dev) -> torch.Tensor:
    return torch.as_tensor(np.asarray(x, dtype=np.float64) if not isinstance(x, torch.Tensor) else x,
                           dtype=torch.float64).to(dev).contiguous()


def _u8(x, dev) -> torch.Tensor:
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x, dtype=bool))
    return t.to(device=dev, dtype=torch.uint8).contiguous()


def regime_codes(labels) -> np.ndarray:
    """Micro-regime labels (None allowed) -> int8 codes (-1 = None)."""
    return np.array([-1 if r is None else _REG_CODE[r] for r in labels], dtype=np.int8)


def micro_regime(trend, above_ema20, above_ema50, rs, bb_width, atr_pct, return_pct, prev_regime=None,
                 prev_strength=None, device=None, stream=None) -> dict[str, torch.Tensor]:
    """Per-symbol micro regime on the device. Inputs: [n] arrays (host or
    device); prev_regime: int8 codes (-1 None) or labels. Returns int8 code
    tensors 'micro_regime' / 'micro_regime_transition' (-1 None) and float64
    'micro_regime_strength' / 'micro_regime_transition_strength'."""
    dev = torch.device(device) if device is not None else (
        trend.device if isinstance(trend, torch.Tensor) else torch.device("cuda"))
    t = _f64(trend, dev)
    n = t.numel()
    ins = [t, _u8(above_ema20, dev), _u8(above_ema50, dev), _f64(rs, dev), _f64(bb_width, dev), _f64(atr_pct, dev),
           _f64(return_pct, dev)]
    pr = ps = None
    if prev_regime is not None:
        codes = prev_regime if isinstance(prev_regime, torch.Tensor) else (
            regime_codes(prev_regime) if np.asarray(prev_regime).dtype == object else np.asarray(prev_regime, np.int8))
        pr = torch.as_tensor(codes, dtype=torch.int8).to(dev).contiguous()
        ps = _f64(np.zeros(n) if prev_strength is None else prev_strength, dev)
    reg = torch.empty(n, dtype=torch.int8, device=dev)
    st = torch.empty(n, dtype=torch.float64, device=dev)
    tr = torch.empty(n, dtype=torch.int8, device=dev)
    tst = torch.empty(n, dtype=torch.float64, device=dev)
    ptr = lambda x: ctypes.c_void_p(x.data_ptr() if x is not None else 0)  # noqa: E731
    status = _lib.load().bq_micro_regime(n, *(ptr(x) for x in ins), ptr(pr), ptr(ps), ptr(reg), ptr(st), ptr(tr),
                                         ptr(tst), engine._stream_handle(stream))
    _lib.check(status, "bq_micro_regime")
    return {"micro_regime": reg, "micro_regime_strength": st, "micro_regime_transition": tr,
            "micro_regime_transition_strength": tst}


def labels(codes, table=MICRO_REGIMES) -> np.ndarray:
    c = codes.cpu().numpy() if isinstance(codes, torch.Tensor) else np.asarray(codes)
    out = np.full(c.shape, None, dtype=object)
    ok = c >= 0
    out[ok] = np.asarray(table, dtype=object)[c[ok]]
    return out


def _canonical(sym: str) -> str:   # models.py:51-52
    return sym.upper().strip().replace("-", "").replace("_", "")


def _get(ctx, name, default=None):
    if ctx is None:
        return default
    return ctx.get(name, default) if isinstance(ctx, Mapping) else getattr(ctx, name, default)


def _symbol_rows(ctx, symbols: Sequence[str]):
    """(rs, trend, found) from the context's symbol_features with the exact
    then canonical lookup of LiveMarketContext.get_symbol_features."""
    sf = _get(ctx, "symbol_features") or {}
    rs = np.zeros(len(symbols))
    tr = np.zeros(len(symbols))
    found = np.zeros(len(symbols), dtype=bool)
    canon = None
    for i, s in enumerate(symbols):
        key = s.strip().upper()
        row = sf.get(key) if hasattr(sf, "get") else None
        if row is None:
            if canon is None:
                canon = {}
                for k in sf:
                    canon.setdefault(_canonical(k), k)
            k = canon.get(_canonical(key))
            row = sf[k] if k is not None else None
        if row is not None:
            rs[i] = float(_get(row, "relative_strength_vs_btc", 0.0))
            tr[i] = float(_get(row, "trend_score", 0.0))
            found[i] = True
    return rs, tr, found


def score_candidates(symbols: Sequence[str], directions: Sequence[str], local_scores, context,
                     context_weight: float = 1.0, risk_weight: float = 0.5, support_weight: float = 0.35,
                     local_features: Sequence[Mapping[str, float] | None] | None = None,
                     emit_threshold=None, device=None, stream=None) -> dict[str, np.ndarray]:
    """Batched score_signal_candidate_with_context: MarketContextScore fields,
    'adjusted_score' and 'emit' per candidate (numpy arrays)."""
    n = len(symbols)
    dev = torch.device(device) if device is not None else torch.device("cuda")
    norm = [d.upper().strip() for d in directions]
    dcode = np.array([0 if d == "LONG" else 1 if d == "SHORT" else 2 for d in norm], dtype=np.int8)
    rs, tr, found = _symbol_rows(context, symbols)
    if local_features is not None:
        for i, lf in enumerate(local_features):
            if lf:
                if "relative_strength_vs_btc" in lf:
                    rs[i] = float(lf["relative_strength_vs_btc"])
                if "trend_score" in lf:
                    tr[i] = float(lf["trend_score"])
    c = _lib.BqContextScalars()
    if context is not None:
        c.present = 1
        for f in ("confidence", "long_tailwind", "short_tailwind", "btc_regime_score", "market_stress_score"):
            setattr(c, f, float(_get(context, f)))
    w = _lib.BqScorerWeights(float(context_weight), float(risk_weight), float(support_weight))
    dd = torch.from_numpy(dcode).to(dev)
    rs_d, tr_d, ls_d = _f64(rs, dev), _f64(tr, dev), _f64(local_scores, dev)
    out = torch.empty((len(SCORE_FIELDS), max(n, 1)), dtype=torch.float64, device=dev)
    status = _lib.load().bq_context_score(
        n, ctypes.c_void_p(dd.data_ptr()), ctypes.c_void_p(rs_d.data_ptr()), ctypes.c_void_p(tr_d.data_ptr()),
        ctypes.c_void_p(ls_d.data_ptr()), ctypes.byref(c), ctypes.byref(w), ctypes.c_void_p(out.data_ptr()),
        max(n, 1), engine._stream_handle(stream))
    _lib.check(status, "bq_context_score")
    o = out[:, :n].cpu().numpy()
    res = dict(zip(SCORE_FIELDS, o))
    res["direction"] = np.array(norm, dtype=object)
    res["symbol_in_snapshot"] = found & (context is not None)
    res["symbol_relative_strength_vs_btc"] = rs
    res["symbol_trend_score"] = tr
    thr = emit_threshold
    if thr is None:
        res["emit"] = np.ones(n, dtype=bool)
    else:
        t = np.array([np.nan if x is None else x for x in (thr if np.ndim(thr) else [thr] * n)], dtype=np.float64)
        res["emit"] = np.isnan(t) | (res["adjusted_score"] >= t)
    return res
