"""Batched device entry points over the C ABI (torch tensors in, torch tensors out).

All tensors are float64 CUDA (HIP) tensors shaped [S, T] with unit stride
along T (any row stride). Launches go on torch's current stream, so results
are ordered with surrounding torch work and can be timed with torch events.
There is no CPU path: non-CUDA input raises.
"""

from __future__ import annotations

import contextlib
import ctypes
import functools
from dataclasses import dataclass, field

import torch

from . import _lib
from ._lib import ENRICH_COLUMNS, FEATURE_COLUMNS, INPUT_FIELDS, PARTIAL_COLUMNS


@dataclass
class IndicatorParams:
    """Python mirror of ``bq_params``; defaults are the reference's windows
    (producers/context_evaluator.py:249-261)."""

    ma_periods: tuple[int, int, int] = (7, 25, 100)
    macd_fast: int = 12
    macd_slow: int = 26
    macd_signal: int = 9
    rsi_window: int = 14
    bb_window: int = 20
    bb_ddof: int = 1
    bb_k: float = 2.0
    atr_window: int = 14
    twap_window: int = 12
    ema_spans: tuple[int, int] = (20, 50)
    mfi_window: int = 14
    extra: dict = field(default_factory=dict)

    def to_c(self) -> _lib.BqParams:
        p = _lib.BqParams()
        for i, v in enumerate(self.ma_periods):
            p.ma_periods[i] = int(v)
        p.macd_fast = int(self.macd_fast)
        p.macd_slow = int(self.macd_slow)
        p.macd_signal = int(self.macd_signal)
        p.rsi_window = int(self.rsi_window)
        p.bb_window = int(self.bb_window)
        p.bb_ddof = int(self.bb_ddof)
        p.atr_window = int(self.atr_window)
        p.twap_window = int(self.twap_window)
        p.ema_spans[0] = int(self.ema_spans[0])
        p.ema_spans[1] = int(self.ema_spans[1])
        p.mfi_window = int(self.mfi_window)
        p.bb_k = float(self.bb_k)
        return p

    def as_oracle_dict(self) -> dict:
        return dict(
            ma_periods=tuple(self.ma_periods),
            macd_fast=self.macd_fast,
            macd_slow=self.macd_slow,
            macd_signal=self.macd_signal,
            rsi_window=self.rsi_window,
            bb_window=self.bb_window,
            bb_ddof=self.bb_ddof,
            bb_k=self.bb_k,
            atr_window=self.atr_window,
            twap_window=self.twap_window,
            ema_spans=tuple(self.ema_spans),
            mfi_window=self.mfi_window,
        )


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream_handle(stream: torch.cuda.Stream | None) -> ctypes.c_void_p:
    """hipStream_t of `stream`, else of torch's current stream on the current
    device (read without building a Stream object: this runs once per launch)."""
    if stream is not None:
        return ctypes.c_void_p(stream.cuda_stream)
    if _raw_stream is not None and _cur_device is not None:
        return ctypes.c_void_p(_raw_stream(_cur_device()))
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _cuda_tensors(obj, out: list) -> list:
    """CUDA tensors among a call's arguments (tensors, and tensors inside
    lists / tuples / dict values one level down)."""
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            out.append(obj)
    elif isinstance(obj, (list, tuple)):
        # sequences of operands are homogeneous: a list whose first entry is
        # not a tensor (e.g. 10k symbol names of a store tick) is not walked
        if obj and isinstance(obj[0], torch.Tensor):
            for x in obj:
                if isinstance(x, torch.Tensor) and x.is_cuda:
                    out.append(x)
    elif isinstance(obj, dict):
        for x in obj.values():
            if isinstance(x, torch.Tensor) and x.is_cuda:
                out.append(x)
    elif isinstance(getattr(obj, "x", None), torch.Tensor) and obj.x.is_cuda:   # Roll / Ewm / Ffill specs
        out.append(obj.x)
    return out


@contextlib.contextmanager
def launch_scope(device: torch.device | None, stream: torch.cuda.Stream | None, tensors=()):
    """Where and when a native launch runs.

    * device — made current for the call: the C ABI launches on the current
      device's stream, and the fused JIT resolves its module per current device.
    * stream — when given, it first waits on the device's current stream (the
      producers of the operands), the call runs under torch.cuda.stream(stream)
      so outputs and temporaries are allocated and produced on it, and every
      CUDA operand is recorded on it so the caching allocator does not hand
      the memory out again before the stream has read it. Later use of the
      outputs on another stream is the caller's to order, as with any torch
      side stream.
    """
    if device is not None and device.type != "cuda":   # host tensors (CPU rehearsal of the collectives)
        yield
        return
    if stream is None:
        if device is None or device.index is None or device.index == (
                _cur_device() if _cur_device else torch.cuda.current_device()):
            yield
            return
        with torch.cuda.device(device):
            yield
        return
    if device is not None:
        # torch.device("cuda") (index None) means the current device
        want = device.index if device.index is not None else torch.cuda.current_device()
        have = stream.device.index if stream.device.index is not None else torch.cuda.current_device()
        if want != have:
            raise ValueError(f"stream is on {stream.device}, operands on {device}")
    with torch.cuda.device(stream.device):
        stream.wait_stream(torch.cuda.current_stream(stream.device))
        for t in tensors:
            t.record_stream(stream)
        with torch.cuda.stream(stream):
            yield


def device_entry(fn):
    """Decorator of the public entry points: runs `fn` on the device holding
    its CUDA operands (all must share one device) and, for `stream=`, under
    launch_scope's stream ordering. The wrapped body always launches on the
    current stream."""

    @functools.wraps(fn)
    def wrapper(*args, stream: torch.cuda.Stream | None = None, **kw):
        ts: list = []
        for a in args:
            _cuda_tensors(a, ts)
        for a in kw.values():
            _cuda_tensors(a, ts)
        dev = ts[0].device if ts else None
        if dev is not None:
            for t in ts:
                if t.device != dev:
                    raise ValueError(f"{fn.__name__}: operands on {dev} and {t.device}; one device per call")
        if stream is None and (dev is None or dev.index == (_cur_device() if _cur_device else -1)):
            return fn(*args, **kw)
        with launch_scope(dev, stream, ts):
            return fn(*args, **kw)

    return wrapper


def _check_panel(x: torch.Tensor, name: str, shape=None) -> torch.Tensor:
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise ValueError(f"{name}: expected a float64 CUDA tensor (no CPU path)")
    if x.dtype != torch.float64:
        raise ValueError(f"{name}: expected dtype float64, got {x.dtype}")
    if x.dim() == 1:
        x = x.unsqueeze(0)
    if x.dim() != 2 or (x.shape[1] > 1 and x.stride(1) != 1):
        raise ValueError(f"{name}: expected [S, T] with unit stride along T")
    if shape is not None and tuple(x.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(x.shape)} != {tuple(shape)}")
    return x


def _row_stride(x: torch.Tensor) -> int:
    return int(x.stride(0)) if x.shape[0] > 1 else int(x.shape[1])


ENRICH_ROW_PAD = 192   # doubles added to each output row's pitch by enrich_outputs (tools/shard_pitch.py)


def enrich_outputs(S: int, T: int, device, columns=ENRICH_COLUMNS) -> dict[str, torch.Tensor]:
    """Output columns for enrich(..., out=...) laid out for HBM: [S, T] views
    into [S, T + ENRICH_ROW_PAD] buffers when the panel is large. With a row
    pitch of exactly T doubles (80 000 B at T = 10 000) the concurrently
    resident workgroups' output streams meet the same HBM channels: the C4
    shard (12 500 x 10 000) ran at 0.666 of 8 TB/s, at 0.711 with a 512-B pad
    (round 5). Round 6 swept the pad on two boxes (profiles/r6d_pitch.txt,
    r6e_pitch.txt): +512 B 0.709 / 0.626, +768 B 0.719 / 0.692, +1 536 B
    0.713 / 0.702 at the shard, the 100k headline indifferent — 192 doubles.
    Small panels get plain [S, T] tensors. enrich() allocates its own outputs
    this way too."""
    pad = ENRICH_ROW_PAD if S >= 1024 and T >= 1024 else 0
    return {k: torch.empty((S, T + pad), dtype=torch.float64, device=device)[:, :T] for k in columns}


@device_entry
def enrich(
    open_: torch.Tensor,
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    volume: torch.Tensor,
    params: IndicatorParams | None = None,
    columns=ENRICH_COLUMNS,
    out: dict[str, torch.Tensor] | None = None,
    stream: torch.cuda.Stream | None = None,
) -> dict[str, torch.Tensor]:
    """Full (or partial) indicator set over a [S, T] panel in ONE kernel launch.

    Replaces ContextEvaluator.indicators_enrichment
    (producers/context_evaluator.py:240-263) applied symbol by symbol.
    Returns {column_name: [S, T] float64 tensor}.
    """
    close = _check_panel(close, "close")
    S, T = close.shape
    ins = [
        _check_panel(t, n, (S, T))
        for t, n in zip((open_, high, low, close, volume), INPUT_FIELDS)
    ]
    ld_in = _row_stride(ins[0])
    if any(_row_stride(t) != ld_in for t in ins):
        ins = [t.contiguous() for t in ins]
        ld_in = T
    cols = tuple(columns)
    unknown = set(cols) - set(ENRICH_COLUMNS)
    if unknown:
        raise ValueError(f"unknown enrich columns: {sorted(unknown)}")
    out = dict(out or {})
    given = [n for n in cols if n in out]
    for name in given:
        _check_panel(out[name], f"out[{name}]", (S, T))
    missing = [n for n in cols if n not in out]
    if missing:
        # the columns this call allocates share the caller's pitch when some
        # are given, else enrich_outputs' rule (a padded pitch on large panels:
        # the layout the bench times is the one every product caller gets)
        if given:
            ld = _row_stride(out[given[0]])
            out.update({n: torch.empty((S, max(ld, T)), dtype=torch.float64, device=close.device)[:, :T]
                        for n in missing})
        else:
            out.update(enrich_outputs(S, T, close.device, missing))
    ld_out = T
    if out:
        strides = {_row_stride(out[n]) for n in cols}
        if len(strides) != 1:
            raise ValueError("all output columns must share one row stride")
        ld_out = strides.pop()
    in_arr = _lib.ptr_array([t.data_ptr() for t in ins])
    out_arr = _lib.ptr_array([out[n].data_ptr() if n in cols else 0 for n in ENRICH_COLUMNS])
    p = (params or IndicatorParams()).to_c()
    st = _lib.load().bq_enrich(
        in_arr, S, T, ld_in, ctypes.byref(p), out_arr, ld_out, _stream_handle(stream)
    )
    _lib.check(st, "bq_enrich")
    return {n: out[n] for n in cols}


@device_entry
def market_features(
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    max_bars: int = 400,
    out: dict[str, torch.Tensor] | None = None,
    stream: torch.cuda.Stream | None = None,
) -> dict[str, torch.Tensor]:
    """_compute_symbol_features at every timestamp of a [S, T] panel
    (market_regime/live_market_context_accumulator.py:244-297) under the
    MarketStateStore history cap ``max_bars`` (klines_provider.py:40,65 uses 400)."""
    close = _check_panel(close, "close")
    S, T = close.shape
    hlc = [_check_panel(t, n, (S, T)) for t, n in zip((high, low, close), ("high", "low", "close"))]
    ld_in = _row_stride(hlc[0])
    if any(_row_stride(t) != ld_in for t in hlc):
        hlc = [t.contiguous() for t in hlc]
        ld_in = T
    out = dict(out or {})
    for name in FEATURE_COLUMNS:
        if name not in out:
            out[name] = torch.empty((S, T), dtype=torch.float64, device=close.device)
        else:
            _check_panel(out[name], f"out[{name}]", (S, T))
    ld_out = _row_stride(out[FEATURE_COLUMNS[0]])
    if any(_row_stride(out[n]) != ld_out for n in FEATURE_COLUMNS):
        raise ValueError("all feature output columns must share one row stride")
    st = _lib.load().bq_market_features(
        _lib.ptr_array([t.data_ptr() for t in hlc]),
        S,
        T,
        ld_in,
        int(max_bars),
        _lib.ptr_array([out[n].data_ptr() for n in FEATURE_COLUMNS]),
        ld_out,
        _stream_handle(stream),
    )
    _lib.check(st, "bq_market_features")
    return out


PUMP_COLUMNS = ("candidate_atr", "momentum_3", "relative_volume", "pre_breakout_compression", "pump_score",
                "prior_high", "close_location", "ema20", "ema50", "trend_score", "momentum_atr", "btc_momentum_3",
                "btc_trend_score", "relative_strength")


@device_entry
def pump_features(
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    volume: torch.Tensor,
    candidate_atr: torch.Tensor,
    ema20: torch.Tensor,
    ema50: torch.Tensor,
    bench_ffill: torch.Tensor,
    bench_ema20: torch.Tensor,
    bench_ema50: torch.Tensor,
    momentum_bars: int = 3,
    volume_lookback: int = 20,
    compression_bars: int = 6,
    stream: torch.cuda.Stream | None = None,
    trend_score: torch.Tensor | None = None,
) -> dict[str, torch.Tensor]:
    """LiquidationSweepPump.compute_pump_score's columns but the two rolling
    quantiles and score_cross (strategies/liquidation_sweep_pump.py:195-268) in
    one pass per row (bq_pump_features): the volume mean, the high / low
    windows and the pad-filled pct_change formed in the kernel. The ewm columns
    (candidate_atr, ema20, ema50) and the benchmark rows ([T]: ffilled close,
    ewm 20, ewm 50) are inputs; the returned ewm columns ARE those input
    tensors (the kernel does not write a copy: 24 B per candle less).
    trend_score: the column already formed with the ewm columns (bq_pump_ewm);
    then the kernel reads neither ema column back and returns it as given."""
    close = _check_panel(close, "close")
    S, T = close.shape
    ins = [_check_panel(t, n, (S, T)).contiguous() for t, n in
           zip((high, low, close, volume, candidate_atr, ema20, ema50),
               ("high", "low", "close", "volume", "candidate_atr", "ema20", "ema50"))]
    if trend_score is not None:
        trend_score = _check_panel(trend_score, "trend_score", (S, T))
    bench = []
    for t, n in zip((bench_ffill, bench_ema20, bench_ema50), ("bench_ffill", "bench_ema20", "bench_ema50")):
        if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float64 or t.numel() != T:
            raise ValueError(f"{n}: expected a float64 CUDA tensor of {T} values")
        bench.append(t.reshape(T).contiguous())
    given = {"candidate_atr": ins[4], "ema20": ins[5], "ema50": ins[6]}
    if trend_score is not None:
        given["trend_score"] = trend_score
    out = {n: given[n] if n in given else torch.empty((S, T), dtype=torch.float64, device=close.device)
           for n in PUMP_COLUMNS}
    iptr = [t.data_ptr() for t in ins]
    if trend_score is not None:
        iptr[5] = iptr[6] = 0   # not read
    st = _lib.load().bq_pump_features(
        _lib.ptr_array(iptr), S, T, T, _lib.ptr_array([t.data_ptr() for t in bench]),
        int(momentum_bars), int(volume_lookback), int(compression_bars),
        _lib.ptr_array([0 if n in given else out[n].data_ptr() for n in PUMP_COLUMNS]), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_pump_features")
    return out


@device_entry
def pump_features_ewm(
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    volume: torch.Tensor,
    bench_ffill: torch.Tensor,
    bench_ema20: torch.Tensor,
    bench_ema50: torch.Tensor,
    momentum_bars: int = 3,
    volume_lookback: int = 20,
    compression_bars: int = 6,
    stream: torch.cuda.Stream | None = None,
) -> dict[str, torch.Tensor]:
    """pump_features with candidate_atr / ema20 / ema50 formed inside the pass
    (bq_pump_features_ewm: the three ewm scans on the row's tiles, no ewm
    column read back; liquidation_sweep_pump.py:206-217, 252-253)."""
    close = _check_panel(close, "close")
    S, T = close.shape
    ins = [_check_panel(t, n, (S, T)).contiguous() for t, n in
           zip((high, low, close, volume), ("high", "low", "close", "volume"))]
    bench = []
    for t, n in zip((bench_ffill, bench_ema20, bench_ema50), ("bench_ffill", "bench_ema20", "bench_ema50")):
        if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float64 or t.numel() != T:
            raise ValueError(f"{n}: expected a float64 CUDA tensor of {T} values")
        bench.append(t.reshape(T).contiguous())
    out = {n: torch.empty((S, T), dtype=torch.float64, device=close.device) for n in PUMP_COLUMNS}
    st = _lib.load().bq_pump_features_ewm(
        _lib.ptr_array([t.data_ptr() for t in ins]), S, T, T, _lib.ptr_array([t.data_ptr() for t in bench]),
        int(momentum_bars), int(volume_lookback), int(compression_bars),
        _lib.ptr_array([out[n].data_ptr() for n in PUMP_COLUMNS]), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_pump_features_ewm")
    return out


@device_entry
def pump_ewm(high: torch.Tensor, low: torch.Tensor, close: torch.Tensor,
             stream: torch.cuda.Stream | None = None, trend: bool = False) -> tuple[torch.Tensor, ...]:
    """LiquidationSweepPump's candidate_atr (TR.ewm(alpha=1/14, min_periods=14))
    and ema20 / ema50 of close in panel mode, one pass per row (bq_pump_ewm:
    the true range formed in the kernel; liquidation_sweep_pump.py:206-217,
    252-253); trend=True adds trend_score = (ema20 - ema50) / ema50 (:254)."""
    close = _check_panel(close, "close").contiguous()
    S, T = close.shape
    high = _check_panel(high, "high", (S, T)).contiguous()
    low = _check_panel(low, "low", (S, T)).contiguous()
    outs = [torch.empty((S, T), dtype=torch.float64, device=close.device) for _ in range(4 if trend else 3)]
    st = _lib.load().bq_pump_ewm(_ptr(high), _ptr(low), _ptr(close), S, T, T, *(_ptr(o) for o in outs[:3]),
                                 _ptr(outs[3] if trend else None), T, _stream_handle(stream))
    _lib.check(st, "bq_pump_ewm")
    return tuple(outs)


BURST_FLOAT_COLUMNS = ("baseline_volume_safe", "volume_ratio", "baseline_quote_volume_safe", "quote_volume_ratio",
                       "price_jump", "range_frac", "body_frac", "close_to_high", "recent_up_closes",
                       "activity_burst_score")
BURST_BOOL_COLUMNS = ("is_bullish", "vol_spike", "quote_vol_spike", "price_jump_flag", "range_expansion_flag",
                      "body_quality_flag", "trend_quality_flag")


@device_entry
def burst_features(
    o: torch.Tensor, h: torch.Tensor, l: torch.Tensor, c: torch.Tensor, v: torch.Tensor,
    qv: torch.Tensor | None, baseline_volume: torch.Tensor, baseline_quote_volume: torch.Tensor | None,
    params, stream: torch.cuda.Stream | None = None,
) -> tuple[dict[str, torch.Tensor], torch.Tensor]:
    """ActivityBurstPump.compute_indicators' columns of
    strategies/activity_burst_pump.py:58-133 in one pass (bq_burst_features),
    given the two baseline medians; returns (columns, the AND of the six flags
    as uint8 for burst_qualify). Without a quote volume the quote baseline and
    its safe column alias the volume's (the reference's fallback)."""
    c = _check_panel(c, "c")
    S, T = c.shape
    has_q = qv is not None
    names = ("o", "h", "l", "c", "v", "qv", "baseline_volume", "baseline_quote_volume")
    ins = []
    for t, n in zip((o, h, l, c, v, qv, baseline_volume, baseline_quote_volume), names):
        ins.append(None if t is None else _check_panel(t, n, (S, T)).contiguous())
    if has_q != (baseline_quote_volume is not None):
        raise ValueError("qv and baseline_quote_volume: give both or neither")
    out = {n: torch.empty((S, T), dtype=torch.float64, device=c.device) for n in BURST_FLOAT_COLUMNS
           if has_q or n != "baseline_quote_volume_safe"}
    flags = {n: torch.empty((S, T), dtype=torch.bool, device=c.device) for n in BURST_BOOL_COLUMNS}
    all_flags = torch.empty((S, T), dtype=torch.uint8, device=c.device)
    pr = _lib.BqBurstParams(float(params.volume_multiplier), float(params.quote_volume_multiplier),
                            float(params.price_threshold), float(params.min_baseline_volume),
                            float(params.min_range_frac), float(params.min_body_frac), float(params.max_close_to_high),
                            int(params.min_recent_up_closes if has_q else 1), 0)
    st = _lib.load().bq_burst_features(
        _lib.ptr_array([0 if t is None else t.data_ptr() for t in ins]), S, T, T, ctypes.byref(pr),
        _lib.ptr_array([out[n].data_ptr() if n in out else 0 for n in BURST_FLOAT_COLUMNS]),
        _lib.ptr_array([flags[n].data_ptr() for n in BURST_BOOL_COLUMNS]), ctypes.c_void_p(all_flags.data_ptr()), T,
        _stream_handle(stream),
    )
    _lib.check(st, "bq_burst_features")
    if not has_q:
        out["baseline_quote_volume_safe"] = out["baseline_volume_safe"]
    out.update(flags)
    return out, all_flags


@device_entry
def burst_qualify(score: torch.Tensor, threshold: torch.Tensor, all_flags: torch.Tensor, cooldown_bars: int = 3,
                  stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """qualified_signal (strategies/activity_burst_pump.py:140-156): raw = the
    six flags & (score >= threshold.fillna(0)), cleared where raw fired in the
    cooldown_bars candles before (bq_burst_qualify). bool [S, T]."""
    score = _check_panel(score, "score")
    S, T = score.shape
    threshold = _check_panel(threshold, "threshold", (S, T)).contiguous()
    score = score.contiguous()
    if not isinstance(all_flags, torch.Tensor) or all_flags.dtype != torch.uint8 or tuple(all_flags.shape) != (S, T):
        raise ValueError("all_flags: expected the uint8 [S, T] tensor of burst_features")
    all_flags = all_flags.contiguous()
    q = torch.empty((S, T), dtype=torch.bool, device=score.device)
    st = _lib.load().bq_burst_qualify(
        ctypes.c_void_p(score.data_ptr()), ctypes.c_void_p(threshold.data_ptr()), ctypes.c_void_p(all_flags.data_ptr()),
        S, T, T, T, int(cooldown_bars), ctypes.c_void_p(q.data_ptr()), _stream_handle(stream),
    )
    _lib.check(st, "bq_burst_qualify")
    return q


SPIKE_BASE_FLOAT = ("price_change", "price_change_abs", "body_size", "body_size_pct", "upper_wick", "lower_wick",
                    "upper_wick_ratio", "lower_wick_ratio", "total_range", "range_pct", "close_open_ratio", "price_ma",
                    "price_zscore", "volume_ma", "volume_ratio", "volume_zscore", "quote_volume_ma",
                    "quote_volume_ratio", "momentum_3", "momentum_5", "close_to_high", "close_to_low",
                    "std_ratio_8_20", "pc_2c", "pc_3c", "pc_pos_count_5", "pc_abs_sum_5", "body_size_pct_ma_10",
                    "body_size_pct_z")
SPIKE_BASE_BOOL = ("is_bullish", "vol_compression_flag", "upward", "downward")
SPIKE_FLAG_FLOAT = ("vol_ratio_slope_3", "vol_ratio_accel", "price_break_threshold_series", "early_spike_proba")
SPIKE_FLAG_BOOL = ("volume_cluster_flag", "price_break_flag", "cumulative_price_break_flag",
                   "cumulative_price_break_short_flag", "accel_spike_flag", "accel_spike_short_flag", "label_pre",
                   "label_short_pre", "early_proba_aug_flag")


def _cols(S, T, dev, names, dtype, given=None):
    given = given or {}
    return {n: given[n] if n in given else torch.empty((S, T), dtype=dtype, device=dev) for n in names}


@device_entry
def spike_base(o, h, l, c, v, qv, close_ffill, price_std, volume_std, std8, std20, body_pct_std, base_window: int = 12,
               streak_length: int = 3, body_size_pct: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> dict[str, torch.Tensor]:
    """FailedSpikeFade's base and early-feature columns
    (strategies/failed_spike_fade.py:260-357) in one pass per row
    (bq_spike_base), given the ffilled close and the rolling std columns;
    body_size_pct: an existing column with the kernel's values (not rewritten)."""
    c = _check_panel(c, "c")
    S, T = c.shape
    ins = [_check_panel(t, n, (S, T)).contiguous() for t, n in zip(
        (o, h, l, c, v, qv, close_ffill, price_std, volume_std, std8, std20, body_pct_std),
        ("o", "h", "l", "c", "v", "qv", "close_ffill", "price_std", "volume_std", "std8", "std20", "body_pct_std"))]
    out = _cols(S, T, c.device, SPIKE_BASE_FLOAT, torch.float64,
                {"body_size_pct": body_size_pct} if body_size_pct is not None else None)
    flags = _cols(S, T, c.device, SPIKE_BASE_BOOL, torch.bool)
    st = _lib.load().bq_spike_base(
        _lib.ptr_array([t.data_ptr() for t in ins]), S, T, T, int(base_window), int(streak_length),
        _lib.ptr_array([0 if (n == "body_size_pct" and body_size_pct is not None) else out[n].data_ptr()
                        for n in SPIKE_BASE_FLOAT]),
        _lib.ptr_array([flags[n].data_ptr() for n in SPIKE_BASE_BOOL]), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_spike_base")
    out.update(flags)
    return out


# bq_spike_base_std's std columns (enum bq_spike_std_col), under their
# FailedSpikeFade.detect names
SPIKE_STD = ("price_std", "volume_std", "rolling_price_std_8", "rolling_price_std_20", "body_size_pct_std_10")


@device_entry
def spike_base_std(o, h, l, c, v, qv, close_ffill, base_window: int = 12, streak_length: int = 3,
                   body_size_pct: torch.Tensor | None = None,
                   stream: torch.cuda.Stream | None = None) -> dict[str, torch.Tensor]:
    """spike_base in panel mode (bq_spike_base_std): the five rolling std
    columns (failed_spike_fade.py:293-339) formed in the same pass as two-pass
    window sums — the window's variance to rounding, where pandas' online
    recurrence (and its bit-exact replay, spike_base's inputs) drifts — and
    returned beside the base columns under their detect() names."""
    c = _check_panel(c, "c")
    S, T = c.shape
    ins = [_check_panel(t, n, (S, T)).contiguous() for t, n in zip(
        (o, h, l, c, v, qv, close_ffill), ("o", "h", "l", "c", "v", "qv", "close_ffill"))]
    out = _cols(S, T, c.device, SPIKE_BASE_FLOAT, torch.float64,
                {"body_size_pct": body_size_pct} if body_size_pct is not None else None)
    flags = _cols(S, T, c.device, SPIKE_BASE_BOOL, torch.bool)
    sd = _cols(S, T, c.device, SPIKE_STD, torch.float64)
    st = _lib.load().bq_spike_base_std(
        _lib.ptr_array([t.data_ptr() for t in ins]), S, T, T, int(base_window), int(streak_length),
        _lib.ptr_array([0 if (n == "body_size_pct" and body_size_pct is not None) else out[n].data_ptr()
                        for n in SPIKE_BASE_FLOAT]),
        _lib.ptr_array([flags[n].data_ptr() for n in SPIKE_BASE_BOOL]),
        _lib.ptr_array([sd[n].data_ptr() for n in SPIKE_STD]), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_spike_base_std")
    out.update(flags)
    out.update(sd)
    return out


_SPIKE_MODES = {"last": 0, "first": 1, "all": 2}


@device_entry
def spike_flags(o, c, close_ffill, volume_ratio, dyn_threshold, vcmr, pbbt, params,
                stream: torch.cuda.Stream | None = None, labels: torch.Tensor | None = None) -> dict[str, torch.Tensor]:
    """FailedSpikeFade's flag columns and preliminary labels
    (strategies/failed_spike_fade.py:360-488) in one pass per row
    (bq_spike_flags): vcmr / pbbt [S] the calibrated thresholds, dyn_threshold
    the |pct change| rolling quantile. labels: an optional bool [2, S, T]
    that receives label_pre / label_short_pre (so one cooldown launch can
    take both as [2S, T] rows)."""
    c = _check_panel(c, "c")
    S, T = c.shape
    ins = [_check_panel(t, n, (S, T)).contiguous() for t, n in zip(
        (o, c, close_ffill, volume_ratio, dyn_threshold), ("o", "c", "close_ffill", "volume_ratio", "dyn_threshold"))]
    vc = vcmr.reshape(S).contiguous().to(torch.float64)
    pb = pbbt.reshape(S).contiguous().to(torch.float64)
    pr = _lib.BqSpikeParams(int(params.volume_cluster_window), int(params.volume_cluster_min_count),
                            int(params.cumulative_price_window), int(params.accel_volume_deriv_window),
                            _SPIKE_MODES[params.volume_cluster_label_mode], int(bool(params.require_both_patterns)),
                            int(bool(params.require_bullish_spike)), 0, float(params.cumulative_price_threshold),
                            float(params.accel_volume_deriv_min), float(params.accel_price_change_min),
                            float(params.body_size_pct_min))
    out = _cols(S, T, c.device, SPIKE_FLAG_FLOAT, torch.float64)
    given = None
    if labels is not None:
        if labels.shape != (2, S, T) or labels.dtype != torch.bool or not labels.is_contiguous() \
                or labels.device != c.device:
            raise ValueError("labels: expected a contiguous bool [2, S, T] tensor on the panel's device")
        given = {"label_pre": labels[0], "label_short_pre": labels[1]}
    flags = _cols(S, T, c.device, SPIKE_FLAG_BOOL, torch.bool, given)
    st = _lib.load().bq_spike_flags(
        _lib.ptr_array([t.data_ptr() for t in ins]), ctypes.c_void_p(vc.data_ptr()), ctypes.c_void_p(pb.data_ptr()),
        S, T, T, ctypes.byref(pr), _lib.ptr_array([out[n].data_ptr() for n in SPIKE_FLAG_FLOAT]),
        _lib.ptr_array([flags[n].data_ptr() for n in SPIKE_FLAG_BOOL]), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_spike_flags")
    out.update(flags)
    return out


@device_entry
def breadth_partial(
    close: torch.Tensor,
    feats: dict[str, torch.Tensor],
    out: torch.Tensor | None = None,
    stream: torch.cuda.Stream | None = None,
) -> torch.Tensor:
    """[T, 10] per-timestamp partial counts/sums over this shard's symbols
    (the reductions of _build_context, live_market_context_accumulator.py:135-163)."""
    close = _check_panel(close, "close")
    S, T = close.shape
    fs = [_check_panel(feats[n], n, (S, T)) for n in FEATURE_COLUMNS]
    ld_f = _row_stride(fs[0])
    if any(_row_stride(t) != ld_f for t in fs):
        raise ValueError("feature columns must share one row stride")
    if out is None:
        out = torch.empty((T, len(PARTIAL_COLUMNS)), dtype=torch.float64, device=close.device)
    elif not (isinstance(out, torch.Tensor) and out.dtype == torch.float64 and out.device == close.device
              and tuple(out.shape) == (T, len(PARTIAL_COLUMNS)) and out.is_contiguous()):
        raise ValueError(f"out: expected a contiguous float64 [{T}, {len(PARTIAL_COLUMNS)}] tensor on {close.device}")
    st = _lib.load().bq_breadth_partial(
        ctypes.c_void_p(close.data_ptr()),
        _lib.ptr_array([t.data_ptr() for t in fs]),
        S,
        T,
        _row_stride(close),
        ld_f,
        ctypes.c_void_p(out.data_ptr()),
        _stream_handle(stream),
    )
    _lib.check(st, "bq_breadth_partial")
    return out


@device_entry
def context_partials(
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    max_bars: int = 400,
    out: torch.Tensor | None = None,
    last: bool = False,
    stream: torch.cuda.Stream | None = None,
):
    """The [T, 10] breadth partials of every timestamp straight from the
    panel (bq_context_partials): market_features + breadth_partial fused, the
    feature columns never written (live_market_context_accumulator.py:95-163
    over _compute_symbol_features :244-297). Counts equal breadth_partial's,
    sums agree to rounding. last=True also returns the features at t = T - 1
    ({name: [S]}, what a context's symbol_features reads); returns
    (partial, last_features | None)."""
    close = _check_panel(close, "close")
    S, T = close.shape
    hlc = [_check_panel(t, n, (S, T)) for t, n in zip((high, low, close), ("high", "low", "close"))]
    ld_in = _row_stride(hlc[0])
    if any(_row_stride(t) != ld_in for t in hlc):
        hlc = [t.contiguous() for t in hlc]
        ld_in = T
    dev = close.device
    if out is None:
        out = torch.empty((T, len(PARTIAL_COLUMNS)), dtype=torch.float64, device=dev)
    elif not (isinstance(out, torch.Tensor) and out.dtype == torch.float64 and out.device == dev
              and tuple(out.shape) == (T, len(PARTIAL_COLUMNS)) and out.is_contiguous()):
        raise ValueError(f"out: expected a contiguous float64 [{T}, {len(PARTIAL_COLUMNS)}] tensor on {dev}")
    lib = _lib.load()
    nbytes = int(lib.bq_context_workspace_bytes(S, T))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)   # caching allocator: 512-B aligned
    lastf = {n: torch.empty(S, dtype=torch.float64, device=dev) for n in FEATURE_COLUMNS} if last else None
    st = lib.bq_context_partials(
        _lib.ptr_array([t.data_ptr() for t in hlc]), S, T, ld_in, int(max_bars),
        ctypes.c_void_p(ws.data_ptr()), nbytes, ctypes.c_void_p(out.data_ptr()),
        _lib.ptr_array([lastf[n].data_ptr() for n in FEATURE_COLUMNS]) if last else None,
        _stream_handle(stream))
    _lib.check(st, "bq_context_partials")
    return out, lastf


class TickState:
    """Device-resident streaming state for S symbols (bq_state).

    ``frame`` is the per-message frame the reference re-enriches on every
    closed kline: KlinesProvider.LIMIT = 400 candles
    (consumers/klines_provider.py:40,201-215 -> producers/context_evaluator.py:
    367-371). Each tick returns the last row of indicators_enrichment over the
    symbol's last ``frame`` candles, the EMA family seeded at the frame's first
    candle exactly as the reference's re-enrichment is. ``frame=0`` keeps
    unbounded-history EMA carries (the full-series pandas EMA) instead."""

    FRAME = 400

    def __init__(self, n_symbols: int, params: IndicatorParams | None = None, frame: int = FRAME):
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        p = (params or IndicatorParams()).to_c()
        # device memory of the state lives on the current device (bq_state_create)
        self.device = torch.device("cuda", torch.cuda.current_device())
        frame = int(frame)
        if frame != 0 and not (_lib.MAX_WINDOW + 2 <= frame <= 1 << 20):
            raise ValueError(f"frame must be 0 or in [{_lib.MAX_WINDOW + 2}, {1 << 20}], got {frame}")
        _lib.check(self._lib.bq_state_create_frame(ctypes.byref(self._h), int(n_symbols), ctypes.byref(p), frame),
                   "bq_state_create_frame")
        self.n_symbols = int(n_symbols)
        self.frame = frame

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.bq_state_destroy(h)
            self._h = None

    @property
    def count(self) -> int:
        return int(self._lib.bq_state_count(self._h))

    @device_entry
    def seed(self, open_, high, low, close, volume, stream=None) -> None:
        close = _check_panel(close, "close")
        S, T = close.shape
        if S != self.n_symbols:
            raise ValueError(f"seed panel has {S} symbols, state has {self.n_symbols}")
        if close.device != self.device:
            raise ValueError(f"seed panel on {close.device}, state on {self.device}")
        ins = [_check_panel(t, n, (S, T)).contiguous() for t, n in zip((open_, high, low, close, volume), INPUT_FIELDS)]
        st = self._lib.bq_state_seed(
            self._h, _lib.ptr_array([t.data_ptr() for t in ins]), T, T, _stream_handle(stream)
        )
        _lib.check(st, "bq_state_seed")

    @device_entry
    def tick(self, new_ohlcv, out: dict[str, torch.Tensor] | None = None, columns=ENRICH_COLUMNS, stream=None):
        """new_ohlcv: sequence of 5 float64 CUDA vectors [S] (open, high, low, close, volume)."""
        vecs = []
        for t, n in zip(new_ohlcv, INPUT_FIELDS):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float64 and t.numel() == self.n_symbols):
                raise ValueError(f"{n}: expected float64 CUDA vector of length {self.n_symbols}")
            if t.device != self.device:
                raise ValueError(f"{n}: on {t.device}, state on {self.device}")
            vecs.append(t.contiguous())
        out = dict(out or {})
        cols = tuple(columns)
        dev = vecs[0].device
        for n in cols:
            if n not in out:
                out[n] = torch.empty(self.n_symbols, dtype=torch.float64, device=dev)
            else:
                o = out[n]
                if not (isinstance(o, torch.Tensor) and o.dtype == torch.float64 and o.device == dev
                        and o.numel() == self.n_symbols and o.is_contiguous()):
                    raise ValueError(f"out[{n}]: expected a contiguous float64 vector of {self.n_symbols} on {dev}")
        st = self._lib.bq_tick(
            self._h,
            _lib.ptr_array([t.data_ptr() for t in vecs]),
            _lib.ptr_array([out[n].data_ptr() if n in cols else 0 for n in ENRICH_COLUMNS]),
            _stream_handle(stream),
        )
        _lib.check(st, "bq_tick")
        return {n: out[n] for n in cols}


@device_entry
def beta_corr(
    close: torch.Tensor,
    btc_close: torch.Tensor,
    window: int = 50,
    stream: torch.cuda.Stream | None = None,
) -> dict[str, torch.Tensor]:
    """Rolling beta / correlation of log returns vs the benchmark at every t
    (ContextEvaluator.dynamic_btc_beta_corr, producers/context_evaluator.py:154-194).
    close: [S, T]; btc_close: [T] index-aligned with the panel."""
    close = _check_panel(close, "close")
    S, T = close.shape
    btc = _check_panel(btc_close.reshape(1, -1), "btc_close", (1, T)).contiguous()
    beta = torch.empty((S, T), dtype=torch.float64, device=close.device)
    corr = torch.empty_like(beta)
    # the benchmark's log returns (log(c / c.shift(1)), :166-169) and window
    # stats once per call, in the kernel's one-workgroup pre-pass (scratch)
    scratch = torch.empty(4 * T, dtype=torch.float64, device=close.device)
    st = _lib.load().bq_beta_corr_ws(
        ctypes.c_void_p(close.data_ptr()), ctypes.c_void_p(btc.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
        S, T, _row_stride(close),
        int(window), ctypes.c_void_p(beta.data_ptr()), ctypes.c_void_p(corr.data_ptr()), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_beta_corr_ws")
    return {"beta": beta, "corr": corr}


def _signal_launch(name: str, ins: list[torch.Tensor], window: int, stream) -> torch.Tensor:
    S, T = ins[-1].shape
    ld = _row_stride(ins[0])
    if any(_row_stride(t) != ld for t in ins):
        ins = [t.contiguous() for t in ins]
        ld = T
    out = torch.empty((S, T), dtype=torch.float64, device=ins[0].device)
    st = getattr(_lib.load(), name)(*[ctypes.c_void_p(t.data_ptr()) for t in ins], S, T, ld, int(window),
                                    ctypes.c_void_p(out.data_ptr()), T, _stream_handle(stream))
    _lib.check(st, name)
    return out


@device_entry
def wilder_rsi(close: torch.Tensor, window: int = 14, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """MeanReversionFade._rsi (strategies/mean_reversion_fade.py:88-109) at
    every t, time-parallel (bq_wilder_rsi; 1e-9 of pandas, finite closes)."""
    close = _check_panel(close, "close")
    return _signal_launch("bq_wilder_rsi", [close], window, stream)


@device_entry
def zscore(close: torch.Tensor, window: int = 20, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """RangeBbRsiMeanReversion._compute_zscore (strategies/range_bb_rsi_mean_reversion.py:132-138)
    at every t, time-parallel (bq_zscore)."""
    close = _check_panel(close, "close")
    return _signal_launch("bq_zscore", [close], window, stream)


@device_entry
def adx(high: torch.Tensor, low: torch.Tensor, close: torch.Tensor, window: int = 14,
        stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """RangeBbRsiMeanReversion._compute_adx (strategies/range_bb_rsi_mean_reversion.py:101-130)
    at every t, time-parallel (bq_adx, window <= 64)."""
    close = _check_panel(close, "close")
    S, T = close.shape
    return _signal_launch("bq_adx", [_check_panel(high, "high", (S, T)), _check_panel(low, "low", (S, T)), close],
                          window, stream)


@device_entry
def rolling(
    x: torch.Tensor,
    window: int,
    stat: str = "mean",
    q: float = 0.5,
    min_periods: int | None = None,
    shift: int = 0,
    out: torch.Tensor | None = None,
    stream: torch.cuda.Stream | None = None,
) -> torch.Tensor:
    """x.shift(shift).rolling(window, min_periods).<stat>() along T of a [S, T]
    panel; stat in {"quantile", "median", "mean", "sum", "var", "std", "max",
    "min", "isum"} (var / std: ddof 1; isum: the sum of an integer-valued
    series such as a flag count — pandas' value, computed without the
    sequential replay)."""
    x = _check_panel(x, "x")
    S, T = x.shape
    if stat == "max":
        stat, q = "quantile", 1.0
    elif stat == "min":
        stat, q = "quantile", 0.0
    if stat not in _lib.ROLL_MODES:
        raise ValueError(f"unknown rolling statistic {stat!r}")
    if out is None:
        out = torch.empty((S, T), dtype=torch.float64, device=x.device)
    st = _lib.load().bq_rolling(
        ctypes.c_void_p(x.data_ptr()), S, T, _row_stride(x), int(window),
        int(window if min_periods is None else min_periods), int(shift), _lib.ROLL_MODES[stat], float(q),
        ctypes.c_void_p(out.data_ptr()), _row_stride(out), _stream_handle(stream),
    )
    _lib.check(st, "bq_rolling")
    return out


@device_entry
def rolling_quantile_cross(
    x: torch.Tensor,
    window: int,
    q: float,
    min_periods: int | None = None,
    shift: int = 0,
    stream: torch.cuda.Stream | None = None,
) -> tuple[torch.Tensor, torch.Tensor]:
    """(thr, cross): thr = x.shift(shift).rolling(window, min_periods).quantile(q)
    and cross = (x >= thr) & (x.shift(1) < thr.shift(1)) (bool) in one pass
    where the sliding-window kernel runs (bq_rolling_quantile_cross) —
    LiquidationSweepPump's score_threshold / score_cross
    (strategies/liquidation_sweep_pump.py:231-239)."""
    x = _check_panel(x, "x")
    S, T = x.shape
    thr = torch.empty((S, T), dtype=torch.float64, device=x.device)
    cross = torch.empty((S, T), dtype=torch.bool, device=x.device)
    st = _lib.load().bq_rolling_quantile_cross(
        ctypes.c_void_p(x.data_ptr()), S, T, _row_stride(x), int(window),
        int(window if min_periods is None else min_periods), int(shift), float(q),
        ctypes.c_void_p(thr.data_ptr()), T, ctypes.c_void_p(cross.data_ptr()), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_rolling_quantile_cross")
    return thr, cross


@device_entry
def ewm(
    x: torch.Tensor,
    alpha: float | None = None,
    span: float | None = None,
    min_periods: int = 0,
    out: torch.Tensor | None = None,
    stream: torch.cuda.Stream | None = None,
) -> torch.Tensor:
    """x.ewm(alpha|span, adjust=False, min_periods).mean() along T (pandas'
    exact recursion, NaN gaps decay the old weight)."""
    x = _check_panel(x, "x")
    S, T = x.shape
    if (alpha is None) == (span is None):
        raise ValueError("give exactly one of alpha / span")
    # pandas: comass from span or alpha, alpha = 1 / (1 + comass)
    com = (float(span) - 1.0) / 2.0 if span is not None else 1.0 / float(alpha) - 1.0
    a = 1.0 / (1.0 + com)
    if out is None:
        out = torch.empty((S, T), dtype=torch.float64, device=x.device)
    st = _lib.load().bq_ewm(
        ctypes.c_void_p(x.data_ptr()), S, T, _row_stride(x), a, int(min_periods),
        ctypes.c_void_p(out.data_ptr()), _row_stride(out), _stream_handle(stream),
    )
    _lib.check(st, "bq_ewm")
    return out


@dataclass
class Roll:
    """One x.shift(shift).rolling(window, min_periods).<stat>() series of a
    rolling_many batch (stat as in rolling())."""

    x: torch.Tensor
    window: int
    stat: str = "mean"
    q: float = 0.5
    min_periods: int | None = None
    shift: int = 0


@dataclass
class Ewm:
    """One x.ewm(alpha|span, adjust=False, min_periods).mean() series of a batch."""

    x: torch.Tensor
    alpha: float | None = None
    span: float | None = None
    min_periods: int = 0


@dataclass
class Ffill:
    """x.ffill() along T (leading NaNs stay) as one series of a batch."""

    x: torch.Tensor


@device_entry
def rolling_many(*specs, exact: bool = True, stream: torch.cuda.Stream | None = None,
                 cross: tuple[int, ...] = ()):
    """Independent Roll / Ewm / Ffill series over one [S, T] shape in as few
    launches as the kernel families allow (bq_rolling_batch): the
    lane-per-symbol replays of different series run side by side instead of
    one launch each. A moment / ewm / ffill series may have fewer rows than
    the panel (e.g. the [1, T] benchmark beside an [S, T] panel): it joins
    the same launch (bq_roll_job.rows) instead of paying a replay walk of
    its own. exact=False: sums / means (window + shift <= 128) and ewm run
    time-parallel (bq_panel.hip, panel mode), within rounding of pandas
    (1e-9) instead of the bit-exact sequential replay; order statistics on
    the tile kernels sort packed keys (the union slot in the key's low bits:
    the selected value is an element within 2^-45 relative of the exact
    order statistic); var / std and the rest are unchanged.
    cross: indices of quantile specs that also get their crossing flags,
    (x >= thr) & (x.shift(1) < thr.shift(1)) as bool [S, T]
    (bq_rolling_batch_cross; liquidation_sweep_pump.py:237-239's score_cross
    form) — then the result is (outs, flags), flags in the order of cross."""
    if not specs:
        return ([], []) if cross else []
    xs = [_check_panel(sp.x, "x") for sp in specs]
    S = max(int(x.shape[0]) for x in xs)
    T = int(xs[0].shape[1])
    outs: list[torch.Tensor] = []
    jobs = []
    keep = []
    for sp, x in zip(specs, xs):
        rows = int(x.shape[0])
        if x.shape[1] != T:
            raise ValueError(f"x: shape {tuple(x.shape)}: every series of a batch needs T = {T}")
        if rows != S and isinstance(sp, Roll) and sp.stat not in ("mean", "sum", "var", "std", "var0", "std0"):
            raise ValueError(f"x: shape {tuple(x.shape)} != {(S, T)} (only moments, ewm and ffill may have fewer rows)")
        out = torch.empty((rows, T), dtype=torch.float64, device=x.device)
        j = _lib.BqRollJob()
        j.x, j.out, j.ld_in, j.ld_out = x.data_ptr(), out.data_ptr(), _row_stride(x), T
        j.rows = rows if rows != S else 0
        j.panel = 0 if exact else 1
        if isinstance(sp, Ffill):
            j.mode = _lib.ROLL_FFILL
        elif isinstance(sp, Ewm):
            if (sp.alpha is None) == (sp.span is None):
                raise ValueError("give exactly one of alpha / span")
            com = (float(sp.span) - 1.0) / 2.0 if sp.span is not None else 1.0 / float(sp.alpha) - 1.0
            j.alpha, j.mode, j.min_periods = 1.0 / (1.0 + com), _lib.ROLL_EWM, int(sp.min_periods)
        else:
            stat, q = sp.stat, sp.q
            if stat == "max":
                stat, q = "quantile", 1.0
            elif stat == "min":
                stat, q = "quantile", 0.0
            if stat not in _lib.ROLL_MODES:
                raise ValueError(f"unknown rolling statistic {stat!r}")
            j.window, j.shift, j.mode, j.q = int(sp.window), int(sp.shift), _lib.ROLL_MODES[stat], float(q)
            j.min_periods = int(sp.window if sp.min_periods is None else sp.min_periods)
        jobs.append(j)
        outs.append(out)
        keep.append(x)
    flags = {}
    for k in cross:
        if not (isinstance(specs[k], Roll) and specs[k].stat == "quantile" and xs[k].shape[0] == S):
            raise ValueError(f"cross: spec {k} is not a quantile over the whole panel")
        flags[k] = torch.empty((S, T), dtype=torch.bool, device=xs[k].device)
    fptr = {id(jobs[k]): flags[k].data_ptr() for k in flags}
    L = _lib.load()
    # a batch call takes MAX_ROLL_JOBS jobs: the sequential replays (moments,
    # ewm — one latency-bound launch per call, whatever its job count) go
    # into the calls first, so 14 replays + 4 order statistics make one replay
    # launch instead of a second one for the replays that spilled into the
    # next call (outputs stay in spec order: each job carries its own pointer)
    _REPLAY = (_lib.ROLL_EWM,) + tuple(_lib.ROLL_MODES[k] for k in ("mean", "sum", "var", "std", "var0", "std0"))
    jobs = sorted(jobs, key=lambda j: 0 if j.mode in _REPLAY else 1)
    for i in range(0, len(jobs), _lib.MAX_ROLL_JOBS):
        chunk = jobs[i : i + _lib.MAX_ROLL_JOBS]
        arr = (_lib.BqRollJob * len(chunk))(*chunk)
        if fptr:
            cp = _lib.ptr_array([fptr.get(id(j), 0) for j in chunk])
            cl = (ctypes.c_int64 * len(chunk))(*([T] * len(chunk)))
            _lib.check(L.bq_rolling_batch_cross(arr, len(chunk), S, T, cp, cl, _stream_handle(stream)),
                       "bq_rolling_batch_cross")
        else:
            _lib.check(L.bq_rolling_batch(arr, len(chunk), S, T, _stream_handle(stream)), "bq_rolling_batch")
    return (outs, [flags[k] for k in cross]) if cross else outs


@device_entry
def row_quantile(x: torch.Tensor, q: float, stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """numpy.quantile(row[~isnan(row)], q) per row (numpy 'linear' method), as
    FailedSpikeFade.auto_calibrate (strategies/failed_spike_fade.py:229-257)
    calls it. Returns [S] float64, NaN for rows without observations."""
    x = _check_panel(x, "x")
    S, T = x.shape
    out = torch.empty((S,), dtype=torch.float64, device=x.device)
    st = _lib.load().bq_row_quantile(
        ctypes.c_void_p(x.data_ptr()), S, T, _row_stride(x), float(q), ctypes.c_void_p(out.data_ptr()),
        _stream_handle(stream),
    )
    _lib.check(st, "bq_row_quantile")
    return out


@device_entry
def cooldown(label: torch.Tensor, bars: int, stream: torch.cuda.Stream | None = None):
    """FailedSpikeFade.apply_cooldown (strategies/failed_spike_fade.py:495-520):
    returns (kept, suppressed) bool [S, T] — a label within `bars` candles of
    the last kept label is cleared and flagged suppressed."""
    if not isinstance(label, torch.Tensor) or not label.is_cuda or label.dtype != torch.bool:
        raise ValueError("label: expected a bool CUDA tensor (no CPU path)")
    if label.dim() == 1:
        label = label.unsqueeze(0)
    label = label.contiguous()
    S, T = label.shape
    kept = torch.empty_like(label)
    sup = torch.empty_like(label)
    st = _lib.load().bq_cooldown(
        ctypes.c_void_p(label.data_ptr()), S, T, T, int(bars), ctypes.c_void_p(kept.data_ptr()),
        ctypes.c_void_p(sup.data_ptr()), T, _stream_handle(stream),
    )
    _lib.check(st, "bq_cooldown")
    return kept, sup


@device_entry
def supertrend(
    high: torch.Tensor,
    low: torch.Tensor,
    close: torch.Tensor,
    period: int = 10,
    multiplier: float = 3.0,
    atr: torch.Tensor | None = None,
    stream: torch.cuda.Stream | None = None,
    exact: bool = True,
) -> dict[str, torch.Tensor]:
    """pybinbot Indicators.set_supertrend (strategies/coinrule/coinrule.py:143-160)
    on a [S, T] panel: {"supertrend": bool (uptrend), "supertrend_upper",
    "supertrend_lower": final bands}. ATR = TR.rolling(period).mean() unless
    given: the default exact=True forms it in the same walk as pandas'
    roll_mean (bq_supertrend_hlc, bit for bit — the live path,
    Indicators.set_supertrend); exact=False is the panel mode
    (bq_supertrend_panel: chunks of each row walked in parallel with verified
    chunk starts, the same recursion) on an ATR equal to pandas' to rounding,
    so bands agree to rounding and flags up to near-ties."""
    high = _check_panel(high, "high")
    S, T = high.shape
    low = _check_panel(low, "low", (S, T))
    close = _check_panel(close, "close", (S, T))
    up = torch.empty((S, T), dtype=torch.bool, device=close.device)
    upper = torch.empty((S, T), dtype=torch.float64, device=close.device)
    lower = torch.empty_like(upper)
    if atr is None:
        ins = [t.contiguous() for t in (high, low, close)]
        L = _lib.load()
        args = [_lib.ptr_array([t.data_ptr() for t in ins]), S, T, T, int(period), float(multiplier),
                ctypes.c_void_p(up.data_ptr()), ctypes.c_void_p(upper.data_ptr()), ctypes.c_void_p(lower.data_ptr()),
                T]
        if exact:
            fn = "bq_supertrend_hlc"
            st = L.bq_supertrend_hlc(*args, _stream_handle(stream))
        else:
            fn = "bq_supertrend_panel"
            st = L.bq_supertrend_panel(*args, _stream_handle(stream))
        _lib.check(st, fn)
    else:
        atr = _check_panel(atr, "atr", (S, T))
        ins = [t.contiguous() for t in (high, low, close, atr)]
        st = _lib.load().bq_supertrend(
            _lib.ptr_array([t.data_ptr() for t in ins]), S, T, T, float(multiplier), ctypes.c_void_p(up.data_ptr()),
            ctypes.c_void_p(upper.data_ptr()), ctypes.c_void_p(lower.data_ptr()), T, _stream_handle(stream),
        )
        _lib.check(st, "bq_supertrend")
    return {"supertrend": up, "supertrend_upper": upper, "supertrend_lower": lower}


# ---- frame plumbing: resample / timestamp joins (bq_frame.hip) -----------------


def _check_ts(ts: torch.Tensor, name: str = "ts") -> torch.Tensor:
    if not isinstance(ts, torch.Tensor) or not ts.is_cuda or ts.dtype != torch.int64:
        raise ValueError(f"{name}: expected an int64 CUDA tensor of ms timestamps (no CPU path)")
    if ts.dim() == 1:
        ts = ts.unsqueeze(0)
    return ts.contiguous()


def _check_lens(lens, S: int, device) -> torch.Tensor | None:
    if lens is None:
        return None
    if not isinstance(lens, torch.Tensor):
        lens = torch.as_tensor(lens, dtype=torch.int64)
    lens = lens.to(device=device, dtype=torch.int64).contiguous()
    if lens.numel() != S:
        raise ValueError(f"lens: expected {S} entries, got {lens.numel()}")
    return lens


def _ptr(t: torch.Tensor | None) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


@device_entry
def resample(
    ts: torch.Tensor,
    fields: dict[str, torch.Tensor],
    aggs: dict[str, str],
    interval_ms: int,
    lens=None,
    max_bins: int | None = None,
    tail: bool = False,
    stream: torch.cuda.Stream | None = None,
) -> tuple[torch.Tensor, dict[str, torch.Tensor], torch.Tensor]:
    """Candles.resample (producers/context_evaluator.py:403-407) on a ragged
    [S, T] panel: pandas resample(interval, origin="start_day").agg(aggs) on
    the open_time index. Returns (bin labels int64 [S, B], {field: [S, B]},
    bins per row int64 [S]); B = the longest row's bin count, read back from
    the device — or, with max_bins (fixed frame geometry, e.g. a captured
    graph: no host synchronisation), B = max_bins, which must be at least
    every row's bin count (bins past a row's count are left unwritten) —
    or, with tail=True (bq_resample_tail), a row with more bins than B keeps
    its newest B bins, so bin min(bins, B) - 1 is always the row's latest
    (the returned bins per row stay the true counts)."""
    ts = _check_ts(ts)
    S, T = ts.shape
    names = list(fields)
    if len(names) > _lib.MAX_RESAMPLE_FIELDS:
        raise ValueError(f"at most {_lib.MAX_RESAMPLE_FIELDS} fields per resample call")
    ins = [_check_panel(fields[n], n, (S, T)).contiguous() for n in names]
    codes = []
    for n in names:
        a = aggs.get(n)
        if a not in _lib.AGG_CODES:
            raise ValueError(f"{n}: aggregation {a!r} not in {sorted(_lib.AGG_CODES)}")
        codes.append(_lib.AGG_CODES[a])
    lens = _check_lens(lens, S, ts.device)
    L = _lib.load()
    out_lens = torch.empty(S, dtype=torch.int64, device=ts.device)
    _lib.check(L.bq_resample_count(_ptr(ts), _ptr(lens), S, T, T, int(interval_ms), _ptr(out_lens),
                                   _stream_handle(stream)), "bq_resample_count")
    if max_bins is not None:
        if max_bins < 0:
            raise ValueError("max_bins must be >= 0")
        B = int(max_bins)
    else:
        B = int(out_lens.max().item()) if S else 0
    out_ts = torch.empty((S, B), dtype=torch.int64, device=ts.device)
    outs = [torch.empty((S, B), dtype=torch.float64, device=ts.device) for _ in names]
    agg_arr = (ctypes.c_int32 * max(1, len(codes)))(*codes)
    st = (L.bq_resample_tail if tail else L.bq_resample)(
        _ptr(ts), _lib.ptr_array([t.data_ptr() for t in ins]), ctypes.cast(agg_arr, ctypes.c_void_p), len(names),
        _ptr(lens), S, T, T, int(interval_ms), _ptr(out_ts), _lib.ptr_array([t.data_ptr() for t in outs]), B,
        _stream_handle(stream),
    )
    _lib.check(st, "bq_resample")
    return out_ts, dict(zip(names, outs)), out_lens


@device_entry
def align(ts: torch.Tensor, bench_ts: torch.Tensor, bench_val: torch.Tensor, lens=None,
          stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """Benchmark value at each candle's timestamp (left merge on open_time,
    duplicates keep "last"; strategies/liquidation_sweep_pump.py:255-263),
    NaN where the benchmark has no candle. ts [S, T] int64, bench_ts [Tb]
    ascending, bench_val [Tb] float64."""
    ts = _check_ts(ts)
    S, T = ts.shape
    bts = _check_ts(bench_ts, "bench_ts").reshape(-1)
    bval = _check_panel(bench_val.reshape(1, -1), "bench_val", (1, bts.numel())).contiguous()
    lens = _check_lens(lens, S, ts.device)
    out = torch.empty((S, T), dtype=torch.float64, device=ts.device)
    st = _lib.load().bq_align(_ptr(ts), _ptr(lens), S, T, T, _ptr(bts), _ptr(bval), bts.numel(), _ptr(out), T,
                              _stream_handle(stream))
    _lib.check(st, "bq_align")
    return out


LEADERSHIP_FUSED = dict(lookback=96, long_max=31)   # bq_leadership's compiled configuration


@device_entry
def leadership(open_time: torch.Tensor, close: torch.Tensor, bench_ts: torch.Tensor, bench_close: torch.Tensor,
               rs_quantile: float = 0.80, lookback: int = 96, min_history: int = 100, min_count: int = 20,
               short: int = 8, long: int = 24, stream: torch.cuda.Stream | None = None):
    """GradualGainerRetest._leadership_allows at every prefix t
    (strategies/gradual_gainer_retest.py:131-196) in one pass (bq_leadership:
    the thresholds are never formed — "rs >= sorted(h)[a]" is a count of the
    window's entries <= rs): returns {"leader": bool [S, T], "rs_2h": [S, T],
    "rs_6h": [S, T]}, or None when the parameters are not the compiled ones
    (RS_LOOKBACK 96, long <= 31): the caller then runs the staged pipeline."""
    if lookback != LEADERSHIP_FUSED["lookback"] or not 0.0 <= rs_quantile < 1.0 \
            or not 1 <= short <= long <= LEADERSHIP_FUSED["long_max"] or min_count < 1 or min_history < 0:
        return None
    close = _check_panel(close, "close").contiguous()
    S, T = close.shape
    ts = _check_ts(open_time)
    if tuple(ts.shape) != (S, T):
        raise ValueError(f"open_time: expected shape {(S, T)}, got {tuple(ts.shape)}")
    bts = _check_ts(bench_ts, "bench_ts").reshape(-1).contiguous()
    bc = _check_panel(bench_close.reshape(1, -1), "bench_close", (1, bts.numel())).contiguous()
    dev = close.device
    leader = torch.empty((S, T), dtype=torch.bool, device=dev)
    rs2 = torch.empty((S, T), dtype=torch.float64, device=dev)
    rs6 = torch.empty_like(rs2)
    lib = _lib.load()
    nbytes = int(lib.bq_leadership_workspace_bytes(S, T))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)   # caching allocator: 512-B aligned
    st = lib.bq_leadership(_ptr(ts), T, _ptr(close), T, S, T, _ptr(bts), _ptr(bc), bts.numel(), float(rs_quantile),
                           int(lookback), int(min_history), int(min_count), int(short), int(long), _ptr(ws), nbytes,
                           _ptr(leader), _ptr(rs2), _ptr(rs6), T, _stream_handle(stream))
    _lib.check(st, "bq_leadership")
    return {"leader": leader, "rs_2h": rs2, "rs_6h": rs6}


def _join_capacity(ts: torch.Tensor, lens: torch.Tensor | None, bts: torch.Tensor) -> int:
    """Largest per-row count of (candle, benchmark row) matches over the
    candles t >= 1 that join (bench_ts ascending): an upper bound on every
    row's joined pairs (dropna only removes some)."""
    S, T = ts.shape
    if S == 0 or T < 2 or bts.numel() == 0:
        return T
    # a benchmark without repeated times joins each candle at most once: T
    # (one small reduction over the benchmark, not a search per candle)
    if bts.numel() < 2 or not bool((bts[1:] == bts[:-1]).any()):
        return T
    keys = ts[:, 1:].contiguous()
    mult = torch.searchsorted(bts, keys, right=True) - torch.searchsorted(bts, keys)
    if lens is not None:
        live = torch.arange(1, T, device=ts.device)[None, :] < lens.reshape(-1, 1)
        mult = torch.where(live, mult, torch.zeros_like(mult))
    return int(mult.sum(dim=1).max().item())


@device_entry
def join_returns(ts: torch.Tensor, close: torch.Tensor, bench_ts: torch.Tensor, bench_close: torch.Tensor,
                 lens=None, capacity: int | None = None, stream: torch.cuda.Stream | None = None):
    """Aligned (symbol, benchmark) log-return pairs of
    ContextEvaluator.dynamic_btc_beta_corr (producers/context_evaluator.py:161-177):
    returns on each frame's own rows, inner join on the timestamp, dropna,
    compacted per row. Returns (x [S, C], y [S, C], pairs per row int64 [S]).
    A benchmark time held k times joins k pairs (pandas' inner join; a frame
    repeating its own time k_l times joins k_l * k times), so a row can hold
    more than T pairs. capacity=None: C = the largest row's joined-row count
    (each candle's benchmark multiplicity, summed per row, on the device: one
    host synchronisation), so no row is ever cut. An int capacity (fixed
    geometry, e.g. a captured graph) gives C = max(T, capacity) without the
    synchronisation; a row with more pairs than C is then cut at C, keeping
    its oldest pairs — size it from the benchmark's repeats. capacity=None
    cannot be used under hipGraph capture (it reads the repeat check back to
    the host): a capturing caller gets a ValueError asking for capacity."""
    ts = _check_ts(ts)
    S, T = ts.shape
    close = _check_panel(close, "close", (S, T)).contiguous()
    bts = _check_ts(bench_ts, "bench_ts").reshape(-1)
    bc = _check_panel(bench_close.reshape(1, -1), "bench_close", (1, bts.numel())).contiguous()
    lens = _check_lens(lens, S, ts.device)
    if capacity is None:
        if torch.cuda.is_current_stream_capturing():
            raise ValueError("join_returns: capacity=None synchronises with the host and cannot run under "
                             "graph capture; pass capacity= (e.g. T when the benchmark repeats no time)")
        capacity = _join_capacity(ts, lens, bts)
    C = max(T, int(capacity))
    x = torch.empty((S, C), dtype=torch.float64, device=ts.device)
    y = torch.empty_like(x)
    n = torch.empty(S, dtype=torch.int64, device=ts.device)
    st = _lib.load().bq_join_returns(_ptr(ts), _ptr(close), _ptr(lens), S, T, T, _ptr(bts), _ptr(bc), bts.numel(),
                                     _ptr(x), _ptr(y), C, _ptr(n), _stream_handle(stream))
    _lib.check(st, "bq_join_returns")
    return x, y, n


@device_entry
def beta_corr_pairs(x: torch.Tensor, y: torch.Tensor, window: int = 50,
                    stream: torch.cuda.Stream | None = None) -> dict[str, torch.Tensor]:
    """Rolling beta / corr over aligned return pairs (join_returns output):
    NaN for rows < window - 1."""
    x = _check_panel(x, "x").contiguous()
    S, T = x.shape
    y = _check_panel(y, "y", (S, T)).contiguous()
    beta = torch.empty((S, T), dtype=torch.float64, device=x.device)
    corr = torch.empty_like(beta)
    st = _lib.load().bq_beta_corr_pairs(_ptr(x), _ptr(y), S, T, T, int(window), _ptr(beta), _ptr(corr), T,
                                        _stream_handle(stream))
    _lib.check(st, "bq_beta_corr_pairs")
    return {"beta": beta, "corr": corr}


@device_entry
def pct_change(x: torch.Tensor, periods: int = 1, fill_method: str | None = "pad") -> torch.Tensor:
    """x.pct_change(periods) along T of a [S, T] panel with pandas 2.3.3's
    default fill_method='pad': f / f.shift(periods) - 1 over the
    forward-filled series f (leading NaNs stay NaN; [1, 2, nan, 4, 5] ->
    [nan, 1, 0, 1, 0.25]) — the BTC 24h change of
    producers/context_evaluator.py:427-430. fill_method=None: the raw series.
    The fill is the device ffill replay (bq_rolling_batch), the quotient the
    same IEEE operations as pandas."""
    x = _check_panel(x, "x")
    if fill_method not in ("pad", "ffill", None):
        raise ValueError(f"fill_method must be 'pad' or None, got {fill_method!r}")
    periods = int(periods)
    if periods < 1:
        raise ValueError(f"periods must be >= 1, got {periods}")
    f = rolling_many(Ffill(x))[0] if fill_method is not None else x
    out = torch.full_like(f, float("nan"))
    if periods < f.shape[1]:
        out[:, periods:] = f[:, periods:] / f[:, :-periods] - 1
    return out