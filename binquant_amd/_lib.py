"""ctypes binding of the gfx950 HIP library (``include/binquant_amd.h``).

The library is built in-tree by ``make`` (or ``__graft_entry__.build()``) into
``binquant_amd/lib/libbinquant_amd.so``. There is no CPU fallback: if the
library is missing, or a call returns a non-zero status, this module raises.

torch is imported first so that the HIP runtime torch ships
(``libamdhip64.so.7``) is the one the loader binds our library to; device
pointers and streams are then shared with torch's allocator and streams.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (binds libamdhip64.so.7 before our library loads)

LIB_PATH = Path(os.environ.get("BQ_LIB_PATH", Path(__file__).resolve().parent / "lib" / "libbinquant_amd.so"))

BQ_OK = 0
BQ_EINVAL = -1
BQ_EHIP = -2
BQ_ESTATE = -4

ENRICH_COLUMNS = (
    "ma_7",
    "ma_25",
    "ma_100",
    "macd",
    "macd_signal",
    "rsi",
    "bb_upper",
    "bb_mid",
    "bb_lower",
    "ATR",
    "twap",
    "ema20",
    "ema50",
    "mfi",
)
INPUT_FIELDS = ("open", "high", "low", "close", "volume")
FEATURE_COLUMNS = ("return_pct", "ema20", "ema50", "trend_score", "atr_pct", "bb_width")
PARTIAL_COLUMNS = (
    "count",
    "advancers",
    "decliners",
    "above_ema20",
    "above_ema50",
    "sum_return",
    "sum_trend",
    "sum_atr_pct",
    "sum_bb_width",
    "tracked",   # 0 from the kernel; market_regime.batch.reduce_partials folds the shard's symbol count in
)
MAX_WINDOW = 126
MAX_RESAMPLE_FIELDS = 12
STORE_MAX_BARS = 512
MICRO_REGIMES = ("TREND_UP", "TREND_DOWN", "RANGE", "VOLATILE", "TRANSITIONAL")
MICRO_TRANSITIONS = ("VOLATILITY_EXPANSION", "BREAKOUT_UP", "BREAKDOWN", "RECOVERY", "MEAN_REVERSION",
                     "ENTERED_TREND_UP", "ENTERED_TREND_DOWN", "ENTERED_RANGE", "ENTERED_TRANSITIONAL")
SCORE_FIELDS = ("confidence", "breadth_score", "btc_alignment_score", "cross_asset_confirmation",
                "followthrough_score", "adverse_excursion_risk", "override_strength", "supportiveness_score",
                "adjusted_score")
AGG_CODES = {"first": 0, "last": 1, "max": 2, "min": 3, "sum": 4}
MAX_ROLLING_WINDOW = 96
ROLL_MODES = {"quantile": 0, "median": 1, "mean": 2, "sum": 3, "var": 4, "std": 5, "var0": 6, "std0": 7,
              "isum": 10,   # isum: sum of an integer-valued series (flag counts), bq_roll_mode BQ_ROLL_ISUM
              "qlower": 11}   # quantile(q, interpolation="lower"), BQ_ROLL_QLOWER
ROLL_EWM = 8
ROLL_FFILL = 9
ROLL_ISUM = 10
MAX_ROLL_JOBS = 16


class BqParams(ctypes.Structure):
    """Mirror of ``bq_params`` (include/binquant_amd.h)."""

    _fields_ = [
        ("ma_periods", ctypes.c_int32 * 3),
        ("macd_fast", ctypes.c_int32),
        ("macd_slow", ctypes.c_int32),
        ("macd_signal", ctypes.c_int32),
        ("rsi_window", ctypes.c_int32),
        ("bb_window", ctypes.c_int32),
        ("bb_ddof", ctypes.c_int32),
        ("atr_window", ctypes.c_int32),
        ("twap_window", ctypes.c_int32),
        ("ema_spans", ctypes.c_int32 * 2),
        ("mfi_window", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("bb_k", ctypes.c_double),
    ]


class BqStoreView(ctypes.Structure):
    """Mirror of ``bq_store_view`` (include/binquant_amd.h)."""

    _fields_ = [
        ("ts", ctypes.c_void_p),
        ("field", ctypes.c_void_p * 5),
        ("head", ctypes.c_void_p),
        ("count", ctypes.c_void_p),
        ("last", ctypes.c_void_p),
        ("capacity", ctypes.c_int64),
        ("max_bars", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


FUSED_MAX_INS = 192
FUSED_MAX_CONST = 32
FUSED_MAX_IN = 16
FUSED_MAX_OUT = 24
FUSED_MAX_REGS = 20
FUSED_MAX_LOADS = 16
FUSED_F64, FUSED_U8 = 0, 1
FUSED_OPS = {name: i for i, name in enumerate(
    ["LD", "CONST", "INRANGE", "ADD", "SUB", "MUL", "DIV", "FMAX", "FMIN", "MAXIMUM", "MINIMUM", "GT", "GE", "LT",
     "LE", "EQ", "NE", "AND", "OR", "NOT", "ABS", "NEG", "ISNAN", "SQRT", "LOG", "WHERE", "ST"], start=1)}


class BqFusedOperand(ctypes.Structure):
    """Mirror of ``bq_fused_operand``."""

    _fields_ = [("ptr", ctypes.c_void_p), ("stride_s", ctypes.c_int64), ("stride_t", ctypes.c_int64),
                ("dtype", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class BqFusedProgram(ctypes.Structure):
    """Mirror of ``bq_fused_program``."""

    _fields_ = [
        ("n_ins", ctypes.c_int32), ("n_loads", ctypes.c_int32), ("n_regs", ctypes.c_int32),
        ("n_in", ctypes.c_int32), ("n_out", ctypes.c_int32), ("n_const", ctypes.c_int32),
        ("ins", ctypes.c_uint64 * FUSED_MAX_INS),
        ("consts", ctypes.c_double * FUSED_MAX_CONST),
        ("inp", BqFusedOperand * FUSED_MAX_IN),
        ("out", BqFusedOperand * FUSED_MAX_OUT),
    ]


class BqRollJob(ctypes.Structure):
    """Mirror of ``bq_roll_job`` (include/binquant_amd.h)."""

    _fields_ = [
        ("x", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("ld_in", ctypes.c_int64),
        ("ld_out", ctypes.c_int64),
        ("window", ctypes.c_int32),
        ("min_periods", ctypes.c_int32),
        ("shift", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("q", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("rows", ctypes.c_int64),
        ("panel", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class BqContextScalars(ctypes.Structure):
    _fields_ = [("confidence", ctypes.c_double), ("long_tailwind", ctypes.c_double),
                ("short_tailwind", ctypes.c_double), ("btc_regime_score", ctypes.c_double),
                ("market_stress_score", ctypes.c_double), ("present", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class BqScorerWeights(ctypes.Structure):
    _fields_ = [("context_weight", ctypes.c_double), ("risk_weight", ctypes.c_double),
                ("support_weight", ctypes.c_double)]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_PP = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); every symbol declared in include/binquant_amd.h
SIGNATURES: dict[str, tuple] = {
    "bq_default_params": (None, [ctypes.POINTER(BqParams)]),
    "bq_version": (ctypes.c_char_p, []),
    "bq_device_arch": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    "bq_enrich": (
        ctypes.c_int,
        [_PP, _I64, _I64, _I64, ctypes.POINTER(BqParams), _PP, _I64, _P],
    ),
    "bq_state_create": (
        ctypes.c_int,
        [ctypes.POINTER(ctypes.c_void_p), _I64, ctypes.POINTER(BqParams)],
    ),
    "bq_state_create_frame": (
        ctypes.c_int,
        [ctypes.POINTER(ctypes.c_void_p), _I64, ctypes.POINTER(BqParams), _I64],
    ),
    "bq_state_destroy": (ctypes.c_int, [_P]),
    "bq_state_seed": (ctypes.c_int, [_P, _PP, _I64, _I64, _P]),
    "bq_tick": (ctypes.c_int, [_P, _PP, _PP, _P]),
    "bq_state_symbols": (_I64, [_P]),
    "bq_state_count": (_I64, [_P]),
    "bq_state_frame": (_I64, [_P]),
    "bq_market_features": (ctypes.c_int, [_PP, _I64, _I64, _I64, _I32, _PP, _I64, _P]),
    "bq_breadth_partial": (ctypes.c_int, [_P, _PP, _I64, _I64, _I64, _I64, _P, _P]),
    "bq_context_workspace_bytes": (ctypes.c_size_t, [_I64, _I64]),
    "bq_context_partials": (ctypes.c_int, [_PP, _I64, _I64, _I64, _I32, _P, ctypes.c_size_t, _P, _PP, _P]),
    "bq_pump_ewm": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _I64, _P]),
    "bq_leadership_workspace_bytes": (ctypes.c_size_t, [_I64, _I64]),
    "bq_leadership": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, _I64, _P, _P, _I64, ctypes.c_double, _I32, _I32, _I32,
                                     _I32, _I32, _P, ctypes.c_size_t, _P, _P, _P, _I64, _P]),
    "bq_beta_corr": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _I32, _P, _P, _I64, _P]),
    "bq_rolling": (ctypes.c_int, [_P, _I64, _I64, _I64, _I32, _I32, _I32, _I32, ctypes.c_double, _P, _I64, _P]),
    "bq_rolling_quantile_cross": (ctypes.c_int, [_P, _I64, _I64, _I64, _I32, _I32, _I32, ctypes.c_double, _P, _I64,
                                                 _P, _I64, _P]),
    "bq_ewm": (ctypes.c_int, [_P, _I64, _I64, _I64, ctypes.c_double, _I32, _P, _I64, _P]),
    "bq_row_quantile": (ctypes.c_int, [_P, _I64, _I64, _I64, ctypes.c_double, _P, _P]),
    "bq_cooldown": (ctypes.c_int, [_P, _I64, _I64, _I64, _I32, _P, _P, _I64, _P]),
    "bq_pump_features": (ctypes.c_int, [_PP, _I64, _I64, _I64, _PP, _I32, _I32, _I32, _PP, _I64, _P]),
    "bq_pump_features_ewm": (ctypes.c_int, [_PP, _I64, _I64, _I64, _PP, _I32, _I32, _I32, _PP, _I64, _P]),
    "bq_burst_features": (ctypes.c_int, [_PP, _I64, _I64, _I64, _P, _PP, _PP, _P, _I64, _P]),
    "bq_burst_qualify": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I64, _I32, _P, _P]),
    "bq_spike_base": (ctypes.c_int, [_PP, _I64, _I64, _I64, _I32, _I32, _PP, _PP, _I64, _P]),
    "bq_spike_base_std": (ctypes.c_int, [_PP, _I64, _I64, _I64, _I32, _I32, _PP, _PP, _PP, _I64, _P]),
    "bq_spike_flags": (ctypes.c_int, [_PP, _P, _P, _I64, _I64, _I64, _P, _PP, _PP, _I64, _P]),
    "bq_supertrend": (ctypes.c_int, [_PP, _I64, _I64, _I64, ctypes.c_double, _P, _P, _P, _I64, _P]),
    "bq_supertrend_hlc": (ctypes.c_int, [_PP, _I64, _I64, _I64, _I32, ctypes.c_double, _P, _P, _P, _I64, _P]),
    "bq_supertrend_panel": (ctypes.c_int, [_PP, _I64, _I64, _I64, _I32, ctypes.c_double, _P, _P, _P, _I64, _P]),
    "bq_resample_count": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _I64, _P, _P]),
    "bq_resample": (ctypes.c_int, [_P, _PP, _P, _I32, _P, _I64, _I64, _I64, _I64, _P, _PP, _I64, _P]),
    "bq_resample_tail": (ctypes.c_int, [_P, _PP, _P, _I32, _P, _I64, _I64, _I64, _I64, _P, _PP, _I64, _P]),
    "bq_align": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _P, _P, _I64, _P, _I64, _P]),
    "bq_join_returns": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _P, _P, _I64, _P, _P, _I64, _P, _P]),
    "bq_beta_corr_bret": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I32, _P, _P, _I64, _P]),
    "bq_beta_corr_ws": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I32, _P, _P, _I64, _P]),
    "bq_beta_corr_pairs": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _I32, _P, _P, _I64, _P]),
    "bq_store_update": (ctypes.c_int, [ctypes.POINTER(BqStoreView), _P, _P, _PP, _P, _I64, _P]),
    "bq_store_features": (ctypes.c_int, [ctypes.POINTER(BqStoreView), _P, _I64, _PP, _P, _P]),
    "bq_store_context_features": (ctypes.c_int, [ctypes.POINTER(BqStoreView), _I64, _P, _I64, _I32, _PP, _P, _P,
                                                 _P, _P]),
    "bq_store_gather": (ctypes.c_int, [ctypes.POINTER(BqStoreView), _P, _I64, _P, _PP, _I64, _P]),
    "bq_rolling_batch": (ctypes.c_int, [ctypes.POINTER(BqRollJob), _I32, _I64, _I64, _P]),
    "bq_rolling_batch_cross": (ctypes.c_int, [ctypes.POINTER(BqRollJob), _I32, _I64, _I64, _PP,
                                              ctypes.POINTER(ctypes.c_int64), _P]),
    "bq_fused_eval": (ctypes.c_int, [ctypes.POINTER(BqFusedProgram), _I64, _I64, _P]),
    "bq_fused_set_native": (ctypes.c_int, [_I32]),
    "bq_fused_set_cache_dir": (ctypes.c_int, [ctypes.c_char_p]),
    "bq_fused_source": (ctypes.c_int, [ctypes.POINTER(BqFusedProgram), ctypes.c_char_p, _I64, ctypes.POINTER(_I64)]),
    "bq_fused_compile": (ctypes.c_int, [ctypes.POINTER(BqFusedProgram)]),
    "bq_fused_stats": (ctypes.c_int, [ctypes.POINTER(_I64)] * 3),
    "bq_wilder_rsi": (ctypes.c_int, [_P, _I64, _I64, _I64, _I32, _P, _I64, _P]),
    "bq_zscore": (ctypes.c_int, [_P, _I64, _I64, _I64, _I32, _P, _I64, _P]),
    "bq_adx": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I64, _I32, _P, _I64, _P]),
    "bq_micro_regime": (ctypes.c_int, [_I64] + [_P] * 13 + [_P]),
    "bq_context_score": (ctypes.c_int, [_I64, _P, _P, _P, _P, ctypes.POINTER(BqContextScalars),
                                        ctypes.POINTER(BqScorerWeights), _P, _I64, _P]),
    "bq_cohort_select": (ctypes.c_int, [_I64, _P, _P, _P, _P, _I32, _P, _P, _P]),
    "bq_parse_kline_events": (ctypes.c_int, [ctypes.c_char_p, _I64, _I64, _P, _I64, _P, _P, _PP, _P, _P, _P]),
}


class NativeLibraryError(RuntimeError):
    pass


_lib: ctypes.CDLL | None = None


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load (once) and type the native library. Raises if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise NativeLibraryError(
            f"binquant_amd native library not found at {p}; run `make` "
            "(or __graft_entry__.build()) — there is no CPU fallback"
        )
    lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # compiled fused programs persist next to the library (bq_fused_jit.hip)
    cache = os.environ.get("BQ_FUSED_CACHE", str(p.parent / "fused_cache"))
    if cache:
        try:
            os.makedirs(cache, exist_ok=True)
            lib.bq_fused_set_cache_dir(cache.encode())
        except OSError:
            pass   # read-only tree: the per-process cache still applies
    if path is None:
        _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status == BQ_OK:
        return
    if status == BQ_EINVAL:
        raise ValueError(f"{what}: invalid argument (status {status})")
    raise RuntimeError(f"{what}: native call failed with status {status}")


def default_params() -> BqParams:
    p = BqParams()
    load().bq_default_params(ctypes.byref(p))
    return p


class BqBurstParams(ctypes.Structure):
    """bq_burst_params (include/binquant_amd.h)"""

    _fields_ = [("volume_multiplier", ctypes.c_double), ("quote_volume_multiplier", ctypes.c_double),
                ("price_threshold", ctypes.c_double), ("min_baseline_volume", ctypes.c_double),
                ("min_range_frac", ctypes.c_double), ("min_body_frac", ctypes.c_double),
                ("max_close_to_high", ctypes.c_double), ("min_recent_up_closes", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class BqSpikeParams(ctypes.Structure):
    """bq_spike_params (include/binquant_amd.h)"""

    _fields_ = [("volume_cluster_window", ctypes.c_int32), ("volume_cluster_min_count", ctypes.c_int32),
                ("cumulative_price_window", ctypes.c_int32), ("accel_volume_deriv_window", ctypes.c_int32),
                ("label_mode", ctypes.c_int32), ("require_both_patterns", ctypes.c_int32),
                ("require_bullish_spike", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("cumulative_price_threshold", ctypes.c_double), ("accel_volume_deriv_min", ctypes.c_double),
                ("accel_price_change_min", ctypes.c_double), ("body_size_pct_min", ctypes.c_double)]


def ptr_array(ptrs) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(ptrs))()
    for i, v in enumerate(ptrs):
        arr[i] = v if v else None
    return arr
