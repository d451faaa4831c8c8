/*
 * binquant_amd — C ABI of the MI355X (gfx950) technical-indicator engine.
 *
 * This is the drop-in boundary for binquant's indicator hot path. Every entry
 * point takes caller-owned DEVICE buffers (plain pointers + sizes), a
 * hipStream_t (passed as void* so this header needs no HIP include), and
 * returns an int status: 0 = ok, < 0 = error (see BQ_E*). No C++ exception
 * crosses this ABI and the library allocates nothing per call.
 *
 * Data layout (all fp64): structure-of-arrays, one array per OHLCV field,
 * each [S][ld] row-major by symbol (candles of one symbol contiguous), i.e.
 * exactly the memory of S pandas float64 columns laid side by side.
 *
 * Reference interfaces replaced (paths relative to carkod/binquant):
 *   bq_enrich          <- ContextEvaluator.indicators_enrichment
 *                         producers/context_evaluator.py:240-263, i.e. the
 *                         pybinbot.Indicators calls at :249-261
 *                         (moving_averages x3, macd, rsi, bollinguer_spreads,
 *                          set_twap, atr) plus Indicators.mfi
 *                         (strategies/coinrule/price_tracker.py:185) and the
 *                         ema20/ema50 columns of
 *                         market_regime/live_market_context_accumulator.py:266-267
 *   bq_tick            <- per-message recompute of the same columns on the
 *                         latest candle (consumers/klines_provider.py:300-380
 *                         -> context_evaluator.py:347-512), as an O(1) state
 *                         update per symbol
 *   bq_market_features <- LiveMarketContextAccumulator._compute_symbol_features
 *                         market_regime/live_market_context_accumulator.py:244-297
 *                         evaluated at every timestamp of a [S][T] panel
 *   bq_beta_corr       <- ContextEvaluator.dynamic_btc_beta_corr
 *                         producers/context_evaluator.py:154-194
 *   bq_supertrend      <- pybinbot Indicators.set_supertrend
 *                         strategies/coinrule/coinrule.py:143-160
 *   bq_resample*       <- pybinbot Candles.resample(df, "1h")
 *                         producers/context_evaluator.py:403-407
 *   bq_align           <- the benchmark left merge of
 *                         strategies/liquidation_sweep_pump.py:255-263
 *   bq_join_returns,   <- the inner join + rolling beta/corr of
 *   bq_beta_corr_pairs    producers/context_evaluator.py:161-194
 *   bq_store_*         <- MarketStateStore (market_regime/market_state_store.py:14-87)
 *                         and _compute_symbol_features on its histories
 *   bq_parse_kline_events <- json.loads + KlineProduceModel of the websocket
 *                         frames, producers/klines_connector.py:77-164 (host)
 *   bq_micro_regime    <- regime_transitions.py:162-232 (per-symbol micro regime)
 *   bq_context_score   <- context_scoring.py:13-114 + signal_context_scorer.py:15-55
 *   bq_cohort_select   <- the portfolio selectors' winner pick
 *                         (liquidation_sweep_pump.py:38-87, gradual_gainer_retest.py:33-70)
 *   bq_breadth_partial <- the per-symbol sums/counts of
 *                         LiveMarketContextAccumulator._build_context
 *                         market_regime/live_market_context_accumulator.py:135-163
 */
#ifndef BINQUANT_AMD_H
#define BINQUANT_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------- */
#define BQ_OK              0
#define BQ_EINVAL         -1   /* bad argument (null pointer, size, window)   */
#define BQ_EHIP           -2   /* HIP runtime error (launch / memcpy)         */
#define BQ_EALIGN         -3   /* reserved: misaligned buffer                 */
#define BQ_ESTATE         -4   /* state handle misuse                         */

/* ---- canonical enrich column set ---------------------------------------- */
/* Order of the `out` pointer array of bq_enrich / bq_tick. A NULL entry
 * skips that column (its bytes are neither computed nor written). */
enum bq_enrich_col {
  BQ_MA_FAST = 0,     /* "ma_7"        close.rolling(7).mean()              */
  BQ_MA_MID,          /* "ma_25"       close.rolling(25).mean()             */
  BQ_MA_SLOW,         /* "ma_100"      close.rolling(100).mean()            */
  BQ_MACD,            /* "macd"        ema12 - ema26 (adjust=False)         */
  BQ_MACD_SIGNAL,     /* "macd_signal" macd.ewm(span=9, adjust=False)       */
  BQ_RSI,             /* "rsi"         SMA-smoothed RSI(14)                 */
  BQ_BB_UPPER,        /* "bb_upper"    mid + k*std                          */
  BQ_BB_MID,          /* "bb_mid"      close.rolling(20).mean()             */
  BQ_BB_LOWER,        /* "bb_lower"    mid - k*std                          */
  BQ_ATR,             /* "ATR"         true_range.rolling(14).mean()        */
  BQ_TWAP,            /* "twap"        ohlc4.rolling(12).mean()             */
  BQ_EMA_FAST,        /* "ema20"       close.ewm(span=20, adjust=False)     */
  BQ_EMA_SLOW,        /* "ema50"       close.ewm(span=50, adjust=False)     */
  BQ_MFI,             /* "mfi"         money-flow index(14)                 */
  BQ_NUM_ENRICH_COLS
};

/* Input field order of the `in` pointer array. */
enum bq_ohlcv_field { BQ_OPEN = 0, BQ_HIGH, BQ_LOW, BQ_CLOSE, BQ_VOLUME, BQ_NUM_INPUTS };

/* Indicator parameters; defaults (bq_default_params) are the reference's. */
typedef struct bq_params {
  int32_t ma_periods[3];   /* 7, 25, 100   (context_evaluator.py:249-251)   */
  int32_t macd_fast;       /* 12                                            */
  int32_t macd_slow;       /* 26                                            */
  int32_t macd_signal;     /* 9                                             */
  int32_t rsi_window;      /* 14                                            */
  int32_t bb_window;       /* 20                                            */
  int32_t bb_ddof;         /* 1 = pandas default std(); 0 = population      */
  int32_t atr_window;      /* 14           (context_evaluator.py:261)       */
  int32_t twap_window;     /* 12                                            */
  int32_t ema_spans[2];    /* 20, 50       (live_market_context_acc.:266)   */
  int32_t mfi_window;      /* 14           (price_tracker.py:185)           */
  int32_t reserved;
  double  bb_k;            /* 2.0                                           */
} bq_params;

/* Largest rolling window any kernel supports (LDS halo - 2). */
#define BQ_MAX_WINDOW 126

void bq_default_params(bq_params* p);

/* Library / device info. */
const char* bq_version(void);
int bq_device_arch(char* buf, int buflen);   /* e.g. "gfx950" */

/*
 * Full indicator set over a [S][T] panel.
 *   in[BQ_NUM_INPUTS]        device pointers, each [S][ld_in] fp64
 *   out[BQ_NUM_ENRICH_COLS]  device pointers, each [S][ld_out] fp64 (NULL = skip)
 * Warm-up rows are NaN exactly where pandas yields NaN (t < window-1).
 * Input contract: finite candles. The panel is what Candles.pre_process /
 * post_process leave (producers/context_evaluator.py:364-371), which has no
 * NaN rows; a symbol missing candles is a ragged row (enrich_frames), not a
 * NaN row. Missing candles in the live feed go through bq_tick, which keeps
 * pandas' NaN-gap rules.
 */
int bq_enrich(const double* const* in, int64_t S, int64_t T, int64_t ld_in,
              const bq_params* params, double* const* out, int64_t ld_out,
              void* stream);

/* ---- streaming tick path ------------------------------------------------- */
typedef struct bq_state bq_state;   /* opaque, device-resident */

/* Candles in the per-message frame the tick path reproduces: the reference
 * re-fetches KlinesProvider.LIMIT = 400 candles and re-enriches them on every
 * closed kline (consumers/klines_provider.py:40,201-215 ->
 * producers/context_evaluator.py:367-371), so its EMAs are seeded at the
 * frame's first candle. */
#define BQ_TICK_FRAME 400

/* Create state for S symbols. Allocates device memory once (not per tick).
 * bq_state_create = bq_state_create_frame(.., BQ_TICK_FRAME). `frame` = 0
 * keeps unbounded-history EMA carries (the full-series pandas EMA) instead;
 * otherwise BQ_MAX_WINDOW + 2 <= frame <= 2^20 (the frame holds every rolling
 * window, so only the EMA family depends on it). */
int bq_state_create(bq_state** st, int64_t S, const bq_params* params);
int bq_state_create_frame(bq_state** st, int64_t S, const bq_params* params, int64_t frame);
int bq_state_destroy(bq_state* st);
/* Seed the state from a [S][T] history panel (T >= 1): ring of the last
 * BQ_MAX_WINDOW+2 candles, and the last `frame` closes (frame mode) or the
 * exact EMA carries at the last candle (frame 0). */
int bq_state_seed(bq_state* st, const double* const* in, int64_t T, int64_t ld_in,
                  void* stream);
/* Append one candle per symbol. new_ohlcv[BQ_NUM_INPUTS] device pointers of
 * length S; out[BQ_NUM_ENRICH_COLS] device pointers of length S (NULL skip).
 * The outputs are the last row of indicators_enrichment over the symbol's
 * frame (the last `frame` candles; all candles when frame = 0): ema20, ema50,
 * macd and macd_signal bit-equal to pandas' ewm(adjust=False) over that frame.
 * A symbol without a candle this tick passes NaN in all five fields: the
 * outputs are then what pandas gives for a frame with that NaN row — EMAs
 * hold their value and decay their old weight by (1 - alpha)
 * (ewm(adjust=False, ignore_na=False)), windows containing the row are NaN,
 * RSI/MFI count its move as 0 (delta.where(...) fills NaN with 0). */
int bq_tick(bq_state* st, const double* const* new_ohlcv, double* const* out,
            void* stream);
int64_t bq_state_symbols(const bq_state* st);
int64_t bq_state_frame(const bq_state* st);   /* 0 = unbounded */
int64_t bq_state_count(const bq_state* st);   /* candles seen per symbol */

/* ---- market context (breadth / regime) ----------------------------------- */
/* Per-symbol feature columns of _compute_symbol_features, order of `feat`. */
enum bq_feature_col {
  BQ_F_RETURN = 0,    /* return_pct = safe_pct(c_t, c_{t-1})               */
  BQ_F_EMA20,         /* ema over the last `max_bars` closes, span 20       */
  BQ_F_EMA50,         /* span 50                                            */
  BQ_F_TREND,         /* (ema20-ema50)/|ema50|                              */
  BQ_F_ATR_PCT,       /* TR.rolling(14,min_periods=1).mean() / close        */
  BQ_F_BB_WIDTH,      /* 4*std(20,ddof=0)/|mid|                             */
  BQ_NUM_FEATURES
};

/* Breadth partial layout per timestamp: [T][BQ_NUM_PARTIALS] fp64. */
enum bq_partial_col {
  BQ_P_COUNT = 0,     /* symbols with features at t (history >= 2 bars)    */
  BQ_P_ADV,           /* return_pct > 0                                    */
  BQ_P_DEC,           /* return_pct < 0                                    */
  BQ_P_ABOVE20,       /* close > ema20                                     */
  BQ_P_ABOVE50,       /* close > ema50                                     */
  BQ_P_SUM_RET,
  BQ_P_SUM_TREND,
  BQ_P_SUM_ATR_PCT,
  BQ_P_SUM_BB_WIDTH,
  BQ_P_RESERVED,
  BQ_NUM_PARTIALS
};

/*
 * Per-symbol market features at every timestamp, with the accumulator's
 * history cap (MarketStateStore max_bars_per_symbol) applied: the features
 * at t see only candles (t-max_bars, t] (15 <= max_bars <= BQ_MAX_HISTORY).
 * hlc = {high, low, close} device pointers, each [S][ld_in].
 * feat[BQ_NUM_FEATURES] device pointers [S][ld_out] (NULL = skip). Row t = 0
 * (fewer than 2 bars of history -> reference returns None) is NaN.
 * Domain: finite high / low / close (a panel of exchange klines). A candle
 * without a close never reaches the reference's features (MarketStateStore
 * drops it, market_state_store.py:84); histories holding candles without a
 * high / low (which the store keeps) go through bq_store_features, the
 * store path's pandas replay. bq_context_partials has the same domain.
 */
#define BQ_MAX_HISTORY 512
int bq_market_features(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in,
                       int32_t max_bars, double* const* feat, int64_t ld_out,
                       void* stream);

/*
 * Cross-symbol partial sums per timestamp over the S symbols of this shard,
 * from the feature columns of bq_market_features (all of BQ_F_RETURN,
 * BQ_F_EMA20, BQ_F_EMA50, BQ_F_TREND, BQ_F_ATR_PCT, BQ_F_BB_WIDTH) and close:
 * partial[T][BQ_NUM_PARTIALS] fp64, overwritten. Deterministic (fixed
 * reduction order, no atomics). Feeds an RCCL all-reduce(sum) across shards,
 * then the scalar scoring of _build_context on the host.
 */
int bq_breadth_partial(const double* close, const double* const* feat, int64_t S, int64_t T,
                       int64_t ld_close, int64_t ld_feat, double* partial, void* stream);

/*
 * Fused panel context build (BASELINE configs[4]): the features of
 * bq_market_features reduced straight into the partials of
 * bq_breadth_partial, without writing the feature columns
 * (live_market_context_accumulator.py:95-163 over :244-297 at every t).
 * Replaces bq_market_features + bq_breadth_partial when only the [T][10]
 * partials (and, optionally, the last timestamp's features) are read.
 * hlc = {high, low, close} [S][ld_in]; partial[T][BQ_NUM_PARTIALS]
 * overwritten (column BQ_P_RESERVED = 0). last_feat: NULL, or
 * BQ_NUM_FEATURES device pointers (each NULL or [S]) receiving the features
 * at t = T - 1. workspace: device memory of bq_context_workspace_bytes(S, T)
 * bytes, 256-byte aligned (group records of 4 symbols; the library
 * allocates nothing). Counts equal bq_breadth_partial's; the sums agree to
 * rounding (another fixed order). Deterministic: no atomics.
 */
size_t bq_context_workspace_bytes(int64_t S, int64_t T);
int bq_context_partials(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in,
                        int32_t max_bars, void* workspace, size_t workspace_bytes,
                        double* partial, double* const* last_feat, void* stream);

/*
 * GradualGainerRetest relative-strength leadership at every prefix t
 * (GradualGainerRetest._leadership_allows + _relative_strengths,
 * strategies/gradual_gainer_retest.py:131-196): open_time [S][ld_ts] int64 ms
 * and close [S][ld_c] of the panel, the benchmark frame bench_ts [nb]
 * (ascending; a duplicated time keeps the later row) / bench_close [nb].
 * Outputs [S][ld_out]: leader (0 / 1 bytes) and rs_2h / rs_6h as the method
 * returns them ((False, 0.0, 0.0) when the strengths are None or the frame
 * is shorter than min_history). One pass: "rs >= sorted(history)[int((n - 1)
 * q)]" is decided by counting the window's entries <= rs (the thresholds are
 * not outputs of the method). Compiled for the strategy's RS_LOOKBACK 96 and
 * long_bars <= 31; other parameters return BQ_EINVAL (the Python layer then
 * runs its staged pipeline). bq_leadership_workspace_bytes returns 0 (the
 * workspace arguments are kept for callers that size one; NULL is fine).
 */
size_t bq_leadership_workspace_bytes(int64_t S, int64_t T);
int bq_leadership(const int64_t* open_time, int64_t ld_ts, const double* close, int64_t ld_c, int64_t S,
                  int64_t T, const int64_t* bench_ts, const double* bench_close, int64_t nb,
                  double rs_quantile, int32_t lookback, int32_t min_history, int32_t min_count,
                  int32_t short_bars, int32_t long_bars, void* workspace, size_t workspace_bytes,
                  uint8_t* leader, double* rs_2h, double* rs_6h, int64_t ld_out, void* stream);

/* ---- benchmark-relative statistics ---------------------------------------- */
/*
 * Rolling beta and correlation of log returns vs the benchmark
 * (ContextEvaluator.dynamic_btc_beta_corr, producers/context_evaluator.py:154-194)
 * at every timestamp: close [S][ld_in], btc_close [T] (index-aligned with the
 * panel), window 2..BQ_MAX_WINDOW (reference: 50). beta/corr [S][ld_out]
 * (NULL = skip). NaN where t < window, beta NaN where var(btc) == 0. Inputs
 * must be finite and positive (the reference dropna()s only the first return).
 */
int bq_beta_corr(const double* close, const double* btc_close, int64_t S, int64_t T, int64_t ld_in,
                 int32_t window, double* beta, double* corr, int64_t ld_out, void* stream);

/* ---- rolling-window statistics (strategy feature pipelines) ---------------- */
#define BQ_MAX_ROLLING_WINDOW 96
enum bq_roll_mode {
  BQ_ROLL_QUANTILE = 0, BQ_ROLL_MEDIAN = 1, BQ_ROLL_MEAN = 2, BQ_ROLL_SUM = 3,
  BQ_ROLL_VAR = 4,   /* ddof 1 */
  BQ_ROLL_STD = 5,   /* ddof 1 */
  BQ_ROLL_VAR0 = 6,  /* ddof 0 */
  BQ_ROLL_STD0 = 7,  /* ddof 0 */
  BQ_ROLL_EWM = 8,   /* bq_rolling_batch only: ewm(alpha, adjust=False, min_periods) */
  BQ_ROLL_FFILL = 9, /* bq_rolling_batch only: ffill() (leading NaNs stay), shift 0;
                        Series.pct_change's default fill_method='pad' */
  BQ_ROLL_ISUM = 10, /* rolling sum of a series whose values are integers with
                        |sum| < 2^53 (counts of boolean flags): pandas' result
                        is then exact in any summation order, so the window is
                        summed directly (no sequential replay); same values,
                        same-value rule and min_periods as BQ_ROLL_SUM */
  BQ_ROLL_QLOWER = 11 /* quantile(q, interpolation="lower"): the int((n-1) q)-th
                        smallest of the window's n values, no interpolation —
                        sorted(history)[int((len(history) - 1) * q)] of
                        GradualGainerRetest._leadership_allows
                        (strategies/gradual_gainer_retest.py:182-187) */
};
/*
 * out = x.shift(shift).rolling(window, min_periods).<mode>() per symbol row,
 * pandas semantics (NaNs skipped, NaN below min_periods; quantile = linear
 * interpolation, q in [0, 1]; q = 0 / 1 give rolling min / max; sum / mean
 * compensated, pandas' same-value rule for mean / sum / var / std; an empty
 * window sums to 0 when min_periods is 0). Replaces the
 * pandas rolling calls of strategies/activity_burst_pump.py:58-63,134-152,
 * strategies/liquidation_sweep_pump.py:218-245, strategies/failed_spike_fade.py:376-378.
 * x, out [S][ld] fp64 device pointers; window <= BQ_MAX_ROLLING_WINDOW;
 * ld_out <= BQ_MAX_ROLL_LD (else BQ_EINVAL).
 */
#define BQ_MAX_ROLL_LD 4194303   /* 64 rows x ld_out x 8 B < 2^31 (32-bit buffer offsets) */
int bq_rolling(const double* x, int64_t S, int64_t T, int64_t ld_in, int32_t window, int32_t min_periods,
               int32_t shift, int32_t mode, double q, double* out, int64_t ld_out, void* stream);

/*
 * out = x.shift(shift).rolling(window, min_periods).quantile(q) as bq_rolling
 * (BQ_ROLL_QUANTILE), and cross[t] = (x[t] >= out[t]) & (x[t-1] < out[t-1])
 * as one byte per candle (pandas comparisons: NaN compares false; 0 at t = 0)
 * — LiquidationSweepPump's score_threshold and score_cross
 * (strategies/liquidation_sweep_pump.py:231-239) in one pass where the
 * sliding-window kernel runs (else the quantile, then a flag pass). cross:
 * uint8 [S][ld_cross] device pointer.
 */
int bq_rolling_quantile_cross(const double* x, int64_t S, int64_t T, int64_t ld_in, int32_t window,
                              int32_t min_periods, int32_t shift, double q, double* out, int64_t ld_out,
                              uint8_t* cross, int64_t ld_cross, void* stream);

/*
 * Many independent rolling / ewm series over one [S][T] shape in one call
 * (the strategy pipelines issue 5-18 of them per frame batch, e.g.
 * strategies/failed_spike_fade.py:260-357): one launch per kernel family
 * instead of one per series, so lane-per-symbol replays of different series
 * run side by side. Jobs are read from HOST memory (copied into the launch).
 */
#define BQ_MAX_ROLL_JOBS 16
typedef struct bq_roll_job {
  const double* x;         /* [S][ld_in] device pointer                        */
  double* out;             /* [S][ld_out] device pointer                       */
  int64_t ld_in, ld_out;
  int32_t window, min_periods, shift, mode;   /* mode: bq_roll_mode            */
  double q;                /* quantile                                         */
  double alpha;            /* BQ_ROLL_EWM                                      */
  int64_t rows;            /* rows of this job's x / out, 1 <= rows <= S (a    */
                           /* benchmark series beside the panel); 0 = all S.  */
                           /* Moments / ewm / ffill only: order statistics    */
                           /* need 0 or S.                                     */
  int32_t panel;           /* 1: sum / mean (window + shift <= 128) and ewm    */
                           /* time-parallel, within rounding of pandas (1e-9) */
                           /* instead of the bit-exact sequential replay      */
  int32_t reserved;
} bq_roll_job;
int bq_rolling_batch(const bq_roll_job* jobs, int32_t n_jobs, int64_t S, int64_t T, void* stream);
/*
 * bq_rolling_batch with crossing flags: for a BQ_ROLL_QUANTILE job i with
 * cross[i] != NULL (uint8 [S][ld_cross[i]] device pointer; the job on all S
 * rows), also cross[i][t] = (x[t] >= out[t]) & (x[t-1] < out[t-1]) as
 * bq_rolling_quantile_cross — formed in the sliding-window kernel's steps
 * where that kernel runs the job. cross / ld_cross: host arrays of n_jobs
 * (cross NULL: none).
 */
int bq_rolling_batch_cross(const bq_roll_job* jobs, int32_t n_jobs, int64_t S, int64_t T, uint8_t* const* cross,
                           const int64_t* ld_cross, void* stream);

/*
 * out = x.ewm(alpha=alpha, adjust=False, min_periods=min_periods).mean()
 * (ignore_na=False: NaN gaps decay the old weight) per symbol row, the exact
 * pandas recursion. Replaces strategies/liquidation_sweep_pump.py:215-217,
 * :265-266 and strategies/mean_reversion_fade.py:94-99.
 */
int bq_ewm(const double* x, int64_t S, int64_t T, int64_t ld_in, double alpha, int32_t min_periods, double* out,
           int64_t ld_out, void* stream);

/*
 * LiquidationSweepPump's per-symbol ewm columns in panel mode (time-parallel,
 * within rounding of pandas; strategies/liquidation_sweep_pump.py:206-217,
 * :252-253): atr = TR.ewm(alpha=1/14, adjust=False, min_periods=14).mean() of
 * the true range of (high, low, close) — formed in the kernel, no TR column —
 * and ema20 / ema50 = close.ewm(span=20 / 50, adjust=False).mean(), in one
 * pass per row; trend_score (NULL = skip) = (ema20 - ema50) / ema50 (:254).
 * Inputs [S][ld_in], outputs [S][ld_out] fp64. Feeds bq_pump_features.
 */
int bq_pump_ewm(const double* high, const double* low, const double* close, int64_t S, int64_t T, int64_t ld_in,
                double* atr, double* ema20, double* ema50, double* trend_score, int64_t ld_out, void* stream);

/* ---- whole-series order statistics and label cooldown ---------------------- */
/*
 * out[s] = numpy.quantile(x[s][~isnan], q) (numpy 'linear' method, numpy's
 * two-sided lerp), NaN for a row without observations. Replaces the
 * np.quantile calls of FailedSpikeFade.auto_calibrate
 * (strategies/failed_spike_fade.py:229-257) and Series.quantile
 * (strategies/relative_strength_reversal_range.py:98). out: S doubles.
 */
int bq_row_quantile(const double* x, int64_t S, int64_t T, int64_t ld_in, double q, double* out, void* stream);

/*
 * FailedSpikeFade.apply_cooldown (strategies/failed_spike_fade.py:495-520):
 * a label (nonzero byte) within `bars` candles of the last kept label is
 * cleared in kept[] and set in suppressed[]. label/kept/suppressed: uint8
 * [S][ld] device pointers.
 */
int bq_cooldown(const uint8_t* label, int64_t S, int64_t T, int64_t ld_in, int32_t bars, uint8_t* kept,
                uint8_t* suppressed, int64_t ld_out, void* stream);

/* ---- fused strategy stages -------------------------------------------------- */
/*
 * LiquidationSweepPump.compute_pump_score (strategies/liquidation_sweep_pump.py:
 * 195-269) in one pass per row, panel mode: every column but the two rolling
 * quantiles (score_threshold / volume_threshold) and score_cross, with the
 * volume.shift(1).rolling(volume_lookback).mean() and the
 * high / low .shift(1).rolling(compression_bars).max() / .min() windows and
 * close.pct_change(momentum_bars) (pad-filled) formed in the kernel.
 * in = {high, low, close, volume, candidate_atr, ema20, ema50} [S][ld_in]
 * fp64 (the three ewm columns from bq_pump_ewm; ema20 / ema50 may both be
 * NULL when out[BQ_PUMP_EMA20 / EMA50 / TREND_SCORE] are NULL); bench = {ffilled
 * benchmark close, its ewm(span=20), ewm(span=50)} [T] fp64 (the benchmark
 * left-merged on the panel's open_time grid); out[BQ_NUM_PUMP_COLS] [S][ld_out]
 * fp64 (NULL = skip). momentum_bars <= 31, volume_lookback and
 * compression_bars <= 30.
 */
enum bq_pump_col {
  BQ_PUMP_CANDIDATE_ATR = 0, BQ_PUMP_MOMENTUM_3, BQ_PUMP_RELATIVE_VOLUME, BQ_PUMP_COMPRESSION, BQ_PUMP_SCORE,
  BQ_PUMP_PRIOR_HIGH, BQ_PUMP_CLOSE_LOCATION, BQ_PUMP_EMA20, BQ_PUMP_EMA50, BQ_PUMP_TREND_SCORE,
  BQ_PUMP_MOMENTUM_ATR, BQ_PUMP_BTC_MOMENTUM_3, BQ_PUMP_BTC_TREND_SCORE, BQ_PUMP_RELATIVE_STRENGTH,
  BQ_NUM_PUMP_COLS
};
int bq_pump_features(const double* const* in, int64_t S, int64_t T, int64_t ld_in, const double* const* bench,
                     int32_t momentum_bars, int32_t volume_lookback, int32_t compression_bars, double* const* out,
                     int64_t ld_out, void* stream);
/*
 * The same pass with the three per-symbol ewm columns formed inside it
 * (candidate_atr = TR.ewm(alpha=1/14, adjust=False, min_periods=14).mean(),
 * ema20 / ema50 = close.ewm(span=20 / 50, adjust=False).mean(),
 * liquidation_sweep_pump.py:206-217, 252-253; within rounding of pandas, a
 * row with a missing / infinite value continuing with pandas' recursion):
 * in = {high, low, close, volume} only; out[BQ_PUMP_CANDIDATE_ATR /
 * BQ_PUMP_EMA20 / BQ_PUMP_EMA50] must be non-NULL.
 */
int bq_pump_features_ewm(const double* const* in, int64_t S, int64_t T, int64_t ld_in, const double* const* bench,
                         int32_t momentum_bars, int32_t volume_lookback, int32_t compression_bars,
                         double* const* out, int64_t ld_out, void* stream);

/*
 * ActivityBurstPump.compute_indicators (strategies/activity_burst_pump.py:51-158)
 * around the score's rolling quantile, bit for bit with the staged pipeline:
 * bq_burst_features forms every column of :58-133 from in = {open, high, low,
 * close, volume, quote_volume, baseline_volume, baseline_quote_volume}
 * [S][ld_in] fp64 (the two baselines: volume.shift(2).rolling(19).median(),
 * bq_rolling_batch; quote_volume and its baseline NULL without a quote
 * volume column: the reference's neutral fallbacks), out_f[BQ_NUM_BURST_F]
 * fp64 and out_b[BQ_NUM_BURST_B] uint8 [S][ld_out] (NULL = skip), all_flags
 * uint8 [S][ld_out]: the AND of the six flags (NULL = skip). bq_burst_qualify:
 * qualified_signal from the score, its threshold (rolling quantile) and
 * all_flags (:140-156), cooldown_bars <= 8; ld_b = the byte arrays' stride.
 */
typedef struct bq_burst_params {
  double volume_multiplier, quote_volume_multiplier, price_threshold, min_baseline_volume;
  double min_range_frac, min_body_frac, max_close_to_high;
  int32_t min_recent_up_closes;   /* the effective minimum (1 without a quote volume) */
  int32_t reserved;
} bq_burst_params;
enum bq_burst_fcol {
  BQ_BURST_BASELINE_VOLUME_SAFE = 0, BQ_BURST_VOLUME_RATIO, BQ_BURST_BASELINE_QUOTE_VOLUME_SAFE,
  BQ_BURST_QUOTE_VOLUME_RATIO, BQ_BURST_PRICE_JUMP, BQ_BURST_RANGE_FRAC, BQ_BURST_BODY_FRAC, BQ_BURST_CLOSE_TO_HIGH,
  BQ_BURST_RECENT_UP_CLOSES, BQ_BURST_SCORE, BQ_NUM_BURST_F
};
enum bq_burst_bcol {
  BQ_BURST_IS_BULLISH = 0, BQ_BURST_VOL_SPIKE, BQ_BURST_QUOTE_VOL_SPIKE, BQ_BURST_PRICE_JUMP_FLAG,
  BQ_BURST_RANGE_EXPANSION_FLAG, BQ_BURST_BODY_QUALITY_FLAG, BQ_BURST_TREND_QUALITY_FLAG, BQ_NUM_BURST_B
};
int bq_burst_features(const double* const* in, int64_t S, int64_t T, int64_t ld_in, const bq_burst_params* p,
                      double* const* out_f, uint8_t* const* out_b, uint8_t* all_flags, int64_t ld_out, void* stream);
int bq_burst_qualify(const double* score, const double* threshold, const uint8_t* all_flags, int64_t S, int64_t T,
                     int64_t ld_in, int64_t ld_b, int32_t cooldown_bars, uint8_t* qualified, void* stream);

/*
 * FailedSpikeFade.detect (strategies/failed_spike_fade.py:260-544) in two
 * passes per row around auto_calibrate. bq_spike_base: in = {open, high, low,
 * close, volume, quote_volume, ffilled close, price_std (close, base window),
 * volume_std (base window), close std 8, close std 20, body_size_pct std 10}
 * [S][ld_in] fp64 (the std columns: bq_rolling_batch's bit-exact replays) ->
 * compute_base_features' and the early features' columns (out_f
 * [BQ_NUM_SPIKE_BASE_F] fp64, out_b [BQ_NUM_SPIKE_BASE_B] uint8, NULL = skip),
 * the rolling means / sums (min_periods = window) formed in the kernel;
 * base_window, streak_length <= 30. bq_spike_flags: in = {open, close, ffilled
 * close, volume_ratio, |pct change| rolling quantile} [S][ld_in], vcmr / pbbt
 * [S] (the calibrated volume-cluster ratio and price-break base) -> the flag
 * columns and preliminary labels of :360-488 (cooldown: bq_cooldown).
 */
typedef struct bq_spike_params {
  int32_t volume_cluster_window, volume_cluster_min_count, cumulative_price_window, accel_volume_deriv_window;
  int32_t label_mode;   /* 0 last, 1 first, 2 all */
  int32_t require_both_patterns, require_bullish_spike, reserved;
  double cumulative_price_threshold, accel_volume_deriv_min, accel_price_change_min, body_size_pct_min;
} bq_spike_params;
enum bq_spike_base_fcol {
  BQ_SPIKE_PRICE_CHANGE = 0, BQ_SPIKE_PRICE_CHANGE_ABS, BQ_SPIKE_BODY_SIZE, BQ_SPIKE_BODY_SIZE_PCT,
  BQ_SPIKE_UPPER_WICK, BQ_SPIKE_LOWER_WICK, BQ_SPIKE_UPPER_WICK_RATIO, BQ_SPIKE_LOWER_WICK_RATIO,
  BQ_SPIKE_TOTAL_RANGE, BQ_SPIKE_RANGE_PCT, BQ_SPIKE_CLOSE_OPEN_RATIO, BQ_SPIKE_PRICE_MA, BQ_SPIKE_PRICE_ZSCORE,
  BQ_SPIKE_VOLUME_MA, BQ_SPIKE_VOLUME_RATIO, BQ_SPIKE_VOLUME_ZSCORE, BQ_SPIKE_QUOTE_VOLUME_MA,
  BQ_SPIKE_QUOTE_VOLUME_RATIO, BQ_SPIKE_MOMENTUM_3, BQ_SPIKE_MOMENTUM_5, BQ_SPIKE_CLOSE_TO_HIGH,
  BQ_SPIKE_CLOSE_TO_LOW, BQ_SPIKE_STD_RATIO_8_20, BQ_SPIKE_PC_2C, BQ_SPIKE_PC_3C, BQ_SPIKE_PC_POS_COUNT_5,
  BQ_SPIKE_PC_ABS_SUM_5, BQ_SPIKE_BODY_SIZE_PCT_MA_10, BQ_SPIKE_BODY_SIZE_PCT_Z, BQ_NUM_SPIKE_BASE_F
};
enum bq_spike_base_bcol {
  BQ_SPIKE_IS_BULLISH = 0, BQ_SPIKE_VOL_COMPRESSION_FLAG, BQ_SPIKE_UPWARD, BQ_SPIKE_DOWNWARD, BQ_NUM_SPIKE_BASE_B
};
enum bq_spike_flag_fcol {
  BQ_SPIKE_VOL_RATIO_SLOPE_3 = 0, BQ_SPIKE_VOL_RATIO_ACCEL, BQ_SPIKE_PRICE_BREAK_THRESHOLD, BQ_SPIKE_EARLY_PROBA,
  BQ_NUM_SPIKE_FLAG_F
};
enum bq_spike_flag_bcol {
  BQ_SPIKE_VOLUME_CLUSTER_FLAG = 0, BQ_SPIKE_PRICE_BREAK_FLAG, BQ_SPIKE_CUM_BREAK_FLAG, BQ_SPIKE_CUM_BREAK_SHORT_FLAG,
  BQ_SPIKE_ACCEL_FLAG, BQ_SPIKE_ACCEL_SHORT_FLAG, BQ_SPIKE_LABEL_PRE, BQ_SPIKE_LABEL_SHORT_PRE,
  BQ_SPIKE_EARLY_AUG_FLAG, BQ_NUM_SPIKE_FLAG_B
};
int bq_spike_base(const double* const* in, int64_t S, int64_t T, int64_t ld_in, int32_t base_window,
                  int32_t streak_length, double* const* out_f, uint8_t* const* out_b, int64_t ld_out, void* stream);
/*
 * bq_spike_base_std: the same pass in panel mode with the five rolling std
 * columns (FailedSpikeFade.compute_base_features' price_std, volume_std,
 * rolling_price_std_8 / _20 and compute_early_features' body_size_pct std 10,
 * failed_spike_fade.py:293-339) formed in the pass — two-pass window sums
 * (the window's variance to rounding) instead of the bit-exact replay of
 * pandas' online recurrence. in = the first 7 inputs of bq_spike_base
 * {open, high, low, close, volume, quote_volume, ffilled close}; out_sd
 * [BQ_NUM_SPIKE_STD] fp64 [S][ld_out] (NULL entries = not written).
 */
enum bq_spike_std_col {
  BQ_SPIKE_STD_PRICE = 0, BQ_SPIKE_STD_VOLUME, BQ_SPIKE_STD_8, BQ_SPIKE_STD_20, BQ_SPIKE_STD_BODY_PCT_10,
  BQ_NUM_SPIKE_STD
};
int bq_spike_base_std(const double* const* in, int64_t S, int64_t T, int64_t ld_in, int32_t base_window,
                      int32_t streak_length, double* const* out_f, uint8_t* const* out_b, double* const* out_sd,
                      int64_t ld_out, void* stream);
int bq_spike_flags(const double* const* in, const double* vcmr, const double* pbbt, int64_t S, int64_t T,
                   int64_t ld_in, const bq_spike_params* p, double* const* out_f, uint8_t* const* out_b,
                   int64_t ld_out, void* stream);

/* ---- sequential state machines (lane = symbol) ----------------------------- */
/*
 * Supertrend trend flag and final bands (pybinbot Indicators.set_supertrend,
 * called at strategies/coinrule/coinrule.py:143 with multiplier 3.0, period 10;
 * the consumer reads bool(df["supertrend"].iloc[-1]) at :160). hlca = {high,
 * low, close, ATR} [S][ld_in] fp64 (ATR = bq_enrich's ATR column with
 * atr_window = period). up: uint8 [S][ld_out] (1 = uptrend); upper/lower:
 * fp64 [S][ld_out] final bands (NULL = skip). Recurrence: see bq_seq.hip.
 */
int bq_supertrend(const double* const* hlca, int64_t S, int64_t T, int64_t ld_in, double multiplier,
                  uint8_t* up, double* upper, double* lower, int64_t ld_out, void* stream);
/*
 * bq_supertrend with the ATR formed in the same walk: hlc = {high, low, close}
 * [S][ld_in] fp64, ATR = TR.rolling(period).mean() replayed as pandas'
 * roll_mean (1 <= period <= BQ_MAX_WINDOW), so flags and bands are pandas'
 * bit for bit; one launch, no ATR column in HBM (engine.supertrend).
 */
int bq_supertrend_hlc(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in, int32_t period,
                      double multiplier, uint8_t* up, double* upper, double* lower, int64_t ld_out, void* stream);
/*
 * bq_supertrend_hlc in panel mode (engine.supertrend(exact=False)): one
 * workgroup per row, each thread walks a chunk of it from a warm-up, then
 * every chunk start is verified against its predecessor's end state (the
 * rare wrong one re-walked), so the flags and bands equal the sequential
 * recursion on the same ATR; the ATR (TR.rolling(period).mean(), min_periods
 * = period, same-value rule) is a direct window sum per candle, equal to
 * pandas' roll_mean to rounding, not bit for bit. Rows longer than 2048
 * candles run bq_supertrend_hlc.
 */
int bq_supertrend_panel(const double* const* hlc, int64_t S, int64_t T, int64_t ld_in, int32_t period,
                        double multiplier, uint8_t* up, double* upper, double* lower, int64_t ld_out, void* stream);

/* ---- frame plumbing: resample and timestamp joins (ragged rows) ------------ */
/* Timestamps are int64 ms, ascending within a row; lens[s] = valid candles of
 * row s (NULL: all T). */
#define BQ_MAX_RESAMPLE_FIELDS 12
enum bq_agg { BQ_AGG_FIRST = 0, BQ_AGG_LAST = 1, BQ_AGG_MAX = 2, BQ_AGG_MIN = 3, BQ_AGG_SUM = 4 };
/*
 * Candles.resample(df, interval="1h") (producers/context_evaluator.py:403-407,
 * pybinbot): pandas resample(interval, origin="start_day", closed/label left)
 * .agg(...) on the open_time index. bq_resample_count writes the number of
 * bins of each row (first candle's bin .. last candle's bin) to out_lens[S];
 * bq_resample fills out_ts (bin labels, NULL = skip) and out_fields
 * [nfields][S][ld_out] (ld_out >= max out_lens) with per-field aggregation
 * aggs[f] (bq_agg; NaN-skipping, SUM Kahan-compensated like pandas group_sum;
 * empty bins NaN, SUM 0).
 */
int bq_resample_count(const int64_t* ts, const int64_t* lens, int64_t S, int64_t T, int64_t ld_in,
                      int64_t interval_ms, int64_t* out_lens, void* stream);
int bq_resample(const int64_t* ts, const double* const* fields, const int32_t* aggs, int32_t nfields,
                const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, int64_t interval_ms, int64_t* out_ts,
                double* const* out_fields, int64_t ld_out, void* stream);
/* bq_resample for a fixed output geometry (a captured graph sizes ld_out on
 * the host): a row with more bins than ld_out — a gap in the candles widens
 * the span, and pandas emits every empty bin of it — keeps its NEWEST ld_out
 * bins (output bin b = the row's bin b + out_lens[s] - ld_out), so the last
 * written bin is always the row's latest, the one process_data reads. */
int bq_resample_tail(const int64_t* ts, const double* const* fields, const int32_t* aggs, int32_t nfields,
                     const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, int64_t interval_ms, int64_t* out_ts,
                     double* const* out_fields, int64_t ld_out, void* stream);
/*
 * Left merge of a benchmark series on the timestamp
 * (strategies/liquidation_sweep_pump.py:255-263, duplicates keep "last"):
 * out[s][t] = bench_val[j] with bench_ts[j] == ts[s][t], NaN if absent.
 * bench_ts ascending, n_bench entries.
 */
int bq_align(const int64_t* ts, const int64_t* lens, int64_t S, int64_t T, int64_t ld_in, const int64_t* bench_ts,
             const double* bench_val, int64_t n_bench, double* out, int64_t ld_out, void* stream);
/*
 * The aligned returns of ContextEvaluator.dynamic_btc_beta_corr
 * (producers/context_evaluator.py:161-177): log(c/c.shift(1)) on each frame's
 * own rows, inner-joined on the timestamp, dropna'd, compacted in order into
 * x (symbol) / y (benchmark) [S][ld_out] with out_lens[s] pairs (NaN tail).
 * A time the benchmark holds k times joins k pairs, in the benchmark's order,
 * each with the return over the benchmark row before it (pandas' inner join
 * on a repeated right index); a row whose pairs would pass ld_out keeps the
 * first ld_out (out_lens[s] = ld_out). bench_ts ascending.
 */
int bq_join_returns(const int64_t* ts, const double* close, const int64_t* lens, int64_t S, int64_t T, int64_t ld_in,
                    const int64_t* bench_ts, const double* bench_close, int64_t n_bench, double* x, double* y,
                    int64_t ld_out, int64_t* out_lens, void* stream);
/*
 * bq_beta_corr on already-aligned return pairs (x, y [S][ld_in], dropna'd
 * prefix of each row): beta/corr of rolling(window) at every row, NaN for
 * rows < window - 1.
 */
/* bq_beta_corr with the benchmark given as its log returns (btc_returns[T],
 * btc_returns[t] = log(btc[t] / btc[t-1]), NaN at t = 0): the returns are
 * formed once per call instead of once per symbol row (engine.beta_corr).
 * scratch: NULL, or 3*T doubles of device memory in which the benchmark's
 * window mean / variance / inverse variance are computed once (a
 * one-workgroup pre-pass) instead of in every symbol's wave. */
int bq_beta_corr_bret(const double* close, const double* btc_returns, double* scratch, int64_t S, int64_t T,
                      int64_t ld_in, int32_t window, double* beta, double* corr, int64_t ld_out, void* stream);
/* bq_beta_corr with a device scratch of 4*T doubles: a one-workgroup
 * pre-pass forms the benchmark's log returns and their window mean /
 * variance / inverse variance once per call, then one wave per symbol row
 * (engine.beta_corr: two launches per call, no host-side returns pass). */
int bq_beta_corr_ws(const double* close, const double* btc_close, double* scratch, int64_t S, int64_t T,
                    int64_t ld_in, int32_t window, double* beta, double* corr, int64_t ld_out, void* stream);
int bq_beta_corr_pairs(const double* x, const double* y, int64_t S, int64_t T, int64_t ld_in, int32_t window,
                       double* beta, double* corr, int64_t ld_out, void* stream);

/* ---- device-resident MarketStateStore -------------------------------------- */
/*
 * market_regime/market_state_store.py:14-87 kept in HBM: per symbol slot a
 * ring of the last max_bars closed candles, sorted by timestamp, unique
 * timestamps (a later update of a timestamp replaces it, keep="last").
 * Caller-owned buffers (the library allocates nothing):
 */
#define BQ_STORE_MAX_BARS 512
typedef struct bq_store_view {
  int64_t* ts;                     /* [capacity][max_bars] candle timestamps (ms)        */
  double*  field[BQ_NUM_INPUTS];   /* open, high, low, close, volume, same layout       */
  int32_t* head;                   /* [capacity] ring index of the oldest candle        */
  int32_t* count;                  /* [capacity] candles held (<= max_bars)             */
  int64_t* last;                   /* [capacity] last closed timestamp (undefined if 0) */
  int64_t  capacity;
  int32_t  max_bars;               /* 2 .. BQ_STORE_MAX_BARS                            */
  int32_t  reserved;
} bq_store_view;
/*
 * MarketStateStore.update for a batch: n_seg runs of candles, run g =
 * [seg_begin[g], seg_begin[g+1]) all for slot[seg_begin[g]], timestamps
 * strictly ascending inside a run, one run per slot per call (the caller
 * sorts and de-duplicates the batch, keep="last"). NaN close / timestamp rows
 * must already be dropped (market_state_store.py:84). slot, ts, seg_begin and
 * the five ohlcv arrays are device pointers.
 */
int bq_store_update(const bq_store_view* st, const int64_t* slot, const int64_t* ts, const double* const* ohlcv,
                    const int64_t* seg_begin, int64_t n_seg, void* stream);
/*
 * LiveMarketContextAccumulator._compute_symbol_features
 * (market_regime/live_market_context_accumulator.py:244-297) on the histories
 * of n_sel slots: feat[BQ_NUM_FEATURES] arrays of n_sel doubles (NULL =
 * skip; NaN rows where a history has < 2 candles, i.e. the reference's None)
 * and close_out[n_sel] (latest close). pandas' ewm / roll_mean / roll_var
 * recurrences are replayed, so values equal pandas' bit for bit.
 */
int bq_store_features(const bq_store_view* st, const int64_t* slots, int64_t n_sel, double* const* feat,
                      double* close_out, void* stream);
/*
 * The per-symbol pass of one live context build
 * (LiveMarketContextAccumulator._build_context,
 * market_regime/live_market_context_accumulator.py:95-133) over ALL n tracked
 * slots [0, n): a slot is fresh when its last closed candle is *fresh_ts
 * (MarketStateStore.get_fresh_symbols, market_state_store.py:49-54; fresh_ts
 * is a device pointer, so a captured graph reads the tick's timestamp).
 * feat / close_out rows: the features of counted fresh slots, NaN otherwise
 * (the benchmark's row only when btc_counted: a sharded store replicates the
 * benchmark and counts it on one rank); fresh_out[n]: 1.0 / 0.0 for those
 * rows; btc_out[8]: the benchmark's features, latest close (whatever its
 * freshness, :105-106) and 1.0 / 0.0 = fresh (unwritten when btc_slot < 0). Same replay as
 * bq_store_features (pandas bit for bit); non-fresh slots are not replayed.
 */
int bq_store_context_features(const bq_store_view* st, int64_t n, const int64_t* fresh_ts, int64_t btc_slot,
                              int btc_counted, double* const* feat, double* close_out, double* fresh_out,
                              double* btc_out, void* stream);
/*
 * MarketStateStore.get_symbol_history / get_all_histories: time-ordered copy
 * of n_sel slots into ts_out / out[BQ_NUM_INPUTS] [n_sel][ld_out]
 * (ld_out >= max_bars; NaN / 0 past each slot's count; NULL = skip).
 */
int bq_store_gather(const bq_store_view* st, const int64_t* slots, int64_t n_sel, int64_t* ts_out,
                    double* const* out, int64_t ld_out, void* stream);

/* ---- signal-generator helpers, time-parallel (bq_signals.hip) --------------- */
/*
 * The inline helpers of the signal generators at every candle of a [S][T]
 * panel (column t = the helper on df.iloc[:t + 1]), split along the time axis
 * (tolerance-exact, 1e-9 relative; the bit-exact replay of the same helpers is
 * the binquant_amd.signals composition with exact=True). Finite prices in,
 * out [S][ld_out] fp64 device pointers.
 *   bq_wilder_rsi  MeanReversionFade._rsi (strategies/mean_reversion_fade.py:88-109):
 *                  ewm(alpha=1/window, min_periods=window, adjust=False) of
 *                  gains / losses, 100 g / (g + l), 50 where g + l == 0
 *   bq_zscore      RangeBbRsiMeanReversion._compute_zscore
 *                  (strategies/range_bb_rsi_mean_reversion.py:132-138): 0 where
 *                  the ddof-0 std is 0 or NaN (warm-up included)
 *   bq_adx         RangeBbRsiMeanReversion._compute_adx (:101-130): 100 where
 *                  the window mean of dx is NaN; window <= 64
 */
int bq_wilder_rsi(const double* close, int64_t S, int64_t T, int64_t ld_in, int32_t window, double* out,
                  int64_t ld_out, void* stream);
int bq_zscore(const double* close, int64_t S, int64_t T, int64_t ld_in, int32_t window, double* out, int64_t ld_out,
              void* stream);
int bq_adx(const double* high, const double* low, const double* close, int64_t S, int64_t T, int64_t ld_in,
           int32_t window, double* out, int64_t ld_out, void* stream);

/* ---- regime annotation, candidate scoring, portfolio selection -------------- */
enum bq_micro_regime_code {   /* models.py:15-21 MicroRegime; -1 = None */
  BQ_MICRO_TREND_UP = 0, BQ_MICRO_TREND_DOWN = 1, BQ_MICRO_RANGE = 2, BQ_MICRO_VOLATILE = 3,
  BQ_MICRO_TRANSITIONAL = 4
};
enum bq_micro_transition_code {   /* models.py:32-42 MicroRegimeTransition; -1 = None */
  BQ_MT_VOLATILITY_EXPANSION = 0, BQ_MT_BREAKOUT_UP, BQ_MT_BREAKDOWN, BQ_MT_RECOVERY, BQ_MT_MEAN_REVERSION,
  BQ_MT_ENTERED_TREND_UP, BQ_MT_ENTERED_TREND_DOWN, BQ_MT_ENTERED_RANGE, BQ_MT_ENTERED_TRANSITIONAL
};
/*
 * RegimeTransitionDetector._annotate_symbol_regime (market_regime/regime_transitions.py:162-232)
 * for n symbols: device arrays of the SymbolMarketFeatures fields; prev_regime
 * (int8, -1 = None; NULL = no previous context) / prev_strength chain the
 * transition. Outputs regime/strength (+ transition / transition_strength,
 * NULL = skip). Bit-exact with the Python floats.
 */
int bq_micro_regime(int64_t n, const double* trend, const uint8_t* above_ema20, const uint8_t* above_ema50,
                    const double* rs, const double* bb_width, const double* atr_pct, const double* return_pct,
                    const int8_t* prev_regime, const double* prev_strength, int8_t* regime, double* strength,
                    int8_t* transition, double* transition_strength, void* stream);

enum bq_direction { BQ_DIR_LONG = 0, BQ_DIR_SHORT = 1, BQ_DIR_OTHER = 2 };   /* direction.upper().strip() */
typedef struct bq_context_scalars {   /* the LiveMarketContext fields the scorer reads */
  double confidence, long_tailwind, short_tailwind, btc_regime_score, market_stress_score;
  int32_t present;                    /* 0: no context (None) */
  int32_t reserved;
} bq_context_scalars;
typedef struct bq_scorer_weights {    /* SignalContextScorer (signal_context_scorer.py:10-13) */
  double context_weight, risk_weight, support_weight;
} bq_scorer_weights;
enum bq_score_field {   /* MarketContextScore fields + the adjusted score; out[field][ld_out] */
  BQ_SC_CONFIDENCE = 0, BQ_SC_BREADTH, BQ_SC_BTC_ALIGNMENT, BQ_SC_CROSS_ASSET, BQ_SC_FOLLOWTHROUGH,
  BQ_SC_ADVERSE, BQ_SC_OVERRIDE, BQ_SC_SUPPORTIVENESS, BQ_SC_ADJUSTED, BQ_NUM_SCORE_FIELDS
};
/*
 * RuleBasedMarketContextModel.evaluate (market_regime/context_scoring.py:13-114)
 * + SignalContextScorer.adjust_score (signal_context_scorer.py:15-28) for n
 * candidates against one context: direction (bq_direction), rs / trend (the
 * candidate's local_features or its snapshot row, resolved by the caller),
 * local_score (NULL = 0). out: BQ_NUM_SCORE_FIELDS x ld_out doubles.
 */
int bq_context_score(int64_t n, const int8_t* direction, const double* rs, const double* trend,
                     const double* local_score, const bq_context_scalars* ctx, const bq_scorer_weights* weights,
                     double* out, int64_t ld_out, void* stream);
/*
 * Portfolio winners (strategies/liquidation_sweep_pump.py:38-87,
 * strategies/gradual_gainer_retest.py:33-70): per cohort (dense ids
 * 0..n_cohorts-1) the accepted candidate (accepted NULL = all) with the
 * largest (score, symbol_rank), the latest submission on a full tie.
 * winner[n_cohorts]: candidate index or -1. scratch: 2*n_cohorts u64 (device).
 */
int bq_cohort_select(int64_t n, const int32_t* cohort, const uint8_t* accepted, const double* score,
                     const int32_t* symbol_rank, int32_t n_cohorts, unsigned long long* scratch, int64_t* winner,
                     void* stream);

/* ---- wire-format ingest (host) ------------------------------------------------ */
/*
 * Binance kline websocket events (one JSON object per '\n'-separated frame,
 * as decoded at producers/klines_connector.py:77-90 and copied into a
 * KlineProduceModel at :148-164) -> arrays, in one native pass: sym
 * [max_rows][sym_stride] NUL-terminated symbols ("s"), open_time ("t"),
 * close_time ("T"), ohlcv[5] ("o","h","l","c","v" via strtod: the same
 * doubles as Python float()), closed ("x"). HOST pointers. Non-kline frames
 * are skipped; malformed kline frames are counted in n_bad and skipped.
 * Returns BQ_EINVAL (with n_rows filled so far) if max_rows is too small.
 */
int bq_parse_kline_events(const char* buf, int64_t len, int64_t max_rows, char* sym, int64_t sym_stride,
                          int64_t* open_time, int64_t* close_time, double* const* ohlcv, uint8_t* closed,
                          int64_t* n_rows, int64_t* n_bad);

/* ---- fused element-wise programs ---------------------------------------------- */
/*
 * The element-wise glue of the strategy pipelines (SURVEY §8a a17-a20:
 * ratios, clips, flags, shifted differences, where-selections between the
 * rolling series — e.g. activity_burst_pump.py:64-133, liquidation_sweep_pump.py:
 * 218-269, failed_spike_fade.py:260-493) evaluated as ONE launch per stage: a
 * straight-line program run per element (s, t) of an [S, T] panel, values in
 * fp64 with IEEE operations in the order the program lists them (the
 * reference's pandas operation order), so results equal the unfused
 * arithmetic bit for bit. Intermediates live in LDS registers, never in HBM.
 *
 * Instruction (uint64): op | dst << 8 | a << 16 | b << 24 | c << 32 | imm << 40
 * (imm: signed 24-bit). The first n_loads instructions are BQ_F_LD, issued
 * together before the rest runs.
 *   LD      dst <- in[b] at t - imm (consts[c] when t - imm is outside [0, T))
 *   CONST   dst <- consts[imm];   INRANGE dst <- 0 <= t - imm < T
 *   binary  dst <- a (op) b;      unary dst <- (op) a
 *   WHERE   dst <- a != 0 ? b : c
 *   (operand k of these ops is consts[k-th index] instead of a register
 *   when bit k of imm is set)
 *   ST      out[imm] <- a (BQ_F_U8 outputs store a != 0)
 * Comparisons give 1.0 / 0.0 (NaN compares false); AND / OR / NOT treat
 * non-zero as true; FMAX / FMIN skip NaN (torch.fmax), MAXIMUM / MINIMUM
 * propagate it (torch.maximum).
 * Operands: element (s, t) at ptr + s * stride_s + t * stride_t elements
 * (stride_t 0: a per-symbol value; stride_s 0: one series for all symbols).
 */
#define BQ_FUSED_MAX_INS 192
#define BQ_FUSED_MAX_CONST 32
#define BQ_FUSED_MAX_IN 16
#define BQ_FUSED_MAX_OUT 24
#define BQ_FUSED_MAX_REGS 20
#define BQ_FUSED_MAX_LOADS 16

enum bq_fused_dtype { BQ_F_F64 = 0, BQ_F_U8 = 1 };

enum bq_fused_op {
  BQ_F_LD = 1, BQ_F_CONST = 2, BQ_F_INRANGE = 3,
  BQ_F_ADD = 4, BQ_F_SUB = 5, BQ_F_MUL = 6, BQ_F_DIV = 7,
  BQ_F_FMAX = 8, BQ_F_FMIN = 9, BQ_F_MAXIMUM = 10, BQ_F_MINIMUM = 11,
  BQ_F_GT = 12, BQ_F_GE = 13, BQ_F_LT = 14, BQ_F_LE = 15, BQ_F_EQ = 16, BQ_F_NE = 17,
  BQ_F_AND = 18, BQ_F_OR = 19, BQ_F_NOT = 20,
  BQ_F_ABS = 21, BQ_F_NEG = 22, BQ_F_ISNAN = 23, BQ_F_SQRT = 24, BQ_F_LOG = 25,
  BQ_F_WHERE = 26, BQ_F_ST = 27
};

typedef struct {
  const void* ptr;
  int64_t stride_s, stride_t;   /* in elements */
  int32_t dtype;                /* bq_fused_dtype */
  int32_t reserved;
} bq_fused_operand;

typedef struct {
  int32_t n_ins, n_loads, n_regs, n_in, n_out, n_const;
  uint64_t ins[BQ_FUSED_MAX_INS];
  double consts[BQ_FUSED_MAX_CONST];
  bq_fused_operand in[BQ_FUSED_MAX_IN];
  bq_fused_operand out[BQ_FUSED_MAX_OUT];
} bq_fused_program;

/* Validates the program (opcodes, register / operand / constant indices,
 * loads first) and runs it over the [S, T] panel. Device operand pointers. */
int bq_fused_eval(const bq_fused_program* prog, int64_t S, int64_t T, void* stream);

/* Native form of the same programs: bq_fused_eval translates the program into
 * straight-line HIP source (operand layouts specialised, constants as exact
 * bit patterns), compiles it for gfx950 with hiprtc on first use and launches
 * the compiled kernel — bit-identical to the interpreter (the default; the
 * environment variable BQ_FUSED_NATIVE=0 or bq_fused_set_native(0) selects
 * the interpreter, -1 restores the environment's choice; returns the previous
 * setting, -1 if unset). Compiled code objects are cached per process and,
 * if a directory is set, on disk (<dir>/<hash>.gfx950.co + its source). */
int bq_fused_set_native(int on);
int bq_fused_set_cache_dir(const char* dir);
/* generated source of a (validated) program: *len = its length; up to cap-1
 * bytes + NUL copied into buf when buf is non-null. No device needed. */
int bq_fused_source(const bq_fused_program* prog, char* buf, int64_t cap, int64_t* len);
/* compile (or find in the caches) without launching. No device needed. */
int bq_fused_compile(const bq_fused_program* prog);
/* counters: hiprtc compiles, disk-cache hits, programs in the process cache */
int bq_fused_stats(int64_t* compiles, int64_t* disk_hits, int64_t* cached);

#ifdef __cplusplus
}
#endif

#endif /* BINQUANT_AMD_H */
