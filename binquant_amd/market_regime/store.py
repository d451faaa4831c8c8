"""Device-resident MarketStateStore and live market-context accumulator
(§8a a13, a14, a16).

``DeviceMarketStateStore`` keeps the API of market_regime/market_state_store.py
(update / get_symbol_history / get_all_histories / get_last_closed_timestamp /
get_tracked_symbols / get_fresh_symbols, same normalisation and errors) but
the histories live in HBM as per-symbol rings (bq_store_view): a closed
candle is an O(1) in-order append on the device instead of a pandas
concat + drop_duplicates + sort + tail (3.9 ms per update),
and ``update_batch`` / ``update_slots`` take a whole tick of symbols in one
launch.

``DeviceLiveMarketContextAccumulator`` keeps the API of
market_regime/live_market_context_accumulator.py (on_closed_candle,
refresh_context_for_timestamp, get_context, get_latest_context). A context
build is: fresh slots (last == ts) on the device -> bq_store_features on
their histories (pandas recurrences replayed bit for bit) ->
bq_breadth_partial (fixed-order sums) -> one all-reduce of 12 doubles when
symbols are sharded over ranks -> host scoring and regime annotation
(regime.py). The reference instead recomputes every fresh symbol's features
in pandas on every message (O(S^2 * 400) per period).
"""

from __future__ import annotations

import ctypes
import functools
from collections import deque
from collections.abc import Mapping, Sequence
from math import ceil
from typing import Any

import numpy as np
import pandas as pd
import torch
import torch.distributed as dist

from .. import _lib, engine
from .._lib import FEATURE_COLUMNS, INPUT_FIELDS
from .._lib import MICRO_TRANSITIONS
from .regime import MIN_COVERAGE_RATIO, REQUIRED_FRESH_SYMBOLS, annotate_market, score_contexts
from .scoring import labels, micro_regime

STORE_COLUMNS = ["timestamp", "open", "high", "low", "close", "volume"]


def normalize_candles(candle: Mapping[str, Any] | pd.Series | pd.DataFrame) -> pd.DataFrame:
    """MarketStateStore._normalize_input (market_regime/market_state_store.py:56-87):
    same defaults (volume 0, open/high/low = close), same ValueErrors, numeric
    coercion, rows without timestamp / close dropped."""
    if isinstance(candle, pd.DataFrame):
        df = candle.copy()
    elif isinstance(candle, pd.Series):
        df = candle.to_frame().T
    else:
        df = pd.DataFrame([dict(candle)])
    if "timestamp" not in df.columns:
        raise ValueError("MarketStateStore.update requires a 'timestamp' column.")
    for column in STORE_COLUMNS:
        if column not in df.columns:
            if column == "volume":
                df[column] = 0.0
            elif column in ("open", "high", "low"):
                df[column] = df["close"] if "close" in df.columns else np.nan
            else:
                raise ValueError(f"Missing required candle field '{column}'.")
    for column in STORE_COLUMNS:
        df[column] = pd.to_numeric(df[column], errors="coerce")
    df = df.dropna(subset=["timestamp", "close"])
    df["timestamp"] = df["timestamp"].astype(int)
    return df[STORE_COLUMNS].copy()


def _device(device) -> torch.device:
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("DeviceMarketStateStore needs a HIP device (no CPU fallback)")
    return torch.device("cuda")


def _on_device(fn):
    """Run a store / accumulator method on the store's device (made current
    for the call) and, for `stream=`, under engine.launch_scope's ordering."""

    @functools.wraps(fn)
    def wrapper(self, *args, stream=None, **kw):
        dev = self.device if hasattr(self, "device") else self.state_store.device
        ts: list = []
        for a in args:
            engine._cuda_tensors(a, ts)
        with engine.launch_scope(dev, stream, ts):
            return fn(self, *args, **kw)

    return wrapper


class SortedNames(Sequence):
    """sorted(names), computed on first access (metadata["fresh_symbols"]);
    `names` is an array or a SymbolFeatureRows (whose names are resolved
    lazily too)."""

    def __init__(self, names):
        self._src, self._sorted = names, None

    def _get(self) -> list[str]:
        if self._sorted is None:
            src = self._src.names if isinstance(self._src, SymbolFeatureRows) else self._src
            self._sorted = sorted(src.tolist())
        return self._sorted

    def __getitem__(self, i):
        return self._get()[i]

    def __len__(self) -> int:
        return len(self._src) if isinstance(self._src, SymbolFeatureRows) else int(self._src.size)

    def __eq__(self, other) -> bool:
        return list(self._get()) == list(other)


class SymbolFeatureRows(Mapping):
    """LiveMarketContext.symbol_features as a read-only mapping symbol -> dict
    (the SymbolMarketFeatures fields of market_regime/models.py:53-83 plus the
    micro-regime annotation), backed by the context pass's per-slot row block,
    which stays in HBM (one device copy per context) until first use: then one
    D2H, `.slots` / `.names` / `.arrays` / `.codes` are cut from it, and a
    per-symbol dict is only built when a symbol is looked up. `rows` may also
    be a host array."""

    def __init__(self, all_names: np.ndarray, rows, count: int, timestamp: int):
        self._all_names, self._rows_t, self._count, self.timestamp = all_names, rows, int(count), timestamp
        self._host = self._slots = self._names = self._arrays = self._codes = None
        self._row: dict[str, int] | None = None

    def _block(self) -> np.ndarray:
        if self._host is None:
            r = self._rows_t
            self._host = r.cpu().numpy() if isinstance(r, torch.Tensor) else np.asarray(r)
            self._rows_t = None
        return self._host

    @property
    def slots(self) -> np.ndarray:
        if self._slots is None:
            R = self._block()
            self._slots = np.flatnonzero((R[_R_FRESH] > 0) & ~np.isnan(R[0]))
        return self._slots

    @property
    def names(self) -> np.ndarray:
        if self._names is None:
            self._names = self._all_names[self.slots]
        return self._names

    @property
    def codes(self) -> np.ndarray:   # int8 micro-regime codes (bq_micro_regime)
        if self._codes is None:
            self._codes = self._block()[_R_REG, self.slots].astype(np.int8)
        return self._codes

    @property
    def arrays(self) -> dict[str, np.ndarray]:
        if self._arrays is None:
            sel = self._block()[:, self.slots]
            nf = len(FEATURE_COLUMNS)
            a = dict(zip(FEATURE_COLUMNS, sel[:nf]))
            a.update(close=sel[_R_CLOSE], relative_strength_vs_btc=sel[_R_RS], above_ema20=sel[_R_A20] > 0,
                     above_ema50=sel[_R_A50] > 0, micro_regime=labels(self.codes),
                     micro_regime_strength=sel[_R_REG_S],
                     micro_regime_transition=labels(sel[_R_TR].astype(np.int8), MICRO_TRANSITIONS),
                     micro_regime_transition_strength=sel[_R_TR_S])
            self._arrays = a
        return self._arrays

    def _index(self) -> dict[str, int]:
        if self._row is None:
            self._row = {n: i for i, n in enumerate(self.names.tolist())}
        return self._row

    def __getitem__(self, symbol: str) -> dict:
        i = self._index()[symbol]
        d = {k: (v[i].item() if hasattr(v[i], "item") else v[i]) for k, v in self.arrays.items()}
        d["symbol"] = symbol
        d["timestamp"] = self.timestamp
        return d

    def __iter__(self):
        return iter(self.names.tolist())

    def __len__(self) -> int:
        return self._count


class DeviceMarketStateStore:
    """MarketStateStore with the histories in HBM (one ring per symbol slot)."""

    def __init__(self, max_bars_per_symbol: int = 200, capacity: int = 1024, device=None) -> None:
        if not 2 <= int(max_bars_per_symbol) <= _lib.STORE_MAX_BARS:
            raise ValueError(f"max_bars_per_symbol must be in [2, {_lib.STORE_MAX_BARS}]")
        self.max_bars_per_symbol = int(max_bars_per_symbol)
        self.device = _device(device)
        self._slots: dict[str, int] = {}
        self._names: list[str] = []
        self._alloc(max(1, int(capacity)))

    # -- storage ----------------------------------------------------------------
    def _alloc(self, cap: int, old=None) -> None:
        M, dev = self.max_bars_per_symbol, self.device
        ts = torch.zeros((cap, M), dtype=torch.int64, device=dev)
        f = torch.full((len(INPUT_FIELDS), cap, M), float("nan"), dtype=torch.float64, device=dev)
        head = torch.zeros(cap, dtype=torch.int32, device=dev)
        count = torch.zeros(cap, dtype=torch.int32, device=dev)
        last = torch.zeros(cap, dtype=torch.int64, device=dev)
        if old is not None:
            n = old["ts"].shape[0]
            ts[:n] = old["ts"]
            f[:, :n] = old["f"]
            head[:n] = old["head"]
            count[:n] = old["count"]
            last[:n] = old["last"]
        self._t = dict(ts=ts, f=f, head=head, count=count, last=last)
        self.capacity = cap
        v = _lib.BqStoreView()
        v.ts = ts.data_ptr()
        for c in range(len(INPUT_FIELDS)):
            v.field[c] = f[c].data_ptr()
        v.head, v.count, v.last = head.data_ptr(), count.data_ptr(), last.data_ptr()
        v.capacity, v.max_bars = cap, M
        self._view = v
        # every (re)allocation is a new generation: anything that baked the
        # ring pointers in (the live context's hipGraph) keys on it
        self.generation = getattr(self, "generation", -1) + 1

    def _slot(self, symbol: str) -> int:
        s = self._slots.get(symbol)
        if s is None:
            s = len(self._names)
            if s >= self.capacity:
                self._alloc(2 * self.capacity, old=self._t)
            self._slots[symbol] = s
            self._names.append(symbol)
        return s

    def slot_of(self, symbol: str) -> int | None:
        return self._slots.get(symbol)

    def symbol_of(self, slot: int) -> str:
        return self._names[slot]

    def names_array(self) -> np.ndarray:
        if getattr(self, "_names_np", None) is None or self._names_np.size != len(self._names):
            self._names_np = np.array(self._names, dtype=object)
        return self._names_np

    def slots_for(self, symbols: Sequence[str]) -> torch.Tensor:
        """Device slot ids of `symbols` (registering new ones); cached for a
        repeated symbol list, so a steady feed pays the lookup once."""
        key = tuple(symbols)
        cached = getattr(self, "_slot_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        ids = [self._slot(s) for s in symbols]
        t = torch.tensor(ids, dtype=torch.int64, device=self.device)
        # strictly increasing ids (the symbols in registration order, as a
        # steady feed sends them): one candle per slot, already in merge order
        self._slot_cache = (key, t, all(a < b for a, b in zip(ids, ids[1:])))
        return t

    @property
    def n_tracked(self) -> int:
        return len(self._names)

    # -- batched updates (device) ---------------------------------------------------
    @_on_device
    def update_slots(self, slots: torch.Tensor, ts: torch.Tensor, fields: Sequence[torch.Tensor], stream=None,
                     unique_sorted: bool = False) -> None:
        """One launch for a batch of candles (arrival order; device tensors):
        rows with NaN close are dropped, each (slot, timestamp) keeps its LAST
        row, runs are sorted by timestamp per slot, then merged into the rings.
        ``unique_sorted`` (internal: update_batch over a cached, strictly
        increasing, registered slot list) skips the sorts and the dedupe, which
        are the identity for such a batch."""
        slots = slots.to(self.device, torch.int64).reshape(-1)
        ts = ts.to(self.device, torch.int64).reshape(-1)
        fields = [x.to(self.device, torch.float64).reshape(-1) for x in fields]
        if len(fields) != len(INPUT_FIELDS) or any(x.numel() != slots.numel() for x in fields) or ts.numel() != slots.numel():
            raise ValueError("update_slots: slots, ts and the five OHLCV fields must have one entry per candle")
        if unique_sorted:
            # one candle per slot in slot order: the kernel drops a candle
            # without a close itself (no host round trip)
            if not slots.numel():
                return
            s3, t3, f3 = slots.contiguous(), ts.contiguous(), [x.contiguous() for x in fields]
            n_seg = s3.numel()
            seg = self._arange(n_seg + 1)
        else:
            if slots.numel() and (int(slots.min()) < 0 or int(slots.max()) >= self.n_tracked):
                raise ValueError("update_slots: slot out of range (register symbols first)")
            ok = ~torch.isnan(fields[INPUT_FIELDS.index("close")])
            idx = torch.nonzero(ok).reshape(-1)
            if idx.numel() == 0:
                return
            order = idx[torch.argsort(ts[idx], stable=True)]
            order = order[torch.argsort(slots[order], stable=True)]
            s2, t2 = slots[order], ts[order]
            last_row = torch.ones_like(s2, dtype=torch.bool)
            last_row[:-1] = (s2[1:] != s2[:-1]) | (t2[1:] != t2[:-1])
            sel = order[last_row]
            s3, t3 = slots[sel].contiguous(), ts[sel].contiguous()
            f3 = [x[sel].contiguous() for x in fields]
            _, counts = torch.unique_consecutive(s3, return_counts=True)
            n_seg = counts.numel()
            seg = torch.zeros(n_seg + 1, dtype=torch.int64, device=self.device)
            seg[1:] = torch.cumsum(counts, 0)
        st = _lib.load().bq_store_update(
            ctypes.byref(self._view), ctypes.c_void_p(s3.data_ptr()), ctypes.c_void_p(t3.data_ptr()),
            _lib.ptr_array([x.data_ptr() for x in f3]), ctypes.c_void_p(seg.data_ptr()), n_seg,
            engine._stream_handle(stream),
        )
        _lib.check(st, "bq_store_update")

    def _arange(self, n: int) -> torch.Tensor:
        a = getattr(self, "_arange_buf", None)
        if a is None or a.numel() < n:
            a = self._arange_buf = torch.arange(max(n, 1024), dtype=torch.int64, device=self.device)
        return a[:n]

    def _staging(self, n: int) -> dict:
        """Two pinned host / device staging slots for update_batch: host
        writes go into the slot whose previous H2D copy has completed (its
        event), so a tick never waits on the device and never races a copy."""
        st = getattr(self, "_stage", None)
        if st is None or st[0]["n"] != n:
            st = self._stage = [dict(n=n, hf=torch.empty((len(INPUT_FIELDS), n), dtype=torch.float64).pin_memory(),
                                     ht=torch.empty(n, dtype=torch.int64).pin_memory(),
                                     df=torch.empty((len(INPUT_FIELDS), n), dtype=torch.float64, device=self.device),
                                     dt=torch.empty(n, dtype=torch.int64, device=self.device), ev=None)
                                for _ in range(2)]
            self._stage_i = 0
        self._stage_i ^= 1
        slot = st[self._stage_i]
        if slot["ev"] is not None:
            slot["ev"].synchronize()
        return slot

    @_on_device
    def update_batch(self, symbols: Sequence[str], timestamp, open_, high, low, close, volume) -> None:
        """Many symbols' candles (host arrays, arrival order) in one launch:
        one pinned H2D of the five columns and the timestamps, one
        bq_store_update, no host synchronisation."""
        slots = self.slots_for(symbols)
        n = slots.numel()
        if n == 0:
            return
        st = self._staging(n)
        hf = st["hf"].numpy()
        for i, x in enumerate((open_, high, low, close, volume)):
            hf[i] = x
        st["ht"].numpy()[:] = timestamp
        st["df"].copy_(st["hf"], non_blocking=True)
        st["dt"].copy_(st["ht"], non_blocking=True)
        ev = st["ev"] = st["ev"] or torch.cuda.Event()
        ev.record()
        self.update_slots(slots, st["dt"], list(st["df"]), unique_sorted=self._slot_cache[2])

    # -- reference API ----------------------------------------------------------------
    @_on_device
    def update(self, symbol: str, candle: Mapping[str, Any] | pd.Series | pd.DataFrame) -> pd.DataFrame:
        normalized = normalize_candles(candle)
        s = self._slot(symbol)
        if len(normalized):
            self.update_slots(
                torch.full((len(normalized),), s, dtype=torch.int64),
                torch.from_numpy(normalized["timestamp"].to_numpy(np.int64)),
                [torch.from_numpy(normalized[c].to_numpy(np.float64)) for c in INPUT_FIELDS],
            )
        history = self.get_symbol_history(symbol)
        if history.empty:
            # the reference stores the empty history and then fails on
            # history.iloc[-1] (market_state_store.py:31)
            raise IndexError("MarketStateStore.update: no candle with a timestamp and a close")
        return history

    @_on_device
    def _gather(self, slots: list[int]) -> tuple[np.ndarray, np.ndarray, dict[str, np.ndarray]]:
        M = self.max_bars_per_symbol
        sl = torch.tensor(slots, dtype=torch.int64, device=self.device)
        ts = torch.empty((len(slots), M), dtype=torch.int64, device=self.device)
        outs = [torch.empty((len(slots), M), dtype=torch.float64, device=self.device) for _ in INPUT_FIELDS]
        st = _lib.load().bq_store_gather(
            ctypes.byref(self._view), ctypes.c_void_p(sl.data_ptr()), len(slots), ctypes.c_void_p(ts.data_ptr()),
            _lib.ptr_array([o.data_ptr() for o in outs]), M, engine._stream_handle(None),
        )
        _lib.check(st, "bq_store_gather")
        counts = self._t["count"][sl].cpu().numpy()
        return counts, ts.cpu().numpy(), {c: o.cpu().numpy() for c, o in zip(INPUT_FIELDS, outs)}

    @staticmethod
    def _frame(n: int, ts: np.ndarray, f: dict[str, np.ndarray], r: int) -> pd.DataFrame:
        d = {"timestamp": ts[r, :n].astype(np.int64)}
        for c in INPUT_FIELDS:
            d[c] = f[c][r, :n]
        return pd.DataFrame(d, columns=STORE_COLUMNS)

    def get_symbol_history(self, symbol: str) -> pd.DataFrame:
        s = self._slots.get(symbol)
        if s is None:
            return pd.DataFrame()
        counts, ts, f = self._gather([s])
        return self._frame(int(counts[0]), ts, f, 0)

    def get_all_histories(self) -> dict[str, pd.DataFrame]:
        if not self._names:
            return {}
        counts, ts, f = self._gather(list(range(self.n_tracked)))
        return {name: self._frame(int(counts[i]), ts, f, i) for i, name in enumerate(self._names)}

    def get_last_closed_timestamp(self, symbol: str) -> int | None:
        s = self._slots.get(symbol)
        if s is None or int(self._t["count"][s]) == 0:
            return None
        return int(self._t["last"][s])

    def get_tracked_symbols(self) -> list[str]:
        return sorted(self._names)

    @_on_device
    def fresh_slots(self, timestamp: int) -> torch.Tensor:
        """Slots whose last closed candle is `timestamp` (ascending slot ids, device)."""
        n = self.n_tracked
        m = (self._t["last"][:n] == int(timestamp)) & (self._t["count"][:n] > 0)
        return torch.nonzero(m).reshape(-1)

    def get_fresh_symbols(self, timestamp: int) -> set[str]:
        return {self._names[i] for i in self.fresh_slots(timestamp).cpu().tolist()}

    # -- features ---------------------------------------------------------------------------
    @_on_device
    def features(self, slots: torch.Tensor, stream=None) -> tuple[dict[str, torch.Tensor], torch.Tensor]:
        """_compute_symbol_features of each slot's history (NaN rows where the
        reference returns None). Returns ({feature: [n]}, latest close [n])."""
        slots = slots.to(self.device, torch.int64).contiguous()
        n = slots.numel()
        feats = {k: torch.empty(n, dtype=torch.float64, device=self.device) for k in FEATURE_COLUMNS}
        close = torch.empty(n, dtype=torch.float64, device=self.device)
        st = _lib.load().bq_store_features(
            ctypes.byref(self._view), ctypes.c_void_p(slots.data_ptr()), n,
            _lib.ptr_array([feats[k].data_ptr() for k in FEATURE_COLUMNS]), ctypes.c_void_p(close.data_ptr()),
            engine._stream_handle(stream),
        )
        _lib.check(st, "bq_store_features")
        return feats, close


class DeviceLiveMarketContextAccumulator:
    """LiveMarketContextAccumulator over a DeviceMarketStateStore.

    With torch.distributed initialised and a symbol-sharded store per rank
    (the benchmark symbol replicated on every rank), the per-timestamp
    partial sums and the tracked / fresh counts are all-reduced in ONE call
    (12 doubles); every rank then scores the same context.
    """

    def __init__(self, state_store: DeviceMarketStateStore, btc_symbol: str, group=None) -> None:
        self.state_store = state_store
        self.btc_symbol = btc_symbol
        self.group = group
        self._contexts_by_timestamp: dict[int, dict] = {}
        self._context_order: deque[int] = deque(maxlen=64)
        self._regimes: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}

    # -- reference API ------------------------------------------------------------------
    @_on_device
    def on_closed_candle(self, symbol: str, candle) -> dict | None:
        history = self.state_store.update(symbol=symbol, candle=candle)
        return self.refresh_context_for_timestamp(int(history.iloc[-1]["timestamp"]))

    @_on_device
    def on_closed_candles(self, symbols: Sequence[str], timestamp, open_, high, low, close, volume,
                          at: int | None = None) -> dict | None:
        """A whole tick in one device update, then one context build (at the
        tick's latest timestamp unless `at` is given)."""
        self.state_store.update_batch(symbols, timestamp, open_, high, low, close, volume)
        ts = int(np.max(np.asarray(timestamp))) if at is None else int(at)
        return self.refresh_context_for_timestamp(ts)

    def get_context(self, timestamp: int) -> dict | None:
        return self._contexts_by_timestamp.get(timestamp)

    def get_latest_context(self) -> dict | None:
        while self._context_order:
            ts = self._context_order[-1]
            ctx = self._contexts_by_timestamp.get(ts)
            if ctx is not None:
                return ctx
            self._context_order.pop()
        return None

    @_on_device
    def refresh_context_for_timestamp(self, timestamp: int) -> dict | None:
        context = self._build_context(int(timestamp))
        if context is None:
            return None
        self._contexts_by_timestamp[int(timestamp)] = context
        if int(timestamp) not in self._context_order:
            self._context_order.append(int(timestamp))
        return context

    def _get_previous_context(self, timestamp: int) -> dict | None:
        for known in reversed(self._context_order):
            if known >= timestamp:
                continue
            ctx = self._contexts_by_timestamp.get(known)
            if ctx is not None:
                return ctx
        return None

    # -- the build --------------------------------------------------------------------------
    def _sharded(self) -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def _bufs(self) -> "_ContextBuffers":
        """Persistent device / pinned buffers of the context pass for the
        store's current shape (re-made when symbols are registered or the
        rings are re-allocated, which also drops a captured graph)."""
        store = self.state_store
        btc_slot = store.slot_of(self.btc_symbol)
        btc_counted = btc_slot is not None and (not self._sharded() or dist.get_rank(self.group) == 0)
        key = (store.n_tracked, store.generation, btc_slot, btc_counted)
        b = getattr(self, "_ctx_bufs", None)
        if b is None or b.key != key:
            tracked = store.n_tracked - (0 if btc_counted or btc_slot is None else 1)
            b = _ContextBuffers(key, store.n_tracked, btc_slot, btc_counted, tracked, store.device)
            self._ctx_bufs = b
        return b

    def _device_pass(self, b: "_ContextBuffers") -> None:
        """Everything of one context build that runs on the device, with no
        host synchronisation (so it can be captured and replayed as one
        hipGraph): fresh mask + features of every tracked slot
        (bq_store_context_features), the breadth partial over the fresh rows
        (bq_breadth_partial, T = 1), the fresh count, relative strength vs
        the benchmark, above-EMA flags, the micro regime with the previous
        context's regimes by slot (bq_micro_regime), and one pinned D2H of the
        per-symbol rows. The timestamp is read from b.ts (device)."""
        store = self.state_store
        n = b.n
        F = b.feat
        st = _lib.load().bq_store_context_features(
            ctypes.byref(store._view), n, ctypes.c_void_p(b.ts.data_ptr()),
            -1 if b.btc_slot is None else int(b.btc_slot), int(b.btc_counted),
            _lib.ptr_array([F[i].data_ptr() for i in range(len(FEATURE_COLUMNS))]),
            ctypes.c_void_p(b.close.data_ptr()), ctypes.c_void_p(b.fresh.data_ptr()),
            ctypes.c_void_p(b.small[_BTC0:].data_ptr()), engine._stream_handle(None))
        _lib.check(st, "bq_store_context_features")
        npart = len(_lib.PARTIAL_COLUMNS)
        fz = {k: F[i].view(n, 1) for i, k in enumerate(FEATURE_COLUMNS)}
        engine.breadth_partial(b.close.view(n, 1), fz, out=b.small[:npart].view(1, npart))
        torch.sum(b.fresh, 0, keepdim=True, out=b.small[npart : npart + 1])
        ret, e20, e50 = F[0], F[1], F[2]
        btc_ret = b.small[_BTC0 : _BTC0 + 1]
        btc_ok = btc_ret == btc_ret
        rs = torch.where(btc_ok, ret - btc_ret, torch.zeros_like(ret))
        if b.btc_slot is not None:
            rs.narrow(0, b.btc_slot, 1).fill_(0.0)   # the benchmark's own relative strength stays 0 (:117-123)
        a20, a50 = b.close > e20, b.close > e50
        ann = micro_regime(F[3], a20, a50, rs, F[5], F[4], ret, prev_regime=b.prev_code,
                           prev_strength=b.prev_strength, device=store.device)
        rows = b.rows
        rows[: len(FEATURE_COLUMNS)].copy_(F)
        rows[_R_CLOSE].copy_(b.close)
        rows[_R_RS].copy_(rs)
        rows[_R_A20].copy_(a20)
        rows[_R_A50].copy_(a50)
        rows[_R_REG].copy_(ann["micro_regime"])
        rows[_R_REG_S].copy_(ann["micro_regime_strength"])
        rows[_R_TR].copy_(ann["micro_regime_transition"])
        rows[_R_TR_S].copy_(ann["micro_regime_transition_strength"])
        rows[_R_FRESH].copy_(b.fresh)
        listed = (b.fresh > 0) & (ret == ret)   # the rows of symbol_features
        torch.where(listed, ann["micro_regime"], torch.full_like(ann["micro_regime"], -1), out=b.code)
        b.strength.copy_(ann["micro_regime_strength"])
        torch.sum(listed, 0, keepdim=True, dtype=torch.float64, out=b.small[_N_LISTED : _N_LISTED + 1])

    def _build_context(self, timestamp: int) -> dict | None:
        store = self.state_store
        b = self._bufs()
        n = b.n
        previous = self._get_previous_context(timestamp)
        prev = self._regimes.get(previous["timestamp"]) if previous is not None else None
        b.set_previous(prev)
        b.ts_host[0] = int(timestamp)
        b.ts.copy_(b.ts_host, non_blocking=True)
        sharded = self._sharded()
        if n and not sharded and _GRAPHS:
            b.run(lambda: self._device_pass(b))
        elif n:
            self._device_pass(b)
        small = b.small
        if sharded:
            # reduce a copy: b.small keeps this rank's tracked count for the next build
            small = small.clone()
            npart = len(_lib.PARTIAL_COLUMNS)
            red = small[: npart + 2]
            if dist.get_backend(self.group) == "gloo":   # CPU rehearsal of the sharded path
                red_c = red.cpu()
                dist.all_reduce(red_c, op=dist.ReduceOp.SUM, group=self.group)
                red.copy_(red_c)
            else:   # RCCL over xGMI: one all-reduce of 12 doubles
                dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group)
        b.small_host.copy_(small, non_blocking=True)
        rows_dev = b.rows.clone()   # this context's row block stays in HBM (read on access)
        torch.cuda.current_stream(store.device).synchronize()
        red_h = b.small_host.numpy()
        npart = len(_lib.PARTIAL_COLUMNS)
        total_fresh, total_tracked = int(red_h[npart]), int(red_h[npart + 1])
        required = max(REQUIRED_FRESH_SYMBOLS, ceil(total_tracked * MIN_COVERAGE_RATIO))
        if total_fresh < required:
            return None
        btc_ret = float(red_h[_BTC0]) if b.btc_slot is not None else float("nan")
        btc_trend = float(red_h[_BTC0 + 3]) if b.btc_slot is not None else float("nan")
        btc_valid = not np.isnan(btc_ret)
        btc_fresh = b.btc_slot is not None and bool(red_h[_BTC0 + 7] > 0)
        batch = score_contexts(
            red_h[None, :npart], np.array([btc_ret if btc_valid else 0.0]),
            np.array([btc_trend if btc_valid else 0.0]), np.array([btc_valid]), total_tracked=total_tracked,
            fresh_count=np.array([total_fresh]), timestamps=np.array([timestamp]),
        )
        batch = annotate_market(batch, previous)
        ctx = batch.context_at(0)
        if ctx is None:
            return None
        ctx["btc_symbol"] = self.btc_symbol
        ctx["confidence"] = 1.0
        ctx["is_provisional"] = False
        # this rank's counted fresh symbols with features: per-symbol rows with
        # relative strength + micro regime (regime_transitions.py:162-232),
        # cut from the row block on access
        sym = SymbolFeatureRows(store.names_array(), rows_dev, int(red_h[_N_LISTED]), int(timestamp))
        ctx["symbol_features"] = sym
        ctx["metadata"] = {
            "btc_fresh": btc_fresh,
            "btc_used_for_regime": btc_valid,
            "fresh_symbols": SortedNames(sym),
            "fresh_symbol_count": int(ctx["fresh_count"]),
        }
        # this context's micro regimes by slot (-1 outside its symbol_features),
        # for the next context's transitions
        self._regimes[int(timestamp)] = (b.code.clone(), b.strength.clone())
        keep = set(self._context_order) | {int(timestamp)}
        for t in [t for t in self._regimes if t not in keep]:
            del self._regimes[t]
        return ctx


# rows of the per-symbol D2H block (_ContextBuffers.rows)
_R_CLOSE, _R_RS, _R_A20, _R_A50, _R_REG, _R_REG_S, _R_TR, _R_TR_S, _R_FRESH = range(6, 15)
_N_ROWS = 15
# small buffer: [10 partials, fresh, tracked, 8 benchmark values, rows listed in symbol_features]
_BTC0 = len(_lib.PARTIAL_COLUMNS) + 2
_N_LISTED = _BTC0 + 8
_GRAPHS = __import__("os").environ.get("BQ_STORE_GRAPH", "1") != "0"


class _ContextBuffers:
    """Fixed-address buffers of one store shape (n tracked slots) for the
    context pass, and its captured hipGraph (built on the second build of the
    same shape: the first runs eagerly and warms the allocator and caches)."""

    def __init__(self, key, n: int, btc_slot, btc_counted: bool, tracked: int, dev) -> None:
        f64 = dict(dtype=torch.float64, device=dev)
        self.key, self.n, self.btc_slot, self.btc_counted = key, n, btc_slot, btc_counted
        self.ts = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ts_host = torch.zeros(1, dtype=torch.int64).pin_memory()
        self.feat = torch.empty((len(FEATURE_COLUMNS), max(n, 1)), **f64)[:, :n]
        self.close = torch.empty(n, **f64)
        self.fresh = torch.empty(n, **f64)
        self.small = torch.full((_N_LISTED + 1,), float("nan"), **f64)
        self.small[: _BTC0].zero_()
        self.small[_BTC0 - 1] = float(tracked)
        self.small[_N_LISTED] = 0.0
        self.small_host = torch.zeros(_N_LISTED + 1, dtype=torch.float64).pin_memory()
        self.prev_code = torch.full((n,), -1, dtype=torch.int8, device=dev)
        self.prev_strength = torch.zeros(n, **f64)
        self.code = torch.full((n,), -1, dtype=torch.int8, device=dev)
        self.strength = torch.zeros(n, **f64)
        self.rows = torch.empty((_N_ROWS, n), **f64)
        self.graph = None
        self.runs = 0

    def set_previous(self, prev) -> None:
        """Copy the previous context's regimes (by slot) into the fixed
        buffers the pass reads; -1 / 0 for slots it did not have."""
        if prev is None:
            self.prev_code.fill_(-1)
            self.prev_strength.zero_()
            return
        code, strength = prev
        m = min(self.n, code.numel())
        self.prev_code[:m].copy_(code[:m])
        self.prev_strength[:m].copy_(strength[:m])
        if m < self.n:
            self.prev_code[m:].fill_(-1)
            self.prev_strength[m:].zero_()

    def run(self, fn) -> None:
        self.runs += 1
        if self.graph is not None:
            self.graph.replay()
            return
        if self.runs < 2:
            fn()
            return
        s = torch.cuda.Stream(device=self.ts.device)
        s.wait_stream(torch.cuda.current_stream(self.ts.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            fn()   # warm-up on the capture stream
            s.synchronize()
            g.capture_begin()
            try:
                fn()
            finally:
                g.capture_end()
        torch.cuda.current_stream(self.ts.device).wait_stream(s)
        self.graph = g
        g.replay()
