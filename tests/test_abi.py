"""CPU checks of the drop-in boundary: the C-ABI library loads and exports
every entry point include/binquant_amd.h declares (no compute without a GPU)."""

import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(bq_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ("bq_enrich", "bq_tick", "bq_state_create", "bq_state_seed", "bq_market_features", "bq_breadth_partial"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from binquant_amd import _lib

    lib = _lib.load()
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, f"symbols declared in include/*.h but not exported: {missing}"
    # the ctypes signature table covers exactly the header
    assert set(_lib.SIGNATURES) == declared_functions()


def test_default_params_match_reference_windows():
    from binquant_amd import _lib

    p = _lib.default_params()
    assert list(p.ma_periods) == [7, 25, 100]          # context_evaluator.py:249-251
    assert (p.macd_fast, p.macd_slow, p.macd_signal) == (12, 26, 9)
    assert p.rsi_window == 14 and p.atr_window == 14    # :255, :261
    assert p.bb_window == 20 and p.bb_k == 2.0
    assert list(p.ema_spans) == [20, 50]                # live_market_context_accumulator.py:266-267
    assert _lib.load().bq_version().startswith(b"binquant_amd")


def test_invalid_arguments_rejected_without_device():
    from binquant_amd import _lib

    lib = _lib.load()
    null = ctypes.c_void_p()
    # null pointer tables are rejected before any HIP call
    assert lib.bq_enrich(None, 1, 1, 1, None, None, 1, null) == _lib.BQ_EINVAL
    assert lib.bq_market_features(None, 1, 1, 1, 400, None, 1, null) == _lib.BQ_EINVAL
    assert lib.bq_breadth_partial(None, None, 1, 1, 1, 1, None, null) == _lib.BQ_EINVAL
    assert lib.bq_tick(None, None, None, null) == _lib.BQ_ESTATE
    h = ctypes.c_void_p()
    assert lib.bq_state_create(ctypes.byref(h), 0, None) == _lib.BQ_EINVAL


def test_roll_job_rows_validated_without_device():
    """bq_roll_job.rows: a job's own row count must lie in [0, S], and only the
    lane-per-row kernels (moments, ewm, ffill) take one below S — the
    validation runs before any HIP call (fake, never dereferenced pointers)."""
    from binquant_amd import _lib

    lib = _lib.load()
    null = ctypes.c_void_p()
    assert ctypes.sizeof(_lib.BqRollJob) == 80   # the header's bq_roll_job (rows, panel, reserved)

    def job(mode, rows, **kw):
        j = _lib.BqRollJob()
        j.x, j.out, j.ld_in, j.ld_out = 0x1000, 0x2000, 100, 100
        j.window, j.min_periods, j.mode, j.rows = 5, 5, mode, rows
        for k, v in kw.items():
            setattr(j, k, v)
        return j

    def call(*jobs, S=8):
        arr = (_lib.BqRollJob * len(jobs))(*jobs)
        return lib.bq_rolling_batch(arr, len(jobs), S, 100, null)

    median = _lib.ROLL_MODES["median"]
    assert call(job(median, 3)) == _lib.BQ_EINVAL                     # order statistics: all S rows
    assert call(job(_lib.ROLL_MODES["isum"], 3)) == _lib.BQ_EINVAL
    assert call(job(_lib.ROLL_MODES["mean"], 9)) == _lib.BQ_EINVAL     # rows > S
    assert call(job(_lib.ROLL_MODES["mean"], -1)) == _lib.BQ_EINVAL
    assert call(job(_lib.ROLL_EWM, 1, alpha=0.0)) == _lib.BQ_EINVAL    # alpha still checked


def test_missing_library_fails_loudly(tmp_path):
    from binquant_amd import _lib

    with pytest.raises(_lib.NativeLibraryError):
        _lib.load(tmp_path / "nope.so")
