"""Benchmark: symbol-candles/s for the full 14-column indicator set on MI355X.

Headline workload: BASELINE.json configs[3] — 100 000 symbols x 10 000 candles
of synthetic fp64 OHLCV resident in HBM, sharded by symbol over the N ranks
(contiguous blocks, market_regime.batch.shard_bounds). At N = 1 the whole
100k x 10k panel sits on one GPU (5 inputs = 40 GB + 14 outputs = 112 GB of
288 GB); at N = 8 each GPU holds the 12 500-symbol C4 shard. Total work is
fixed as N grows ("scaling": "strong"). One step = one bq_enrich launch over
the rank's shard (reads 5 inputs, writes 14 columns). Ranks share no data
(symbols are independent); the only collective is the MAX of the timings.

Also reported (same JSON line):
  roofline     — algorithmic bytes (152 B/candle) / mean enrich_kernel time
                 (HIP events on the launch stream) vs 8 TB/s HBM peak; traffic
                 from the committed rocprofv3 PMC summary of this workload;
  shard        — the fixed 12 500 x 10 000 C4 shard per GPU (weak-scaling
                 figure, same kernel);
  cpu_baseline — the oracle's pandas per-symbol path in the reference's call
                 pattern at C1 (500-candle frame: indicators_enrichment +
                 _compute_symbol_features per symbol) over a
                 process pool sized to the host's CPU share, rank 0 at every
                 N (after the timed legs), time-bounded sample;
  tick         — C3: 10k symbols, one candle per tick, H2D + bq_tick + D2H
                 latency p50/p99;
  breadth      — C5 (configs[4]) end to end: market_context_batch = the fused
                 panel context build (bq_context_partials: features reduced
                 straight into the [T x 10] partials) + ONE all-reduce of the
                 partials (tracked count folded in) + host scoring and regime
                 annotation of all T contexts; the kernel's roofline on
                 24 B/candle, the reduction and scoring times, the unfused pair
                 timed beside it;
  rows         — every other SURVEY §8 row on the device at 12 500 x 2 000
                 (HIP-event time per call, algorithmic bytes -> GB/s and
                 fraction of HBM peak) with a bounded CPU timing of the
                 oracle's per-symbol path where the oracle restates the row;
  store        — §8f row 1: device MarketStateStore + live context at 10k
                 symbols x 400-bar histories, per-tick latency p50/p99;
  cohort       — one message cohort end to end (process_data for 1000
                 symbols' 5m + 15m frames + the context refresh), eager and as
                 one hipGraph, beside the reference's per-symbol cost x S.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

import numpy as np
import pandas as pd
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from binquant_amd import engine  # noqa: E402
from binquant_amd._lib import ENRICH_COLUMNS  # noqa: E402
from binquant_amd.market_regime.batch import reduce_partials, shard_bounds  # noqa: E402
from binquant_amd.synth import device_panel  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_CANDLE = 8 * (5 + len(ENRICH_COLUMNS))   # 5 inputs read + 14 columns written = 152 B


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--symbols", type=int, default=100_000, help="total symbols, sharded over the ranks")
    ap.add_argument("--candles", type=int, default=10_000)
    ap.add_argument("--shard-symbols", type=int, default=12_500, help="per-GPU symbols of the weak-scaling leg")
    ap.add_argument("--shard-steps", type=int, default=10)
    ap.add_argument("--no-shard", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-workers", type=int, default=0, help="0: the host's CPU share (see host_cores)")
    ap.add_argument("--cpu-candles", type=int, default=500, help="C1 frame length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tick-symbols", type=int, default=10_000)
    ap.add_argument("--ticks", type=int, default=2000)
    ap.add_argument("--no-tick", action="store_true")
    ap.add_argument("--no-breadth", action="store_true")
    ap.add_argument("--breadth-steps", type=int, default=3)
    ap.add_argument("--no-rows", action="store_true")
    ap.add_argument("--row-symbols", type=int, default=12_500)
    ap.add_argument("--row-candles", type=int, default=2_000)
    ap.add_argument("--store-ticks", type=int, default=300)
    ap.add_argument("--live-symbols", type=int, default=1000)
    return ap.parse_args()


def launch_ranks(args) -> int | None:
    """`bench.py --gpus N` run by itself (no WORLD_SIZE in the environment,
    N > 1): start N fresh child interpreters of this script, one per GPU
    (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1 at a free
    port), poll them and return 0 when all succeed; rank 0 prints the JSON
    line. The first rank to exit non-zero ends the run: the others (which
    would otherwise wait in the rendezvous or a collective for the missing
    rank) are terminated and that rank's code is returned. Called before
    anything touches the GPU in this process (the children are new
    processes, not an exec of this one). Returns None when this process is
    itself a rank."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for i in range(args.gpus):
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            print(f"bench.py: a rank exited with code {bad[0]}; the other ranks were stopped", file=sys.stderr)
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def setup_dist(args):
    """One process per GPU, RCCL ("nccl") over xGMI. BQ_BENCH_BACKEND=gloo
    rehearses the multi-rank path on fewer GPUs (ranks share devices round-robin,
    collectives over gloo on host copies): same sharding, same single
    all-reduce per breadth build, same timing reduction."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s); "
                         "run `bench.py --gpus N` alone (it starts N ranks) or under "
                         "torch.distributed.run --nproc-per-node N")
    fail = os.environ.get("BQ_BENCH_FAIL_RANK", "")   # test hook: "rank:code" exits that rank at start-up
    if fail and int(fail.split(":")[0]) == rank:
        raise SystemExit(int(fail.split(":")[1]))
    backend = os.environ.get("BQ_BENCH_BACKEND", "nccl")
    timeout = timedelta(seconds=float(os.environ.get("BQ_BENCH_PG_TIMEOUT", "600")))
    if backend == "gloo":
        # rendezvous first: a rank that never arrives leaves the others in
        # init_process_group, before any device call (launch_ranks stops them)
        if world > 1:
            dist.init_process_group("gloo", timeout=timeout)
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        return world, rank, local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _cpu_worker(args):
    """One host process: the reference's per-message call pattern at C1 — one
    pandas frame per symbol through indicators_enrichment
    (producers/context_evaluator.py:240-263, oracle restatement) plus
    _compute_symbol_features on the store's last 400 bars
    (market_regime/live_market_context_accumulator.py:244-297) — until the
    time budget ends."""
    seed, T, budget = args
    import pandas as pd

    from binquant_amd.synth import numpy_symbol
    from oracle import indicators_ref as ref
    from oracle import market_ref

    done, spent, s = 0, 0.0, 0
    while spent < budget:
        sym = numpy_symbol(T, seed * 100_000 + s, scale=100.0)
        df = pd.DataFrame(sym)
        t0 = time.perf_counter()
        ref.indicators_enrichment(df)
        market_ref.symbol_features(sym["high"][-400:], sym["low"][-400:], sym["close"][-400:])
        spent += time.perf_counter() - t0
        done += T
        s += 1
    return done, spent, s


def host_cores() -> dict:
    """The host CPU share this process may use: the cgroup CPU quota when one
    is set, else the scheduler affinity mask; os.cpu_count() (the whole
    machine) is reported beside it. On the GPU pool the box's share is also
    published as OMP_NUM_THREADS, which caps the count when present."""
    total = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    share = quota if quota is not None else affinity
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        share = min(share, int(omp))
    return {"os_cpu_count": total, "affinity": affinity, "cgroup_quota": quota,
            "omp_num_threads": int(omp) if omp.isdigit() else None, "share": max(1, share)}


def cpu_model() -> str | None:
    """The host CPU's model name (/proc/cpuinfo), e.g. for BASELINE.md's plan."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(args):
    import multiprocessing as mp

    cores = host_cores()
    workers = args.cpu_workers if args.cpu_workers > 0 else cores["share"]
    T = args.cpu_candles
    # single core, alone on the host (before the pool): the same call pattern in this process
    sc_done, sc_spent, sc_syms = _cpu_worker((999, T, min(4.0, args.cpu_seconds)))
    ctx = mp.get_context("spawn")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, [(i, T, args.cpu_seconds) for i in range(workers)])
    wall = time.perf_counter() - t0
    candles = sum(r[0] for r in res)
    busy = max(r[1] for r in res)
    syms = sum(r[2] for r in res)
    return {
        "value": candles / busy,
        "unit": "symbol-candles/s",
        "cores": workers,
        "kind": "port",
        "cpu_model": cpu_model(),
        "single_core": {"value": sc_done / sc_spent, "unit": "symbol-candles/s", "cores": 1,
                        "sample": f"{sc_syms} symbols x {T}-candle frames, one process alone on the host"},
        "host": cores,
        "sample": f"C1: {syms} symbols x {T}-candle frames, per symbol pandas indicators_enrichment (14 columns) "
        f"+ _compute_symbol_features on the last 400 bars (oracle restatement of the reference call pattern), "
        f"{workers} processes x ~{args.cpu_seconds:.0f}s (wall {wall:.1f}s)",
    }


def pmc_entry(kernel: str, candles: int) -> dict:
    """The committed rocprofv3 PMC summary of this workload
    (profiles/pmc_traffic.json); empty when it was taken on another panel
    size (the source tag is kept)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f).get(kernel, {})
    except (OSError, ValueError):
        return {}
    if d.get("candles_per_launch") != candles:
        return {"source": d.get("source")}
    return d


def pmc_traffic(kernel: str, candles: int):
    """HBM bytes per launch from the committed PMC summary (pmc_entry); null
    when the summary was taken on another panel size."""
    d = pmc_entry(kernel, candles)
    return d.get("bytes_per_launch"), d.get("source")


def bench_tick(args, dev):
    S = args.tick_symbols
    hist = device_panel(S, 400, device=dev, seed=7)
    st = engine.TickState(S)
    st.seed(hist["open"], hist["high"], hist["low"], hist["close"], hist["volume"])
    rng = np.random.default_rng(0)
    host_in = torch.empty((5, S), dtype=torch.float64).pin_memory()
    dev_in = torch.empty((5, S), dtype=torch.float64, device=dev)
    outs = {k: torch.empty(S, dtype=torch.float64, device=dev) for k in ENRICH_COLUMNS}
    host_out = torch.empty((len(ENRICH_COLUMNS), S), dtype=torch.float64).pin_memory()
    dev_out = torch.empty((len(ENRICH_COLUMNS), S), dtype=torch.float64, device=dev)
    outs = {k: dev_out[i] for i, k in enumerate(ENRICH_COLUMNS)}
    last = hist["close"][:, -1].cpu().numpy()
    lat = []
    n = args.ticks
    for i in range(n + 50):
        c = last * np.exp(rng.normal(0, 0.002, S))
        o = last
        hi = np.maximum(o, c) * 1.001
        lo = np.minimum(o, c) * 0.999
        v = rng.lognormal(3, 1, S)
        host_in.numpy()[:] = np.stack([o, hi, lo, c, v])
        last = c
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev_in.copy_(host_in, non_blocking=True)
        st.tick([dev_in[j] for j in range(5)], out=outs)
        host_out.copy_(dev_out, non_blocking=True)
        torch.cuda.synchronize()
        if i >= 50:
            lat.append(time.perf_counter() - t0)
    lat = np.array(lat) * 1e3
    return {
        "symbols": S,
        "ticks": n,
        "p50_ms": float(np.percentile(lat, 50)),
        "p99_ms": float(np.percentile(lat, 99)),
        "max_ms": float(lat.max()),
        "includes": "H2D 5xS fp64 (pinned) + bq_tick + D2H 14xS fp64, synchronized",
    }


CONTEXT_BYTES_PER_CANDLE = 3 * 8   # C5: high, low, close read once; the [T x 10] partials are O(T)


def bench_breadth(args, panel, world, dev):
    """C5 (BASELINE configs[4]): breadth / context SCORING at every timestamp
    of the shard, end to end through the product API
    market_regime.batch.market_context_batch(keep_features=False):
    bq_context_partials (features reduced straight into the [T x 10]
    partials, the feature columns never written) -> ONE all-reduce(sum) of
    the partials (tracked-symbol count folded into the spare column;
    reduce_partials, RCCL over xGMI at N > 1) -> the benchmark's feature row
    -> D2H of the partials -> host scoring (score_contexts) and market-regime
    annotation (annotate_market) of all T contexts. Roofline on the kernel's
    algorithmic bytes: 3 fp64 inputs per candle (the group records the
    kernel's passes exchange are intermediate); the unfused features +
    breadth_partial pair is timed beside it."""
    from binquant_amd.market_regime.batch import contexts_from_partials, market_context_batch

    h, l, c = panel["high"], panel["low"], panel["close"]
    S, T = c.shape
    btc_hlc = (h[:1], l[:1], c[:1])   # the benchmark row (replicated on every rank)
    tss = 1_700_000_000_000 + 900_000 * np.arange(T, dtype=np.int64)
    part, _ = engine.context_partials(h, l, c, max_bars=400)
    steps = max(1, args.breadth_steps)
    stream = torch.cuda.current_stream()
    # (1) the kernel alone, HIP events on its stream (the roofline)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    barrier(world)
    for i in range(steps):
        evs[i][0].record(stream)
        engine.context_partials(h, l, c, max_bars=400, out=part)
        evs[i][1].record(stream)
    barrier(world)
    kern_ms = max_over_ranks(float(np.mean([a.elapsed_time(b) for a, b in evs])), world)
    achieved = S * T * CONTEXT_BYTES_PER_CANDLE / (kern_ms * 1e-3) / 1e9
    # (2) the whole C5 step: partials + all-reduce + scoring + annotation of T contexts
    market_context_batch(h, l, c, btc_hlc, timestamps=tss, keep_features=False)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        res = market_context_batch(h, l, c, btc_hlc, timestamps=tss, keep_features=False)
    barrier(world)
    dt = max_over_ranks(time.perf_counter() - t0, world) / steps
    n_total = int(res.contexts.fields["total_tracked_symbols"][-1]) if res.contexts.valid.any() else S * world
    # the parts: the reduction alone, and host scoring + annotation (from the reduced partials on the host)
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(steps):
        _, n_red = reduce_partials(part, S)
    barrier(world)
    reduce_ms = max_over_ranks(time.perf_counter() - t0, world) / steps * 1e3
    ph = res.partial.cpu().numpy()
    bret = np.zeros(T)
    t0 = time.perf_counter()
    for _ in range(steps):
        contexts_from_partials(ph, bret, bret, total_tracked=n_red, timestamps=tss)
    scoring_ms = (time.perf_counter() - t0) / steps * 1e3
    # the unfused pair (what round 2 ran): features written, re-read by breadth_partial
    feats = engine.market_features(h, l, c, max_bars=400)
    up = engine.breadth_partial(c, feats)
    unfused_ms = _time_call(lambda: (engine.market_features(h, l, c, max_bars=400, out=feats),
                                     engine.breadth_partial(c, feats, out=up)), reps=2)
    del feats, up
    # traffic / VALU from the committed PMC of all three passes per call at
    # this shape (tools/row_profile.sh context + tools/context_traffic.py)
    pe = pmc_entry("context_partials", S * T)
    traffic, traffic_src = pe.get("bytes_per_launch"), pe.get("source")
    return {
        "value": n_total * T / dt,
        "unit": "symbol-candles/s",
        "ms_per_step": dt * 1e3,
        "kernel_ms": kern_ms,
        "reduce_ms": reduce_ms,
        "scoring_ms": scoring_ms,
        "contexts": T,
        "valid_contexts": int(res.contexts.valid.sum()),
        "tracked_symbols": n_total,
        "workload": f"{S} symbols x {T} candles per GPU, max_bars 400: market_context_batch(keep_features=False) = "
                    f"fused features -> [T x 10] partials, "
                    + ("one RCCL all_reduce, " if world > 1 else "")
                    + "benchmark features, D2H, score_contexts + annotate_market of all T contexts",
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_scope": pe.get("scope"),
                     "traffic_by_pass": {k: v.get("traffic_bytes") for k, v in (pe.get("kernels") or {}).items()},
                     "kernel": "bq_context_partials (passes 1 + 2 + 3)", "kernel_ms": kern_ms,
                     "algorithmic_bytes_per_candle": CONTEXT_BYTES_PER_CANDLE, "candles_per_launch": S * T,
                     # pass 1 is bound by its instruction stream as much as by HBM
                     "valu": {k: v for k, v in (pe.get("valu") or {}).items()
                              if k in ("kernel", "valu_lane_ops_per_candle", "valu_busy_est", "valu_active_share")}
                     or None},
        "unfused_ms": unfused_ms,
    }


def _time_call(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def output_bytes(res) -> int:
    """Bytes of every tensor a call returns (dicts, tuples, lists walked)."""
    if isinstance(res, torch.Tensor):
        return res.numel() * res.element_size()
    if isinstance(res, dict):
        return sum(output_bytes(v) for v in res.values())
    if isinstance(res, (tuple, list)):
        return sum(output_bytes(v) for v in res)
    return 0


def _cpu_rate(fn, candles_per_call, budget=1.0):
    """Candles/s of a single-core oracle call pattern, time-bounded."""
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget:
        fn()
        n += 1
    return n * candles_per_call / (time.perf_counter() - t0)


def bench_rows(args, dev):
    """Per-row device timings (SURVEY §8a/§8f rows beyond the headline)."""
    import pandas as pd

    from binquant_amd import signals, strategies
    from binquant_amd.synth import numpy_symbol
    from oracle import frame_ref, indicators_ref, market_ref

    S, T = args.row_symbols, args.row_candles
    p = device_panel(S, T, device=dev, seed=99)
    o, h, l, c, v = (p[k] for k in ("open", "high", "low", "close", "volume"))
    qv = v * c
    btc = c[0].clone()
    ts = (1_700_000_000_000 + 900_000 * torch.arange(T, device=dev, dtype=torch.int64)).expand(S, T).contiguous()
    agg = {"open": "first", "high": "max", "low": "min", "close": "last", "volume": "sum"}
    # name -> (device call, input bytes read per candle, row reference). The
    # algorithmic bytes are those inputs read once plus every output the call
    # returns written once at its dtype (bool columns 1 B, [S] / [T] results
    # counted too): output_bytes() of the call's own result.
    rows = {
        "a11_beta_corr": (lambda: engine.beta_corr(c, btc, 50), 8, "producers/context_evaluator.py:154-194"),
        "a13_market_features": (lambda: engine.market_features(h, l, c, max_bars=400), 24,
                                "live_market_context_accumulator.py:244-297"),
        "a17_activity_burst": (lambda: strategies.activity_burst_features(o, h, l, c, v, qv), 48,
                               "strategies/activity_burst_pump.py:51-158"),
        "a18_pump_score": (lambda: strategies.pump_score_features(o, h, l, c, v, btc), 32,
                           "strategies/liquidation_sweep_pump.py:195-269"),
        "a19_failed_spike": (lambda: strategies.failed_spike_features(o, h, l, c, v, qv), 48,
                             "strategies/failed_spike_fade.py:260-544"),
        "a20_wilder_rsi": (lambda: signals.wilder_rsi(c), 8, "strategies/mean_reversion_fade.py:88-109"),
        "a20_adx": (lambda: signals.adx(h, l, c), 24, "strategies/range_bb_rsi_mean_reversion.py:101-122"),
        "a20_zscore": (lambda: signals.zscore(c), 8, "strategies/range_bb_rsi_mean_reversion.py:124-138"),
        "a20_leadership": (lambda: signals.gradual_gainer_leadership(ts, c, ts[0], btc), 16,
                           "strategies/gradual_gainer_retest.py:131-196"),
        "supertrend": (lambda: engine.supertrend(h, l, c, exact=False), 24, "strategies/coinrule/coinrule.py:143"),
        "a9_resample_1h": (lambda: engine.resample(ts, {"open": o, "high": h, "low": l, "close": c, "volume": v},
                                                   agg, 3_600_000), 48, "producers/context_evaluator.py:403-407"),
        # fixed geometry, as a live caller passes it (the benchmark repeats no
        # time): no capacity probe inside the timed call
        "f4_btc_join_returns": (lambda: engine.join_returns(ts, c, ts[0], btc, capacity=ts.shape[1]), 16,
                                "producers/context_evaluator.py:161-177"),
    }
    out = {"workload": f"{S} symbols x {T} candles (synthetic, HBM-resident)",
           "bytes_rule": "inputs read once + every returned output written once at its dtype"}
    for name, (fn, in_bpc, ref) in rows.items():
        bpc = in_bpc + output_bytes(fn()) / (S * T)
        ms = _time_call(fn)
        gbs = S * T * bpc / (ms * 1e-3) / 1e9
        out[name] = {"ms": ms, "value": S * T / (ms * 1e-3), "unit": "symbol-candles/s", "GBps": gbs,
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_candle": bpc, "reference": ref}
    del p, o, h, l, c, v, qv, ts
    torch.cuda.empty_cache()
    if args.no_cpu_baseline:
        return out
    # bounded single-core CPU timings of the oracle restatements (pandas, the reference's library)
    sym = numpy_symbol(400, 1)
    df = pd.DataFrame(sym)
    bc = numpy_symbol(400, 2)["close"]
    tsv = 1_700_000_000_000 + 900_000 * np.arange(400)
    df_r = df.assign(open_time=tsv)
    cpu = {
        "a11_beta_corr": lambda: indicators_ref.beta_corr_series(sym["close"], bc, 50),
        "a13_market_features": lambda: market_ref.symbol_features(sym["high"], sym["low"], sym["close"]),
        "supertrend": lambda: indicators_ref.supertrend(df.copy(), 3.0, 10),
        "a9_resample_1h": lambda: frame_ref.resample(df_r, "1h", agg),
        "f4_btc_join_returns": lambda: frame_ref.joined_returns(tsv, sym["close"], tsv, bc),
    }
    for name, fn in cpu.items():
        rate = _cpu_rate(fn, 400 if name != "a13_market_features" else 1)
        out[name]["cpu_oracle"] = {"value": rate, "unit": "symbol-candles/s" if name != "a13_market_features"
                                   else "symbol-features/s (one latest-candle feature row per call)",
                                   "cores": 1, "sample": "one 400-candle frame per call, ~1 s"}
    return out


def bench_live(args, dev):
    """Live-path strategy pipelines: S symbols x 400-bar frames per message
    (SURVEY §3.2), eager launches vs one hipGraph replay (binquant_amd.graphs).
    reference_cpu_ms_estimate: the reference's per-symbol pandas cost x S
     — an ESTIMATE measured in the survey container through the
    real modules, not on this host (the oracle does not restate these
    pipelines; their parity rests on the reference's fixtures)."""
    from binquant_amd import signals, strategies
    from binquant_amd.graphs import CapturedPipeline

    S, T = args.live_symbols, 400
    p = device_panel(S, T, device=dev, seed=31)
    ins = [p[k] for k in ("open", "high", "low", "close", "volume")]
    pipes = {
        "a17_activity_burst": (lambda o, h, l, c, v: strategies.activity_burst_features(o, h, l, c, v, v * c), 9.1),
        "a18_pump_score": (lambda o, h, l, c, v: strategies.pump_score_features(o, h, l, c, v, c[0], exact=True),
                           9.8),
        "a19_failed_spike": (lambda o, h, l, c, v: strategies.failed_spike_features(o, h, l, c, v, v * c, exact=True),
                             24.3),
        "a20_top_gainer": (lambda o, h, l, c, v: signals.top_gainer_features(o, h, l, c, v, v * c), None),
    }
    out = {"workload": f"{S} symbols x {T}-bar frames (one message cohort)"}
    for name, (fn, ref_ms) in pipes.items():
        eager = _time_call(lambda: fn(*ins), reps=5)
        g = CapturedPipeline(fn, *ins)
        graph = _time_call(lambda: g(*ins), reps=5)
        out[name] = {"eager_ms": eager, "graph_ms": graph,
                     "reference_cpu_ms_estimate": None if ref_ms is None else ref_ms * S}
        del g
    return out


# the reference's single-core pandas cost per symbol of one message (BASELINE.md
# rows, measured through the real modules): indicators_enrichment on the 5m and
# 15m frames (5.1 ms each), the store features (2.2), ActivityBurstPump (9.1),
# LiquidationSweepPump (9.8), FailedSpikeFade (24.3)
REF_COHORT_MS_PER_SYMBOL = 5.1 * 2 + 2.2 + 9.1 + 9.8 + 24.3


def bench_cohort(args, dev):
    """One message cohort end to end (binquant_amd.cohort.process_cohort:
    ContextEvaluator.process_data for every symbol of a 15-minute cohort,
    producers/context_evaluator.py:347-512, with the context refresh of
    klines_provider.py:181-199): S symbols x 400-bar 5m and 15m frames, eager
    and replayed as one captured hipGraph, next to the reference's per-symbol
    pandas cost x S on one core."""
    from binquant_amd.cohort import process_cohort
    from binquant_amd.graphs import CapturedPipeline

    S, T = args.live_symbols, 400
    p5 = device_panel(S, T, device=dev, seed=41)
    p15 = device_panel(S, T, device=dev, seed=43)
    ts15 = (1_700_000_000_000 + 900_000 * torch.arange(T, device=dev, dtype=torch.int64)).expand(S, T).contiguous()
    ins = [p5[k] for k in ("open", "high", "low", "close", "volume")] + \
          [p15[k] for k in ("open", "high", "low", "close", "volume")] + [ts15, ts15[0].clone(), p15["close"][0].clone()]
    eager = _time_call(lambda: process_cohort(*ins), reps=3)
    g = CapturedPipeline(process_cohort, *ins)
    graph = _time_call(lambda: g(*ins), reps=10)
    del g
    # the part of the cohort the oracle restates, timed here on this host's
    # core: indicators_enrichment of the 5m and 15m frames + the store features
    # per symbol, on a bounded sample of the cohort's own frames
    from oracle import indicators_ref, market_ref

    n_sample = min(24, S)
    h5 = {k: p5[k][:n_sample].cpu().numpy() for k in ("open", "high", "low", "close", "volume")}
    h15 = {k: p15[k][:n_sample].cpu().numpy() for k in ("open", "high", "low", "close", "volume")}
    t0 = time.perf_counter()
    for s in range(n_sample):
        for fr in (h5, h15):
            indicators_ref.indicators_enrichment(pd.DataFrame({k: fr[k][s] for k in fr}))
        market_ref.symbol_features(h15["high"][s], h15["low"][s], h15["close"][s])
    oracle_ms_sym = (time.perf_counter() - t0) * 1e3 / n_sample
    return {"workload": f"{S} symbols x {T}-bar 5m + 15m frames (one message cohort): enrich x2, 1h resample, "
                        "beta/corr + BTC change, context partials + last features, burst / pump / spike / top gainer "
                        "/ leadership features (exact replays)",
            "eager_ms": eager, "graph_ms": graph,
            "oracle_cpu_ms_measured": oracle_ms_sym * S,
            "oracle_cpu_basis": f"measured on this host, 1 core, {n_sample}-symbol sample x {S}: the oracle's pandas "
                                "indicators_enrichment (5m + 15m frames) + _compute_symbol_features per symbol — the "
                                "part of the cohort the oracle restates",
            "reference_cpu_ms_estimate": REF_COHORT_MS_PER_SYMBOL * S,
            "reference_cpu_estimate_basis": "NOT measured here: BASELINE.md per-symbol pandas costs of the real "
                                            "modules in the survey container (incl. the burst / pump / spike "
                                            "pipelines the oracle does not restate) x symbols, 1 core"}


def bench_store(args, dev):
    """§8f row 1: DeviceMarketStateStore at 10k symbols x 400-bar histories;
    one tick = a new closed candle per symbol (host arrays, one device update)
    + the live context build (fresh slots, features, breadth, scoring)."""
    from binquant_amd.market_regime.store import DeviceLiveMarketContextAccumulator, DeviceMarketStateStore

    S, M = args.tick_symbols, 400
    syms = ["BTCUSDT"] + [f"S{i:05d}USDT" for i in range(1, S)]
    store = DeviceMarketStateStore(max_bars_per_symbol=M, capacity=S)
    acc = DeviceLiveMarketContextAccumulator(store, "BTCUSDT")
    rng = np.random.default_rng(0)
    price = 10 ** rng.uniform(-2, 3, S)
    t0 = 1_700_000_000_000
    hist = device_panel(S, M, device=dev, seed=5)
    slots = torch.arange(S, dtype=torch.int64, device=dev).repeat_interleave(M)
    for s in syms:
        store._slot(s)
    tsh = (t0 + 900_000 * torch.arange(M, device=dev, dtype=torch.int64)).repeat(S)
    store.update_slots(slots, tsh, [hist[k].reshape(-1) for k in ("open", "high", "low", "close", "volume")])
    del hist, slots, tsh
    lat = []
    vol = np.ones(S)
    for k in range(args.store_ticks + 20):   # 20 untimed warm-up ticks
        ts = t0 + 900_000 * (M + k)
        price *= np.exp(rng.normal(0, 0.002, S))
        c = price
        torch.cuda.synchronize()
        a = time.perf_counter()
        ctx = acc.on_closed_candles(syms, np.full(S, ts), c, c * 1.001, c * 0.999, c, vol, at=ts)
        torch.cuda.synchronize()
        if k >= 20:
            lat.append(time.perf_counter() - a)
    sl = store.fresh_slots(ts)
    fms = _time_call(lambda: store.features(sl), reps=5)
    lat = np.array(lat) * 1e3
    return {
        "symbols": S, "max_bars": M, "ticks": len(lat),
        "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
        "features_kernel_ms": fms,
        "features_GBps": S * M * 24 / (fms * 1e-3) / 1e9,
        "context_valid": ctx is not None,
        "includes": "host candle arrays -> pinned H2D + one bq_store_update, then the context pass as one "
                    "replayed hipGraph (fresh mask + bq_store_context_features over all slots + breadth + micro "
                    "regime), one D2H of the reduced partials, host scoring/annotation; synchronized",
    }


def time_enrich(panel, steps: int, warmup: int, world: int):
    """Wall time per step (barrier + synchronize on both sides, max over
    ranks) and mean enrich_kernel time (HIP events on the launch stream)."""
    S, T = panel["close"].shape
    dev = panel["close"].device
    out = engine.enrich_outputs(S, T, dev)   # padded row pitch (engine.enrich_outputs)
    stream = torch.cuda.current_stream()

    def step():
        engine.enrich(panel["open"], panel["high"], panel["low"], panel["close"], panel["volume"], out=out)

    for _ in range(warmup):
        step()
    barrier(world)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    barrier(world)
    wall = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    del out
    return max_over_ranks(wall, world) / steps, max_over_ranks(kern_ms, world)


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", local)
    lo, hi = shard_bounds(args.symbols, world, rank)
    S, T = hi - lo, args.candles
    panel = device_panel(S, T, device=dev, seed=1234 + rank)
    step_s, kern_ms = time_enrich(panel, args.steps, args.warmup, world)
    value = args.symbols * T / step_s
    bytes_launch = S * T * BYTES_PER_CANDLE
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic("enrich_kernel", S * T)

    result = {
        "metric": "symbol-candles/s for full indicator set (14 fp64 columns)",
        "value": value,
        "unit": "symbol-candles/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8d random-walk klines generated in HBM)",
        "config": {
            "workload": f"configs[3]: {args.symbols} symbols x {T} candles, symbol-sharded over {world} GPU(s) "
                        f"({S} symbols x {T} candles on rank 0)",
            "symbols": args.symbols,
            "symbols_per_gpu": S,
            "candles": T,
            "columns": list(ENRICH_COLUMNS),
            "parallelism": f"symbol-sharded x{world}, no data-path collective",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": "enrich_kernel",
            "kernel_ms": kern_ms,
            "algorithmic_bytes_per_candle": BYTES_PER_CANDLE,
            "candles_per_launch": S * T,
        },
    }
    if not args.no_breadth:
        result["breadth"] = bench_breadth(args, panel, world, dev)
    del panel
    torch.cuda.empty_cache()
    if not args.no_shard:
        shard = device_panel(args.shard_symbols, T, device=dev, seed=4321 + rank)
        sh_step, sh_kern = time_enrich(shard, args.shard_steps, 2, world)
        result["shard"] = {
            "workload": f"C4 shard: {args.shard_symbols} symbols x {T} candles per GPU (weak scaling)",
            "value": args.shard_symbols * T * world / sh_step,
            "unit": "symbol-candles/s",
            "scaling": "weak",
            "ms_per_step": sh_step * 1e3,
            "kernel_ms": sh_kern,
            "frac": args.shard_symbols * T * BYTES_PER_CANDLE / (sh_kern * 1e-3) / 1e9 / HBM_PEAK_GBS,
        }
        del shard
        torch.cuda.empty_cache()
    # rank 0 only, after every timed multi-rank leg (the other ranks wait in
    # the closing barrier): C3 and the store tick are one-GPU latencies, so
    # they run at every world size; the per-row legs at N = 1 only; the CPU
    # baseline at every world size (north_star: the reference CPU path beside
    # the GPU figure at 1, 2, 4 and 8 GPUs)
    if rank == 0 and not args.no_tick:
        result["tick"] = bench_tick(args, dev)
        result["store"] = bench_store(args, dev)
    if rank == 0 and world == 1 and not args.no_rows:
        result["rows"] = bench_rows(args, dev)
        result["live"] = bench_live(args, dev)
        result["cohort"] = bench_cohort(args, dev)
    result["cpu_baseline"] = cpu_baseline(args) if rank == 0 and not args.no_cpu_baseline else None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
