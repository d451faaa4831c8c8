"""Fold the rocprofv3 evidence of the C5 context build (tools/row_profile.sh
<tag> context, ROW_S=100000 ROW_T=10000) into profiles/pmc_traffic.json's
"context_partials" entry — the figures bench.py's breadth roofline reports.

The bench times `engine.context_partials` whole (kernel_ms: passes 1 + 2 + 3),
so `bytes_per_launch` is the HBM traffic of all three kernels per call
(FETCH_SIZE x 2 on gfx950 for 16-byte streaming reads, WRITE_SIZE; KiB ->
bytes), with the split per kernel beside it. Pass 1 is bound by its
instruction stream as much as by HBM, so its VALU figures go
in too. Pass 2 reads 8-byte lanes (lane = timestamp), a width the guide's
x2 rule is not calibrated for: its x1 figure is kept beside the x2 one, and
its algorithmic read (the group records: 34 B per 4 symbols and candle) is
the check of which one holds.
Pass-1 VALU figures:
  valu_lane_ops_per_candle = SQ_INSTS_VALU x 64 / (S x T)
  valu_busy_est            = 4 cycles x SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
                             (a wave64 fp64 VALU instruction occupies a 16-lane SIMD 4 cycles)
  valu_active_share        = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES

    python tools/context_traffic.py <rows_summary.json> <pmc_traffic.json> <tag>
"""
import json
import sys

PASSES = ("context_partials_kernel", "context_group_reduce_kernel", "context_chunk_reduce_kernel")


def main():
    src, dst, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    row = json.load(open(src))["context"]
    S, T = row["shape"]
    by_k = row["counters_per_call_by_kernel"]
    kernels = {}
    total_f = total_w = 0.0
    p1 = None
    for name, cnt in by_k.items():
        short = next((p for p in PASSES if p in name), None)
        if short is None:
            continue
        f = cnt.get("FETCH_SIZE", 0.0) * 1024 * 2
        w = cnt.get("WRITE_SIZE", 0.0) * 1024
        total_f += f
        total_w += w
        us = next((k["per_call_us"] for n, k in row["kernels"].items() if short in n), None)
        kernels[short] = {"name": name, "us_per_call": us, "fetch_bytes_x2": f, "fetch_bytes_x1": f / 2,
                          "write_bytes": w,
                          "traffic_bytes": f + w}
        if short == PASSES[0]:
            p1 = cnt
    valu = None
    if p1 and p1.get("SQ_INSTS_VALU") and p1.get("GRBM_GUI_ACTIVE"):
        simd_cycles = p1["GRBM_GUI_ACTIVE"] / 8 * 1024
        valu = {"kernel": PASSES[0],
                "valu_lane_ops_per_candle": p1["SQ_INSTS_VALU"] * 64 / (S * T),
                "valu_busy_est": 4 * p1["SQ_INSTS_VALU"] / simd_cycles,
                "valu_active_share": p1["SQ_ACTIVE_INST_VALU"] / p1["SQ_WAVE_CYCLES"]
                if p1.get("SQ_WAVE_CYCLES") else None,
                "wait_share": p1["SQ_WAIT_ANY"] / p1["SQ_WAVE_CYCLES"] if p1.get("SQ_WAVE_CYCLES") else None,
                "sq_insts_valu": p1["SQ_INSTS_VALU"], "grbm_gui_active": p1["GRBM_GUI_ACTIVE"]}
    try:
        allk = json.load(open(dst))
    except (OSError, ValueError):
        allk = {}
    allk["context_partials"] = {
        "source": tag,
        "bytes_per_launch": total_f + total_w,
        "candles_per_launch": S * T,
        "fetch_bytes_corrected": total_f,
        "write_bytes": total_w,
        "traffic_over_algorithmic": (total_f + total_w) / (24.0 * S * T),
        "scope": "all three passes per engine.context_partials call (what bench kernel_ms times)",
        "kernels": kernels,
        "valu": valu,
        "note": "FETCH_SIZE x2 (gfx950 half-count for 16B/lane streaming reads), KiB -> bytes",
    }
    json.dump(allk, open(dst, "w"), indent=1)
    print(json.dumps(allk["context_partials"], indent=1))


if __name__ == "__main__":
    main()
