#!/usr/bin/env python3
"""Summary of the last k_live dispatch of two rocprofv3 PMC passes (SQ counters, FETCH_SIZE):
VALU instructions per wave, VALU busy, effective clock, HBM read traffic against the 16 B events.
usage: scripts/pmc_live_summary.py <sq.csv> <fetch.csv>"""
import csv
import json
import sys

CUS, SIMDS, XCDS = 256, 4, 8
K, E = 1 << 20, 1024
EVB = int(sys.argv[3]) if len(sys.argv) > 3 else 16  # bytes per event (32: FP64 events)


def last(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        if "k_live" in r["Kernel_Name"]:
            d = rows.setdefault(int(r["Dispatch_Id"]), {})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return rows[max(rows)], len(rows)


s, n = last(sys.argv[1])
f, _ = last(sys.argv[2])
clk = s["GRBM_GUI_ACTIVE"] / XCDS / (s["_ns"] * 1e-9)
out = {"kernel": "k_live<false> (pekf_live_dev)", "dispatches": n, "summarised": "the last (steady state)",
       "config": {"filters": K, "events_per_filter": E}, "kernel_ns_sq_pass": s["_ns"], "kernel_ns_fetch_pass": f["_ns"],
       "valu_insts_per_wave": s["SQ_INSTS_VALU"] / s["SQ_WAVES"],
       "valu_busy": 4 * s["SQ_ACTIVE_INST_VALU"] / (CUS * SIMDS * s["GRBM_GUI_ACTIVE"] / XCDS),
       "effective_clock_ghz": clk / 1e9, "sq_wait_any_frac": s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"],
       "traffic_bytes": 2.0 * f["FETCH_SIZE"] * 1024, "algorithmic_bytes": EVB * K * E,
       "note": "traffic = 2 x FETCH_SIZE x 1024 (gfx950); valu_busy = 4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8)"}
out["traffic_over_algorithmic"] = out["traffic_bytes"] / out["algorithmic_bytes"]
print(json.dumps(out, indent=1))
