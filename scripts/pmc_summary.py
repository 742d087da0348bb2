#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the fused kernel into profiles/<round>/pmc_summary.json.

usage: scripts/pmc_summary.py <fetch_csv> <sq_csv> <batch> <records> <out.json>

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports exactly half the
bytes of a wide coalesced streaming read on gfx950, so traffic = 2 * FETCH_SIZE * 1024.
SQ_* wave/active counters are in quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import csv
import json
import sys

CUS, SIMDS_PER_CU, XCDS = 256, 4, 8


def counters(path, kernel="k_run"):
    out = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            out.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
            out[r["Dispatch_Id"]]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return list(out.values())


def main():
    fetch_csv, sq_csv, batch, records, dst = sys.argv[1:6]
    batch, records = int(batch), int(records)
    f = counters(fetch_csv)[0]
    s = counters(sq_csv)[0]
    algo = batch * records * 40
    traffic = 2.0 * f["FETCH_SIZE"] * 1024
    waves = s["SQ_WAVES"]
    clk = s["GRBM_GUI_ACTIVE"] / XCDS / (s["_ns"] * 1e-9)
    valu_busy = 4 * s["SQ_ACTIVE_INST_VALU"] / (CUS * SIMDS_PER_CU * s["GRBM_GUI_ACTIVE"] / XCDS)
    summary = {
        "kernel": "k_run<false> (pekf_run_dev)",
        "config": {"batch": batch, "records": records},
        "algorithmic_read_bytes": algo,
        "fetch_size_kib": f["FETCH_SIZE"],
        "hbm_traffic_bytes": traffic,
        "traffic_over_algorithmic": traffic / algo,
        "kernel_ns_fetch_pass": f["_ns"],
        "kernel_ns_sq_pass": s["_ns"],
        "effective_clock_ghz": clk / 1e9,
        "valu_busy": valu_busy,
        "valu_insts_per_wave_step": s["SQ_INSTS_VALU"] / (waves * records),
        "sq_wait_inst_any_frac": s["SQ_WAIT_INST_ANY"] / s["SQ_WAVE_CYCLES"],
        "sq_wait_any_frac": s["SQ_WAIT_ANY"] / s["SQ_WAVE_CYCLES"],
        "note": "traffic = 2 x FETCH_SIZE x 1024 (gfx950 FETCH_SIZE halves wide streaming reads); "
                "valu_busy = 4 x SQ_ACTIVE_INST_VALU (quad-cycles) / (1024 SIMDs x GRBM_GUI_ACTIVE/8)",
    }
    json.dump(summary, open(dst, "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
