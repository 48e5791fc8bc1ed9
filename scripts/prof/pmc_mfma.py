#!/usr/bin/env python3
"""Per-kernel MFMA / wave-state summary of a rocprofv3 --pmc CSV pass
(counter_collection.csv) taken with
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
  SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT

mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs x SIMDs): the
share of SIMD cycles with the matrix pipe busy while the GPU ran the dispatch
(GRBM_GUI_ACTIVE is summed over the 8 XCDs' GRBMs: 1.76M for a 91.6 us
dispatch = 8 x 220K shader cycles; MFMA busy cycles are per SIMD, e.g.
113M for the fp32 tower forward = its 6.86 GFLOP / 64 FLOP per SIMD cycle); wait /
inst-stall / active are the shares of wave cycles (disjoint, MI355X_MICROARCH
PMC table).

    python scripts/prof/pmc_mfma.py gpurun_out/pmc_tower/pmc_counter_collection.csv --simds 1024
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--simds", type=int, default=1024)  # 256 CUs x 4 SIMDs
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    if a.csv.endswith(".db"):  # rocprofv3's default rocpd database: its counters_collection view
        import sqlite3

        con = sqlite3.connect(a.csv)
        rows_in = [{"Kernel_Name": k, "Counter_Name": n, "Counter_Value": v, "Dispatch_Id": d}
                   for (k, n, v, d) in con.execute(
                       "select kernel_name, counter_name, value, dispatch_id from counters_collection")]
    else:
        with open(a.csv) as f:
            rows_in = list(csv.DictReader(f))
    if True:
        for r in rows_in:
            k = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            k = k.replace("pbx::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    rows = []
    for k, c in per.items():
        act = c.get("GRBM_GUI_ACTIVE", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        rows.append((c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), k, len(disp[k]),
                     c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (act / a.xcds * a.simds) if act else 0.0,
                     c.get("SQ_WAIT_ANY", 0.0) / wc, c.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                     c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc))
    rows.sort(reverse=True)
    print(f"| kernel | dispatches | mfma_util | wave wait | inst stall | active |")
    print(f"|---|---|---|---|---|---|")
    for _, k, n, u, w, i, ac in rows[:a.top]:
        print(f"| {k} | {n} | {u:.3f} | {w:.3f} | {i:.3f} | {ac:.3f} |")


if __name__ == "__main__":
    main()
