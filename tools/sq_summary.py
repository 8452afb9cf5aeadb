"""Per-GEMM-class summary of tools/profile_sq.sh passes (rocprofv3 --pmc csv).

python tools/sq_summary.py gpurun_out/<TAG>   -> one JSON object per class with
summed counters, launches and the ratios used in DESIGN.md:
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMD)   (matrix-core duty)
  wait_any / wait_inst / active_any = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY
                                       per SQ_WAVE_CYCLES
  clock_ghz  = GRBM_GUI_ACTIVE / 8 XCD / kernel time
  hbm_bytes  = 2 FETCH_SIZE + WRITE_SIZE (KB, gfx950 FETCH correction, MI355X_MICROARCH.md)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_prof import tag_of  # noqa: E402


def main(d):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(float)
    for path in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(path)):
            t = tag_of(row["Kernel_Name"]) or row["Kernel_Name"].split("(")[0][-40:]
            acc[t][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[(t, os.path.basename(os.path.dirname(path)))].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    for path in glob.glob(os.path.join(d, "a", "run_kernel_trace.csv")):
        for row in csv.DictReader(open(path)):
            t = tag_of(row["Kernel_Name"]) or row["Kernel_Name"].split("(")[0][-40:]
            dur[t] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    out = {}
    for t, c in acc.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        r = {k: v for k, v in c.items()}
        if "SQ_BUSY_CYCLES" in c and c["SQ_BUSY_CYCLES"]:
            r["mfma_busy"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (4.0 * c["SQ_BUSY_CYCLES"])
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
            if k in c:
                r[k.lower().replace("sq_", "") + "_per_wave_cycle"] = c[k] / wc
        if dur.get(t) and "GRBM_GUI_ACTIVE" in c:
            r["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8.0 / dur[t] / 1e9
        if "FETCH_SIZE" in c:
            r["hbm_bytes"] = (2 * c["FETCH_SIZE"] + c.get("WRITE_SIZE", 0.0)) * 1024
        r["kernel_s"] = dur.get(t)
        out[t] = r
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
