"""Summarise a tools/profile_r01.sh run into profiles/ (committed evidence).

Writes
  profiles/<round>_kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary
  profiles/<round>_pmc_summary.json   -- per tagged GEMM class: launches, average
      duration, FETCH_SIZE / WRITE_SIZE per launch and the corrected HBM bytes
      per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB * 1024; the factor 2 is the
      gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md "HBM" for wide
      coalesced reads)
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAGS = {1: "df_exchange_contract", 2: "xc_forward_u", 3: "xc_back_l", 4: "xc_forward_w", 5: "xc_back_m"}


def tag_of(name):
    """GEMM class of a dgemm_kernel<BM, BN, WGM, WGN, BK, MINW, A_KC, B_KC, TAG, MODE> symbol."""
    if "dgemm_kernel<" not in name:
        return None
    t = int(name.split("dgemm_kernel<")[1].split(">")[0].split(",")[8])
    return TAGS.get(t)


def counters(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def durations(path):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            per[row["Kernel_Name"]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return per


def main(prof_dir, rnd="r01"):
    # the bench line names tag 1 after the exchange mode it ran
    try:
        with open(os.path.join(prof_dir, "trace.log")) as f:
            line = [l for l in f if l.startswith("{")][-1]
        if "mo_exchange_stored" in json.loads(line).get("gemm_classes", {}):
            TAGS[1] = "mo_exchange_stored"
    except Exception:
        pass
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(prof_dir, "trace", "run_kernel_stats.csv"),
                os.path.join(out, f"{rnd}_kernel_stats.csv"))
    fetch = counters(os.path.join(prof_dir, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(prof_dir, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    dur = durations(os.path.join(prof_dir, "trace", "run_kernel_trace.csv"))
    summary = {}
    for name in set(fetch) | set(write) | set(dur):
        tag = tag_of(name)
        if tag is None:
            continue
        s = summary.setdefault(tag, dict(kernels=[], launches=0, fetch_kb=0.0, write_kb=0.0,
                                         dur_ns=0.0, traced=0))
        s["kernels"].append(name)
        s["launches"] += len(fetch.get(name, []))
        s["fetch_kb"] += sum(fetch.get(name, []))
        s["write_kb"] += sum(write.get(name, []))
        s["dur_ns"] += sum(dur.get(name, []))
        s["traced"] += len(dur.get(name, []))
    for tag, s in summary.items():
        n = max(1, s["launches"])
        s["fetch_bytes_per_launch_raw"] = s["fetch_kb"] * 1024 / n
        s["write_bytes_per_launch"] = s["write_kb"] * 1024 / n
        s["hbm_bytes_per_launch"] = 2 * s["fetch_kb"] * 1024 / n + s["write_kb"] * 1024 / n
        s["avg_duration_ms_trace"] = s["dur_ns"] / max(1, s["traced"]) / 1e6
    with open(os.path.join(out, f"{rnd}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
