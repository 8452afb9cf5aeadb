"""Summarise a tools/evidence.sh run into profiles/ (committed evidence).

python tools/parse_prof.py gpurun_out/<TAG> r02   writes, per bench config C
found under gpurun_out/<TAG>/C/:
  profiles/r02_<C>_kernel_stats.csv  -- rocprofv3 --kernel-trace --stats summary
  profiles/r02_<C>_bench.json        -- the bench line of that config (if run)
and merges into profiles/r02_pmc_summary.json  {C: {class: {...}}} per tagged
kernel class: launches, average traced duration, FETCH_SIZE / WRITE_SIZE per
launch and the corrected HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE
(KB * 1024; the factor 2 is the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md "HBM" for wide coalesced reads).  Untagged kernels (the
XC point kernels, J, embedding) are summarised under their own names.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAGS = {1: "df_exchange_contract", 2: "xc_forward_u", 3: "xc_back_l", 4: "xc_forward_w", 5: "xc_back_m"}


def tag_of(name, stored=False):
    """Class of a kernel symbol: dgemm_kernel<BM, BN, WGM, WGN, BK, MINW, A_KC,
    B_KC, TAG, MODE, MAP> by its TAG; the skinny exchange kernels as the stored
    exchange class."""
    if "k_skinny" in name:
        return "mo_exchange_stored"
    if "k_xc_rho_w" in name:
        return "xc_forward_w"
    if "k_xc_back_m" in name:          # the dedicated kernel and its split reduce
        return "xc_back_m"
    if "dgemm_kernel<" not in name:
        return None
    t = int(name.split("dgemm_kernel<")[1].split(">")[0].split(",")[8])
    if t == 1 and stored:
        return "mo_exchange_stored"
    return TAGS.get(t)


def is_aux(name):
    """helper launches of a class (counted in its bytes and time, not its launches)"""
    return ("k_skinny_reduce" in name or "k_skinny_transpose" in name or "k_xc_back_m_reduce" in name
            or "k_xsf_split4" in name or "k_xsf_combine4" in name)


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()[-60:]


def rows(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return list(csv.DictReader(f))


def bench_line(path):
    try:
        with open(path) as f:
            return json.loads([l for l in f if l.startswith("{")][-1])
    except (OSError, IndexError, ValueError):
        return None


def summarise(cdir):
    line = bench_line(os.path.join(cdir, "trace.log"))
    stored = bool(line and "mo_exchange_stored" in line.get("gemm_classes", {}))
    steps = (line or {}).get("steps", 1)
    acc = {}

    def slot(name):
        key = tag_of(name, stored) or short(name)
        return key, acc.setdefault(key, dict(kernels=set(), launches=0, fetch_kb=0.0, write_kb=0.0,
                                             dur_ns=0.0, traced=0))

    for r in rows(os.path.join(cdir, "trace", "run_kernel_trace.csv")):
        _, s = slot(r["Kernel_Name"])
        s["kernels"].add(r["Kernel_Name"])
        s["dur_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        s["traced"] += 0 if is_aux(r["Kernel_Name"]) else 1
    for p, field in (("FETCH_SIZE", "fetch_kb"), ("WRITE_SIZE", "write_kb")):
        seen = defaultdict(int)
        for r in rows(os.path.join(cdir, p, "run_counter_collection.csv")):
            if r["Counter_Name"] != p:
                continue
            key, s = slot(r["Kernel_Name"])
            s[field] += float(r["Counter_Value"])
            seen[key] += 0 if is_aux(r["Kernel_Name"]) else 1
        for key, n in seen.items():
            acc[key].setdefault("pmc_launches", {})[p] = n
    out = {}
    for key, s in acc.items():
        n = max(s.get("pmc_launches", {}).values() or [0]) or 1
        s["kernels"] = sorted(s["kernels"])
        s["launches_pmc"] = n
        s["fetch_bytes_per_launch_raw"] = s["fetch_kb"] * 1024 / n
        s["write_bytes_per_launch"] = s["write_kb"] * 1024 / n
        s["hbm_bytes_per_launch"] = (2 * s["fetch_kb"] + s["write_kb"]) * 1024 / n
        s["avg_duration_ms_trace"] = s["dur_ns"] / max(1, s["traced"]) / 1e6
        s["ms_per_step_trace"] = s["dur_ns"] / 1e6 / max(1, steps + (line or {}).get("warmup", 0))
        s.pop("pmc_launches", None)
        out[key] = s
    return out, line


def main(tag_dir, rnd="r02"):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    path = os.path.join(prof, f"{rnd}_pmc_summary.json")
    try:
        with open(path) as f:
            summary = json.load(f)
    except (OSError, ValueError):
        summary = {}
    for c in sorted(os.listdir(tag_dir)):
        cdir = os.path.join(tag_dir, c)
        if not os.path.isdir(os.path.join(cdir, "trace")):
            continue
        st = os.path.join(cdir, "trace", "run_kernel_stats.csv")
        if os.path.exists(st):
            shutil.copy(st, os.path.join(prof, f"{rnd}_{c}_kernel_stats.csv"))
        b = bench_line(os.path.join(cdir, "bench.log"))
        if b:
            with open(os.path.join(prof, f"{rnd}_{c}_bench.json"), "w") as f:
                f.write(json.dumps(b) + "\n")
        summary[c], _ = summarise(cdir)
        print(c, {k: (round(v["avg_duration_ms_trace"], 3), round(v["hbm_bytes_per_launch"] / 1e9, 3))
                  for k, v in summary[c].items() if v["traced"]})
    with open(path, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
