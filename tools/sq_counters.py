"""Per-GEMM-class summary of an SQ counter pass (rocprofv3 --pmc ... csv)."""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from parse_prof import tag_of  # noqa: E402

path = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(int)
for row in csv.DictReader(open(path)):
    t = tag_of(row["Kernel_Name"]) or row["Kernel_Name"][:40]
    acc[t][row["Counter_Name"]] += float(row["Counter_Value"])
    n[(t, row["Counter_Name"])] += 1
for t, d in sorted(acc.items()):
    wc = d.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    parts = [f"{k}={v / wc:.3f}" for k, v in sorted(d.items()) if k != "SQ_WAVE_CYCLES"]
    print(f"{t:28s} wave_cycles={wc:.3e} " + " ".join(parts))
