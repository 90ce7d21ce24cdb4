"""Summarize a rocprofv3 kernel_stats.csv: per-kernel average ms and share."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    name = r["Name"]
    short = name.split("(")[0].replace("void ", "")
    if "rocprim" in name:
        m = re.search(r"wrapped_(\w+?)_config", name)
        short = "rocprim::" + (m.group(1) if m else "init_lookback" if "init_lookback" in name else name[:40])
    print(f"{short[:48]:48s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f} "
          f"total_ms={float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f}%")
print("total ms", round(tot / 1e6, 2))
