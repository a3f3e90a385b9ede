"""Per-kernel statistics (calls, total / average ns, share) from a rocprofv3 SQLite output (.db),
in the column layout of rocprofv3 --stats' kernel_stats.csv.  Usage: python tools/rocpd_stats.py <out.db|dir> [csv]"""
import collections
import csv
import glob
import os
import sqlite3
import sys

src = sys.argv[1]
db = src if src.endswith(".db") else glob.glob(os.path.join(src, "**", "*.db"), recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                 "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
agg = collections.defaultdict(list)
for name, a, b in rows:
    agg[name].append(b - a)
tot = sum(sum(v) for v in agg.values())
out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")]
for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    out.append((name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)))
w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
w.writerows(out)
