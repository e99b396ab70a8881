"""Per-kernel duration stats from a rocprofv3 results database (the default rocpd SQLite
output): name, calls, average / min / max us, total ms.  Usage: prof_db_stats.py DB [filter]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = db.execute("select s.kernel_name, d.end - d.start, d.grid_size_x, d.workgroup_size_x "
                  "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
st = collections.defaultdict(list)
for name, dur, gx, wx in rows:
    if flt in name:
        st[(name, gx // max(wx, 1))].append(dur / 1000.0)
print("%-70s %6s %6s %9s %9s %9s %9s" % ("kernel", "wgs", "calls", "avg_us", "min_us", "max_us", "total_ms"))
for (name, wg), d in sorted(st.items(), key=lambda kv: -sum(kv[1])):
    print("%-70s %6d %6d %9.2f %9.2f %9.2f %9.3f" % (name[:70], wg, len(d), sum(d) / len(d), min(d), max(d),
                                                     sum(d) / 1000))
