"""Per-kernel dispatch count / average / total ms from a rocprofv3 rocpd
database (rocprofv3 -d DIR -o NAME writes NAME_results.db)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
q = """select s.kernel_name, count(*), avg(d.end - d.start) / 1e6, sum(d.end - d.start) / 1e6
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
       group by s.kernel_name order by sum(d.end - d.start) desc"""
print("calls,avg_ms,total_ms,kernel")
for name, n, avg, tot in db.execute(q).fetchall()[: int(sys.argv[2]) if len(sys.argv) > 2 else 15]:
    print(f"{n},{avg:.4f},{tot:.3f},{name[:120]}")
