"""Per-kernel duration summary from a rocprofv3 SQLite (rocpd) output database.

    python tools/kstats.py <results.db> [--csv out.csv] [--top N]
"""
import argparse
import csv
import sqlite3


def kernel_stats(db: str):
    con = sqlite3.connect(db)
    cur = con.cursor()
    rows = cur.execute(
        "select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
        "max(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
        "group by s.kernel_name order by sum(d.end - d.start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": r[3], "Percentage": 100.0 * r[2] / tot,
             "MinNs": r[4], "MaxNs": r[5]} for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    st = kernel_stats(a.db)
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0]))
            w.writeheader()
            w.writerows(st)
    for r in st[: a.top]:
        print(f"{r['Percentage']:6.2f}% {r['Calls']:6d} {r['AverageNs'] / 1e3:10.1f} us  {r['Name'][:110]}")


if __name__ == "__main__":
    main()
