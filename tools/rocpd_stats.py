"""Per-kernel stats CSV from a rocprofv3 rocpd SQLite database (``top_kernels`` view).

    python tools/rocpd_stats.py gpurun_out/prof11/run_results.db > profiles/.../kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    # the rocpd views report durations in microseconds (a 1 GiB HBM check reads ~250 here:
    # 4.2 TB/s; 250 ns would be 4 PB/s)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, total, avg, pct in c.execute("select * from top_kernels"):
        w.writerow([name, calls, round(total, 1), round(avg, 1), round(pct, 2)])


if __name__ == "__main__":
    main(sys.argv[1])
