"""Median duration per (kernel, grid) from a rocprofv3 --kernel-trace SQLite database (rocpd tables).
Usage: python tools/rocpd_medians.py run_results.db [kernel-substring ...]"""
import collections
import sqlite3
import sys

import numpy as np


def medians(db, keys=()):
    con = sqlite3.connect(db)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    q = ("select s.kernel_name, d.start, d.end, d.grid_size_x from %s d join %s s on d.kernel_id = s.id" % (kd, ks))
    by = collections.defaultdict(list)
    for name, st, en, gx in cur.execute(q):
        if not keys or any(k in name for k in keys):
            by[(name, gx)].append((en - st) / 1e3)
    return {k: (len(v), float(np.median(v)), float(np.mean(v))) for k, v in by.items()}


if __name__ == "__main__":
    for (name, gx), (n, med, avg) in sorted(medians(sys.argv[1], sys.argv[2:]).items(), key=lambda x: -x[1][0] * x[1][1]):
        print("%-60s grid %9d  n %4d  median %9.2f us  avg %9.2f us" % (name[:60], gx, n, med, avg))
