#!/usr/bin/env python3
"""Timeline of the last N kernel dispatches of a rocprofv3 run whose output is the rocpd
SQLite database (run_results.db): name, the idle gap before it on the GPU, its duration.
Usage: python tools/rocpd_timeline.py <run_results.db> [N]"""
import sqlite3,sys,re
db=sys.argv[1]
c=sqlite3.connect(db)
cols=[r[1] for r in c.execute("pragma table_info(kernels)")]
rows=c.execute("select * from kernels order by start").fetchall()
ix={k:i for i,k in enumerate(cols)}
def short(n):
    n=n.replace("(anonymous namespace)::","");m=re.search(r"\b(k_\w+(<[^()]*>)?)",n);return m.group(1) if m else n[:40]
name_k=[k for k in cols if 'name' in k.lower()][0]
# last N dispatches
N=int(sys.argv[2]) if len(sys.argv)>2 else 40
sel=rows[-N:]
prev=None
for r in sel:
    st,en=r[ix['start']],r[ix['end']]
    g=r[ix.get('grid_size_x',0)] if 'grid_size_x' in ix else ''
    print(f"{short(r[ix[name_k]])[:40]:40s} gap {(st-prev)/1e3 if prev else 0:8.2f} dur {(en-st)/1e3:8.2f} grid {g}")
    prev=en
