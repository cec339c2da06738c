"""Markdown kernel summary from a rocprofv3 SQLite database (--kernel-trace
without --output-format csv).  usage: python tools/parse_prof_db.py DB [title]"""
import sqlite3
import sys

db = sys.argv[1]
title = sys.argv[2] if len(sys.argv) > 2 else db
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration) "
                 "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[5] for r in rows)
print(f"# {title}\n")
print("| kernel | calls | avg µs | min µs | max µs | total ms | % |")
print("|---|---|---|---|---|---|---|")
for name, n, avg, mn, mx, sm in rows:
    short = name.split("(")[0].replace("void ", "")
    print(f"| `{short}` | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {sm / 1e6:.3f} | {100 * sm / tot:.1f} |")
seq = c.execute("select name, grid_x, duration from kernels where name like '%k_pw_%' order by start").fetchall()
if seq:
    print("\n## Wavefront launches in order (grid = threads)\n")
    print("| kernel | grid | µs |")
    print("|---|---|---|")
    for name, g, d in seq[:24]:
        print(f"| `{name.split('(')[0].replace('void ', '')}` | {g} | {d / 1e3:.1f} |")
