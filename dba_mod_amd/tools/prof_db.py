"""Summarise a rocprofv3 rocpd sqlite database: per-kernel totals over the last N dispatches."""
import sqlite3, sys, re, collections
def short(n):
    n = n.replace('(anonymous namespace)::', '')
    n = re.sub(r'^void ', '', n)
    n = re.sub(r'\(.*', '', n)
    return n[:70]
def summary(path, last=None):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    if last: rows = rows[-last:]
    tot = collections.defaultdict(lambda: [0.0, 0])
    for n, s, e in rows:
        t = tot[short(n)]; t[0] += (e - s) / 1e3; t[1] += 1
    span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0
    return tot, span, len(rows)
if __name__ == "__main__":
    last = int(sys.argv[2]) if len(sys.argv) > 2 else None
    tot, span, n = summary(sys.argv[1], last)
    print(f"{n} dispatches, span {span:.1f} us, kernel sum {sum(v[0] for v in tot.values()):.1f} us")
    for k, (us, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"{us:10.1f} us {c:6d}  {k}")
