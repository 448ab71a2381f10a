"""HIP API call counts from a rocprofv3 --hip-trace database (rocpd SQLite):
which runtime calls (hipMemcpyAsync, hipMemsetAsync, ...) a run issued.

    python tools/api_counts.py <run_results.db> [PATTERN]
"""
import sqlite3
import sys
from collections import Counter


def main():
    con = sqlite3.connect(sys.argv[1])
    pat = sys.argv[2].lower() if len(sys.argv) > 2 else ""
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table', 'view')")]
    for t in tabs:
        cols = [r[1] for r in con.execute(f"pragma table_info('{t}')")]
        if "name" not in cols:
            continue
        try:
            cnt = Counter(r[0] for r in con.execute(f"select name from '{t}'"))
        except sqlite3.Error:
            continue
        hits = [(n, c) for n, c in cnt.most_common() if isinstance(n, str) and pat in n.lower()]
        if hits:
            print(f"# {t}")
            for n, c in hits[:25]:
                print(f"{c:8d}  {n[:120]}")


def timeline(path, pat, bins=10):
    """per-tenth-of-the-run counts of the matching calls (setup vs steady state)"""
    con = sqlite3.connect(path)
    cols = [r[1] for r in con.execute("pragma table_info('regions')")]
    st = "start" if "start" in cols else cols[cols.index("name") + 1]
    rows = [(n, t) for n, t in con.execute(f"select name, {st} from regions") if isinstance(n, str)]
    t0, t1 = min(t for _, t in rows), max(t for _, t in rows)
    per = Counter()
    for n, t in rows:
        if pat in n.lower():
            per[(n, min(bins - 1, int((t - t0) * bins / max(1, t1 - t0))))] += 1
    for n in sorted({n for n, _ in per}):
        print(f"{n:28s}", " ".join(f"{per[(n, b)]:5d}" for b in range(bins)))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[3] == "--timeline":
        timeline(sys.argv[1], sys.argv[2].lower())
        sys.exit(0)
    main()
