"""Summarise a rocprofv3 SQLite kernel trace: per-kernel stats and the last step's timeline."""
import sqlite3
import sys


def main(db, timeline=True):
    c = sqlite3.connect(db)
    q = "select name, count(*), avg(end-start), sum(end-start) from kernels group by name order by sum(end-start) desc"
    print(f"{'kernel':40s} {'calls':>5s} {'avg_us':>9s} {'total_ms':>9s}")
    for n, k, a, s in c.execute(q):
        print(f"{n.split('(')[0][:40]:40s} {k:5d} {a / 1e3:9.1f} {s / 1e6:9.2f}")
    if not timeline:
        return
    rows = list(c.execute("select name, start, end, grid_x, grid_y, workgroup_x, vgpr_count, lds_size, scratch_size "
                          "from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if 'k_gray' in r[0]][-1]
    t0 = rows[idx][1]
    print("\nlast step:")
    for r in rows[idx:]:
        if 'rocclr' in r[0]:
            continue
        print(f"{r[0].split('(')[0][:26]:26s} +{(r[1] - t0) / 1e3:8.1f} {(r[2] - r[1]) / 1e3:7.1f}us "
              f"grid {r[3]}x{r[4]} wg {r[5]} vgpr {r[6]} lds {r[7]} scr {r[8]}")


if __name__ == "__main__":
    main(sys.argv[1], len(sys.argv) < 3)
