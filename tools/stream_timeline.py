"""Per-stream timeline of the last few steps of a rocprofv3 kernel trace (sqlite)."""
import sqlite3
import sys


def main(db, nsteps=2):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, stream_id from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if 'k_gray' in r[0]]
    i0 = idx[-1 - nsteps]
    t0 = rows[i0][1]
    for r in rows[i0:]:
        if 'rocclr' in r[0]:
            continue
        print(f"{r[0].split('(')[0].replace('odo::', '')[:20]:20s} s{r[3]} +{(r[1] - t0) / 1e3:8.1f} "
              f"{(r[2] - r[1]) / 1e3:7.1f}  end {(r[2] - t0) / 1e3:8.1f}")
    g = [rows[i][1] for i in idx[-1 - nsteps:]]
    print("step starts (us):", [round((x - t0) / 1e3, 1) for x in g])


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
