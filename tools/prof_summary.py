"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a per-kernel table.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--skip N]
Prints: calls, mean/median us, total us, share, VGPR/SGPR/LDS per kernel, and the per-step sum
for the kernels that appear once per training step.
"""
import argparse
import sqlite3
import statistics
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-calls", type=int, default=10, help="kernels called fewer times are setup noise")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, end-start, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, grid_x, grid_y, grid_z,"
                     " workgroup_x from kernels").fetchall()
    by = {}
    for name, d, v, av, sg, lds, gx, gy, gz, wx in rows:
        e = by.setdefault(name, {"d": [], "meta": (v, av, sg, lds, gx * gy * gz // max(wx, 1))})
        e["d"].append(d / 1000.0)
    tot = sum(sum(e["d"]) for e in by.values() if len(e["d"]) >= a.min_calls)
    print(f"{'kernel':60s} {'calls':>6s} {'mean_us':>8s} {'med_us':>8s} {'total_us':>10s} {'share':>6s} "
          f"{'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'lds':>6s} {'wgs':>6s}")
    step = 0.0
    for name, e in sorted(by.items(), key=lambda kv: -sum(kv[1]["d"])):
        if len(e["d"]) < a.min_calls:
            continue
        d = e["d"]
        v, av, sg, lds, wgs = e["meta"]
        short = name.replace("tfd::(anonymous namespace)::", "")[:60]
        med = statistics.median(d)
        step += med
        print(f"{short:60s} {len(d):6d} {sum(d)/len(d):8.2f} {med:8.2f} {sum(d):10.1f} {sum(d)/tot*100:5.1f}% "
              f"{v:5d} {av:5d} {sg:5d} {lds:6d} {wgs:6d}")
    print(f"sum of per-kernel medians (one step if each kernel runs once per step): {step:.2f} us")


if __name__ == "__main__":
    sys.exit(main())
