"""Per-step kernel timeline from a rocprofv3 kernel-trace database (rocpd sqlite).

    python tools/prof_timeline.py gpurun_out/prof/run_results.db [--anchor mnist_adam_kernel]

Splits the trace into steps at each end of the anchor kernel (the step's last kernel), then prints,
per kernel of a step, the median start / end offsets from the previous step's anchor end and the
median gap to the kernel that finished just before it started. This shows where a step's time goes
that a per-kernel duration table cannot: launch gaps and the overlap of forked streams.
"""
import argparse
import sqlite3
import statistics
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="mnist_adam_kernel")
    ap.add_argument("--skip", type=int, default=20, help="steps to skip at the start (warmup)")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    rows = [(n.replace("tfd::(anonymous namespace)::", "").split("(")[0], s, e) for n, s, e in rows]
    steps, cur, t0 = [], [], None
    for n, s, e in rows:
        if t0 is None:
            if a.anchor in n:
                t0 = e
            continue
        cur.append((n, s - t0, e - t0))
        if a.anchor in n:
            steps.append(cur)
            cur, t0 = [], e
    steps = steps[a.skip:]
    if not steps:
        print("no complete steps found")
        return 1
    sig = [tuple(k[0] for k in st) for st in steps]
    common = max(set(sig), key=sig.count)
    sel = [st for st, sg in zip(steps, sig) if sg == common]
    print(f"{len(steps)} steps, {len(sel)} with the common kernel sequence; times in us from the previous "
          f"step's {a.anchor} end")
    print(f"{'kernel':28s} {'start':>8s} {'end':>8s} {'dur':>7s} {'gap':>7s}")
    for i, name in enumerate(common):
        st = statistics.median(s[i][1] for s in sel) / 1e3
        en = statistics.median(s[i][2] for s in sel) / 1e3
        # gap: start minus the latest end among kernels that ended before this one started
        gaps = []
        for s in sel:
            prev = [k[2] for j, k in enumerate(s) if j != i and k[2] <= s[i][1]]
            gaps.append((s[i][1] - (max(prev) if prev else 0)) / 1e3)
        print(f"{name[:28]:28s} {st:8.2f} {en:8.2f} {en - st:7.2f} {statistics.median(gaps):7.2f}")
    tot = statistics.median(s[-1][2] for s in sel) / 1e3
    print(f"step (anchor end to anchor end): {tot:.2f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
