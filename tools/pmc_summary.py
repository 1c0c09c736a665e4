"""Per-kernel averages of rocprofv3 PMC counters from a rocpd sqlite database.

    python tools/pmc_summary.py gpurun_out/pmc1/<...>/run_results.db
"""
import sqlite3
import sys
from collections import defaultdict


def main(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    q = f"select {name_col}, counter_name, value, dispatch_id from counters_collection"
    acc = defaultdict(lambda: defaultdict(list))
    for kname, cname, val, did in c.execute(q):
        acc[kname][cname].append(val)
    dur = defaultdict(list)
    for n, d in c.execute("select name, end-start from kernels"):
        dur[n].append(d / 1000.0)
    counters = sorted({cn for k in acc.values() for cn in k})
    print("kernel".ljust(40), "dur_us".rjust(8), " ".join(cn[:16].rjust(16) for cn in counters))
    for kname in sorted(acc, key=lambda k: -sum(dur.get(k, [0])) / max(len(dur.get(k, [1])), 1)):
        if len(dur.get(kname, [])) < 5:
            continue
        d = sum(dur[kname]) / len(dur[kname])
        short = kname.replace("tfd::(anonymous namespace)::", "").split("(")[0][:40]
        vals = [sum(acc[kname][cn]) / max(len(acc[kname][cn]), 1) if cn in acc[kname] else float("nan") for cn in counters]
        print(short.ljust(40), f"{d:8.2f}", " ".join(f"{v:16.4g}" for v in vals))


if __name__ == "__main__":
    main(sys.argv[1])
