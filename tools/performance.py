"""Regenerate the reference's ``performance`` table (``/root/reference/performance:1-6``: global
steps vs training time vs validation accuracy at Adam lr 0.01, 1 PS + 2 sync workers, 128 images
per worker step) on this framework.

    python tools/performance.py [--num_workers 2] [--num_gpus 0] [--steps 40,60,80,100,120] [--out performance.md]

One cluster run to the last milestone; the chief pauses the clock and runs the 5 x 1000 validation
pass at every milestone (``--eval_at_steps``), printing one table row each.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tensorflow_distributed_amd import launch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--num_ps", type=int, default=1)
    ap.add_argument("--num_workers", type=int, default=2)
    ap.add_argument("--num_gpus", type=int, default=0)
    ap.add_argument("--steps", default="40,60,80,100,120")
    ap.add_argument("--data_dir", default="/tmp/mnist-data")
    ap.add_argument("--out", default="")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args(argv)
    last = max(int(s) for s in a.steps.split(","))
    args = [f"--train_steps={last}", f"--eval_at_steps={a.steps}", f"--num_gpus={a.num_gpus}", "--quiet",
            f"--data_dir={a.data_dir}"] + a.extra
    r = launch.launch(a.num_ps, a.num_workers, args, echo=False, timeout_s=7200)
    chief = "".join(v for k, v in r["outputs"].items() if k.startswith("worker:0#"))
    if not r["ok"]:
        print(chief)
        return 1
    table = chief[chief.index("Steps ,Time ,Accuracy, Learning rate"):]
    print(table, end="")
    if a.out:
        with open(a.out, "w") as f:
            f.write(table)
    return 0


if __name__ == "__main__":
    sys.exit(main())
