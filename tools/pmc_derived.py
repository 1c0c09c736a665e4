"""Derived per-kernel metrics from the pass tables that scripts/gpu_run.sh pmc= steps print
(tools/pmc_summary.py output, one table per counter pass, concatenated).

    python tools/pmc_derived.py profiles/pmc_kernels_r3_base.txt [--clock_ghz 2.4]

Columns:
  us            kernel duration (mean of the passes; counter collection inflates it a little)
  mfma_busy%    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x clock): share of the chip's
                matrix-pipe cycles spent in MFMAs (SQ_VALU_MFMA_BUSY_CYCLES sums busy cycles over
                SIMDs: 16 per v_mfma_f32_16x16x32_bf16 = 16 K FLOP, checked against
                SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP). At the max clock this is a lower bound.
  TFLOP/s       SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP / duration
  lds_conf/inst SQ_LDS_BANK_CONFLICT (extra LDS cycles) per LDS wave-instruction
  wait%         SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  GB/s          (2 x FETCH_SIZE + WRITE_SIZE) / duration: FETCH_SIZE reports half the bytes of
                wide streaming reads on gfx950 (MI355X_MICROARCH.md, HBM), so it is doubled; an
                upper-bound estimate for kernels whose reads are not 16-B streams
  L2 hit%       TCC_HIT / (TCC_HIT + TCC_MISS)
"""
import argparse
import collections
import math


def parse(path):
    vals = collections.defaultdict(dict)
    durs = collections.defaultdict(list)
    cols = None
    for line in open(path):
        if line.startswith("#") or not line.strip():
            continue
        parts = line.split()
        if parts[0] == "kernel":
            cols = parts[2:]
            continue
        if cols is None:
            continue
        name = line[:40].strip().replace("void ", "")  # fixed-width name column (templates hold spaces)
        nums = parts[-(len(cols) + 1):]
        try:
            d = float(nums[0])
            xs = [float(v) for v in nums[1:]]
        except ValueError:
            continue
        durs[name].append(d)
        for c, v in zip(cols, xs):
            vals[name][c] = v
    return vals, {k: sum(v) / len(v) for k, v in durs.items()}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--clock_ghz", type=float, default=2.4)
    a = ap.parse_args(argv)
    vals, dur = parse(a.path)

    def g(k, c):  # pmc_summary.py truncates counter names to 16 characters
        return vals[k].get(c, vals[k].get(c[:16], math.nan))

    hdr = f"{'kernel':34s} {'us':>6s} {'mfma_busy%':>10s} {'TFLOP/s':>8s} {'lds_conf/inst':>13s} {'wait%':>6s} {'GB/s':>7s} {'L2hit%':>7s}"
    print(hdr)
    for k in sorted(dur, key=lambda k: -dur[k]):
        if k.startswith("__amd") or k.startswith("void"):
            continue
        us = dur[k]
        cyc = us * 1e-6 * a.clock_ghz * 1e9
        busy = g(k, "SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * cyc) * 100
        tf = g(k, "SQ_INSTS_VALU_MFMA_MOPS_BF16") * 512 / (us * 1e-6) / 1e12
        lds = g(k, "SQ_LDS_BANK_CONFLICT") / g(k, "SQ_INSTS_LDS") if g(k, "SQ_INSTS_LDS") else math.nan
        wait = g(k, "SQ_WAIT_ANY") / g(k, "SQ_WAVE_CYCLES") * 100
        gbs = (2 * g(k, "FETCH_SIZE") + g(k, "WRITE_SIZE")) * 1e3 / (us * 1e-6) / 1e9
        hit = g(k, "TCC_HIT_sum") / (g(k, "TCC_HIT_sum") + g(k, "TCC_MISS_sum")) * 100
        print(f"{k:34s} {us:6.2f} {busy:10.1f} {tf:8.0f} {lds:13.2f} {wait:6.1f} {gbs:7.0f} {hit:7.1f}")


if __name__ == "__main__":
    main()
