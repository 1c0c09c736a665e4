"""Where do a kernel's prologue loads get waited for? Compiles a HIP source for gfx950 with
--save-temps (into a scratch directory) and prints, per kernel, the instruction stream up to its
first MFMA (or the first N lines) reduced to vector loads (global / buffer / LDS-DMA), s_waitcnt
vmcnt, barriers and branches, so a wait issued in the middle of a load batch -- an exec-masked load
merged by a phi, a hoisted compare, a dependent index chain -- shows up before any timing run.
(The round-6 MNIST finds: docs/DESIGN.md §8.)

    python tools/isa_waits.py csrc/kernels/mnist.hip [--kernel fc1_fwd] [--lines 400]
    python tools/isa_waits.py csrc/kernels/mnist.hip --masked   # per kernel: exec-masked loads that wait
                                                               # inside their branch (each a serial round trip)
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-O3", "-fPIC", "-std=c++17", "-x", "hip", "--offload-arch=gfx950", "-D__HIP_PLATFORM_AMD__=1",
         "-ffp-contract=fast", "-munsafe-fp-atomics", "-Wno-unused-result", "-Xclang", "-target-feature", "-Xclang",
         "-packed-fp32-ops", "--save-temps"]
KEEP = re.compile(r"^\s*(global_load|buffer_load|global_load_lds|s_waitcnt vmcnt|s_barrier|s_cbranch|v_mfma)")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--kernel", default="", help="substring of the kernel's mangled name")
    ap.add_argument("--lines", type=int, default=600, help="asm lines scanned per kernel when it has no MFMA")
    ap.add_argument("--masked", action="store_true", help="count exec-masked branches (s_and_saveexec ... s_or_b64 exec)"
                    " that hold a load AND a wait: the conv1 weight reads of round 6 were ten of these in a row")
    a = ap.parse_args(argv)
    src = os.path.abspath(a.src)
    with tempfile.TemporaryDirectory() as d:
        cmd = [os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), *FLAGS, "-I",
               os.path.join(ROOT, "csrc"), "-c", src, "-o", os.path.join(d, "k.o")]
        p = subprocess.run(cmd, cwd=d, capture_output=True, text=True)
        if p.returncode:
            sys.exit(p.stderr[-2000:])
        asm = open(glob.glob(os.path.join(d, "*gfx950*.s"))[0]).read().splitlines()
    if a.masked:
        return masked_waits(asm, a.kernel)
    starts = [i for i, ln in enumerate(asm) if re.match(r"^_Z\S+:", ln) and "GLOBAL__N" in ln or
              re.match(r"^_Z\S+:\s", ln)]
    for s in starts:
        name = asm[s].split(":")[0]
        if a.kernel and a.kernel not in name:
            continue
        end = next((j for j in range(s + 1, len(asm)) if asm[j].strip().startswith("s_endpgm")), len(asm))
        body = asm[s + 1:end]
        mf = next((j for j, ln in enumerate(body) if "v_mfma" in ln), None)
        stop = mf + 1 if mf is not None else min(len(body), a.lines)
        loads = 0
        print(f"== {name}  ({end - s} lines; first MFMA at +{mf})")
        for j, ln in enumerate(body[:stop]):
            if not KEEP.match(ln):
                continue
            t = ln.strip()
            if "load" in t.split()[0]:
                loads += 1
            print(f"  +{j:5d} [{loads:3d} loads] {t[:90]}")


def masked_waits(asm, kernel=""):
    cur, counts = None, {}
    for i, ln in enumerate(asm):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            cur = m.group(1)
        if cur is None or "s_and_saveexec" not in ln or (kernel and kernel not in cur):
            continue
        blk = asm[i:i + 12]
        end = next((j for j, b in enumerate(blk) if "s_or_b64 exec" in b), None)
        if end is None:
            continue
        inner = "\n".join(blk[:end])
        if re.search(r"ds_read|global_load|buffer_load", inner) and "s_waitcnt" in inner:
            counts[cur] = counts.get(cur, 0) + 1
    for k, v in sorted(counts.items(), key=lambda x: -x[1]):
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
