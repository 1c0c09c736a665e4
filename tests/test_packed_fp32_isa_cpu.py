"""Packed-fp32 nondeterminism: what the built code says.

Round 2 found that a build WITH packed fp32 VALU ops (``v_pk_fma_f32``, the default instruction
selection) gave repeat-to-repeat differences in the VALU conv1 kernel (``conv1_pool_fwd``) only
when four processes time-sliced one GPU -- never in one process, never in the default build
(``profiles/packed_fp32_probe_r2.log``), and only in the second channel of a packed channel pair.

The kernel-side explanation that fits that signature is a packed instruction reading a register
half that nothing in the kernel wrote: its value would be whatever the previous wave on that SIMD
left, stable when every wave is this kernel, different when other processes' waves run between.
This test rules it out in the code object: it compiles the kernels with packed fp32 ops, builds
the control-flow graph of the SLP-vectorised ``head_kernel`` (the VALU ``conv1_pool_fwd`` is gone) and runs
a must-be-written dataflow over the VGPRs (a packed operand counts only the halves its
``op_sel``/``op_sel_hi`` select). No path reads a VGPR before writing it, and the kernel's LDS
use is barrier-separated (stage -> __syncthreads -> read, no LDS reuse), so the divergence is
not an uninitialised register or an LDS race in this kernel; what remains is the wave
save/restore across processes of the packed-fp32 path, which the build avoids
(``_build.py``: ``-packed-fp32-ops``). docs/DESIGN.md section 6.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
SRC = os.path.join(ROOT, "csrc", "kernels", "mnist.hip")

pytestmark = pytest.mark.skipif(not (os.path.exists(os.path.join(LLVM, "llvm-objdump"))
                                     and os.path.exists("/opt/rocm/bin/hipcc")), reason="no ROCm toolchain")

STORES = ("global_store", "buffer_store", "ds_write", "flat_store", "global_atomic", "buffer_atomic", "scratch_store")
LOADS = ("global_load", "buffer_load", "ds_read", "flat_load", "scratch_load")


def _regs(tok):
    out = []
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", tok):
        out += [int(m.group(3))] if m.group(3) else list(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def _defs_uses(code):
    """(VGPRs written, VGPRs read) of one instruction; packed ops read only the selected halves."""
    op, _, args = code.partition(" ")
    sel = re.search(r"op_sel:\[([01,]+)\]", args)
    sel_hi = re.search(r"op_sel_hi:\[([01,]+)\]", args)
    args = re.sub(r"\s(op_sel|op_sel_hi|neg_lo|neg_hi):\[[^\]]*\]", "", args)
    ops = [a.strip() for a in re.split(r",(?![^\[]*\])", args.strip())] if args.strip() else []
    if op.startswith(STORES) or op.startswith("s_"):
        return [], sum((_regs(a) for a in ops), [])
    if op.startswith(("v_cmp", "v_readfirstlane", "v_readlane")) and not op.startswith("v_cmpx"):
        return [], sum((_regs(a) for a in ops[1:]), [])
    if not (op.startswith(LOADS) or op.startswith("v_")) or not ops:
        return [], []
    uses = []
    if op.startswith("v_pk_") and "v_pk_mov" not in op:
        lo = [int(x) for x in sel.group(1).split(",")] if sel else [0, 0, 0]
        hi = [int(x) for x in sel_hi.group(1).split(",")] if sel_hi else [1, 1, 1]
        for i, a in enumerate(ops[1:]):
            r = _regs(a)
            if len(r) == 2 and i < len(lo):
                uses += [r[h] for h in sorted({lo[i], hi[i]})]
            else:
                uses += r
    elif op.startswith("v_pk_mov_b32"):  # D.lo = S0[op_sel[0]], D.hi = S1[op_sel[1]]
        s = [int(x) for x in sel.group(1).split(",")] if sel else [0, 1]
        for i, a in enumerate(ops[1:3]):
            r = _regs(a)
            uses += [r[s[i]]] if len(r) == 2 else r
    else:
        uses = sum((_regs(a) for a in ops[1:]), [])
    return _regs(ops[0]), uses


def _parse(asm, func):
    ins, on = [], False
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            on = m.group(1) == func
            continue
        if not on or not line.startswith("\t"):
            continue
        code, _, cmt = line.partition("//")
        am = re.match(r"\s*([0-9A-F]+):", cmt)
        if code.strip() and am:
            tm = re.search(r"<[^>]*\+0x([0-9a-f]+)>", cmt)
            ins.append((int(am.group(1), 16), code.strip(), int(tm.group(1), 16) if tm else None))
    return ins


def maybe_uninitialised_reads(ins, init=frozenset([0])):
    """Reads of VGPRs that are not written on every path from the kernel entry (v0 = work-item ids)."""
    base = ins[0][0]
    at = {a: i for i, (a, _, _) in enumerate(ins)}
    leaders = {0}
    for i, (_, c, t) in enumerate(ins):
        if c.startswith(("s_branch", "s_cbranch")):
            if t is not None and base + t in at:
                leaders.add(at[base + t])
            leaders.add(i + 1)
    starts = sorted(x for x in leaders if x < len(ins))
    blocks = [(s, starts[k + 1] if k + 1 < len(starts) else len(ins)) for k, s in enumerate(starts)]
    bid = {s: k for k, (s, _) in enumerate(blocks)}
    succ = {k: [] for k in range(len(blocks))}
    for k, (s, e) in enumerate(blocks):
        _, c, t = ins[e - 1]
        if c.startswith("s_endpgm"):
            continue
        if c.startswith(("s_branch", "s_cbranch")):
            succ[k].append(bid[at[base + t]])
        if not c.startswith("s_branch") and e < len(ins):
            succ[k].append(bid[e])
    pred = {k: [p for p in succ if k in succ[p]] for k in succ}
    full = frozenset(range(512))
    IN = {k: (frozenset(init) if k == 0 else full) for k in succ}
    OUT = {}

    def run(k):
        w, bad = set(IN[k]), []
        for i in range(*blocks[k]):
            d, u = _defs_uses(ins[i][1])
            bad += [(ins[i][0], r, ins[i][1]) for r in u if r not in w]
            w |= set(d)
        return frozenset(w), bad

    changed = True
    while changed:
        changed = False
        for k in succ:
            if k:
                new = frozenset.intersection(*[OUT.get(p, full) for p in pred[k]]) if pred[k] else frozenset(init)
                if new != IN[k]:
                    IN[k], changed = new, True
            o, _ = run(k)
            if OUT.get(k) != o:
                OUT[k], changed = o, True
    return [b for k in succ for b in run(k)[1]]


@pytest.fixture(scope="module")
def packed_asm(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("pk") / "mnist_pk.co")
    subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output",
                    "-O3", "-std=c++17", "-I", os.path.join(ROOT, "csrc"), "-ffp-contract=fast", "-munsafe-fp-atomics",
                    "-c", SRC, "-o", out], check=True, capture_output=True)
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", out], check=True,
                          capture_output=True, text=True).stdout


def test_packed_build_reads_no_unwritten_vgpr(packed_asm):
    """The SLP-vectorised head kernel in the packed build (the VALU conv1 kernel that showed the
    divergence was replaced in round 4 by conv1 on the matrix core inside conv12_fwd_lds, whose
    packed build has no packed FMAs). The dataflow model covers VALU / LDS / flat-global
    instructions, which is what these two kernels are made of -- not the buffer-load GEMM cores."""
    func = next(m for m in re.findall(r"^[0-9a-f]+ <(.+)>:$", packed_asm, re.M) if "head_kernel" in m)
    ins = _parse(packed_asm, func)
    assert len(ins) > 200
    assert any(c.startswith("v_pk_fma_f32") for _, c, _ in ins), "expected packed fp32 FMAs in this build"
    bad = maybe_uninitialised_reads(ins)
    assert not bad, [f"{a:x} v{r}: {c}" for a, r, c in bad[:10]]
    conv12 = next(m for m in re.findall(r"^[0-9a-f]+ <(.+)>:$", packed_asm, re.M) if "conv12_fwd_lds" in m)
    assert not any(c.startswith("v_pk_fma_f32") for _, c, _ in _parse(packed_asm, conv12))


def test_analysis_flags_an_unwritten_packed_half():
    """The checker itself: a packed FMA whose src0 high half (v3) was never written is flagged; with
    op_sel_hi:[0,1,1] (src0's low half feeds both results) it is not."""
    body = [(0x0, "v_mov_b32_e32 v2, 1.0", None), (0x4, "v_mov_b32_e32 v4, 1.0", None),
            (0x8, "v_mov_b32_e32 v5, 1.0", None), (0xc, "v_pk_fma_f32 v[6:7], v[2:3], v[4:5], v[4:5]", None),
            (0x14, "s_endpgm", None)]
    bad = maybe_uninitialised_reads(body)
    assert [r for _, r, _ in bad] == [3]
    body[3] = (0xc, "v_pk_fma_f32 v[6:7], v[2:3], v[4:5], v[4:5] op_sel_hi:[0,1,1]", None)
    assert maybe_uninitialised_reads(body) == []
