"""The cross-device IPC protocol's memory ordering, pinned in the built gfx950 code object.

The one-shot collectives (csrc/comm/ipc_allreduce.hip) hand staging data to peer GPUs over xGMI.
With two ranks on one device L2 coherence hides a missing fence, so the one-GPU tests cannot
catch one; the code object can. For every rank count W = 2..8 of each collective kernel this
test disassembles the object that is linked into ``_C.so`` (``build/native/ipc_allreduce.hip.o``,
or the same source compiled with the build's flags) and checks the START barrier and the call
counter:

* release: the START flag store to a peer is a system-scope store (``sc0 sc1``) preceded by a
  system-scope L2 write-back (``buffer_wbl2 sc0 sc1``) and a ``s_waitcnt vmcnt(0)`` that drains it,
  with no store between them (the staging stores are visible before the flag). The compiler
  drops the wait after the write-back of a release store whose vmcnt it believes empty
  (MI355X_MICROARCH.md, "Compiler hazard"); the kernel's explicit fence + inline-asm wait is what
  this pins;
* acquire: after the time-bounded spin on the peers' flags (``sc0 sc1`` loads), a system-scope
  invalidate (``buffer_inv sc0 sc1``) and its ``vmcnt(0)`` come before the workgroup barrier that
  releases the block to read the peers' staging;
* the call-counter bump is a system-scope atomic preceded by a system-scope write-back.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
SRC = os.path.join(ROOT, "csrc", "comm", "ipc_allreduce.hip")
OBJ = os.path.join(ROOT, "build", "native", "ipc_allreduce.hip.o")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-objdump")), reason="no ROCm llvm tools")

STORE = re.compile(r"^\s*(global_store|global_atomic|buffer_store|buffer_atomic|flat_store|flat_atomic)")


def _disassemble(co):
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                         capture_output=True, text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
        elif cur is not None and line.strip():
            funcs[cur].append(line.split("//")[0].strip())
    return funcs


def _compile(src, root, out):
    subprocess.run(["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "--no-gpu-bundle-output",
                    "-O3", "-std=c++17", "-I", os.path.join(root, "csrc"), "-ffp-contract=fast", "-munsafe-fp-atomics",
                    "-c", src, "-o", out], check=True, capture_output=True)
    return out


def _device_object(tmp):
    """gfx950 code object of the IPC kernels: unbundled from the linked build object when present,
    else compiled from the source with the build's device flags."""
    if os.path.exists(OBJ):
        local = os.path.join(tmp, "ipc.o")
        shutil.copy(OBJ, local)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], check=True, capture_output=True,
                       cwd=tmp)
        cands = [f for f in os.listdir(tmp) if "gfx950" in f]
        assert cands, os.listdir(tmp)
        return os.path.join(tmp, cands[0])
    return _compile(SRC, ROOT, os.path.join(tmp, "ipc.co"))


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    tmp = str(tmp_path_factory.mktemp("isa"))
    return _disassemble(_device_object(tmp))


def _kernel(funcs, name, w):
    key = [k for k in funcs if name in k and f"ILi{w}E" in k]
    assert len(key) == 1, (name, w, [k for k in funcs if name in k])
    return funcs[key[0]]


@pytest.mark.parametrize("name", ["ipc_allreduce_kernel", "ipc_reduce_scatter_kernel", "ipc_all_gather_kernel"])
@pytest.mark.parametrize("w", [2, 3, 4, 5, 6, 7, 8])
def test_start_barrier_release_acquire(kernels, name, w):
    body = _kernel(kernels, name, w)
    spin = [i for i, s in enumerate(body) if s.startswith("s_sleep")]
    assert spin, "no time-bounded spin (s_sleep) in the START barrier"
    s0 = spin[0]
    # release: the last system-scope store before the spin is the flag store
    stores = [i for i in range(s0) if body[i].startswith("global_store") and body[i].endswith("sc0 sc1")]
    assert stores, "no system-scope flag store before the spin"
    st = stores[-1]
    # the nearest system-scope write-back that a vmcnt(0) wait drains before the flag store, with no
    # vector-memory store or atomic in between (loads of peer pointers may sit there; a second,
    # redundant wbl2 that the compiler emits for the release store itself is allowed)
    drained = [i for i in range(st) if body[i].startswith("buffer_wbl2 sc0 sc1")
               and any(x.startswith("s_waitcnt") and "vmcnt(0)" in x for x in body[i + 1:st])]
    assert drained, "flag store without a drained system-scope write-back before it"
    between = body[drained[-1] + 1:st]
    assert not [x for x in between if STORE.match(x)], f"a store between the drained wbl2 and the flag store: {between}"
    # the polls are system-scope loads
    polls = [s for s in body[max(0, s0 - 40):s0 + 10] if s.startswith("global_load_dword")]
    assert polls and all(s.endswith("sc0 sc1") for s in polls), polls
    # acquire: buffer_inv sc0 sc1 + vmcnt(0) after the spin, before the next workgroup barrier
    bar = [i for i in range(s0, len(body)) if body[i].startswith("s_barrier")]
    assert bar, "no workgroup barrier after the START spin"
    seg = body[s0:bar[0]]
    inv = [i for i, s in enumerate(seg) if s.startswith("buffer_inv sc0 sc1")]
    assert inv, f"no system-scope invalidate between the spin and the barrier: {seg[-12:]}"
    assert any(s.startswith("s_waitcnt") and "vmcnt(0)" in s for s in seg[inv[-1] + 1:]), seg[inv[-1]:]


@pytest.mark.parametrize("name", ["ipc_allreduce_kernel", "ipc_reduce_scatter_kernel", "ipc_all_gather_kernel"])
def test_call_counter_bump_is_system_release(kernels, name):
    body = _kernel(kernels, name, 8)
    atom = [i for i, s in enumerate(body) if s.startswith("global_atomic_add") and s.endswith("sc1") and "sc0" not in s.split()[-1]]
    assert atom, "no system-scope call-counter atomic"
    i = atom[-1]
    prior = body[max(0, i - 6):i]
    assert any(s.startswith("buffer_wbl2 sc0 sc1") for s in prior), prior


def test_checker_rejects_a_missing_release(tmp_path):
    """Mutation check of the checker itself: the same source without the explicit release fence
    (and with a relaxed flag store) must fail the release assertion."""
    root = tmp_path / "mut"
    shutil.copytree(os.path.join(ROOT, "csrc"), root / "csrc")
    src = root / "csrc" / "comm" / "ipc_allreduce.hip"
    text = src.read_text()
    fence = '    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");\n    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");\n    flag_store'
    assert fence in text
    text = text.replace(fence, "    flag_store").replace(
        "__hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM)",
        "__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)")
    src.write_text(text)
    funcs = _disassemble(_compile(str(src), str(root), str(tmp_path / "mut.co")))
    with pytest.raises(AssertionError, match="drained system-scope write-back"):
        test_start_barrier_release_acquire(funcs, "ipc_allreduce_kernel", 8)
