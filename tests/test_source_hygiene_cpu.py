"""Kernel-source hygiene: production kernels carry no timing-only experiment switches (arms that
produce wrong results on purpose) and no losing A/B arms of the MNIST step; the A/B evidence
lives in profiles/ab_*.log and docs/DESIGN.md, not in the kernels."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = sorted(glob.glob(os.path.join(ROOT, "csrc", "**", "*.hip"), recursive=True)
                 + glob.glob(os.path.join(ROOT, "csrc", "**", "*.h"), recursive=True)
                 + glob.glob(os.path.join(ROOT, "csrc", "**", "*.cpp"), recursive=True))


def test_no_wrong_result_experiment_switches():
    bad = []
    for p in SOURCES:
        for i, ln in enumerate(open(p), 1):
            if re.search(r"TFD_(EXP|DIAG)_", ln):
                bad.append(f"{os.path.relpath(p, ROOT)}:{i}: {ln.strip()}")
    assert not bad, "\n".join(bad)


def test_mnist_kernels_have_no_ab_switches():
    """The bf16 MNIST step's kernels keep exactly one configurable switch: the phase-clock
    profiling build (TFD_STAMP, off by default, no effect on results)."""
    src = open(os.path.join(ROOT, "csrc", "kernels", "mnist.hip")).read()
    switches = set(re.findall(r"#if(?:n?def)?\s+!?\(?(TFD_\w+)", src))
    assert switches <= {"TFD_STAMP"}, switches
    assert len(src.splitlines()) < 1700


def test_removed_engine_paths_stay_removed():
    eng = open(os.path.join(ROOT, "csrc", "runtime", "mnist_engine.cpp")).read()
    for name in ("set_fc_adam", "set_conv_unfused", "pbf_alt", "mnist_backward_a_adam"):
        assert name not in eng, name
