"""Calibration of the ResNet oracle tests' relative-L2 bounds (tests/test_resnet_gpu.py REL_BOUND,
E2E_FC_BOUND): every block case and the end-to-end fc gradients against the fp32 PyTorch reference,
in row mode (the tests' mode) and slot mode (the training default), per tensor.

    python tools/debug/resnet_oracle_rel.py
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from tensorflow_distributed_amd import _native  # noqa: E402

import test_resnet_gpu as T  # noqa: E402

CASES = [(50, 0, 16), (50, 1, 16), (50, 3, 16), (50, 13, 4), (18, 0, 16), (18, 2, 16)]


def main():
    _native.require()
    cuda = torch.device("cuda", 0)
    old = torch.ops.tfd.bn_part_slots()
    try:
        for slots in (0, 4):
            torch.ops.tfd.set_bn_part_slots(slots)
            worst = {}
            for depth, bi, hw in CASES:
                pairs = T.block_case(cuda, depth, bi, hw)
                rels = {k: round(T.rel_l2(a, b), 5) for k, (a, b) in pairs.items()}
                norms = {k: float("%.3g" % b.double().norm().item()) for k, (a, b) in pairs.items()}
                for k, r in rels.items():
                    kd = T._kind(k)
                    worst[kd] = max(worst.get(kd, 0.0), r)
                print(json.dumps({"slots": slots, "case": [depth, bi, hw], "rel_l2": rels, "ref_norm": norms}), flush=True)
            for depth, nb, hw in ((18, 4, 64), (50, 4, 64), (18, 8, 128), (50, 8, 128), (50, 16, 128)):
                from tensorflow_distributed_amd.models.resnet import ResNet

                torch.manual_seed(0)
                m = ResNet(depth, num_classes=16, device=cuda, seed=1, width=16, zero_init_residual=False)
                x = torch.randn(nb, hw, hw, 3)
                lab = torch.randint(0, 16, (nb,), dtype=torch.int32)
                loss, _ = m.loss(x.to(cuda), lab.to(cuda))
                loss.backward()
                torch.cuda.synchronize()
                lref, P = T._ref_forward(m, x.to(torch.bfloat16).float(), lab)
                lref.backward()
                r = {"loss": abs(loss.item() - lref.item()) / lref.item(),
                     "fc": T.rel_l2(m.fp.g("fc").float().cpu(), P["fc"].grad),
                     "fc/bias": T.rel_l2(m.fp.g("fc/bias").float().cpu(), P["fc/bias"].grad)}
                key = "e2e_fc_%d_%d" % (nb, hw)
                worst[key] = max(worst.get(key, 0.0), r["fc"], r["fc/bias"])
                print(json.dumps({"slots": slots, "e2e": [depth, nb, hw], "rel": {k: round(v, 5) for k, v in r.items()}}),
                      flush=True)
            print(json.dumps({"slots": slots, "worst": worst}), flush=True)
    finally:
        torch.ops.tfd.set_bn_part_slots(old)


if __name__ == "__main__":
    main()
