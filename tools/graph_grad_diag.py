"""One-step gradients of a graph replay vs an eager step from identical weights (finetune, B=256,
production weight-gradient routing); prints the segments whose gradients disagree.

    python tools/graph_grad_diag.py [--order graph_first|eager_first]"""

import argparse
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
from test_graph_gpu import _batches, _finetune  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="eager_first")
    ap.add_argument("--B", type=int, default=256)
    a = ap.parse_args()
    from jumbo_mae_tpu_amd.runtime.graph import GraphedTrainStep

    data = _batches(3, B=a.B)
    m1, t1 = _finetune(0.0, 0.0)
    m2, t2 = _finetune(0.0, 0.0)
    gs = GraphedTrainStep(t2, [data[0]], warmup=3, restore=True)
    for i in (1, 2):
        if a.order == "eager_first":
            la = t1.train_step([data[i]])["loss"].item()
            lb = gs([data[i]])["loss"].item()
        else:
            lb = gs([data[i]])["loss"].item()
            la = t1.train_step([data[i]])["loss"].item()
        torch.cuda.synchronize()
        bad = []
        for seg in m1.store.segments:
            sl = slice(seg.offset, seg.offset + seg.numel)
            g1, g2 = m1.store.grad[sl], m2.store.grad[sl]
            err = (g1 - g2).abs()
            sc = g1.abs().max().item()
            if err.max().item() > 2e-2 * sc + 1e-7:
                nbad = int((err > 2e-2 * sc + 1e-7).sum().item())
                idx = int(err.argmax().item())
                bad.append(f"{seg.key} shape {seg.shape} bad {nbad}/{seg.numel} first-max at {idx} "
                           f"g1 {g1[idx].item():.3e} g2 {g2[idx].item():.3e}")
        print(f"[{a.order} {os.environ.get('JMAE_STORE_GRADS', '-')}/{os.environ.get('JMAE_PAIR_WGRAD', '-')}] "
              f"step {i} loss {la:.6f} {lb:.6f}; bad segments: {len(bad)}", flush=True)
        for b in bad:
            print("   ", b, flush=True)


if __name__ == "__main__":
    main()
