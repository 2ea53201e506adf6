"""Graph replay vs eager at production weight-gradient routing (finetune, B = 256): per-segment
count of master weights that moved apart by > 1e-5, for eager vs eager and eager vs graph, to tell
atomic-order noise (scattered, present in both) from a stale captured buffer (whole segments).

    python tools/graph_diag.py [--B 256] [--steps 5]"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_graph_gpu import _batches, _finetune  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from jumbo_mae_tpu_amd.runtime.graph import GraphedTrainStep

    data = _batches(a.steps + 3, B=a.B)
    m1, t1 = _finetune(0.0, 0.0)
    m2, t2 = _finetune(0.0, 0.0)
    m3, t3 = _finetune(0.0, 0.0)
    gs = GraphedTrainStep(t2, [data[0]], warmup=3)
    for _ in range(3):
        t1.train_step([data[0]])
        t3.train_step([data[0]])
    torch.cuda.synchronize()
    for i in range(1, a.steps + 1):
        la = t1.train_step([data[i]])["loss"].item()
        lc = t3.train_step([data[i]])["loss"].item()
        lb = gs([data[i]])["loss"].item()
        print(f"step {i}: eager {la:.6f} eager2 {lc:.6f} graph {lb:.6f}")
    torch.cuda.synchronize()
    tot = {"eager2": 0, "graph": 0}
    for seg in m1.store.segments:
        sl = slice(seg.offset, seg.offset + seg.numel)
        row = []
        for name, m in (("eager2", m3), ("graph", m2)):
            d = (m1.store.master[sl] - m.store.master[sl]).abs()
            n = int((d > 1e-5).sum().item())
            tot[name] += n
            row.append(f"{name} {n:7d} max {d.max().item():.2e}")
        print(f"{seg.key:48s} {seg.numel:9d}  " + "  ".join(row))
    print("total", tot, "of", m1.store.total)


if __name__ == "__main__":
    main()
