"""Graph replay vs eager train steps on a tiny finetune model: per-parameter max |dw| (diagnostic)."""
import sys

import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_graph_gpu import _batches, _finetune  # noqa: E402

from jumbo_mae_tpu_amd.runtime.graph import GraphedTrainStep  # noqa: E402

data = _batches(8)
m1, t1 = _finetune(0.0, 0.0)
m2, t2 = _finetune(0.0, 0.0)
gs = GraphedTrainStep(t2, [data[0]], warmup=3)
for _ in range(3):
    t1.train_step([data[0]])
torch.cuda.synchronize()
print("after warmup max|dw|", (m1.store.master - m2.store.master).abs().max().item())
for i in range(1, 6):
    a = t1.train_step([data[i]])
    b = gs([data[i]])
    torch.cuda.synchronize()
    print(i, "loss", a["loss"].item(), b["loss"].item(), "max|dw|", (m1.store.master - m2.store.master).abs().max().item())
d = (m1.store.master - m2.store.master).abs()
top = torch.topk(d, 10)
segs = sorted(m1.store.segments, key=lambda sg: sg.offset)
for v, ix in zip(top.values.tolist(), top.indices.tolist()):
    seg = [sg for sg in segs if sg.offset <= ix][-1]
    print(f"{v:.3e} {seg.key} (+{ix - seg.offset})")
