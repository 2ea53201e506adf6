"""Convert a PyTorch (timm-style) state dict to a Flax msgpack tree usable with --pretrained-ckpt.

Reference CLI: scripts/convert_pytorch_to_flax.py ckpt [--num-heads N] [--from-timm] [--exclude-heads].
``--from-timm`` needs the timm package and network access, neither of which exists offline; pass a
local .pth/.pt file instead (loaded with torch.load(weights_only=True): nothing is executed).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jumbo_mae_tpu_amd.ckpt.checkpoint import write_bytes  # noqa: E402
from jumbo_mae_tpu_amd.ckpt.convert import torch_to_flax  # noqa: E402
from jumbo_mae_tpu_amd.ckpt.msgpack_flax import msgpack_serialize  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("checkpoint")
    ap.add_argument("--num-heads", type=int, default=6)
    ap.add_argument("--from-timm", action="store_true", default=False)
    ap.add_argument("--exclude-heads", action="store_true", default=False)
    ap.add_argument("--sincos-posemb", action="store_true", help="drop pos_embed (model uses fixed sincos2d)")
    ap.add_argument("--output", default=None)
    a = ap.parse_args(argv)
    if a.from_timm:
        try:
            import timm  # noqa: F401
        except ImportError:
            raise SystemExit("--from-timm needs timm (not installed); convert a local state-dict file instead")
        model = timm.create_model(a.checkpoint, pretrained=True)
        sd = model.state_dict()
    else:
        sd = torch.load(a.checkpoint, map_location="cpu", weights_only=True)
        if "model" in sd and isinstance(sd["model"], dict):
            sd = sd["model"]
    sd = {k: v.float().numpy() for k, v in sd.items() if isinstance(v, torch.Tensor)}
    tree = torch_to_flax(sd, a.num_heads, exclude_heads=a.exclude_heads, learnable_posemb=not a.sincos_posemb)
    out = a.output or (os.path.splitext(os.path.basename(a.checkpoint))[0] + ".msgpack")
    write_bytes(out, msgpack_serialize(tree))
    print(f"wrote {out}")
    return out


if __name__ == "__main__":
    main()
