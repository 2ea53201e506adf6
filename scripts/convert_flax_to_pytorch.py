"""Convert a Flax msgpack checkpoint (ours or the reference's) to a PyTorch state dict (.pth).

Jumbo-aware (3 CLS tokens, shared jumbo MLP, norm3 / ls3); standard parts keep timm names.
Reference CLI: scripts/convert_flax_to_pytorch.py ckpt.msgpack [--exclude-heads].
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jumbo_mae_tpu_amd.ckpt.checkpoint import load_params  # noqa: E402
from jumbo_mae_tpu_amd.ckpt.convert import flax_to_torch  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("checkpoint")
    ap.add_argument("--exclude-heads", action="store_true", default=False)
    ap.add_argument("--output", default=None)
    ap.add_argument("--image-size", type=int, default=224,
                    help="input resolution of a sincos-posemb model (sets the exported pos_embed grid)")
    a = ap.parse_args(argv)
    sd = flax_to_torch(load_params(a.checkpoint), exclude_heads=a.exclude_heads, image_size=a.image_size)
    out = a.output or a.checkpoint.replace(".msgpack", ".pth")
    torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, out)
    print(f"wrote {len(sd)} tensors to {out}")
    return out


if __name__ == "__main__":
    main()
