"""Finetune / linear-probe entry point (same flags as the reference's src/main_finetune.py).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 src/main_finetune.py --mode linear ...
"""
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
warnings.filterwarnings("ignore")

from jumbo_mae_tpu_amd.train.finetune import cli  # noqa: E402

if __name__ == "__main__":
    cli()
