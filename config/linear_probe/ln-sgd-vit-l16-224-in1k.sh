#!/usr/bin/env bash
# Linear probe ViT-L/16, SGD(momentum 0.9), batch 4096, lr 3.0, no warmup, 90 epochs.
BS=4096 OPT=sgd LR=3.0 WARMUP_EP=0 MODEL_FLAGS="--layers 24 --dim 1024 --heads 16" NAME="$(basename "$0" .sh)" \
  exec "$(dirname "$0")/ln-lars-vit-b16-224-in1k.sh" "$@"
