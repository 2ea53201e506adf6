#!/usr/bin/env bash
# Linear probe ViT-B/16, SGD(momentum 0.9), batch 4096, lr 3.0 (not batch-scaled), no warmup, 90 epochs.
BS=4096 OPT=sgd LR=3.0 WARMUP_EP=0 NAME="$(basename "$0" .sh)" \
  exec "$(dirname "$0")/ln-lars-vit-b16-224-in1k.sh" "$@"
